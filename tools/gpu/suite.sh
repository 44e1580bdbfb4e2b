#!/bin/bash
# GPU check: the -m gpu suite (or TESTS="tests/test_x.py ..."; one process, per-test time limit), then one bench
# line (BENCH_ARGS; NO_BENCH=1 skips it). Logs under gpurun_out/ (TAG prefixes their names).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
T=${TAG:-run}
mkdir -p $O
export TMPDIR=/tmp
cd $R
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $O/${T}_pytest_gpu.log 2>&1; rc=$?
  tail -5 $O/${T}_pytest_gpu.log
  [ $rc -ne 0 ] && { echo "pytest failed rc=$rc"; grep -E "FAILED|Error|error" $O/${T}_pytest_gpu.log | head -20; exit 1; }
fi
[ -n "$NO_BENCH" ] && { echo ALLDONE; exit 0; }
timeout -k 10 ${BENCH_TIMEOUT:-600} python -u bench.py ${BENCH_ARGS:-} > $O/${T}_bench.log 2>&1 || { echo "bench failed rc=$?"; tail -30 $O/${T}_bench.log; exit 1; }
tail -1 $O/${T}_bench.log | cut -c1-800
echo ALLDONE
