#!/bin/bash
# Round GPU check: the whole -m gpu suite (one process, per-test time limit), then one default bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $O/pytest_gpu.log 2>&1; rc=$?
tail -5 $O/pytest_gpu.log
[ $rc -ne 0 ] && { echo "pytest failed rc=$rc"; grep -E "FAILED|Error|error" $O/pytest_gpu.log | head -20; exit 1; }
[ -n "$NO_BENCH" ] && { echo ALLDONE; exit 0; }
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $O/bench.log 2>&1 || { echo "bench failed rc=$?"; tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-600
echo ALLDONE
