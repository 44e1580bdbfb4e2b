#!/bin/bash
# One GPU iteration: a subset of the parity tests (TESTS, default all), then optionally a bench line
# (BENCH=1, BENCH_ARGS) and a kernel-trace profile of it (PROFILE=1). Every GPU step has its own time
# limit and the steps are chained: the first failure ends the call.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 180 --timeout-method thread ${PYTEST_ARGS:-} > $O/pytest_gpu.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest_gpu.log | tail -60
[ $rc -ne 0 ] && { echo "pytest failed rc=$rc"; tail -60 $O/pytest_gpu.log; exit 1; }
if [ -n "$BENCH" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-500} python -u bench.py ${BENCH_ARGS:-} > $O/bench.log 2>&1 || { echo "bench failed rc=$?"; tail -40 $O/bench.log; exit 1; }
  tail -1 $O/bench.log
fi
if [ -n "$PROFILE" ]; then
  cd /tmp
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt -o run -- python3 $R/bench.py ${PROF_ARGS:---steps 3 --warmup 1 --no-cpu-baseline --no-host} > $O/prof_kt.log 2>&1 || { echo "prof failed rc=$?"; tail -30 $O/prof_kt.log; exit 1; }
  head -16 $O/prof_kt/run_kernel_stats.csv | cut -c1-160
fi
echo ALLDONE
