#!/bin/bash
# GPU round trip: parity tests, one bench line, a kernel-trace profile of the bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > $O/pytest_gpu.log 2>&1; rc=$?
tail -15 $O/pytest_gpu.log
[ $rc -ne 0 ] && { echo "pytest failed rc=$rc"; exit 1; }
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > $O/bench.log 2>&1 || { echo "bench failed rc=$?"; tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log
if [ -n "$PROFILE" ]; then
  cd /tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host > $O/prof_kt.log 2>&1 || { echo "prof failed rc=$?"; tail -30 $O/prof_kt.log; exit 1; }
  head -8 $O/prof_kt/run_kernel_stats.csv | cut -c1-200
fi
echo ALLDONE
