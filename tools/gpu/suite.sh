#!/bin/bash
# The one GPU-iteration script (run through gpurun from the repo root). Steps, each under its own time limit and
# chained so that the first failure ends the call; logs under gpurun_out/, names prefixed with TAG:
#   0. the address-guarded sampler suite (tests/test_gpu_guard.py on libflexpai_xcheck.so; NO_GUARD=1 skips);
#   1. the -m gpu parity tests (TESTS="tests/test_x.py ..." for a subset; NO_TESTS=1 skips), one process;
#   2. one bench line (BENCH_ARGS; NO_BENCH=1 skips);
#   3. PROF=1: a rocprofv3 --kernel-trace --stats profile of bench.py $PROF_ARGS (summary: ${TAG}_prof/run_kernel_stats.csv);
#   4. PMC="FETCH_SIZE WRITE_SIZE ...": one rocprofv3 --pmc pass per counter set (sets separated by ';'), each with
#      --kernel-trace only (MI355X_MICROARCH.md's HBM section: separate passes), over bench.py $PMC_ARGS.
# Any other environment (FLEXPAI_FBS=1, FLEXPAI_FB_WINDOW=...) is exported by the caller and reaches every step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
T=${TAG:-run}
mkdir -p $O
export TMPDIR=/tmp
cd $R
if [ -z "$NO_TESTS" ] && [ -z "$NO_GUARD" ]; then
  # the guarded samplers first (csrc/guard.hpp, the test build): a kernel draft whose indices leave their buffers fails
  # here with the site named, before any unguarded kernel of the draft runs
  timeout -k 10 300 python -u -m pytest tests/test_gpu_guard.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/${T}_guard.log 2>&1 || { echo "guarded suite failed"; grep -E "FAILED|Error|error" $O/${T}_guard.log | head -20; exit 1; }
  tail -1 $O/${T}_guard.log
fi
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $O/${T}_pytest_gpu.log 2>&1; rc=$?
  tail -5 $O/${T}_pytest_gpu.log
  [ $rc -ne 0 ] && { echo "pytest failed rc=$rc"; grep -E "FAILED|Error|error" $O/${T}_pytest_gpu.log | head -20; exit 1; }
fi
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-600} python -u bench.py ${BENCH_ARGS:-} > $O/${T}_bench.log 2>&1 || { echo "bench failed rc=$?"; tail -30 $O/${T}_bench.log; exit 1; }
  tail -1 $O/${T}_bench.log | cut -c1-800
fi
PA=${PROF_ARGS:---steps 5 --warmup 2 --no-cpu-baseline --no-host --no-public --no-add8 --no-strong --no-contention}
if [ -n "$PROF" ]; then
  timeout -k 10 ${PROF_TIMEOUT:-400} rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof -o run -- python3 bench.py $PA > $O/${T}_prof.log 2>&1 || { echo "prof failed rc=$?"; tail -20 $O/${T}_prof.log; exit 1; }
  tail -1 $O/${T}_prof.log | cut -c1-400
  head -12 $O/${T}_prof/run_kernel_stats.csv | cut -c1-160
fi
if [ -n "$PMC" ]; then
  MA=${PMC_ARGS:---steps 1 --warmup 0 --no-cpu-baseline --no-decrypt --no-host --no-public --no-add8 --no-strong --no-contention}
  i=0
  IFS=';' read -ra SETS <<< "$PMC"
  for set in "${SETS[@]}"; do
    i=$((i+1))
    timeout -s KILL ${PMC_TIMEOUT:-180} rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/${T}_pmc$i -o run -- python3 bench.py $MA > $O/${T}_pmc$i.log 2>&1 || { echo "pmc pass $i ($set) failed rc=$?"; tail -20 $O/${T}_pmc$i.log; exit 1; }
    echo "pmc pass $i: $set"
  done
fi
echo ALLDONE
