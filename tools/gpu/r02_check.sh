#!/bin/bash
# Full GPU suite, the default bench line (encrypt, decrypt, public key, configs[2] leg) and kernel stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_check.log 2>&1 || { echo "tests failed rc=$?"; grep -E "FAILED|Error|assert" $O/pytest_check.log | head -20; tail -5 $O/pytest_check.log; exit 1; }
tail -2 $O/pytest_check.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-host > $O/bench_check.log 2>&1 || { echo "bench failed rc=$?"; tail -30 $O/bench_check.log; exit 1; }
tail -1 $O/bench_check.log | cut -c1-300
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_check -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-host > $O/prof_check.log 2>&1 || { echo "prof failed rc=$?"; tail -30 $O/prof_check.log; exit 1; }
head -12 $O/prof_check/run_kernel_stats.csv | cut -c1-150
echo ALLDONE
