#!/bin/bash
# The fixed-base path alone: its parity tests, then kernel stats of the encrypt-only bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_fixed_base.py tests/test_gpu_pair_paths.py -x -q --timeout 200 --timeout-method thread > $O/pytest_fin.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $O/pytest_fin.log; exit 1; }
tail -2 $O/pytest_fin.log
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_fin -o run -- python3 $R/bench.py --steps 8 --warmup 1 --no-cpu-baseline --no-host --no-decrypt --no-public --no-add8 > $O/prof_fin.log 2>&1 || { echo "prof failed rc=$?"; tail -30 $O/prof_fin.log; exit 1; }
grep -E "k_fbp|k_fb_digits" $O/prof_fin/run_kernel_stats.csv | cut -c1-160
tail -1 $O/prof_fin.log | cut -c1-250
echo ALLDONE
