#!/bin/bash
# k_sgp parity (4096-bit fixed base, public fixed base), then its configs[4] HBM traffic (FETCH / WRITE passes).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_fixed_base_4096.py tests/test_gpu_public_fixed_base.py -x -v --timeout 300 --timeout-method thread > $O/pytest_sgp.log 2>&1; rc=$?
tail -3 $O/pytest_sgp.log
[ $rc -ne 0 ] && { echo "pytest failed rc=$rc"; grep -E "FAILED|Error|error|assert" $O/pytest_sgp.log | head -30; exit 1; }
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc4_$c -o run -- python3 $R/bench.py --config 4 --steps 1 --warmup 0 --no-cpu-baseline --no-decrypt --no-public --no-host --no-strong > $O/pmc4_$c.log 2>&1 || { echo "pmc4 $c failed rc=$?"; tail -20 $O/pmc4_$c.log; exit 1; }
done
cd $R
python3 tools/pmc_traffic.py $O/pmc4_FETCH_SIZE/run_counter_collection.csv $O/pmc4_WRITE_SIZE/run_counter_collection.csv --kernel k_sgp --n 4194304 --nb 4096 --window 21 -o $O/pmc_k_sgp.json || exit 1
echo ALLDONE
