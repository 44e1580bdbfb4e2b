#!/bin/bash
# Round-1 checkpoint on the GPU: parity tests, smoke, bench line, kernel-trace stats, and the HBM
# PMC passes (FETCH_SIZE / WRITE_SIZE in separate runs) for the bench's dominant kernels.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { echo "bench failed rc=$?"; tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-600
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host > $O/prof_kt.log 2>&1 || { echo "prof failed rc=$?"; tail -30 $O/prof_kt.log; exit 1; }
head -12 $O/prof_kt/run_kernel_stats.csv | cut -c1-160
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_$c -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-decrypt --no-public --no-host > $O/pmc_$c.log 2>&1 || { echo "pmc $c failed rc=$?"; tail -20 $O/pmc_$c.log; exit 1; }
done
cd $R
for k in k_fb k_crt_fin; do
  python3 tools/pmc_traffic.py $O/pmc_FETCH_SIZE/run_counter_collection.csv $O/pmc_WRITE_SIZE/run_counter_collection.csv --kernel $k --n 1048576 --nb 2048 -o $O/pmc_${k}_latest.json || exit 1
done
echo ALLDONE
