#!/bin/bash
# Pair-path parity (pairs vs the kernels they replace), then configs[4]: a bench line with decryption, a
# kernel-trace/stats profile, and the HBM traffic of k_fbgp (separate FETCH_SIZE / WRITE_SIZE passes).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_pair_paths.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_pp.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|ERROR|Error" $O/pytest_pp.log | tail -8
[ $rc -ne 0 ] && { tail -40 $O/pytest_pp.log; exit 1; }
timeout -k 10 500 python -u bench.py --config 4 --steps 2 --warmup 1 > $O/bench_c4.log 2>&1 || { echo "bench c4 failed rc=$?"; tail -20 $O/bench_c4.log; exit 1; }
tail -1 $O/bench_c4.log | cut -c1-300
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o run -- python3 $R/bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline --no-host --no-public > $O/prof_c4.log 2>&1 || { echo "prof failed rc=$?"; tail -30 $O/prof_c4.log; exit 1; }
head -12 $O/prof_c4/run_kernel_stats.csv | cut -c1-150
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc4_$c -o run -- python3 $R/bench.py --config 4 --steps 1 --warmup 0 --no-cpu-baseline --no-decrypt --no-public --no-host > $O/pmc4_$c.log 2>&1 || { echo "pmc $c failed rc=$?"; tail -20 $O/pmc4_$c.log; exit 1; }
done
cd $R
python3 tools/pmc_traffic.py $O/pmc4_FETCH_SIZE/run_counter_collection.csv $O/pmc4_WRITE_SIZE/run_counter_collection.csv --kernel k_fbgp --n 4194304 --nb 4096 --window 21 -o $O/pmc_k_fbgp_latest.json || exit 1
cat $O/pmc_k_fbgp_latest.json
echo ALLDONE
