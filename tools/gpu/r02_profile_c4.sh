#!/bin/bash
# configs[4] (nb = 4096, 4M elements, fixed-base on the group engine): bench line, kernel-trace/stats
# profile and HBM traffic of k_fbg / k_crt_fin (separate FETCH_SIZE / WRITE_SIZE passes, gfx950
# correction of MI355X_MICROARCH.md).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o run -- python3 $R/bench.py --config 4 --steps 3 --warmup 1 --no-cpu-baseline --no-decrypt --no-public > $O/prof_c4.log 2>&1 || { echo "prof failed rc=$?"; tail -30 $O/prof_c4.log; exit 1; }
tail -1 $O/prof_c4.log | cut -c1-300
head -12 $O/prof_c4/run_kernel_stats.csv | cut -c1-150
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc4_$c -o run -- python3 $R/bench.py --config 4 --steps 1 --warmup 0 --no-cpu-baseline --no-decrypt --no-public > $O/pmc4_$c.log 2>&1 || { echo "pmc $c failed rc=$?"; tail -20 $O/pmc4_$c.log; exit 1; }
done
cd $R
python3 tools/pmc_traffic.py $O/pmc4_FETCH_SIZE/run_counter_collection.csv $O/pmc4_WRITE_SIZE/run_counter_collection.csv --kernel k_fbg --n 4194304 --nb 4096 --window 21 -o $O/pmc_k_fbg_latest.json || exit 1
for k in k_crt_fin k_fb_digits; do
  python3 tools/pmc_traffic.py $O/pmc4_FETCH_SIZE/run_counter_collection.csv $O/pmc4_WRITE_SIZE/run_counter_collection.csv --kernel $k --n 4194304 --nb 4096 -o $O/pmc_${k}_4096_latest.json || exit 1
done
echo ALLDONE
