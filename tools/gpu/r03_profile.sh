#!/bin/bash
# Round-3 profiles of the committed tree: kernel-trace/stats of the default bench, HBM traffic (separate
# FETCH_SIZE / WRITE_SIZE passes, tools/pmc_traffic.py) of k_fbp / k_fbp_fin / k_fb_digits (configs[1]) and
# k_add (configs[2]), k_sgp (configs[4]), SQ issue counters of the configs[1] kernels, then the default bench line (which now finds the
# fresh traffic files of this very library).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host > $O/prof_kt.log 2>&1 || { echo "prof failed rc=$?"; tail -30 $O/prof_kt.log; exit 1; }
head -16 $O/prof_kt/run_kernel_stats.csv | cut -c1-150
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_$c -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-decrypt --no-public --no-host --no-add8 --no-strong > $O/pmc_$c.log 2>&1 || { echo "pmc $c failed rc=$?"; tail -20 $O/pmc_$c.log; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc2_$c -o run -- python3 $R/bench.py --config 2 --steps 1 --warmup 0 --no-cpu-baseline --no-public --no-strong > $O/pmc2_$c.log 2>&1 || { echo "pmc2 $c failed rc=$?"; tail -20 $O/pmc2_$c.log; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc4_$c -o run -- python3 $R/bench.py --config 4 --steps 1 --warmup 0 --no-cpu-baseline --no-decrypt --no-public --no-host --no-strong > $O/pmc4_$c.log 2>&1 || { echo "pmc4 $c failed rc=$?"; tail -20 $O/pmc4_$c.log; exit 1; }
done
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmcsq -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-public --no-host --no-add8 --no-strong > $O/pmcsq.log 2>&1 || { echo "pmc sq failed rc=$?"; tail -20 $O/pmcsq.log; exit 1; }
cd $R
python3 tools/pmc_traffic.py $O/pmc_FETCH_SIZE/run_counter_collection.csv $O/pmc_WRITE_SIZE/run_counter_collection.csv --kernel k_fbp --n 1048576 --nb 2048 --window 23 -o profiles/pmc_k_fbp_latest.json || exit 1
for k in k_fbp_fin k_fb_digits; do
  python3 tools/pmc_traffic.py $O/pmc_FETCH_SIZE/run_counter_collection.csv $O/pmc_WRITE_SIZE/run_counter_collection.csv --kernel $k --n 1048576 --nb 2048 -o profiles/pmc_${k}_latest.json || exit 1
done
python3 tools/pmc_traffic.py $O/pmc2_FETCH_SIZE/run_counter_collection.csv $O/pmc2_WRITE_SIZE/run_counter_collection.csv --kernel k_add --n 1048576 --nb 2048 -o profiles/pmc_k_add_latest.json || exit 1
python3 tools/pmc_traffic.py $O/pmc4_FETCH_SIZE/run_counter_collection.csv $O/pmc4_WRITE_SIZE/run_counter_collection.csv --kernel k_sgp --n 4194304 --nb 4096 --window 21 -o profiles/pmc_k_sgp_latest.json || exit 1
mkdir -p $O/pmcjson && cp profiles/pmc_*_latest.json $O/pmcjson/
python3 tools/pmc_sq_summary.py $O/pmcsq/run_counter_collection.csv > $O/pmc_sq_summary.txt 2>&1 || true
head -30 $O/pmc_sq_summary.txt
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { echo "bench failed rc=$?"; tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-600
echo ALLDONE
