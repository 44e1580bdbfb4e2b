#!/bin/bash
# HBM traffic of the bench's dominant kernels (separate FETCH_SIZE / WRITE_SIZE passes, per
# MI355X_MICROARCH.md §HBM) + the step-0 integer-throughput microbenchmark.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 $R/tools/microbench/int_throughput > $O/int_throughput.txt 2>&1 || { echo "microbench failed"; cat $O/int_throughput.txt; exit 1; }
cat $O/int_throughput.txt
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_$c -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-decrypt --no-public --no-host > $O/pmc_$c.log 2>&1 || { echo "pmc $c failed rc=$?"; tail -20 $O/pmc_$c.log; exit 1; }
done
cd $R
for k in k_crt_a k_crt_b k_crt_fin; do
  python3 tools/pmc_traffic.py $O/pmc_FETCH_SIZE/run_counter_collection.csv $O/pmc_WRITE_SIZE/run_counter_collection.csv --kernel $k --n 1048576 --nb 2048 -o $O/pmc_${k}_latest.json || exit 1
done
echo ALLDONE
