#!/bin/bash
# One default bench line plus a kernel-trace/stats profile of the same command.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > $O/bench.log 2>&1 || { echo "bench failed rc=$?"; tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host > $O/prof_kt.log 2>&1 || { echo "prof failed rc=$?"; tail -30 $O/prof_kt.log; exit 1; }
head -14 $O/prof_kt/run_kernel_stats.csv | cut -c1-150
echo ALLDONE
