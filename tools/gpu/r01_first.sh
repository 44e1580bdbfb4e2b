#!/bin/bash
# Round-1 first GPU pass: parity tests, bench line, rocprofv3 kernel-trace stats, HBM PMC passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 500 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { echo "bench failed rc=$?"; tail -30 $O/bench.log; exit 1; }
tail -2 $O/bench.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_kt.log 2>&1 || { echo "prof failed rc=$?"; tail -30 $O/prof_kt.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/prof_fetch -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-decrypt > $O/prof_fetch.log 2>&1 || { echo "pmc fetch failed rc=$?"; tail -30 $O/prof_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/prof_write -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-decrypt > $O/prof_write.log 2>&1 || { echo "pmc write failed rc=$?"; tail -30 $O/prof_write.log; exit 1; }
find $O -name "*.csv" | head -50
echo ALLDONE
