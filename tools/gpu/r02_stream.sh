#!/bin/bash
# k_fbp with rows streamed behind the reads: fixed-base parity tests, then the default bench line and its stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_fixed_base.py tests/test_gpu_pair_paths.py -x -q --timeout 200 --timeout-method thread > $O/pytest_stream.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $O/pytest_stream.log; exit 1; }
tail -2 $O/pytest_stream.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-host > $O/bench_stream.log 2>&1 || { echo "bench failed rc=$?"; tail -30 $O/bench_stream.log; exit 1; }
tail -1 $O/bench_stream.log | cut -c1-400
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_stream -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-host --no-decrypt --no-public --no-add8 > $O/prof_stream.log 2>&1 || { echo "prof failed rc=$?"; tail -30 $O/prof_stream.log; exit 1; }
head -6 $O/prof_stream/run_kernel_stats.csv | cut -c1-150
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmcsq_stream -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-public --no-host --no-add8 --no-decrypt > $O/pmcsq_stream.log 2>&1 || { echo "pmc sq failed rc=$?"; tail -20 $O/pmcsq_stream.log; exit 1; }
cd $R
python3 tools/pmc_sq_summary.py $O/pmcsq_stream/run_counter_collection.csv > $O/pmc_sq_stream.txt 2>&1 || true
grep k_fbp $O/pmc_sq_stream.txt
echo ALLDONE
