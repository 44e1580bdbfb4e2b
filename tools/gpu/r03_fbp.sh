#!/bin/bash
# Fixed-base (k_fbp) parity + a bench line with a kernel-trace profile.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_fixed_base.py tests/test_gpu_pair_paths.py ${PYTEST_EXTRA:-} -x -q --timeout 300 --timeout-method thread > $O/pytest_fbp.log 2>&1; rc=$?
tail -5 $O/pytest_fbp.log
[ $rc -ne 0 ] && { echo "pytest failed rc=$rc"; grep -E "FAILED|Error|error" $O/pytest_fbp.log | head -20; exit 1; }
timeout -k 10 400 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $O/bench_fbp.log 2>&1 || { echo "bench failed rc=$?"; tail -30 $O/bench_fbp.log; exit 1; }
tail -1 $O/bench_fbp.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']); print(d['extra'].get('stages')); print(d.get('setup'))"
[ -n "$NO_PROF" ] && { echo ALLDONE; exit 0; }
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_fbp -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host > $O/prof_fbp.log 2>&1 || { echo "prof failed rc=$?"; tail -30 $O/prof_fbp.log; exit 1; }
head -12 $O/prof_fbp/run_kernel_stats.csv | cut -c1-160
echo ALLDONE
