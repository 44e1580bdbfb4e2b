#!/bin/bash
# Split-pair sampler (kernels_sgp.hpp): 4096-bit fixed-base and public fixed-base parity, then the configs[4] bench
# (k_sgp for k_fbgp) and the default bench (public fixed-base leg), with a kernel trace of the configs[4] run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_fixed_base_4096.py tests/test_gpu_public_fixed_base.py -x -v --timeout 300 --timeout-method thread > $O/pytest_sgp.log 2>&1; rc=$?
tail -5 $O/pytest_sgp.log
[ $rc -ne 0 ] && { echo "pytest failed rc=$rc"; grep -E "FAILED|Error|error|assert" $O/pytest_sgp.log | head -30; exit 1; }
[ -n "$NO_BENCH" ] && { echo ALLDONE; exit 0; }
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o run -- python3 $R/bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_c4.log 2>&1 || { echo "bench c4 failed rc=$?"; tail -30 $O/bench_c4.log; exit 1; }
head -14 $O/prof_c4/run_kernel_stats.csv | cut -c1-150
tail -1 $O/bench_c4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']; print(d['value'], d['roofline']['kernel'], d['roofline']['kernel_ms'], d['roofline']['frac']); print({k: e[k] for k in ('decrypt_per_s_per_gpu','roundtrip_exact') if k in e})"
cd $R
timeout -k 10 600 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { echo "bench failed rc=$?"; tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']; print(d['value']); print({k: v for k, v in e.items() if 'public' in k or 'pfb' in k})"
echo ALLDONE
