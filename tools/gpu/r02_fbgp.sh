#!/bin/bash
# 4096-bit pair-group sampler: parity tests, then configs[4] bench lines with k_fbgp and with k_fbg.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_fixed_base_4096.py tests/test_gpu_dec4.py tests/test_gpu_native.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_fbgp.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|ERROR|Error" $O/pytest_fbgp.log | tail -15
[ $rc -ne 0 ] && { tail -40 $O/pytest_fbgp.log; exit 1; }
for v in 1 0; do
  FLEXPAI_FB_PAIR=$v timeout -k 10 500 python -u bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline --no-host --no-decrypt > $O/bench_c4_p$v.log 2>&1 || { echo "bench c4 p=$v failed rc=$?"; tail -20 $O/bench_c4_p$v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_c4_p$v.log').read().strip().splitlines()[-1]); print('pair=$v', round(d['value']), d['roofline']['kernel'], round(d['roofline']['kernel_ms'],1), round(d['roofline']['frac'],3), d['extra'].get('stages'), d['setup'].get('fixed_base_build_wall_ms'))"
done
echo ALLDONE
