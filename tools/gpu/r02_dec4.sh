#!/bin/bash
# 4096-bit split-pair decryption: parity tests, then the configs[4] bench line (decrypt rate in extra).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_dec4.py tests/test_gpu_native.py tests/test_gpu_dec_lane.py tests/test_gpu_fixed_base_4096.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_dec4.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|ERROR|Error" $O/pytest_dec4.log | tail -15
[ $rc -ne 0 ] && { tail -40 $O/pytest_dec4.log; exit 1; }
timeout -k 10 500 python -u bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline --no-host > $O/bench_c4.log 2>&1 || { echo "bench c4 failed rc=$?"; tail -20 $O/bench_c4.log; exit 1; }
python3 - $O/bench_c4.log <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e=d['extra']
print('value', round(d['value']), d['roofline']['kernel'], round(d['roofline']['kernel_ms'],1), round(d['roofline']['frac'],3))
print('dec', e.get('decrypt_path'), e.get('decrypt_per_s_per_gpu'), e.get('decrypt_kernel_ms'), e.get('decrypt_int_mac_frac'), e.get('roundtrip_exact'))
PY
echo ALLDONE
