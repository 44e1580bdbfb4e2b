#!/bin/bash
# Pair kernels everywhere: the full GPU suite, the default bench, and the same bench on the 2S-limb kernels.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -5 $O/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/pytest_gpu.log | head -30; exit 1; }
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_pair.log 2>&1 || { echo "bench failed rc=$?"; tail -20 $O/bench_pair.log; exit 1; }
FLEXPAI_PAIR=0 FLEXPAI_FB_PAIR=0 timeout -k 10 400 python bench.py --no-cpu-baseline --no-host > $O/bench_nopair.log 2>&1 || { echo "bench nopair failed rc=$?"; tail -20 $O/bench_nopair.log; exit 1; }
for f in bench_pair bench_nopair; do
python3 - $O/$f.log <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e=d['extra']
print(sys.argv[1].split('/')[-1], 'value', round(d['value']), 'dom', d['roofline']['kernel'], round(d['roofline']['kernel_ms'],2), 'frac', round(d['roofline']['frac'],3))
print('  dec', e.get('decrypt_path'), round(e['decrypt_per_s_per_gpu']), 'ms', round(e['decrypt_kernel_ms'],1), 'frac', round(e['decrypt_int_mac_frac'],3), e.get('decrypt_stages'))
g=e.get('generic_crt_path',{}); print('  generic', round(g.get('value',0)), g.get('stages_ms'), g.get('k_crt_b_int_mac_frac'))
c=e.get('config2_add8',{}); print('  cfg2', round(c.get('elements_per_s',0)), c.get('decrypt_ms'), c.get('k_add_ms'), c.get('statuses_ok'), 'rt', e.get('roundtrip_exact'))
PY
done
echo ALLDONE
