#!/bin/bash
# Pair fixed-base sampler: parity tests, then encrypt-only bench lines with the pair kernel and with k_fb.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_fixed_base.py tests/test_gpu_package.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_pair.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|ERROR|Error" $O/pytest_pair.log | tail -15
[ $rc -ne 0 ] && { tail -40 $O/pytest_pair.log; exit 1; }
for v in 1 0; do
  FLEXPAI_FB_PAIR=$v timeout -k 10 300 python bench.py --steps 5 --no-cpu-baseline --no-host --no-public --no-add8 > $O/bench_pair$v.log 2>&1 || { echo "bench pair=$v failed rc=$?"; tail -20 $O/bench_pair$v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_pair$v.log').read().strip().splitlines()[-1]); print('pair=$v', d['value'], d['roofline']['kernel'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['extra'].get('stages'), d['extra'].get('roundtrip_exact'))"
done
echo ALLDONE
