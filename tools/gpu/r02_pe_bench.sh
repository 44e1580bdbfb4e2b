#!/bin/bash
# The public-key leg of the default bench with the split-pair kernels and with k_encrypt.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
for v in 1 0; do
  FLEXPAI_PAIR=$v timeout -k 10 400 python -u bench.py --steps 3 --no-cpu-baseline --no-host --no-add8 --no-decrypt > $O/bench_pe$v.log 2>&1 || { echo "bench failed rc=$?"; tail -20 $O/bench_pe$v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_pe$v.log').read().strip().splitlines()[-1]); e=d['extra']; print('pair=$v', round(d['value']), e.get('public_key_path'))"
done
echo ALLDONE
