#!/bin/bash
# Fixed-base window sweep with the pair sampler (encrypt-only bench lines).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
for w in 20 21 22 23; do
  timeout -k 10 300 python bench.py --fb-window $w --steps 5 --no-cpu-baseline --no-host --no-public --no-add8 --no-decrypt > $O/fbw_$w.log 2>&1 || { echo "w=$w failed rc=$?"; tail -20 $O/fbw_$w.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/fbw_$w.log').read().strip().splitlines()[-1]); print($w, round(d['value']), round(d['roofline']['kernel_ms'],2), d['extra']['fixed_base'], d['setup'].get('fixed_base_table_bytes'))"
done
echo ALLDONE
