#!/bin/bash
# Fixed-base digit window sweep (8/12/16 bits): encrypt-only bench lines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
for w in ${WINDOWS:-8 12 16}; do
  FLEXPAI_FB_WINDOW=$w timeout -k 10 300 python bench.py --fb-window $w --steps 5 --no-cpu-baseline --no-host --no-public --no-add8 --no-decrypt > $O/fbw_$w.log 2>&1 || { echo "w=$w failed rc=$?"; tail -20 $O/fbw_$w.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/fbw_$w.log').read().strip().splitlines()[-1]); print($w, d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['extra']['fixed_base'])"
done
echo ALLDONE
