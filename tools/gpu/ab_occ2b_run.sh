#!/bin/bash
# Same-box A/B: k_crt_a (engine_lane.hip, FPAI_LANE_OCC = 2) and k_fbg_garner (engine_grp.hip, FPAI_GARNER_OCC = 2) at two
# waves per SIMD (ab/libflexpai_occ2b.so) against the product: the generic CRT leg of configs[1] and the configs[4] step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/abocc2b
mkdir -p $O
cd $R
BA="--steps 2 --warmup 1 --no-cpu-baseline --no-host --no-add8 --no-strong --no-contention --no-public --no-decrypt"
for rep in 1 2; do
  for v in base occ2b; do
    L=""; [ $v = occ2b ] && L=$R/ab/libflexpai_occ2b.so
    FLEXPAI_LIB=$L timeout -k 10 300 python -u bench.py $BA > $O/c1_${v}_$rep.log 2>&1 || { echo "bench c1 $v failed"; tail -5 $O/c1_${v}_$rep.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e=d['extra']; print('c1', sys.argv[2], sys.argv[3], round(e['generic_crt_path']['value']/1e6,4), json.dumps(e['generic_crt_path']['stages_ms']))" $O/c1_${v}_$rep.log $v $rep
    FLEXPAI_LIB=$L timeout -k 10 300 python -u bench.py --config 4 $BA > $O/c4_${v}_$rep.log 2>&1 || { echo "bench c4 $v failed"; tail -5 $O/c4_${v}_$rep.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e=d['extra']; print('c4', sys.argv[2], sys.argv[3], round(d['value']/1e6,4), json.dumps({k: round(v['kernel_ms'],2) for k,v in e['stages'].items()}))" $O/c4_${v}_$rep.log $v $rep
  done
done
echo ALLDONE
