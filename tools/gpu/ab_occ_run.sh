#!/bin/bash
# Same-box A/B of the pair exponentiation kernels' occupancy (engine_pair.hip built with FPAI_LANE_OCC = 2 into
# ab/libflexpai_occ2.so): decrypt and the generic CRT encrypt of the bench, product vs occ2, interleaved twice.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/abocc
mkdir -p $O
cd $R
BA="--steps 2 --warmup 1 --no-cpu-baseline --no-host --no-add8 --no-strong --no-contention --no-public"
for rep in 1 2; do
  for v in base occ2; do
    L=""; [ $v = occ2 ] && L=$R/ab/libflexpai_occ2.so
    FLEXPAI_LIB=$L timeout -k 10 300 python -u bench.py $BA > $O/bench_${v}_$rep.log 2>&1 || { echo "bench $v failed"; tail -5 $O/bench_${v}_$rep.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e=d['extra']; print(sys.argv[2], sys.argv[3], round(e['decrypt_per_s_per_gpu']/1e6,4), round(e['decrypt_stages']['k_dec_pow']['kernel_ms'],2), round(e['generic_crt_path']['value']/1e6,4), json.dumps(e['generic_crt_path']['stages_ms']), e['roundtrip_exact'])" $O/bench_${v}_$rep.log $v $rep
  done
done
echo ALLDONE
