#!/bin/bash
# Same-box A/B: the 4096-bit decryption kernel k_dec4_pow at one wave per SIMD (FPAI_DEC4_OCC = 1,
# ab/libflexpai_dec4occ1.so: 256 VGPRs + 134 AGPRs, no spills) against the product (two waves, 540 B of scratch).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/abdec4
mkdir -p $O
cd $R
BA="--config 4 --n 1048576 --steps 1 --warmup 0 --no-cpu-baseline --no-host --no-add8 --no-strong --no-contention --no-public"
for rep in 1 2; do
  for v in base occ1; do
    L=""; [ $v = occ1 ] && L=$R/ab/libflexpai_dec4occ1.so
    FLEXPAI_LIB=$L timeout -k 10 300 python -u bench.py $BA > $O/c4_${v}_$rep.log 2>&1 || { echo "bench $v failed"; tail -5 $O/c4_${v}_$rep.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e=d['extra']; print(sys.argv[2], sys.argv[3], round(e['decrypt_per_s_per_gpu']/1e3,2), json.dumps({k: round(v['kernel_ms'],1) for k,v in e['decrypt_stages'].items()}), e.get('roundtrip_exact'))" $O/c4_${v}_$rep.log $v $rep
  done
done
echo ALLDONE
