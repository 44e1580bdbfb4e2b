#!/bin/bash
# GPU side of tools/ab_fbs_digits.sh: the fused-digit library's fixed-base suite once, then base / D interleaved three
# times on one box (bench.py, headline config, legs off; the D run with decrypt on: its round trip must be exact).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab05d
mkdir -p $O
export TMPDIR=/tmp
cd $R
FLEXPAI_LIB=$R/ab/libflexpai_abD.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fbs.py tests/test_gpu_fixed_base.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_D.log 2>&1 || { echo "D suite failed"; tail -15 $O/pytest_D.log; exit 1; }
tail -1 $O/pytest_D.log
BA="--steps 10 --warmup 2 --no-cpu-baseline --no-host --no-public --no-add8 --no-strong --no-contention --no-decrypt"
for rep in 1 2 3; do
  for v in base D; do
    L=""; [ $v = D ] && L=$R/ab/libflexpai_abD.so
    A="$BA"; [ $v = D ] && [ $rep = 1 ] && A="--steps 10 --warmup 2 --no-cpu-baseline --no-host --no-public --no-add8 --no-strong --no-contention"
    FLEXPAI_LIB=$L timeout -k 10 240 python -u bench.py $A > $O/bench_${v}_$rep.log 2>&1 || { echo "bench $v failed"; tail -5 $O/bench_${v}_$rep.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e=d['extra']; print(sys.argv[2], sys.argv[3], round(d['value']/1e6,3), round(d['ms_per_step'],3), json.dumps({k: round(v['kernel_ms'],3) for k, v in e['stages'].items()}), e.get('roundtrip_exact'))" $O/bench_${v}_$rep.log $v $rep
  done
done
echo ALLDONE
