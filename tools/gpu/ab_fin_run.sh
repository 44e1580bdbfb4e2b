#!/bin/bash
# Same-box A/B of a k_fbp_fin variant (ab/libflexpai_fin2acc.so) against the product: the headline bench, interleaved
# three times (legs off), k_fbp_fin's HIP-event time and the step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/abfin
mkdir -p $O
cd $R
BA="--steps 10 --warmup 2 --no-cpu-baseline --no-host --no-public --no-add8 --no-strong --no-contention --no-decrypt"
for rep in 1 2 3; do
  for v in base v; do
    L=""; [ $v = v ] && L=$R/ab/libflexpai_fin2acc.so
    FLEXPAI_LIB=$L timeout -k 10 240 python -u bench.py $BA > $O/b_${v}_$rep.log 2>&1 || { echo "bench $v failed"; tail -5 $O/b_${v}_$rep.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e=d['extra']; print(sys.argv[2], sys.argv[3], round(d['value']/1e6,3), round(d['ms_per_step'],3), json.dumps({k: round(v['kernel_ms'],3) for k, v in e['stages'].items()}))" $O/b_${v}_$rep.log $v $rep
  done
done
FLEXPAI_LIB=$R/ab/libflexpai_fin2acc.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fixed_base.py tests/test_gpu_fbs.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_v.log 2>&1; tail -1 $O/pytest_v.log
echo ALLDONE
