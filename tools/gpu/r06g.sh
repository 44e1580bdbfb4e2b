set -o pipefail
O=gpurun_out; mkdir -p $O
T=r06g
timeout -k 10 600 python -u -m pytest tests/test_gpu_sgs.py tests/test_gpu_fixed_base_4096.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/${T}_sgs_tests.log 2>&1 || { echo "sgs tests failed"; tail -40 $O/${T}_sgs_tests.log; exit 1; }
tail -1 $O/${T}_sgs_tests.log
FLEXPAI_LIB=$PWD/ab/libflexpai_bfin1.so timeout -k 10 600 python -u -m pytest tests/test_gpu_sgs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/${T}_bfin1_tests.log 2>&1 || { echo "bfin1 tests failed"; tail -20 $O/${T}_bfin1_tests.log; exit 1; }
tail -1 $O/${T}_bfin1_tests.log
B="--config 4 --steps 3 --warmup 1 --no-cpu-baseline --no-host --no-public --no-decrypt"
for rep in 1 2; do for v in prefold fold bfin1; do
  L=""; [ $v != fold ] && L=$PWD/ab/libflexpai_$v.so
  FLEXPAI_LIB=$L timeout -k 10 240 python -u bench.py $B > $O/${T}_c4ab_${v}_$rep.log 2>&1 || { echo "c4 ab $v failed"; tail -5 $O/${T}_c4ab_${v}_$rep.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e=d['extra']; print(sys.argv[2], sys.argv[3], round(d['value']/1e6,3), round(d['ms_per_step'],2), {k:round(v['kernel_ms'],2) for k,v in e['stages'].items()}, d['extra'].get('roundtrip_exact'))" $O/${T}_c4ab_${v}_$rep.log $v $rep
done; done
echo ALLDONE
