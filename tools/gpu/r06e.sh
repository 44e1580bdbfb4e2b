set -o pipefail
O=gpurun_out; mkdir -p $O
T=r06e
timeout -k 10 300 python -u -m pytest tests/test_gpu_guard.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/${T}_guard.log 2>&1 || { echo "guard failed"; tail -30 $O/${T}_guard.log; exit 1; }
tail -1 $O/${T}_guard.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/${T}_pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/${T}_pytest_gpu.log; exit 1; }
tail -1 $O/${T}_pytest_gpu.log
FLEXPAI_LIB=$PWD/ab/libflexpai_sgs3.so timeout -k 10 400 python -u -m pytest tests/test_gpu_sgs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/${T}_sgs3_tests.log 2>&1 || { echo "sgs3 tests failed"; tail -20 $O/${T}_sgs3_tests.log; exit 1; }
tail -1 $O/${T}_sgs3_tests.log
B="--config 4 --steps 3 --warmup 1 --no-cpu-baseline --no-host --no-public --no-decrypt"
for rep in 1 2; do for v in base sgs3; do
  L=""; [ $v != base ] && L=$PWD/ab/libflexpai_$v.so
  FLEXPAI_LIB=$L timeout -k 10 240 python -u bench.py $B > $O/${T}_c4ab_${v}_$rep.log 2>&1 || { echo "c4 ab $v failed"; tail -5 $O/${T}_c4ab_${v}_$rep.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e=d['extra']; print(sys.argv[2], sys.argv[3], round(d['value']/1e6,3), round(d['ms_per_step'],2), {k:round(v['kernel_ms'],2) for k,v in e['stages'].items()})" $O/${T}_c4ab_${v}_$rep.log $v $rep
done; done
timeout -k 10 300 python -u tools/pfb_breakeven.py > $O/${T}_pfb_breakeven.log 2>&1 || { echo "breakeven failed"; tail -5 $O/${T}_pfb_breakeven.log; exit 1; }
tail -1 $O/${T}_pfb_breakeven.log
echo ALLDONE
