set -o pipefail
O=gpurun_out; mkdir -p $O
T=r06d
timeout -k 10 300 python -u -m pytest tests/test_gpu_guard.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/${T}_guard.log 2>&1 || { echo "guard failed"; tail -30 $O/${T}_guard.log; exit 1; }
tail -1 $O/${T}_guard.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/${T}_pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/${T}_pytest_gpu.log; exit 1; }
tail -1 $O/${T}_pytest_gpu.log
A="--steps 20 --warmup 2 --no-cpu-baseline --no-host --no-add8 --no-contention --no-strong --no-nb1024 --no-decrypt"
FLEXPAI_TABLE_POOL=0 timeout -k 10 300 python -u bench.py $A > $O/${T}_ab_plain.log 2>&1 || { echo "ab plain failed"; tail -20 $O/${T}_ab_plain.log; exit 1; }
timeout -k 10 300 python -u bench.py $A > $O/${T}_ab_pool.log 2>&1 || { echo "ab pool failed"; tail -20 $O/${T}_ab_pool.log; exit 1; }
FLEXPAI_TABLE_POOL=0 timeout -k 10 300 python -u bench.py $A > $O/${T}_ab_plain2.log 2>&1 || { echo "ab plain2 failed"; exit 1; }
timeout -k 10 300 python -u bench.py $A > $O/${T}_ab_pool2.log 2>&1 || { echo "ab pool2 failed"; exit 1; }
for f in plain pool plain2 pool2; do python3 -c "
import json,sys; d=json.loads(open('$O/${T}_ab_$f.log').read().strip().splitlines()[-1]); e=d['extra']
print('$f', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), 'ms', {k:round(v['kernel_ms'],3) for k,v in e['stages'].items()}, 'pfb', round(e['public_key_fixed_base']['setup_ms']), 'ms setup', round(e['public_key_fixed_base']['value']/1e6,2))"; done
FLEXPAI_SETUP_TRACE=1 timeout -k 10 300 python -u tools/pfb_setup_trace.py --repeat 2 > $O/${T}_pfb.log 2>&1 || { echo pfb failed; tail -20 $O/${T}_pfb.log; exit 1; }
grep -E "public tables|holder tables|uploads" $O/${T}_pfb.log
timeout -k 10 600 python -u bench.py > $O/${T}_bench.log 2>&1 || { echo "bench failed"; tail -30 $O/${T}_bench.log; exit 1; }
tail -1 $O/${T}_bench.log | cut -c1-300
FLEXPAI_LIB=$PWD/ab/libflexpai_ab40.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fbs.py tests/test_gpu_guard.py -m gpu -x -q --timeout 120 --timeout-method thread -k "not inject" > $O/${T}_ab40_tests.log 2>&1 || { echo "ab40 tests failed"; tail -20 $O/${T}_ab40_tests.log; exit 1; }
tail -1 $O/${T}_ab40_tests.log
B="--steps 10 --warmup 2 --no-cpu-baseline --no-host --no-public --no-add8 --no-strong --no-contention --no-nb1024"
for rep in 1 2 3; do for v in base 8 40; do
  L=""; [ $v != base ] && L=$PWD/ab/libflexpai_ab$v.so
  FLEXPAI_LIB=$L timeout -k 10 240 python -u bench.py $B > $O/${T}_fbsab_${v}_$rep.log 2>&1 || { echo "ab $v failed"; tail -5 $O/${T}_fbsab_${v}_$rep.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], round(d['value']/1e6,3), round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3), d['extra']['roundtrip_exact'])" $O/${T}_fbsab_${v}_$rep.log $v $rep
done; done
echo ALLDONE
