set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
FLEXPAI_LIB=$R/ibond-flex_amd/flex/crypto/paillier/_native/libflexpai_occ2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_dec_lane.py tests/test_gpu_crt.py tests/test_gpu_pair_paths.py -x -q --timeout 300 --timeout-method thread > $O/pytest_occ2.log 2>&1 || { echo "pytest failed"; tail -20 $O/pytest_occ2.log; exit 1; }
tail -2 $O/pytest_occ2.log
for L in libflexpai.so libflexpai_occ2.so libflexpai.so libflexpai_occ2.so; do
FLEXPAI_LIB=$R/ibond-flex_amd/flex/crypto/paillier/_native/$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-host --no-strong --no-public > $O/bench_$L.log 2>&1 || { echo "bench failed $L"; tail -20 $O/bench_$L.log; exit 1; }
tail -1 $O/bench_$L.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']; print('$L', round(d['value']/1e6,2), 'dec', round(e['decrypt_per_s_per_gpu']/1e6,3), e['decrypt_kernel_ms'], 'crt', round(e['generic_crt_path']['value']/1e6,3), 'c2', round(e['config2_add8']['elements_per_s']/1e6,3))"
done
echo ALLDONE
