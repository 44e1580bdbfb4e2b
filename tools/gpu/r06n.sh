set -o pipefail
O=gpurun_out; mkdir -p $O
T=r06n
timeout -k 10 400 python -u -m pytest tests/test_gpu_crt_rows.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/${T}_rows_tests.log 2>&1 || { echo "rows tests failed"; grep -E "FAILED|Error|assert" $O/${T}_rows_tests.log | head -20; tail -30 $O/${T}_rows_tests.log; exit 1; }
tail -1 $O/${T}_rows_tests.log
timeout -k 10 400 python -u tools/gpu/latency_1k.py > $O/${T}_latency.log 2>&1 || { echo "latency failed"; tail -20 $O/${T}_latency.log; exit 1; }
grep '^{' $O/${T}_latency.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_dec4.py tests/test_gpu_fixed_base_4096.py tests/test_gpu_sgs.py tests/test_gpu_crt.py tests/test_gpu_engine.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/${T}_4096_tests.log 2>&1 || { echo "4096 tests failed"; grep -E "FAILED|Error" $O/${T}_4096_tests.log | head; tail -20 $O/${T}_4096_tests.log; exit 1; }
tail -1 $O/${T}_4096_tests.log
echo ALLDONE
