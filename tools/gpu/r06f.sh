set -o pipefail
O=gpurun_out; mkdir -p $O
T=r06f
timeout -k 10 300 python -u -m pytest tests/test_gpu_crt_rows.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/${T}_rows_tests.log 2>&1 || { echo "rows tests failed"; tail -40 $O/${T}_rows_tests.log; exit 1; }
tail -1 $O/${T}_rows_tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_crt.py tests/test_gpu_guard.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/${T}_crt_tests.log 2>&1 || { echo "crt tests failed"; tail -30 $O/${T}_crt_tests.log; exit 1; }
tail -1 $O/${T}_crt_tests.log
timeout -k 10 300 python -u tools/gpu/crt_rows_sweep.py --nb 2048 > $O/${T}_sweep2048.log 2>&1 || { echo "sweep failed"; tail -20 $O/${T}_sweep2048.log; exit 1; }
cat $O/${T}_sweep2048.log | grep '^{'
timeout -k 10 300 python -u tools/gpu/crt_rows_sweep.py --nb 1024 > $O/${T}_sweep1024.log 2>&1 || { echo "sweep1024 failed"; tail -20 $O/${T}_sweep1024.log; exit 1; }
cat $O/${T}_sweep1024.log | grep '^{'
timeout -k 10 300 python -u tools/fresh_key_trace.py --keys 3 --n 1000 > $O/${T}_fresh1k.log 2>&1 || { echo "fresh failed"; tail -20 $O/${T}_fresh1k.log; exit 1; }
grep "^key" $O/${T}_fresh1k.log
timeout -k 10 300 python -u tools/fresh_key_trace.py --keys 3 --n 1000 --nb 1024 > $O/${T}_fresh1k_1024.log 2>&1 || { echo "fresh1024 failed"; exit 1; }
grep "^key" $O/${T}_fresh1k_1024.log
echo ALLDONE
