set -o pipefail
O=gpurun_out; mkdir -p $O
T=r06i
timeout -k 10 300 python -u -m pytest tests/test_gpu_crt_rows.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/${T}_rows_tests.log 2>&1 || { echo "rows tests failed"; tail -40 $O/${T}_rows_tests.log; exit 1; }
tail -1 $O/${T}_rows_tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_dec_lane.py tests/test_gpu_crt.py tests/test_gpu_engine.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/${T}_dec_tests.log 2>&1 || { echo "dec tests failed"; tail -30 $O/${T}_dec_tests.log; exit 1; }
tail -1 $O/${T}_dec_tests.log
timeout -k 10 300 python -u tools/gpu/crt_rows_sweep.py --nb 2048 --sizes 256,1024,2048,4096,8192 > $O/${T}_sweep2048.log 2>&1 || { echo "sweep failed"; tail -20 $O/${T}_sweep2048.log; exit 1; }
grep '^{' $O/${T}_sweep2048.log
timeout -k 10 300 python -u tools/gpu/crt_rows_sweep.py --nb 1024 --sizes 256,1024,4096,8192 > $O/${T}_sweep1024.log 2>&1 || { echo "sweep1024 failed"; tail -20 $O/${T}_sweep1024.log; exit 1; }
grep '^{' $O/${T}_sweep1024.log
echo ALLDONE
