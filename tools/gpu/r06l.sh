set -o pipefail
O=gpurun_out; mkdir -p $O
T=r06l
timeout -k 10 300 python -u -m pytest tests/test_gpu_crt_rows.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/${T}_rows_tests.log 2>&1 || { echo "rows tests failed"; grep -E "FAILED|Error|assert" $O/${T}_rows_tests.log | head -20; tail -30 $O/${T}_rows_tests.log; exit 1; }
tail -1 $O/${T}_rows_tests.log
timeout -k 10 300 python -u tools/gpu/latency_1k.py > $O/${T}_latency.log 2>&1 || { echo "latency failed"; tail -20 $O/${T}_latency.log; exit 1; }
grep '^{' $O/${T}_latency.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/${T}_pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/${T}_pytest_gpu.log | head; tail -30 $O/${T}_pytest_gpu.log; exit 1; }
tail -1 $O/${T}_pytest_gpu.log
echo ALLDONE
