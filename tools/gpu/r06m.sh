set -o pipefail
O=gpurun_out; mkdir -p $O
T=r06m
timeout -k 10 300 python -u -m pytest tests/test_gpu_guard.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/${T}_guard.log 2>&1 || { echo "guard failed"; tail -30 $O/${T}_guard.log; exit 1; }
tail -1 $O/${T}_guard.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/${T}_pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/${T}_pytest_gpu.log | head; tail -30 $O/${T}_pytest_gpu.log; exit 1; }
tail -1 $O/${T}_pytest_gpu.log
echo ALLDONE
