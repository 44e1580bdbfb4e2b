set -o pipefail
O=gpurun_out; mkdir -p $O
T=r06q
timeout -k 10 400 python -u -m pytest tests/test_gpu_pe1.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/${T}_pe1_tests.log 2>&1 || { echo "pe1 tests failed"; grep -E "FAILED|Error|assert" $O/${T}_pe1_tests.log | head -20; tail -30 $O/${T}_pe1_tests.log; exit 1; }
tail -1 $O/${T}_pe1_tests.log
timeout -k 10 300 python -u tools/gpu/pe1_rate.py > $O/${T}_pe1_rate.log 2>&1 || { echo "rate failed"; tail -20 $O/${T}_pe1_rate.log; exit 1; }
grep '^{' $O/${T}_pe1_rate.log
echo ALLDONE
