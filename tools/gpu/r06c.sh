set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_fixed_base.py tests/test_gpu_fbs.py tests/test_gpu_sgs.py tests/test_gpu_fixed_base_4096.py tests/test_gpu_window_policy.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/r06c_pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/r06c_pytest.log; exit 1; }
tail -2 $O/r06c_pytest.log
FLEXPAI_SETUP_TRACE=1 timeout -k 10 200 python -u tools/fresh_key_trace.py --keys 3 > $O/r06c_fresh1M.log 2>&1 || { echo fresh1M failed; tail -20 $O/r06c_fresh1M.log; exit 1; }
FLEXPAI_SETUP_TRACE=1 timeout -k 10 200 python -u tools/fresh_key_trace.py --keys 3 --n 1000 > $O/r06c_fresh1k.log 2>&1 || { echo fresh1k failed; tail -20 $O/r06c_fresh1k.log; exit 1; }
grep "^key" $O/r06c_fresh1M.log $O/r06c_fresh1k.log
FLEXPAI_SETUP_TRACE=1 timeout -k 10 300 python -u tools/pfb_setup_trace.py --repeat 2 > $O/r06c_pfb.log 2>&1 || { echo pfb failed; tail -20 $O/r06c_pfb.log; exit 1; }
FLEXPAI_SETUP_TRACE=1 timeout -k 10 300 python -u tools/pfb_setup_trace.py --repeat 2 --no-holder > $O/r06c_pfb_noholder.log 2>&1 || { echo pfb2 failed; tail -20 $O/r06c_pfb_noholder.log; exit 1; }
grep -E "public tables|holder tables" $O/r06c_pfb.log $O/r06c_pfb_noholder.log
timeout -k 10 400 python -u tools/gpu/nb1024_sweep.py > $O/r06c_nb1024_sweep.log 2>&1 || { echo sweep failed; tail -20 $O/r06c_nb1024_sweep.log; exit 1; }
cat $O/r06c_nb1024_sweep.log | grep window_requested
echo ALLDONE
