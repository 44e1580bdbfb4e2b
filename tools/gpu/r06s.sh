set -o pipefail
O=gpurun_out; mkdir -p $O
FLEXPAI_LIB=$PWD/ab/libflexpai_fbs19o4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fbs.py tests/test_gpu_fixed_base.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/r06s_o4_tests.log 2>&1 || { echo "o4 tests failed"; tail -20 $O/r06s_o4_tests.log; exit 1; }
tail -1 $O/r06s_o4_tests.log
for rep in 1 2 3; do for v in base o4; do
  L=""; [ $v = o4 ] && L=$PWD/ab/libflexpai_fbs19o4.so
  FLEXPAI_LIB=$L timeout -k 10 300 python -u tools/gpu/nb1024_sweep.py --windows 23 > $O/r06s_${v}_$rep.log 2>&1 || { echo "$v failed"; tail -5 $O/r06s_${v}_$rep.log; exit 1; }
  echo "$v $rep $(grep '^{' $O/r06s_${v}_$rep.log)"
done; done
echo ALLDONE
