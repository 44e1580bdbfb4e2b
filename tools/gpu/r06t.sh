set -o pipefail
O=gpurun_out; mkdir -p $O
FLEXPAI_LIB=$PWD/ab/libflexpai_crta2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_crt.py tests/test_gpu_crt_rows.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/r06t_tests.log 2>&1 || { echo "tests failed"; tail -20 $O/r06t_tests.log; exit 1; }
tail -1 $O/r06t_tests.log
for rep in 1 2 3; do for v in base crta2; do
  L=""; [ $v = crta2 ] && L=$PWD/ab/libflexpai_crta2.so
  FLEXPAI_LIB=$L timeout -k 10 200 python -u tools/gpu/crt_rate.py > $O/r06t_${v}_$rep.log 2>&1 || { echo "$v failed"; tail -5 $O/r06t_${v}_$rep.log; exit 1; }
  grep '^{' $O/r06t_${v}_$rep.log
done; done
echo ALLDONE
