set -o pipefail
export TMPDIR=/tmp
TAG=r04c TESTS="tests/test_gpu_fbs.py tests/test_gpu_full_size.py::test_config3_full_size_sharded" NO_BENCH=1 bash tools/gpu/suite.sh || exit 1
BA="--steps 5 --warmup 2 --no-cpu-baseline --no-public --no-add8 --no-host --no-strong"
export FLEXPAI_FBS=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04c_prof_fbs -o run -- python bench.py $BA > gpurun_out/r04c_bench_fbs.log 2>&1 || { echo "fbs bench rc=$?"; tail -20 gpurun_out/r04c_bench_fbs.log; exit 1; }
tail -1 gpurun_out/r04c_bench_fbs.log | cut -c1-600
unset FLEXPAI_FBS
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04c_prof_fbp -o run -- python bench.py $BA > gpurun_out/r04c_bench_fbp.log 2>&1 || { echo "fbp bench rc=$?"; tail -20 gpurun_out/r04c_bench_fbp.log; exit 1; }
tail -1 gpurun_out/r04c_bench_fbp.log | cut -c1-600
echo ALLDONE
