# one-off (round 4): signed-MAC rate, Shoup rows with unsigned step 2, SQ counters of k_fbs against k_fbp
set -o pipefail
timeout -k 10 120 tools/microbench/int_throughput > gpurun_out/r04d_int_throughput.txt 2>&1 || exit 1
grep -E "mad|fma_f32" gpurun_out/r04d_int_throughput.txt
export TAG=r04d TESTS="tests/test_gpu_fbs.py" NO_BENCH=1
bash tools/gpu/suite.sh || exit 1
export NO_TESTS=1
FLEXPAI_FBS=1 TAG=r04d_fbs PROF=1 PMC="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY GRBM_GUI_ACTIVE" bash tools/gpu/suite.sh || exit 1
TAG=r04d_fbp PMC="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY GRBM_GUI_ACTIVE" bash tools/gpu/suite.sh || exit 1
