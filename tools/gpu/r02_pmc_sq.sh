#!/bin/bash
# SQ issue/stall counters of the round-2 kernels: configs[2] (k_fb, k_fb_fin, k_add, decrypt) and configs[4]
# (k_fbg, k_crt_fin<8>), one counter pass each (7 SQ + 1 GRBM counters: within one pass's limits).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
SET="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE"
timeout -s KILL 240 rocprofv3 --pmc $SET --kernel-trace --output-format csv -d $O/sq_c2 -o run -- python3 $R/bench.py --config 2 --steps 1 --warmup 0 --no-cpu-baseline --no-public > $O/sq_c2.log 2>&1 || { echo "sq c2 failed rc=$?"; tail -20 $O/sq_c2.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc $SET --kernel-trace --output-format csv -d $O/sq_c4 -o run -- python3 $R/bench.py --config 4 --steps 1 --warmup 0 --no-cpu-baseline --no-decrypt --no-public > $O/sq_c4.log 2>&1 || { echo "sq c4 failed rc=$?"; tail -20 $O/sq_c4.log; exit 1; }
cd $R
python3 tools/pmc_sq_summary.py $O/sq_c2/run_counter_collection.csv $O/sq_c4/run_counter_collection.csv > $O/r02_pmc_sq.txt || exit 1
cat $O/r02_pmc_sq.txt
echo ALLDONE
