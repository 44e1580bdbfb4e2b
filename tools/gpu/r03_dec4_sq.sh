#!/bin/bash
# SQ issue counters of the 4096-bit decryption kernels (tools/gpu/stage_times.py at NB = 4096, one rep).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
NB=4096 N=262144 REPS=1 timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmcsq4 -o run -- python3 $R/tools/gpu/stage_times.py > $O/pmcsq4.log 2>&1 || { echo "pmc failed rc=$?"; tail -20 $O/pmcsq4.log; exit 1; }
cd $R
python3 tools/pmc_sq_summary.py $O/pmcsq4/run_counter_collection.csv > $O/pmc_sq4_summary.txt 2>&1 || true
cat $O/pmc_sq4_summary.txt
tail -3 $O/pmcsq4.log
echo ALLDONE
