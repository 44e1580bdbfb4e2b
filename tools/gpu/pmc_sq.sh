#!/bin/bash
# SQ issue/stall counters and the effective clock of the encrypt + decrypt kernels (one rep of
# tools/gpu/stage_times.py per counter pass).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
           "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  REPS=1 timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/pmcsq_$i -o run -- python3 $R/tools/gpu/stage_times.py > $O/pmcsq_$i.log 2>&1 || { echo "pass $i failed"; tail -20 $O/pmcsq_$i.log; exit 1; }
done
echo ALLDONE
