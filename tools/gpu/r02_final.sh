#!/bin/bash
# Round-end state: the full GPU suite, then the pair profiling script (bench lines, stats, traffic, SQ).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -4 $O/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/pytest_gpu.log | head -20; exit 1; }
bash tools/gpu/r02_profile_pair.sh
