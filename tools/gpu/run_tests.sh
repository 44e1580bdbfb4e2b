#!/bin/bash
# GPU parity tests only (optionally a subset: TESTS="tests/test_x.py ..."), one process.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR" $O/pytest_gpu.log | tail -40
tail -30 $O/pytest_gpu.log | grep -v PASSED
exit $rc
