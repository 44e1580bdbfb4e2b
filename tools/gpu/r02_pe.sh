#!/bin/bash
# Public-key encryption on split pairs: parity tests, then the bench's public-key leg.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_pe.py tests/test_gpu_dec4.py tests/test_gpu_crt.py tests/test_gpu_pair_paths.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_pe.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|ERROR|Error" $O/pytest_pe.log | tail -15
[ $rc -ne 0 ] && { tail -50 $O/pytest_pe.log; exit 1; }
timeout -k 10 500 python -u bench.py --steps 3 --no-cpu-baseline --no-host --no-add8 > $O/bench_pe.log 2>&1 || { echo "bench failed rc=$?"; tail -20 $O/bench_pe.log; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_pe.log').read().strip().splitlines()[-1]); e=d['extra']; print(d['value'], e.get('public_key_path'), e.get('decrypt_per_s_per_gpu'))"
echo ALLDONE
