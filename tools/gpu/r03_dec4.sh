#!/bin/bash
# 4096-bit decryption parity (split pairs) + the configs[4] bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_dec4.py tests/test_gpu_pe.py -x -q --timeout 300 --timeout-method thread > $O/pytest_dec4.log 2>&1; rc=$?
tail -5 $O/pytest_dec4.log
[ $rc -ne 0 ] && { echo "pytest failed rc=$rc"; grep -E "FAILED|Error|error" $O/pytest_dec4.log | head -20; exit 1; }
timeout -k 10 600 python -u bench.py --config 4 --no-cpu-baseline ${BENCH_ARGS:-} > $O/bench_c4.log 2>&1 || { echo "bench failed rc=$?"; tail -30 $O/bench_c4.log; exit 1; }
tail -1 $O/bench_c4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']; print(d['value'], d['roofline']['kernel_ms'], d['roofline']['frac']); print({k: e[k] for k in ('decrypt_per_s_per_gpu','decrypt_kernel_ms','decrypt_int_mac_frac','roundtrip_exact') if k in e})"
echo ALLDONE
