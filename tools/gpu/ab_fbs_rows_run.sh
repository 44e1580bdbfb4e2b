#!/bin/bash
# GPU side of tools/ab_fbs_rows.sh: base / T / I / TI interleaved twice on one box (bench.py, headline config, legs off,
# no decrypt: T's ciphertexts are wrong by construction), then per variant a FETCH_SIZE pass (HBM reads of k_fbs) and a
# GRBM_GUI_ACTIVE / SQ pass (the kernel's clock and issue), each a run of its own.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab05
mkdir -p $O
export TMPDIR=/tmp
cd $R
BA="--steps 10 --warmup 2 --no-cpu-baseline --no-host --no-public --no-add8 --no-strong --no-contention --no-decrypt"
lib() { case $1 in base) echo "";; T) echo "$R/ab/libflexpai_ab1.so";; I) echo "$R/ab/libflexpai_ab2.so";; TI) echo "$R/ab/libflexpai_ab3.so";; esac; }
for rep in 1 2; do
  for v in base T I TI; do
    FLEXPAI_LIB=$(lib $v) timeout -k 10 240 python -u bench.py $BA > $O/bench_${v}_$rep.log 2>&1 || { echo "bench $v failed"; tail -5 $O/bench_${v}_$rep.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['value'], d['roofline']['kernel_ms'])" $O/bench_${v}_$rep.log $v $rep
  done
done
MA="--steps 1 --warmup 0 --no-cpu-baseline --no-decrypt --no-host --no-public --no-add8 --no-strong --no-contention"
for v in base T I TI; do
  FLEXPAI_LIB=$(lib $v) timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmcf_$v -o run -- python3 bench.py $MA > $O/pmcf_$v.log 2>&1 || { echo "pmc fetch $v failed"; tail -5 $O/pmcf_$v.log; exit 1; }
  FLEXPAI_LIB=$(lib $v) timeout -s KILL 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d $O/pmcs_$v -o run -- python3 bench.py $MA > $O/pmcs_$v.log 2>&1 || { echo "pmc sq $v failed"; tail -5 $O/pmcs_$v.log; exit 1; }
  echo "pmc $v done"
done
echo ALLDONE
