# Round-6 final library, part A: tests, smoke, kernel statistics and the PMC traffic passes (separate FETCH_SIZE /
# WRITE_SIZE runs, --kernel-trace only) for configs[1] (k_fbs) and configs[4] (k_sgs).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
T=r06_final
timeout -k 10 300 python -u -m pytest tests/test_gpu_guard.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/${T}_guard.log 2>&1 || { echo "guard failed"; tail -30 $O/${T}_guard.log; exit 1; }
tail -1 $O/${T}_guard.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/${T}_pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/${T}_pytest_gpu.log | head; tail -30 $O/${T}_pytest_gpu.log; exit 1; }
tail -1 $O/${T}_pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/${T}_smoke.log; exit 1; }
tail -1 $O/${T}_smoke.log
PA="--steps 5 --warmup 2 --no-cpu-baseline --no-host --no-public --no-add8 --no-strong --no-contention --no-nb1024"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof -o run -- python3 bench.py $PA > $O/${T}_prof.log 2>&1 || { echo "prof failed"; tail -20 $O/${T}_prof.log; exit 1; }
head -8 $O/${T}_prof/run_kernel_stats.csv | cut -c1-140
MA="--steps 1 --warmup 0 --no-cpu-baseline --no-decrypt --no-host --no-public --no-add8 --no-strong --no-contention --no-nb1024"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/${T}_pmc_$c -o run -- python3 bench.py $MA > $O/${T}_pmc_$c.log 2>&1 || { echo "pmc $c failed"; tail -5 $O/${T}_pmc_$c.log; exit 1; }
  echo "pmc $c done"
done
MC="--config 4 --steps 1 --warmup 0 --no-cpu-baseline --no-decrypt --no-host --no-public"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/${T}_pmc4_$c -o run -- python3 bench.py $MC > $O/${T}_pmc4_$c.log 2>&1 || { echo "pmc4 $c failed"; tail -5 $O/${T}_pmc4_$c.log; exit 1; }
  echo "pmc4 $c done"
done
echo ALLDONE
