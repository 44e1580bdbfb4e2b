# Round-6 final library, part B: the bench lines (with roofline.traffic from part A's PMC files of this binary).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
T=r06_final
timeout -k 10 600 python -u bench.py > $O/${T}_bench.log 2>&1 || { echo "bench failed"; tail -30 $O/${T}_bench.log; exit 1; }
tail -1 $O/${T}_bench.log | cut -c1-300
timeout -k 10 600 python -u bench.py --config 4 > $O/${T}_bench_config4.log 2>&1 || { echo "bench c4 failed"; tail -30 $O/${T}_bench_config4.log; exit 1; }
tail -1 $O/${T}_bench_config4.log | cut -c1-300
timeout -k 10 300 python -u bench.py --config 0 > $O/${T}_bench_config0.log 2>&1 || { echo "bench c0 failed"; tail -30 $O/${T}_bench_config0.log; exit 1; }
tail -1 $O/${T}_bench_config0.log | cut -c1-300
echo ALLDONE
