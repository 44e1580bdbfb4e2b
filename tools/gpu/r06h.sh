set -o pipefail
O=gpurun_out; mkdir -p $O
T=r06h
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in bfin1s bfin2s; do
  FLEXPAI_LIB=$PWD/ab/libflexpai_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_sgs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/${T}_${v}_tests.log 2>&1 || { echo "$v tests failed"; tail -20 $O/${T}_${v}_tests.log; exit 1; }
  tail -1 $O/${T}_${v}_tests.log
done
B="--config 4 --steps 2 --warmup 1 --no-cpu-baseline --no-host --no-public --no-decrypt"
for v in prefold bfin1s bfin2s; do
  FLEXPAI_LIB=$PWD/ab/libflexpai_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof_$v -o run -- python3 bench.py $B > $O/${T}_prof_$v.log 2>&1 || { echo "prof $v failed"; tail -5 $O/${T}_prof_$v.log; exit 1; }
  python3 -c "
import csv,glob,sys
f=glob.glob('$O/${T}_prof_$v/**/run_kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
  n=r['Name']
  if 'sgs' in n or 'sgp' in n or 'fbg' in n: print('$v', n[:40], r['Calls'], round(float(r['AverageNs'])/1e6,3))
"
done
B="--config 4 --steps 3 --warmup 1 --no-cpu-baseline --no-host --no-public --no-decrypt"
for rep in 1 2; do for v in prefold bfin1s bfin2s; do
  FLEXPAI_LIB=$PWD/ab/libflexpai_$v.so timeout -k 10 240 python -u bench.py $B > $O/${T}_c4ab_${v}_$rep.log 2>&1 || { echo "c4 ab $v failed"; tail -5 $O/${T}_c4ab_${v}_$rep.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e=d['extra']; print(sys.argv[2], sys.argv[3], round(d['value']/1e6,3), round(d['ms_per_step'],2), {k:round(v['kernel_ms'],2) for k,v in e['stages'].items()})" $O/${T}_c4ab_${v}_$rep.log $v $rep
done; done
echo ALLDONE
