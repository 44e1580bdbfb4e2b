#!/bin/bash
# Row-layout A/B of k_fbs: builds three measurement-only libraries next to the product --
# the product's objects with engine_fbs.hip recompiled under FBS_AB = 1 (T: 384-B row stride, three-line rows, the
# bytes of packed rows), 2 (I: + v_alignbit/v_and per a and a' digit, the instructions of packed rows) and 3 (both:
# packed 384-B rows without the periodic reductions R' = 2^1024 would also need) -- into ab/. Run on the CPU:
#     bash tools/ab_fbs_rows.sh
# then on the GPU box: bash tools/gpu/ab_fbs_rows_run.sh (bench.py with FLEXPAI_LIB=ab/..., same box, interleaved).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
cd "$R"
python -c "import __graft_entry__ as g; g.build_native()"
mkdir -p ab build/ab
OBJS=$(ls build/obj/*.o | grep -v '/engine_fbs.o$')
for v in 1 2 3; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c -DFBS_AB=$v -I include -I build/gmpinc ibond-flex_amd/csrc/engine_fbs.hip -o build/ab/engine_fbs_ab$v.o &
done
wait
for v in 1 2 3; do
  hipcc --offload-arch=gfx950 -shared -fPIC $OBJS build/ab/engine_fbs_ab$v.o /usr/lib/x86_64-linux-gnu/libgmp.so.10 -o ab/libflexpai_ab$v.so
done
ls -la ab/
