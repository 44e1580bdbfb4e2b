#!/bin/bash
# Digit-fusion A/B of k_fbs: a measurement-only library next to the product -- flexpai.hip,
# engine_fbs.hip and engine_fbp.hip recompiled under FBS_AB = 4 (k_fbs draws its own exponent digits in a prologue,
# no k_fb_digits launch; kernels_fbs.hpp) -- into ab/libflexpai_abD.so. Run on the CPU:
#     bash tools/ab_fbs_digits.sh
# then on the GPU box: bash tools/gpu/ab_fbs_digits_run.sh (bench.py with FLEXPAI_LIB=ab/..., same box, interleaved).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
cd "$R"
python -c "import __graft_entry__ as g; g.build_native()"
mkdir -p ab build/ab
OBJS=$(ls build/obj/*.o | grep -v -E '/(flexpai|engine_fbs|engine_fbp)\.o$')
for u in flexpai engine_fbs engine_fbp; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c -DFBS_AB=4 -I include -I build/gmpinc ibond-flex_amd/csrc/$u.hip -o build/ab/${u}_abD.o &
done
wait
hipcc --offload-arch=gfx950 -shared -fPIC $OBJS build/ab/flexpai_abD.o build/ab/engine_fbs_abD.o build/ab/engine_fbp_abD.o \
  /usr/lib/x86_64-linux-gnu/libgmp.so.10 -o ab/libflexpai_abD.so
ls -la ab/libflexpai_abD.so
