// Host interface of the fixed-base obfuscation translation unit (engine_fb.hip).
#pragma once
#include "kernels_fb.hpp"

namespace fpai {

// blocks per CU of k_fb<sb> and k_fb_fin<sb>; -1 if sb is unsupported (37: 1024-bit keys, 74: 2048-bit keys)
int fb_occupancy(int sb, int* occ_fb, int* occ_fin);
hipError_t fb_launch(int sb, const FbParams& p, int gx, hipStream_t st);
hipError_t fb_launch_digits(const FbDigitParams& p, int gx, hipStream_t st);
hipError_t fb_launch_fin(int sb, const FbFinParams& p, int gx, hipStream_t st);
// builds both halves' tables (K digit positions of W bits) on `st`
hipError_t fb_build_tables(int sb, const FbHalf* d_halves, uint4* t0, uint4* t1, int K, int W, hipStream_t st);

}  // namespace fpai
