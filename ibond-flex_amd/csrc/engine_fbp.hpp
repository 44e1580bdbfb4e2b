// Host interface of the pair fixed-base translation unit (engine_fbp.hip).
#pragma once
#include "kernels_fbp.hpp"

namespace fpai {

// blocks per CU of k_fbp<s>; -1 if s is unsupported (19: 1024-bit keys, 37: 2048-bit keys)
int fbp_occupancy(int s, int* occ);
hipError_t fbp_launch(int s, const FbpParams& p, int gx, hipStream_t st);
// blocks per CU of k_fbp_fin<s>, and its launch
int fbp_fin_occupancy(int s, int* occ);
hipError_t fbp_launch_fin(int s, const FbpFinParams& p, int gx, hipStream_t st);
// builds both halves' factored pair tables (K digit positions of W bits) on `st`, in two phases around the host's
// inversion of the chain products (FbpHalf::cval, pair_host_invert)
hipError_t fbp_build_phase1(int s, const FbpHalf* d_halves, int K, int W, hipStream_t st);
hipError_t fbp_build_phase2(int s, const FbpHalf* d_halves, uint4* t0, uint4* t1, int K, int W, hipStream_t st);

}  // namespace fpai
