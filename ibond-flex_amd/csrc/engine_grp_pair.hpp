// Host interface of the pair-group sampler for 4096-bit keys (engine_grp_pair.hip, kernels_grp_pair.hpp).
#pragma once
#include "kernels_grp_pair.hpp"

namespace fpai {

int fbgp_occupancy(int* occ);
// launches on grid (gx, 2): blockIdx.y = half
hipError_t fbgp_launch(const FbgpParams& p, int gx, hipStream_t st);
hipError_t fbgp_launch_w(const FbgpParams& p, int gx, hipStream_t st);
// table construction in two phases around the host's inversion of the chain products (FbgpHalf::cval)
hipError_t fbgp_build_phase1(const FbgpHalf* d_halves, int K, int W, hipStream_t st);
hipError_t fbgp_build_phase2(const FbgpHalf* d_halves, uint32_t* t0, uint32_t* t1, int K, int W, hipStream_t st);

}  // namespace fpai
