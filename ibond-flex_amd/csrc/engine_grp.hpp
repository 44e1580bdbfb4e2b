// Host interface of the group-engine key-holder translation unit (engine_grp.hip): the fixed-base sampler for keys whose p^2 exceeds one lane (nb = 4096), kernels_grp.hpp.
#pragma once
#include "kernels_grp.hpp"

namespace fpai {

constexpr int GRP_TPI = 4;                  // S = 148 limbs: p_h^2 of a 4096-bit key

int grp_occupancy(int* occ_fb);
// launches on grid (gx, 2): blockIdx.y = half
hipError_t grp_launch_fb(const FbParams& p, int gx, hipStream_t st);
hipError_t grp_launch_garner(const FbgGarnerParams& p, int gx, hipStream_t st);
hipError_t grp_launch_fin(const FbgFinParams& p, int gx, hipStream_t st);   // TPI 8 (n^2 of a 4096-bit key)
int grp_fin_occupancy(int* occ_garner, int* occ_fin);
hipError_t grp_build_tables(const FbHalf* d_halves, uint32_t* t0, uint32_t* t1, int K, int W, hipStream_t st);
size_t grp_lds_bytes();

}  // namespace fpai
