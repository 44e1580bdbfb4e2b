// Host interface of the group-engine Garner translation unit (engine_grp.hip, kernels_grp.hpp): the recombination of the
// 4096-bit key holder's halves.
#pragma once
#include "kernels_grp.hpp"

namespace fpai {

constexpr int GRP_TPI = 4;                  // S = 148 limbs: p_h^2 of a 4096-bit key

hipError_t grp_launch_garner(const FbgGarnerParams& p, int gx, hipStream_t st);
hipError_t grp_launch_fin(const FbgFinParams& p, int gx, hipStream_t st);   // TPI 8 (n^2 of a 4096-bit key)
int grp_fin_occupancy(int* occ_garner, int* occ_fin);
size_t grp_lds_bytes();

}  // namespace fpai
