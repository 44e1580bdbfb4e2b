// Host interface of the split-pair fixed-base sampler (engine_sgp.hip, kernels_sgp.hpp).
#pragma once
#include "kernels_sgp.hpp"

namespace fpai {

int sgp_occupancy(int* occ);
// grid (gx, halves): blockIdx.y = half, SGP_PAIRS elements per block
hipError_t sgp_launch(const SgpParams& p, int gx, int halves, hipStream_t st);

}  // namespace fpai
