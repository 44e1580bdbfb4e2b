// Host interface of the split-pair fixed-base sampler (engine_sgp.hip, kernels_sgp.hpp).
#pragma once
#include "kernels_sgp.hpp"

namespace fpai {

int sgp_occupancy(int* occ);
// grid (gx, halves): blockIdx.y = half, SGP_PAIRS elements per block
hipError_t sgp_launch(const SgpParams& p, int gx, int halves, hipStream_t st);
// the pairs -> w_h = A + p_h B mod p_h^2 in place (k_sgp_w, the Garner kernels' input), grid (.., halves)
hipError_t sgp_launch_w(const SgpParams& p, int halves, int cus, hipStream_t st);
// Garner's last step c = w_q + q^2 h on lanes (k_sgp_fin)
hipError_t sgp_launch_fin(const SgpFinParams& p, int cus, hipStream_t st);

}  // namespace fpai
