// Host interface of the Shoup-row split-pair sampler (engine_sgs.hip, kernels_sgs.hpp; the default where it prices
// lower, flexpai.hip fb_choose).
#pragma once
#include "kernels_sgs.hpp"

namespace fpai {

int sgs_occupancy(int* occ);
// the Shoup rows of both halves from their factored rows (rows = K 2^W per half)
hipError_t sgs_launch_conv(const SgsHalf* halves, size_t rows, uint4* atab0, uint4* atab1, hipStream_t st);
// the sampler, grid (gx, halves): SGP_PAIRS elements per block
hipError_t sgs_launch(const SgsParams& p, int gx, int halves, hipStream_t st);
// the b sums applied in place: the pairs k_sgp_w / k_pe_fin take
hipError_t sgs_launch_bfin(const SgsFinParams& p, int halves, int cus, hipStream_t st);

}  // namespace fpai
