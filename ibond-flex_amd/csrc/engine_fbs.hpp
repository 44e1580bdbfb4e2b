// Host interface of the Shoup-row fixed-base translation unit (engine_fbs.hip).
#pragma once
#include "kernels_fbs.hpp"

namespace fpai {

// bytes of one Shoup row (kernels_fbs.hpp, fbs_row_quads): 448 at s = 37, 224 at s = 19; 0 if s is unsupported
int fbs_row_bytes(int s);
// blocks per CU of k_fbs<s>; -1 if s is unsupported
int fbs_occupancy(int s, int* occ);
// k_fbs<s> over grid (gx, 2): LANE_BLOCK / 2 elements per block and sweep
hipError_t fbs_launch(int s, const FbpParams& p, int gx, hipStream_t st);
// phase 2 of the table construction for Shoup rows (after the host wrote the chain inverses): the inverse tables
// (k_fbp_inv_bwd), then the rows (k_fbs_fill); cst: device array of the two halves' FbsConst; g: the address guard (guard.hpp)
hipError_t fbs_build_phase2(int s, const FbpHalf* d_halves, const FbsConst* cst, uint4* t0, uint4* t1, int K, int W,
                            hipStream_t st, const GuardArgs& g);

}  // namespace fpai
