// Host interface of the public-key fixed-base unit (engine_pfb.hip, kernels_pfb.hpp).
#pragma once
#include "kernels_pfb.hpp"

namespace fpai {

int pfb_occupancy(int* occ);
// per-key construction: chain (bases), lohi, the inversion's forward pass | host inverts the chain products
// (FbgpHalf::cval) | backward pass, fill
hipError_t pfb_build_phase1(const PfbConst* d_c, int nbases, int K, int W, hipStream_t st);
hipError_t pfb_build_phase2(const PfbConst* d_c, int K, int W, uint4* table, hipStream_t st);
hipError_t pfb_launch_digits(const PfbDigitParams& p, int gx, hipStream_t st);
hipError_t pfb_launch(const PfbParams& p, int gx, hipStream_t st);

}  // namespace fpai
