// Host interface of the 1024-bit public-key pair encryption translation unit (engine_pe1.hip, kernels_pe1.hpp).
#pragma once
#include <algorithm>

#include "kernels_pe1.hpp"

namespace fpai {

constexpr int PE1_S = 37;   // limbs of n (n <= 1024 bits: R = 2^1036 >= 2^12 n)
// blocks per CU of k_pe1_pow
int pe1_occupancy(int* occ);
// k_pe1_words, k_dec_pre_pair<37> (pre: one half, n in place of p_h), k_pe1_pow (grid gx), k_pe1_fin on `st`;
// ev[0..3] (nullable) recorded before the words and after the pre, the chain and the finish
hipError_t pe1_launch(const Pe1Params& p, const DecPairPreParams& pre, int gx, int cus, hipStream_t st, hipEvent_t* ev);

}  // namespace fpai
