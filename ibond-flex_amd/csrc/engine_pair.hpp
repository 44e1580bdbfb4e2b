// Host interface of the pair exponentiation translation unit (engine_pair.hip): lane-engine CRT decryption
// and stage B of the generic CRT encryption on p-adic pairs (kernels_pair.hpp).
#pragma once
#include <algorithm>

#include "engine_dec.hpp"
#include "kernels_pair.hpp"

namespace fpai {

// s: limbs of p_h (19 for 1024-bit keys, 37 for 2048-bit keys); -1 if unsupported. Grid sizes are for
// `chunk` elements (callers clamp them); the work buffer holds [2][2s][chunk] words.
// factored: the B-free chain (k_dec_pow_pair<s, true>, the product); false: the general chain (test build only)
int dec_pair_geometry(int s, int cus, long long chunk, DecLaneGeom* g, bool factored = true);
// k_dec_pre_pair, k_dec_pow_pair (both halves on blockIdx.y), k_dec_fin_pair on `st`; ev[0..3] nullable
hipError_t dec_pair_launch(int s, const DecPairPreParams& pre, const CrtParams& pw, const DecPairFinParams& f,
                           const DecLaneGeom& g, hipStream_t st, hipEvent_t* ev, bool factored = true);
// k_dec_fin_pair<s> alone (grid gx), for pairs another kernel produced (k_dec_w)
hipError_t dec_pair_launch_fin(int s, const DecPairFinParams& f, int gx, hipStream_t st);
// blocks per CU of k_crt_b_pair<s> (-1 if unsupported) and its launch (grid gx x 2 halves)
int crt_b_pair_occupancy(int s, int* occ);
hipError_t crt_b_pair_launch(int s, const CrtParams& p, int gx, hipStream_t st);

}  // namespace fpai
