// Types of the lane-engine decryption (kernels_dec.hpp): the 2S-limb lane kernels k_dec_pre/pow/fin were retired in
// round 6 (the pair kernels, engine_pair.hip, decrypt 1024/2048-bit keys; the group engine the rest).
#pragma once
#include <algorithm>

#include "kernels_dec.hpp"

namespace fpai {

struct DecLaneGeom {          // launch geometry of a lane-engine decryption (engine_pair.hip's pair kernels)
  int gx_pre = 0;            // blocks per half for the pre kernel
  int gx_pow = 0;            // blocks per half for the exponentiation (resident lanes: the tiles are per lane)
  int gx_fin = 0;            // blocks for the fin kernel
  size_t scratch_bytes = 0;  // per-lane tiles of the exponentiation
};

}  // namespace fpai
