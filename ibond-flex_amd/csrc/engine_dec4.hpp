// Host interface of the 4096-bit split-pair decryption unit (engine_dec4.hip, kernels_dec4.hpp).
#pragma once
#include <algorithm>

#include "kernels_dec4.hpp"

namespace fpai {

struct Dec4Geom {
  int gx_pre = 0, gx_pow = 0, gx_L = 0, gx_fin = 0;   // blocks (per half for pre/pow/L)
  size_t lds_fin = 0;                                   // dynamic LDS of k_dec4_fin
  size_t scratch_bytes = 0;                             // per-lane tiles of k_dec4_pow
};
int dec4_geometry(int cus, long long chunk, Dec4Geom* g);
// k_dec4_pre, k_dec4_pow, k_dec4_L (halves on blockIdx.y), k_dec4_fin on `st`; ev[0..3] nullable
hipError_t dec4_launch(const Dec4Params& p, const DecParams& f, const Dec4Geom& g, hipStream_t st, hipEvent_t* ev);
// k_dec4_L + k_dec4_fin alone, on pairs another kernel left in p.x (k_dec_w<74, 148>)
hipError_t dec4_launch_tail(const Dec4Params& p, const DecParams& f, const Dec4Geom& g, hipStream_t st);

}  // namespace fpai
