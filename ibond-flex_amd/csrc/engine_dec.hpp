// Host interface of the lane-engine decryption translation unit (engine_dec.hip).
#pragma once
#include <algorithm>

#include "kernels_dec.hpp"

namespace fpai {

struct DecLaneGeom {
  int gx_pre = 0;            // blocks per half for k_dec_pre
  int gx_pow = 0;            // blocks per half for k_dec_pow (resident lanes: the tiles are per lane)
  int gx_fin = 0;            // blocks for k_dec_fin
  size_t scratch_bytes = 0;  // per-lane tiles of k_dec_pow
};

// sa: lane limbs of p (19 for 1024-bit keys, 37 for 2048-bit keys); returns -1 if unsupported.
// Grid sizes are for `chunk` elements; callers clamp them to smaller chunks.
int dec_lane_geometry(int sa, int cus, long long chunk, DecLaneGeom* g);
// k_dec_pre, k_dec_pow (both halves on blockIdx.y), k_dec_fin on `st`; ev[0..3] (each nullable)
// are recorded before, between and after the kernels.
hipError_t dec_lane_launch(int sa, const DecPreParams& pre, const CrtParams& pw, const DecFinParams& f,
                           const DecLaneGeom& g, hipStream_t st, hipEvent_t* ev);

}  // namespace fpai
