// Host interface of the 16-lane-row CRT encryption translation unit (engine_crtw.hip).
#pragma once
#include <algorithm>

#include "kernels_crtw.hpp"

namespace fpai {

// k_crt_w<sa, 2 sa> (sa = 19, 37, 74) over p.n elements, both halves (grid blocks x 2); hipErrorInvalidValue for other sizes
hipError_t crtw_launch(int sa, const crtw::Params& p, hipStream_t st);
// k_dec_w<sa, 2 sa>: the pairs k_dec_fin_pair takes, for p.n elements, both halves
hipError_t decw_launch(int sa, const crtw::DecParams& p, hipStream_t st);
// k_pe_w<k> (k = limbs of n^2: 74, 148 or 296) over p.n elements with the op list over n; hipErrorInvalidValue otherwise
hipError_t pew_launch(int k, const EncParams& p, const uint32_t* prog, int nprog, hipStream_t st);

}  // namespace fpai
