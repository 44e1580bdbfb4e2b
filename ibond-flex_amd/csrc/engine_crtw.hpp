// Host interface of the 16-lane-row CRT encryption translation unit (engine_crtw.hip).
#pragma once
#include <algorithm>

#include "kernels_crtw.hpp"

namespace fpai {

// k_crt_w<sa, 2 sa> over p.n elements, both halves (grid blocks x 2); hipErrorInvalidValue for other sizes
hipError_t crtw_launch(int sa, const crtw::Params& p, hipStream_t st);

}  // namespace fpai
