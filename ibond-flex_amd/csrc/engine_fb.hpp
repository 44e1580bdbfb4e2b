// Host interface of the fixed-base obfuscation translation unit (engine_fb.hip): the exponent digits.
#pragma once
#include "kernels_fb.hpp"

namespace fpai {

hipError_t fb_launch_digits(const FbDigitParams& p, int gx, hipStream_t st);

}  // namespace fpai
