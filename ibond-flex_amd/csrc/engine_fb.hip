// Fixed-base obfuscation kernels (kernels_fb.hpp): the exponent digits' instantiations and launch (the round-1 sampler
// k_fb / k_fb_fin and its table builders were retired in round 6).
#include "engine_fb.hpp"

namespace fpai {

hipError_t fb_launch_digits(const FbDigitParams& p, int gx, hipStream_t st) {
  const int rw = (p.raw_bits + 31) / 32;
  if (rw + 3 <= 21) hipLaunchKernelGGL(k_fb_digits<21>, dim3(gx, 2), dim3(FB_DIG_BLOCK), 0, st, p);
  else if (rw + 3 <= 37) hipLaunchKernelGGL(k_fb_digits<37>, dim3(gx, 2), dim3(FB_DIG_BLOCK), 0, st, p);
  else if (rw + 3 <= 69) hipLaunchKernelGGL(k_fb_digits<69>, dim3(gx, 2), dim3(FB_DIG_BLOCK), 0, st, p);
  else hipLaunchKernelGGL(k_fb_digits<FB_RAW_MAX + 3>, dim3(gx, 2), dim3(FB_DIG_BLOCK), 0, st, p);
  return hipGetLastError();
}

}  // namespace fpai
