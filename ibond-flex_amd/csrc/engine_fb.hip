// Fixed-base obfuscation kernels (kernels_fb.hpp): instantiations and launches.
#include "engine_fb.hpp"
#ifndef FLEXPAI_XCHECK
#define FLEXPAI_XCHECK 0   // 1: the test-only library (flexpai.hip: xcheck_env)
#endif

namespace fpai {

#if FLEXPAI_XCHECK
int fb_occupancy(int sb, int* occ_fb, int* occ_fin) {
  hipError_t e1, e2;
  if (sb == 37) {
    e1 = hipOccupancyMaxActiveBlocksPerMultiprocessor(occ_fb, k_fb<37>, LANE_BLOCK, 0);
    e2 = hipOccupancyMaxActiveBlocksPerMultiprocessor(occ_fin, k_fb_fin<37>, LANE_BLOCK, 0);
  } else if (sb == 74) {
    e1 = hipOccupancyMaxActiveBlocksPerMultiprocessor(occ_fb, k_fb<74>, LANE_BLOCK, 0);
    e2 = hipOccupancyMaxActiveBlocksPerMultiprocessor(occ_fin, k_fb_fin<74>, LANE_BLOCK, 0);
  } else {
    return -1;
  }
  if (e1 != hipSuccess || *occ_fb < 1) *occ_fb = 1;
  if (e2 != hipSuccess || *occ_fin < 1) *occ_fin = 1;
  return 0;
}
#endif

#if FLEXPAI_XCHECK
hipError_t fb_launch(int sb, const FbParams& p, int gx, hipStream_t st) {
  if (sb == 37) hipLaunchKernelGGL(k_fb<37>, dim3(gx, 2), dim3(LANE_BLOCK), 0, st, p);
  else if (sb == 74) hipLaunchKernelGGL(k_fb<74>, dim3(gx, 2), dim3(LANE_BLOCK), 0, st, p);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}
#endif

hipError_t fb_launch_digits(const FbDigitParams& p, int gx, hipStream_t st) {
  const int rw = (p.raw_bits + 31) / 32;
  if (rw + 3 <= 21) hipLaunchKernelGGL(k_fb_digits<21>, dim3(gx, 2), dim3(FB_DIG_BLOCK), 0, st, p);
  else if (rw + 3 <= 37) hipLaunchKernelGGL(k_fb_digits<37>, dim3(gx, 2), dim3(FB_DIG_BLOCK), 0, st, p);
  else if (rw + 3 <= 69) hipLaunchKernelGGL(k_fb_digits<69>, dim3(gx, 2), dim3(FB_DIG_BLOCK), 0, st, p);
  else hipLaunchKernelGGL(k_fb_digits<FB_RAW_MAX + 3>, dim3(gx, 2), dim3(FB_DIG_BLOCK), 0, st, p);
  return hipGetLastError();
}

#if FLEXPAI_XCHECK
hipError_t fb_launch_fin(int sb, const FbFinParams& p, int gx, hipStream_t st) {
  if (sb == 37) hipLaunchKernelGGL(k_fb_fin<37>, dim3(gx), dim3(LANE_BLOCK), 0, st, p);
  else if (sb == 74) hipLaunchKernelGGL(k_fb_fin<74>, dim3(gx), dim3(LANE_BLOCK), 0, st, p);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}
#endif

#if FLEXPAI_XCHECK
hipError_t fb_build_tables(int sb, const FbHalf* d_halves, uint4* t0, uint4* t1, int K, int W, hipStream_t st) {
  const int per = ((1 << W) + LANE_BLOCK - 1) / LANE_BLOCK;
  if (sb == 37) {
    hipLaunchKernelGGL(k_fb_lohi<37>, dim3(K, 2), dim3(LANE_BLOCK), 0, st, d_halves, K, W);
    hipLaunchKernelGGL(k_fb_fill<37>, dim3(K * per, 2), dim3(LANE_BLOCK), 0, st, d_halves, K, W, t0, t1);
  } else if (sb == 74) {
    hipLaunchKernelGGL(k_fb_lohi<74>, dim3(K, 2), dim3(LANE_BLOCK), 0, st, d_halves, K, W);
    hipLaunchKernelGGL(k_fb_fill<74>, dim3(K * per, 2), dim3(LANE_BLOCK), 0, st, d_halves, K, W, t0, t1);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
#endif

}  // namespace fpai
