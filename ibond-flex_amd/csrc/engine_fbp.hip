// Pair fixed-base kernels (kernels_fbp.hpp): instantiations and launches.
#include "engine_fbp.hpp"
#ifndef FLEXPAI_XCHECK
#define FLEXPAI_XCHECK 0   // 1: the test-only library (flexpai.hip: xcheck_env)
#endif

namespace fpai {

#if FLEXPAI_XCHECK
int fbp_occupancy(int s, int* occ) {
  hipError_t e;
  if (s == 19) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(occ, k_fbp<19>, LANE_BLOCK, 0);
  else if (s == 37) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(occ, k_fbp<37>, LANE_BLOCK, 0);
  else return -1;
  if (e != hipSuccess || *occ < 1) *occ = 1;
  return 0;
}
#endif

#if FLEXPAI_XCHECK
hipError_t fbp_launch(int s, const FbpParams& p, int gx, hipStream_t st) {
  if (s == 19) hipLaunchKernelGGL(k_fbp<19>, dim3(gx, 2), dim3(LANE_BLOCK), 0, st, p);
  else if (s == 37) hipLaunchKernelGGL(k_fbp<37>, dim3(gx, 2), dim3(LANE_BLOCK), 0, st, p);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}
#endif

int fbp_fin_occupancy(int s, int* occ) {
  hipError_t e;
  if (s == 19) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(occ, k_fbp_fin<19>, LANE_BLOCK, 0);
  else if (s == 37) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(occ, k_fbp_fin<37>, LANE_BLOCK, 0);
  else return -1;
  if (e != hipSuccess || *occ < 1) *occ = 1;
  return 0;
}

hipError_t fbp_launch_fin(int s, const FbpFinParams& p, int gx, hipStream_t st) {
  if (s == 19) hipLaunchKernelGGL(k_fbp_fin<19>, dim3(gx), dim3(LANE_BLOCK), 0, st, p);
  else if (s == 37) hipLaunchKernelGGL(k_fbp_fin<37>, dim3(gx), dim3(LANE_BLOCK), 0, st, p);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

// table construction, phase 1: lo/hi half-digit powers, then the forward pass of the batch inversion (the chain
// products land in FbpHalf::cval for the host's inversion)
hipError_t fbp_build_phase1(int s, const FbpHalf* d_halves, int K, int W, hipStream_t st) {
  const dim3 ig((2 * K + 63) / 64, 2);
  if (s == 19) {
    hipLaunchKernelGGL(k_fbp_lohi<19>, dim3(K, 2), dim3(LANE_BLOCK), 0, st, d_halves, K, W);
    hipLaunchKernelGGL(k_fbp_inv_fwd<19>, ig, dim3(64), 0, st, d_halves, K, W);
  } else if (s == 37) {
    hipLaunchKernelGGL(k_fbp_lohi<37>, dim3(K, 2), dim3(LANE_BLOCK), 0, st, d_halves, K, W);
    hipLaunchKernelGGL(k_fbp_inv_fwd<37>, ig, dim3(64), 0, st, d_halves, K, W);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// phase 2 (after the host wrote the chain inverses): the inverse tables, then the factored rows
#if FLEXPAI_XCHECK
hipError_t fbp_build_phase2(int s, const FbpHalf* d_halves, uint4* t0, uint4* t1, int K, int W, hipStream_t st) {
  const int per = ((1 << W) + LANE_BLOCK - 1) / LANE_BLOCK;
  const dim3 ig((2 * K + 63) / 64, 2);
  if (s == 19) {
    hipLaunchKernelGGL(k_fbp_inv_bwd<19>, ig, dim3(64), 0, st, d_halves, K, W);
    hipLaunchKernelGGL(k_fbp_fill<19>, dim3(K * per, 2), dim3(LANE_BLOCK), 0, st, d_halves, K, W, t0, t1);
  } else if (s == 37) {
    hipLaunchKernelGGL(k_fbp_inv_bwd<37>, ig, dim3(64), 0, st, d_halves, K, W);
    hipLaunchKernelGGL(k_fbp_fill<37>, dim3(K * per, 2), dim3(LANE_BLOCK), 0, st, d_halves, K, W, t0, t1);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
#endif

}  // namespace fpai
