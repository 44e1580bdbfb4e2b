// Shoup-row fixed-base kernels (kernels_fbs.hpp): instantiations and launches.
#ifndef FLEXPAI_XCHECK
#define FLEXPAI_XCHECK 0   // 1: the test-only library (address guards, guard.hpp)
#endif
#include "engine_fbs.hpp"

namespace fpai {

int fbs_row_bytes(int s) {
  if (s == 19) return fbs_row_quads<19>() * 16;
  if (s == 37) return fbs_row_quads<37>() * 16;
  return 0;
}

int fbs_occupancy(int s, int* occ) {
  hipError_t e;
  if (s == 19) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(occ, k_fbs<19>, LANE_BLOCK, 0);
  else if (s == 37) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(occ, k_fbs<37>, LANE_BLOCK, 0);
  else return -1;
  if (e != hipSuccess || *occ < 1) *occ = 1;
  return 0;
}

hipError_t fbs_launch(int s, const FbpParams& p, int gx, hipStream_t st) {
  if (s == 19) hipLaunchKernelGGL(k_fbs<19>, dim3(gx, 2), dim3(LANE_BLOCK), 0, st, p);
  else if (s == 37) hipLaunchKernelGGL(k_fbs<37>, dim3(gx, 2), dim3(LANE_BLOCK), 0, st, p);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t fbs_build_phase2(int s, const FbpHalf* d_halves, const FbsConst* cst, uint4* t0, uint4* t1, int K, int W,
                            hipStream_t st, const GuardArgs& g) {
  const int per = ((1 << W) + LANE_BLOCK - 1) / LANE_BLOCK;
  const dim3 ig((2 * K + 63) / 64, 2);
  if (s == 19) {
    hipLaunchKernelGGL(k_fbp_inv_bwd<19>, ig, dim3(64), 0, st, d_halves, K, W);
    hipLaunchKernelGGL(k_fbs_fill<19>, dim3(K * per, 2), dim3(LANE_BLOCK), 0, st, d_halves, cst, K, W, t0, t1, g);
  } else if (s == 37) {
    hipLaunchKernelGGL(k_fbp_inv_bwd<37>, ig, dim3(64), 0, st, d_halves, K, W);
    hipLaunchKernelGGL(k_fbs_fill<37>, dim3(K * per, 2), dim3(LANE_BLOCK), 0, st, d_halves, cst, K, W, t0, t1, g);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace fpai
