// Split-pair fixed-base sampler (kernels_sgp.hpp): instantiation and launch. LDS is static (rows + b sums).
#ifndef FLEXPAI_XCHECK
#define FLEXPAI_XCHECK 0   // 1: the test-only library (address guards, guard.hpp)
#endif
#include "engine_sgp.hpp"

namespace fpai {

int sgp_occupancy(int* occ) {
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(occ, k_sgp<SGP_S>, LANE_BLOCK, 0) != hipSuccess || *occ < 1) *occ = 1;
  return 0;
}

hipError_t sgp_launch_w(const SgpParams& p, int halves, int cus, hipStream_t st) {
  const long long nb = (p.n + LANE_BLOCK - 1) / LANE_BLOCK;
  hipLaunchKernelGGL(k_sgp_w<SGP_S>, dim3((unsigned)std::max<long long>(1, std::min<long long>(nb, 4LL * cus)), halves),
                     dim3(LANE_BLOCK), 0, st, p);
  return hipGetLastError();
}

hipError_t sgp_launch_fin(const SgpFinParams& p, int cus, hipStream_t st) {
  const long long nb = (p.n + LANE_BLOCK - 1) / LANE_BLOCK;
  hipLaunchKernelGGL(k_sgp_fin<SGP_S>, dim3((unsigned)std::max<long long>(1, std::min<long long>(nb, 2LL * cus))), dim3(LANE_BLOCK), 0,
                     st, p);
  return hipGetLastError();
}

hipError_t sgp_launch(const SgpParams& p, int gx, int halves, hipStream_t st) {
  hipLaunchKernelGGL(k_sgp<SGP_S>, dim3(gx, halves), dim3(LANE_BLOCK), 0, st, p);
  return hipGetLastError();
}

}  // namespace fpai
