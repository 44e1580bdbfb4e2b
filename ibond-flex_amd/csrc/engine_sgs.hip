// Shoup-row split-pair sampler (kernels_sgs.hpp): instantiations and launches. LDS is static.
#ifndef FLEXPAI_XCHECK
#define FLEXPAI_XCHECK 0   // 1: the test-only library (address guards, guard.hpp)
#endif
#include "engine_sgs.hpp"

namespace fpai {

int sgs_occupancy(int* occ) {
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(occ, k_sgs<SGP_S>, LANE_BLOCK, 0) != hipSuccess || *occ < 1) *occ = 1;
  return 0;
}

hipError_t sgs_launch_conv(const SgsHalf* halves, size_t rows, uint4* atab0, uint4* atab1, hipStream_t st) {
  hipLaunchKernelGGL(k_sgs_conv<SGP_S>, dim3((unsigned)((rows + LANE_BLOCK - 1) / LANE_BLOCK), 2), dim3(LANE_BLOCK), 0, st, halves,
                     rows, atab0, atab1);
  return hipGetLastError();
}

hipError_t sgs_launch(const SgsParams& p, int gx, int halves, hipStream_t st) {
  hipLaunchKernelGGL(k_sgs<SGP_S>, dim3(gx, halves), dim3(LANE_BLOCK), 0, st, p);
  return hipGetLastError();
}

hipError_t sgs_launch_bfin(const SgsFinParams& p, int halves, int cus, hipStream_t st) {
  const long long nb = (p.n + SGP_PAIRS - 1) / SGP_PAIRS;
  hipLaunchKernelGGL(k_sgs_bfin<SGP_S>, dim3((unsigned)std::max<long long>(1, std::min<long long>(nb, 2LL * cus)), halves),
                     dim3(LANE_BLOCK), 0, st, p);
  return hipGetLastError();
}

}  // namespace fpai
