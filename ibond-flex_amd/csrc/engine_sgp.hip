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

hipError_t sgp_launch(const SgpParams& p, int gx, int halves, hipStream_t st) {
  hipLaunchKernelGGL(k_sgp<SGP_S>, dim3(gx, halves), dim3(LANE_BLOCK), 0, st, p);
  return hipGetLastError();
}

}  // namespace fpai
