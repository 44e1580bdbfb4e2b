// Lane-engine CRT encryption kernels (kernels_crt.hpp): instantiations, occupancy and launches,
// in their own translation unit so the engine builds in parallel.
#include "engine_lane.hpp"
#ifndef FLEXPAI_XCHECK
#define FLEXPAI_XCHECK 0   // 1: the test-only library (flexpai.hip: xcheck_env)
#endif

namespace fpai {

template <typename K>
static int occupancy(K kernel) {
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kernel, LANE_BLOCK, 0) != hipSuccess || occ < 1) occ = 1;
  return occ;
}

int crt_lane_occupancy(int sa, int* occ_a, int* occ_b) {
  if (sa == 19) {
    *occ_a = occupancy(k_crt_a<19>);
#if FLEXPAI_XCHECK
    *occ_b = occupancy(k_crt_b<19, 37>);
#else
    *occ_b = 1;   // stage B runs k_crt_b_pair (engine_pair.hip)
#endif
  } else if (sa == 37) {
    *occ_a = occupancy(k_crt_a<37>);
#if FLEXPAI_XCHECK
    *occ_b = occupancy(k_crt_b<37, 74>);
#else
    *occ_b = 1;   // stage B runs k_crt_b_pair (engine_pair.hip)
#endif
  } else {
    return -1;
  }
  return 0;
}

hipError_t crt_launch_a(int sa, const CrtParams& p, int gx, hipStream_t st) {
  if (sa == 19) hipLaunchKernelGGL(k_crt_a<19>, dim3(gx, 2), dim3(LANE_BLOCK), 0, st, p);
  else if (sa == 37) hipLaunchKernelGGL(k_crt_a<37>, dim3(gx, 2), dim3(LANE_BLOCK), 0, st, p);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

#if FLEXPAI_XCHECK
hipError_t crt_launch_b(int sa, const CrtParams& p, int gx, hipStream_t st) {
  if (sa == 19) hipLaunchKernelGGL((k_crt_b<19, 37>), dim3(gx, 2), dim3(LANE_BLOCK), 0, st, p);
  else if (sa == 37) hipLaunchKernelGGL((k_crt_b<37, 74>), dim3(gx, 2), dim3(LANE_BLOCK), 0, st, p);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}
#endif

}  // namespace fpai
