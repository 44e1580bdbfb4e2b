// Lane-engine CRT encryption kernels (kernels_crt.hpp): instantiations, occupancy and launches,
// in their own translation unit so the engine builds in parallel.
#include "engine_lane.hpp"

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
    *occ_b = 1;   // stage B runs k_crt_b_pair (engine_pair.hip)
  } else if (sa == 37) {
    *occ_a = occupancy(k_crt_a<37>);
    *occ_b = 1;   // stage B runs k_crt_b_pair (engine_pair.hip)
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


}  // namespace fpai
