// Host interface of the lane-engine CRT encryption translation unit (engine_lane.hip): stage A
// (k_crt_a) and stage B (k_crt_b) instantiations, occupancy and launches.
#pragma once
#include "kernels_crt.hpp"

namespace fpai {

// blocks per CU the kernels reach (hipOccupancyMaxActiveBlocksPerMultiprocessor); -1 if unsupported
int crt_lane_occupancy(int sa, int* occ_a, int* occ_b);
// k_crt_a<sa> / k_crt_b<sa, 2 sa> on grid (gx, 2)
hipError_t crt_launch_a(int sa, const CrtParams& p, int gx, hipStream_t st);

}  // namespace fpai
