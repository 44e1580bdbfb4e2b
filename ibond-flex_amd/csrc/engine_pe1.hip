// 1024-bit public-key encryption on p-adic pairs (kernels_pe1.hpp): instantiations and launches.
#include "engine_pe1.hpp"

namespace fpai {

int pe1_occupancy(int* occ) {
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(occ, k_pe1_pow<PE1_S>, LANE_BLOCK, 0) != hipSuccess || *occ < 1) *occ = 1;
  return 0;
}

hipError_t pe1_launch(const Pe1Params& p, const DecPairPreParams& pre, int gx, int cus, hipStream_t st, hipEvent_t* ev) {
  const long long lb = (p.n + LANE_BLOCK - 1) / LANE_BLOCK;
  const int gl = (int)std::max<long long>(1, std::min<long long>(lb, 8ll * cus));
  if (ev && ev[0]) (void)hipEventRecord(ev[0], st);
  hipLaunchKernelGGL(k_pe1_words<0>, dim3(gl), dim3(LANE_BLOCK), 0, st, p);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_dec_pre_pair<PE1_S>, dim3(gl, 1), dim3(LANE_BLOCK), 0, st, pre);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (ev && ev[1]) (void)hipEventRecord(ev[1], st);
  hipLaunchKernelGGL(k_pe1_pow<PE1_S>, dim3((int)std::min<long long>(gx, lb)), dim3(LANE_BLOCK), 0, st, p);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (ev && ev[2]) (void)hipEventRecord(ev[2], st);
  hipLaunchKernelGGL(k_pe1_fin<PE1_S>, dim3(gl), dim3(LANE_BLOCK), 0, st, p);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (ev && ev[3]) (void)hipEventRecord(ev[3], st);
  return hipSuccess;
}

}  // namespace fpai
