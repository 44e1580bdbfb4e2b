// 4096-bit split-pair decryption (kernels_dec4.hpp): instantiations, geometry, launches.
#include "engine_dec4.hpp"

namespace fpai {

template <typename K>
static int occupancy(K kernel, int block, size_t lds) {
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kernel, block, lds) != hipSuccess || occ < 1) occ = 1;
  return occ;
}

int dec4_geometry(int cus, long long chunk, Dec4Geom* g) {
  const long long pb = (chunk + D4_PAIRS - 1) / D4_PAIRS, lb = (chunk + LANE_BLOCK - 1) / LANE_BLOCK;
  auto clamp = [](long long v, long long cap) { return (int)std::max<long long>(1, std::min<long long>(v, cap)); };
  g->gx_pre = clamp(pb, (long long)occupancy(k_dec4_pre<D4_S>, LANE_BLOCK, 0) * cus / 2);
  g->gx_pow = clamp(pb, (long long)occupancy(k_dec4_pow<D4_S>, LANE_BLOCK, 0) * cus / 2);
  g->gx_L = clamp(lb, (long long)occupancy(k_dec4_L<D4_S>, LANE_BLOCK, 0) * cus / 2);
  constexpr int GPB = BLOCK / 4;
  g->lds_fin = (size_t)GPB * 4 * L * 4;
  g->gx_fin = clamp((chunk + GPB - 1) / GPB, (long long)occupancy(k_dec4_fin<4>, BLOCK, g->lds_fin) * cus);
  g->scratch_bytes = (size_t)2 * g->gx_pow * LANE_BLOCK * lane_scratch_words<D4_S>() * 4;
  return 0;
}

hipError_t dec4_launch_tail(const Dec4Params& p, const DecParams& f, const Dec4Geom& g, hipStream_t st) {
  const long long lb = (p.n + LANE_BLOCK - 1) / LANE_BLOCK;
  constexpr int GPB = BLOCK / 4;
  const long long fb = (p.n + GPB - 1) / GPB;
  hipLaunchKernelGGL(k_dec4_L<D4_S>, dim3((int)std::min<long long>(g.gx_L, lb), 2), dim3(LANE_BLOCK), 0, st, p);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_dec4_fin<4>, dim3((int)std::min<long long>(g.gx_fin, fb)), dim3(BLOCK), g.lds_fin, st, f,
                     (const uint32_t*)p.mh);
  return hipGetLastError();
}

hipError_t dec4_launch(const Dec4Params& p, const DecParams& f, const Dec4Geom& g, hipStream_t st, hipEvent_t* ev) {
  const long long pb = (p.n + D4_PAIRS - 1) / D4_PAIRS, lb = (p.n + LANE_BLOCK - 1) / LANE_BLOCK;
  constexpr int GPB = BLOCK / 4;
  const long long fb = (p.n + GPB - 1) / GPB;
  if (ev && ev[0]) (void)hipEventRecord(ev[0], st);
  hipLaunchKernelGGL(k_dec4_pre<D4_S>, dim3((int)std::min<long long>(g.gx_pre, pb), 2), dim3(LANE_BLOCK), 0, st, p);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (ev && ev[1]) (void)hipEventRecord(ev[1], st);
  hipLaunchKernelGGL(k_dec4_pow<D4_S>, dim3((int)std::min<long long>(g.gx_pow, pb), 2), dim3(LANE_BLOCK), 0, st, p);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (ev && ev[2]) (void)hipEventRecord(ev[2], st);
  hipLaunchKernelGGL(k_dec4_L<D4_S>, dim3((int)std::min<long long>(g.gx_L, lb), 2), dim3(LANE_BLOCK), 0, st, p);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(k_dec4_fin<4>, dim3((int)std::min<long long>(g.gx_fin, fb)), dim3(BLOCK), g.lds_fin, st, f,
                     (const uint32_t*)p.mh);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (ev && ev[3]) (void)hipEventRecord(ev[3], st);
  return hipSuccess;
}

}  // namespace fpai
