// Public-key split-pair encryption (kernels_pe.hpp): instantiations, geometry, launches.
#include "engine_pe.hpp"

namespace fpai {

template <typename K>
static int occupancy(K kernel) {
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kernel, LANE_BLOCK, 0) != hipSuccess || occ < 1) occ = 1;
  return occ;
}

int pe_geometry(int cus, long long chunk, Dec4Geom* g) {
  const long long pb = (chunk + D4_PAIRS - 1) / D4_PAIRS, lb = (chunk + LANE_BLOCK - 1) / LANE_BLOCK;
  auto clamp = [](long long v, long long cap) { return (int)std::max<long long>(1, std::min<long long>(v, cap)); };
  g->gx_pre = clamp(pb, (long long)occupancy(k_pe_pre<D4_S>) * cus);
  g->gx_pow = clamp(pb, (long long)std::min(occupancy(k_pe_pow<D4_S>), occupancy(k_pe_pow_f<D4_S>)) * cus);
  g->gx_L = clamp(lb, (long long)occupancy(k_pe_fin<D4_S>) * cus);
  g->scratch_bytes = (size_t)g->gx_pow * LANE_BLOCK * lane_scratch_words<D4_S>() * 4;
  return 0;
}

hipError_t pe_launch_pre_aw(const PeParams& p, const Dec4Geom& g, hipStream_t st, hipEvent_t* ev) {
  const long long pb = (p.n + D4_PAIRS - 1) / D4_PAIRS, lb = (p.n + LANE_BLOCK - 1) / LANE_BLOCK;
  if (ev && ev[0]) (void)hipEventRecord(ev[0], st);
  hipLaunchKernelGGL(k_pe_pre<D4_S>, dim3((int)std::min<long long>(g.gx_pre, pb)), dim3(LANE_BLOCK), 0, st, p);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_pe_awords<D4_S>, dim3((int)std::min<long long>(g.gx_L, lb)), dim3(LANE_BLOCK), 0, st, p);
  return hipGetLastError();
}

hipError_t pe_launch_iota_pow_f(const PeParams& p, const Dec4Geom& g, hipStream_t st, hipEvent_t* ev) {
  const long long pb = (p.n + D4_PAIRS - 1) / D4_PAIRS, lb = (p.n + LANE_BLOCK - 1) / LANE_BLOCK;
  hipLaunchKernelGGL(k_pe_iota<D4_S>, dim3((int)std::min<long long>(g.gx_pre, pb)), dim3(LANE_BLOCK), 0, st, p);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (ev && ev[1]) (void)hipEventRecord(ev[1], st);
  hipLaunchKernelGGL(k_pe_pow_f<D4_S>, dim3((int)std::min<long long>(g.gx_pow, pb)), dim3(LANE_BLOCK), 0, st, p);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (p.noinv) {   // the general chain, which exits at once unless the chunk had no inverse (PeParams::noinv)
    hipLaunchKernelGGL(k_pe_pow<D4_S>, dim3((int)std::min<long long>(g.gx_pow, pb)), dim3(LANE_BLOCK), 0, st, p);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  if (ev && ev[2]) (void)hipEventRecord(ev[2], st);
  hipLaunchKernelGGL(k_pe_fin<D4_S>, dim3((int)std::min<long long>(g.gx_L, lb)), dim3(LANE_BLOCK), 0, st, p);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (ev && ev[3]) (void)hipEventRecord(ev[3], st);
  return hipSuccess;
}

hipError_t pe_launch(const PeParams& p, const Dec4Geom& g, hipStream_t st, hipEvent_t* ev) {
  const long long pb = (p.n + D4_PAIRS - 1) / D4_PAIRS, lb = (p.n + LANE_BLOCK - 1) / LANE_BLOCK;
  if (ev && ev[0]) (void)hipEventRecord(ev[0], st);
  hipLaunchKernelGGL(k_pe_pre<D4_S>, dim3((int)std::min<long long>(g.gx_pre, pb)), dim3(LANE_BLOCK), 0, st, p);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (ev && ev[1]) (void)hipEventRecord(ev[1], st);
  hipLaunchKernelGGL(k_pe_pow<D4_S>, dim3((int)std::min<long long>(g.gx_pow, pb)), dim3(LANE_BLOCK), 0, st, p);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (ev && ev[2]) (void)hipEventRecord(ev[2], st);
  hipLaunchKernelGGL(k_pe_fin<D4_S>, dim3((int)std::min<long long>(g.gx_L, lb)), dim3(LANE_BLOCK), 0, st, p);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (ev && ev[3]) (void)hipEventRecord(ev[3], st);
  return hipSuccess;
}

hipError_t pe_launch_fin(const PeParams& p, int cus, hipStream_t st) {
  const long long lb = (p.n + LANE_BLOCK - 1) / LANE_BLOCK;
  const int gx = (int)std::max<long long>(1, std::min<long long>(lb, (long long)occupancy(k_pe_fin<D4_S>) * cus));
  hipLaunchKernelGGL(k_pe_fin<D4_S>, dim3(gx), dim3(LANE_BLOCK), 0, st, p);
  return hipGetLastError();
}

}  // namespace fpai
