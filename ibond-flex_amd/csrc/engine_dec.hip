// Lane-engine CRT decryption: kernel instantiations and launch geometry (own translation unit so
// the engine builds in parallel; the context and the C ABI live in flexpai.hip).
#include "engine_dec.hpp"
#ifndef FLEXPAI_XCHECK
#define FLEXPAI_XCHECK 0   // 1: the test-only library (flexpai.hip: xcheck_env)
#endif

namespace fpai {
#if FLEXPAI_XCHECK

template <typename K>
static int occupancy(K kernel) {
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kernel, LANE_BLOCK, 0) != hipSuccess || occ < 1) occ = 1;
  return occ;
}

template <int SA, int SB>
static void geometry(int cus, long long chunk, DecLaneGeom* g) {
  const long long blocks = (chunk + LANE_BLOCK - 1) / LANE_BLOCK;
  auto clamp = [&](long long cap) { return (int)std::max<long long>(1, std::min<long long>(blocks, cap)); };
  g->gx_pre = clamp((long long)occupancy(k_dec_pre<SB>) * cus / 2);
  g->gx_pow = clamp((long long)occupancy(k_dec_pow<SB>) * cus / 2);
  g->gx_fin = clamp((long long)occupancy(k_dec_fin<SA, SB>) * cus);
  g->scratch_bytes = (size_t)2 * g->gx_pow * LANE_BLOCK * lane_scratch_words<SB>() * 4;
}

int dec_lane_geometry(int sa, int cus, long long chunk, DecLaneGeom* g) {
  if (sa == 19) geometry<19, 37>(cus, chunk, g);
  else if (sa == 37) geometry<37, 74>(cus, chunk, g);
  else return -1;
  return 0;
}

template <int SA, int SB>
static hipError_t launch(const DecPreParams& pre, const CrtParams& pw, const DecFinParams& f, const DecLaneGeom& g,
                         hipStream_t st, hipEvent_t* ev) {
  const long long blocks = (f.n + LANE_BLOCK - 1) / LANE_BLOCK;
  auto clamp = [&](int gx) { return (int)std::min<long long>(gx, blocks); };
  if (ev && ev[0]) (void)hipEventRecord(ev[0], st);
  hipLaunchKernelGGL(k_dec_pre<SB>, dim3(clamp(g.gx_pre), 2), dim3(LANE_BLOCK), 0, st, pre);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (ev && ev[1]) (void)hipEventRecord(ev[1], st);
  hipLaunchKernelGGL(k_dec_pow<SB>, dim3(clamp(g.gx_pow), 2), dim3(LANE_BLOCK), 0, st, pw);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (ev && ev[2]) (void)hipEventRecord(ev[2], st);
  hipLaunchKernelGGL((k_dec_fin<SA, SB>), dim3(clamp(g.gx_fin)), dim3(LANE_BLOCK), 0, st, f);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (ev && ev[3]) (void)hipEventRecord(ev[3], st);
  return hipSuccess;
}

hipError_t dec_lane_launch(int sa, const DecPreParams& pre, const CrtParams& pw, const DecFinParams& f,
                           const DecLaneGeom& g, hipStream_t st, hipEvent_t* ev) {
  if (sa == 19) return launch<19, 37>(pre, pw, f, g, st, ev);
  if (sa == 37) return launch<37, 74>(pre, pw, f, g, st, ev);
  return hipErrorInvalidValue;
}

#endif
}  // namespace fpai
