// Pair exponentiation kernels (kernels_pair.hpp): instantiations, launch geometry and launches.
#ifndef FLEXPAI_XCHECK
#define FLEXPAI_XCHECK 0   // 1: the test-only library, which also holds the general decryption chain (k_dec_pow_pair<s, false>)
#endif
#include "engine_pair.hpp"

namespace fpai {

template <typename K>
static int occupancy(K kernel) {
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kernel, LANE_BLOCK, 0) != hipSuccess || occ < 1) occ = 1;
  return occ;
}

template <int S>
static void geometry(int cus, long long chunk, DecLaneGeom* g, bool factored) {
  const long long blocks = (chunk + LANE_BLOCK - 1) / LANE_BLOCK;
  auto clamp = [&](long long cap) { return (int)std::max<long long>(1, std::min<long long>(blocks, cap)); };
  g->gx_pre = clamp((long long)occupancy(k_dec_pre_pair<S>) * cus / 2);
#if FLEXPAI_XCHECK
  if (!factored) g->gx_pow = clamp((long long)occupancy(k_dec_pow_pair<S, false>) * cus / 2);
  else
#endif
    g->gx_pow = clamp((long long)occupancy(k_dec_pow_pair<S, true>) * cus / 2);
  (void)factored;
  g->gx_fin = clamp((long long)occupancy(k_dec_fin_pair<S>) * cus);
  g->scratch_bytes = (size_t)2 * g->gx_pow * LANE_BLOCK * lane_scratch_words<2 * S>() * 4;
}

int dec_pair_geometry(int s, int cus, long long chunk, DecLaneGeom* g, bool factored) {
  if (s == 19) geometry<19>(cus, chunk, g, factored);
  else if (s == 37) geometry<37>(cus, chunk, g, factored);
  else return -1;
  return 0;
}

template <int S>
static hipError_t launch(const DecPairPreParams& pre, const CrtParams& pw, const DecPairFinParams& f, const DecLaneGeom& g,
                         hipStream_t st, hipEvent_t* ev, bool factored) {
  const long long blocks = (f.n + LANE_BLOCK - 1) / LANE_BLOCK;
  auto clamp = [&](int gx) { return (int)std::min<long long>(gx, blocks); };
  if (ev && ev[0]) (void)hipEventRecord(ev[0], st);
  hipLaunchKernelGGL(k_dec_pre_pair<S>, dim3(clamp(g.gx_pre), 2), dim3(LANE_BLOCK), 0, st, pre);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (ev && ev[1]) (void)hipEventRecord(ev[1], st);
#if FLEXPAI_XCHECK
  if (!factored) hipLaunchKernelGGL((k_dec_pow_pair<S, false>), dim3(clamp(g.gx_pow), 2), dim3(LANE_BLOCK), 0, st, pw);
  else
#endif
    hipLaunchKernelGGL((k_dec_pow_pair<S, true>), dim3(clamp(g.gx_pow), 2), dim3(LANE_BLOCK), 0, st, pw);
  (void)factored;
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (ev && ev[2]) (void)hipEventRecord(ev[2], st);
  hipLaunchKernelGGL(k_dec_fin_pair<S>, dim3(clamp(g.gx_fin)), dim3(LANE_BLOCK), 0, st, f);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (ev && ev[3]) (void)hipEventRecord(ev[3], st);
  return hipSuccess;
}

hipError_t dec_pair_launch(int s, const DecPairPreParams& pre, const CrtParams& pw, const DecPairFinParams& f,
                           const DecLaneGeom& g, hipStream_t st, hipEvent_t* ev, bool factored) {
  if (s == 19) return launch<19>(pre, pw, f, g, st, ev, factored);
  if (s == 37) return launch<37>(pre, pw, f, g, st, ev, factored);
  return hipErrorInvalidValue;
}

hipError_t dec_pair_launch_fin(int s, const DecPairFinParams& f, int gx, hipStream_t st) {
  if (s == 19) hipLaunchKernelGGL(k_dec_fin_pair<19>, dim3(gx), dim3(LANE_BLOCK), 0, st, f);
  else if (s == 37) hipLaunchKernelGGL(k_dec_fin_pair<37>, dim3(gx), dim3(LANE_BLOCK), 0, st, f);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

int crt_b_pair_occupancy(int s, int* occ) {
  if (s == 19) *occ = occupancy(k_crt_b_pair<19>);
  else if (s == 37) *occ = occupancy(k_crt_b_pair<37>);
  else return -1;
  return 0;
}

hipError_t crt_b_pair_launch(int s, const CrtParams& p, int gx, hipStream_t st) {
  if (s == 19) hipLaunchKernelGGL(k_crt_b_pair<19>, dim3(gx, 2), dim3(LANE_BLOCK), 0, st, p);
  else if (s == 37) hipLaunchKernelGGL(k_crt_b_pair<37>, dim3(gx, 2), dim3(LANE_BLOCK), 0, st, p);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace fpai
