// Pair-group fixed-base kernels for 4096-bit keys (kernels_grp_pair.hpp): instantiations and launches.
#include "engine_grp_pair.hpp"
#ifndef FLEXPAI_XCHECK
#define FLEXPAI_XCHECK 0   // 1: the test-only library (flexpai.hip: xcheck_env)
#endif

namespace fpai {

static size_t pg_lds() { return ((size_t)(BLOCK / FBGP_TPI) * 2 * FBGP_S + FBGP_S) * 4; }
static size_t main_lds() { return pg_lds(); }   // + the static row staging (pair_table_products)
static size_t w_lds() { return (size_t)(BLOCK / 4) * 4 * L * 4; }

#if FLEXPAI_XCHECK
int fbgp_occupancy(int* occ) {
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(occ, k_fbgp<FBGP_TPI, FBGP_LL>, BLOCK, main_lds()) != hipSuccess ||
      *occ < 1)
    *occ = 1;
  return 0;
}
#endif

#if FLEXPAI_XCHECK
hipError_t fbgp_launch(const FbgpParams& p, int gx, hipStream_t st) {
  hipLaunchKernelGGL((k_fbgp<FBGP_TPI, FBGP_LL>), dim3(gx, 2), dim3(BLOCK), main_lds(), st, p);
  return hipGetLastError();
}
#endif

hipError_t fbgp_launch_w(const FbgpParams& p, int gx, hipStream_t st) {
  hipLaunchKernelGGL(k_fbgp_w<4>, dim3(gx, 2), dim3(BLOCK), w_lds(), st, p);
  return hipGetLastError();
}

// table construction, phase 1: lo/hi half-digit powers, then the forward pass of the batch inversion (the chain
// products land in FbgpHalf::cval for the host's inversion)
hipError_t fbgp_build_phase1(const FbgpHalf* d_halves, int K, int W, hipStream_t st) {
  constexpr int GPB = BLOCK / FBGP_TPI;
  const int LO = W / 2, HI = W - LO;
  const int nent = (1 << LO) + (1 << HI);
  hipLaunchKernelGGL((k_fbgp_lohi<FBGP_TPI, FBGP_LL>), dim3((nent + GPB - 1) / GPB, K, 2), dim3(BLOCK), pg_lds(), st,
                     d_halves, K, W);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((k_pair_inv_fwd<FBGP_TPI, FBGP_LL>), dim3((2 * K + GPB - 1) / GPB, 2), dim3(BLOCK),
                     (size_t)GPB * FBGP_S * 4, st, d_halves, K, W);
  return hipGetLastError();
}

// phase 2 (after the host wrote the chain inverses): the inverse tables, then the factored rows
hipError_t fbgp_build_phase2(const FbgpHalf* d_halves, uint32_t* t0, uint32_t* t1, int K, int W, hipStream_t st) {
  constexpr int GPB = BLOCK / FBGP_TPI;
  hipLaunchKernelGGL((k_pair_inv_bwd<FBGP_TPI, FBGP_LL>), dim3((2 * K + GPB - 1) / GPB, 2), dim3(BLOCK),
                     (size_t)GPB * FBGP_S * 4, st, d_halves, K, W);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((k_fbgp_fill<FBGP_TPI, FBGP_LL>), dim3(((1 << W) + GPB - 1) / GPB, K, 2), dim3(BLOCK), pg_lds(), st,
                     d_halves, K, W, t0, t1);
  return hipGetLastError();
}

}  // namespace fpai
