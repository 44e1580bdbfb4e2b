// Public-key fixed-base kernels (kernels_pfb.hpp): instantiations and launches.
#include "engine_pfb.hpp"
#ifndef FLEXPAI_XCHECK
#define FLEXPAI_XCHECK 0   // 1: the test-only library (flexpai.hip: xcheck_env)
#endif

namespace fpai {

static size_t pg_lds() { return ((size_t)(BLOCK / PFB_TPI) * 2 * PFB_S + PFB_S) * 4; }
static size_t main_lds() { return pg_lds(); }   // + the static row staging (kernels_grp_pair.hpp)

#if FLEXPAI_XCHECK
int pfb_occupancy(int* occ) {
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(occ, k_pfb<PFB_TPI, PFB_LL>, BLOCK, main_lds()) != hipSuccess ||
      *occ < 1)
    *occ = 1;
  return 0;
}
#endif

hipError_t pfb_build_phase1(const PfbConst* d_c, int nbases, int K, int W, hipStream_t st) {
  constexpr int GPB = BLOCK / PFB_TPI;
  hipLaunchKernelGGL((k_pfb_chain<PFB_TPI, PFB_LL>), dim3((nbases + GPB - 1) / GPB), dim3(BLOCK), pg_lds(), st, d_c);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int LO = W / 2, HI = W - LO;
  const int nent = (1 << LO) + (1 << HI);
  // the lohi builder of the 4096-bit key holder's tables, on one "half": the modulus n (PfbConst::g)
  hipLaunchKernelGGL((k_fbgp_lohi<PFB_TPI, PFB_LL>), dim3((nent + GPB - 1) / GPB, K, 1), dim3(BLOCK), pg_lds(), st,
                     &d_c->g, K, W);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL((k_pair_inv_fwd<PFB_TPI, PFB_LL>), dim3((2 * K + GPB - 1) / GPB, 1), dim3(BLOCK),
                     (size_t)GPB * PFB_S * 4, st, &d_c->g, K, W);
  return hipGetLastError();
}

hipError_t pfb_build_phase2(const PfbConst* d_c, int K, int W, uint4* table, hipStream_t st) {
  constexpr int GPB = BLOCK / PFB_TPI;
  hipLaunchKernelGGL((k_pair_inv_bwd<PFB_TPI, PFB_LL>), dim3((2 * K + GPB - 1) / GPB, 1), dim3(BLOCK),
                     (size_t)GPB * PFB_S * 4, st, &d_c->g, K, W);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((k_pfb_fill<PFB_TPI, PFB_LL>), dim3(((1 << W) + GPB - 1) / GPB, K), dim3(BLOCK), pg_lds(), st,
                     d_c, K, W, table);
  return hipGetLastError();
}

hipError_t pfb_launch_digits(const PfbDigitParams& p, int gx, hipStream_t st) {
  hipLaunchKernelGGL(k_pfb_digits<0>, dim3(gx), dim3(PFB_DIG_BLOCK), 0, st, p);
  return hipGetLastError();
}

#if FLEXPAI_XCHECK
hipError_t pfb_launch(const PfbParams& p, int gx, hipStream_t st) {
  hipLaunchKernelGGL((k_pfb<PFB_TPI, PFB_LL>), dim3(gx), dim3(BLOCK), main_lds(), st, p);
  return hipGetLastError();
}
#endif

}  // namespace fpai
