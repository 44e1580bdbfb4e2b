// Group-engine key-holder kernels for 4096-bit keys (kernels_grp.hpp): instantiations and launches.
#include "engine_grp.hpp"
#ifndef FLEXPAI_XCHECK
#define FLEXPAI_XCHECK 0   // 1: the test-only library (flexpai.hip: xcheck_env)
#endif

namespace fpai {

size_t grp_lds_bytes() { return (size_t)(BLOCK / GRP_TPI) * GRP_TPI * L * 4; }

#if FLEXPAI_XCHECK
int grp_occupancy(int* occ_fb) {
  const size_t lds = grp_lds_bytes();
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(occ_fb, k_fbg<GRP_TPI>, BLOCK, lds) != hipSuccess || *occ_fb < 1)
    *occ_fb = 1;
  return 0;
}
#endif

#if FLEXPAI_XCHECK
hipError_t grp_launch_fb(const FbParams& p, int gx, hipStream_t st) {
  hipLaunchKernelGGL(k_fbg<GRP_TPI>, dim3(gx, 2), dim3(BLOCK), grp_lds_bytes(), st, p);
  return hipGetLastError();
}
#endif

static size_t fin_lds_bytes() { return (size_t)(BLOCK / 8) * 8 * L * 4; }

int grp_fin_occupancy(int* occ_garner, int* occ_fin) {
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(occ_garner, k_fbg_garner<GRP_TPI>, BLOCK, grp_lds_bytes()) !=
          hipSuccess || *occ_garner < 1)
    *occ_garner = 1;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(occ_fin, k_fbg_fin<8>, BLOCK, fin_lds_bytes()) != hipSuccess ||
      *occ_fin < 1)
    *occ_fin = 1;
  return 0;
}

hipError_t grp_launch_garner(const FbgGarnerParams& p, int gx, hipStream_t st) {
  hipLaunchKernelGGL(k_fbg_garner<GRP_TPI>, dim3(gx), dim3(BLOCK), grp_lds_bytes(), st, p);
  return hipGetLastError();
}

hipError_t grp_launch_fin(const FbgFinParams& p, int gx, hipStream_t st) {
  hipLaunchKernelGGL(k_fbg_fin<8>, dim3(gx), dim3(BLOCK), fin_lds_bytes(), st, p);
  return hipGetLastError();
}

#if FLEXPAI_XCHECK
hipError_t grp_build_tables(const FbHalf* d_halves, uint32_t* t0, uint32_t* t1, int K, int W, hipStream_t st) {
  constexpr int GPB = BLOCK / GRP_TPI;
  const int LO = W / 2, HI = W - LO;
  const int nent = (1 << LO) + (1 << HI);
  hipLaunchKernelGGL(k_fbg_lohi<GRP_TPI>, dim3((nent + GPB - 1) / GPB, K, 2), dim3(BLOCK), grp_lds_bytes(), st,
                     d_halves, K, W);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_fbg_fill<GRP_TPI>, dim3(((1 << W) + GPB - 1) / GPB, K, 2), dim3(BLOCK), grp_lds_bytes(), st,
                     d_halves, K, W, t0, t1);
  return hipGetLastError();
}
#endif

}  // namespace fpai
