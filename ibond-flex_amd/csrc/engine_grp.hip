// Group-engine key-holder kernels for 4096-bit keys (kernels_grp.hpp): instantiations and launches.
#include "engine_grp.hpp"

namespace fpai {

size_t grp_lds_bytes() { return (size_t)(BLOCK / GRP_TPI) * GRP_TPI * L * 4; }

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

}  // namespace fpai
