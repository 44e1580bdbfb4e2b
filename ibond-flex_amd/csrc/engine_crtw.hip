// CRT encryption on 16-lane rows (kernels_crtw.hpp): instantiations and launch.
#include "engine_crtw.hpp"

namespace fpai {

hipError_t crtw_launch(int sa, const crtw::Params& p, hipStream_t st) {
  const long long blocks = (p.n + crtw::GPW - 1) / crtw::GPW;
  const int gx = (int)std::min<long long>(blocks, 1ll << 20);
  if (sa == 19) hipLaunchKernelGGL((crtw::k_crt_w<19, 37>), dim3(gx, 2), dim3(crtw::BLOCK_W), 0, st, p);
  else if (sa == 37) hipLaunchKernelGGL((crtw::k_crt_w<37, 74>), dim3(gx, 2), dim3(crtw::BLOCK_W), 0, st, p);
  else if (sa == 74) hipLaunchKernelGGL((crtw::k_crt_w<74, 148>), dim3(gx, 2), dim3(crtw::BLOCK_W), 0, st, p);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t decw_launch(int sa, const crtw::DecParams& p, hipStream_t st) {
  const long long blocks = (p.n + crtw::GPW - 1) / crtw::GPW;
  const int gx = (int)std::min<long long>(blocks, 1ll << 20);
  if (sa == 19) hipLaunchKernelGGL((crtw::k_dec_w<19, 37>), dim3(gx, 2), dim3(crtw::BLOCK_W), 0, st, p);
  else if (sa == 37) hipLaunchKernelGGL((crtw::k_dec_w<37, 74>), dim3(gx, 2), dim3(crtw::BLOCK_W), 0, st, p);
  else if (sa == 74) hipLaunchKernelGGL((crtw::k_dec_w<74, 148>), dim3(gx, 2), dim3(crtw::BLOCK_W), 0, st, p);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t pew_launch(int k, const EncParams& p, const uint32_t* prog, int nprog, hipStream_t st) {
  const long long blocks = (p.n + crtw::GPW - 1) / crtw::GPW;
  const int gx = (int)std::min<long long>(blocks, 1ll << 20);
  if (k == 74) hipLaunchKernelGGL((crtw::k_pe_w<74>), dim3(gx), dim3(crtw::BLOCK_W), 0, st, p, prog, nprog);
  else if (k == 148) hipLaunchKernelGGL((crtw::k_pe_w<148>), dim3(gx), dim3(crtw::BLOCK_W), 0, st, p, prog, nprog);
  else if (k == 296) hipLaunchKernelGGL((crtw::k_pe_w<296>), dim3(gx), dim3(crtw::BLOCK_W), 0, st, p, prog, nprog);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace fpai
