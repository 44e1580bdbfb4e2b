// Ciphertext x plaintext kernels (kernels_mul.hpp): instantiations and launches.
#include "engine_mul.hpp"

#include <algorithm>

namespace fpai {

int mul_occupancy(int tpi, int* occ) {
  hipError_t e;
  if (tpi == 2) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(occ, k_mul<2>, BLOCK, mul_lds_bytes());
  else if (tpi == 4) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(occ, k_mul<4>, BLOCK, mul_lds_bytes());
  else if (tpi == 8) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(occ, k_mul<8>, BLOCK, mul_lds_bytes());
  else return -1;
  if (e != hipSuccess || *occ < 1) *occ = 1;
  return 0;
}

hipError_t mul_launch(int tpi, const MulParams& p, int grid, hipStream_t st) {
  const size_t lds = mul_lds_bytes();
  if (tpi == 2) hipLaunchKernelGGL(k_mul<2>, dim3(grid), dim3(BLOCK), lds, st, p);
  else if (tpi == 4) hipLaunchKernelGGL(k_mul<4>, dim3(grid), dim3(BLOCK), lds, st, p);
  else if (tpi == 8) hipLaunchKernelGGL(k_mul<8>, dim3(grid), dim3(BLOCK), lds, st, p);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t plain_launch(int tpi, const PlainParams& p, long long units, int cus, hipStream_t st) {
  const size_t lds = mul_lds_bytes();
  const long long gpb = BLOCK / tpi;
  const int grid = (int)std::max<long long>(1, std::min<long long>((units + gpb - 1) / gpb, 8ll * cus));
  if (tpi == 2) hipLaunchKernelGGL(k_plain<2>, dim3(grid), dim3(BLOCK), lds, st, p);
  else if (tpi == 4) hipLaunchKernelGGL(k_plain<4>, dim3(grid), dim3(BLOCK), lds, st, p);
  else if (tpi == 8) hipLaunchKernelGGL(k_plain<8>, dim3(grid), dim3(BLOCK), lds, st, p);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t inv_launch(int tpi, bool up, const InvParams& p, int grid, hipStream_t st) {
  const size_t lds = mul_lds_bytes();
  if (tpi == 2) {
    if (up) hipLaunchKernelGGL(k_inv_up<2>, dim3(grid), dim3(BLOCK), lds, st, p);
    else hipLaunchKernelGGL(k_inv_down<2>, dim3(grid), dim3(BLOCK), lds, st, p);
  } else if (tpi == 4) {
    if (up) hipLaunchKernelGGL(k_inv_up<4>, dim3(grid), dim3(BLOCK), lds, st, p);
    else hipLaunchKernelGGL(k_inv_down<4>, dim3(grid), dim3(BLOCK), lds, st, p);
  } else if (tpi == 8) {
    if (up) hipLaunchKernelGGL(k_inv_up<8>, dim3(grid), dim3(BLOCK), lds, st, p);
    else hipLaunchKernelGGL(k_inv_down<8>, dim3(grid), dim3(BLOCK), lds, st, p);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace fpai
