// Host interface of the ciphertext x plaintext translation unit (engine_mul.hip, kernels_mul.hpp).
#pragma once
#include "kernels_mul.hpp"

namespace fpai {

// dynamic LDS bytes of k_mul / k_inv_* (one S-limb slot per lane group)
constexpr size_t mul_lds_bytes() { return (size_t)BLOCK * L * 4; }
// blocks per CU of k_mul<tpi> (-1: unsupported group size)
int mul_occupancy(int tpi, int* occ);
hipError_t mul_launch(int tpi, const MulParams& p, int grid, hipStream_t st);
hipError_t plain_launch(int tpi, const PlainParams& p, long long units, int cus, hipStream_t st);
hipError_t inv_launch(int tpi, bool up, const InvParams& p, int grid, hipStream_t st);

}  // namespace fpai
