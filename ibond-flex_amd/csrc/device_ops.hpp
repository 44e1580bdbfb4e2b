// Per-element device helpers shared by the Paillier kernels: fixed-point encode
// (flex/crypto/paillier/fixedpoint_number.py:46-90), ChaCha20 obfuscator generation and the
// c0 = 1 + n*m construction (raw_encrypt.py:22-49).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "bn_group.hpp"

namespace fpai {

enum { ST_OK = 0, ST_INT = 1, ST_INT_BIG = 2, ST_OVERFLOW = 3, ST_FLOAT_OVF = 4, ST_ENC_RANGE = 5 };

// floor(a / b) for b > 0
__device__ __forceinline__ int floor_div(int a, int b) { return (a >= 0) ? a / b : -((-a + b - 1) / b); }

// FixedPointNumber.encode for a float value (float32 is widened exactly). precision=None:
// e = floor((53 - frexp(v).exp) / 4); m = round_half_even(v * 16^e) computed exactly
// (numpy-1.x semantics). |v| < 1e-200 encodes as the int 0 with e = 0.
__device__ __forceinline__ int encode_float(double v, bool fixed, int fexp, int64_t& M, int& e) {
  if (fabs(v) < 1e-200) {
    M = 0;
    e = fixed ? fexp : 0;
    return ST_OK;
  }
  if (!fixed) {
    int fe;
    (void)frexp(v, &fe);
    e = floor_div(53 - fe, 4);
  } else {
    e = fexp;
  }
  const double s = rint(ldexp(v, 4 * e));   // exact scaling, then ties-to-even
  if (!(fabs(s) < 9.223372036854775e18)) return ST_ENC_RANGE;
  M = (int64_t)s;
  return ST_OK;
}

__device__ __forceinline__ int encode_int(int64_t v, bool fixed, int fexp, int64_t& M, int& e) {
  if (!fixed || fexp == 0) {
    M = v;
    e = fixed ? fexp : 0;
    return ST_OK;
  }
  e = fexp;
  if (fexp > 0) {
    if (fexp >= 16) return v == 0 ? (M = 0, ST_OK) : ST_ENC_RANGE;
    const __int128 w = (__int128)v << (4 * fexp);
    if (w > (__int128)INT64_MAX || w < -(__int128)INT64_MAX) return ST_ENC_RANGE;
    M = (int64_t)w;
    return ST_OK;
  }
  const double s = rint(ldexp((double)v, 4 * fexp));
  M = (int64_t)s;
  return ST_OK;
}

// ---------------------------------------------------------------- ChaCha20 (RFC 8439 §2.3)
__device__ __forceinline__ uint32_t rotl32(uint32_t v, int c) { return (v << c) | (v >> (32 - c)); }
#define FPAI_QR(a, b, c, d)            \
  a += b; d = rotl32(d ^ a, 16);       \
  c += d; b = rotl32(b ^ c, 12);       \
  a += b; d = rotl32(d ^ a, 8);        \
  c += d; b = rotl32(b ^ c, 7);

__device__ __forceinline__ void chacha20_block(const uint32_t key[8], uint32_t counter, uint32_t n0, uint32_t n1,
                                               uint32_t n2, uint32_t out[16]) {
  uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key[0], key[1], key[2], key[3],
                    key[4],      key[5],      key[6],      key[7],      counter, n0,     n1,     n2};
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = s[i];
#pragma unroll 1
  for (int r = 0; r < 10; ++r) {
    FPAI_QR(x[0], x[4], x[8], x[12]);
    FPAI_QR(x[1], x[5], x[9], x[13]);
    FPAI_QR(x[2], x[6], x[10], x[14]);
    FPAI_QR(x[3], x[7], x[11], x[15]);
    FPAI_QR(x[0], x[5], x[10], x[15]);
    FPAI_QR(x[1], x[6], x[11], x[12]);
    FPAI_QR(x[2], x[7], x[8], x[13]);
    FPAI_QR(x[3], x[4], x[9], x[14]);
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) out[i] = x[i] + s[i];
}
#undef FPAI_QR

}  // namespace fpai
