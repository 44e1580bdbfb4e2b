// Shared pieces of the CRT decryptions: the per-half constants of the lane engine (DecLaneHalf: p_h, h_h R, p_h - 1,
// read by the pair kernels' setup) and the decode of the recombined plaintext (decode_lane: FixedPointNumber.decode,
// fixedpoint_number.py:92-107, with the reference's overflow checks), used by k_dec_fin_pair (kernels_pair.hpp).
// (The 2S-limb lane kernels k_dec_pre / k_dec_pow / k_dec_fin that first held them were retired in round 6.)
#pragma once
#include "kernels_crt.hpp"

namespace fpai {

struct DecLaneHalf {
  const uint32_t* m2;     // p_h^2, SB limbs
  const uint32_t* cK;     // R_B^(K+1) mod p_h^2, K = ciphertext chunks (SB limbs)
  uint32_t mprime2;       // -p_h^-2 mod 2^LB
  uint32_t pinv;          // p_h^-1 mod 2^LB (exact division)
  uint32_t mprime1;       // -p_h^-1 mod 2^LB
  uint32_t pad;
  const uint32_t* ph;     // p_h, SA limbs
  const uint32_t* hR;     // h_h * R_A mod p_h, SA limbs
  const uint32_t* pm1;    // p_h - 1, SA limbs (L for x == 0: (0 - 1) // p == -1 == p - 1 mod p)
};

// ---------------------------------------------------------------- CRT recombination + decode
template <int S>
__device__ __forceinline__ int cmp_limbs(const uint32_t (&a)[S], const uint32_t (&b)[S]) {
  int c = 0;
#pragma unroll
  for (int k = 0; k < S; ++k) c = (a[k] > b[k]) ? 1 : ((a[k] < b[k]) ? -1 : c);
  return c;
}

// FixedPointNumber.decode (fixedpoint_number.py:92-107) of x in [0, n), x in S canonical limbs:
// float(mantissa) correctly rounded (half even, Python int -> float), times 16^-e.
template <int S>
__device__ __forceinline__ void decode_lane(const uint32_t (&x)[S], const uint32_t (&nl)[S], const uint32_t (&mx)[S],
                                            int e, double& val, int64_t& mant, int& st) {
  uint32_t mag[S];
  bool neg = false;
  st = ST_OK;
  if (cmp_limbs<S>(x, mx) <= 0) {
#pragma unroll
    for (int k = 0; k < S; ++k) mag[k] = x[k];
  } else {
    (void)lane::sub<S>(nl, x, mag);   // n - x (x < n)
    if (cmp_limbs<S>(mag, mx) > 0) st = ST_OVERFLOW;
    neg = true;
  }
  val = 0.0;
  mant = 0;
  if (st != ST_OK) return;
  int top = 0;
  uint32_t xt = 0;
#pragma unroll
  for (int k = 0; k < S; ++k)
    if (mag[k]) {
      top = k;
      xt = mag[k];
    }
  const int B = xt == 0 ? 0 : top * lane::LB + (32 - __clz(xt));   // bit length
  const int lo_bit = B > 64 ? B - 64 : 0;
  uint64_t hi64 = 0;
  bool sticky = false;
#pragma unroll
  for (int k = 0; k < S; ++k) {
    const uint64_t v = mag[k];
    const int sh = k * lane::LB - lo_bit;
    if (sh >= 64) continue;
    if (sh >= 0) {
      hi64 |= v << sh;
    } else if (sh > -lane::LB) {
      hi64 |= v >> (-sh);
      sticky |= (v & ((1ull << (-sh)) - 1ull)) != 0;
    } else {
      sticky |= v != 0;
    }
  }
  double d;
  if (B <= 53) {
    d = (double)hi64;
  } else {
    const int drop = (B > 64 ? 64 : B) - 53;
    uint64_t keep = hi64 >> drop;
    const uint64_t rem = hi64 & ((1ull << drop) - 1ull);
    const uint64_t halfv = 1ull << (drop - 1);
    if (rem > halfv || (rem == halfv && (sticky || (keep & 1ull)))) keep += 1;
    d = ldexp((double)keep, lo_bit + drop);
  }
  if (e > 0) {
    if (isinf(d) || B > 1024) st = ST_FLOAT_OVF;
    else val = (neg ? -d : d) * ldexp(1.0, -4 * e);
  } else {
    val = ldexp(neg ? -d : d, -4 * e);
    const int sh = -4 * e;
    if (B + sh <= 63) {
      const int64_t mm = (int64_t)(hi64 << sh);
      mant = neg ? -mm : mm;
      st = ST_INT;
    } else {
      st = ST_INT_BIG;
    }
  }
}

}  // namespace fpai
