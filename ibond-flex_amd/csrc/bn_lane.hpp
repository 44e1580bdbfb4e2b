// Lane-per-element big-number engine for gfx950: one modulus-sized number entirely in ONE lane
// (S limbs of LB = 28 bits), 64 independent numbers per wavefront, no cross-lane traffic.
//
// Why a second engine next to the lane-group one (bn_group.hpp): squarings dominate every
// exponentiation on the Paillier path (~85% of products), and a square needs only the upper
// triangle a_i*a_j (i >= j, doubled off the diagonal): S(S+1)/2 + S^2 MACs instead of 2S^2.
// Inside a lane the triangle is a compile-time shape, so the saving is real; across the lanes of
// a group the lanes below the diagonal would idle in SIMD lock-step and nothing is saved. The
// price is registers (2S accumulator VGPRs + S for a + S for m), so it is used for moduli up to
// ~2072 bits (S <= 74): the CRT halves mod p / p^2 of 1024- and 2048-bit keys.
//
// CIOS with a rotating register map: at iteration j, relative accumulator position i lives in
// P[(i + j) % S]; after the reduction the lowest position is retired (its carry moves up) and
// becomes the new, empty top. After S iterations the map is the identity again. Accumulator
// bound: an accumulator lives S iterations and receives per iteration at most one a*b product
// (< 2^57 when doubled) and one q*m product (< 2^56), plus one carry (< 2^36):
// S * 1.5 * 2^57 + 2^36 < 2^64 for S <= 74.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

namespace fpai {
namespace lane {

constexpr int LB = 28;
constexpr uint32_t LMASK = (1u << LB) - 1u;

template <int S>
struct Mod {
  uint32_t m[S];      // modulus limbs
  uint32_t mprime;    // -m^-1 mod 2^LB
};

template <int S>
__device__ __forceinline__ void pin(uint64_t (&P)[S]) {
#pragma unroll
  for (int i = 0; i < S; ++i) asm volatile("" : "+v"(P[i]));
}

// reduction half of iteration J (shared by square and multiply)
template <int S, int J>
__device__ __forceinline__ void reduce_step(uint64_t (&P)[S], const uint32_t (&m)[S], uint32_t mprime) {
  const uint32_t q = ((uint32_t)P[J] * mprime) & LMASK;
#pragma unroll
  for (int i = 0; i < S; ++i) P[(i + J) % S] += (uint64_t)q * m[i];
  const uint64_t v0 = P[J];
  P[(J + 1) % S] += v0 >> LB;
  P[J] = 0;
  pin<S>(P);
  __builtin_amdgcn_sched_barrier(0);
}

template <int S, int J>
__device__ __forceinline__ void sqr_step(uint64_t (&P)[S], const uint32_t (&a)[S], const uint32_t (&m)[S],
                                         uint32_t mprime) {
  const uint32_t aj = a[J];
  const uint32_t aj2 = aj << 1;
  P[(2 * J) % S] += (uint64_t)aj * aj;
#pragma unroll
  for (int i = J + 1; i < S; ++i) P[(i + J) % S] += (uint64_t)a[i] * aj2;
  reduce_step<S, J>(P, m, mprime);
}

template <int S, int J>
__device__ __forceinline__ void mul_step(uint64_t (&P)[S], const uint32_t (&a)[S], uint32_t bj, const uint32_t (&m)[S],
                                         uint32_t mprime) {
#pragma unroll
  for (int i = 0; i < S; ++i) P[(i + J) % S] += (uint64_t)a[i] * bj;
  reduce_step<S, J>(P, m, mprime);
}

// A limb cut from a 64-bit sum by an explicit v_and_b32 into a fresh 32-bit register. Left to LLVM, the mask is
// applied to the 64-bit sum and the limb stays the low half of a live register pair: every loop-carried limb then
// holds two VGPRs (k_fbp: 236 VGPRs instead of ~160 for the same live values).
__device__ __forceinline__ uint32_t limb32(uint64_t v) {
  uint32_t r;
  asm("v_and_b32 %0, 0xfffffff, %1" : "=v"(r) : "v"((uint32_t)v));
  return r;
}

template <int S>
__device__ __forceinline__ void normalize(const uint64_t (&P)[S], uint32_t (&r)[S]) {
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < S; ++i) {
    const uint64_t v = P[i] + c;
    r[i] = limb32(v);
    c = v >> LB;
  }
}

template <int S, int... Js>
__device__ __forceinline__ void sqr_all(uint64_t (&P)[S], const uint32_t (&a)[S], const uint32_t (&m)[S],
                                        uint32_t mprime, std::integer_sequence<int, Js...>) {
  (sqr_step<S, Js>(P, a, m, mprime), ...);
}
template <int S, int... Js>
__device__ __forceinline__ void mul_all(uint64_t (&P)[S], const uint32_t (&a)[S], const uint32_t (&b)[S],
                                        const uint32_t (&m)[S], uint32_t mprime, std::integer_sequence<int, Js...>) {
  (mul_step<S, Js>(P, a, b[Js], m, mprime), ...);
}

// One CIOS pass over S digits of b, accumulating into P (no normalisation): K passes over the
// chunks of a K*S-limb b compute a * b * R^-K mod m (used to reduce wide inputs).
template <int S>
__device__ __forceinline__ void mul_pass(uint64_t (&P)[S], const uint32_t (&a)[S], const uint32_t (&b)[S],
                                         const uint32_t (&m)[S], uint32_t mprime) {
  mul_all<S>(P, a, b, m, mprime, std::make_integer_sequence<int, S>{});
}

// a <- a^2 R^-1 mod m   (a < 2m, R = 2^(LB*S) > 4m  ->  result < 2m, canonical limbs)
template <int S>
__device__ __forceinline__ void mont_sqr(uint32_t (&a)[S], const uint32_t (&m)[S], uint32_t mprime) {
  uint64_t P[S];
#pragma unroll
  for (int i = 0; i < S; ++i) P[i] = 0;
  sqr_all<S>(P, a, m, mprime, std::make_integer_sequence<int, S>{});
  normalize<S>(P, a);
}

// a <- a b R^-1 mod m   (a, b < 2m -> result < 2m)
template <int S>
__device__ __forceinline__ void mont_mul(uint32_t (&a)[S], const uint32_t (&b)[S], const uint32_t (&m)[S],
                                         uint32_t mprime) {
  uint64_t P[S];
#pragma unroll
  for (int i = 0; i < S; ++i) P[i] = 0;
  mul_all<S>(P, a, b, m, mprime, std::make_integer_sequence<int, S>{});
  normalize<S>(P, a);
}

// a <- a b R^-1 mod m with the multiplier b in LDS, one column of 16-byte quads per lane:
// limbs 4g..4g+3 at bq[g * BSTRIDE] (layout [quad][lane]: conflict-free ds_read_b128). Quad g+1 is
// read while quad g's steps run, so the LDS latency hides behind the MACs and b never occupies
// S VGPRs.
template <int S, int BSTRIDE, int J>
__device__ __forceinline__ void mul_step_lds(uint64_t (&P)[S], const uint32_t (&a)[S], uint4& cur, uint4& nxt,
                                             const uint4* __restrict__ bq, const uint32_t (&m)[S], uint32_t mprime) {
  if constexpr (J % 4 == 0) {
    cur = nxt;
    if constexpr (J / 4 + 1 < (S + 3) / 4) nxt = bq[(J / 4 + 1) * BSTRIDE];
  }
  const uint32_t bj = (J % 4 == 0) ? cur.x : (J % 4 == 1) ? cur.y : (J % 4 == 2) ? cur.z : cur.w;
#pragma unroll
  for (int i = 0; i < S; ++i) P[(i + J) % S] += (uint64_t)a[i] * bj;
  reduce_step<S, J>(P, m, mprime);
}
template <int S, int BSTRIDE, int... Js>
__device__ __forceinline__ void mul_all_lds(uint64_t (&P)[S], const uint32_t (&a)[S], const uint4* __restrict__ bq,
                                            const uint32_t (&m)[S], uint32_t mprime, std::integer_sequence<int, Js...>) {
  uint4 cur, nxt = bq[0];
  (mul_step_lds<S, BSTRIDE, Js>(P, a, cur, nxt, bq, m, mprime), ...);
}
template <int S, int BSTRIDE>
__device__ __forceinline__ void mont_mul_lds(uint32_t (&a)[S], const uint4* __restrict__ bq, const uint32_t (&m)[S],
                                             uint32_t mprime) {
  uint64_t P[S];
#pragma unroll
  for (int i = 0; i < S; ++i) P[i] = 0;
  mul_all_lds<S, BSTRIDE>(P, a, bq, m, mprime, std::make_integer_sequence<int, S>{});
  normalize<S>(P, a);
}

// d = a - b over S canonical limbs; returns the borrow out (true when a < b, d then wraps)
template <int S>
__device__ __forceinline__ bool sub(const uint32_t (&a)[S], const uint32_t (&b)[S], uint32_t (&d)[S]) {
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < S; ++i) {
    const int32_t v = (int32_t)a[i] - (int32_t)b[i] + c;
    d[i] = (uint32_t)v & LMASK;
    c = v >> LB;
  }
  return c != 0;
}

// a <- a - m if a >= m
template <int S>
__device__ __forceinline__ void cond_sub(uint32_t (&a)[S], const uint32_t (&m)[S]) {
  uint32_t d[S];
  const bool neg = sub<S>(a, m, d);
#pragma unroll
  for (int i = 0; i < S; ++i) a[i] = neg ? a[i] : d[i];
}

// Limb i of the integer held as little-endian 32-bit words w[0..nw) (compile-time limb index,
// so the word index and shift are constants; words past nw read as 0).
template <typename W>
__device__ __forceinline__ uint32_t limb_from_words(const W& w, int nw, int limb) {
  const int bit = limb * LB, wi = bit >> 5, sh = bit & 31;
  const uint64_t lo = wi < nw ? (uint64_t)w(wi) : 0ull;
  const uint64_t hi = (wi + 1 < nw && sh + LB > 32) ? (uint64_t)w(wi + 1) : 0ull;
  return (uint32_t)(((hi << 32) | lo) >> sh) & LMASK;
}

}  // namespace lane
}  // namespace fpai
