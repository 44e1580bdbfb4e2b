// p-adic pairs (bn_pair.hpp) on lane groups (bn_group.hpp's layout) with LL limbs per lane: a residue mod
// p^2 as (A, B), v = A + p B, each of A, B spread over the TPI lanes of a group (lane t owns limbs
// [LL t, LL t + LL)), S = TPI LL limbs of p. For 4096-bit keys p has 2048 bits: TPI = 4, LL = 19, S = 76, and
// a pair product costs 5 S^2 = 28.9 k lane-MACs against 2 (148)^2 = 43.8 k for the Montgomery product over the
// 148 limbs of p^2 that k_fbg runs (TPI = 4, L = 37). (TPI = 2 with L = 37 per lane does not fit: A, B, two
// accumulator rows and the modulus take 259 VGPRs.)
//
// One CIOS digit j, multiplier digits (a2j, b2j) broadcast from the group's LDS slot [A2: S][B2: S]:
//   P1 += A a2j,  P2 += B a2j + A b2j                  (square: P1 += A a_j, P2 += A (2 b_j))
//   q1 = P1_low mprime (group lane 0, DPP broadcast);  P2_low += LMASK - q1  (group lane 0)
//   q2 = P2_low mprime;  P1 += q1 p, P2 += q2 p;  both rows shift one limb across the group (DPP).
// The digits LMASK - q1_j sum to (R - 1) - m, so with P2 started at X = (1 - R) mod p (R = 2^(28 S)) the second
// row computes REDC(A1 B2 + A2 B1 - m) with every accumulator non-negative (kernels_dec4.hpp uses the same
// device). Bounds: operands < 2p, R >= 2^24 p: outputs < 2p; a physical accumulator lives LL digits and takes
// at most three products (< 2^57 for a doubled digit) per digit.
#pragma once
#include "bn_group.hpp"

namespace fpai {
namespace pgrp {

// a limb cut from a 64-bit sum into a fresh 32-bit register (see bn_lane.hpp limb32)
__device__ __forceinline__ uint32_t cut28(uint64_t v) {
  uint32_t r;
  asm("v_and_b32 %0, 0xfffffff, %1" : "=v"(r) : "v"((uint32_t)v));
  return r;
}

template <int TPI, int LL>
__device__ __forceinline__ void normalize(const uint64_t (&P)[LL], uint32_t (&r)[LL], int lane, int tig) {
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < LL; ++i) {
    const uint64_t v = P[i] + c;
    r[i] = cut28(v);
    c = v >> LB;
  }
  uint32_t inlo = dpp_from_prev((uint32_t)c);
  uint32_t inhi = dpp_from_prev((uint32_t)(c >> 32));
  if (tig == 0) { inlo = 0; inhi = 0; }
  c = ((uint64_t)inhi << 32) | inlo;
  {
    const uint64_t v = (uint64_t)r[0] + c;
    r[0] = (uint32_t)v & LMASK;
    c = v >> LB;
  }
  uint32_t c32 = (uint32_t)c;
#pragma unroll
  for (int i = 1; i < LL; ++i) {
    const uint32_t v = r[i] + c32;
    r[i] = v & LMASK;
    c32 = v >> LB;
  }
  if (ballot(c32 != 0) != 0ull) {
    bool all_ones = true;
#pragma unroll
    for (int i = 0; i < LL; ++i) all_ones &= (r[i] == LMASK);
    uint32_t ci = lookahead_carry_in<TPI>(c32 != 0, all_ones, lane);
#pragma unroll
    for (int i = 0; i < LL; ++i) {
      const uint32_t v = r[i] + ci;
      r[i] = v & LMASK;
      ci = v >> LB;
    }
  }
}

// d = a - b; true (group-uniform) when a < b
template <int TPI, int LL>
__device__ __forceinline__ bool sub_limbs(const uint32_t (&a)[LL], const uint32_t (&b)[LL], uint32_t (&d)[LL], int lane, int tig) {
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < LL; ++i) {
    const int32_t v = (int32_t)a[i] - (int32_t)b[i] + c;
    d[i] = (uint32_t)v & LMASK;
    c = v >> LB;
  }
  const int32_t b1 = c;
  int32_t bin = (int32_t)dpp_from_prev((uint32_t)c);
  if (tig == 0) bin = 0;
#pragma unroll
  for (int i = 0; i < LL; ++i) {
    const int32_t v = (int32_t)d[i] + bin;
    d[i] = (uint32_t)v & LMASK;
    bin = v >> LB;
  }
  bool all_zero = true;
#pragma unroll
  for (int i = 0; i < LL; ++i) all_zero &= (d[i] == 0u);
  const bool gen = (bin != 0);
  const uint32_t bi = lookahead_carry_in<TPI>(gen, all_zero, lane);
  if (ballot(bi != 0) != 0ull) {
    int32_t b2 = -(int32_t)bi;
#pragma unroll
    for (int i = 0; i < LL; ++i) {
      const int32_t v = (int32_t)d[i] + b2;
      d[i] = (uint32_t)v & LMASK;
      b2 = v >> LB;
    }
  }
  const bool neg_here = (tig == TPI - 1) && (b1 != 0 || gen || (all_zero && bi));
  const uint64_t NB = ballot(neg_here);
  const int gbase = lane - tig;
  return ((NB >> (gbase + TPI - 1)) & 1ull) != 0ull;
}

template <int TPI, int LL>
__device__ __forceinline__ void cond_sub(uint32_t (&r)[LL], const uint32_t (&m)[LL], int lane, int tig) {
  uint32_t d[LL];
  const bool neg = sub_limbs<TPI, LL>(r, m, d, lane, tig);
  if (!neg) {
#pragma unroll
    for (int i = 0; i < LL; ++i) r[i] = d[i];
  }
}

template <int TPI, int LL, bool SQR, bool B2Z, int S_>
__device__ __forceinline__ void step(uint64_t (&P1)[LL], uint64_t (&P2)[LL], const uint32_t (&A)[LL], const uint32_t (&B)[LL],
                                     const uint32_t* __restrict__ Ao, const uint32_t* __restrict__ Bo, uint32_t& acur,
                                     uint32_t& bcur, const uint32_t (&m)[LL], uint32_t mprime, int tig) {
  const uint32_t aj = acur, bj = bcur;
  if constexpr (S_ + 1 < LL) {
    acur = Ao[S_ + 1];
    if constexpr (SQR || !B2Z) bcur = Bo[S_ + 1];
  }
  (void)bj;
  if constexpr (SQR) {
    const uint32_t bj2 = bj << 1;
#pragma unroll
    for (int i = 0; i < LL; ++i) {
      P1[(i + S_) % LL] += (uint64_t)A[i] * aj;
      P2[(i + S_) % LL] += (uint64_t)A[i] * bj2;
    }
  } else {
#pragma unroll
    for (int i = 0; i < LL; ++i) {
      P1[(i + S_) % LL] += (uint64_t)A[i] * aj;
      P2[(i + S_) % LL] += (uint64_t)B[i] * aj;
      if constexpr (!B2Z) {
        asm volatile("" : "+v"(P2[(i + S_) % LL]));   // keeps both products accumulating MACs (LLVM would
        P2[(i + S_) % LL] += (uint64_t)A[i] * bj;      // otherwise sum them first and add: 3 instructions)
      }
    }
  }
  const uint32_t q1 = bcast0<TPI>(((uint32_t)P1[S_] * mprime) & LMASK);
  P2[S_] += tig == 0 ? (uint64_t)(LMASK - q1) : 0ull;
  const uint32_t q2 = bcast0<TPI>(((uint32_t)P2[S_] * mprime) & LMASK);
#pragma unroll
  for (int i = 0; i < LL; ++i) {
    P1[(i + S_) % LL] += (uint64_t)q1 * m[i];
    P2[(i + S_) % LL] += (uint64_t)q2 * m[i];
  }
  const uint64_t v1 = P1[S_], v2 = P2[S_];
  P1[(S_ + 1) % LL] += v1 >> LB;
  P2[(S_ + 1) % LL] += v2 >> LB;
  P1[S_] = (uint64_t)dpp_from_next((uint32_t)v1 & LMASK);
  P2[S_] = (uint64_t)dpp_from_next((uint32_t)v2 & LMASK);
#pragma unroll
  for (int i = 0; i < LL; ++i) asm volatile("" : "+v"(P1[i]), "+v"(P2[i]));
  __builtin_amdgcn_sched_barrier(0);
}

template <int TPI, int LL, bool SQR, bool B2Z, int... Ss>
__device__ __forceinline__ void outer(uint64_t (&P1)[LL], uint64_t (&P2)[LL], const uint32_t (&A)[LL], const uint32_t (&B)[LL],
                                      const uint32_t* __restrict__ Ao, const uint32_t* __restrict__ Bo, const uint32_t (&m)[LL],
                                      uint32_t mprime, int tig, std::integer_sequence<int, Ss...>) {
  uint32_t acur = Ao[0], bcur = (SQR || !B2Z) ? Bo[0] : 0u;
  (step<TPI, LL, SQR, B2Z, Ss>(P1, P2, A, B, Ao, Bo, acur, bcur, m, mprime, tig), ...);
}

// (A, B) <- (A, B) (A2, B2) R^-1, (A2, B2) in the group's LDS slot [A2: S][B2: S] (SQR: the slot holds (A, B)
// itself); xs: (1 - R) mod p in LDS (S limbs). B2Z: the multiplier is (A2, 0) (its B half is not read): the B row
// drops the A B2 term, 4 S^2 lane-MACs instead of 5 S^2 (factored table rows, kernels_grp_pair.hpp).
template <int TPI, int LL, bool SQR, bool B2Z = false>
__device__ __forceinline__ void montmul(uint32_t (&A)[LL], uint32_t (&B)[LL], const uint32_t* slot, const uint32_t* xs,
                                        const uint32_t (&m)[LL], uint32_t mprime, int lane, int tig) {
  constexpr int S = TPI * LL;
  uint64_t P1[LL], P2[LL];
#pragma unroll
  for (int i = 0; i < LL; ++i) {
    P1[i] = 0;
    P2[i] = xs[tig * LL + i];
  }
  for (int o = 0; o < TPI; ++o)
    outer<TPI, LL, SQR, B2Z>(P1, P2, A, B, slot + o * LL, slot + S + o * LL, m, mprime, tig, std::make_integer_sequence<int, LL>{});
  normalize<TPI, LL>(P1, A, lane, tig);
  normalize<TPI, LL>(P2, B, lane, tig);
}

// ---- single-row Montgomery products mod p on the group (table construction and the final correction)
template <int TPI, int LL, int S_>
__device__ __forceinline__ void step1(uint64_t (&P)[LL], const uint32_t (&A)[LL], const uint32_t* __restrict__ Ao, uint32_t& acur,
                                      const uint32_t (&m)[LL], uint32_t mprime) {
  const uint32_t aj = acur;
  if constexpr (S_ + 1 < LL) acur = Ao[S_ + 1];
#pragma unroll
  for (int i = 0; i < LL; ++i) P[(i + S_) % LL] += (uint64_t)A[i] * aj;
  const uint32_t q = bcast0<TPI>(((uint32_t)P[S_] * mprime) & LMASK);
#pragma unroll
  for (int i = 0; i < LL; ++i) P[(i + S_) % LL] += (uint64_t)q * m[i];
  const uint64_t v = P[S_];
  P[(S_ + 1) % LL] += v >> LB;
  P[S_] = (uint64_t)dpp_from_next((uint32_t)v & LMASK);
#pragma unroll
  for (int i = 0; i < LL; ++i) asm volatile("" : "+v"(P[i]));
  __builtin_amdgcn_sched_barrier(0);
}
template <int TPI, int LL, int... Ss>
__device__ __forceinline__ void outer1(uint64_t (&P)[LL], const uint32_t (&A)[LL], const uint32_t* __restrict__ Ao,
                                       const uint32_t (&m)[LL], uint32_t mprime, std::integer_sequence<int, Ss...>) {
  uint32_t acur = Ao[0];
  (step1<TPI, LL, Ss>(P, A, Ao, acur, m, mprime), ...);
}
// A <- A X R^-1 mod p (< 2p for A, X < 2p), X = the S limbs at `slot`
template <int TPI, int LL>
__device__ __forceinline__ void montmul1(uint32_t (&A)[LL], const uint32_t* slot, const uint32_t (&m)[LL], uint32_t mprime,
                                         int lane, int tig) {
  uint64_t P[LL];
#pragma unroll
  for (int i = 0; i < LL; ++i) P[i] = 0;
  for (int o = 0; o < TPI; ++o) outer1<TPI, LL>(P, A, slot + o * LL, m, mprime, std::make_integer_sequence<int, LL>{});
  normalize<TPI, LL>(P, A, lane, tig);
}

// canonical pair: A - p + p (B + 1) == A + p B; then B mod p (B <= 2p)
template <int TPI, int LL>
__device__ __forceinline__ void canon(uint32_t (&A)[LL], uint32_t (&B)[LL], const uint32_t (&m)[LL], int lane, int tig) {
  uint32_t d[LL];
  const bool lt = sub_limbs<TPI, LL>(A, m, d, lane, tig);
  uint64_t P[LL];
#pragma unroll
  for (int i = 0; i < LL; ++i) {
    A[i] = lt ? A[i] : d[i];
    P[i] = (uint64_t)B[i] + ((!lt && tig == 0 && i == 0) ? 1u : 0u);
  }
  normalize<TPI, LL>(P, B, lane, tig);
  cond_sub<TPI, LL>(B, m, lane, tig);
  cond_sub<TPI, LL>(B, m, lane, tig);
}

}  // namespace pgrp
}  // namespace fpai
