// p-adic pair arithmetic mod p^2 in one lane (lane engine sizes: S limbs of p, LB = 28).
//
// A residue v mod p^2 is held as a pair (A, B), 0 <= A, B < 2p (S canonical limbs each), with
//   v == A + p B  (mod p^2).
// With R = 2^(LB S) (the radix of p, not of p^2), the CIOS product of the A parts gives
// A1 A2 = U R - m p exactly (U = (A1 A2 + m p) / R, m the q-digits of the reduction), so
//   (A1 + p B1)(A2 + p B2) R^-1 == U + p (A1 B2 + A2 B1 - m) R^-1        (mod p^2)
// and the Montgomery product mod p^2 with radix R is the pair
//   (U, REDC_p(A1 B2 + A2 B1 - m)).
// Both CIOS run in lock-step over the digits j: the second consumes the first's digit q1_j at the
// position where it is produced. Cost 5 S^2 MACs (square: 3.5 S^2) against 2 (2S)^2 (square
// 1.5 (2S)^2) for a Montgomery product over the 2S limbs of p^2: 0.625x (0.58x) of the work, with the
// register footprint of a 2S-limb lane product (A, B: 2S; two accumulators: 4S VGPRs).
//
// Bounds (checked limb by limb in tools/pair_model.py): with R > 8p and operands < 2p, U < 2p and
// REDC(.) < (A1 B2 + A2 B1) / R + p < 2p. The subtraction of q1_j is never executed: the second row picks q2_j
// so that its position J becomes q1_j (mod 2^28) instead of 0 -- q2_j = (P2_J - q1_j) mprime -- and the shift
// that retires position J drops those low 28 bits, which is exactly the subtraction (its value is >= 0 because
// (Z + q2 p) / R > -m / R > -1). So both rows stay non-negative with unsigned carries, and no 64-bit subtraction
// (two instructions and a carry hazard) runs per digit. A position receives per digit at most two a*b products
// and one q2*p product (< 2^57 + 2^57 + 2^56 for a square's doubled digit), so S * 1.25 * 2^58 < 2^64 for S <= 37.
#pragma once
#include "bn_lane.hpp"

#include <type_traits>

namespace fpai {
namespace pair {

using lane::LB;
using lane::LMASK;

// pins every accumulator but position Z, which was just cleared: the compiler then sees the zero and starts
// that position's next sum with a product instead of moving 0 into it first
template <int S, int Z>
__device__ __forceinline__ void pin2(uint64_t (&P1)[S], uint64_t (&P2)[S]) {
#pragma unroll
  for (int i = 0; i < S; ++i)
    if (i != Z) asm volatile("" : "+v"(P1[i]), "+v"(P2[i]));
}

// reductions of digit J: P1 by q1 (its own digit), P2 by q2 with q1 dropped at position J (above)
template <int S, int J>
__device__ __forceinline__ void red2(uint64_t (&P1)[S], uint64_t (&P2)[S], const uint32_t (&m)[S], uint32_t mprime) {
  const uint32_t q1 = ((uint32_t)P1[J] * mprime) & LMASK;
  const uint32_t q2 = (((uint32_t)P2[J] - q1) * mprime) & LMASK;
#pragma unroll
  for (int i = 0; i < S; ++i) {
    P1[(i + J) % S] += (uint64_t)q1 * m[i];
    P2[(i + J) % S] += (uint64_t)q2 * m[i];
  }
  P1[(J + 1) % S] += P1[J] >> LB;
  P2[(J + 1) % S] += P2[J] >> LB;   // its low 28 bits are q1: the subtraction of m
  P1[J] = 0;
  P2[J] = 0;
  pin2<S, J>(P1, P2);
  __builtin_amdgcn_sched_barrier(0);
}

// digit J of a product with the multiplier's digits (a2j, b2j)
template <int S, int J>
__device__ __forceinline__ void mul_digit(uint64_t (&P1)[S], uint64_t (&P2)[S], const uint32_t (&A)[S], const uint32_t (&B)[S],
                                          uint32_t a2j, uint32_t b2j) {
#pragma unroll
  for (int i = 0; i < S; ++i) {
    P1[(i + J) % S] += (uint64_t)A[i] * a2j;
    P2[(i + J) % S] += (uint64_t)B[i] * a2j + (uint64_t)A[i] * b2j;
  }
}

// digit J of a square: upper triangle of A^2, and 2 A B (B's digit doubled)
template <int S, int J>
__device__ __forceinline__ void sqr_digit(uint64_t (&P1)[S], uint64_t (&P2)[S], const uint32_t (&A)[S], const uint32_t (&B)[S]) {
  const uint32_t aj = A[J], aj2 = aj << 1, bj2 = B[J] << 1;
  P1[(2 * J) % S] += (uint64_t)aj * aj;
#pragma unroll
  for (int i = J + 1; i < S; ++i) P1[(i + J) % S] += (uint64_t)A[i] * aj2;
#pragma unroll
  for (int i = 0; i < S; ++i) P2[(i + J) % S] += (uint64_t)A[i] * bj2;
}

template <int S>
__device__ __forceinline__ void zero2(uint64_t (&P1)[S], uint64_t (&P2)[S]) {
#pragma unroll
  for (int i = 0; i < S; ++i) P1[i] = P2[i] = 0;
}

// (A, B) <- (A, B)^2 R^-1
template <int S, int... Js>
__device__ __forceinline__ void sqr_all(uint64_t (&P1)[S], uint64_t (&P2)[S], const uint32_t (&A)[S], const uint32_t (&B)[S],
                                        const uint32_t (&m)[S], uint32_t mprime, std::integer_sequence<int, Js...>) {
  ((sqr_digit<S, Js>(P1, P2, A, B), red2<S, Js>(P1, P2, m, mprime)), ...);
}
template <int S>
__device__ __forceinline__ void mont_sqr(uint32_t (&A)[S], uint32_t (&B)[S], const uint32_t (&m)[S], uint32_t mprime) {
  uint64_t P1[S], P2[S];
  zero2<S>(P1, P2);
  sqr_all<S>(P1, P2, A, B, m, mprime, std::make_integer_sequence<int, S>{});
  lane::normalize<S>(P1, A);
  lane::normalize<S>(P2, B);
}

// (A, B) <- (A, B) (A2, B2) R^-1 with the multiplier's digit pair J from get(J) (a uint2: x = A2[J],
// y = B2[J]); get is called once per digit, in order.
template <int S, int J, class Get>
__device__ __forceinline__ void mul_step(uint64_t (&P1)[S], uint64_t (&P2)[S], const uint32_t (&A)[S], const uint32_t (&B)[S],
                                         Get& get, const uint32_t (&m)[S], uint32_t mprime) {
  const uint2 d = get(std::integral_constant<int, J>{});
  mul_digit<S, J>(P1, P2, A, B, d.x, d.y);
  red2<S, J>(P1, P2, m, mprime);
}
template <int S, class Get, int... Js>
__device__ __forceinline__ void mul_all(uint64_t (&P1)[S], uint64_t (&P2)[S], const uint32_t (&A)[S], const uint32_t (&B)[S],
                                        Get& get, const uint32_t (&m)[S], uint32_t mprime, std::integer_sequence<int, Js...>) {
  (mul_step<S, Js>(P1, P2, A, B, get, m, mprime), ...);
}
template <int S, class Get>
__device__ __forceinline__ void mont_mul(uint32_t (&A)[S], uint32_t (&B)[S], Get&& get, const uint32_t (&m)[S], uint32_t mprime) {
  uint64_t P1[S], P2[S];
  zero2<S>(P1, P2);
  mul_all<S>(P1, P2, A, B, get, m, mprime, std::make_integer_sequence<int, S>{});
  lane::normalize<S>(P1, A);
  lane::normalize<S>(P2, B);
}

// ---- (A, B) <- (A, B)(a, 0) R^-1 in lock-step (the factored decryption chain, kernels_pair.hpp decf_run): both rows
// take the multiplier's one digit a_J, P1 += A a_J, P2 += B a_J (the A1 B2 term is gone), then red2 -- 4 S^2 MACs
// against mont_mul's 5 S^2, one LDS word per digit instead of two, same registers and bounds. get(J) returns a_J.
template <int S, int J, class Get>
__device__ __forceinline__ void mul_b0_step(uint64_t (&P1)[S], uint64_t (&P2)[S], const uint32_t (&A)[S], const uint32_t (&B)[S],
                                            Get& get, const uint32_t (&m)[S], uint32_t mprime) {
  const uint32_t a = get(std::integral_constant<int, J>{});
#pragma unroll
  for (int i = 0; i < S; ++i) {
    P1[(i + J) % S] += (uint64_t)A[i] * a;
    P2[(i + J) % S] += (uint64_t)B[i] * a;
  }
  red2<S, J>(P1, P2, m, mprime);
}
template <int S, class Get, int... Js>
__device__ __forceinline__ void mul_b0_all(uint64_t (&P1)[S], uint64_t (&P2)[S], const uint32_t (&A)[S], const uint32_t (&B)[S],
                                           Get& get, const uint32_t (&m)[S], uint32_t mprime, std::integer_sequence<int, Js...>) {
  (mul_b0_step<S, Js>(P1, P2, A, B, get, m, mprime), ...);
}
template <int S, class Get>
__device__ __forceinline__ void mont_mul_b0(uint32_t (&A)[S], uint32_t (&B)[S], Get&& get, const uint32_t (&m)[S], uint32_t mprime) {
  uint64_t P1[S], P2[S];
  zero2<S>(P1, P2);
  mul_b0_all<S>(P1, P2, A, B, get, m, mprime, std::make_integer_sequence<int, S>{});
  lane::normalize<S>(P1, A);
  lane::normalize<S>(P2, B);
}

// ---- two B-free operands against two pair constants at once: (X1, 0) C1 + (X2, 0) C2, times R^-1 (k_fbp_fin's
// w_q q^-2 = A_q q^-2 + B_q q^-1). Lock-step rows as in mont_mul: P1 += X1 c1a_J + X2 c2a_J, P2 += X1 c1b_J + X2 c2b_J,
// one reduction for both products (6 S^2 MACs, against 4 S^2 + 4 S^2 for two products); per position and digit at most
// two products and one reduction product, within mont_mul's bound. get(J) returns (c1a, c1b, c2a, c2b) of digit J.
template <int S, int J, class Get>
__device__ __forceinline__ void mul2_step(uint64_t (&P1)[S], uint64_t (&P2)[S], const uint32_t (&X1)[S], const uint32_t (&X2)[S],
                                          Get& get, const uint32_t (&m)[S], uint32_t mprime) {
  const uint4 d = get(std::integral_constant<int, J>{});
#pragma unroll
  for (int i = 0; i < S; ++i) {
    P1[(i + J) % S] += (uint64_t)X1[i] * d.x + (uint64_t)X2[i] * d.z;
    P2[(i + J) % S] += (uint64_t)X1[i] * d.y + (uint64_t)X2[i] * d.w;
  }
  red2<S, J>(P1, P2, m, mprime);
}
template <int S, class Get, int... Js>
__device__ __forceinline__ void mul2_all(uint64_t (&P1)[S], uint64_t (&P2)[S], const uint32_t (&X1)[S], const uint32_t (&X2)[S],
                                         Get& get, const uint32_t (&m)[S], uint32_t mprime, std::integer_sequence<int, Js...>) {
  (mul2_step<S, Js>(P1, P2, X1, X2, get, m, mprime), ...);
}
// (X1, X2) <- the pair (U, V) of (X1 C1 + X2 C2) R^-1 mod p^2 (X1, X2 < 2p; C1, C2 canonical pairs): U, V < 2p
template <int S, class Get>
__device__ __forceinline__ void mont_mul2_a0(uint32_t (&X1)[S], uint32_t (&X2)[S], Get&& get, const uint32_t (&m)[S],
                                             uint32_t mprime) {
  uint64_t P1[S], P2[S];
  zero2<S>(P1, P2);
  mul2_all<S>(P1, P2, X1, X2, get, m, mprime, std::make_integer_sequence<int, S>{});
  lane::normalize<S>(P1, X1);
  lane::normalize<S>(P2, X2);
}

// ---- products by a pair (a, 0): a factored table row (kernels_fbp.hpp)
// (A + p B) a R^-1 == U + p REDC(B a - m) (mod p^2): the A1 B2 term is gone, 4 S^2 MACs. Run as two CIOS passes
// over the digits of a -- U = REDC(A a), handing each reduction digit q1_j to put(j, q1_j), then REDC(B a - m),
// m = sum q1_j 2^(28 j), with gb(j) returning (a_j, q1_j) -- so that only one 64-bit accumulator row (2S VGPRs)
// is live at a time; the caller keeps the digits where it has room. Bounds as above (the second pass is the
// second row of the lock-step product with one product per position and digit fewer).
template <int S, int Z>
__device__ __forceinline__ void pin1(uint64_t (&P)[S]) {
#pragma unroll
  for (int i = 0; i < S; ++i)
    if (i != Z) asm volatile("" : "+v"(P[i]));
}

template <int S, int J, class Get, class Put>
__device__ __forceinline__ void a0_step_u(uint64_t (&P)[S], const uint32_t (&A)[S], Get& get, Put& put, const uint32_t (&m)[S],
                                          uint32_t mprime) {
  const uint32_t aj = get(std::integral_constant<int, J>{});
#pragma unroll
  for (int i = 0; i < S; ++i) P[(i + J) % S] += (uint64_t)A[i] * aj;
  const uint32_t q = ((uint32_t)P[J] * mprime) & LMASK;
  put(std::integral_constant<int, J>{}, q);
#pragma unroll
  for (int i = 0; i < S; ++i) P[(i + J) % S] += (uint64_t)q * m[i];
  P[(J + 1) % S] += P[J] >> LB;
  P[J] = 0;
  pin1<S, J>(P);
  __builtin_amdgcn_sched_barrier(0);
}

template <int S, int J, class Get>
__device__ __forceinline__ void a0_step_b(uint64_t (&P)[S], const uint32_t (&B)[S], Get& get, const uint32_t (&m)[S],
                                          uint32_t mprime) {
  const uint2 d = get(std::integral_constant<int, J>{});   // (a_J, q1_J)
#pragma unroll
  for (int i = 0; i < S; ++i) P[(i + J) % S] += (uint64_t)B[i] * d.x;
  const uint32_t q2 = (((uint32_t)P[J] - d.y) * mprime) & LMASK;
#pragma unroll
  for (int i = 0; i < S; ++i) P[(i + J) % S] += (uint64_t)q2 * m[i];
  P[(J + 1) % S] += P[J] >> LB;   // its low 28 bits are q1_J: the subtraction of m
  P[J] = 0;
  pin1<S, J>(P);
  __builtin_amdgcn_sched_barrier(0);
}

template <int S, class Get, class Put, int... Js>
__device__ __forceinline__ void a0_pass_u(uint64_t (&P)[S], const uint32_t (&A)[S], Get& get, Put& put, const uint32_t (&m)[S],
                                          uint32_t mprime, std::integer_sequence<int, Js...>) {
  (a0_step_u<S, Js>(P, A, get, put, m, mprime), ...);
}
template <int S, class Get, int... Js>
__device__ __forceinline__ void a0_pass_b(uint64_t (&P)[S], const uint32_t (&B)[S], Get& get, const uint32_t (&m)[S],
                                          uint32_t mprime, std::integer_sequence<int, Js...>) {
  (a0_step_b<S, Js>(P, B, get, m, mprime), ...);
}

// (A, B) <- (A, B)(a, 0) R^-1 (above)
template <int S, class GetU, class Put, class GetB>
__device__ __forceinline__ void mont_mul_a0(uint32_t (&A)[S], uint32_t (&B)[S], GetU&& ga, Put&& put, GetB&& gb,
                                            const uint32_t (&m)[S], uint32_t mprime) {
  uint64_t P[S];
#pragma unroll
  for (int i = 0; i < S; ++i) P[i] = 0;
  a0_pass_u<S>(P, A, ga, put, m, mprime, std::make_integer_sequence<int, S>{});
  lane::normalize<S>(P, A);
#pragma unroll
  for (int i = 0; i < S; ++i) P[i] = 0;
  a0_pass_b<S>(P, B, gb, m, mprime, std::make_integer_sequence<int, S>{});
  lane::normalize<S>(P, B);
}

// ---- one row: X <- REDC(init + X y) mod p with y's digits from get(J) (a uint32_t), P holding init on entry (< 2^56
// per limb); the factored decryption's closing Horner sum (kernels_pair.hpp decf_run)
template <int S, class Get>
__device__ __forceinline__ void redc_row(uint64_t (&P)[S], uint32_t (&X)[S], Get&& get, const uint32_t (&m)[S], uint32_t mprime) {
  auto nop = [](auto, uint32_t) {};
  a0_pass_u<S>(P, X, get, nop, m, mprime, std::make_integer_sequence<int, S>{});
  lane::normalize<S>(P, X);
}

// (A, B) with A, B < 2p -> the canonical pair A < p, B < p of the same residue mod p^2
// (A - p + p (B + 1) == A + p B)
template <int S>
__device__ __forceinline__ void canon(uint32_t (&A)[S], uint32_t (&B)[S], const uint32_t (&m)[S]) {
  uint32_t d[S];
  const bool lt = lane::sub<S>(A, m, d);
  uint32_t c = lt ? 0u : 1u;
#pragma unroll
  for (int i = 0; i < S; ++i) {
    A[i] = lt ? A[i] : d[i];
    const uint32_t v = B[i] + c;
    B[i] = v & LMASK;
    c = v >> LB;
  }
  lane::cond_sub<S>(B, m);   // B <= 2p
  lane::cond_sub<S>(B, m);
}

}  // namespace pair
}  // namespace fpai
