// Exponentiations mod p_h^2 on p-adic pairs (bn_pair.hpp): CRT decryption (decryptor.py:55-61) and
// stage B of the generic CRT encryption (kernels_crt.hpp), with every square and product mod p_h^2
// done over the S limbs of p_h. A residue is the pair (A, B), v = A + p_h B; the lane machine of
// kernels_crt.hpp runs unchanged on tiles of 2S limbs (A then B: the size of a 2S-limb p_h^2 tile).
//
//   k_dec_pre_pair<S>   c~ = c R mod p_h^2 as a pair: one CIOS over the K S 28-bit digits of the ciphertext
//                       c with the constant pair of R^(K+1) in registers (the pair form of lane::mul_pass)
//   k_dec_pow_pair<S>   x_h = c~^(p_h - 1) * (1, 0) R^-1 = c^(p_h - 1) mod p_h^2 (plain pair)
//   k_dec_fin_pair<S>   canonical pair (A, B) of x_h == 1 mod p_h: A = 1 and L_h = (x_h - 1) // p_h = B
//                       (A = 0, B = 0 for c == 0 mod p_h: L_h = -1, the reference's floor division);
//                       then m_h = L_h h_h mod p_h, CRT and decode exactly as k_dec_fin
//   k_crt_b_pair<S>     u_h = (y R)^(p_h) * coef R^-1 mod p_h^2, written as A + p_h B (k_crt_b's SB limbs)
#pragma once
#include "bn_pair.hpp"
#include "kernels_dec.hpp"
#include "kernels_fbp.hpp"

namespace fpai {

// limb t of the 2S-limb tile image of a pair
template <int S, int T>
__device__ __forceinline__ uint32_t pair_limb(const uint32_t (&A)[S], const uint32_t (&B)[S]) {
  if constexpr (T < S) return A[T];
  else if constexpr (T < 2 * S) return B[T - S];
  else return 0u;
}
template <int S, int G>
__device__ __forceinline__ uint4 pack_pair_quad(const uint32_t (&A)[S], const uint32_t (&B)[S]) {
  return make_uint4(pair_limb<S, 4 * G>(A, B), pair_limb<S, 4 * G + 1>(A, B), pair_limb<S, 4 * G + 2>(A, B),
                    pair_limb<S, 4 * G + 3>(A, B));
}
template <int S, int T>
__device__ __forceinline__ void set_pair_limb(uint32_t (&A)[S], uint32_t (&B)[S], uint32_t v) {
  if constexpr (T < S) A[T] = v;
  else if constexpr (T < 2 * S) B[T - S] = v;
}
template <int S, int G>
__device__ __forceinline__ void unpack_pair_quad(const uint4 v, uint32_t (&A)[S], uint32_t (&B)[S]) {
  set_pair_limb<S, 4 * G>(A, B, v.x);
  set_pair_limb<S, 4 * G + 1>(A, B, v.y);
  set_pair_limb<S, 4 * G + 2>(A, B, v.z);
  set_pair_limb<S, 4 * G + 3>(A, B, v.w);
}
template <int S, int... Gs>
__device__ __forceinline__ void ptile_load(const LaneScratch& t, int k, uint32_t (&A)[S], uint32_t (&B)[S],
                                           std::integer_sequence<int, Gs...>) {
  constexpr int TQ = tile_quads<2 * S>();
  (unpack_pair_quad<S, Gs>(t.quad(k * TQ + Gs), A, B), ...);
}
template <int S, int... Gs>
__device__ __forceinline__ void ptile_store(const LaneScratch& t, int k, const uint32_t (&A)[S], const uint32_t (&B)[S],
                                            std::integer_sequence<int, Gs...>) {
  constexpr int TQ = tile_quads<2 * S>();
  ((t.quad(k * TQ + Gs) = pack_pair_quad<S, Gs>(A, B)), ...);
}
template <int S, int... Gs>
__device__ __forceinline__ void pcol_store(uint4* bcol, const uint32_t (&A)[S], const uint32_t (&B)[S],
                                           std::integer_sequence<int, Gs...>) {
  ((bcol[Gs * LANE_BLOCK] = pack_pair_quad<S, Gs>(A, B)), ...);
}

// The multiplier pair from this lane's LDS column ([quad][lane], 2S limbs: A then B), digit J+1's two
// words read while digit J multiplies.
template <int S>
struct PairLdsDigits {
  const uint4* bcol;
  uint32_t na, nb;
  __device__ __forceinline__ uint32_t word(int t) const {
    return reinterpret_cast<const uint32_t*>(bcol + (t >> 2) * LANE_BLOCK)[t & 3];
  }
  __device__ __forceinline__ explicit PairLdsDigits(const uint4* c) : bcol(c) {
    na = word(0);
    nb = word(S);
  }
  template <int J>
  __device__ __forceinline__ uint2 operator()(std::integral_constant<int, J>) {
    const uint2 r = make_uint2(na, nb);
    if constexpr (J + 1 < S) {
      na = word(J + 1);
      nb = word(S + J + 1);
    }
    return r;
  }
};

// The lane machine of kernels_crt.hpp (run_lane_program) on pairs: same op list and tile indices.
template <int S>
__device__ __forceinline__ void run_pair_program(uint32_t (&A)[S], uint32_t (&B)[S], const LaneScratch& t,
                                                 const uint32_t* __restrict__ prog, int nprog,
                                                 const uint32_t* __restrict__ c1, const uint32_t (&m)[S], uint32_t mprime) {
  constexpr int TQ = tile_quads<2 * S>();
  using Q = std::make_integer_sequence<int, TQ>;
  __shared__ uint4 ldsb[TQ * LANE_BLOCK];
  uint4* bcol = ldsb + threadIdx.x;
  uint4* brow = ldsb + (threadIdx.x & ~63u);
  for (int i = 0; i <= nprog; ++i) {
    const uint32_t op = (i < nprog) ? lane_op(prog, i) : LOP_B_CONST;
    if (op & LOP_A_FROM_T) {
      ptile_load<S>(t, (op >> 16) & 0xFF, A, B, Q{});
#pragma unroll
      for (int j = 0; j < S; ++j) asm volatile("" : "+v"(A[j]), "+v"(B[j]));
    }
    if (op & LOP_SQR) {
      if (op & LOP_PREFETCH) ltile_to_lds<2 * S>(t, (op >> 8) & 0xFF, brow);
      pair::mont_sqr<S>(A, B, m, mprime);
    } else {
      if (op & LOP_B_CONST) {
        uint32_t ca[S], cb[S];
#pragma unroll
        for (int j = 0; j < S; ++j) {
          ca[j] = c1[j];
          cb[j] = c1[S + j];
        }
        pcol_store<S>(bcol, ca, cb, Q{});
      } else if (!(op & LOP_B_READY)) {
        ltile_to_lds<2 * S>(t, (op >> 8) & 0xFF, brow);
      }
      lds_dma_wait();
      pair::mont_mul<S>(A, B, PairLdsDigits<S>(bcol), m, mprime);
    }
    if (op & LOP_STORE) ptile_store<S>(t, op >> 24, A, B, Q{});
    if (op & LOP_B_SET) pcol_store<S>(bcol, A, B, Q{});
  }
}

struct DecPairHalf {
  const uint32_t* p;      // p_h, S limbs
  const uint32_t* cK;     // pair of R^(K+1) mod p_h^2 (2S limbs), K = ciphertext chunks of S limbs
  const uint32_t* hR;     // h_h R mod p_h, S limbs
  const uint32_t* pm1;    // p_h - 1, S limbs
  uint32_t mprime;        // -p_h^-1 mod 2^LB
  uint32_t pad;
};

struct DecPairPreParams {
  const DecPairHalf* halves;   // [2]
  long long n;
  const uint32_t* ct;
  int ct_words;
  int kchunks;
  uint32_t* out;               // [2][2S][n]
};

// one digit of the long CIOS: the constant pair (A, B) in registers times the ciphertext digit cj
template <int S, int J>
__device__ __forceinline__ void pre_step(uint64_t (&P1)[S], uint64_t (&P2)[S], uint32_t (&A)[S], uint32_t (&B)[S],
                                         uint32_t cj, const uint32_t (&m)[S], uint32_t mprime) {
#pragma unroll
  for (int i = 0; i < S; ++i) asm volatile("" : "+v"(A[i]), "+v"(B[i]));   // (else LLVM hoists 64-bit zero-extended copies)
  pair::mul_digit<S, J>(P1, P2, A, B, cj, 0u);
  pair::red2<S, J>(P1, P2, m, mprime);
}
// the ciphertext's 28-bit digits from its words, read one digit ahead (no S-digit array beside the two rows)
struct PreDigits {
  const uint32_t* cw;
  int nw, bit;       // words; bit of the next digit
  uint32_t cur;
  __device__ __forceinline__ uint32_t fetch() {   // (clamped loads and selects: no branch inside the pass)
    const int wi = bit >> 5, sh = bit & 31;
    const uint32_t l = cw[wi < nw ? wi : nw - 1], h = cw[wi + 1 < nw ? wi + 1 : nw - 1];
    const uint64_t lo = wi < nw ? (uint64_t)l : 0ull;
    const uint64_t hi = wi + 1 < nw ? (uint64_t)h : 0ull;
    bit += lane::LB;
    return (uint32_t)(((hi << 32) | lo) >> sh) & lane::LMASK;
  }
  __device__ __forceinline__ uint32_t next() {
    const uint32_t v = cur;
    cur = fetch();
    return v;
  }
};
template <int S, int... Js>
__device__ __forceinline__ void pre_pass(uint64_t (&P1)[S], uint64_t (&P2)[S], uint32_t (&A)[S], uint32_t (&B)[S],
                                         PreDigits& dg, const uint32_t (&m)[S], uint32_t mprime, std::integer_sequence<int, Js...>) {
  (pre_step<S, Js>(P1, P2, A, B, dg.next(), m, mprime), ...);
}

template <int S>
__global__ __launch_bounds__(LANE_BLOCK, 2) void k_dec_pre_pair(DecPairPreParams p) {
  const int half = blockIdx.y;
  const DecPairHalf* H = p.halves + half;
  const uint32_t mprime = H->mprime;
  for (long long i = (long long)blockIdx.x * LANE_BLOCK + threadIdx.x; i < p.n; i += (long long)gridDim.x * LANE_BLOCK) {
    const uint32_t* cw = p.ct + i * p.ct_words;
    uint32_t m[S], A[S], B[S];
#pragma unroll
    for (int j = 0; j < S; ++j) {
      m[j] = (uint32_t)__builtin_amdgcn_readfirstlane(H->p[j]);   // SGPRs (as VGPRs the pass spilled 202 of them)
      A[j] = H->cK[j];
      B[j] = H->cK[S + j];
    }
    uint64_t P1[S], P2[S];
    pair::zero2<S>(P1, P2);
    PreDigits dg{cw, p.ct_words, 0, 0u};
    dg.cur = dg.fetch();
#pragma unroll 1
    for (int k = 0; k < p.kchunks; ++k) pre_pass<S>(P1, P2, A, B, dg, m, mprime, std::make_integer_sequence<int, S>{});
    uint32_t xa[S], xb[S];
    lane::normalize<S>(P1, xa);
    lane::normalize<S>(P2, xb);
#pragma unroll
    for (int j = 0; j < S; ++j) {
      p.out[((size_t)half * 2 * S + j) * p.n + i] = xa[j];
      p.out[((size_t)half * 2 * S + S + j) * p.n + i] = xb[j];
    }
  }
}

// ---- the factored chain (round 5; tools/decf_model.py restates the algebra, tests/test_decf_model.py checks it)
// The window table keeps FULL pairs (a general pair product costs 5 S^2 here against 4 S^2 for a B-free one, so the
// 15 table products stay general), but the chain's multipliers are B-free: entry P_t = a_t (1 + p b_t), the chain
// multiplies by (a_t, 0) (mont_mul_b0) and the dropped factors, 1 + p s with s = sum_t K_t b_t, are restored at the end
// from the chain's own Fermat inverse -- it runs p - 2, so its result's A component is iota = A~^-1 R^2 mod p:
//   Y'       chain over p - 2, multipliers (a_t, 0) (the first load takes the full pair)
//   1 + p G  = mm(mm(Y', (A~, 0)), (1, 0))      (the closing (A~, 0) drops (1 + p u) = (1 + p b_1): slot 1's weight + 1)
//   delta    = REDC(acc iota), acc = Horner over j = 15..0 of c_j = REDC(H_{2j+1} K'_{2j+1}) in w = REDC(iota iota)
//   output   (A, G + delta), B reduced below 2p
// Per 1024-bit p_h: ~170 chain multiplies at 4 S^2 instead of 5 S^2, against 34 one-row passes (2 S^2) of the Horner
// sum and one more product. iota and w live in the lane's LDS column (the multiplier digits read only its A half
// once the chain is over: w at words 0 .. S-1, iota at DECF_IOTA ..), K'_t comes from global memory (uniform), the
// pair (1 + p G) waits in the spare tile DECF_G.
constexpr uint32_t LOP_BFREE = 1u << 15;   // MUL op: the multiplier is the B-free (a_t, 0) of the tile in the column
constexpr int DECF_G = LANE_NTILE;         // spare tile (the lane scratch's staging area): the pair (1 + p G)
template <int S>
constexpr int decf_iota() { return S + 1; }   // column word of iota's limb 0 (limb S - 1 of the A half stays intact)
static_assert(tile_quads<2 * 37>() * 4 >= 37 + 1 + 37 && tile_quads<2 * 19>() * 4 >= 19 + 1 + 19, "iota fits the column");

template <int S>
struct PairLdsDigitA {   // the multiplier's A digits a_J from this lane's LDS column (word J), one ahead
  const uint4* bcol;
  int off;
  uint32_t na;
  __device__ __forceinline__ uint32_t word(int t) const {
    return reinterpret_cast<const uint32_t*>(bcol + (t >> 2) * LANE_BLOCK)[t & 3];
  }
  __device__ __forceinline__ PairLdsDigitA(const uint4* c, int o) : bcol(c), off(o) { na = word(off); }
  template <int J>
  __device__ __forceinline__ uint32_t operator()(std::integral_constant<int, J>) {
    const uint32_t r = na;
    if constexpr (J + 1 < S) na = word(off + J + 1);
    return r;
  }
};
template <int S>
__device__ __forceinline__ void col_put(uint4* bcol, int off, const uint32_t (&x)[S]) {
#pragma unroll
  for (int j = 0; j < S; ++j) reinterpret_cast<uint32_t*>(bcol + ((off + j) >> 2) * LANE_BLOCK)[(off + j) & 3] = x[j];
}
template <int S, int G0, int... Gs>   // the B limbs of a pair tile (limbs S .. 2S-1 of its 2S-limb image)
__device__ __forceinline__ void ptile_load_b(const LaneScratch& t, int k, uint32_t (&B)[S], std::integer_sequence<int, Gs...>) {
  constexpr int TQ = tile_quads<2 * S>();
  uint32_t A[S];
  (unpack_pair_quad<S, G0 + Gs>(t.quad(k * TQ + G0 + Gs), A, B), ...);
}

template <int S>
__device__ __forceinline__ void decf_run(uint32_t (&A)[S], uint32_t (&B)[S], const LaneScratch& t, const uint32_t* __restrict__ prog,
                                         int nprog, const uint32_t* __restrict__ kf, const uint32_t (&m)[S], uint32_t mprime) {
  constexpr int TQ = tile_quads<2 * S>();
  constexpr int IO = decf_iota<S>();
  using Q = std::make_integer_sequence<int, TQ>;
  __shared__ uint4 ldsb[TQ * LANE_BLOCK];
  uint4* bcol = ldsb + threadIdx.x;
  uint4* brow = ldsb + (threadIdx.x & ~63u);
  // the table (ops 0 .. LANE_NTILE - 1: x~^2 into the column, then general products by it), then the chain and the two
  // closing products (squares and B-free products only) -- two loops, so that neither holds three product bodies
  int i = 0;
  for (; i < LANE_NTILE && i < nprog; ++i) {
    const uint32_t op = lane_op(prog, i);
    if (op & LOP_A_FROM_T) {
      ptile_load<S>(t, (op >> 16) & 0xFF, A, B, Q{});
#pragma unroll
      for (int j = 0; j < S; ++j) asm volatile("" : "+v"(A[j]), "+v"(B[j]));
    }
    if (op & LOP_SQR) {
      pair::mont_sqr<S>(A, B, m, mprime);
    } else {
      lds_dma_wait();
      pair::mont_mul<S>(A, B, PairLdsDigits<S>(bcol), m, mprime);
    }
    if (op & LOP_STORE) ptile_store<S>(t, op >> 24, A, B, Q{});
    if (op & LOP_B_SET) pcol_store<S>(bcol, A, B, Q{});
  }
  for (; i < nprog; ++i) {
    const uint32_t op = lane_op(prog, i);
    const int bidx = (op >> 8) & 0x7F;
    if (op & LOP_A_FROM_T) {
      ptile_load<S>(t, (op >> 16) & 0xFF, A, B, Q{});
#pragma unroll
      for (int j = 0; j < S; ++j) asm volatile("" : "+v"(A[j]), "+v"(B[j]));
    }
    if (op & LOP_SQR) {
      if (op & LOP_PREFETCH) ltile_to_lds<2 * S>(t, bidx, brow);
      pair::mont_sqr<S>(A, B, m, mprime);
    } else {
      if (op & LOP_B_CONST) {   // (1, 0): the A half only (iota sits above it)
        uint32_t one[S];
#pragma unroll
        for (int j = 0; j < S; ++j) one[j] = j == 0 ? 1u : 0u;
        col_put<S>(bcol, 0, one);
      } else if (!(op & LOP_B_READY)) {
        ltile_to_lds<2 * S>(t, bidx, brow);
      }
      lds_dma_wait();
      if (op & LOP_IOTA) col_put<S>(bcol, IO, A);   // iota = Y' mod p (after the DMA of the multiplier's tile)
      pair::mont_mul_b0<S>(A, B, PairLdsDigitA<S>(bcol, 0), m, mprime);   // every product here is by a B-free (a_t, 0)
    }
  }
  ptile_store<S>(t, DECF_G, A, B, Q{});   // 1 + p G
  // w = REDC(iota iota) -> the column's A half
  {
    uint32_t X[S];
    PairLdsDigitA<S> rd(bcol, IO);
#pragma unroll
    for (int j = 0; j < S; ++j) X[j] = rd.word(IO + j);
    uint64_t P[S];
#pragma unroll
    for (int j = 0; j < S; ++j) P[j] = 0;
    pair::redc_row<S>(P, X, rd, m, mprime);
    col_put<S>(bcol, 0, X);
  }
  // acc = Horner over j = 15 .. 0 of c_j = REDC(H_{2j+1} K'_j) in w; A holds acc
#pragma unroll 1
  for (int j = LANE_NTILE - 1; j >= 0; --j) {
    uint64_t P[S];
    {
      ptile_load_b<S, S / 4>(t, j, B, std::make_integer_sequence<int, TQ - S / 4>{});
#pragma unroll
      for (int i = 0; i < S; ++i) P[i] = 0;
      uint32_t kd[S];   // K'_j: all S words requested at once (a load per digit would expose S memory latencies)
      const uint32_t* kj = kf + (size_t)j * S;
#pragma unroll
      for (int i = 0; i < S; ++i) kd[i] = kj[i];
      pair::redc_row<S>(P, B, [&](auto J) { return kd[decltype(J)::value]; }, m, mprime);   // c_j
    }
#pragma unroll
    for (int i = 0; i < S; ++i) P[i] = B[i];
    if (j == LANE_NTILE - 1) {
#pragma unroll
      for (int i = 0; i < S; ++i) A[i] = 0;
    }
    pair::redc_row<S>(P, A, PairLdsDigitA<S>(bcol, 0), m, mprime);   // acc = REDC(c_j + acc w)
  }
  {   // delta = REDC(acc iota)
    uint64_t P[S];
#pragma unroll
    for (int i = 0; i < S; ++i) P[i] = 0;
    pair::redc_row<S>(P, A, PairLdsDigitA<S>(bcol, IO), m, mprime);
  }
  // (A_G, G + delta): G, delta < 2p; B reduced below 2p for k_dec_fin_pair
  {
    uint32_t ga[S];
#pragma unroll
    for (int j = 0; j < S; ++j) ga[j] = A[j];
    ptile_load<S>(t, DECF_G, A, B, Q{});
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < S; ++j) {
      const uint32_t v = B[j] + ga[j] + c;
      B[j] = v & lane::LMASK;
      c = v >> lane::LB;
    }
    lane::cond_sub<S>(B, m);
    lane::cond_sub<S>(B, m);
  }
}

// x_h = c~^(p_h - 1) * (1, 0) R^-1: the plain pair of c^(p_h - 1) mod p_h^2. FACTORED: the B-free chain (decf_run, the
// product); otherwise the general chain (run_pair_program; the test build's cross-check)
// Two waves per SIMD (round 5): the allocator then spills ~20 values per chain step that one wave per SIMD keeps in 386
// registers, and the second wave covers those reloads and the reduction digits' dependency chains -- measured on one
// box, 443 -> 412 ms per 1M, 2.31 -> 2.48 M dec/s (profiles/r05_ab_dec_pair_occupancy.txt; k_crt_b_pair, with heavier
// spills, lost 5 % the same way and keeps LANE_OCC).
constexpr int DEC_PAIR_OCC = 2;
// The 1024-bit key's chain (S = 19) at three waves (round 6): 168 VGPRs and 36 spilled against 237 at two waves;
// same box, interleaved x3: 66.1-67.0 -> 63.1-63.5 ms per 1M, 15.5 -> 16.3 M dec/s (profiles/r06r_ab_dec19_occupancy.txt)
#ifndef DEC_PAIR_OCC19
#define DEC_PAIR_OCC19 3
#endif
template <int S, bool FACTORED>
__global__ __launch_bounds__(LANE_BLOCK, S == 19 ? DEC_PAIR_OCC19 : DEC_PAIR_OCC) void k_dec_pow_pair(CrtParams p) {
  const int half = blockIdx.y;
  const CrtHalf* H = p.halves + half;
  uint32_t m[S];
#pragma unroll
  for (int j = 0; j < S; ++j) m[j] = H->m[j];
  const uint32_t mprime = H->mprime;
  const int nprog = H->nprog;
  const uint32_t* prog = H->prog;
  const uint32_t* c1 = H->c1;
  const LaneScratch tl = lane_scratch(p.scratch);
  for (long long base = (long long)blockIdx.x * LANE_BLOCK; base < p.n; base += (long long)gridDim.x * LANE_BLOCK) {
    const long long i = base + threadIdx.x;
    const long long ii = i < p.n ? i : p.n - 1;
    uint32_t A[S], B[S];
#pragma unroll
    for (int j = 0; j < S; ++j) {
      A[j] = p.yin[((size_t)half * 2 * S + j) * p.n + ii];
      B[j] = p.yin[((size_t)half * 2 * S + S + j) * p.n + ii];
    }
    ptile_store<S>(tl, 0, A, B, std::make_integer_sequence<int, tile_quads<2 * S>()>{});
    if constexpr (FACTORED) decf_run<S>(A, B, tl, prog, nprog, H->c0, m, mprime);
    else run_pair_program<S>(A, B, tl, prog, nprog, c1, m, mprime);
    if (i < p.n) {
#pragma unroll
      for (int j = 0; j < S; ++j) {
        p.out[((size_t)half * 2 * S + j) * p.n + i] = A[j];
        p.out[((size_t)half * 2 * S + S + j) * p.n + i] = B[j];
      }
    }
  }
}

// m_h = L(x_h, p_h) h_h mod p_h from the plain pair of x_h (decryptor.py:55-61, keypair.py:81-90)
template <int S>
__device__ __forceinline__ void dec_half_pair(const DecPairHalf* __restrict__ H, const uint32_t* __restrict__ xh, long long n,
                                              long long i, uint32_t (&mh)[S]) {
  uint32_t A[S], pl[S];
#pragma unroll
  for (int j = 0; j < S; ++j) {
    A[j] = xh[(size_t)j * n + i];
    mh[j] = xh[(size_t)(S + j) * n + i];
    pl[j] = H->p[j];
  }
  pair::canon<S>(A, mh, pl);   // x_h = A + p_h mh, A, mh < p_h
  uint32_t nz = 0;
#pragma unroll
  for (int j = 0; j < S; ++j) nz |= A[j];
  if (nz == 0) {   // x_h == 0 mod p_h: L = floor((p_h mh - 1) / p_h) = mh - 1 (mod p_h)
    uint32_t one[S];
#pragma unroll
    for (int j = 0; j < S; ++j) one[j] = j == 0 ? 1u : 0u;
    uint32_t d[S];
    const bool neg = lane::sub<S>(mh, one, d);
#pragma unroll
    for (int j = 0; j < S; ++j) mh[j] = neg ? H->pm1[j] : d[j];
  }
  uint32_t hb[S];
#pragma unroll
  for (int j = 0; j < S; ++j) hb[j] = H->hR[j];
  lane::mont_mul<S>(mh, hb, pl, H->mprime);   // L_h h_h mod p_h (< 2 p_h)
  lane::cond_sub<S>(mh, pl);
}

struct DecPairFinParams {
  const DecPairHalf* halves;  // [2]
  long long n;
  const uint32_t* xh;         // [2][2S][n] plain pairs of c^(p_h - 1) mod p_h^2
  const int32_t* exp;
  const uint32_t* p;          // S limbs
  const uint32_t* q;
  const uint32_t* qinvR;      // q^-1 R mod p
  uint32_t pprime;
  const uint32_t* nlimb;      // n, 2S limbs
  const uint32_t* maxint;     // n // 3 - 1, 2S limbs
  double* val;
  int64_t* mant;
  int32_t* status;
  uint32_t* raw;
  int pt_words;
};

template <int S>
__global__ __launch_bounds__(LANE_BLOCK) void k_dec_fin_pair(DecPairFinParams p) {
  constexpr int SA = S, SB = 2 * S;
  for (long long i = (long long)blockIdx.x * LANE_BLOCK + threadIdx.x; i < p.n; i += (long long)gridDim.x * LANE_BLOCK) {
    uint32_t mp[SA], mq[SA], pl[SA];
    dec_half_pair<S>(p.halves, p.xh, p.n, i, mp);
    dec_half_pair<S>(p.halves + 1, p.xh + (size_t)SB * p.n, p.n, i, mq);
#pragma unroll
    for (int j = 0; j < SA; ++j) pl[j] = p.p[j];
    // u = (mp - mq) q^-1 mod p
    uint32_t a1[SA], a2[SA], qi[SA], u[SA];
#pragma unroll
    for (int j = 0; j < SA; ++j) {
      qi[j] = p.qinvR[j];
      a1[j] = mp[j];
      a2[j] = mq[j];
    }
    lane::mont_mul<SA>(a1, qi, pl, p.pprime);
    lane::cond_sub<SA>(a1, pl);
    lane::mont_mul<SA>(a2, qi, pl, p.pprime);
    lane::cond_sub<SA>(a2, pl);
    {
      const bool neg = lane::sub<SA>(a1, a2, u);
      uint64_t c = 0;
#pragma unroll
      for (int j = 0; j < SA; ++j) {
        const uint64_t v = (uint64_t)u[j] + (neg ? pl[j] : 0u) + c;
        u[j] = (uint32_t)v & lane::LMASK;
        c = v >> lane::LB;
      }
    }
    // x = mq + u q (< n)
    uint32_t x[SB];
    {
      uint64_t X[SB];
#pragma unroll
      for (int k = 0; k < SB; ++k) X[k] = k < SA ? (uint64_t)mq[k] : 0ull;
#pragma unroll
      for (int j = 0; j < SA; ++j) {
        const uint32_t qj = p.q[j];
#pragma unroll
        for (int t = 0; t < SA; ++t) X[t + j] += (uint64_t)u[t] * qj;
      }
      lane::normalize<SB>(X, x);
    }
    uint32_t nl[SB], mx[SB];
#pragma unroll
    for (int k = 0; k < SB; ++k) {
      nl[k] = p.nlimb[k];
      mx[k] = p.maxint[k];
    }
    double val;
    int64_t mant;
    int st;
    decode_lane<SB>(x, nl, mx, p.exp[i], val, mant, st);
    p.val[i] = val;
    if (p.mant) p.mant[i] = mant;
    p.status[i] = st;
    if (p.raw) {
      uint32_t* out = p.raw + i * p.pt_words;
#pragma unroll
      for (int w = 0; w < (SB * lane::LB + 31) / 32; ++w) {
        const int bit = 32 * w, k = bit / lane::LB, sh = bit - k * lane::LB;
        uint64_t v = (uint64_t)x[k] >> sh;
        if (k + 1 < SB) v |= (uint64_t)x[k + 1] << (lane::LB - sh);
        if (k + 2 < SB && 2 * lane::LB - sh < 32) v |= (uint64_t)x[k + 2] << (2 * lane::LB - sh);
        if (w < p.pt_words) out[w] = (uint32_t)v;
      }
    }
  }
}

// ---------------------------------------------------------------- CRT encryption, stage B on pairs
// u_h = (y R)^(p_h) * coef R^-1 mod p_h^2 from y (stage A, < 2 p_h): (y, 0) * pair(R^2) R^-1 = y R, the lane
// machine with the exponent p_h, the final product with the pair of coef; out as A + p_h B, SB limbs.
template <int S>
__global__ __launch_bounds__(LANE_BLOCK, LANE_OCC) void k_crt_b_pair(CrtParams p) {
  constexpr int SB = FbpGeom<S>::SB;   // limbs of u_h < 2 p_h^2 (k_crt_fin's layout)
  const int half = blockIdx.y;
  const CrtHalf* H = p.halves + half;
  uint32_t m[S];
#pragma unroll
  for (int j = 0; j < S; ++j) m[j] = H->m[j];
  const uint32_t mprime = H->mprime;
  const int nprog = H->nprog;
  const uint32_t* prog = H->prog;
  const uint32_t* c1 = H->c1;
  const uint32_t* c0 = H->c0;
  const LaneScratch tl = lane_scratch(p.scratch);
  for (long long base = (long long)blockIdx.x * LANE_BLOCK; base < p.n; base += (long long)gridDim.x * LANE_BLOCK) {
    const long long i = base + threadIdx.x;
    const long long ii = i < p.n ? i : p.n - 1;
    uint32_t A[S], B[S];
#pragma unroll
    for (int j = 0; j < S; ++j) {
      A[j] = p.yin[((size_t)half * S + j) * p.n + ii];
      B[j] = 0u;
    }
    pair::mont_mul<S>(A, B, [&](auto J) { return make_uint2(c0[decltype(J)::value], c0[S + decltype(J)::value]); }, m,
                      mprime);                                      // y R
    ptile_store<S>(tl, 0, A, B, std::make_integer_sequence<int, tile_quads<2 * S>()>{});
    run_pair_program<S>(A, B, tl, prog, nprog, c1, m, mprime);     // y^(p_h) coef
    if (i < p.n) {
      pair::canon<S>(A, B, m);
      fbp_store_w<S, SB>(A, B, m, p.out + (size_t)half * SB * p.n + i, p.n, std::make_integer_sequence<int, SB>{});
    }
  }
}

}  // namespace fpai
