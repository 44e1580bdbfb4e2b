// Fixed-base sampler on split pairs (round 3): kernels_dec4.hpp's lane-pair layout for the two 2048-bit-modulus
// samplers that ran on TPI = 4 pair groups -- the 4096-bit key holder's w_h = c0 G_h^(a_h) mod p_h^2 (k_fbgp,
// kernels_grp_pair.hpp) and the public-key r^n = prod_j h_j^(e_j) mod n^2 (k_pfb, kernels_pfb.hpp). Same tables
// (factored rows a (1 + m b), kernels_grp_pair.hpp), same digits, same canonical pairs out, so k_fbgp_w / Garner
// and k_pe_fin follow unchanged and the ciphertexts are bit-identical.
//
// Element e on lanes 2e, 2e+1: the even lane keeps A, the odd lane B, each in registers (74 limbs), and one product
// by a row (a, 0) is ONE split CIOS pass over the row's 74 digits on both lanes:
//   even: A' = REDC(A a)            (reduction digit q1_j)
//   odd : B' = REDC(B a - m)        (m = the even lane's q1 stream, taken by DPP and dropped by the retiring
//                                    shift, bn_pair.hpp)
// i.e. 2 S^2 lane-MACs per lane and 4 S^2 per element, with S = 74 against the group engine's 76 and none of its
// per-digit cross-lane traffic. The row's a half streams HBM -> LDS by DMA (the one LDS operand, read as 28-bit
// digits straight from its 32-bit words); its b half goes to registers and into the pair's running sum in LDS.
//
// Montgomery radix: this engine's R' = 2^(28 74) while the rows hold T R with R = 2^(28 76) (the table builders run
// on the group engine), so every product leaves a factor 2^56. The start value absorbs all K of them: the pair
// c0 C with C = 2^(-56 K) mod m^2 -- (C_A, C_B + gamma C_A) for c0 = (1, gamma), from constants precomputed on
// the host -- and the b-sum correction REDC'(A sum_k b_k R) = A bs 2^56 is divided by 2^56 (two zero-digit REDC
// steps) before the odd lane adds it.
#pragma once
#include "kernels_dec4.hpp"   // (and kernels_fb.hpp: opaque_uniform)
#include "kernels_grp_pair.hpp"

namespace fpai {

constexpr int SGP_S = 74;                      // limbs of the modulus (p_h of a 4096-bit key, a 2048-bit n)
constexpr int SGP_PAIRS = LANE_BLOCK / 2;      // elements per block
constexpr int SGP_AW = FBGP_PW;                // 32-bit words of a row's a half
constexpr int SGP_GROUP = 4 * SGP_AW + 16;     // LDS words per DMA group of 4 pairs (+16: bank offset per group)
constexpr int SGP_WAVE_ROWS = 8 * SGP_GROUP;   // per wave (32 pairs)
constexpr int SGP_BW = FBGP_PW + 4;            // words of a pair's b sum (< 2^(32 PW + 9)), 16-B aligned
static_assert(LB * (FBGP_S - SGP_S) == 56, "radix gap of the tables");

struct SgpHalf {
  const uint4* table;      // [K][2^W] factored rows of FBGP_ROW4 uint4 (T R mod m^2, R = 2^(28 FBGP_S))
  const uint32_t* p;       // modulus m, S limbs
  const uint32_t* ca;      // C mod m, C = 2^(-56 K) mod m^2
  const uint32_t* cb;      // C div m
  const uint32_t* nmc;     // [4][S]: w 2^(16 c) C_A mod m (gamma = w |M|; w = n / p_h, or 1 for the public n)
  const uint32_t* pbig;    // 2^20 m
  uint32_t mprime;         // -m^-1 mod 2^28
};

struct SgpParams {
  const SgpHalf* halves;   // [gridDim.y]
  long long n;
  int K, W;
  const uint32_t* digits;  // [gridDim.y][K][n]
  uint32_t* out;           // [gridDim.y][2 S][n]: the pair [A: S][B: S], A < 2m, B < 4m
  const void* x;
  int dtype, exp_mode, fexp;
  int32_t* exp;            // written by half 0
  int32_t* status;
  GuardArgs g;             // test build (guard.hpp): rows = K 2^W, digits = halves K n, out = halves 2 S n
};

// LDS word of a row's a half: DMA group g = pair >> 2 at g SGP_GROUP; within it word w of pair j = pair & 3 at
// 16 (w >> 2) + 4 j + (w & 3) (lane L of a DMA instruction fetches 16 B of pair L & 3, column L >> 2), so the four
// pairs of a group read a digit from four different banks.
template <bool SWZ>
constexpr int sgp_word_off(int w) { return SWZ ? 16 * (w >> 2) + (w & 3) : w; }

// 28-bit digit J of a little-endian word array (NW words, zero beyond)
template <int NW, bool SWZ, int J>
__device__ __forceinline__ uint32_t sgp_digit(const uint32_t* w) {
  constexpr int b = LB * J, i = b >> 5, o = b & 31;
  const uint32_t lo = i < NW ? w[sgp_word_off<SWZ>(i)] : 0u;
  if constexpr (o + LB <= 32) {
    return (lo >> o) & LMASK;
  } else {
    const uint32_t hi = i + 1 < NW ? w[sgp_word_off<SWZ>(i + 1)] : 0u;
    return __builtin_amdgcn_alignbit(hi, lo, (uint32_t)o) & LMASK;
  }
}

// digit J of the split pass (kernels_dec4.hpp d4_step, digits cut from words)
template <int S, int NW, bool SWZ, int J>
__device__ __forceinline__ void sgp_step(uint64_t (&P)[S], const uint32_t (&a)[S], const uint32_t* __restrict__ w, uint32_t& cur,
                                         const uint32_t (&m)[S], uint32_t mprime, bool odd) {
  const uint32_t y = cur;
  if constexpr (J + 1 < S) cur = sgp_digit<NW, SWZ, J + 1>(w);
#pragma unroll
  for (int i = 0; i < S; ++i) P[(i + J) % S] += (uint64_t)a[i] * y;
  const uint32_t q0 = ((uint32_t)P[J] * mprime) & LMASK;
  const uint32_t q1 = __builtin_amdgcn_update_dpp(0u, q0, 0xA0, 0xF, 0xF, false);   // the even lane's q
  const uint32_t q = (((uint32_t)P[J] - (odd ? q1 : 0u)) * mprime) & LMASK;
#pragma unroll
  for (int i = 0; i < S; ++i) P[(i + J) % S] += (uint64_t)q * m[i];
  P[(J + 1) % S] += P[J] >> LB;   // odd lane: the low 28 bits are q1, dropped
  P[J] = 0;
  lane::pin<S>(P);
  __builtin_amdgcn_sched_barrier(0);
}
template <int S, int NW, bool SWZ, int... Js>
__device__ __forceinline__ void sgp_pass(uint64_t (&P)[S], const uint32_t (&a)[S], const uint32_t* __restrict__ w,
                                         const uint32_t (&m)[S], uint32_t mprime, bool odd, std::integer_sequence<int, Js...>) {
  uint32_t cur = sgp_digit<NW, SWZ, 0>(w);
  (sgp_step<S, NW, SWZ, Js>(P, a, w, cur, m, mprime, odd), ...);
}

// the a halves of the wave's 32 rows of product k -> LDS (8 DMA instructions of 1 KB, 4 pairs each); lane L of
// instruction g fetches column L >> 2 of pair 4 g + (L & 3), whose row index it takes from that pair's even lane
__device__ __forceinline__ void sgp_rows_dma(const uint4* __restrict__ table, size_t k, int W, uint32_t d,
                                             const uint32_t* wave_rows, int lane, GuardArgs gd) {
  typedef __attribute__((address_space(3))) uint32_t lds_u32;
  const uint32_t lb = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(lds_u32*)wave_rows);
  const size_t kb = k << W;
  int ln = lane;
  asm volatile("" : "+v"(ln));   // (lane-derived offsets recomputed here, not kept live across the products)
  const int col = ln >> 2, jj = ln & 3;
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    const uint32_t dg = (uint32_t)__builtin_amdgcn_ds_bpermute((8 * g + 2 * jj) * 4, (int)d);
    const uint4* src = table + FPAI_GUARD_IDX(gd, GS_SGP_ROW, kb + dg, gd.rows, (long long)k) * FBGP_ROW4 + col;
    uint32_t dst = lb + (uint32_t)(g * SGP_GROUP * 4);
    asm volatile("" : "+s"(dst));
    __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(size_t)dst, 16, 0, 0);
  }
}

// this lane's 32 words of the row's b half (b R words [32 tig, 32 tig + 32))
__device__ __forceinline__ void sgp_b_load(const uint4* __restrict__ table, size_t k, int W, uint32_t d, int tig, uint4 (&bv)[8],
                                           GuardArgs gd) {
  const uint4* src = table + FPAI_GUARD_IDX(gd, GS_SGP_ROW, (k << W) + d, gd.rows, (long long)k) * FBGP_ROW4 + (FBGP_PW / 4) + 8 * tig;
#pragma unroll
  for (int q = 0; q < 8; ++q) bv[q] = src[q];
}

// bs[32 tig, 32 tig + 32) += the lane's b words; the carry out counts in cc (enters at word 32 (tig + 1))
__device__ __forceinline__ void sgp_bsum_add(uint32_t* bs, const uint4 (&bv)[8], int tig, uint32_t& cc) {
  uint4* acc = reinterpret_cast<uint4*>(bs) + 8 * tig;
  uint32_t w[32], a[32];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const uint4 u = acc[q];
    a[4 * q] = u.x, a[4 * q + 1] = u.y, a[4 * q + 2] = u.z, a[4 * q + 3] = u.w;
    w[4 * q] = bv[q].x, w[4 * q + 1] = bv[q].y, w[4 * q + 2] = bv[q].z, w[4 * q + 3] = bv[q].w;
  }
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    uint32_t co;
    a[i] = __builtin_addc(a[i], w[i], c, &co);
    c = co;
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) acc[q] = make_uint4(a[4 * q], a[4 * q + 1], a[4 * q + 2], a[4 * q + 3]);
  cc += c;
}

// z <- z 2^-56 mod m: two REDC steps with zero digits (z < 2p in, < 2p out)
template <int S>
__device__ __forceinline__ void sgp_div56(uint32_t (&z)[S], const uint32_t (&m)[S], uint32_t mprime) {
  uint64_t Q[S];
#pragma unroll
  for (int i = 0; i < S; ++i) Q[i] = z[i];
#pragma unroll
  for (int J = 0; J < 2; ++J) {
    const uint32_t q = ((uint32_t)Q[J] * mprime) & LMASK;
#pragma unroll
    for (int i = 0; i < S; ++i) Q[(i + J) % S] += (uint64_t)q * m[i];
    Q[J + 1] += Q[J] >> LB;
    Q[J] = 0;
  }
  uint64_t R[S];
#pragma unroll
  for (int i = 0; i < S; ++i) R[i] = Q[(i + 2) % S];   // limb i of the quotient
  lane::normalize<S>(R, z);
}

#if FLEXPAI_XCHECK
// test build (guard.hpp): digit k of element ee in half h, its offset and value checked
__device__ __forceinline__ uint32_t sgp_guard_digit(const SgpParams& p, int h, int k, long long ee) {
  const uint32_t d = p.digits[FPAI_GUARD_IDX(p.g, GS_SGP_DIGIT, ((size_t)h * p.K + k) * p.n + ee, p.g.digits, ee)];
  return (uint32_t)FPAI_GUARD_IDX(p.g, GS_SGP_DVAL, d, 1ull << p.W, ee);
}
#define SGP_DIGIT(k) sgp_guard_digit(p, half, (k), ee)
#else
#define SGP_DIGIT(k) dg[(size_t)(k) * p.n]
#endif

template <int S>
__global__ __launch_bounds__(LANE_BLOCK, 2) void k_sgp(SgpParams p) {
  __shared__ __attribute__((aligned(16))) uint32_t rows[(LANE_BLOCK / 64) * SGP_WAVE_ROWS];
  __shared__ __attribute__((aligned(16))) uint32_t bsum[SGP_PAIRS * SGP_BW];
  const int half = blockIdx.y;
  const SgpHalf* H = p.halves + half;
  uint32_t m[S];
#pragma unroll
  for (int j = 0; j < S; ++j) m[j] = H->p[j];
  const uint32_t mprime = H->mprime;
  const int lane = threadIdx.x & 63;
  const int tig = threadIdx.x & 1;
  const bool odd = tig != 0;
  const int pib = threadIdx.x >> 1;
  const int pw = pib & 31;   // pair within the wave
  const uint32_t* wave_rows = rows + (threadIdx.x >> 6) * SGP_WAVE_ROWS;
  const uint32_t* my_row = wave_rows + (pw >> 2) * SGP_GROUP + 4 * (pw & 3);
  uint32_t* bs = bsum + pib * SGP_BW;
  const uint4* table = H->table;
  const int K = p.K, W = p.W;
  for (long long base = (long long)blockIdx.x * SGP_PAIRS; base < p.n; base += (long long)gridDim.x * SGP_PAIRS) {
    const long long e = base + pib;
    const bool valid = e < p.n;
    const long long ee = valid ? e : p.n - 1;
    int64_t M = 0;
    int ex = 0, stt;
    const bool fixed = p.exp_mode != 0;
    if (p.dtype == 0) stt = encode_float((double)((const float*)p.x)[ee], fixed, p.fexp, M, ex);
    else if (p.dtype == 1) stt = encode_float(((const double*)p.x)[ee], fixed, p.fexp, M, ex);
    else stt = encode_int(((const int64_t*)p.x)[ee], fixed, p.fexp, M, ex);
    if (half == 0 && valid && !odd) {
      p.exp[e] = ex;
      if (p.status) p.status[e] = stt;
    }
    // the start: c0 C = (C_A, C_B + gamma C_A); gamma C_A = sum_c nmc_c |M|_c (16-bit chunks, < 2^18 m), negative
    // M: 2^20 m - that sum
    uint32_t x[S];
    {
      const bool neg = M < 0;
      const uint64_t mag = neg ? (uint64_t)0 - (uint64_t)M : (uint64_t)M;
      // (opaque pointers: the constants are re-read per element, not hoisted out of the loop into SGPRs)
      const uint32_t* nmc = opaque_uniform(H->nmc);
      const uint32_t* pbg = opaque_uniform(H->pbig);
      const uint32_t* cbg = opaque_uniform(H->cb);
      const uint32_t* cag = opaque_uniform(H->ca);
      uint64_t P[S];
#pragma unroll
      for (int i = 0; i < S; ++i) {
        uint64_t v = 0;
#pragma unroll
        for (int c = 0; c < 4; ++c) v += (uint64_t)nmc[c * S + i] * ((uint32_t)(mag >> (16 * c)) & 0xFFFFu);
        P[i] = v;
      }
      uint32_t Xs[S], D[S], pb[S];
      lane::normalize<S>(P, Xs);
#pragma unroll
      for (int i = 0; i < S; ++i) pb[i] = pbg[i];
      (void)lane::sub<S>(pb, Xs, D);
#pragma unroll
      for (int i = 0; i < S; ++i) P[i] = (uint64_t)cbg[i] + (neg ? D[i] : Xs[i]);
      lane::normalize<S>(P, Xs);
#pragma unroll
      for (int i = 0; i < S; ++i) x[i] = odd ? Xs[i] : cag[i];
    }
    const uint32_t* dg = p.digits + (size_t)half * K * p.n + ee;
    (void)dg;
    wave_lds_fence();   // the previous element's reads of rows / bs are done
    for (int i = tig; i < SGP_BW; i += 2) bs[i] = 0u;
    uint32_t cc = 0;
    uint4 bv[8];
    {
      const uint32_t d0 = SGP_DIGIT(0);
      sgp_rows_dma(table, 0, W, d0, wave_rows, lane, p.g);
      sgp_b_load(table, 0, W, d0, tig, bv, p.g);
    }
    uint32_t dn = K > 1 ? SGP_DIGIT(1) : 0u;
    for (int k = 0; k < K; ++k) {
      lds_dma_wait();   // row k's a half in LDS, its b words in bv, digit k+1 in dn
      sgp_bsum_add(bs, bv, tig, cc);
      uint64_t P[S];
#pragma unroll
      for (int i = 0; i < S; ++i) P[i] = 0;
      sgp_pass<S, SGP_AW, true>(P, x, my_row, m, mprime, odd, std::make_integer_sequence<int, S>{});
      if (k + 1 < K) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the rows are consumed before they are overwritten
        sgp_rows_dma(table, (size_t)(k + 1), W, dn, wave_rows, lane, p.g);
      }
      __builtin_amdgcn_sched_barrier(0);
      lane::normalize<S>(P, x);
      __builtin_amdgcn_sched_barrier(0);
      if (k + 1 < K) {   // (after the normalization: the b words do not share registers with P)
        sgp_b_load(table, (size_t)(k + 1), W, dn, tig, bv, p.g);
        dn = k + 2 < K ? SGP_DIGIT(k + 2) : 0u;
      } else {           // (defined on every path, or bv stays live -- and spilled -- across the product)
#pragma unroll
        for (int q = 0; q < 8; ++q) bv[q] = make_uint4(0u, 0u, 0u, 0u);
      }
    }
    // the b sum: lane 1's carry count enters at word 64, lane 0's at word 32 (rippling through lane 1's words)
    wave_lds_fence();
    if (odd) bs[2 * 32] = cc;
    wave_lds_fence();
    if (!odd) {
      uint64_t c = cc;
      for (int w = 32; c != 0 && w < SGP_BW; ++w) {
        const uint64_t v = (uint64_t)bs[w] + c;
        bs[w] = (uint32_t)v;
        c = v >> 32;
      }
    }
    wave_lds_fence();
    // B += A bs: z = REDC'(A bs R) 2^-56 on the even lane (the odd lane's pass is discarded), taken by DPP
    {
      uint64_t P[S];
#pragma unroll
      for (int i = 0; i < S; ++i) P[i] = 0;
      sgp_pass<S, SGP_BW, false>(P, x, bs, m, mprime, false, std::make_integer_sequence<int, S>{});
      uint32_t z[S];
      lane::normalize<S>(P, z);
      sgp_div56<S>(z, m, mprime);
      uint32_t c = 0;   // (32-bit carries: a 64-bit view of x here turns every limb of x into a register pair)
#pragma unroll
      for (int j = 0; j < S; ++j) {
        const uint32_t zb = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)z[j], 0xA0, 0xF, 0xF, false);
        const uint32_t v = x[j] + (odd ? zb : 0u) + c;
        x[j] = v & LMASK;
        c = v >> LB;
      }   // A < 2p (even), B < 4p (odd): what k_fbgp_w and k_pe_fin take
    }
    if (valid && FPAI_GUARD_OK(p.g, GS_SGP_OUT, ((size_t)half * 2 * S + tig * S + S - 1) * p.n + e, p.g.out, e)) {
#pragma unroll
      for (int i = 0; i < S; ++i) p.out[((size_t)half * 2 * S + tig * S + i) * p.n + e] = x[i];
    }
  }
}

// ---------------------------------------------------------------- the pairs -> w_h for Garner (nb = 4096)
// w_h = A + p_h B mod p_h^2 from k_sgp's pair (A < 2p, B < 4p), in place in the [half][2S][n] rows: the pair made
// canonical (A < p, B < p: A's multiple of p moved into B, then B mod p), then A + p_h B < p_h^2 by product scanning
// -- one lane per element-half, p_h and B in VGPRs, A's limbs read as their columns come (A - f p_h, f = [A >= p_h],
// with its borrow chain on the way), the limbs of w written as they complete (row c of w replaces row c of the pair,
// read by then). S^2 plain MACs per element-half (round 5: in place of k_fbgp_w's Montgomery product mod p_h^2 on the
// TPI = 4 group engine, 4 S^2 plus cross-lane traffic).
template <int S, int C, int I>
__device__ __forceinline__ void sgpw_mac(uint64_t& acc, const uint32_t (&b)[S], const uint32_t (&m)[S]) {
  if constexpr (C - I >= 0 && C - I < S) acc += (uint64_t)b[I] * m[C - I];
}
template <int S, int C, int... Is>
__device__ __forceinline__ void sgpw_col(uint64_t& acc, const uint32_t (&b)[S], const uint32_t (&m)[S], std::integer_sequence<int, Is...>) {
  (sgpw_mac<S, C, Is>(acc, b, m), ...);
}
typedef __attribute__((address_space(1))) uint32_t sgpw_g32;   // (global, not flat: a pointer through an asm stays global)
template <int S, int C>
__device__ __forceinline__ void sgpw_step(uint64_t& acc, int32_t& br, uint32_t fm, const uint32_t (&b)[S], const uint32_t (&m)[S],
                                          sgpw_g32*& out, size_t stride) {
  if constexpr (C < S) {   // limb C of A - f p_h (>= 0 as a whole), read from the row that w's limb C replaces
    const int32_t v = (int32_t)*out - (int32_t)(m[C] & fm) + br;
    br = v >> LB;
    acc += (uint32_t)v & LMASK;
  }
  sgpw_col<S, C>(acc, b, m, std::make_integer_sequence<int, S>{});
  *out = (uint32_t)acc & LMASK;
  out += stride;
  asm volatile("" : "+v"(out));   // (one running address: 2S precomputed 64-bit offsets would not fit)
  acc >>= LB;
}
template <int S, int... Cs>
__device__ __forceinline__ void sgpw_all(uint32_t fm, const uint32_t (&b)[S], const uint32_t (&m)[S], sgpw_g32* out, size_t stride,
                                         std::integer_sequence<int, Cs...>) {
  uint64_t acc = 0;
  int32_t br = 0;
  (sgpw_step<S, Cs>(acc, br, fm, b, m, out, stride), ...);
}
// x >= m over S canonical limbs
template <int S>
__device__ __forceinline__ bool sgpw_ge(const uint32_t (&x)[S], const uint32_t (&m)[S]) {
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < S; ++i) c = ((int32_t)x[i] - (int32_t)m[i] + c) >> LB;
  return c == 0;
}

template <int S>
__global__ __launch_bounds__(LANE_BLOCK, 2) void k_sgp_w(SgpParams p) {
  const int half = blockIdx.y;
  const SgpHalf* H = p.halves + half;
  uint32_t m[S];
#pragma unroll
  for (int j = 0; j < S; ++j) {
    m[j] = H->p[j];
    asm volatile("" : "+v"(m[j]));   // VGPRs (in SGPRs, with the rest, 53 spilled and every use became a readlane)
  }
  const size_t stride = (size_t)p.n;
  for (long long e = (long long)blockIdx.x * LANE_BLOCK + threadIdx.x; e < p.n; e += (long long)gridDim.x * LANE_BLOCK) {
    sgpw_g32* col = (sgpw_g32*)(p.out + (size_t)half * 2 * S * stride + e);
    // the pair's rows, all loads issued before the first use; f = [A >= p_h] (A then dropped: its limbs are read
    // again, from L1/L2, as the product's columns come)
    uint32_t b[S];
    uint32_t f;
    {
      const sgpw_g32* r = col;
#pragma unroll
      for (int i = 0; i < S; ++i) {
        b[i] = *r;
        r += stride;
        asm volatile("" : "+v"(r));
      }
      int32_t c = 0;
#pragma unroll
      for (int i = 0; i < S; ++i) c = ((int32_t)b[i] - (int32_t)m[i] + c) >> LB;
      f = c == 0 ? 1u : 0u;
#pragma unroll
      for (int i = 0; i < S; ++i) {
        b[i] = *r;
        r += stride;
        asm volatile("" : "+v"(r));
      }
    }
    {   // B + f, then B mod p_h (B + f <= 4 p_h)
      uint32_t cy = f;
#pragma unroll
      for (int i = 0; i < S; ++i) {
        const uint32_t v = b[i] + cy;
        b[i] = v & LMASK;
        cy = v >> LB;
      }
    }
#pragma unroll 1
    for (int rep = 0; rep < 4; ++rep) {
      const uint32_t fm = sgpw_ge<S>(b, m) ? LMASK : 0u;
      int32_t br = 0;
#pragma unroll
      for (int i = 0; i < S; ++i) {
        const int32_t v = (int32_t)b[i] - (int32_t)(m[i] & fm) + br;
        b[i] = (uint32_t)v & LMASK;
        br = v >> LB;
      }
    }
    sgpw_all<S>(f ? LMASK : 0u, b, m, col, stride, std::make_integer_sequence<int, 2 * S>{});
  }
}

// ---------------------------------------------------------------- Garner's last step (nb = 4096)
// c = w_q + q^2 h (exact: < n^2), h < p^2 and w_q < q^2 from k_fbg_garner / k_sgp_w, as two plain products by q on
// one lane per element: t = q h (74 x 148 limbs), then u = q t (74 x 222), each by operand scanning with a rotating
// window of S = 74 64-bit column accumulators (q in VGPRs: 74 + 148 registers; column J is complete after operand limb
// J and leaves the window then -- the lazy-CIOS shape of bn_lane.hpp without a reduction), the operand's limbs loaded
// SGPF_D limbs ahead; then c = w_q + u, cut into words. The intermediates go through memory, limb J of a product over
// limb J of its operand once that was read: t over h's rows (and the digit buffer, dead by then, for t's top S rows),
// u over t's (and the digit buffer's next S rows). 27.4 k plain MACs per element (round 5: in place of k_fbg_fin's
// Montgomery product at S = 296 on the TPI = 8 group engine, 175 k).
struct SgpFinParams {
  uint32_t* w;             // [2][2S][n]: h (half 0's rows, < p^2), w_q (half 1's rows, < q^2)
  uint32_t* t_hi;          // [2S][n]: the digit buffer (dead after k_sgp): t's rows 2S .. 3S-1, u's rows 3S .. 4S-1
  long long n;
  const uint32_t* q;       // S limbs
  uint32_t* ct;
  int ct_words;
};
constexpr int SGPF_D = 4;   // operand limbs in flight
constexpr int SGPF_CT_WORDS = 256;   // words of a ciphertext (c < n^2, nb = 4096; the host checks ct_words)

typedef __attribute__((address_space(1))) uint32_t sgpf_g32;
// a limb this lane stored earlier in the kernel: read at device scope (sc1: from L2, where the write-through store
// went, not from a vector-L1 line the lane may have fetched before the store -- ordering the kernel does not want to
// rest on the L1's store-hit policy)
template <bool COH>
__device__ __forceinline__ uint32_t sgpf_ld(const sgpf_g32* p) {
  if constexpr (COH) return __scoped_atomic_load_n(p, __ATOMIC_RELAXED, __MEMORY_SCOPE_DEVICE);
  else return *p;
}
template <class T>
__device__ __forceinline__ T* sgpf_adv(T* p, size_t n) {   // one running row address (precomputed ones would not fit)
  p += n;
  asm volatile("" : "+v"(p));
  return p;
}

// operand limb JJ of a block (x), its S MACs into the window, column JJ leaves: its limb -> *ks; the next load issued
template <int S, bool COH, int JJ>
__device__ __forceinline__ void sgpf_step(uint64_t (&P)[S], uint32_t (&q)[S], uint32_t (&ring)[SGPF_D], const sgpf_g32*& xs,
                                          sgpf_g32*& ks, size_t n) {
#pragma unroll
  for (int i = 0; i < S; ++i) asm volatile("" : "+s"(q[i]));   // (else LLVM hoists the 64-bit zero-extended q: 148 registers)
  const uint32_t x = ring[JJ % SGPF_D];
  if constexpr (JJ + SGPF_D < S) {
    ring[JJ % SGPF_D] = sgpf_ld<COH>(xs);   // limb JJ + D
    xs = sgpf_adv(xs, n);
  }
#pragma unroll
  for (int i = 0; i < S; ++i) P[(i + JJ) % S] += (uint64_t)q[i] * x;
  const uint64_t v = P[JJ % S];
  P[(JJ + 1) % S] += v >> LB;
  P[JJ % S] = 0;
  *ks = (uint32_t)v & LMASK;
  ks = sgpf_adv(ks, n);
#pragma unroll
  for (int i = 0; i < S; ++i)
    if (i != JJ % S) asm volatile("" : "+v"(P[i]));
  __builtin_amdgcn_sched_barrier(0);
}
template <int S, bool COH, int... Js>
__device__ __forceinline__ void sgpf_block(uint64_t (&P)[S], uint32_t (&q)[S], const sgpf_g32* xs, sgpf_g32* ks, size_t n,
                                           std::integer_sequence<int, Js...>) {
  uint32_t ring[SGPF_D];
#pragma unroll
  for (int d = 0; d < SGPF_D; ++d) {
    ring[d] = sgpf_ld<COH>(xs);
    xs = sgpf_adv(xs, n);
  }
  (sgpf_step<S, COH, Js>(P, q, ring, xs, ks, n), ...);
}
// the last S columns: no operand limb
template <int S>
__device__ __forceinline__ void sgpf_tail(uint64_t (&P)[S], sgpf_g32* ks, size_t n) {
#pragma unroll
  for (int jj = 0; jj < S; ++jj) {
    const uint64_t v = P[jj];
    if (jj + 1 < S) P[jj + 1] += v >> LB;
    *ks = (uint32_t)v & LMASK;
    ks = sgpf_adv(ks, n);
  }
}

// c = w_q + u (limbs of u: rows at a (2S), b (S), b2 (S); w_q: 2S rows) -> the NW ciphertext words (compile-time
// packing; the 4S limbs span NW + 3 words, the top ones zero since c < n^2 -- and not stored: they are the next
// element's first words). The limbs are loaded SGPF_WD ahead (a load right before its use waited out an L2 round
// trip per limb: 441 waits per element).
constexpr int SGPF_WD = 8;
template <int S>
struct SgpfWordSrc {
  const sgpf_g32 *ua, *ub, *uc, *wq;
  size_t n;
  template <int J>
  __device__ __forceinline__ uint32_t u() {   // limb J of u (in order)
    const sgpf_g32*& p = J < 2 * S ? ua : (J < 3 * S ? ub : uc);
    const uint32_t v = sgpf_ld<true>(p);
    p = sgpf_adv(p, n);
    return v;
  }
  template <int J>
  __device__ __forceinline__ uint32_t w() {   // limb J of w_q (J < 2S)
    const uint32_t v = *wq;
    wq = sgpf_adv(wq, n);
    return v;
  }
};
template <int S, int NW, int J>
__device__ __forceinline__ void sgpf_word_step(SgpfWordSrc<S>& src, uint32_t (&ru)[SGPF_WD], uint32_t (&rw)[SGPF_WD], uint64_t& buf,
                                               uint64_t& cy, sgpf_g32* ct) {
  constexpr int NB = (LB * J) % 32;   // bits in buf before this limb
  uint64_t v = (uint64_t)ru[J % SGPF_WD] + cy;
  if constexpr (J < 2 * S) v += rw[J % SGPF_WD];
  if constexpr (J + SGPF_WD < 4 * S) ru[J % SGPF_WD] = src.template u<J + SGPF_WD>();
  if constexpr (J + SGPF_WD < 2 * S) rw[J % SGPF_WD] = src.template w<J + SGPF_WD>();
  cy = v >> LB;
  buf |= (v & LMASK) << NB;
  if constexpr (NB + LB >= 32) {
    constexpr int WI = (LB * J) / 32;   // word completed by this limb
    if constexpr (WI < NW) ct[WI] = (uint32_t)buf;
    buf >>= 32;
  }
}
template <int S, int NW, int... Js>
__device__ __forceinline__ void sgpf_words_all(SgpfWordSrc<S>& src, sgpf_g32* ct, std::integer_sequence<int, Js...>) {
  uint32_t ru[SGPF_WD], rw[SGPF_WD];
#pragma unroll
  for (int d = 0; d < SGPF_WD; ++d) {
    ru[d] = sgpf_ld<true>(src.ua);
    src.ua = sgpf_adv(src.ua, src.n);
    rw[d] = *src.wq;
    src.wq = sgpf_adv(src.wq, src.n);
  }
  uint64_t buf = 0, cy = 0;
  (sgpf_word_step<S, NW, Js>(src, ru, rw, buf, cy, ct), ...);
}

template <int S>
__global__ __launch_bounds__(LANE_BLOCK, 2) void k_sgp_fin(SgpFinParams p) {
  static_assert(S == SGP_S, "n^2 of a 4096-bit key: 4 S limbs, 256 words");
  uint32_t q[S];
#pragma unroll
  for (int i = 0; i < S; ++i) q[i] = (uint32_t)__builtin_amdgcn_readfirstlane(p.q[i]);   // SGPRs
  const size_t n = (size_t)p.n;
  using Js = std::make_integer_sequence<int, S>;
  for (long long e = (long long)blockIdx.x * LANE_BLOCK + threadIdx.x; e < p.n; e += (long long)gridDim.x * LANE_BLOCK) {
    sgpf_g32* h = (sgpf_g32*)(p.w + e);                 // rows 0 .. 2S-1
    sgpf_g32* th = (sgpf_g32*)(p.t_hi + e);             // rows 2S .. 3S-1
    sgpf_g32* th2 = (sgpf_g32*)(p.t_hi + S * n + e);    // rows 3S .. 4S-1
    uint64_t P[S];
    // t = q h: h's 2S limbs (two blocks), t's 3S limbs
#pragma unroll
    for (int i = 0; i < S; ++i) P[i] = 0;
#pragma unroll 1
    for (int blk = 0; blk < 2; ++blk) sgpf_block<S, false>(P, q, h + (size_t)blk * S * n, h + (size_t)blk * S * n, n, Js{});
    sgpf_tail<S>(P, th, n);
    // u = q t: t's 3S limbs, u's 4S limbs
#pragma unroll
    for (int i = 0; i < S; ++i) P[i] = 0;
#pragma unroll 1
    for (int blk = 0; blk < 3; ++blk) {
      sgpf_g32* rows = blk < 2 ? h + (size_t)blk * S * n : th;
      sgpf_block<S, true>(P, q, rows, rows, n, Js{});
    }
    sgpf_tail<S>(P, th2, n);
    // c = w_q + u -> words
    {
      SgpfWordSrc<S> src{h, th, th2, (const sgpf_g32*)(p.w + (size_t)2 * S * n + e), n};
      sgpf_words_all<S, SGPF_CT_WORDS>(src, (sgpf_g32*)(p.ct + (size_t)e * SGPF_CT_WORDS), std::make_integer_sequence<int, 4 * S>{});
    }
  }
}

}  // namespace fpai
