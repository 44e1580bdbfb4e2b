// PROTOTYPE (measurement only, tools/microbench/sgs_stream.hip; not part of the library): the split-pair fixed-base
// sampler with Shoup rows. kernels_sgp.hpp's lane-pair layout (element-half e on lanes 2e, 2e+1:
// the even lane keeps A, the odd lane B, V = A + m B mod m^2) with each product by a row (a, 0) done as
// kernels_fbs.hpp's Shoup product instead of a Montgomery split pass, at S = 74:
//   step 1: Q = floor(X a' / R), R = 2^(28 S), from the columns >= S - 1 of X a' (75 accumulators, S (S + 1) / 2 MACs);
//   step 2: X' = X a + Q (R - m) mod R (= X a - Q m), S (S + 1) MACs; the odd lane adds the even lane's Q_A (DPP):
//           V a = r_A + m (Q_A + B a).
// Per lane 1.5 S^2 + 1.5 S MACs against the Montgomery pass's 2 S^2. At S = 74 the step-2 accumulator row does not fit
// next to X and Q (4 S = 296 VGPRs); step 2 therefore runs in two parts split by the index i of X_i and Q_i:
//   part H: i in [37, 74) -- it reaches only the columns [37, 74) (digits a_0 .. a_36): 37 accumulators, X, Q;
//   part L: i in [0, 37)  -- all 74 columns: 74 accumulators, X_L, Q_L (X_H, Q_H are dead after part H);
// 222 VGPRs at either peak, nothing parked. Q_A enters as the odd lane's accumulator start. Two waves per SIMD.
//
// Rows: entry (k, d) = the S limbs of a (plain) in quads 0 .. 18 and of a' = floor(a R / m) in quads 19 .. 37, 40 quads
// apart. BS = 1: the b half of row k (16 quads of b R words, from a second table) streams by DMA into the pair's a'
// quads once step 1 has read them, and after the product each lane adds its 32 words to its part of the element's b
// sum in global memory ([half][16 quads][n], the carry-outs counted in a register and written at the end).
#pragma once
#include "kernels_sgp.hpp"

namespace fpai {

constexpr int SGS_NQ = (SGP_S + 3) / 4;        // quads per number (19)
constexpr int SGS_ROW_Q = 40;                  // quads between table rows (38 used)
constexpr int SGS_WAVE_Q = 2 * SGS_NQ * 32;    // LDS quads per wave: [a, a'][quad][pair of the wave]

struct SgsHalf {
  const uint4* atab;       // [K][2^W] rows of SGS_ROW_Q quads
  const uint32_t* p;       // modulus m, S limbs
  const uint4* btab;       // BS: b R quads of entry r at btab + r * bstride (16 quads)
  int bstride;
};

struct SgsParams {
  const SgsHalf* halves;   // [gridDim.y]
  long long n;
  int K, W;
  const uint32_t* digits;  // [gridDim.y][K][n]
  uint32_t* out;           // [gridDim.y][2 S][n]
  uint4* bsum;             // BS: [gridDim.y][16][n]
  uint32_t* bcc;           // BS: [gridDim.y][2][n] carry counts
  GuardArgs g;             // test build: rows = K 2^W, digits = halves K n, out = halves 2 S n
};

template <int J>
__device__ __forceinline__ uint32_t sgs_qword(const uint4& v) {
  return J == 0 ? v.x : J == 1 ? v.y : J == 2 ? v.z : v.w;
}

// step 1, consumption index T (digit J = S - 1 - T of a', quads read descending one ahead)
template <int S, int T>
__device__ __forceinline__ void sgs_q_digit(uint64_t (&P)[S + 1], const uint32_t (&X)[S], const uint4* q, uint4& cur, uint4& nxt) {
  constexpr int J = S - 1 - T;
  if constexpr (T > 0 && J % 4 == 3) cur = nxt;
  if constexpr ((T == 0 || J % 4 == 3) && J / 4 > 0) nxt = q[(J / 4 - 1) * 32];
  const uint32_t d = sgs_qword<J % 4>(cur);
#pragma unroll
  for (int i = S - 1 - J; i < S; ++i) P[i + J - (S - 1)] += (uint64_t)X[i] * d;
#pragma unroll
  for (int i = 0; i <= S; ++i) asm volatile("" : "+v"(P[i]));
  __builtin_amdgcn_sched_barrier(0);
}
template <int S, int... Ts>
__device__ __forceinline__ void sgs_q_all(uint64_t (&P)[S + 1], const uint32_t (&X)[S], const uint4* q, std::integer_sequence<int, Ts...>) {
  uint4 cur = q[(SGS_NQ - 1) * 32], nxt;
  (sgs_q_digit<S, Ts>(P, X, q, cur, nxt), ...);
}

// the wave's 32 rows of product k -> LDS: instruction i fetches quad 2i on lanes 0-31 and 2i+1 on lanes 32-63, for
// pair L & 31 (its row index from that pair's even lane), landing at [quad][pair]
__device__ __forceinline__ void sgs_rows_dma(const uint4* __restrict__ atab, size_t k, int W, uint32_t d, uint32_t lb, int lane,
                                             GuardArgs gd) {
  int ln = lane;
  asm volatile("" : "+v"(ln));   // (lane-derived offsets recomputed here, not kept live across the products)
  const uint32_t dp = (uint32_t)__builtin_amdgcn_ds_bpermute((ln & 31) * 8, (int)d);
  const uint4* src = atab + FPAI_GUARD_IDX(gd, GS_SGP_ROW, (k << W) + dp, gd.rows, (long long)k) * SGS_ROW_Q + (ln >> 5);
#pragma unroll
  for (int i = 0; i < SGS_NQ; ++i) {
    uint32_t dst = lb + (uint32_t)(i * 1024);
    asm volatile("" : "+s"(dst));
    __builtin_amdgcn_global_load_lds((const void*)(src + 2 * i), (__attribute__((address_space(3))) void*)(size_t)dst, 16, 0, 0);
  }
}

#if FLEXPAI_XCHECK
#define SGS_DIGIT(k) sgp_guard_digit_s(p, half, (k), ee)
__device__ __forceinline__ uint32_t sgp_guard_digit_s(const SgsParams& p, int h, int k, long long ee) {
  const uint32_t d = p.digits[FPAI_GUARD_IDX(p.g, GS_SGP_DIGIT, ((size_t)h * p.K + k) * p.n + ee, p.g.digits, ee)];
  return (uint32_t)FPAI_GUARD_IDX(p.g, GS_SGP_DVAL, d, 1ull << p.W, ee);
}
#else
#define SGS_DIGIT(k) dg[(size_t)(k) * p.n]
#endif

// step 1 as a sweep over the columns [C0, C0 + NC) of X a' only (digits J = S-1 down to JMIN, a' quads descending
// one ahead): P[c - C0] += X_i a'_J for i + J = c
template <int S, int C0, int NC, int JMIN, int T>
__device__ __forceinline__ void sgs_q2_digit(uint64_t (&P)[NC], const uint32_t (&X)[S], const uint4* q, uint4& cur, uint4& nxt) {
  constexpr int J = S - 1 - T;
  if constexpr (T > 0 && J % 4 == 3) cur = nxt;
  if constexpr ((T == 0 || J % 4 == 3) && J / 4 > JMIN / 4) nxt = q[(J / 4 - 1) * 32];
  const uint32_t d = sgs_qword<J % 4>(cur);
  constexpr int lo = C0 - J > 0 ? C0 - J : 0, hi = C0 + NC - 1 - J < S - 1 ? C0 + NC - 1 - J : S - 1;
#pragma unroll
  for (int i = lo; i <= hi; ++i) P[i + J - C0] += (uint64_t)X[i] * d;
#pragma unroll
  for (int i = 0; i < NC; ++i) asm volatile("" : "+v"(P[i]));
  __builtin_amdgcn_sched_barrier(0);
}
template <int S, int C0, int NC, int JMIN, int... Ts>
__device__ __forceinline__ void sgs_q2_all(uint64_t (&P)[NC], const uint32_t (&X)[S], const uint4* q, std::integer_sequence<int, Ts...>) {
  uint4 cur = q[(SGS_NQ - 1) * 32], nxt;
  (sgs_q2_digit<S, C0, NC, JMIN, Ts>(P, X, q, cur, nxt), ...);
}

// step 2 part H / part L, digit J of a: P[i + J] += X_i a_J, then += Q_i mbar_J (mbar = R - m) for i in [I0, I1] with
// i + J < S
template <int S, int I0, int I1, int PLO, int J>
__device__ __forceinline__ void sgs_s2_digit(uint64_t (&P)[S], const uint32_t (&X)[S], const uint32_t (&Q)[S], const uint32_t (&m)[S],
                                             const uint4* a, uint4& cur, uint4& nxt, int njq) {
  (void)njq;
  constexpr int NQJ = I0 == 0 ? SGS_NQ : (S - I0 + 3) / 4;   // quads of a this part reads
  if constexpr (J % 4 == 0) {
    if constexpr (J > 0) cur = nxt;
    if constexpr (J / 4 + 1 < NQJ) nxt = a[(J / 4 + 1) * 32];
  }
  const uint32_t d = sgs_qword<J % 4>(cur);
  const uint32_t mb = J == 0 ? (lane::LMASK + 1u) - m[0] : lane::LMASK - m[J];
  constexpr int hi = I1 < S - 1 - J ? I1 : S - 1 - J;
#pragma unroll
  for (int i = I0; i <= hi; ++i) P[i + J] += (uint64_t)X[i] * d;
#pragma unroll
  for (int i = I0; i <= hi; ++i) P[i + J] += (uint64_t)Q[i] * mb;
#pragma unroll
  for (int i = PLO; i < S; ++i) asm volatile("" : "+v"(P[i]));
  __builtin_amdgcn_sched_barrier(0);
}
template <int S, int I0, int I1, int PLO, int... Js>
__device__ __forceinline__ void sgs_s2_all(uint64_t (&P)[S], const uint32_t (&X)[S], const uint32_t (&Q)[S], const uint32_t (&m)[S],
                                           const uint4* a, std::integer_sequence<int, Js...>) {
  uint4 cur = a[0], nxt;
  (sgs_s2_digit<S, I0, I1, PLO, Js>(P, X, Q, m, a, cur, nxt, 0), ...);
}

// the pair's b half of row k (16 quads) -> its a' quads: instruction i = quads 2i (lanes 0-31) and 2i+1 (lanes 32-63)
__device__ __forceinline__ void sgs_b_dma(const uint4* __restrict__ btab, int bstride, size_t k, int W, uint32_t d, uint32_t lb,
                                          int lane) {
  int ln = lane;
  asm volatile("" : "+v"(ln));
  const uint32_t dp = (uint32_t)__builtin_amdgcn_ds_bpermute((ln & 31) * 8, (int)d);
  const uint4* src = btab + ((k << W) + dp) * (size_t)bstride + (ln >> 5);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint32_t dst = lb + (uint32_t)(SGS_NQ * 512 + i * 1024);
    asm volatile("" : "+s"(dst));
    __builtin_amdgcn_global_load_lds((const void*)(src + 2 * i), (__attribute__((address_space(3))) void*)(size_t)dst, 16, 0, 0);
  }
}

template <int S, int BS>
__global__ __launch_bounds__(LANE_BLOCK, 2) void k_sgs(SgsParams p) {
  static_assert(S == SGP_S, "rows of 19 quads");
  constexpr int IH = 37;   // part H: i >= IH
  __shared__ __attribute__((aligned(16))) uint4 lrows[(LANE_BLOCK / 64) * SGS_WAVE_Q];
  const int half = blockIdx.y;
  const SgsHalf* H = p.halves + half;
  uint32_t m[S];
#pragma unroll
  for (int j = 0; j < S; ++j) m[j] = H->p[j];
  const uint4* atab = H->atab;
  const int K = p.K, W = p.W;
  const int lane = threadIdx.x & 63, tig = threadIdx.x & 1, pw = lane >> 1;
  const bool odd = tig != 0;
  const uint4* wq = lrows + (threadIdx.x >> 6) * SGS_WAVE_Q;
  typedef __attribute__((address_space(3))) uint4 lds_q;
  const uint32_t lb = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(lds_q*)wq);
  const uint4* ar = wq + pw;                        // the pair's a quads (stride 32)
  const uint4* apr = wq + SGS_NQ * 32 + pw;         // its a' quads (BS: then its b quads)
  uint32_t ob = odd ? 1u : 0u;
  asm volatile("" : "+v"(ob));   // (a multiplier, not a select)
  constexpr int PAIRS = LANE_BLOCK / 2;
  for (long long base = (long long)blockIdx.x * PAIRS; base < p.n; base += (long long)gridDim.x * PAIRS) {
    const long long e = base + (threadIdx.x >> 1);
    const bool valid = e < p.n;
    const long long ee = valid ? e : p.n - 1;
    const uint32_t* dg = p.digits + (size_t)half * K * p.n + ee;
    (void)dg;
    uint4* bsp = p.bsum + ((size_t)half * 16 + 8 * tig) * p.n + ee;   // this lane's 8 quads, n apart
    uint32_t cc = 0;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the previous element's LDS reads are done
    uint32_t dcur = SGS_DIGIT(0);
    sgs_rows_dma(atab, 0, W, dcur, lb, lane, p.g);
    uint32_t dn = K > 1 ? SGS_DIGIT(1) : 0u;
    lds_dma_wait();
    uint32_t X[S];   // (a_0, 0)
#pragma unroll
    for (int g = 0; g < SGS_NQ; ++g) {
      const uint4 v = ar[g * 32];
      if (4 * g < S) X[4 * g] = odd ? 0u : v.x;
      if (4 * g + 1 < S) X[4 * g + 1] = odd ? 0u : v.y;
      if (4 * g + 2 < S) X[4 * g + 2] = odd ? 0u : v.z;
      if (4 * g + 3 < S) X[4 * g + 3] = odd ? 0u : v.w;
    }
    if constexpr (BS) {   // b_0: the sum's start
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      sgs_b_dma(H->btab, H->bstride, 0, W, dcur, lb, lane);
      lds_dma_wait();
      if (valid) {
#pragma unroll
        for (int q = 0; q < 8; ++q) bsp[(size_t)q * p.n] = apr[(8 * tig + q) * 32];
      }
    }
    for (int k = 1; k < K; ++k) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // row k-1's reads are done
      sgs_rows_dma(atab, (size_t)k, W, dn, lb, lane, p.g);
      dcur = dn;
      dn = k + 1 < K ? SGS_DIGIT(k + 1) : 0u;
      lds_dma_wait();   // row k in LDS, digit k+1 in dn
      uint32_t Q[S];
      {
        uint64_t P[S + 1];
#pragma unroll
        for (int i = 0; i <= S; ++i) P[i] = 0;
        sgs_q_all<S>(P, X, apr, std::make_integer_sequence<int, S>{});
        uint64_t c = P[0] >> lane::LB;
#pragma unroll
        for (int i = 1; i <= S; ++i) {
          const uint64_t t = P[i] + c;
          Q[i - 1] = lane::limb32(t);
          c = t >> lane::LB;
        }
      }
      if constexpr (BS) {   // a' is read: row k's b half into its quads
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        sgs_b_dma(H->btab, H->bstride, (size_t)k, W, dcur, lb, lane);
      }
      uint64_t P[S];
#pragma unroll
      for (int i = IH; i < S; ++i) P[i] = (uint64_t)((uint32_t)__builtin_amdgcn_update_dpp(0, (int)Q[i], 0xA0, 0xF, 0xF, false) * ob);
      sgs_s2_all<S, IH, S - 1, IH>(P, X, Q, m, ar, std::make_integer_sequence<int, S - IH>{});
#pragma unroll
      for (int i = 0; i < IH; ++i) P[i] = (uint64_t)((uint32_t)__builtin_amdgcn_update_dpp(0, (int)Q[i], 0xA0, 0xF, 0xF, false) * ob);
      sgs_s2_all<S, 0, IH - 1, 0>(P, X, Q, m, ar, std::make_integer_sequence<int, S>{});
      {
        uint64_t c = 0;   // (mod R: the carry out of limb S - 1 is dropped)
#pragma unroll
        for (int i = 0; i < S; ++i) {
          const uint64_t t = P[i] + c;
          X[i] = lane::limb32(t);
          c = t >> lane::LB;
        }
      }
      if constexpr (BS) {   // this lane's 32 words of the b sum += the row's (carry-outs counted in cc)
        uint4 s[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) s[q] = bsp[(size_t)q * p.n];
        lds_dma_wait();
        unsigned int c = 0;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const uint4 b = apr[(8 * tig + q) * 32];
          s[q].x = __builtin_addc(s[q].x, b.x, c, &c);
          s[q].y = __builtin_addc(s[q].y, b.y, c, &c);
          s[q].z = __builtin_addc(s[q].z, b.z, c, &c);
          s[q].w = __builtin_addc(s[q].w, b.w, c, &c);
        }
        cc += c;
        if (valid) {   // (clamped lanes alias element n - 1)
#pragma unroll
          for (int q = 0; q < 8; ++q) bsp[(size_t)q * p.n] = s[q];
        }
      }
    }
    if (valid && FPAI_GUARD_OK(p.g, GS_SGP_OUT, ((size_t)half * 2 * S + tig * S + S - 1) * p.n + e, p.g.out, e)) {
#pragma unroll
      for (int i = 0; i < S; ++i) p.out[((size_t)half * 2 * S + tig * S + i) * p.n + e] = X[i];
      if constexpr (BS) p.bcc[((size_t)half * 2 + tig) * p.n + e] = cc;
    }
  }
}

// BS = 2 form: step 1 as two column sweeps ([73, 110) then [110, 147): Q's low limbs out of the first, X, 37
// accumulators and them live in the second: 185 VGPRs) and step 2 in four parts by the index of X_i / Q_i (i >= 56,
// >= 37, >= 18, >= 0: at most 186 live), so that the element's b sum (32 words and a carry count per lane) stays in
// registers and the row's b words come from LDS (DMA'd into the a' quads after step 1): no global round trip.
template <int S, int LO, int HI>
__device__ __forceinline__ void sgs_part(uint64_t (&P)[S], const uint32_t (&X)[S], const uint32_t (&Q)[S], const uint32_t (&m)[S],
                                         const uint4* ar, uint32_t ob) {
#pragma unroll
  for (int i = LO; i <= HI; ++i) P[i] = (uint64_t)((uint32_t)__builtin_amdgcn_update_dpp(0, (int)Q[i], 0xA0, 0xF, 0xF, false) * ob);
  sgs_s2_all<S, LO, HI, LO>(P, X, Q, m, ar, std::make_integer_sequence<int, S - LO>{});
}

template <int S>
__global__ __launch_bounds__(LANE_BLOCK, 2) void k_sgs2(SgsParams p) {
  static_assert(S == SGP_S, "rows of 19 quads");
  constexpr int C1 = S - 1 + 37;   // step 1's second sweep starts at column 110
  __shared__ __attribute__((aligned(16))) uint4 lrows[(LANE_BLOCK / 64) * SGS_WAVE_Q];
  const int half = blockIdx.y;
  const SgsHalf* H = p.halves + half;
  uint32_t m[S];
#pragma unroll
  for (int j = 0; j < S; ++j) m[j] = H->p[j];
  const uint4* atab = H->atab;
  const int K = p.K, W = p.W;
  const int lane = threadIdx.x & 63, tig = threadIdx.x & 1, pw = lane >> 1;
  const bool odd = tig != 0;
  const uint4* wq = lrows + (threadIdx.x >> 6) * SGS_WAVE_Q;
  typedef __attribute__((address_space(3))) uint4 lds_q;
  const uint32_t lb = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(lds_q*)wq);
  const uint4* ar = wq + pw;
  const uint4* apr = wq + SGS_NQ * 32 + pw;
  uint32_t ob = odd ? 1u : 0u;
  asm volatile("" : "+v"(ob));
  constexpr int PAIRS = LANE_BLOCK / 2;
  for (long long base = (long long)blockIdx.x * PAIRS; base < p.n; base += (long long)gridDim.x * PAIRS) {
    const long long e = base + (threadIdx.x >> 1);
    const bool valid = e < p.n;
    const long long ee = valid ? e : p.n - 1;
    const uint32_t* dg = p.digits + (size_t)half * K * p.n + ee;
    (void)dg;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    uint32_t dcur = SGS_DIGIT(0);
    sgs_rows_dma(atab, 0, W, dcur, lb, lane, p.g);
    uint32_t dn = K > 1 ? SGS_DIGIT(1) : 0u;
    lds_dma_wait();
    uint32_t X[S];
#pragma unroll
    for (int g = 0; g < SGS_NQ; ++g) {
      const uint4 v = ar[g * 32];
      if (4 * g < S) X[4 * g] = odd ? 0u : v.x;
      if (4 * g + 1 < S) X[4 * g + 1] = odd ? 0u : v.y;
      if (4 * g + 2 < S) X[4 * g + 2] = odd ? 0u : v.z;
      if (4 * g + 3 < S) X[4 * g + 3] = odd ? 0u : v.w;
    }
    uint32_t bsw[32], cc = 0;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    sgs_b_dma(H->btab, H->bstride, 0, W, dcur, lb, lane);
    lds_dma_wait();
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const uint4 b = apr[(8 * tig + q) * 32];
      bsw[4 * q] = b.x, bsw[4 * q + 1] = b.y, bsw[4 * q + 2] = b.z, bsw[4 * q + 3] = b.w;
    }
    for (int k = 1; k < K; ++k) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      sgs_rows_dma(atab, (size_t)k, W, dn, lb, lane, p.g);
      dcur = dn;
      dn = k + 1 < K ? SGS_DIGIT(k + 1) : 0u;
      lds_dma_wait();
      uint32_t Q[S];
      {
        uint64_t c;
        {
          uint64_t P[37];
#pragma unroll
          for (int i = 0; i < 37; ++i) P[i] = 0;
          sgs_q2_all<S, S - 1, 37, 0>(P, X, apr, std::make_integer_sequence<int, S>{});
          c = P[0] >> lane::LB;
#pragma unroll
          for (int i = 1; i < 37; ++i) {
            const uint64_t t = P[i] + c;
            Q[i - 1] = lane::limb32(t);
            c = t >> lane::LB;
          }
        }
        {
          uint64_t P[37];
#pragma unroll
          for (int i = 0; i < 37; ++i) P[i] = 0;
          sgs_q2_all<S, C1, 37, C1 - (S - 1)>(P, X, apr, std::make_integer_sequence<int, 2 * S - 1 - C1>{});
#pragma unroll
          for (int i = 0; i < 37; ++i) {
            const uint64_t t = P[i] + c;
            Q[36 + i] = lane::limb32(t);
            c = t >> lane::LB;
          }
          Q[S - 1] = lane::limb32(c);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      sgs_b_dma(H->btab, H->bstride, (size_t)k, W, dcur, lb, lane);
      uint64_t P[S];
      sgs_part<S, 56, S - 1>(P, X, Q, m, ar, ob);
      sgs_part<S, 37, 55>(P, X, Q, m, ar, ob);
      sgs_part<S, 18, 36>(P, X, Q, m, ar, ob);
      sgs_part<S, 0, 17>(P, X, Q, m, ar, ob);
      {
        uint64_t c = 0;
#pragma unroll
        for (int i = 0; i < S; ++i) {
          const uint64_t t = P[i] + c;
          X[i] = lane::limb32(t);
          c = t >> lane::LB;
        }
      }
      lds_dma_wait();
      {
        unsigned int c = 0;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const uint4 b = apr[(8 * tig + q) * 32];
          bsw[4 * q] = __builtin_addc(bsw[4 * q], b.x, c, &c);
          bsw[4 * q + 1] = __builtin_addc(bsw[4 * q + 1], b.y, c, &c);
          bsw[4 * q + 2] = __builtin_addc(bsw[4 * q + 2], b.z, c, &c);
          bsw[4 * q + 3] = __builtin_addc(bsw[4 * q + 3], b.w, c, &c);
        }
        cc += c;
      }
    }
    if (valid && FPAI_GUARD_OK(p.g, GS_SGP_OUT, ((size_t)half * 2 * S + tig * S + S - 1) * p.n + e, p.g.out, e)) {
#pragma unroll
      for (int i = 0; i < S; ++i) p.out[((size_t)half * 2 * S + tig * S + i) * p.n + e] = X[i];
      uint4* bsp = p.bsum + ((size_t)half * 16 + 8 * tig) * p.n + e;
#pragma unroll
      for (int q = 0; q < 8; ++q) bsp[(size_t)q * p.n] = make_uint4(bsw[4 * q], bsw[4 * q + 1], bsw[4 * q + 2], bsw[4 * q + 3]);
      p.bcc[((size_t)half * 2 + tig) * p.n + e] = cc;
    }
  }
}

}  // namespace fpai
