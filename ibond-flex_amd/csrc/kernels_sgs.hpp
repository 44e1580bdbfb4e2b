// Split-pair fixed-base sampler on Shoup rows (round 5; the default where it prices lower,
// flexpai.hip fb_choose; $FLEXPAI_SGS=0 keeps k_sgp): kernels_sgp.hpp's lane-pair layout -- element-half e on lanes
// 2e, 2e+1, the even lane keeps A, the odd lane B, V = A + m B mod m^2 --
// with each product by a row (a, 0) done as kernels_fbs.hpp's Shoup product instead of a Montgomery split pass, at
// S = 74 (the 2048-bit p_h of a 4096-bit key):
//   step 1: Q = floor(X a' / R), R = 2^(28 S), from the columns >= S - 1 of X a' (Q at most S + 1 below the floor);
//   step 2: X' = X a + Q (R - m) mod R (= X a - Q m); the odd lane's accumulators start at the even lane's Q_A
//           (DPP): V a = r_A + m (Q_A + B a).
// 1.5 S^2 + 1.5 S lane-MACs per product against the Montgomery pass's 2 S^2. Registers (4 S = 296 VGPRs would hold
// X, Q and one step-2 accumulator row): step 1 runs as two sweeps of columns ([73, 110), then [110, 147) with Q's
// low limbs already out: 185 live) and step 2 in four parts by the index of X_i / Q_i (i >= 56, >= 37, >= 18, >= 0:
// a part reaches only the columns >= its lowest i, and X_i, Q_i are dead after their part: at most 186 live). That
// leaves room for the element's b sum in registers (32 words and a carry count per lane); the row's b words come by
// DMA into the pair's a' quads once step 1 has read them. Two waves per SIMD, 19 KB of LDS per wave.
// Measured (tools/microbench/sgs_stream.hip, profiles/r05_ab_sgs_prototype_stream.txt): 0.82-0.84 of k_sgp's time
// for the same rows at equal W.
//
// Tables. The factored rows k_fbgp_fill built hold T R = a (1 + m b) mod m^2 (R = 2^(28 76), Montgomery form for
// k_sgp) as the words of a and of b R; the Shoup rows (k_sgs_conv) take the same a -- entry (k, d) = the S limbs of a in
// quads 0 .. 18 and of a' = floor(a 2^(28 S) / m) in quads 19 .. 37, SGS_ROW_Q quads apart -- and the b halves stay in
// the factored table. Plain Shoup products of those a then give prod_k T_k R, i.e. the product times R^K, which
// k_sgs_bfin removes with one constant: R^-K mod m^2 = c_A (1 + m beta), c_A by one split Montgomery pass by the
// integer y = c_A R' mod m (which multiplies by c_A (1 + m delta)^-1, c_A R' mod m^2 = y (1 + m delta)), beta + delta
// joining the b sum. The first row is the start: c0 T_0 R = (1 + m gamma) a_0 (1 + m b_0) is the
// pair (a_0, 0) with b_0 in the b sum; k_sgs_bfin adds gamma and beta to it and applies it: B += A (gamma + beta +
// sum_k b_k) mod m, leaving A < m, B < m for k_sgp_w / k_pe_fin.
#pragma once
#include "kernels_fbs.hpp"   // fbs_ap_all / fbs_apt_all / fbs_store_limbs / fbs_reduce_est
#include "kernels_sgp.hpp"

namespace fpai {

constexpr int SGS_NQ = (SGP_S + 3) / 4;        // quads per number (19)
constexpr int SGS_ROW_Q = 40;                  // quads between Shoup rows (38 used; 640 B, five 128-B lines)
constexpr int SGS_WAVE_Q = 2 * SGS_NQ * 32;    // LDS quads per wave: [a, a'][quad][pair of the wave]

struct SgsHalf {
  const uint4* atab;       // [K][2^W] Shoup rows
  const uint4* fac;        // the factored rows (FBGP_ROW4 quads: a R words, then b R words)
  const uint32_t* p;       // modulus m, S limbs
  const uint32_t* nmr;     // [4][S]: w 2^(16 c) R mod m, R = 2^(28 FBGP_S) (gamma = w |M| mod m; w = n / p_h, or 1)
  const uint32_t* pbig;    // 2^20 m
  const uint32_t* mu;      // floor(2^(56 S) / m), S + 2 limbs (k_sgs_conv)
  const uint32_t* cy;      // 64 words: y = c_A R' mod m (R^-K mod m^2 = c_A (1 + m beta), R' = 2^(28 S))
  const uint32_t* bR;      // S limbs: (beta + delta) R mod m
  uint32_t mprime;         // -m^-1 mod 2^28
};

struct SgsParams {
  const SgsHalf* halves;   // [gridDim.y]
  long long n;
  int K, W;
  const uint32_t* digits;  // [gridDim.y][K][n]
  uint32_t* out;           // [gridDim.y][2 S][n]: the pair after the K - 1 products, A < (S + 3) m, B < 2 (S + 3) m
  uint4* bsum;             // [gridDim.y][16][n]: the b sum's 64 words (lane t: quads 8 t .. 8 t + 7)
  uint32_t* bcc;           // [gridDim.y][2][n]: their carry counts (lane 0's enter at word 32, lane 1's at word 64)
  GuardArgs g;             // test build: rows = K 2^W, digits = halves K n, out = halves 2 S n
};

struct SgsFinParams {
  const SgsHalf* halves;
  long long n;
  uint32_t* out;           // in: k_sgs's pairs; out: A < m, B < m (k_sgp_w's / k_pe_fin's input)
  const uint4* bsum;
  const uint32_t* bcc;
  const void* x;
  int dtype, exp_mode, fexp;
  int32_t* exp;            // written by half 0
  int32_t* status;
  int dbg;                 // test-build debugging: 3 = write the b sum's words over the pair rows and stop, 4 = the pair times c_A
};

template <int J>
__device__ __forceinline__ uint32_t sgs_qword(const uint4& v) {
  return J == 0 ? v.x : J == 1 ? v.y : J == 2 ? v.z : v.w;
}

// step 1 as a sweep over the columns [C0, C0 + NC) of X a' (digits J = S-1 down to JMIN, a' quads descending one
// ahead): P[c - C0] += X_i a'_J for i + J = c
template <int S, int C0, int NC, int JMIN, int T>
__device__ __forceinline__ void sgs_q_digit(uint64_t (&P)[NC], const uint32_t (&X)[S], const uint4* q, uint4& cur, uint4& nxt) {
  constexpr int J = S - 1 - T;
  if constexpr (T > 0 && J % 4 == 3) cur = nxt;
  if constexpr ((T == 0 || J % 4 == 3) && J / 4 > JMIN / 4) nxt = q[(J / 4 - 1) * 32];
  const uint32_t d = sgs_qword<J % 4>(cur);
  constexpr int lo = C0 - J > 0 ? C0 - J : 0, hi = C0 + NC - 1 - J < S - 1 ? C0 + NC - 1 - J : S - 1;
#pragma unroll
  for (int i = lo; i <= hi; ++i) P[i + J - C0] += (uint64_t)X[i] * d;
#pragma unroll
  for (int i = 0; i < NC; ++i) asm volatile("" : "+v"(P[i]));
  // (round 6: without these pins and with Q_A by a mask instead of the multiply below -- k_fbs's two changes -- the loop
  // lost 272 of its 9607 instructions per product but not a measurable microsecond: profiles/r06e_ab_sgs_pins_mask.txt)
  __builtin_amdgcn_sched_barrier(0);
}
template <int S, int C0, int NC, int JMIN, int... Ts>
__device__ __forceinline__ void sgs_q_all(uint64_t (&P)[NC], const uint32_t (&X)[S], const uint4* q, std::integer_sequence<int, Ts...>) {
  uint4 cur = q[(SGS_NQ - 1) * 32], nxt;
  (sgs_q_digit<S, C0, NC, JMIN, Ts>(P, X, q, cur, nxt), ...);
}

// step 2, the part i in [I0, I1], digit J of a (ascending, quads one ahead): P[i + J] += X_i a_J, then += Q_i mbar_J
// (mbar = R - m: limbs 2^28 - m_0, then 2^28 - 1 - m_j) for i + J < S; the part's columns are those >= I0
template <int S, int I0, int I1, int J>
__device__ __forceinline__ void sgs_r_digit(uint64_t (&P)[S], const uint32_t (&X)[S], const uint32_t (&Q)[S], const uint32_t (&m)[S],
                                            const uint4* a, uint4& cur, uint4& nxt) {
  constexpr int NQJ = (S - I0 + 3) / 4;   // quads of a the part reads (digits 0 .. S - 1 - I0)
  if constexpr (J % 4 == 0) {
    if constexpr (J > 0) cur = nxt;
    if constexpr (J / 4 + 1 < NQJ) nxt = a[(J / 4 + 1) * 32];
  }
  const uint32_t d = sgs_qword<J % 4>(cur);
  const uint32_t mb = J == 0 ? (LMASK + 1u) - m[0] : LMASK - m[J];
  constexpr int hi = I1 < S - 1 - J ? I1 : S - 1 - J;
  // (all X_i a_J first, then all Q_i mbar_J: no back-to-back MACs into one accumulator)
#pragma unroll
  for (int i = I0; i <= hi; ++i) P[i + J] += (uint64_t)X[i] * d;
#pragma unroll
  for (int i = I0; i <= hi; ++i) P[i + J] += (uint64_t)Q[i] * mb;
#pragma unroll
  for (int i = I0; i < S; ++i) asm volatile("" : "+v"(P[i]));
  __builtin_amdgcn_sched_barrier(0);
}
template <int S, int I0, int I1, int... Js>
__device__ __forceinline__ void sgs_r_all(uint64_t (&P)[S], const uint32_t (&X)[S], const uint32_t (&Q)[S], const uint32_t (&m)[S],
                                          const uint4* a, std::integer_sequence<int, Js...>) {
  uint4 cur = a[0], nxt;
  (sgs_r_digit<S, I0, I1, Js>(P, X, Q, m, a, cur, nxt), ...);
}
// part [I0, I1]: its columns' accumulators start at the even lane's Q_A limbs on the odd lane (0 on the even)
template <int S, int I0, int I1>
__device__ __forceinline__ void sgs_part(uint64_t (&P)[S], const uint32_t (&X)[S], const uint32_t (&Q)[S], const uint32_t (&m)[S],
                                         const uint4* ar, uint32_t ob) {
#pragma unroll
  for (int i = I0; i <= I1; ++i) P[i] = (uint64_t)((uint32_t)__builtin_amdgcn_update_dpp(0, (int)Q[i], 0xA0, 0xF, 0xF, false) * ob);
  sgs_r_all<S, I0, I1>(P, X, Q, m, ar, std::make_integer_sequence<int, S - I0>{});
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
// the b half of the pair's factored row (k, d) (16 quads) -> its a' quads (same instruction shape)
__device__ __forceinline__ void sgs_b_dma(const uint4* __restrict__ fac, size_t k, int W, uint32_t d, uint32_t lb, int lane,
                                          GuardArgs gd) {
  int ln = lane;
  asm volatile("" : "+v"(ln));
  const uint32_t dp = (uint32_t)__builtin_amdgcn_ds_bpermute((ln & 31) * 8, (int)d);
  const uint4* src = fac + FPAI_GUARD_IDX(gd, GS_SGP_ROW, (k << W) + dp, gd.rows, (long long)k) * FBGP_ROW4 + FBGP_PW / 4 + (ln >> 5);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint32_t dst = lb + (uint32_t)(SGS_NQ * 512 + i * 1024);
    asm volatile("" : "+s"(dst));
    __builtin_amdgcn_global_load_lds((const void*)(src + 2 * i), (__attribute__((address_space(3))) void*)(size_t)dst, 16, 0, 0);
  }
}

#if FLEXPAI_XCHECK
__device__ __forceinline__ uint32_t sgs_guard_digit(const SgsParams& p, int h, int k, long long ee) {
  const uint32_t d = p.digits[FPAI_GUARD_IDX(p.g, GS_SGP_DIGIT, ((size_t)h * p.K + k) * p.n + ee, p.g.digits, ee)];
  return (uint32_t)FPAI_GUARD_IDX(p.g, GS_SGP_DVAL, d, 1ull << p.W, ee);
}
#define SGS_DIGIT(k) sgs_guard_digit(p, half, (k), ee)
#else
#define SGS_DIGIT(k) dg[(size_t)(k) * p.n]
#endif

template <int S>
__global__ __launch_bounds__(LANE_BLOCK, 2) void k_sgs(SgsParams p) {
  static_assert(S == SGP_S, "rows of 19 quads");
  constexpr int C1 = S - 1 + 37;   // step 1's second sweep starts at column 110
  __shared__ __attribute__((aligned(16))) uint4 lrows[(LANE_BLOCK / 64) * SGS_WAVE_Q];
  const int half = blockIdx.y;
  const SgsHalf* H = p.halves + half;
  uint32_t m[S];
#pragma unroll
  for (int j = 0; j < S; ++j) m[j] = H->p[j];
  const uint4* atab = H->atab;
  const uint4* fac = H->fac;
  const int K = p.K, W = p.W;
  const int lane = threadIdx.x & 63, tig = threadIdx.x & 1, pw = lane >> 1;
  const bool odd = tig != 0;
  const uint4* wq = lrows + (threadIdx.x >> 6) * SGS_WAVE_Q;
  typedef __attribute__((address_space(3))) uint4 lds_q;
  const uint32_t lb = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(lds_q*)wq);
  const uint4* ar = wq + pw;                  // the pair's a quads (stride 32)
  const uint4* apr = wq + SGS_NQ * 32 + pw;   // its a' quads, then its b quads
  uint32_t ob = odd ? 1u : 0u;
  asm volatile("" : "+v"(ob));   // (a multiplier, not a select)
  constexpr int PAIRS = LANE_BLOCK / 2;
  for (long long base = (long long)blockIdx.x * PAIRS; base < p.n; base += (long long)gridDim.x * PAIRS) {
    const long long e = base + (threadIdx.x >> 1);
    const bool valid = e < p.n;
    const long long ee = valid ? e : p.n - 1;
    const uint32_t* dg = p.digits + (size_t)half * K * p.n + ee;
    (void)dg;
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
    uint32_t bsw[32], cc = 0;   // this lane's 32 words of the b sum, from b_0
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    sgs_b_dma(fac, 0, W, dcur, lb, lane, p.g);
    lds_dma_wait();
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const uint4 b = apr[(8 * tig + q) * 32];
      bsw[4 * q] = b.x, bsw[4 * q + 1] = b.y, bsw[4 * q + 2] = b.z, bsw[4 * q + 3] = b.w;
    }
    for (int k = 1; k < K; ++k) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // row k-1's reads are done
      sgs_rows_dma(atab, (size_t)k, W, dn, lb, lane, p.g);
      dcur = dn;
      dn = k + 1 < K ? SGS_DIGIT(k + 1) : 0u;
      lds_dma_wait();   // row k in LDS, digit k+1 in dn
      uint32_t Q[S];
      {
        uint64_t c;
        {
          uint64_t P[37];
#pragma unroll
          for (int i = 0; i < 37; ++i) P[i] = 0;
          sgs_q_all<S, S - 1, 37, 0>(P, X, apr, std::make_integer_sequence<int, S>{});
          c = P[0] >> LB;   // (column S - 1: its carry only)
#pragma unroll
          for (int i = 1; i < 37; ++i) {
            const uint64_t t = P[i] + c;
            Q[i - 1] = lane::limb32(t);
            c = t >> LB;
          }
        }
        {
          uint64_t P[37];
#pragma unroll
          for (int i = 0; i < 37; ++i) P[i] = 0;
          sgs_q_all<S, C1, 37, C1 - (S - 1)>(P, X, apr, std::make_integer_sequence<int, 2 * S - 1 - C1>{});
#pragma unroll
          for (int i = 0; i < 37; ++i) {
            const uint64_t t = P[i] + c;
            Q[36 + i] = lane::limb32(t);
            c = t >> LB;
          }
          Q[S - 1] = lane::limb32(c);   // (Q < X < R)
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // a' read by both lanes: row k's b half into its quads
      sgs_b_dma(fac, (size_t)k, W, dcur, lb, lane, p.g);
      uint64_t P[S];
      sgs_part<S, 56, S - 1>(P, X, Q, m, ar, ob);
      sgs_part<S, 37, 55>(P, X, Q, m, ar, ob);
      sgs_part<S, 18, 36>(P, X, Q, m, ar, ob);
      sgs_part<S, 0, 17>(P, X, Q, m, ar, ob);
      {
        uint64_t c = 0;   // (mod R: the carry out of limb S - 1 is dropped)
#pragma unroll
        for (int i = 0; i < S; ++i) {
          const uint64_t t = P[i] + c;
          X[i] = lane::limb32(t);
          c = t >> LB;
        }
      }
      lds_dma_wait();   // the b quads
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

// ---------------------------------------------------------------- the b sum applied
// Per element-half on a lane pair (k_sgp's tail): bs = gamma R + sum_k b_k R (words, in LDS; gamma R = sum_c nmr_c
// |M|_c, or 2^20 m minus that for M < 0: < 2^19 m with the K <= 128 rows, so bs fits the S digits REDC' reads), A to
// A mod m (its multiples t of m into B), z = REDC'(A bs) 2^-56 = A bs mod m (< 2 m, the pass's R' = 2^(28 S) against
// the rows' R = 2^(28 76)), B + t + z to B mod m. Out: A < m, B < m.
template <int S>
__global__ __launch_bounds__(LANE_BLOCK, 2) void k_sgs_bfin(SgsFinParams p) {
  __shared__ __attribute__((aligned(16))) uint32_t bsum[SGP_PAIRS * SGP_BW];
  __shared__ uint32_t cyl[FBGP_PW];
  const int half = blockIdx.y;
  const SgsHalf* H = p.halves + half;
  for (int i = threadIdx.x; i < FBGP_PW; i += blockDim.x) cyl[i] = H->cy[i];
  __syncthreads();
  uint32_t m[S];
#pragma unroll
  for (int j = 0; j < S; ++j) m[j] = H->p[j];
  const uint32_t mprime = H->mprime;
  const int tig = threadIdx.x & 1;
  const bool odd = tig != 0;
  uint32_t* bs = bsum + (threadIdx.x >> 1) * SGP_BW;
  for (long long base = (long long)blockIdx.x * SGP_PAIRS; base < p.n; base += (long long)gridDim.x * SGP_PAIRS) {
    const long long e = base + (threadIdx.x >> 1);
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
    wave_lds_fence();   // the previous element's reads of bs are done
    {   // this lane's 32 words of the sum; lane 1's carry count at word 64
      const uint4* bsp = p.bsum + ((size_t)half * 16 + 8 * tig) * p.n + ee;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const uint4 v = bsp[(size_t)q * p.n];
        bs[32 * tig + 4 * q] = v.x, bs[32 * tig + 4 * q + 1] = v.y, bs[32 * tig + 4 * q + 2] = v.z, bs[32 * tig + 4 * q + 3] = v.w;
      }
      if (odd) {
        bs[64] = p.bcc[((size_t)half * 2 + 1) * p.n + ee];
        for (int w = 65; w < SGP_BW; ++w) bs[w] = 0u;
      }
    }
    wave_lds_fence();
    if (!odd) {   // lane 0's carry count from word 32, then gamma R (limbs -> words) on top
      uint64_t c = p.bcc[((size_t)half * 2) * p.n + ee];
      for (int w = 32; w < SGP_BW; ++w) {
        const uint64_t v = (uint64_t)bs[w] + c;
        bs[w] = (uint32_t)v;
        c = v >> 32;
      }
      const bool neg = M < 0;
      const uint64_t mag = neg ? (uint64_t)0 - (uint64_t)M : (uint64_t)M;
      const uint32_t* nmr = opaque_uniform(H->nmr);
      const uint32_t* pbg = opaque_uniform(H->pbig);
      uint64_t P[S];
#pragma unroll
      for (int i = 0; i < S; ++i) {
        uint64_t v = 0;
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4) v += (uint64_t)nmr[c4 * S + i] * ((uint32_t)(mag >> (16 * c4)) & 0xFFFFu);
        P[i] = v;
      }
      uint32_t g[S], pb[S], D[S];
      lane::normalize<S>(P, g);
      if (neg) {
#pragma unroll
        for (int i = 0; i < S; ++i) pb[i] = pbg[i];
        (void)lane::sub<S>(pb, g, D);
#pragma unroll
        for (int i = 0; i < S; ++i) g[i] = D[i];
      }
      {   // + beta R
        const uint32_t* br = opaque_uniform(H->bR);
        uint32_t cy = 0;
#pragma unroll
        for (int i = 0; i < S; ++i) {
          const uint32_t v = g[i] + br[i] + cy;
          g[i] = v & LMASK;
          cy = v >> LB;
        }
      }
      // bs += g
      {
        // limbs -> words by a running 64-bit window: 28 bits in per limb, 32 out per word
        uint64_t acc = 0;
        int have = 0, w = 0;
        uint64_t carry = 0;
#pragma unroll
        for (int i = 0; i < S; ++i) {
          acc |= (uint64_t)g[i] << have;
          have += LB;
          if (have >= 32) {
            const uint64_t v = (uint64_t)bs[w] + (uint32_t)acc + carry;
            bs[w] = (uint32_t)v;
            carry = v >> 32;
            acc >>= 32;
            have -= 32;
            ++w;
          }
        }
        for (; w < SGP_BW; ++w) {
          const uint64_t v = (uint64_t)bs[w] + (uint32_t)acc + carry;
          bs[w] = (uint32_t)v;
          carry = v >> 32;
          acc >>= 32;
        }
      }
    }
    wave_lds_fence();
    if (p.dbg == 3) {
      if (valid && !odd)
        for (int w = 0; w < SGP_BW; ++w) p.out[((size_t)half * 2 * S + w) * p.n + e] = bs[w];
      continue;
    }
    // the pair times c_A: one split Montgomery pass by c_A R' (A < (S + 3) m, B < 2 (S + 3) m in; A < 2 m, B < 4 m out)
    uint32_t x[S];
#pragma unroll
    for (int i = 0; i < S; ++i) x[i] = p.out[((size_t)half * 2 * S + tig * S + i) * p.n + ee];
    {
      uint64_t P[S];
#pragma unroll
      for (int i = 0; i < S; ++i) P[i] = 0;
      sgp_pass<S, FBGP_PW, false>(P, x, cyl, m, mprime, odd, std::make_integer_sequence<int, S>{});
      lane::normalize<S>(P, x);
    }
    if (p.dbg == 4) {
      if (valid)
        for (int i = 0; i < S; ++i) p.out[((size_t)half * 2 * S + tig * S + i) * p.n + e] = x[i];
      continue;
    }
    // A to A mod m on the even lane, its multiples t to the odd lane
    uint32_t t = 0;
    if (!odd) fbs_reduce_est<S>(x, m, t);
    const uint32_t tb = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)t, 0xA0, 0xF, 0xF, false);
    uint32_t z[S];
    {   // z = REDC'(x bs) on both lanes (the odd lane's discarded)
      uint64_t P[S];
#pragma unroll
      for (int i = 0; i < S; ++i) P[i] = 0;
      sgp_pass<S, SGP_BW, false>(P, x, bs, m, mprime, false, std::make_integer_sequence<int, S>{});
      lane::normalize<S>(P, z);
      sgp_div56<S>(z, m, mprime);
    }
    {   // odd: B + t + z (< 2 (S + 3) m + 2^7 + 2 m < 2^8 m), then mod m
      uint32_t c = odd ? tb : 0u;
#pragma unroll
      for (int j = 0; j < S; ++j) {
        const uint32_t zb = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)z[j], 0xA0, 0xF, 0xF, false);
        const uint32_t v = x[j] + (odd ? zb : 0u) + c;
        x[j] = v & LMASK;
        c = v >> LB;
      }
      uint32_t t2 = 0;
      if (odd) fbs_reduce_est<S>(x, m, t2);
    }
    if (valid) {
#pragma unroll
      for (int i = 0; i < S; ++i) p.out[((size_t)half * 2 * S + tig * S + i) * p.n + e] = x[i];
    }
  }
}

// ---------------------------------------------------------------- Shoup rows from the factored rows

// One row per thread: the factored row's a (words -> limbs, canonical), then a' = floor(a R' / m), R' = 2^(28 S), by
// kernels_fbs.hpp's product scanning with mu = floor(R'^2 / m) and one correction.
template <int S>
__global__ __launch_bounds__(LANE_BLOCK) void k_sgs_conv(const SgsHalf* halves, size_t rows, uint4* atab0, uint4* atab1) {
  const size_t r = (size_t)blockIdx.x * LANE_BLOCK + threadIdx.x;
  if (r >= rows) return;
  const SgsHalf* H = halves + blockIdx.y;
  uint4* atab = blockIdx.y ? atab1 : atab0;
  uint32_t m[S];
#pragma unroll
  for (int i = 0; i < S; ++i) m[i] = (uint32_t)__builtin_amdgcn_readfirstlane(H->p[i]);
  uint32_t A[S];
  {
    uint32_t w[FBGP_PW];
    const uint4* src = H->fac + r * FBGP_ROW4;
#pragma unroll
    for (int q = 0; q < FBGP_PW / 4; ++q) {
      const uint4 v = src[q];
      w[4 * q] = v.x, w[4 * q + 1] = v.y, w[4 * q + 2] = v.z, w[4 * q + 3] = v.w;
    }
#pragma unroll
    for (int i = 0; i < S; ++i) A[i] = lane::limb_from_words([&](int j) { return w[j]; }, FBGP_PW, i);
  }
  lane::cond_sub<S>(A, m);
  uint32_t ap[S + 1];
  {
    fbs_ap_all<S>(ap, A, H->mu, std::make_integer_sequence<int, 2 * S + 1>{});
    uint32_t tl[S + 1];
    fbs_apt_all<S>(tl, ap, A, m, std::make_integer_sequence<int, S + 1>{});
    int32_t bw = 0;
#pragma unroll
    for (int t2 = 0; t2 < S + 1; ++t2) {
      const int32_t v = (int32_t)tl[t2] - (int32_t)(t2 < S ? m[t2] : 0u) + bw;
      bw = v >> LB;
    }
    uint32_t inc = bw == 0 ? 1u : 0u;
#pragma unroll
    for (int t2 = 0; t2 < S + 1; ++t2) {
      const uint32_t v = ap[t2] + inc;
      ap[t2] = v & LMASK;
      inc = v >> LB;
    }
  }
  uint4* dst = atab + r * SGS_ROW_Q;
  fbs_store_limbs<S>(dst, A, std::make_integer_sequence<int, SGS_NQ>{});
  fbs_store_limbs<S>(dst + SGS_NQ, ap, std::make_integer_sequence<int, SGS_NQ>{});   // a' < R: limb S is zero
}

}  // namespace fpai
