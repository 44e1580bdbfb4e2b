// Fixed-base obfuscation with Shoup-form rows (round 4): the sampler of kernels_fbp.hpp with each product by a
// table row done as Shoup's fixed-multiplier product instead of a Montgomery pass. Same distribution, same
// canonical pairs out, so k_fbp_fin recombines them unchanged and the ciphertexts are bit-identical to k_fbp's.
//
// Rows. A table entry T = T_k[d] mod p_h^2 (PLAIN, not Montgomery form) is stored factored as T = a (1 + p_h b),
// a = T mod p_h, together with Shoup's quotient a' = floor(a R / p_h) < R, R = 2^(28 S): the S 28-bit limbs of a
// (one per 32-bit word, QA quads), the S limbs of a' (QAP quads), then the PW 32-bit words of b R mod p_h (QB quads)
// -- 448 B per row at nb = 2048 (28 quads). Limbs, not packed words, so that a digit is a register of the quad that
// holds it (no shift or align per digit). The a and a' quads stream into LDS by DMA one product ahead, the b R quads
// into registers (summed into bs at once).
//
// Product of the running pair (A, B), V = A + p B (mod p^2), by a (tools/shoup_model.py checks every bound):
//   V a = A a + p B a = r_A + p (Q_A + B a),   A a = r_A + Q_A p
// and for each component X in {A, B} two steps:
//   step 1: Q = floor(X a' / R) from the columns >= S - 1 of X a' only: S (S + 1) / 2 MACs, Q at most S + 1
//           below the exact floor (the dropped columns are worth < S R);
//   step 2: X' = init + X a - Q p from the columns 0 .. S - 1, as init + X a + Q (R - p) mod R (unsigned 64-bit
//           accumulators): S (S + 1) MACs, exact because the true value lies in [0, R).
// Shoup's bound A a / p - A a' / R in [0, A / R) keeps A < (S + 3) p and B < 2 (S + 3) p, far below R.
// 3 S^2 + 3 S MACs per product against 4 S^2 for the Montgomery pass pair (and no q_j multiplications).
// The first row is the start: c0 T_0 = (1 + p gamma) a_0 (1 + p b_0) is the pair (a_0, 0) with gamma R and b_0 R in the
// b sum (fbs_gamma_words), so K - 1 products follow. After them the b sum is applied once (fbp_apply_bsum), then the
// pair is reduced to canonical.
#pragma once
#include "kernels_fbp.hpp"

namespace fpai {

template <int S>
struct FbsGeom;
template <>
struct FbsGeom<19> {   // 1024-bit keys: p_h < 2^512, R = 2^532
  static constexpr int PW = 16, QA = 5, QAP = 5, QB = 4;
};
template <>
struct FbsGeom<37> {   // 2048-bit keys: p_h < 2^1024, R = 2^1036
  static constexpr int PW = 32, QA = 10, QAP = 10, QB = 8;
};
template <int S>
constexpr int fbs_row_quads() { return FbsGeom<S>::QA + FbsGeom<S>::QAP + FbsGeom<S>::QB; }

// Row-layout A/B (round 5; tools/ab_fbs_rows.sh): builds of this header with FBS_AB set are
// measurement-only libraries, never the product. FBS_AB & 1 ("T", traffic): rows addressed at a 384-B stride (three
// aligned 128-B lines) and only the b R quads that fit in them fetched (the rest zero) -- the bytes of packed 384-B
// rows, wrong ciphertexts; FBS_AB & 2 ("I", instructions): every digit of a and a' costs the v_alignbit + v_and that
// cutting a 28-bit digit out of packed 32-bit words costs (on the same digit: same ciphertexts).
// FBS_AB & 4 ("D"): k_fb_digits fused into k_fbs -- each element-half's even lane draws and reduces
// its exponent and cuts the digits in a prologue (kernels_fb.hpp fb_digits_elem, staged in the wave's second row
// buffer), stores them, and the product loop reads them back from L2 (agent-scope loads: another block may hold the
// line in its L1); the host launches no k_fb_digits. Same digits, same ciphertexts.
#ifndef FBS_AB
#define FBS_AB 0
#endif
template <int S>
constexpr int fbs_row_stride() { return (FBS_AB & 1) && S == 37 ? 24 : fbs_row_quads<S>(); }   // quads between rows
template <int S>
constexpr int fbs_b_fetch() { return (FBS_AB & 1) ? FbsGeom<S>::QB / 4 : FbsGeom<S>::QB / 2; }   // b R quads per lane
__device__ __forceinline__ uint32_t fbs_ab_extract(uint32_t d) {
#if FBS_AB & 2
  uint32_t r, z = 0;
  asm volatile("v_alignbit_b32 %0, %1, %2, %3" : "=v"(r) : "v"(d), "v"(d), "v"(z));
  asm volatile("v_and_b32 %0, 0x0fffffff, %0" : "+v"(r));
  return r;
#else
  return d;
#endif
}
template <int S>
constexpr int fbs_lds_quads() { return FbsGeom<S>::QA + FbsGeom<S>::QAP; }

// step 1, digit J of a' (columns >= S - 1): P[k - (S - 1)] for k = i + J >= S - 1
template <int S, int T, class Rd>
__device__ __forceinline__ void fbs_q_digit(uint64_t (&P)[S + 1], const uint32_t (&X)[S], Rd& rd) {
  constexpr int J = S - 1 - T;
  const uint32_t d = rd(std::integral_constant<int, T>{});
#pragma unroll
  for (int i = S - 1 - J; i < S; ++i) P[i + J - (S - 1)] += (uint64_t)X[i] * d;
  // (no empty-asm pins here, unlike step 2: one MAC per column and digit leaves LLVM nothing to re-associate, and
  // each pinned block cost an s_nop before the next MAC -- round 6, profiles/r06d_ab_fbs_pins_startcols.txt)
  __builtin_amdgcn_sched_barrier(0);
}
template <int S, class Rd, int... Ts>
__device__ __forceinline__ void fbs_q_all(uint64_t (&P)[S + 1], const uint32_t (&X)[S], Rd& rd, std::integer_sequence<int, Ts...>) {
  (fbs_q_digit<S, Ts>(P, X, rd), ...);
}
// Q: the limbs of floor(X a' / R) (truncated, above); rd yields the digits of a', J = S-1 .. 0
template <int S, class Rd>
__device__ __forceinline__ void fbs_quotient(const uint32_t (&X)[S], Rd& rd, uint32_t (&q)[S]) {
  uint64_t P[S + 1];
#pragma unroll
  for (int i = 0; i <= S; ++i) P[i] = 0;
  fbs_q_all<S>(P, X, rd, std::make_integer_sequence<int, S>{});
  uint64_t c = P[0] >> lane::LB;
#pragma unroll
  for (int i = 1; i <= S; ++i) {
    const uint64_t v = P[i] + c;
    q[i - 1] = lane::limb32(v);
    c = v >> lane::LB;
  }
}

// step 2, digit J of a: P[i + J] += X_i a_J + Q_i pbar_J for i + J < S, pbar = R - p (limbs 2^28 - p_0, then
// 2^28 - 1 - p_j): X a + Q (R - p) = X a - Q p mod R, all unsigned (v_mad_u64_u32 only; columns < 2 S 2^56 < 2^64)
template <int S, int J, class Rd>
__device__ __forceinline__ void fbs_r_digit(uint64_t (&P)[S], const uint32_t (&X)[S], const uint32_t (&q)[S],
                                            const uint32_t (&m)[S], Rd& rd) {
  const uint32_t d = rd(std::integral_constant<int, J>{});
  const uint32_t pb = J == 0 ? (lane::LMASK + 1u) - m[0] : lane::LMASK - m[J];
#pragma unroll
  for (int i = 0; i + J < S; ++i) {
    P[i + J] += (uint64_t)X[i] * d;
    P[i + J] += (uint64_t)q[i] * pb;
  }
#pragma unroll
  for (int i = J; i < S; ++i) asm volatile("" : "+v"(P[i]));   // (without them LLVM fuses the two MACs into mul_lo + add3)
  __builtin_amdgcn_sched_barrier(0);
}
template <int S, class Rd, int... Js>
__device__ __forceinline__ void fbs_r_all(uint64_t (&P)[S], const uint32_t (&X)[S], const uint32_t (&q)[S], const uint32_t (&m)[S],
                                          Rd& rd, std::integer_sequence<int, Js...>) {
  (fbs_r_digit<S, Js>(P, X, q, m, rd), ...);
}

// x <- x mod m for x < 2^7 m, counting the multiples into t: the quotient estimated from the top two limbs
// (fb_shoup_possible: m > 2^(28 (S - 1)), so the estimate's error is far below one), subtracted in one signed pass,
// then at most two conditional subtractions (in place of 6-7 shift-and-subtract passes).
template <int S>
__device__ __forceinline__ void fbs_reduce_est(uint32_t (&x)[S], const uint32_t (&m)[S], uint32_t& t) {
  const double xt = (double)x[S - 1] * 268435456.0 + (double)x[S - 2];
  const double mt = (double)m[S - 1] * 268435456.0 + (double)m[S - 2] + 1.0;
  const double qe = xt / mt - 1.0 / 1048576.0;
  const int32_t q = qe > 0.0 ? (int32_t)qe : 0;   // floor(x / m) - 1 <= q <= floor(x / m)
  {
    int64_t c = 0;
    const int32_t nq = -q;
#pragma unroll
    for (int i = 0; i < S; ++i) {
      const int64_t v = (int64_t)x[i] + (int64_t)nq * (int32_t)m[i] + c;
      x[i] = (uint32_t)v & lane::LMASK;
      c = v >> lane::LB;
    }
  }
  t += (uint32_t)q;
#pragma unroll 1
  for (int r = 0; r < 2; ++r) {
    int32_t c = 0;
    uint32_t d[S];
#pragma unroll
    for (int i = 0; i < S; ++i) {
      const int32_t v = (int32_t)x[i] - (int32_t)m[i] + c;
      d[i] = (uint32_t)v & lane::LMASK;
      c = v >> lane::LB;
    }
    const bool lt = c != 0;
#pragma unroll
    for (int i = 0; i < S; ++i) x[i] = lt ? x[i] : d[i];
    t += lt ? 0u : 1u;
  }
}

// the S limbs of a from the pair's row (a reader over quads 0 .. QA-1)
template <int S, class Rd, int... Ts>
__device__ __forceinline__ void fbs_read_limbs(uint32_t (&x)[S], Rd& rd, std::integer_sequence<int, Ts...>) {
  ((x[Ts] = rd(std::integral_constant<int, Ts>{})), ...);
}

template <int S, int HW, int... Js>
__device__ __forceinline__ void fbs_gamma_pick(const uint32_t (&g)[S], bool odd, uint32_t (&w)[HW], uint32_t& wc,
                                               std::integer_sequence<int, Js...>) {
  ((w[Js] = odd ? fb_word<S, HW + Js>(g) : fb_word<S, Js>(g)), ...);
  wc = odd ? fb_word<S, 2 * HW>(g) : 0u;
}

// The start of the b sum: c0 = 1 + n M = 1 + p_h gamma, gamma = (n / p_h) M mod p_h, is the factored value
// 1 (1 + p_h gamma), so the product starts from the first row's (a_0, 0) and gamma R joins the b R words: this lane's
// words tig HW .. tig HW + HW - 1 of gamma R (unreduced: a sum of 8-bit chunks of |M| times (n / p_h) 2^(8 c) R mod p_h,
// < 2040 p_h, or 2^11 p_h minus that for M < 0) and, in the odd lane, word PW as the carry word. With the K rows'
// b R words (< p_h each) the sum stays below 2^12 p_h <= R = 2^(28 S): fbp_apply_bsum's S-limb operand.
template <int S, int HW>
__device__ __forceinline__ void fbs_gamma_words(int64_t M, const FbpHalf* __restrict__ H, bool odd, uint32_t (&w)[HW],
                                                uint32_t& wc) {
  const bool neg = M < 0;
  const uint64_t mag = neg ? (uint64_t)0 - (uint64_t)M : (uint64_t)M;
  uint32_t mc[FBP_NC];
#pragma unroll
  for (int c = 0; c < FBP_NC; ++c) mc[c] = (uint32_t)((mag >> (FBP_CB * c)) & ((1ull << FBP_CB) - 1ull));
  const uint32_t* nm = opaque_uniform(H->nmR);
  const uint32_t* pb = opaque_uniform(H->pbig);
  uint32_t g[S];
  int64_t carry = 0;
#pragma unroll
  for (int j = 0; j < S; ++j) {
    uint64_t s = 0;
#pragma unroll
    for (int c = 0; c < FBP_NC; ++c) s += (uint64_t)nm[c * S + j] * mc[c];
    const int64_t v = carry + (neg ? (int64_t)pb[j] - (int64_t)s : (int64_t)s);
    g[j] = (uint32_t)v & lane::LMASK;
    carry = v >> lane::LB;
  }
  fbs_gamma_pick<S, HW>(g, odd, w, wc, std::make_integer_sequence<int, HW>{});
}
// ---------------------------------------------------------------- the sampler on split pairs
// Element-half e on lanes 2e, 2e+1 (kernels_sgp.hpp's layout): the even lane keeps A, the odd lane B, and both run
// the same Shoup pass on their own component at once -- step 1 (their quotient), then step 2, the odd lane's
// accumulator starting at the even lane's Q_A (one DPP per limb). Per lane: the component, Q and one accumulator
// row (148 VGPRs in step 2) and half of the b sum (16 words + a carry).
//
// Rows in LDS, double-buffered (product k reads buffer k & 1 while row k+1 streams into the other): DMA instruction
// g of a wave fetches quad 2g + t of pair p's row on lane 2p + t, landing at [g][lane] (1 KB per instruction), so
// quad Q of the pair's row sits at (Q / 2) KB + (Q & 1) 16 B from the pair's base: both lanes of a pair read the same
// addresses (a broadcast), consecutive pairs consecutive 32 B. The b R quads go to registers (QB / 2 per lane).
// At S = 37: 10 DMA instructions, 2 x 10 KB per wave, 80 KB per block -- two blocks fill the CU's 160 KB.
template <int S>
constexpr int fbs_dma_insts() { return (FbsGeom<S>::QA + FbsGeom<S>::QAP + 1) / 2; }
template <int S>
constexpr int fbs_wave_buf_bytes() { return fbs_dma_insts<S>() * 1024; }
template <int Q>
constexpr int fbs_pair_off() { return (Q >> 1) * 1024 + (Q & 1) * 16; }

// limbs of a' (quads QA .. QA+QAP-1 of the row, consumed J = S-1 .. 0) or of a (quads 0 .. QA-1, J = 0 .. S-1) from
// the pair's row in LDS: limb J is word J % 4 of quad J / 4. Quads are read DQ ahead in consumption order, with exact
// lgkmcnt waits (only these reads are in flight: the row DMA and the digit loads count in vmcnt).
template <int S, int NQ, int Q0, bool DESC, int DQ>
struct FbsPairReader {
  static_assert(4 * NQ >= S, "limbs per number");
  uint32_t addr;
  fbp_u32x4 q[NQ];
  static constexpr int dig(int t) { return DESC ? S - 1 - t : t; }
  static constexpr int rank(int qd) { return DESC ? NQ - 1 - qd : qd; }
  static constexpr int quad_at(int r) { return DESC ? NQ - 1 - r : r; }
  static constexpr int need(int t) { return rank(dig(t) / 4); }   // monotone in t
  static constexpr int issued(int t) { return t < 0 ? -1 : (need(t) + DQ < NQ - 1 ? need(t) + DQ : NQ - 1); }
  template <int R0, int... Rs>
  __device__ __forceinline__ void issue(std::integer_sequence<int, Rs...>) {
    ((q[quad_at(R0 + Rs)] = lds_quad_rd<fbs_pair_off<Q0 + quad_at(R0 + Rs)>()>(addr)), ...);
  }
  template <int T>
  __device__ __forceinline__ uint32_t operator()(std::integral_constant<int, T>) {
    constexpr int from = issued(T - 1) + 1, to = issued(T);
    issue<from>(std::make_integer_sequence<int, (to >= from ? to - from + 1 : 0)>{});
    constexpr int J = dig(T), g = J / 4;
    if constexpr (T == 0 || need(T) > need(T - 1)) {
      constexpr int pending = to - need(T);
      static_assert(pending >= 0 && pending <= 15, "lgkmcnt range");
      asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(q[g]) : "i"(pending));
    }
    return fbs_ab_extract(quad_word<J % 4>(q[g]));
  }
};

// row `row` (this pair's) -> the wave's LDS buffer at lb (wave-uniform): quads 2g + t on lane 2p + t; and this lane's
// half of the b R quads (QB / 2: lane t takes words t PW / 2 .. (t + 1) PW / 2 - 1) into bv
template <int S>
__device__ __forceinline__ void fbs_row_fetch(const uint4* row, uint32_t lb, int tig, fbp_u32x4 (&bv)[FbsGeom<S>::QB / 2]) {
  using G = FbsGeom<S>;
  const uint4* src = row + tig;
#pragma unroll
  for (int g = 0; g < fbs_dma_insts<S>(); ++g) {
    uint32_t dst = lb + (uint32_t)(g * 1024);
    asm volatile("" : "+s"(dst));
    __builtin_amdgcn_global_load_lds((const void*)(src + 2 * g), (__attribute__((address_space(3))) void*)(size_t)dst, 16, 0, 0);
  }
  constexpr int QH = G::QB / 2, QF = fbs_b_fetch<S>();
  const fbp_u32x4* b = reinterpret_cast<const fbp_u32x4*>(row + G::QA + G::QAP + QF * tig);
#pragma unroll
  for (int q = 0; q < QH; ++q) bv[q] = q < QF ? b[q] : fbp_u32x4{0u, 0u, 0u, 0u};
}

#if FLEXPAI_XCHECK
// test build (guard.hpp): digit k of element ee in half h, its offset and value checked; the row index checked
__device__ __forceinline__ uint32_t fbs_guard_digit(const FbpParams& p, int h, int k, long long ee, unsigned int s_off,
                                                    unsigned int s_val) {
  const uint32_t d = p.digits[FPAI_GUARD_IDX(p.g, s_off, ((size_t)h * p.K + k) * p.n + ee, p.g.digits, ee)];
  return (uint32_t)FPAI_GUARD_IDX(p.g, s_val, d, 1ull << p.W, ee);
}
#define FBS_DIGIT(k) fbs_guard_digit(p, half, (k), ee, GS_FBS_DIGIT, GS_FBS_DVAL)
#define FBS_ROW(k, d) FPAI_GUARD_IDX(p.g, GS_FBS_ROW, ((size_t)(k) << W) + (d), p.g.rows, ee)
#elif FBS_AB & 4
#define FBS_DIGIT(k) __hip_atomic_load(const_cast<uint32_t*>(dg + (size_t)(k) * p.n), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
#define FBS_ROW(k, d) (((size_t)(k) << W) + (d))
#else
#define FBS_DIGIT(k) dg[(size_t)(k) * p.n]
#define FBS_ROW(k, d) (((size_t)(k) << W) + (d))
#endif

template <int S>
__global__ __launch_bounds__(LANE_BLOCK, 2) void k_fbs(FbpParams p) {
  using G = FbsGeom<S>;
  constexpr int PW = G::PW, TQ = fbs_row_stride<S>(), WB = fbs_wave_buf_bytes<S>();
  static_assert(PW == 32 || PW == 16, "b sum halves");
  constexpr int HW = PW / 2;   // b sum words per lane
  __shared__ __attribute__((aligned(16))) uint8_t lbuf[(LANE_BLOCK / 64) * 2 * WB];
  const int half = blockIdx.y;
  const FbpHalf* H = p.halves + half;
  uint32_t m[S];
#pragma unroll
  for (int j = 0; j < S; ++j) m[j] = H->p[j];
  const uint32_t mprime = H->mprime;
  const uint4* table = H->table;
  const int K = p.K, W = p.W;
  const int lane = threadIdx.x & 63;
  const int tig = threadIdx.x & 1;
  const bool odd = tig != 0;
  const int pib = threadIdx.x >> 1;
  typedef __attribute__((address_space(3))) uint8_t lds_u8;
  const uint32_t wbase = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(lds_u8*)(lbuf + (threadIdx.x >> 6) * 2 * WB));
  const uint32_t pbase = wbase + (uint32_t)((lane >> 1) * 32);   // this pair's quad 0 in buffer 0
  constexpr int PAIRS = LANE_BLOCK / 2;
  for (long long base = (long long)blockIdx.x * PAIRS; base < p.n; base += (long long)gridDim.x * PAIRS) {
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
    uint32_t X[S];   // even lane: A; odd lane: B -- (a_0, 0) from the first row (below)
    const uint32_t* dg = p.digits + (size_t)half * K * p.n + ee;
    (void)dg;
    uint32_t bsw[HW], bcc;   // this lane's half of the b sum, started at gamma R (c0 = 1 (1 + p gamma), factored)
    fbs_gamma_words<S, HW>(M, H, odd, bsw, bcc);
    static_assert(G::QB / 2 == HW / 4, "b R quads per lane");
    fbp_u32x4 bv[G::QB / 2];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the previous element's reads of both buffers are done
#if FBS_AB & 4
    {   // this element-half's digits (the even lane; staged in the wave's second row buffer), stored and waited
      // (the parameters from device memory through an opaque pointer: held in registers across the element loop, they
      // had spilled 140 VGPRs, 15 scratch accesses of them inside the product loop)
      const FbDigitParams* dp = reinterpret_cast<const FbDigitParams*>(opaque_uniform(reinterpret_cast<const uint32_t*>(p.dig)));
      const FbDigitKey dk = fb_digit_key(*dp, half);
      uint32_t* arow = reinterpret_cast<uint32_t*>(lbuf + (threadIdx.x >> 6) * 2 * WB + WB) + (lane >> 1) * 37;
      if (!odd) fb_digits_elem<37>(*dp, dk, half, ee, arow);
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    }
#endif
    fbs_row_fetch<S>(table + (size_t)FBS_ROW(0, FBS_DIGIT(0)) * TQ, wbase, tig, bv);
    uint32_t dn = K > 1 ? FBS_DIGIT(1) : 0u;
    for (int k = 0; k < K; ++k) {
      lds_dma_wait();                                     // row k in buffer k & 1, its b R in bv, digit k+1 in dn
      {                                                   // this lane's half of the b sum
        unsigned int c = 0;
#pragma unroll
        for (int q = 0; q < HW / 4; ++q) {
          bsw[4 * q] = __builtin_addc(bsw[4 * q], bv[q].x, c, &c);
          bsw[4 * q + 1] = __builtin_addc(bsw[4 * q + 1], bv[q].y, c, &c);
          bsw[4 * q + 2] = __builtin_addc(bsw[4 * q + 2], bv[q].z, c, &c);
          bsw[4 * q + 3] = __builtin_addc(bsw[4 * q + 3], bv[q].w, c, &c);
        }
        bcc += c;
      }
      const uint32_t cur = pbase + (uint32_t)((k & 1) * WB);
      if (k + 1 < K) {                                    // row k+1 -> the other buffer (read two products ago: done)
        fbs_row_fetch<S>(table + FBS_ROW(k + 1, dn) * TQ, wbase + (uint32_t)(((k + 1) & 1) * WB), tig, bv);
        dn = k + 2 < K ? FBS_DIGIT(k + 2) : 0u;
      } else {
#pragma unroll
        for (int q = 0; q < G::QB / 2; ++q) bv[q] = fbp_u32x4{0u, 0u, 0u, 0u};
      }
      __builtin_amdgcn_sched_barrier(0);
      if (k == 0) {   // c0 T_0 = (1 + p gamma) a_0 (1 + p b_0): the pair (a_0, 0), the factors in the b sum -- no product
        FbsPairReader<S, G::QA, 0, false, 1> ra{cur};
        fbs_read_limbs<S>(X, ra, std::make_integer_sequence<int, S>{});
#pragma unroll
        for (int i = 0; i < S; ++i) X[i] = odd ? 0u : X[i];
        continue;
      }
      uint32_t q[S];
      {
        FbsPairReader<S, G::QAP, G::QA, true, 1> r1{cur};
        fbs_quotient<S>(X, r1, q);
      }
      {   // step 2; the odd lane's accumulator columns start at the even lane's Q_A (one DPP'd AND per limb, before the
        // digits: round 6, against one DPP, one MAC by 0 / 1 and a DPP hazard nop per limb in the normalisation)
        uint64_t P[S];
        uint32_t om = odd ? ~0u : 0u;
        asm volatile("" : "+v"(om));   // (a mask, not a select)
#pragma unroll
        for (int i = 0; i < S; ++i)
          P[i] = (uint64_t)((uint32_t)__builtin_amdgcn_update_dpp(0, (int)q[i], 0xA0, 0xF, 0xF, false) & om);   // quad_perm [0,0,2,2]
        FbsPairReader<S, G::QA, 0, false, 1> r2{cur};
        fbs_r_all<S>(P, X, q, m, r2, std::make_integer_sequence<int, S>{});
        uint64_t c = 0;   // (mod R: the carry out of limb S - 1 is dropped)
#pragma unroll
        for (int i = 0; i < S; ++i) {
          const uint64_t v = P[i] + c;
          X[i] = lane::limb32(v);
          c = v >> lane::LB;
        }
      }
    }
    // the even lane: A < (S + 3) p to canonical (its multiples of p move into B), B from the odd lane, the b sum
    // (its high half from the odd lane), B + REDC(A bs R), B to canonical
    uint32_t B[S], bs[PW], bc;
#pragma unroll
    for (int j = 0; j < S; ++j) B[j] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)X[j], 0xF5, 0xF, 0xF, false);   // [1,1,3,3]
    {
      uint32_t c = 0;   // bs = lo + 2^(32 HW) (hi + c_lo) + 2^(32 PW) c_hi
#pragma unroll
      for (int j = 0; j < HW; ++j) {
        bs[j] = bsw[j];
        const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)bsw[j], 0xF5, 0xF, 0xF, false);
        const uint64_t v = (uint64_t)hi + (j == 0 ? bcc : 0u) + c;
        bs[HW + j] = (uint32_t)v;
        c = (uint32_t)(v >> 32);
      }
      bc = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)bcc, 0xF5, 0xF, 0xF, false) + c;
    }
    if (!odd && valid) {
      uint32_t t = 0;
      fbs_reduce_est<S>(X, m, t);                         // (S + 3) p < 2^7 p
      {
        uint32_t c = t;
#pragma unroll
        for (int j = 0; j < S; ++j) {
          const uint32_t v = B[j] + c;
          B[j] = v & lane::LMASK;
          c = v >> lane::LB;
        }
      }
      fbp_apply_bsum<S, PW>(X, B, bs, bc, m, mprime);     // B + REDC(A bs R) < 2 (S + 3) p + 64 + 2 p < 128 p
      uint32_t tb = 0;
      fbs_reduce_est<S>(B, m, tb);
      uint32_t* o = p.out + fbp_pair_index<S>(e, half, p.n);
      if (FPAI_GUARD_OK(p.g, GS_FBS_OUT, fbp_pair_index<S>(e, half, p.n) + (2 * S - 1) * 64, p.g.out, e)) {
#pragma unroll
        for (int j = 0; j < 2 * S; ++j) o[j * 64] = j < S ? X[j] : B[j - S];
      }
    }
  }
}

// ---------------------------------------------------------------- Shoup-form rows from the pair tables' lo/hi
// entries and inverses (k_fbp_lohi, k_fbp_inv_fwd/bwd): per entry T R = lo hi R^-1 as a pair, T = (T R)(1, 0) R^-1
// canonical (A_T, B_T); a = A_T; b = B_T A_T^-1 = REDC(B_T X) with X = REDC(inv_lo inv_hi) = A_T^-1 R (the lo/hi
// entries and their inverses are R-forms of l_lo, l_hi and their inverses, A_T = l_lo l_hi mod p), b R =
// REDC(b R^2); a' = floor(a R / p) from floor(a mu / R), mu = floor(R^2 / p), raised by one when a R - a' p >= p.
struct FbsConst {
  const uint32_t* mu;      // floor(R^2 / p_h): S + 1 limbs (+ 1 spare)
  const uint32_t* r2;      // R^2 mod p_h, S limbs
};

template <int S, int... Gs>
__device__ __forceinline__ void fbs_store_words(uint4* __restrict__ dst, const uint32_t (&x)[S], std::integer_sequence<int, Gs...>) {
  ((dst[Gs] = make_uint4(fb_word<S, 4 * Gs>(x), fb_word<S, 4 * Gs + 1>(x), fb_word<S, 4 * Gs + 2>(x), fb_word<S, 4 * Gs + 3>(x))),
   ...);
}
template <int N, int I>
__device__ __forceinline__ uint32_t fbs_limb_or0(const uint32_t (&x)[N]) {
  if constexpr (I < N) return x[I];
  else return 0u;
}
template <int S, int N, int... Gs>   // limbs 0 .. S-1 of x, one per word, zero-padded to whole quads
__device__ __forceinline__ void fbs_store_limbs(uint4* __restrict__ dst, const uint32_t (&x)[N], std::integer_sequence<int, Gs...>) {
  ((dst[Gs] = make_uint4(4 * Gs < S ? fbs_limb_or0<N, 4 * Gs>(x) : 0u, 4 * Gs + 1 < S ? fbs_limb_or0<N, 4 * Gs + 1>(x) : 0u,
                         4 * Gs + 2 < S ? fbs_limb_or0<N, 4 * Gs + 2>(x) : 0u, 4 * Gs + 3 < S ? fbs_limb_or0<N, 4 * Gs + 3>(x) : 0u)),
   ...);
}

// a' = floor(a mu / R) by product scanning (fbs_fill_body): column T of A mu, A: S limbs, mu: S + 1 limbs, one running
// 64-bit sum (at most S + 1 products < 2^56 per column plus a carry < 2^36); columns S .. 2S are a'. Compile-time
// columns (a loop over 2S + 1 x S candidate products is too long for the unroller, which then left a branch per MAC).
template <int S, int T, int I>
__device__ __forceinline__ void fbs_ap_mac(uint64_t& acc, const uint32_t (&A)[S], const uint32_t* mu) {
  if constexpr (T - I >= 0 && T - I < S + 1) acc += (uint64_t)A[I] * mu[T - I];
}
template <int S, int T, int... Is>
__device__ __forceinline__ void fbs_ap_column(uint64_t& acc, const uint32_t (&A)[S], const uint32_t* mu,
                                              std::integer_sequence<int, Is...>) {
  (fbs_ap_mac<S, T, Is>(acc, A, mu), ...);
}
template <int S, int T>
__device__ __forceinline__ void fbs_ap_step(uint64_t& acc, uint32_t (&ap)[S + 1], const uint32_t (&A)[S], const uint32_t* mu) {
  fbs_ap_column<S, T>(acc, A, mu, std::make_integer_sequence<int, S>{});
  if constexpr (T >= S) ap[T - S] = (uint32_t)acc & lane::LMASK;
  acc >>= lane::LB;
}
template <int S, int... Ts>
__device__ __forceinline__ void fbs_ap_all(uint32_t (&ap)[S + 1], const uint32_t (&A)[S], const uint32_t* mu,
                                           std::integer_sequence<int, Ts...>) {
  uint64_t acc = 0;
  (fbs_ap_step<S, Ts>(acc, ap, A, mu), ...);
}
// the low S + 1 limbs of a R - a' p (signed running sum: at most S + 1 products < 2^56 subtracted per column)
template <int S, int T, int I>
__device__ __forceinline__ void fbs_apt_mac(int64_t& acc, const uint32_t (&ap)[S + 1], const uint32_t (&m)[S]) {
  if constexpr (T - I >= 0 && T - I < S) acc -= (int64_t)((uint64_t)ap[I] * m[T - I]);
}
template <int S, int T, int... Is>
__device__ __forceinline__ void fbs_apt_step(int64_t& acc, uint32_t (&tl)[S + 1], const uint32_t (&ap)[S + 1],
                                             const uint32_t (&A)[S], const uint32_t (&m)[S], std::integer_sequence<int, Is...>) {
  if constexpr (T == S) acc += (int64_t)A[0];
  (fbs_apt_mac<S, T, Is>(acc, ap, m), ...);
  tl[T] = (uint32_t)acc & lane::LMASK;
  acc >>= lane::LB;
}
template <int S, int... Ts>
__device__ __forceinline__ void fbs_apt_all(uint32_t (&tl)[S + 1], const uint32_t (&ap)[S + 1], const uint32_t (&A)[S],
                                            const uint32_t (&m)[S], std::integer_sequence<int, Ts...>) {
  int64_t acc = 0;
  (fbs_apt_step<S, Ts>(acc, tl, ap, A, m, std::make_integer_sequence<int, S + 1>{}), ...);
}

// One row per thread. UNI: every thread of the block shares the hi entry (2^(W/2) >= LANE_BLOCK, i.e. W >= 16), whose
// pair and inverse, with mu and R^2, the block stages once in LDS (sh); otherwise they come from global memory (round 5:
// a global load per digit of the hi entry, each waited, had made the fill latency-bound at 4.0 ns per row -- 34 ms of a
// fresh key's 95 ms at W = 16, 1.57 s of the W = 22 build).
template <int S, bool UNI>
__device__ __forceinline__ void fbs_fill_body(const FbpHalf* halves, const FbsConst* cst, int W, uint4* table0, uint4* table1,
                                              const GuardArgs& g, const uint32_t* sh) {
  using G = FbsGeom<S>;
  constexpr int TQ = fbs_row_quads<S>();
  const int ent = 1 << W;
  const int per = (ent + LANE_BLOCK - 1) / LANE_BLOCK;
  const int k = blockIdx.x / per;
  const int d = (blockIdx.x % per) * LANE_BLOCK + threadIdx.x;
  if (d >= ent) return;
  const int half = blockIdx.y;
  const FbpHalf* H = halves + half;
  const FbsConst* C = cst + half;
  uint4* table = half ? table1 : table0;
  const int LO = W / 2;
  const int dl = (int)FPAI_GUARD_IDX(g, GS_FILL_LOHI, (unsigned)(d & ((1 << LO) - 1)), FB_LO, d),
            dh = (int)FPAI_GUARD_IDX(g, GS_FILL_LOHI, (unsigned)(d >> LO), FB_LO, d);
  const uint32_t* lo = H->lohi + (((size_t)k * 2 + 0) * FB_LO + dl) * 2 * S;
  const uint32_t* hi = UNI ? sh : H->lohi + (((size_t)k * 2 + 1) * FB_LO + dh) * 2 * S;
  const uint32_t* ih = UNI ? sh + 2 * S : H->inv + (((size_t)k * 2 + 1) * FB_LO + dh) * S;
  const uint32_t* mu = UNI ? sh + 3 * S : C->mu;
  const uint32_t* r2 = UNI ? sh + 4 * S + 2 : C->r2;
  uint32_t m[S], A[S], B[S];
#pragma unroll
  for (int i = 0; i < S; ++i) {
    m[i] = (uint32_t)__builtin_amdgcn_readfirstlane(H->p[i]);   // uniform: SGPRs, not 37 VGPRs of the pair product's budget
    A[i] = lo[i];
    B[i] = lo[S + i];
  }
  pair::mont_mul<S>(A, B, [&](auto J) { return make_uint2(hi[decltype(J)::value], hi[S + decltype(J)::value]); }, m, H->mprime);
  pair::mont_mul<S>(A, B, [&](auto J) { return make_uint2(decltype(J)::value == 0 ? 1u : 0u, 0u); }, m, H->mprime);   // T R -> T
  pair::canon<S>(A, B, m);
  // a' = floor(a R / p): the high part of a mu, then one correction. Product scanning, one running 64-bit column sum
  // (a column takes at most S + 1 products < 2^56 plus a carry < 2^36: below 2^63), so no 2S-column array is live
  // (round 5: the row-scanning form kept 2S + 2 64-bit columns and spilled 624 B)
  uint32_t ap[S + 1];
  {
    fbs_ap_all<S>(ap, A, mu, std::make_integer_sequence<int, 2 * S + 1>{});
    // t = a R - a' p over the low S + 1 limbs (exact: 0 <= t < 2 p); a' += 1 when t >= p
    uint32_t tl[S + 1];
    fbs_apt_all<S>(tl, ap, A, m, std::make_integer_sequence<int, S + 1>{});
    // t >= p ?
    int32_t bw = 0;
#pragma unroll
    for (int t2 = 0; t2 < S + 1; ++t2) {
      const int32_t v = (int32_t)tl[t2] - (int32_t)(t2 < S ? m[t2] : 0u) + bw;
      bw = v >> lane::LB;
    }
    uint32_t inc = bw == 0 ? 1u : 0u;
#pragma unroll
    for (int t2 = 0; t2 < S + 1; ++t2) {
      const uint32_t v = ap[t2] + inc;
      ap[t2] = v & lane::LMASK;
      inc = v >> lane::LB;
    }
  }
  uint4* dst = table + FPAI_GUARD_IDX(g, GS_FILL_ROW, (size_t)k * ent + d, g.rows, d) * TQ;
  fbs_store_limbs<S>(dst, A, std::make_integer_sequence<int, G::QA>{});
  fbs_store_limbs<S>(dst + G::QA, ap, std::make_integer_sequence<int, G::QAP>{});   // a' < R: limb S is zero
  // b = B_T A_T^-1, b R: after a and a' are stored (their registers free again)
  uint32_t bR[S];
  {
    const uint32_t* il = H->inv + (((size_t)k * 2 + 0) * FB_LO + dl) * S;
    uint32_t X[S], Y[S];
#pragma unroll
    for (int i = 0; i < S; ++i) {
      X[i] = il[i];
      Y[i] = ih[i];
      bR[i] = B[i];
    }
    lane::mont_mul<S>(X, Y, m, H->mprime);               // A_T^-1 R
    lane::mont_mul<S>(bR, X, m, H->mprime);              // b = B_T A_T^-1
#pragma unroll
    for (int i = 0; i < S; ++i) Y[i] = r2[i];
    lane::mont_mul<S>(bR, Y, m, H->mprime);              // b R
    lane::cond_sub<S>(bR, m);
  }
  fbs_store_words<S>(dst + G::QA + G::QAP, bR, std::make_integer_sequence<int, G::QB>{});
}

template <int S>
__global__ __launch_bounds__(LANE_BLOCK, 2) void k_fbs_fill(const FbpHalf* halves, const FbsConst* cst, int K, int W, uint4* table0,
                                                         uint4* table1, GuardArgs g) {
  __shared__ uint32_t sh[5 * S + 2];   // hi pair [2S], its inverse [S], mu [S + 2], R^2 mod p [S]
  (void)K;
  const int LO = W / 2;
  if ((1 << LO) >= LANE_BLOCK) {   // block-uniform (W is a kernel argument)
    const int per = (1 << W) / LANE_BLOCK, k = blockIdx.x / per;
    const int dh = (int)FPAI_GUARD_IDX(g, GS_FILL_LOHI, (unsigned)(((blockIdx.x % per) * LANE_BLOCK) >> LO), FB_LO, k);
    const FbpHalf* H = halves + blockIdx.y;
    const FbsConst* C = cst + blockIdx.y;
    const uint32_t* hi = H->lohi + (((size_t)k * 2 + 1) * FB_LO + dh) * 2 * S;
    const uint32_t* ih = H->inv + (((size_t)k * 2 + 1) * FB_LO + dh) * S;
    for (int i = threadIdx.x; i < 5 * S + 2; i += LANE_BLOCK)
      sh[i] = i < 2 * S ? hi[i] : i < 3 * S ? ih[i - 2 * S] : i < 4 * S + 2 ? C->mu[i - 3 * S] : C->r2[i - 4 * S - 2];
    __syncthreads();
    fbs_fill_body<S, true>(halves, cst, W, table0, table1, g, sh);
  } else {
    fbs_fill_body<S, false>(halves, cst, W, table0, table1, g, nullptr);
  }
}

}  // namespace fpai
