// CRT decryption for 4096-bit keys on p-adic pairs split over a lane pair (bn_pair.hpp's algebra).
//
// p_h has 2048 bits, S = 74 limbs: a pair (A, B) with v = A + p_h B (mod p_h^2) and its two CIOS rows
// (2 x 74 64-bit accumulators) do not fit one lane next to the operand, so the rows go to the two lanes of a
// lane pair (element-half e: lanes 2e, 2e+1). Both lanes run the same instruction stream; the even lane computes
// the A row, the odd lane the B row, taking the even lane's reduction digit q1_j by one DPP step per digit:
//   even lane: P += a y_j + q1 p           (U = REDC(A1 A2), the A row)
//   odd lane : P += a y_j + q2 p, q2 = (P_J - q1) mprime   (the B row: REDC(a y - m) with m the even lane's
//              reduction digits q1_j, which the retiring shift drops instead of subtracting them, bn_pair.hpp)
// k_dec4_pre (and k_pe_pre) hold the same register operand in both lanes and stream different digits from LDS. The
// exponentiation (d4r_run, below) keeps each lane's own component in registers: a square (A, B)^2 takes A's digits
// from the even lane by DPP (P_even += A A_j, P_odd += B 2A_j): 2 x 2 S^2 lane-MACs against 2 (2S)^2 for the
// Montgomery square over the 148 limbs of p_h^2 that the TPI = 4 group engine runs (k_decrypt); a product x t
// takes two passes, z = REDC(A_x B_t) on the even lane, then REDC(A_x A_t) | REDC(B_x A_t - m) + z (< 4p, a valid
// operand: R >= 2^24 p_h).
//
//   k_dec4_pre  per element-half: c R as a pair (one split CIOS over the ciphertext's limbs against the
//               constant pair of R^(K+1))
//   k_dec4_pow  per element-half: c^(p_h - 1) on split pairs with B-free window multipliers (d4f_run, below),
//               left in plain form by a product with (1, 0)                     (decryptor.py:55-61)
//   k_dec4_L    per element-half: L_h = B of the canonical pair (A = 1; A = 0 for c == 0 mod p_h, L = B - 1),
//               m_h = L_h h_h mod p_h
//   k_dec4_fin  per element (lane group of 4, the bn_group engine): CRT (gmpy_math.py:31-40) and
//               FixedPointNumber.decode, as k_decrypt's last steps
#pragma once
#include "kernels_fb.hpp"   // opaque_uniform

namespace fpai {

constexpr int D4_S = 74;                     // limbs of p_h
constexpr int D4_PAIRS = LANE_BLOCK / 2;     // element-halves per block
constexpr int D4_SLOT = 4 * D4_S;            // LDS words per element-half: x [A][B], t [A][B]

struct Dec4Half {
  const uint32_t* p;       // p_h, S limbs
  const uint32_t* X1;      // (1 - R) mod p_h
  const uint32_t* XK;      // (1 - R^K) mod p_h, K = ciphertext chunks of S limbs
  const uint32_t* cK;      // pair of R^(K+1) mod p_h^2 ([A: S][B: S])
  const uint32_t* hR;      // h_h R mod p_h
  const uint32_t* prog;    // op list of the factored chain (d4f_run): table, p_h - 2, the two closing products
  int nprog;
  uint32_t mprime;
  const uint32_t* kf;      // [16][S] K'_t of the closing Horner sum (d4f_run; slot 0: -R mod p_h)
};

struct Dec4Params {
  const Dec4Half* halves;  // [2]
  long long n;
  const uint32_t* ct;
  int ct_words;
  int kchunks;
  uint32_t* x;             // [2][2S][n]: pairs (A: limbs 0..S-1, B: S..2S-1)
  uint32_t* mh;            // [2][S][n]
  uint32_t* scratch;       // per-lane tiles (LaneScratch, tile_quads<S> quads per tile)
};

template <int S, int J>
__device__ __forceinline__ void d4_step(uint64_t (&P)[S], const uint32_t (&a)[S], const uint32_t* __restrict__ dig,
                                        uint32_t& cur, int sh, const uint32_t (&m)[S], uint32_t mprime, bool subq) {
  const uint32_t y = cur << sh;
  if constexpr (J + 1 < S) cur = dig[J + 1];
#pragma unroll
  for (int i = 0; i < S; ++i) P[(i + J) % S] += (uint64_t)a[i] * y;
  const uint32_t q0 = ((uint32_t)P[J] * mprime) & lane::LMASK;
  const uint32_t q1 = __builtin_amdgcn_update_dpp(0u, q0, 0xA0, 0xF, 0xF, false);   // quad_perm [0,0,2,2]: even lane's q
  const uint32_t q = (((uint32_t)P[J] - (subq ? q1 : 0u)) * mprime) & lane::LMASK;
#pragma unroll
  for (int i = 0; i < S; ++i) P[(i + J) % S] += (uint64_t)q * m[i];
  P[(J + 1) % S] += P[J] >> lane::LB;   // B row: the low 28 bits are q1, dropped (bn_pair.hpp)
  P[J] = 0;
  lane::pin<S>(P);
  __builtin_amdgcn_sched_barrier(0);
}
// S digits dig[0..S) (shifted left by sh) against the register operand a; subq: this lane is the B row of a
// pair pass (it drops q1 of its even neighbour at each digit)
template <int S, int... Js>
__device__ __forceinline__ void d4_pass(uint64_t (&P)[S], const uint32_t (&a)[S], const uint32_t* __restrict__ dig, int sh,
                                        const uint32_t (&m)[S], uint32_t mprime, bool subq, std::integer_sequence<int, Js...>) {
  uint32_t cur = dig[0];
  (d4_step<S, Js>(P, a, dig, cur, sh, m, mprime, subq), ...);
}

__device__ __forceinline__ void d4_fence() { wave_lds_fence(); }

// ---------------------------------------------------------------- c~ = c R mod p_h^2 as a pair
// The constant pair of R^(K+1) (A in the even lane, B in the odd) times the ciphertext's K S digits (staged
// in LDS), R^-K: one split CIOS, the odd row started at (1 - R^K) mod p_h.
template <int S>
__global__ __launch_bounds__(LANE_BLOCK, 1) void k_dec4_pre(Dec4Params p) {
  __shared__ uint32_t lds[D4_PAIRS * D4_SLOT];
  const int half = blockIdx.y;
  const Dec4Half* H = p.halves + half;
  uint32_t m[S];
#pragma unroll
  for (int j = 0; j < S; ++j) m[j] = H->p[j];
  const uint32_t mprime = H->mprime;
  const int tig = threadIdx.x & 1;
  const bool odd = tig != 0;
  const int pib = threadIdx.x >> 1;
  uint32_t* sx = lds + pib * D4_SLOT;
  for (long long base = (long long)blockIdx.x * D4_PAIRS; base < p.n; base += (long long)gridDim.x * D4_PAIRS) {
    const long long e = base + pib;
    const bool valid = e < p.n;
    const long long ee = valid ? e : p.n - 1;
    {
      const uint32_t* cw = p.ct + ee * p.ct_words;
      const int nw = p.ct_words;
      d4_fence();
      for (int k = tig; k < p.kchunks * S; k += 2) {
        const int bit = k * lane::LB, wi = bit >> 5, sh = bit & 31;
        const uint64_t lo = wi < nw ? (uint64_t)cw[wi] : 0ull;
        const uint64_t hi = wi + 1 < nw ? (uint64_t)cw[wi + 1] : 0ull;
        sx[k] = (uint32_t)(((hi << 32) | lo) >> sh) & lane::LMASK;
      }
      d4_fence();
    }
    uint32_t a[S];
#pragma unroll
    for (int i = 0; i < S; ++i) a[i] = H->cK[tig * S + i];
    uint64_t P[S];
#pragma unroll
    for (int i = 0; i < S; ++i) P[i] = 0;
#pragma unroll 1
    for (int k = 0; k < p.kchunks; ++k)
      d4_pass<S>(P, a, sx + k * S, 0, m, mprime, odd, std::make_integer_sequence<int, S>{});
    uint32_t y[S];
    lane::normalize<S>(P, y);
    if (valid) {
#pragma unroll
      for (int i = 0; i < S; ++i) p.x[((size_t)half * 2 * S + tig * S + i) * p.n + e] = y[i];
    }
  }
}

// ---------------------------------------------------------------- x_h = c~^(p_h - 1), plain pair
// The lane machine of kernels_crt.hpp (same op list: SQR, MUL with the multiplier from a tile, the constant,
// or as set, A_FROM_T, STORE, B_SET) on split pairs. Each lane keeps its own component of every tile (the
// even lane A, the odd lane B).
template <int S, int... Gs>
__device__ __forceinline__ void d4_tile_store(const LaneScratch& t, int k, const uint32_t* src, std::integer_sequence<int, Gs...>) {
  constexpr int TQ = tile_quads<S>();
  ((t.quad(k * TQ + Gs) = make_uint4(4 * Gs < S ? src[4 * Gs] : 0u, 4 * Gs + 1 < S ? src[4 * Gs + 1] : 0u,
                                     4 * Gs + 2 < S ? src[4 * Gs + 2] : 0u, 4 * Gs + 3 < S ? src[4 * Gs + 3] : 0u)),
   ...);
}
template <int S, int... Gs>
__device__ __forceinline__ void d4_tile_load(const LaneScratch& t, int k, uint32_t* dst, std::integer_sequence<int, Gs...>) {
  constexpr int TQ = tile_quads<S>();
  uint4 v[sizeof...(Gs)];
  ((v[Gs] = t.quad(k * TQ + Gs)), ...);
  d4_fence();
  (((4 * Gs < S ? (dst[4 * Gs] = v[Gs].x) : 0u), (4 * Gs + 1 < S ? (dst[4 * Gs + 1] = v[Gs].y) : 0u),
    (4 * Gs + 2 < S ? (dst[4 * Gs + 2] = v[Gs].z) : 0u), (4 * Gs + 3 < S ? (dst[4 * Gs + 3] = v[Gs].w) : 0u)),
   ...);
  d4_fence();
}

// ---- k_dec4_pow: the components in registers (round 3)
// Each lane keeps ITS component of x in registers (the even lane A, the odd lane B), so a square needs no LDS: the
// digits are the even lane's own limbs, A[j], broadcast to the odd lane by one DPP per digit and doubled there
// (P_even += A A_j, P_odd += B 2A_j). A product x t (t in the LDS multiplier st = [A_t][B_t]) runs two passes:
//   pass A: P += a B_t[j] on both lanes; the even lane's z = REDC(A_x B_t) is written over st's B half (the odd
//           lane's product is discarded);
//   pass 1: P += a A_t[j] with the split reduction (the odd lane drops the even lane's q1); then the odd lane adds
//           z, so B' = REDC(B_x A_t - m) + REDC(A_x B_t) < 4p and the even lane's A' = REDC(A_x A_t).
// Only the multiplier lives in LDS (2S words per lane pair instead of 4S): two blocks of 256 lanes per CU, two
// waves per SIMD. A multiplier kept across products (LOP_B_READY without a prefetch: the table's x~^2) has its B
// half clobbered by z: LOP_B_SET also stores it in a spare tile, reloaded before each later product that keeps it.
constexpr int D4R_SLOT = 2 * D4_S;       // LDS words per element-half: the multiplier [A][B]
constexpr int D4R_KEPT = LANE_NTILE;     // spare tile (in the lane scratch's stage-A buffer, unused here)
static_assert((LANE_NTILE + 1) * tile_quads<D4_S>() <= LANE_NTILE * tile_quads<D4_S>() + RBUF_WORDS / 4,
              "the spare tile fits the lane scratch");

template <int S, int J>
__device__ __forceinline__ void d4r_sqr_step(uint64_t (&P)[S], const uint32_t (&a)[S], int tig, const uint32_t (&m)[S],
                                             uint32_t mprime, bool odd) {
  const uint32_t y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a[J], 0xA0, 0xF, 0xF, false) << tig;   // 2^tig A_J
#pragma unroll
  for (int i = 0; i < S; ++i) P[(i + J) % S] += (uint64_t)a[i] * y;
  const uint32_t q0 = ((uint32_t)P[J] * mprime) & lane::LMASK;
  const uint32_t q1 = __builtin_amdgcn_update_dpp(0u, q0, 0xA0, 0xF, 0xF, false);
  P[J] += odd ? (uint64_t)(lane::LMASK - q1) : 0ull;   // (the odd row started at (1 - R) mod p: non-negative)
  const uint32_t q = ((uint32_t)P[J] * mprime) & lane::LMASK;
#pragma unroll
  for (int i = 0; i < S; ++i) P[(i + J) % S] += (uint64_t)q * m[i];
  P[(J + 1) % S] += P[J] >> lane::LB;
  P[J] = 0;
  lane::pin<S>(P);
  __builtin_amdgcn_sched_barrier(0);
}
template <int S, int... Js>
__device__ __forceinline__ void d4r_sqr_pass(uint64_t (&P)[S], const uint32_t (&a)[S], int tig, const uint32_t (&m)[S],
                                             uint32_t mprime, bool odd, std::integer_sequence<int, Js...>) {
  (d4r_sqr_step<S, Js>(P, a, tig, m, mprime, odd), ...);
}

template <int S, int... Gs>
__device__ __forceinline__ void d4r_tile_store(const LaneScratch& t, int k, const uint32_t (&x)[S], std::integer_sequence<int, Gs...>) {
  constexpr int TQ = tile_quads<S>();
  ((t.quad(k * TQ + Gs) = make_uint4(4 * Gs < S ? x[4 * Gs] : 0u, 4 * Gs + 1 < S ? x[4 * Gs + 1] : 0u,
                                     4 * Gs + 2 < S ? x[4 * Gs + 2] : 0u, 4 * Gs + 3 < S ? x[4 * Gs + 3] : 0u)),
   ...);
}
template <int S, int... Gs>
__device__ __forceinline__ void d4r_tile_load(const LaneScratch& t, int k, uint32_t (&x)[S], std::integer_sequence<int, Gs...>) {
  constexpr int TQ = tile_quads<S>();
  uint4 v[sizeof...(Gs)];
  ((v[Gs] = t.quad(k * TQ + Gs)), ...);
  (((4 * Gs < S ? (x[4 * Gs] = v[Gs].x) : 0u), (4 * Gs + 1 < S ? (x[4 * Gs + 1] = v[Gs].y) : 0u),
    (4 * Gs + 2 < S ? (x[4 * Gs + 2] = v[Gs].z) : 0u), (4 * Gs + 3 < S ? (x[4 * Gs + 3] = v[Gs].w) : 0u)),
   ...);
}

// The op list (kernels_crt.hpp) on register components; st = this pair's multiplier [A][B] in LDS.
template <int S, class FinalB>
__device__ __forceinline__ void d4r_run(uint32_t (&a)[S], uint32_t* st, const LaneScratch& tl, const uint32_t* __restrict__ prog,
                                        int nprog, const uint32_t* x1, const uint32_t (&m)[S], uint32_t mprime, int tig,
                                        FinalB&& final_b) {
  constexpr int TQ = tile_quads<S>();
  using Q = std::make_integer_sequence<int, TQ>;
  const bool odd = tig != 0;
  const uint32_t oddmask = odd ? 0xFFFFFFFFu : 0u;
  bool bclob = false;   // st's B half holds a product's z, not the kept multiplier
  for (int i = 0; i <= nprog; ++i) {
    const uint32_t op = (i < nprog) ? lane_op(prog, i) : LOP_B_CONST;
    if (op & LOP_A_FROM_T) d4r_tile_load<S>(tl, (op >> 16) & 0xFF, a, Q{});
    const bool sqr = (op & LOP_SQR) != 0;
    if (sqr && (op & LOP_PREFETCH)) {
      d4_tile_load<S>(tl, (op >> 8) & 0xFF, st + tig * S, Q{});   // the next MUL's multiplier (B_READY)
      bclob = false;
    }
    uint64_t P[S];
    if (sqr) {
#pragma unroll
      for (int j = 0; j < S; ++j) P[j] = odd ? (uint64_t)x1[j] : 0ull;
      d4r_sqr_pass<S>(P, a, tig, m, mprime, odd, std::make_integer_sequence<int, S>{});
      lane::normalize<S>(P, a);
    } else {
      if (op & LOP_B_CONST) {
        d4_fence();
        final_b(st + tig * S);
        d4_fence();
      } else if (!(op & LOP_B_READY)) {
        d4_tile_load<S>(tl, (op >> 8) & 0xFF, st + tig * S, Q{});
      } else if (bclob) {
        d4_tile_load<S>(tl, D4R_KEPT, st + tig * S, Q{});
      }
      // pass A: z = REDC(A_x B_t) on the even lane, over st's B half
#pragma unroll
      for (int j = 0; j < S; ++j) P[j] = 0;
      d4_pass<S>(P, a, st + S, 0, m, mprime, false, std::make_integer_sequence<int, S>{});
      {
        uint32_t z[S];
        lane::normalize<S>(P, z);
        d4_fence();
        if (!odd) {
#pragma unroll
          for (int j = 0; j < S; ++j) st[S + j] = z[j];
        }
        d4_fence();
      }
      bclob = true;
      // pass 1: A' = REDC(A_x A_t) (even), REDC(B_x A_t - m) + z (odd)
#pragma unroll
      for (int j = 0; j < S; ++j) P[j] = 0;
      d4_pass<S>(P, a, st, 0, m, mprime, odd, std::make_integer_sequence<int, S>{});
#pragma unroll
      for (int j = 0; j < S; ++j) P[j] += (uint64_t)(st[S + j] & oddmask);
      lane::normalize<S>(P, a);
    }
    if (op & LOP_STORE) d4r_tile_store<S>(tl, op >> 24, a, Q{});
    if (op & LOP_B_SET) {
      d4_fence();
#pragma unroll
      for (int j = 0; j < S; ++j) st[tig * S + j] = a[j];
      d4_fence();
      d4r_tile_store<S>(tl, D4R_KEPT, a, Q{});
      bclob = false;
    }
  }
}

// ---- k_dec4_pow: B-free window multipliers (round 4)
// A product by a pair (a, 0) is one pass on both lanes (U = REDC(A_x a) | REDC(B_x a - m)); by a general pair it is
// two. So the window table is factored, P_t = a_t (1 + p b_t) (a_t, H_t its components, b_t = H_t / a_t mod p), the
// chain multiplies by (a_t, 0) only, and the dropped factors are put back at the end, where they commute: squares
// double them, so they total 1 + p s, s = sum_t K_t b_t with K_t = sum over the chain's multiplies by entry t of
// 2^(squares after it), a constant of the key (the host's build_dec4f_program). b_t needs a_t^-1, and the chain
// provides it: it runs the exponent p - 2, whose result Y' is A~^-1 R^2 mod p (Fermat) -- iota. With the ciphertext
// pair c~ = A~ + p B_c = A~ (1 + p u) (the base is B-free: (A~, 0), u = B_c / A~):
//   P_t      = mm-powers of (A~, 0): 30 one-pass products, odd t stored in tiles 0..15 (tile 0 keeps B_c in the odd
//              lane's component)
//   Y'       = the chain over p - 2 (first load: the full pair P_first)
//   1 + p G  = mm(mm(Y', (A~, 0)), (1, 0))                             (Y' A~ == 1 mod p: c~^(p-1) in plain form)
//   delta    = s - u = REDC(acc iota), acc = sum_j c_j (w R^-1)^j by Horner, w = REDC(iota iota),
//              c_j = REDC(H_{2j+1} K'_{2j+1}) R^-1 (K'_t = K_t R), c_0 = -B_c R^-1 (K'_1 = -R: b_1 = 0)
//   output   = (A, G + delta): c^(p-1) mod p^2 = (1 + p G)(1 + p delta)   (tools/dec4f_model.py checks the algebra)
// Per 2048-bit p_h: 2043 squares + 341 one-pass products + 30 (table) + 2 + 34 (Horner) passes, against
// 2043 + 2 x 341 + 33 before. The Horner passes run in the odd lane (the even lane's copy is discarded); K'_t is
// staged per step through a block-wide LDS row, so the loop over steps is block-uniform.
constexpr int D4F_G = LANE_NTILE;         // spare tile: the pair (1 + p G)
constexpr int D4F_ACC = LANE_NTILE + 1;   // spare tile: the Horner accumulator
constexpr int D4F_HORNER = 2 * LANE_NTILE + 2;   // passes after the chain: w, 16 x (c_j, acc), delta
static_assert((LANE_NTILE + 2) * tile_quads<D4_S>() <= LANE_NTILE * tile_quads<D4_S>() + RBUF_WORDS / 4,
              "the two spare tiles fit the lane scratch");

// the even lane's component of tile k -> LDS row dst (the odd lane's copy is not needed: B-free multipliers)
template <int S, int... Gs>
__device__ __forceinline__ void d4f_mult_load(const LaneScratch& t, int k, uint32_t* dst, bool odd, std::integer_sequence<int, Gs...>) {
  constexpr int TQ = tile_quads<S>();
  d4_fence();
  if (!odd) {
    uint4 v[sizeof...(Gs)];
    ((v[Gs] = t.quad(k * TQ + Gs)), ...);
    (((4 * Gs < S ? (dst[4 * Gs] = v[Gs].x) : 0u), (4 * Gs + 1 < S ? (dst[4 * Gs + 1] = v[Gs].y) : 0u),
      (4 * Gs + 2 < S ? (dst[4 * Gs + 2] = v[Gs].z) : 0u), (4 * Gs + 3 < S ? (dst[4 * Gs + 3] = v[Gs].w) : 0u)),
     ...);
  }
  d4_fence();
}

// The public-key encryption's inputs to the factored chain (k_pe_pow_f, kernels_pe.hpp; PE = true below): the chain
// runs the exponent n over the B-free base (A_r, 0) -- x^n mod n^2 depends on x mod n only, so the base's B part is
// dropped outright -- iota = A_r^-1 R^2 mod n comes from a batch inversion instead of a Fermat chain (n's factors are
// not known), and the closing multiplies by c0 = 1 + n M: the output is (A_Z, B_Z + A_Z (delta + M)) mod n.
struct PefIn {
  const uint32_t* iota;    // [S][n] limbs of A_r^-1 R^2 mod n
  const uint32_t* r2n;     // R^2 mod n, S limbs (t R = REDC(t R^2))
  const uint32_t* nl;      // n, S limbs
  long long n, ee;         // elements, this element
  int64_t M;               // the encoding: c0 = 1 + n M
};

template <int S, bool PE = false>
__device__ __forceinline__ void d4f_run(uint32_t (&a)[S], uint32_t* st, uint32_t* kb, const LaneScratch& tl,
                                        const uint32_t* __restrict__ prog, int nprog, const uint32_t* __restrict__ kf,
                                        const uint32_t* x1, const uint32_t (&m)[S], uint32_t mprime, int tig,
                                        const PefIn& pe = PefIn{}) {
  constexpr int TQ = tile_quads<S>();
  using Q = std::make_integer_sequence<int, TQ>;
  const bool odd = tig != 0;
  if constexpr (PE) {   // (A_r, B_r) -> (A_r, 0): the base's B part does not change x^n mod n^2
#pragma unroll
    for (int j = 0; j < S; ++j) a[j] = odd ? 0u : a[j];
  }
  // the table's base (A~, 0), the multiplier A~ kept in the LDS A row by the table's products (LOP_B_READY)
  d4r_tile_store<S>(tl, 0, a, Q{});
  d4_fence();
  if (!odd) {
#pragma unroll
    for (int j = 0; j < S; ++j) st[j] = a[j];
    if constexpr (PE) {   // iota into the B row now (the chain's B-free multipliers use only the A row)
#pragma unroll
      for (int j = 0; j < S; ++j) st[S + j] = pe.iota[(size_t)j * pe.n + pe.ee];
    }
  }
#pragma unroll
  for (int j = 0; j < S; ++j) a[j] = odd ? 0u : a[j];
  d4_fence();
#pragma unroll 1
  for (int i = 0; i < nprog; ++i) {
    const uint32_t op = lane_op(prog, i);
    if (op & LOP_A_FROM_T) {
      const int k = (op >> 16) & 0xFF;
      d4r_tile_load<S>(tl, k, a, Q{});
      if (k == 0) {   // tile 0's odd component is B_c; the entry is (A~, 0)
#pragma unroll
        for (int j = 0; j < S; ++j) a[j] = odd ? 0u : a[j];
      }
    }
    if (op & LOP_IOTA) {   // iota = Y' mod p (any representative < 2p) -> the LDS B row
      d4_fence();
      if (!odd) {
#pragma unroll
        for (int j = 0; j < S; ++j) st[S + j] = a[j];
      }
      d4_fence();
    }
    uint64_t P[S];
    if (op & LOP_SQR) {
      if (op & LOP_PREFETCH) d4f_mult_load<S>(tl, (op >> 8) & 0xFF, st, odd, Q{});
#pragma unroll
      for (int j = 0; j < S; ++j) P[j] = odd ? (uint64_t)x1[j] : 0ull;
      d4r_sqr_pass<S>(P, a, tig, m, mprime, odd, std::make_integer_sequence<int, S>{});
    } else {
      if (op & LOP_B_CONST) {
        d4_fence();
        if (!odd) {
#pragma unroll
          for (int j = 0; j < S; ++j) st[j] = j == 0 ? 1u : 0u;
        }
        d4_fence();
      } else if (!(op & LOP_B_READY)) {
        d4f_mult_load<S>(tl, (op >> 8) & 0xFF, st, odd, Q{});
      }
      // (A_x + p B_x)(a, 0): U = REDC(A_x a) (even), REDC(B_x a - m) (odd)
#pragma unroll
      for (int j = 0; j < S; ++j) P[j] = 0;
      d4_pass<S>(P, a, st, 0, m, mprime, odd, std::make_integer_sequence<int, S>{});
    }
    lane::normalize<S>(P, a);
    if (op & LOP_STORE) d4r_tile_store<S>(tl, op >> 24, a, Q{});
  }
  // the closing Horner sum (odd lane; LDS: st = [w][iota], kb = K'_t); a holds (1 + p G), also in tile D4F_G
#pragma unroll 1
  for (int s = 0; s < D4F_HORNER; ++s) {
    const bool first = s == 0, last = s == D4F_HORNER - 1;
    const bool cj = !first && !last && (s & 1);   // c_j = REDC(H_t K'_t)
    const int j = LANE_NTILE - 1 - (s - 1) / 2;
    uint64_t P[S];
    const uint32_t* dig;
    if (cj) {
      __syncthreads();
      for (int i = threadIdx.x; i < S; i += blockDim.x) kb[i] = kf[j * S + i];
      __syncthreads();
      d4r_tile_load<S>(tl, j, a, Q{});
#pragma unroll
      for (int i = 0; i < S; ++i) P[i] = 0;
      dig = kb;
    } else if (first) {   // w = REDC(iota iota)
#pragma unroll
      for (int i = 0; i < S; ++i) a[i] = st[S + i];
#pragma unroll
      for (int i = 0; i < S; ++i) P[i] = 0;
      dig = st + S;
    } else if (!last) {   // acc = REDC(c_j + acc w)
#pragma unroll
      for (int i = 0; i < S; ++i) P[i] = a[i];
      if (j == LANE_NTILE - 1) {
#pragma unroll
        for (int i = 0; i < S; ++i) a[i] = 0;
      } else {
        d4r_tile_load<S>(tl, D4F_ACC, a, Q{});
      }
      dig = st;
    } else {              // delta = REDC(acc iota)
      d4r_tile_load<S>(tl, D4F_ACC, a, Q{});
#pragma unroll
      for (int i = 0; i < S; ++i) P[i] = 0;
      dig = st + S;
    }
    d4_pass<S>(P, a, dig, 0, m, mprime, false, std::make_integer_sequence<int, S>{});
    lane::normalize<S>(P, a);
    if (first) {
      d4_fence();
      if (!odd) {
#pragma unroll
        for (int i = 0; i < S; ++i) st[i] = a[i];
      }
      d4_fence();
    } else if (!last && !cj) {
      d4r_tile_store<S>(tl, D4F_ACC, a, Q{});
    }
  }
  if constexpr (!PE) {   // output (A, G + delta): G < 2p, delta < 2p
    uint32_t g[S];
    d4r_tile_load<S>(tl, D4F_G, g, Q{});
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < S; ++i) {
      const uint32_t v = g[i] + (odd ? a[i] : 0u) + c;
      a[i] = v & lane::LMASK;
      c = v >> lane::LB;
    }
  } else {   // (A_Z, B_Z + A_Z t), t = delta + M mod n: u = REDC(t R^2) = t R over R^2's digits (kb), then REDC(u A_Z)
    {
      const int64_t M = pe.M;
      const bool neg = M < 0;
      const uint64_t mag = neg ? (uint64_t)0 - (uint64_t)M : (uint64_t)M;
      int64_t c = 0;
#pragma unroll
      for (int j = 0; j < S; ++j) {   // a (the odd lane's delta < 2n) + M, or + n - |M|: < 3n
        const uint32_t mj = j < 3 ? (uint32_t)(mag >> (lane::LB * j)) & lane::LMASK : 0u;
        const int64_t v = (int64_t)a[j] + (neg ? (int64_t)pe.nl[j] - (int64_t)mj : (int64_t)mj) + c;
        a[j] = (uint32_t)v & lane::LMASK;
        c = v >> lane::LB;
      }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < S; i += blockDim.x) kb[i] = pe.r2n[i];
    __syncthreads();
    uint64_t P[S];
#pragma unroll
    for (int i = 0; i < S; ++i) P[i] = 0;
    d4_pass<S>(P, a, kb, 0, m, mprime, false, std::make_integer_sequence<int, S>{});
    lane::normalize<S>(P, a);            // u = t R (< 2n)
    uint32_t g[S];
    d4r_tile_load<S>(tl, D4F_G, g, Q{});   // (A_Z, B_Z)
    d4_fence();
    if (!odd) {
#pragma unroll
      for (int i = 0; i < S; ++i) st[i] = g[i];   // A_Z's digits for the odd lane's last pass
    }
    d4_fence();
#pragma unroll
    for (int i = 0; i < S; ++i) P[i] = 0;
    d4_pass<S>(P, a, st, 0, m, mprime, false, std::make_integer_sequence<int, S>{});
    lane::normalize<S>(P, a);            // t A_Z (< 2n)
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < S; ++i) {         // even: A_Z; odd: B_Z + t A_Z (< 4n)
      const uint32_t v = g[i] + (odd ? a[i] : 0u) + c;
      a[i] = v & lane::LMASK;
      c = v >> lane::LB;
    }
  }
}

template <int S>
#ifndef FPAI_DEC4_OCC
#define FPAI_DEC4_OCC 2   // waves per SIMD (measurement builds: tools/gpu/ab_dec4_occ_run.sh)
#endif
__global__ __launch_bounds__(LANE_BLOCK, FPAI_DEC4_OCC) void k_dec4_pow(Dec4Params p) {
  constexpr int TQ = tile_quads<S>();
  using Q = std::make_integer_sequence<int, TQ>;
  __shared__ uint32_t lds[D4_PAIRS * D4R_SLOT + 2 * S];
  const int half = blockIdx.y;
  const Dec4Half* H = p.halves + half;
  uint32_t m[S];
#pragma unroll
  for (int j = 0; j < S; ++j) m[j] = H->p[j];
  const uint32_t mprime = H->mprime;
  const int nprog = H->nprog;
  const uint32_t* prog = H->prog;
  const uint32_t* kf = H->kf;
  uint32_t* x1 = lds + D4_PAIRS * D4R_SLOT;   // (1 - R) mod p_h: the odd row's start in squares (LDS: no SGPRs)
  uint32_t* kb = x1 + S;                       // K'_t of the current Horner step (block-wide)
  for (int i = threadIdx.x; i < S; i += blockDim.x) x1[i] = H->X1[i];
  __syncthreads();
  const int tig = threadIdx.x & 1;
  const int pib = threadIdx.x >> 1;
  uint32_t* st = lds + pib * D4R_SLOT;
  const LaneScratch tl = lane_scratch(p.scratch);
  for (long long base = (long long)blockIdx.x * D4_PAIRS; base < p.n; base += (long long)gridDim.x * D4_PAIRS) {
    const long long e = base + pib;
    const bool valid = e < p.n;
    const long long ee = valid ? e : p.n - 1;
    uint32_t a[S];
#pragma unroll
    for (int i = 0; i < S; ++i) a[i] = p.x[((size_t)half * 2 * S + tig * S + i) * p.n + ee];
    d4f_run<S>(a, st, kb, tl, prog, nprog, kf, x1, m, mprime, tig);
    if (valid) {
#pragma unroll
      for (int i = 0; i < S; ++i) p.x[((size_t)half * 2 * S + tig * S + i) * p.n + e] = a[i];
    }
  }
}

// ---------------------------------------------------------------- m_h = L_h h_h mod p_h
// one lane per element-half: the canonical pair of x_h (A < 2p, B < 4p on entry) gives L_h = B (A = 1), or
// B - 1 (A = 0: c == 0 mod p_h, the reference's floor division); then REDC(L_h h_h R) with h_h R's digits
// broadcast from LDS.
template <int S>
__global__ __launch_bounds__(LANE_BLOCK) void k_dec4_L(Dec4Params p) {
  __shared__ uint32_t hr[S];
  const int half = blockIdx.y;
  const Dec4Half* H = p.halves + half;
  for (int i = threadIdx.x; i < S; i += blockDim.x) hr[i] = H->hR[i];
  __syncthreads();
  uint32_t m[S];
#pragma unroll
  for (int j = 0; j < S; ++j) m[j] = H->p[j];
  for (long long e = (long long)blockIdx.x * LANE_BLOCK + threadIdx.x; e < p.n; e += (long long)gridDim.x * LANE_BLOCK) {
    uint32_t a[S], b[S], d[S];
#pragma unroll
    for (int i = 0; i < S; ++i) {
      a[i] = p.x[((size_t)half * 2 * S + i) * p.n + e];
      b[i] = p.x[((size_t)half * 2 * S + S + i) * p.n + e];
    }
    const bool lt = lane::sub<S>(a, m, d);
    uint32_t c = lt ? 0u : 1u;
#pragma unroll
    for (int i = 0; i < S; ++i) {
      a[i] = lt ? a[i] : d[i];
      const uint32_t v = b[i] + c;
      b[i] = v & lane::LMASK;
      c = v >> lane::LB;
    }
#pragma unroll 1
    for (int r = 0; r < 4; ++r) lane::cond_sub<S>(b, m);
    uint32_t nz = 0;
#pragma unroll
    for (int i = 0; i < S; ++i) nz |= a[i];
    if (nz == 0) {
      uint32_t one[S];
#pragma unroll
      for (int i = 0; i < S; ++i) one[i] = i == 0 ? 1u : 0u;
      const bool neg = lane::sub<S>(b, one, d);
#pragma unroll
      for (int i = 0; i < S; ++i) b[i] = neg ? m[i] - (i == 0 ? 1u : 0u) : d[i];
    }
    uint64_t P[S];
#pragma unroll
    for (int i = 0; i < S; ++i) P[i] = 0;
    d4_pass<S>(P, b, hr, 0, m, H->mprime, false, std::make_integer_sequence<int, S>{});
    lane::normalize<S>(P, b);
    lane::cond_sub<S>(b, m);
#pragma unroll
    for (int i = 0; i < S; ++i) p.mh[((size_t)half * S + i) * p.n + e] = b[i];
  }
}

// CRT + decode from m_p, m_q ([2][74][n]) on a lane group of TPI = 4 (S = 148), k_decrypt's steps 8-9
template <int TPI>
__global__ __launch_bounds__(BLOCK) void k_dec4_fin(DecParams p, const uint32_t* __restrict__ mh) {
  constexpr int S = TPI * L;
  constexpr int GPB = BLOCK / TPI;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int lane = threadIdx.x & 63;
  const int tig = threadIdx.x % TPI;
  const int gib = threadIdx.x / TPI;
  uint32_t* eslot = smem + gib * S;
  const DecHalf* H0 = p.halves;
  for (long long base = (long long)blockIdx.x * GPB; base < p.n; base += (long long)gridDim.x * GPB) {
    const long long inst = base + gib;
    const bool valid = inst < p.n;
    const long long ii = valid ? inst : p.n - 1;
    uint32_t mp[L], mq[L];
    {
      int t = tig;
      asm volatile("" : "+v"(t));
#pragma unroll
      for (int i = 0; i < L; ++i) {
        const int limb = t * L + i;
        mp[i] = limb < D4_S ? mh[(size_t)limb * p.n + ii] : 0u;
        mq[i] = limb < D4_S ? mh[((size_t)D4_S + limb) * p.n + ii] : 0u;
      }
    }
    uint32_t p0[L], a1[L], a2[L], u[L];
    load_limbs_g<TPI>(H0->ph, p0, tig);
    copy_g_to_lds<TPI>(eslot, p.qinvR, tig);
    montmul<TPI>(a1, mp, eslot, TPI, p0, H0->pprime, lane, tig);
    cond_sub<TPI>(a1, p0, lane, tig);
    montmul<TPI>(a2, mq, eslot, TPI, p0, H0->pprime, lane, tig);
    cond_sub<TPI>(a2, p0, lane, tig);
    {
      const bool neg = sub_limbs<TPI>(a1, a2, u, lane, tig);
      uint64_t P[L];
#pragma unroll
      for (int i = 0; i < L; ++i) P[i] = (uint64_t)u[i] + (neg ? p0[i] : 0u);
      normalize<TPI>(P, u, lane, tig);
    }
    uint32_t nlm[L], uq[L], x[L];
    load_limbs_g<TPI>(p.nlimb, nlm, tig);
    copy_g_to_lds<TPI>(eslot, p.qRn, tig);
    montmul<TPI>(uq, u, eslot, TPI, nlm, p.nprime, lane, tig);
    cond_sub<TPI>(uq, nlm, lane, tig);
    {
      uint64_t P[L];
#pragma unroll
      for (int i = 0; i < L; ++i) P[i] = (uint64_t)uq[i] + mq[i];
      normalize<TPI>(P, x, lane, tig);
    }
    write_limbs_lds<TPI>(eslot, x, tig);
    if (valid && p.raw) {
      for (int j = tig; j < p.pt_words; j += TPI) p.raw[ii * p.pt_words + j] = limbs_word(eslot, S, j);
    }
    if (valid && tig == 0) decode_element(eslot, p, ii);
    wave_lds_fence();
  }
}

}  // namespace fpai
