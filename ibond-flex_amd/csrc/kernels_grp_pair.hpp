// Fixed-base sampler for 4096-bit keys on pair groups (bn_pgroup.hpp: TPI = 4 lanes x LL = 19 limbs, S = 76
// limbs of p_h): kernels_grp.hpp's k_fbg with every product mod p_h^2 a pair product, 5 S^2 = 28.9 k lane-MACs
// against k_fbg's 2 (148)^2 = 43.8 k. Same distribution and ciphertext bits.
//
//   k_fbgp       w_h = c0 G_h^(a_h) mod p_h^2 as the canonical pair (A, B) (c0 = the pair (1, (n/p_h) M))
//   k_fbgp_w     w_h = A + p_h B mod p_h^2 (one product mod p_h^2 on the L = 37 group engine, in place), so
//                k_fbg_garner and k_fbg_fin recombine exactly as after k_fbg
//   k_fbgp_lohi / k_fbgp_fill   the per-key tables: rows of the canonical pair of T_k[d] R mod p_h^2 as the
//                32-bit words of A then of B (512 B, below)
#pragma once
#include "bn_pgroup.hpp"
#include "kernels_grp.hpp"

namespace fpai {

constexpr int FBGP_TPI = 4, FBGP_LL = 19, FBGP_S = FBGP_TPI * FBGP_LL;   // 76 limbs >= the 74 of a 2048-bit p_h
constexpr int FBGP_SP = 74;                                               // limbs of A and of B that can be non-zero
constexpr int FBGP_PW = 64;                 // 32-bit words of A and of B in a table row (a canonical pair: A, B < 2^2048)
constexpr int FBGP_ROW4 = 2 * FBGP_PW / 4;  // uint4 per row: 512 B, four aligned 128-B lines

struct FbgpHalf {
  const uint32_t* table;   // [K][2^W] rows of FBGP_ROW4 uint4: canonical pair of T_k[d] R mod p_h^2 (words)
  const uint32_t* p;       // p_h, S limbs
  const uint32_t* X;       // (1 - R) mod p_h, S limbs (R = 2^(28 S))
  const uint32_t* oneR;    // pair of R mod p_h^2 ([A: S][B: S])
  const uint32_t* bases;   // [K][2][2S] pairs of B_k R and B_k^(2^LO) R mod p_h^2
  uint32_t* lohi;          // [K][2][FB_LO][2S] scratch
  const uint32_t* nm;      // [4][S] (n / p_h) 2^(16 c) mod p_h
  const uint32_t* pbig;    // [S] 2^20 p_h
  const uint32_t* p2;      // p_h^2, 148 limbs (k_fbgp_w)
  const uint32_t* pR2;     // p_h R' mod p_h^2, R' = 2^(28 148), 148 limbs (k_fbgp_w)
  uint32_t mprime;         // -p_h^-1 mod 2^28
  uint32_t mprime2;        // -p_h^-2 mod 2^28
  // factored rows (below): inverses of the lo/hi entries' A parts, and the construction scratch
  uint32_t* inv;           // [K][2][FB_LO][S]: (A of lo/hi entry)^-1 R mod p_h
  uint32_t* pre;           // [2K][2^HI][S] prefix products of the batch inversion (scratch)
  uint32_t* cval;          // [2K][S]: each chain's product (k_pair_inv_fwd), then its inverse R^2 (host)
};

struct FbgpParams {
  const FbgpHalf* halves;  // [2]
  long long n;
  int K, W;
  const uint32_t* digits;  // [2][K][n]
  uint32_t* out;           // [2][148][n]: the pair [A: 74][B: 74], then w_h in place (k_fbgp_w)
  const void* x;
  int dtype, exp_mode, fexp;
  int32_t* exp;
  int32_t* status;
};

template <int TPI, int LL>
__device__ __forceinline__ void fbgp_load(const uint32_t* __restrict__ g, uint32_t (&x)[LL], int tig) {
#pragma unroll
  for (int i = 0; i < LL; ++i) x[i] = g[tig * LL + i];
}
// a pair ([A: stride][B: stride], the first SP limbs of each) -> the group's slot [A: S][B: S]
template <int TPI, int LL>
__device__ __forceinline__ void fbgp_pair_to_slot(uint32_t* slot, const uint32_t* __restrict__ g, int stride, int tig) {
  constexpr int S = TPI * LL;
  int t = tig;
  asm volatile("" : "+v"(t));
  uint32_t a[LL], b[LL];
#pragma unroll
  for (int i = 0; i < LL; ++i) {
    const int idx = t * LL + i;
    a[i] = idx < FBGP_SP ? g[idx] : 0u;
    b[i] = idx < FBGP_SP ? g[stride + idx] : 0u;
  }
  wave_lds_fence();
#pragma unroll
  for (int i = 0; i < LL; ++i) {
    slot[t * LL + i] = a[i];
    slot[S + t * LL + i] = b[i];
  }
  wave_lds_fence();
}
template <int TPI, int LL>
__device__ __forceinline__ void pfb_store_limbs(uint32_t* dst, const uint32_t (&x)[LL], int tig) {
#pragma unroll
  for (int i = 0; i < LL; ++i) dst[tig * LL + i] = x[i];
}
template <int TPI, int LL>
__device__ __forceinline__ void fbgp_regs_to_slot(uint32_t* slot, const uint32_t (&A)[LL], const uint32_t (&B)[LL], int tig) {
  constexpr int S = TPI * LL;
  wave_lds_fence();
#pragma unroll
  for (int i = 0; i < LL; ++i) {
    slot[tig * LL + i] = A[i];
    slot[S + tig * LL + i] = B[i];
  }
  wave_lds_fence();
}

// ---------------------------------------------------------------- table rows as 32-bit words
// A row is the canonical pair (A, B) of T_k[d] R as the 32-bit words of A then of B (512 B). The limb-row layout
// of the first version (74 + 74 28-bit limbs, 592 B) straddled 128-B lines and read 1.21x its bytes from HBM.

// canonical pair (registers) -> the group's slot -> lane t stores words [32 t, 32 t + 32) of the row (16-byte
// stores). Word w of a component = limbs i, i + 1 (i = 32 w / 28, shift 32 w mod 28 = 4 w mod 28 <= 24). row
// may be null (the group only takes part in the slot traffic).
template <int TPI, int LL>
__device__ __forceinline__ void pair_store_row(uint4* row, uint32_t* slot, const uint32_t (&A)[LL], const uint32_t (&B)[LL],
                                               int tig) {
  constexpr int S = TPI * LL;
  static_assert(TPI * 32 == 2 * FBGP_PW, "one lane per 32 row words");
  fbgp_regs_to_slot<TPI, LL>(slot, A, B, tig);
  uint32_t wv[32];
#pragma unroll
  for (int q = 0; q < 32; ++q) {
    const int w = tig * 32 + q;
    const int comp = w / FBGP_PW, ww = w % FBGP_PW;
    const int i = (32 * ww) / LB, o = (32 * ww) % LB;
    const uint32_t* cs = slot + comp * S;
    wv[q] = (cs[i] >> o) | (cs[i + 1] << (LB - o));
  }
  if (row) {
    row += tig * 8;
#pragma unroll
    for (int q = 0; q < 8; ++q) row[q] = make_uint4(wv[4 * q], wv[4 * q + 1], wv[4 * q + 2], wv[4 * q + 3]);
  }
  wave_lds_fence();
}

// ---- rows stream HBM -> LDS by DMA, one product ahead, without registers
// A wave holds 16 groups; one global_load_lds writes 16 B per lane at M0 + 16 lane, i.e. 1 KB: lanes 0-31 fetch
// the 512-B row of group 2q, lanes 32-63 that of group 2q + 1, so eight instructions land the wave's 16 rows
// contiguously (group g's row at wave_stage + 512 g). The row index of a group comes from its lane 0 by
// readlane. The staging array is its own __shared__ object: the compiler then does not order the product's
// slot reads behind the DMA in flight (they cannot alias), so the row of product k+1 streams in during k.
constexpr int FBGP_STAGE_WORDS = 16 * 2 * FBGP_PW + 4;   // per wave (+4: the conversion's last read past a row)

__device__ __forceinline__ void pair_rows_dma(const uint4* __restrict__ table, size_t k, int W, uint32_t d,
                                              const uint32_t* wave_stage, int lane) {
  typedef __attribute__((address_space(3))) uint32_t lds_u32;
  const uint32_t lb = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(lds_u32*)wave_stage);
  const size_t kb = k << W;
  const int hi = lane >> 5, col = lane & 31;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const uint32_t d0 = __builtin_amdgcn_readlane(d, 8 * q), d1 = __builtin_amdgcn_readlane(d, 8 * q + 4);
    const uint4* src = table + (kb + (hi ? d1 : d0)) * FBGP_ROW4 + col;
    uint32_t dst = lb + (uint32_t)(q * 1024);
    asm volatile("" : "+s"(dst));
    __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(size_t)dst, 16, 0, 0);
  }
}

// The group's staged row (contiguous words) -> limbs in the slot [A: S][B: S]. Lane t owns limbs [LL t, LL t + LL)
// of each component, i.e. bits from 28 LL t: it reads the 18 words from word (28 LL t) / 32, shifts them down by
// (28 LL t) mod 32 (one funnel shift per word, the lane's own amount) and cuts 28-bit limbs at compile-time
// offsets. Limbs >= FBGP_SP are zero.
template <int TPI, int LL, int NCOMP = 2, int CW = FBGP_PW>
__device__ __forceinline__ void pair_stage_to_slot(uint32_t* slot, const uint32_t* row, int tig) {
  constexpr int S = TPI * LL;
  constexpr int NW = (LB * LL + 31) / 32 + 1;   // 18 words cover a lane's 19 limbs at any bit offset
  static_assert(LL == 19 && NW == 18, "geometry");
  const uint32_t bit0 = (uint32_t)(LB * LL) * (uint32_t)tig;
  const uint32_t w0 = bit0 >> 5, sh = bit0 & 31u;
#pragma unroll
  for (int comp = 0; comp < NCOMP; ++comp) {
    const uint32_t* src = row + comp * FBGP_PW + w0;
    uint32_t v[NW];
#pragma unroll
    for (int k = 0; k < NW; ++k) v[k] = src[k];
    uint32_t u[NW - 1];
#pragma unroll
    for (int k = 0; k + 1 < NW; ++k) u[k] = __builtin_amdgcn_alignbit(v[k + 1], v[k], sh);
    uint32_t* dst = slot + comp * S + tig * LL;
#pragma unroll
    for (int r = 0; r < LL; ++r) {
      const int b = LB * r, w = b >> 5, o = b & 31;
      const uint32_t lo = u[w], hi = (w + 1 < NW - 1) ? u[w + 1] : 0u;
      uint32_t limb = __builtin_amdgcn_alignbit(hi, lo, (uint32_t)o) & LMASK;
      if (r + (TPI - 1) * LL >= 32 * CW / LB) {
        // limbs at or past bit 32 CW of the component: keep only its own bits (the words read past the component
        // are the other component's, or the next row's)
        const int lim = 32 * CW - LB * (tig * LL + r);
        limb = lim >= LB ? limb : lim > 0 ? (limb & ((1u << lim) - 1u)) : 0u;
      }
      dst[r] = limb;
    }
  }
}

// ---- factored rows
// A table entry T' = T R mod p^2 is stored as T' = a (1 + p b) with a = T' mod p and b = (T' div p) a^-1 mod p
// (rows: the words of a, then of b R mod p). The product of the K entries an element selects is then
//   prod_k T'_k = (prod_k a_k) (1 + p sum_k b_k)   (mod p^2)
// so the loop multiplies by the pairs (a_k, 0) -- the B row loses its A B2 term: 4 S^2 lane-MACs instead of
// 5 S^2 -- while each lane adds its quarter of the b R words into a running sum (16 words + a carry count),
// and one correction at the end applies the factor: (A + p B)(1 + p bs) = A + p (B + A bs) (mod p^2),
// B += REDC(A (bs R)). Same value, same ciphertext bits.

// the bR words of the group's staged row (words PW .. 2 PW) into this lane's quarter of the running sum, which
// lives in the slot's B half (the B2 = 0 products never read it): 16 words at slot + S + 16 t, the carry count
// at slot + S + PW + t
template <int TPI, int LL>
__device__ __forceinline__ void pair_bsum_add(uint32_t* slot, const uint32_t* row, int tig) {
  constexpr int S = TPI * LL, NB = FBGP_PW / TPI;
  const uint4* src = reinterpret_cast<const uint4*>(row + FBGP_PW) + tig * (NB / 4);
  uint4* acc = reinterpret_cast<uint4*>(slot + S) + tig * (NB / 4);
  uint32_t w[NB], a[NB];
#pragma unroll
  for (int q = 0; q < NB / 4; ++q) {
    const uint4 v = src[q], u = acc[q];
    w[4 * q] = v.x, w[4 * q + 1] = v.y, w[4 * q + 2] = v.z, w[4 * q + 3] = v.w;
    a[4 * q] = u.x, a[4 * q + 1] = u.y, a[4 * q + 2] = u.z, a[4 * q + 3] = u.w;
  }
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const uint64_t v = (uint64_t)a[i] + w[i] + c;
    a[i] = (uint32_t)v;
    c = v >> 32;
  }
#pragma unroll
  for (int q = 0; q < NB / 4; ++q) acc[q] = make_uint4(a[4 * q], a[4 * q + 1], a[4 * q + 2], a[4 * q + 3]);
  slot[S + FBGP_PW + tig] += (uint32_t)c;
}

// (A, B) <- (A, B) prod_k T_k[dg[k stride]] over K factored word rows of 2^W entries; row k+1 streams in by DMA
// during product k. wave_stage: this wave's FBGP_STAGE_WORDS words (its own __shared__ object). Leaves the
// running b sum in the slot's B half for pair_apply_bsum.
template <int TPI, int LL>
__device__ __forceinline__ void pair_table_products(uint32_t (&A)[LL], uint32_t (&B)[LL], const uint4* __restrict__ table,
                                                    const uint32_t* __restrict__ dg, long long stride, int K, int W,
                                                    uint32_t* slot, const uint32_t* wave_stage, const uint32_t* xs,
                                                    const uint32_t (&m)[LL], uint32_t mprime, int lane, int tig) {
  constexpr int S = TPI * LL;
  const uint32_t* row = wave_stage + (lane / TPI) * 2 * FBGP_PW;
  wave_lds_fence();
  for (int i = tig; i < FBGP_PW + TPI; i += TPI) slot[S + i] = 0u;   // the b sum and its carry counts
  pair_rows_dma(table, 0, W, dg[0], wave_stage, lane);
  uint32_t dn = K > 1 ? dg[(size_t)stride] : 0u;
  for (int k = 0; k < K; ++k) {
    lds_dma_wait();                                   // row k landed, digit k+1 loaded
    wave_lds_fence();
    pair_stage_to_slot<TPI, LL, 1>(slot, row, tig);   // a (the B half of the slot is not read)
    pair_bsum_add<TPI, LL>(slot, row, tig);
    wave_lds_fence();
    if (k + 1 < K) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the staged row is consumed before it is overwritten
      pair_rows_dma(table, (size_t)(k + 1), W, dn, wave_stage, lane);
      dn = k + 2 < K ? dg[(size_t)(k + 2) * stride] : 0u;
    }
    pgrp::montmul<TPI, LL, false, true>(A, B, slot, xs, m, mprime, lane, tig);
  }
}

// B += REDC(A bsR) with bsR = sum_k b_k R (the lanes' words plus their carries, < 2^(32 PW + 7)): then
// A + p B == (A + p B)(1 + p sum b_k) (mod p^2). Uses the group's staging row and slot. B < 4p on exit.
template <int TPI, int LL>
__device__ __forceinline__ void pair_apply_bsum(uint32_t (&A)[LL], uint32_t (&B)[LL], uint32_t* slot, uint32_t* row,
                                                const uint32_t (&m)[LL], uint32_t mprime, int lane, int tig) {
  constexpr int S = TPI * LL, NB = FBGP_PW / TPI;
  constexpr int CW = FBGP_PW + 4;   // the sum's words (carries above word PW)
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  wave_lds_fence();
  for (int i = tig; i < FBGP_PW; i += TPI) row[i] = slot[S + i];
  for (int i = FBGP_PW + tig; i < CW + 2; i += TPI) row[i] = 0u;
  wave_lds_fence();
  // carry count of lane t enters at word NB (t + 1): applied one lane at a time (a few words ripple at most)
  for (int t = 0; t < TPI; ++t) {
    if (tig == t) {
      uint64_t c = slot[S + FBGP_PW + t];
      for (int w = NB * (t + 1); c != 0 && w < CW; ++w) {
        const uint64_t v = (uint64_t)row[w] + c;
        row[w] = (uint32_t)v;
        c = v >> 32;
      }
    }
    wave_lds_fence();
  }
  pair_stage_to_slot<TPI, LL, 1, CW>(slot, row, tig);
  wave_lds_fence();
  uint32_t U[LL];
#pragma unroll
  for (int i = 0; i < LL; ++i) U[i] = A[i];
  pgrp::montmul1<TPI, LL>(U, slot, m, mprime, lane, tig);   // A bs mod p, < 2p
  uint64_t P[LL];
#pragma unroll
  for (int i = 0; i < LL; ++i) P[i] = (uint64_t)B[i] + U[i];
  pgrp::normalize<TPI, LL>(P, B, lane, tig);
}

template <int TPI, int LL>
__global__ __launch_bounds__(BLOCK, 2) void k_fbgp(FbgpParams p) {
  constexpr int S = TPI * LL;
  constexpr int GPB = BLOCK / TPI;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int lane = threadIdx.x & 63;
  const int tig = threadIdx.x % TPI;
  const int gib = threadIdx.x / TPI;
  const int half = blockIdx.y;
  const FbgpHalf* H = p.halves + half;
  __shared__ __attribute__((aligned(16))) uint32_t stage[(BLOCK / 64) * FBGP_STAGE_WORDS];
  uint32_t* slot = smem + gib * 2 * S;
  const uint32_t* wstage = stage + (threadIdx.x / 64) * FBGP_STAGE_WORDS;
  uint32_t* xs = smem + GPB * 2 * S;
  for (int i = threadIdx.x; i < S; i += BLOCK) xs[i] = H->X[i];
  __syncthreads();
  uint32_t m[LL];
  fbgp_load<TPI, LL>(H->p, m, tig);
  const uint32_t mprime = H->mprime;
  const int K = p.K, W = p.W;
  const uint4* table = reinterpret_cast<const uint4*>(H->table);
  for (long long base = (long long)blockIdx.x * GPB; base < p.n; base += (long long)gridDim.x * GPB) {
    const long long inst = base + gib;
    const bool valid = inst < p.n;
    const long long ii = valid ? inst : p.n - 1;
    const uint32_t* dg = p.digits + (size_t)half * K * p.n + ii;
    int64_t M = 0;
    int e = 0, st;
    const bool fixed = p.exp_mode != 0;
    if (p.dtype == 0) st = encode_float((double)((const float*)p.x)[ii], fixed, p.fexp, M, e);
    else if (p.dtype == 1) st = encode_float(((const double*)p.x)[ii], fixed, p.fexp, M, e);
    else st = encode_int(((const int64_t*)p.x)[ii], fixed, p.fexp, M, e);
    if (half == 0 && valid && tig == 0) {
      p.exp[ii] = e;
      if (p.status) p.status[ii] = st;
    }
    // c0 = the pair (1, (n / p_h) M mod p_h): the sum over the 16-bit chunks of |M| (< 2^18 p_h; negative M:
    // 2^20 p_h - sum), a valid operand (R >= 2^24 p_h)
    uint32_t A[LL], B[LL];
    {
      const bool neg = M < 0;
      const uint64_t mag = neg ? (uint64_t)0 - (uint64_t)M : (uint64_t)M;
      int t = tig;
      asm volatile("" : "+v"(t));
      uint64_t P[LL];
#pragma unroll
      for (int i = 0; i < LL; ++i) {
        uint64_t v = 0;
#pragma unroll
        for (int c = 0; c < 4; ++c) v += (uint64_t)H->nm[c * S + t * LL + i] * ((uint32_t)(mag >> (16 * c)) & 0xFFFFu);
        P[i] = v;
      }
      uint32_t Xs[LL], Pb[LL], D[LL];
      pgrp::normalize<TPI, LL>(P, Xs, lane, tig);
      fbgp_load<TPI, LL>(H->pbig, Pb, tig);
      (void)pgrp::sub_limbs<TPI, LL>(Pb, Xs, D, lane, tig);
#pragma unroll
      for (int i = 0; i < LL; ++i) {
        B[i] = neg ? D[i] : Xs[i];
        A[i] = (tig == 0 && i == 0) ? 1u : 0u;
      }
    }
    pair_table_products<TPI, LL>(A, B, table, dg, p.n, K, W, slot, wstage, xs, m, mprime, lane, tig);
    pair_apply_bsum<TPI, LL>(A, B, slot, const_cast<uint32_t*>(wstage) + (lane / TPI) * 2 * FBGP_PW, m, mprime, lane, tig);
    pgrp::cond_sub<TPI, LL>(B, m, lane, tig);   // B < 4p -> < 2p: canon takes B + 1 <= 2p
    pgrp::cond_sub<TPI, LL>(B, m, lane, tig);
    pgrp::canon<TPI, LL>(A, B, m, lane, tig);
    if (valid) {
#pragma unroll
      for (int i = 0; i < LL; ++i) {
        const int idx = tig * LL + i;
        if (idx < FBGP_SP) {
          p.out[((size_t)half * 2 * FBGP_SP + idx) * p.n + ii] = A[i];
          p.out[((size_t)half * 2 * FBGP_SP + FBGP_SP + idx) * p.n + ii] = B[i];
        }
      }
    }
  }
}

// w_h = A + (B (p_h R') R'^-1 mod p_h^2) (< p_h^2 after two conditional subtractions), in place
template <int TPI>
__global__ __launch_bounds__(BLOCK) void k_fbgp_w(FbgpParams p) {
  constexpr int S = TPI * L;
  constexpr int GPB = BLOCK / TPI;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int lane = threadIdx.x & 63;
  const int tig = threadIdx.x % TPI;
  const int gib = threadIdx.x / TPI;
  const int half = blockIdx.y;
  const FbgpHalf* H = p.halves + half;
  uint32_t* slot = smem + gib * S;
  uint32_t m[L];
  load_limbs_g<TPI>(H->p2, m, tig);
  for (long long base = (long long)blockIdx.x * GPB; base < p.n; base += (long long)gridDim.x * GPB) {
    const long long inst = base + gib;
    const bool valid = inst < p.n;
    const long long ii = valid ? inst : p.n - 1;
    uint32_t a[L], b[L], t[L];
    {
      int tt = tig;
      asm volatile("" : "+v"(tt));
#pragma unroll
      for (int i = 0; i < L; ++i) {
        const int idx = tt * L + i;
        a[i] = idx < FBGP_SP ? p.out[((size_t)half * 2 * FBGP_SP + idx) * p.n + ii] : 0u;
        b[i] = idx < FBGP_SP ? p.out[((size_t)half * 2 * FBGP_SP + FBGP_SP + idx) * p.n + ii] : 0u;
      }
    }
    copy_g_to_lds<TPI>(slot, H->pR2, tig);
    montmul<TPI>(t, b, slot, TPI, m, H->mprime2, lane, tig);   // p_h B mod p_h^2 (< 2 p_h^2)
    uint64_t P[L];
#pragma unroll
    for (int i = 0; i < L; ++i) P[i] = (uint64_t)t[i] + a[i];
    normalize<TPI>(P, t, lane, tig);
    cond_sub<TPI>(t, m, lane, tig);
    cond_sub<TPI>(t, m, lane, tig);
    if (valid) {
#pragma unroll
      for (int i = 0; i < L; ++i) p.out[((size_t)half * S + tig * L + i) * p.n + ii] = t[i];
    }
  }
}

// ---- construction of factored rows
// lo[j], hi[j] represent L_j R, H_j R mod p^2 (their A parts: A_j == L_j R mod p); the fill's pair product gives
// the canonical (A, B) of T' = L H R, A == L H R (mod p). The factored row needs b R = B A^-1 R = B (L H)^-1 mod p.
// With inv_x = L_x^-1 R (k_pair_inv, R-forms): X = mont(inv_lo, inv_hi) = (L H)^-1 R, and mont(B, X) = B (L H)^-1.
template <int TPI, int LL>
__device__ __forceinline__ void pair_factor_row(uint32_t (&B)[LL], const FbgpHalf* H, int k, int d, int W, uint32_t* slot,
                                                const uint32_t (&m)[LL], int lane, int tig) {
  constexpr int S = TPI * LL;
  const int LO = W / 2;
  const uint32_t* il = H->inv + (((size_t)k * 2 + 0) * FB_LO + (d & ((1 << LO) - 1))) * S;
  const uint32_t* ih = H->inv + (((size_t)k * 2 + 1) * FB_LO + (d >> LO)) * S;
  uint32_t X[LL], Y[LL];
  fbgp_load<TPI, LL>(il, X, tig);
  fbgp_load<TPI, LL>(ih, Y, tig);
  wave_lds_fence();
#pragma unroll
  for (int i = 0; i < LL; ++i) slot[tig * LL + i] = Y[i];
  wave_lds_fence();
  pgrp::montmul1<TPI, LL>(X, slot, m, H->mprime, lane, tig);   // X = (L H)^-1 R
  wave_lds_fence();
#pragma unroll
  for (int i = 0; i < LL; ++i) slot[tig * LL + i] = X[i];
  wave_lds_fence();
  pgrp::montmul1<TPI, LL>(B, slot, m, H->mprime, lane, tig);   // b R = B (L H)^-1
  pgrp::cond_sub<TPI, LL>(B, m, lane, tig);
}

// Batch inversion of the lo/hi entries' A parts (Montgomery's trick), one group per chain (half, k, lo|hi), in
// R-forms throughout. k_pair_inv_fwd: prefix products P_j = (L_0 .. L_j) R (scratch) and the chain's product
// P = (L_0 .. L_EM-1) R; the host inverts the 2K chain products of a half at once (one extended-Euclid inversion,
// batch trick) -- the modulus may be composite (n, for the public fixed bases), so no Fermat -- and writes back
// I = P^-1 R^2 = (L_0 .. L_EM-1)^-1 R; k_pair_inv_bwd: inv_j = I_j P_(j-1), I_(j-1) = I_j x_j, i.e.
// inv_j = L_j^-1 R. Every group runs the longest chain (wave-uniform trip counts: the groups' DPP shifts read their
// neighbours); shorter chains are padded with the Montgomery one.
template <int TPI, int LL>
struct PairInvChain {
  int k, sp, E, EM;
  bool valid;
  const uint32_t* lh;
  uint32_t* pre;
  __device__ PairInvChain(const FbgpHalf* H, int K, int W, int gib) {
    const int c0 = blockIdx.x * (BLOCK / TPI) + gib;
    valid = c0 < 2 * K;
    const int c = valid ? c0 : 0;
    k = c >> 1;
    sp = c & 1;
    const int LO = W / 2, HI = W - LO;
    E = 1 << (sp ? HI : LO);
    EM = 1 << (HI > LO ? HI : LO);
    constexpr int S = TPI * LL;
    lh = H->lohi + ((size_t)k * 2 + sp) * FB_LO * 2 * S;
    pre = H->pre + (size_t)c * EM * S;
  }
};

template <int TPI, int LL>
__device__ __forceinline__ void pair_inv_mul(uint32_t (&a)[LL], const uint32_t (&b)[LL], uint32_t* slot, const uint32_t (&m)[LL],
                                             uint32_t mprime, int lane, int tig) {
  wave_lds_fence();
#pragma unroll
  for (int i = 0; i < LL; ++i) slot[tig * LL + i] = b[i];
  wave_lds_fence();
  pgrp::montmul1<TPI, LL>(a, slot, m, mprime, lane, tig);
}

template <int TPI, int LL>
__global__ __launch_bounds__(BLOCK) void k_pair_inv_fwd(const FbgpHalf* halves, int K, int W) {
  constexpr int S = TPI * LL;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int lane = threadIdx.x & 63, tig = threadIdx.x % TPI, gib = threadIdx.x / TPI;
  uint32_t* slot = smem + gib * S;
  const FbgpHalf* H = halves + blockIdx.y;
  const PairInvChain<TPI, LL> ch(H, K, W, gib);
  uint32_t m[LL], one[LL], acc[LL], x[LL];
  fbgp_load<TPI, LL>(H->p, m, tig);
  fbgp_load<TPI, LL>(H->oneR, one, tig);          // R mod p: the Montgomery one
  for (int j = 0; j < ch.EM; ++j) {
    if (j < ch.E) fbgp_load<TPI, LL>(ch.lh + (size_t)j * 2 * S, x, tig);
    else {
#pragma unroll
      for (int i = 0; i < LL; ++i) x[i] = one[i];
    }
    if (j == 0) {
#pragma unroll
      for (int i = 0; i < LL; ++i) acc[i] = x[i];
    } else {
      pair_inv_mul<TPI, LL>(acc, x, slot, m, H->mprime, lane, tig);
    }
    if (ch.valid) pfb_store_limbs<TPI, LL>(ch.pre + (size_t)j * S, acc, tig);
  }
  pgrp::cond_sub<TPI, LL>(acc, m, lane, tig);
  if (ch.valid) pfb_store_limbs<TPI, LL>(H->cval + (size_t)(2 * ch.k + ch.sp) * S, acc, tig);
}

template <int TPI, int LL>
__global__ __launch_bounds__(BLOCK) void k_pair_inv_bwd(const FbgpHalf* halves, int K, int W) {
  constexpr int S = TPI * LL;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int lane = threadIdx.x & 63, tig = threadIdx.x % TPI, gib = threadIdx.x / TPI;
  uint32_t* slot = smem + gib * S;
  const FbgpHalf* H = halves + blockIdx.y;
  const PairInvChain<TPI, LL> ch(H, K, W, gib);
  uint32_t m[LL], one[LL], I[LL], x[LL];
  fbgp_load<TPI, LL>(H->p, m, tig);
  fbgp_load<TPI, LL>(H->oneR, one, tig);
  fbgp_load<TPI, LL>(H->cval + (size_t)(2 * ch.k + ch.sp) * S, I, tig);
  uint32_t* out = H->inv + ((size_t)ch.k * 2 + ch.sp) * FB_LO * S;
  for (int j = ch.EM - 1; j >= 1; --j) {
    uint32_t t[LL];
    fbgp_load<TPI, LL>(ch.pre + (size_t)(j - 1) * S, x, tig);
#pragma unroll
    for (int i = 0; i < LL; ++i) t[i] = I[i];
    pair_inv_mul<TPI, LL>(t, x, slot, m, H->mprime, lane, tig);
    pgrp::cond_sub<TPI, LL>(t, m, lane, tig);
    if (ch.valid && j < ch.E) pfb_store_limbs<TPI, LL>(out + (size_t)j * S, t, tig);
    if (j < ch.E) fbgp_load<TPI, LL>(ch.lh + (size_t)j * 2 * S, x, tig);
    else {
#pragma unroll
      for (int i = 0; i < LL; ++i) x[i] = one[i];
    }
    pair_inv_mul<TPI, LL>(I, x, slot, m, H->mprime, lane, tig);
  }
  pgrp::cond_sub<TPI, LL>(I, m, lane, tig);
  if (ch.valid) pfb_store_limbs<TPI, LL>(out, I, tig);
}

// lo[j] = B_k^j R (j < 2^LO), hi[j] = (B_k^(2^LO))^j R (j < 2^(W - LO)): one group per entry, square-and-
// multiply with wave-uniform control (a group whose bit is clear multiplies by R, the Montgomery one)
template <int TPI, int LL>
__global__ __launch_bounds__(BLOCK) void k_fbgp_lohi(const FbgpHalf* halves, int K, int W) {
  constexpr int S = TPI * LL;
  constexpr int GPB = BLOCK / TPI;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int lane = threadIdx.x & 63;
  const int tig = threadIdx.x % TPI;
  const int gib = threadIdx.x / TPI;
  uint32_t* slot = smem + gib * 2 * S;
  uint32_t* xs = smem + GPB * 2 * S;
  const int half = blockIdx.z;
  const int k = blockIdx.y;
  const FbgpHalf* H = halves + half;
  for (int i = threadIdx.x; i < S; i += BLOCK) xs[i] = H->X[i];
  __syncthreads();
  const int LO = W / 2, HI = W - LO;
  const int nlo = 1 << LO, nent = nlo + (1 << HI);
  const int e = blockIdx.x * GPB + gib;
  const bool valid = e < nent;
  const int s = valid && e >= nlo ? 1 : 0;
  const uint32_t j = valid ? (uint32_t)(s ? e - nlo : e) : 0u;
  const int bits = s ? HI : LO;
  uint32_t m[LL], A[LL], B[LL], xa[LL], xb[LL], oa[LL], ob[LL];
  fbgp_load<TPI, LL>(H->p, m, tig);
  const uint32_t* xg = H->bases + ((size_t)k * 2 + s) * 2 * S;
  fbgp_load<TPI, LL>(xg, xa, tig);
  fbgp_load<TPI, LL>(xg + S, xb, tig);
  fbgp_load<TPI, LL>(H->oneR, oa, tig);
  fbgp_load<TPI, LL>(H->oneR + S, ob, tig);
#pragma unroll
  for (int i = 0; i < LL; ++i) {
    A[i] = oa[i];
    B[i] = ob[i];
  }
  for (int b = max(LO, HI) - 1; b >= 0; --b) {
    fbgp_regs_to_slot<TPI, LL>(slot, A, B, tig);
    pgrp::montmul<TPI, LL, true>(A, B, slot, xs, m, H->mprime, lane, tig);
    const bool mul = b < bits && ((j >> b) & 1u);
    uint32_t ta[LL], tb[LL];
#pragma unroll
    for (int i = 0; i < LL; ++i) {
      ta[i] = mul ? xa[i] : oa[i];
      tb[i] = mul ? xb[i] : ob[i];
    }
    fbgp_regs_to_slot<TPI, LL>(slot, ta, tb, tig);
    pgrp::montmul<TPI, LL, false>(A, B, slot, xs, m, H->mprime, lane, tig);
  }
  if (valid) {
    uint32_t* o = H->lohi + (((size_t)k * 2 + s) * FB_LO + j) * 2 * S;
#pragma unroll
    for (int i = 0; i < LL; ++i) {
      o[tig * LL + i] = A[i];
      o[S + tig * LL + i] = B[i];
    }
  }
}

template <int TPI, int LL>
__global__ __launch_bounds__(BLOCK) void k_fbgp_fill(const FbgpHalf* halves, int K, int W, uint32_t* table0, uint32_t* table1) {
  constexpr int S = TPI * LL;
  constexpr int GPB = BLOCK / TPI;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int lane = threadIdx.x & 63;
  const int tig = threadIdx.x % TPI;
  const int gib = threadIdx.x / TPI;
  uint32_t* slot = smem + gib * 2 * S;
  uint32_t* xs = smem + GPB * 2 * S;
  const int half = blockIdx.z;
  const int k = blockIdx.y;
  const FbgpHalf* H = halves + half;
  for (int i = threadIdx.x; i < S; i += BLOCK) xs[i] = H->X[i];
  __syncthreads();
  const int ent = 1 << W, LO = W / 2;
  const int d0 = blockIdx.x * GPB + gib;
  const bool valid = d0 < ent;
  const int d = valid ? d0 : ent - 1;
  uint32_t m[LL], A[LL], B[LL];
  fbgp_load<TPI, LL>(H->p, m, tig);
  const uint32_t* lo = H->lohi + (((size_t)k * 2 + 0) * FB_LO + (d & ((1 << LO) - 1))) * 2 * S;
  const uint32_t* hi = H->lohi + (((size_t)k * 2 + 1) * FB_LO + (d >> LO)) * 2 * S;
  fbgp_load<TPI, LL>(lo, A, tig);
  fbgp_load<TPI, LL>(lo + S, B, tig);
  {
    uint32_t ha[LL], hb[LL];
    fbgp_load<TPI, LL>(hi, ha, tig);
    fbgp_load<TPI, LL>(hi + S, hb, tig);
    fbgp_regs_to_slot<TPI, LL>(slot, ha, hb, tig);
  }
  pgrp::montmul<TPI, LL, false>(A, B, slot, xs, m, H->mprime, lane, tig);
  pgrp::canon<TPI, LL>(A, B, m, lane, tig);
  pair_factor_row<TPI, LL>(B, H, k, d, W, slot, m, lane, tig);
  uint4* t = reinterpret_cast<uint4*>(half ? table1 : table0);
  pair_store_row<TPI, LL>(valid ? t + ((size_t)k * ent + d) * FBGP_ROW4 : nullptr, slot, A, B, tig);
}

}  // namespace fpai
