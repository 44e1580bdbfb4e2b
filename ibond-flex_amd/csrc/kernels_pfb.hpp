// Public-key fixed-base obfuscators (DESIGN.md §3 "Fixed bases without the private key"): a party that
// holds only n draws r = g_0^e_0 * g_1^e_1 * ... * g_32^e_32 mod n from bases g_j it picked itself and
// uniform exponents (e_0: nb + 64 bits, e_1..e_32: 96 bits), so that
//   r^n mod n^2 = prod_j h_j^e_j,  h_j = g_j^n mod n^2,
// a product of K table rows T_k[d] = h_j(k)^(d 2^(W pos(k))) instead of the 2047 squarings + ~410 products of
// r^n (obfuscator.py:36). The ciphertext is the reference's encryption under that r (raw_encrypt.py:22-49,
// obfuscator.py:23-37): c = c0 r^n mod n^2, c0 = 1 + n M.
//
// Every product mod n^2 is a p-adic pair product (bn_pgroup.hpp) over the 76 limbs of n on a lane group of
// 4 x 19 limbs: v = A + n B. Nothing in the pair algebra needs n prime (kernels_pe.hpp).
//
//   k_pfb_chain   once per key: one group per base: h_j R = (g_j R)^n by square-and-multiply, then the digit
//                 bases B_k R = (h_j R)^(2^(W pos)) and B_k^(2^LO) R, canonical pairs, for k_fbgp_lohi
//   k_fbgp_lohi   (kernels_grp_pair.hpp, one "half") lo/hi half-digit powers
//   k_pair_inv   (kernels_grp_pair.hpp) batch inversion of the lo/hi entries' A parts
//   k_pfb_fill    T_k[d] R = lo * hi as a factored row a (1 + n b): the words of a, then of b R mod n
//                 (512 B per row at nb = 2048: four aligned 128-B lines; kernels_grp_pair.hpp "factored rows")
//   k_pfb_digits  per element: the ChaCha20 stream (nonce: index, 0x70666230) cut into K W-bit digits
//   k_pfb         per element: encode, c0 = the pair (1, M mod n), K products by (a_k, 0) + the b sum, the
//                 correction (1 + n sum b_k), canonical pair -> xw
//   k_pe_fin      (kernels_pe.hpp) c = A + n B -> ciphertext words
#pragma once
#include "kernels_grp_pair.hpp"
#include "kernels_pe.hpp"

namespace fpai {

constexpr int PFB_TPI = 4, PFB_LL = 19, PFB_S = PFB_TPI * PFB_LL;   // 76 limbs: R = 2^2128 >= 2^24 n
constexpr int PFB_SHORT = 32;        // bases with short exponents (subgroup coverage)
constexpr int PFB_TBITS = 96;        // bits of a short exponent (rounded up to whole digits)
constexpr int PFB_E0_EXTRA = 64;     // e_0 has nb + 64 bits (rounded up to whole digits)
constexpr int PFB_NBASES = 1 + PFB_SHORT;
constexpr int PFB_PW = FBGP_PW;      // 32-bit words of A and of B in a table row (n < 2^2048)
constexpr int PFB_SP = 74;           // limbs of A and of B written for k_pe_fin (n < 2^(28 74))
constexpr int PFB_ROW4 = FBGP_ROW4;  // uint4 per table row
constexpr int PFB_DIG_BLOCK = 128;

struct PfbConst {
  FbgpHalf g;              // modulus n: p = n limbs, X = (1 - R) mod n, oneR = pair of R mod n^2, bases, lohi
  const uint4* table;      // [K][2^W] rows of PFB_ROW4 uint4
  const uint32_t* gl;      // [nbases][S] limbs of the bases g_j (< n)
  const uint32_t* r2;      // pair of R^2 mod n^2 [A: S][B: S]
  const uint32_t* nw;      // n as 32-bit words (the exponent of k_pfb_chain), PFB_PW words
  int nbits;               // bits of n
  int nbases;
  int K, W, K0, KS;        // digits: K = K0 + (nbases - 1) KS; base 0 owns slots [0, K0)
};

struct PfbParams {
  const PfbConst* c;
  long long n;
  const uint32_t* digits;  // [K][n]
  const void* x;
  int dtype, exp_mode, fexp;
  int32_t* exp;
  int32_t* status;
  uint32_t* xw;            // [2 PFB_SP][n]: canonical pair limbs for k_pe_fin
};

struct PfbDigitParams {
  long long n;
  uint32_t rng_key[8];
  unsigned long long index_base;
  int K, W;
  uint32_t* digits;        // [K][n]
};

// ---------------------------------------------------------------- per-key table construction
template <int TPI, int LL>
__device__ __forceinline__ void pfb_store_pair(uint32_t* dst, const uint32_t (&A)[LL], const uint32_t (&B)[LL], int tig) {
  constexpr int S = TPI * LL;
#pragma unroll
  for (int i = 0; i < LL; ++i) {
    dst[tig * LL + i] = A[i];
    dst[S + tig * LL + i] = B[i];
  }
}

// One group per base: h_j R = (g_j R)^n (left-to-right binary, the bits of n are wave-uniform), then for each
// of its digit slots k: bases[k][0] = B_k R, bases[k][1] = B_k^(2^LO) R (canonical pairs), B_(k+1) = B_k^(2^W).
template <int TPI, int LL>
__global__ __launch_bounds__(BLOCK) void k_pfb_chain(const PfbConst* c) {
  constexpr int S = TPI * LL;
  constexpr int GPB = BLOCK / TPI;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int lane = threadIdx.x & 63;
  const int tig = threadIdx.x % TPI;
  const int gib = threadIdx.x / TPI;
  uint32_t* slot = smem + gib * 2 * S;
  uint32_t* xs = smem + GPB * 2 * S;
  const FbgpHalf* H = &c->g;
  for (int i = threadIdx.x; i < S; i += BLOCK) xs[i] = H->X[i];
  __syncthreads();
  const int j0 = blockIdx.x * GPB + gib;
  const bool valid = j0 < c->nbases;
  const int j = valid ? j0 : 0;
  uint32_t m[LL], A[LL], B[LL], xa[LL], xb[LL];
  fbgp_load<TPI, LL>(H->p, m, tig);
  const uint32_t mprime = H->mprime;
  // x = (g_j, 0) R: the plain pair times the pair of R^2
  fbgp_load<TPI, LL>(c->gl + (size_t)j * S, xa, tig);
#pragma unroll
  for (int i = 0; i < LL; ++i) xb[i] = 0u;
  {
    uint32_t ra[LL], rb[LL];
    fbgp_load<TPI, LL>(c->r2, ra, tig);
    fbgp_load<TPI, LL>(c->r2 + S, rb, tig);
    fbgp_regs_to_slot<TPI, LL>(slot, ra, rb, tig);
    pgrp::montmul<TPI, LL, false>(xa, xb, slot, xs, m, mprime, lane, tig);
  }
  fbgp_load<TPI, LL>(H->oneR, A, tig);
  fbgp_load<TPI, LL>(H->oneR + S, B, tig);
  for (int b = c->nbits - 1; b >= 0; --b) {
    fbgp_regs_to_slot<TPI, LL>(slot, A, B, tig);
    pgrp::montmul<TPI, LL, true>(A, B, slot, xs, m, mprime, lane, tig);
    if ((c->nw[b >> 5] >> (b & 31)) & 1u) {
      fbgp_regs_to_slot<TPI, LL>(slot, xa, xb, tig);
      pgrp::montmul<TPI, LL, false>(A, B, slot, xs, m, mprime, lane, tig);
    }
  }
  // wave-uniform trip counts (the groups' DPP shifts read their neighbours): every group runs base 0's K0
  // positions and stores only its own
  const int k0 = j == 0 ? 0 : c->K0 + (j - 1) * c->KS;
  const int len = j == 0 ? c->K0 : c->KS;
  const int W = c->W, LO = W / 2;
  for (int pos = 0; pos < c->K0; ++pos) {
    const bool mine = valid && pos < len;
    uint32_t ca[LL], cb[LL];
#pragma unroll
    for (int i = 0; i < LL; ++i) {
      ca[i] = A[i];
      cb[i] = B[i];
    }
    pgrp::canon<TPI, LL>(ca, cb, m, lane, tig);
    if (mine) pfb_store_pair<TPI, LL>(const_cast<uint32_t*>(H->bases) + ((size_t)(k0 + pos) * 2 + 0) * 2 * S, ca, cb, tig);
    for (int q = 0; q < W; ++q) {
      fbgp_regs_to_slot<TPI, LL>(slot, A, B, tig);
      pgrp::montmul<TPI, LL, true>(A, B, slot, xs, m, mprime, lane, tig);
      if (q + 1 == LO) {
#pragma unroll
        for (int i = 0; i < LL; ++i) {
          ca[i] = A[i];
          cb[i] = B[i];
        }
        pgrp::canon<TPI, LL>(ca, cb, m, lane, tig);
        if (mine) pfb_store_pair<TPI, LL>(const_cast<uint32_t*>(H->bases) + ((size_t)(k0 + pos) * 2 + 1) * 2 * S, ca, cb, tig);
      }
    }
  }
}

// T_k[d] R = lo[d mod 2^LO] hi[d >> LO] R^-1, canonical, as the 32-bit words of A then of B. The canonical pair
// goes through the group's LDS slot; lane t writes words [32 t, 32 t + 32) of the row (16-byte stores).
template <int TPI, int LL>
__global__ __launch_bounds__(BLOCK) void k_pfb_fill(const PfbConst* c, int K, int W, uint4* table) {
  constexpr int S = TPI * LL;
  constexpr int GPB = BLOCK / TPI;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int lane = threadIdx.x & 63;
  const int tig = threadIdx.x % TPI;
  const int gib = threadIdx.x / TPI;
  uint32_t* slot = smem + gib * 2 * S;
  uint32_t* xs = smem + GPB * 2 * S;
  const FbgpHalf* H = &c->g;
  const int k = blockIdx.y;
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
  if (valid) pair_store_row<TPI, LL>(table + ((size_t)k * ent + d) * FBGP_ROW4, slot, A, B, tig);
  else pair_store_row<TPI, LL>(nullptr, slot, A, B, tig);
}

// ---------------------------------------------------------------- per element
// digits[k][i] = bits [W k, W k + W) of the element's ChaCha20 stream (key, counter 0.., nonce = (index lo,
// index hi, 0x70666230)); the stream is consumed in order through a 64-bit bit buffer (W <= 24).
template <int DUMMY = 0>   // (a template only so the header can be included by several units)
__global__ __launch_bounds__(PFB_DIG_BLOCK) void k_pfb_digits(PfbDigitParams p) {
  const uint32_t mask = (1u << p.W) - 1u;
  for (long long i = (long long)blockIdx.x * PFB_DIG_BLOCK + threadIdx.x; i < p.n;
       i += (long long)gridDim.x * PFB_DIG_BLOCK) {
    const unsigned long long g = p.index_base + (unsigned long long)i;
    uint64_t acc = 0;
    int have = 0, k = 0;
    for (uint32_t b = 0; k < p.K; ++b) {
      uint32_t blk[16];
      chacha20_block(p.rng_key, b, (uint32_t)g, (uint32_t)(g >> 32), 0x70666230u, blk);
#pragma unroll
      for (int w = 0; w < 16; ++w) {
        acc |= (uint64_t)blk[w] << have;
        have += 32;
        while (have >= p.W && k < p.K) {
          p.digits[(size_t)k * p.n + i] = (uint32_t)acc & mask;
          acc >>= p.W;
          have -= p.W;
          ++k;
        }
      }
    }
  }
}

template <int TPI, int LL>
__global__ __launch_bounds__(BLOCK, 2) void k_pfb(PfbParams p) {
  constexpr int S = TPI * LL;
  constexpr int GPB = BLOCK / TPI;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int lane = threadIdx.x & 63;
  const int tig = threadIdx.x % TPI;
  const int gib = threadIdx.x / TPI;
  const PfbConst* C = p.c;
  const FbgpHalf* H = &C->g;
  __shared__ __attribute__((aligned(16))) uint32_t stage[(BLOCK / 64) * FBGP_STAGE_WORDS];
  uint32_t* slot = smem + gib * 2 * S;
  const uint32_t* wstage = stage + (threadIdx.x / 64) * FBGP_STAGE_WORDS;
  uint32_t* xs = smem + GPB * 2 * S;
  for (int i = threadIdx.x; i < S; i += BLOCK) xs[i] = H->X[i];
  __syncthreads();
  uint32_t m[LL];
  fbgp_load<TPI, LL>(H->p, m, tig);
  const uint32_t mprime = H->mprime;
  const int K = C->K, W = C->W;
  const uint4* table = C->table;
  for (long long base = (long long)blockIdx.x * GPB; base < p.n; base += (long long)gridDim.x * GPB) {
    const long long inst = base + gib;
    const bool valid = inst < p.n;
    const long long ii = valid ? inst : p.n - 1;
    const uint32_t* dg = p.digits + ii;
    int64_t M = 0;
    int e = 0, st;
    const bool fixed = p.exp_mode != 0;
    if (p.dtype == 0) st = encode_float((double)((const float*)p.x)[ii], fixed, p.fexp, M, e);
    else if (p.dtype == 1) st = encode_float(((const double*)p.x)[ii], fixed, p.fexp, M, e);
    else st = encode_int(((const int64_t*)p.x)[ii], fixed, p.fexp, M, e);
    if (valid && tig == 0) {
      p.exp[ii] = e;
      if (p.status) p.status[ii] = st;
    }
    // c0 = 1 + n M: the pair (1, M mod n) (M < 0: n - |M|)
    uint32_t A[LL], B[LL];
    {
      const bool neg = M < 0;
      const uint64_t mag = neg ? (uint64_t)0 - (uint64_t)M : (uint64_t)M;
      uint32_t ml[LL];
#pragma unroll
      for (int i = 0; i < LL; ++i) {
        ml[i] = (tig == 0 && i < 3) ? (uint32_t)(mag >> (LB * i)) & LMASK : 0u;
        A[i] = (tig == 0 && i == 0) ? 1u : 0u;
      }
      uint32_t D[LL];
      (void)pgrp::sub_limbs<TPI, LL>(m, ml, D, lane, tig);
#pragma unroll
      for (int i = 0; i < LL; ++i) B[i] = neg ? D[i] : ml[i];
    }
    pair_table_products<TPI, LL>(A, B, table, dg, p.n, K, W, slot, wstage, xs, m, mprime, lane, tig);
    pair_apply_bsum<TPI, LL>(A, B, slot, const_cast<uint32_t*>(wstage) + (lane / TPI) * 2 * FBGP_PW, m, mprime, lane, tig);
    pgrp::cond_sub<TPI, LL>(B, m, lane, tig);   // B < 4p -> < 2p
    pgrp::cond_sub<TPI, LL>(B, m, lane, tig);
    pgrp::canon<TPI, LL>(A, B, m, lane, tig);
    if (valid) {
#pragma unroll
      for (int i = 0; i < LL; ++i) {
        const int idx = tig * LL + i;
        if (idx < PFB_SP) {
          p.xw[(size_t)idx * p.n + ii] = A[i];
          p.xw[((size_t)PFB_SP + idx) * p.n + ii] = B[i];
        }
      }
    }
  }
}

}  // namespace fpai
