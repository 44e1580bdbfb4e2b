// Fixed-base sampler for 4096-bit keys on pair groups (bn_pgroup.hpp: TPI = 4 lanes x LL = 19 limbs, S = 76
// limbs of p_h): kernels_grp.hpp's k_fbg with every product mod p_h^2 a pair product, 5 S^2 = 28.9 k lane-MACs
// against k_fbg's 2 (148)^2 = 43.8 k. Same distribution and ciphertext bits.
//
//   k_fbgp       w_h = c0 G_h^(a_h) mod p_h^2 as the canonical pair (A, B) (c0 = the pair (1, (n/p_h) M))
//   k_fbgp_w     w_h = A + p_h B mod p_h^2 (one product mod p_h^2 on the L = 37 group engine, in place), so
//                k_fbg_garner and k_fbg_fin recombine exactly as after k_fbg
//   k_fbgp_lohi / k_fbgp_fill   the per-key tables: rows of [A: 74][B: 74] limbs of T_k[d] R mod p_h^2 (the
//                148-limb row size of k_fbg's tables)
#pragma once
#include "bn_pgroup.hpp"
#include "kernels_grp.hpp"

namespace fpai {

constexpr int FBGP_TPI = 4, FBGP_LL = 19, FBGP_S = FBGP_TPI * FBGP_LL;   // 76 limbs >= the 74 of a 2048-bit p_h
constexpr int FBGP_SP = 74;                                               // limbs of A and of B in a table row

struct FbgpHalf {
  const uint32_t* table;   // [K][2^W][2 SP] rows: canonical pair of T_k[d] R mod p_h^2
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
  uint32_t* slot = smem + gib * 2 * S;
  uint32_t* xs = smem + GPB * 2 * S;
  for (int i = threadIdx.x; i < S; i += BLOCK) xs[i] = H->X[i];
  __syncthreads();
  uint32_t m[LL];
  fbgp_load<TPI, LL>(H->p, m, tig);
  const uint32_t mprime = H->mprime;
  const int K = p.K, W = p.W;
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
    for (int k = 0; k < K; ++k) {
      fbgp_pair_to_slot<TPI, LL>(slot, H->table + (((size_t)k << W) + dg[(size_t)k * p.n]) * 2 * FBGP_SP, FBGP_SP, tig);
      pgrp::montmul<TPI, LL, false>(A, B, slot, xs, m, mprime, lane, tig);
    }
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
  if (valid) {
    uint32_t* row = (half ? table1 : table0) + ((size_t)k * ent + d) * 2 * FBGP_SP;
#pragma unroll
    for (int i = 0; i < LL; ++i) {
      const int idx = tig * LL + i;
      if (idx < FBGP_SP) {
        row[idx] = A[i];
        row[FBGP_SP + idx] = B[i];
      }
    }
  }
}

}  // namespace fpai
