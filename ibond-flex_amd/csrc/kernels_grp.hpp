// Key-holder encryption for keys whose CRT squares p^2, q^2 do not fit one lane (nb = 4096: p_h^2 has
// 4096 bits = 148 limbs of 28 bits, against the lane engine's 74): the per-half work moves to the
// lane-group engine (bn_group.hpp), TPI = 4 lanes x 37 limbs per number, with c0 folded into the first
// product, and the halves are recombined by Garner (k_fbg_garner mod p^2, k_fbg_fin mod n^2). Only the
// fixed-base sampler exists at this size: an explicit r, or device-RNG encryption without resident
// tables, runs the public-key path (k_encrypt<8>).
//
//   k_fbg<TPI>     fixed-base sampler (kernels_fb.hpp's distribution and digits): w_h = c0 G_h^(a_h) mod p_h^2,
//                  K table products per half, no squarings; rows are the S canonical 28-bit limbs of
//                  T_k[d] R (lane t of a group loads its 37 limbs)
//   k_fbg_lohi / k_fbg_fill   the per-key tables, built like kernels_fb.hpp's (lo/hi half-digit powers,
//                  then one product per entry), on the group engine
// blockIdx.y selects the half (p or q), so modulus, exponent schedule and constants are wave-uniform.
#pragma once
#include "kernels_crt.hpp"
#include "kernels_fb.hpp"

namespace fpai {

// ---------------------------------------------------------------- fixed-base sampler
// FbHalf fields as used here: table = rows of S limbs ([K][2^W][S] u32, as uint4*), m, mprime, nm = [4][S]
// n 2^(16 c) mod p_h^2 and pbig = 2^20 p_h^2 (c0 folding); R2 / oneR / bases / lohi for the table build.
template <int TPI>
__device__ __forceinline__ void fbg_row_load(const uint32_t* __restrict__ row, uint32_t (&x)[L], int tig) {
  int t = tig;
  asm volatile("" : "+v"(t));
#pragma unroll
  for (int i = 0; i < L; ++i) x[i] = row[t * L + i];
}

// A operand of the first product: c0 = 1 + n M as the unreduced sum 1 + sum_c (n 2^(16 c) mod p_h^2) M_c
// over the 16-bit chunks of |M| (negative M: 1 + 2^20 p_h^2 - sum), < 2^21 p_h^2 < R / 4 (R = 2^(28 S),
// p_h^2 < 2^4096): a valid CIOS operand, so c0 costs no product (kernels_fb.hpp fb_c0, group layout).
template <int TPI>
__device__ __forceinline__ void fbg_c0(int64_t M, const uint32_t* __restrict__ nm, const uint32_t* __restrict__ pbig,
                                       uint32_t (&a)[L], int lane, int tig) {
  constexpr int S = TPI * L;
  const bool neg = M < 0;
  const uint64_t mag = neg ? (uint64_t)0 - (uint64_t)M : (uint64_t)M;
  uint32_t mc[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) mc[c] = (uint32_t)(mag >> (16 * c)) & 0xFFFFu;
  int t = tig;
  asm volatile("" : "+v"(t));
  uint64_t P[L];
#pragma unroll
  for (int i = 0; i < L; ++i) {
    uint64_t v = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) v += (uint64_t)nm[c * S + t * L + i] * mc[c];
    P[i] = v;
  }
  uint32_t X[L], B[L], D[L];
  normalize<TPI>(P, X, lane, tig);
  load_limbs_g<TPI>(pbig, B, tig);
  (void)sub_limbs<TPI>(B, X, D, lane, tig);             // 2^20 p_h^2 - sum (only used when M < 0)
#pragma unroll
  for (int i = 0; i < L; ++i) P[i] = (uint64_t)(neg ? D[i] : X[i]) + ((tig == 0 && i == 0) ? 1u : 0u);
  normalize<TPI>(P, a, lane, tig);
}

// Per element and half: w_h = c0 G_h^(a_h) mod p_h^2 (< p_h^2). The first product takes the unreduced c0
// (fbg_c0) as A and row T_0[d_0] (Montgomery form) as B, which leaves the Montgomery domain at once; every
// later product multiplies by a Montgomery-form row and keeps the plain domain. The halves are recombined
// by Garner (k_fbg_garner, k_fbg_fin). The p-half writes the exponent and status.
template <int TPI>
__global__ __launch_bounds__(BLOCK, 2) void k_fbg(FbParams p) {
  constexpr int S = TPI * L;
  constexpr int GPB = BLOCK / TPI;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int lane = threadIdx.x & 63;
  const int tig = threadIdx.x % TPI;
  const int gib = threadIdx.x / TPI;
  const int half = blockIdx.y;
  const FbHalf* H = p.halves + half;
  uint32_t* slot = smem + gib * S;
  uint32_t m[L];
  load_limbs_g<TPI>(H->m, m, tig);
  const uint32_t* table = reinterpret_cast<const uint32_t*>(H->table);
  const int K = p.K, W = p.W;
  for (long long base = (long long)blockIdx.x * GPB; base < p.n; base += (long long)gridDim.x * GPB) {
    const long long inst = base + gib;
    const bool valid = inst < p.n;
    const long long ii = valid ? inst : p.n - 1;
    const uint32_t* dg = p.digits + (size_t)half * K * p.n + ii;   // digit k at dg[k * n]
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
    uint32_t a[L];
    fbg_c0<TPI>(M, H->nm, H->pbig, a, lane, tig);
    for (int k = 0; k < K; ++k) {
      // no register prefetch of the next row (37 more VGPRs spill the product): one product is ~40k
      // cycles per wave, the row's HBM latency hides behind the other resident wave of the SIMD
      uint32_t b[L];
      fbg_row_load<TPI>(table + (((size_t)k << W) + dg[(size_t)k * p.n]) * S, b, tig);
      write_limbs_lds<TPI>(slot, b, tig);
      montmul<TPI>(a, a, slot, TPI, m, H->mprime, lane, tig);
    }
    cond_sub<TPI>(a, m, lane, tig);
    if (valid) {
#pragma unroll
      for (int i = 0; i < L; ++i) p.out[((size_t)half * S + tig * L + i) * p.n + ii] = a[i];
    }
  }
}

// Garner, step 1 (mod p^2, S = 148): h = (w_p - w_q) (q^2)^-1 mod p^2 = (w_p + 8 p^2 - w_q) coefR R^-1
// (w_q < q^2 < 4 p^2 for balanced primes; the sum < 9 p^2 < R / 4), reduced to < p^2; written over w_p.
struct FbgGarnerParams {
  uint32_t* w;              // [2][S][n] (k_fbg): w_p, w_q; h replaces w_p
  long long n;
  const uint32_t* m;        // p^2
  const uint32_t* m8;       // 8 p^2
  const uint32_t* coefR;    // (q^2)^-1 R mod p^2
  uint32_t mprime;
};
template <int TPI>
__global__ __launch_bounds__(BLOCK) void k_fbg_garner(FbgGarnerParams p) {
  constexpr int S = TPI * L;
  constexpr int GPB = BLOCK / TPI;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int lane = threadIdx.x & 63;
  const int tig = threadIdx.x % TPI;
  const int gib = threadIdx.x / TPI;
  uint32_t* slot = smem + gib * S;
  uint32_t m[L];
  load_limbs_g<TPI>(p.m, m, tig);
  for (long long base = (long long)blockIdx.x * GPB; base < p.n; base += (long long)gridDim.x * GPB) {
    const long long inst = base + gib;
    const bool valid = inst < p.n;
    const long long ii = valid ? inst : p.n - 1;
    uint32_t wp[L], wq[L], t[L];
#pragma unroll
    for (int i = 0; i < L; ++i) {
      wp[i] = p.w[((size_t)tig * L + i) * p.n + ii];
      wq[i] = p.w[((size_t)S + tig * L + i) * p.n + ii];
    }
    load_limbs_g<TPI>(p.m8, t, tig);
    (void)sub_limbs<TPI>(t, wq, t, lane, tig);           // 8 p^2 - w_q > 0
    uint64_t P[L];
#pragma unroll
    for (int i = 0; i < L; ++i) P[i] = (uint64_t)t[i] + wp[i];
    normalize<TPI>(P, t, lane, tig);
    copy_g_to_lds<TPI>(slot, p.coefR, tig);
    montmul<TPI>(t, t, slot, TPI, m, p.mprime, lane, tig);
    cond_sub<TPI>(t, m, lane, tig);
    if (valid) {
#pragma unroll
      for (int i = 0; i < L; ++i) p.w[((size_t)tig * L + i) * p.n + ii] = t[i];
    }
  }
}

// Garner, step 2 (mod n^2, S = 296): c = w_q + q^2 h = w_q + h (q^2 R) R^-1 (exact: h q^2 < n^2, and the
// sum is the CRT value < n^2), streamed to the ciphertext words.
struct FbgFinParams {
  const uint32_t* w;        // [2][SH][n]: h, w_q
  int sh;                   // limbs of a half (148)
  long long n;
  const uint32_t* N;        // n^2 (S limbs)
  const uint32_t* q2R;      // q^2 R mod n^2
  uint32_t mprime;
  uint32_t* ct;
  int ct_words;
};
template <int TPI>
__global__ __launch_bounds__(BLOCK, 1) void k_fbg_fin(FbgFinParams p) {
  constexpr int S = TPI * L;
  constexpr int GPB = BLOCK / TPI;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int lane = threadIdx.x & 63;
  const int tig = threadIdx.x % TPI;
  const int gib = threadIdx.x / TPI;
  uint32_t* slot = smem + gib * S;
  uint32_t m[L];
  load_limbs_g<TPI>(p.N, m, tig);
  for (long long base = (long long)blockIdx.x * GPB; base < p.n; base += (long long)gridDim.x * GPB) {
    const long long inst = base + gib;
    const bool valid = inst < p.n;
    const long long ii = valid ? inst : p.n - 1;
    uint32_t a[L];
    int t = tig;
    asm volatile("" : "+v"(t));
#pragma unroll
    for (int i = 0; i < L; ++i) {
      const int limb = t * L + i;
      a[i] = limb < p.sh ? p.w[(size_t)limb * p.n + ii] : 0u;
    }
    copy_g_to_lds<TPI>(slot, p.q2R, tig);
    montmul<TPI>(a, a, slot, TPI, m, p.mprime, lane, tig);
    cond_sub<TPI>(a, m, lane, tig);
    uint64_t P[L];
#pragma unroll
    for (int i = 0; i < L; ++i) {
      const int limb = t * L + i;
      P[i] = (uint64_t)a[i] + (limb < p.sh ? p.w[((size_t)p.sh + limb) * p.n + ii] : 0u);
    }
    normalize<TPI>(P, a, lane, tig);
    emit_words<TPI>(slot, a, p.ct + ii * p.ct_words, p.ct_words, valid, tig);
  }
}

// lo[j] = B_k^j R (j < 2^LO), hi[j] = B_k^(2^LO j) R (j < 2^(W - LO)): one group per entry, square-and-
// multiply with wave-uniform control (a group whose bit is clear multiplies by R, the Montgomery one)
template <int TPI>
__global__ __launch_bounds__(BLOCK) void k_fbg_lohi(const FbHalf* halves, int K, int W) {
  constexpr int S = TPI * L;
  constexpr int GPB = BLOCK / TPI;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int lane = threadIdx.x & 63;
  const int tig = threadIdx.x % TPI;
  const int gib = threadIdx.x / TPI;
  uint32_t* slot = smem + gib * S;
  const int half = blockIdx.z;
  const int k = blockIdx.y;
  const FbHalf* H = halves + half;
  const int LO = W / 2, HI = W - LO;
  const int nlo = 1 << LO, nent = nlo + (1 << HI);
  const int e = blockIdx.x * GPB + gib;                              // entry: lo[e] or hi[e - nlo]
  const bool valid = e < nent;
  const int s = valid && e >= nlo ? 1 : 0;
  const uint32_t j = valid ? (uint32_t)(s ? e - nlo : e) : 0u;
  const int bits = s ? HI : LO;
  uint32_t m[L], x[L], acc[L];
  load_limbs_g<TPI>(H->m, m, tig);
  // x~ = B_k R, then B_k^(2^LO) R for the hi half
  load_limbs_g<TPI>(H->bases + (size_t)k * S, x, tig);
  copy_g_to_lds<TPI>(slot, H->R2, tig);
  montmul<TPI>(x, x, slot, TPI, m, H->mprime, lane, tig);
  for (int q = 0; q < LO; ++q) {
    const bool sq = s == 1;
    uint32_t one[L];
    load_limbs_g<TPI>(H->oneR, one, tig);
#pragma unroll
    for (int i = 0; i < L; ++i) one[i] = sq ? x[i] : one[i];
    write_limbs_lds<TPI>(slot, one, tig);
    montmul<TPI>(x, x, slot, TPI, m, H->mprime, lane, tig);
  }
  load_limbs_g<TPI>(H->oneR, acc, tig);
  for (int b = max(LO, HI) - 1; b >= 0; --b) {
    write_limbs_lds<TPI>(slot, acc, tig);
    montmul<TPI>(acc, acc, slot, TPI, m, H->mprime, lane, tig);
    const bool mul = b < bits && ((j >> b) & 1u);
    uint32_t t[L];
    load_limbs_g<TPI>(H->oneR, t, tig);
#pragma unroll
    for (int i = 0; i < L; ++i) t[i] = mul ? x[i] : t[i];
    write_limbs_lds<TPI>(slot, t, tig);
    montmul<TPI>(acc, acc, slot, TPI, m, H->mprime, lane, tig);
  }
  if (valid) {
    uint32_t* o = H->lohi + (((size_t)k * 2 + s) * FB_LO + j) * S;
#pragma unroll
    for (int i = 0; i < L; ++i) o[tig * L + i] = acc[i];
  }
}

template <int TPI>
__global__ __launch_bounds__(BLOCK) void k_fbg_fill(const FbHalf* halves, int K, int W, uint32_t* table0, uint32_t* table1) {
  constexpr int S = TPI * L;
  constexpr int GPB = BLOCK / TPI;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int lane = threadIdx.x & 63;
  const int tig = threadIdx.x % TPI;
  const int gib = threadIdx.x / TPI;
  uint32_t* slot = smem + gib * S;
  const int half = blockIdx.z;
  const int k = blockIdx.y;
  const FbHalf* H = halves + half;
  const int ent = 1 << W, LO = W / 2;
  const int d0 = blockIdx.x * GPB + gib;
  const bool valid = d0 < ent;
  const int d = valid ? d0 : ent - 1;
  uint32_t m[L], a[L];
  load_limbs_g<TPI>(H->m, m, tig);
  load_limbs_g<TPI>(H->lohi + (((size_t)k * 2 + 0) * FB_LO + (d & ((1 << LO) - 1))) * S, a, tig);
  copy_g_to_lds<TPI>(slot, H->lohi + (((size_t)k * 2 + 1) * FB_LO + (d >> LO)) * S, tig);
  montmul<TPI>(a, a, slot, TPI, m, H->mprime, lane, tig);
  cond_sub<TPI>(a, m, lane, tig);
  if (valid) {
    uint32_t* row = (half ? table1 : table0) + ((size_t)k * ent + d) * S;
#pragma unroll
    for (int i = 0; i < L; ++i) row[tig * L + i] = a[i];
  }
}

}  // namespace fpai
