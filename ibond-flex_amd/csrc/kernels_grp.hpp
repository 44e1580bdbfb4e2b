// Key-holder encryption for keys whose CRT squares p^2, q^2 do not fit one lane (nb = 4096: p_h^2 has
// 4096 bits = 148 limbs of 28 bits, against the lane engine's 74): the per-half work moves to the
// lane-group engine (bn_group.hpp), TPI = 4 lanes x 37 limbs per number, and the recombination with c0
// is k_crt_fin<8> (kernels_crt.hpp) over n^2. Only the fixed-base sampler exists at this size: an
// explicit r, or device-RNG encryption without resident tables, runs the public-key path (k_encrypt<8>).
//
//   k_fbg<TPI>     fixed-base sampler (kernels_fb.hpp's distribution and digits): u_h = G_h^(a_h) coef_h,
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
// FbHalf fields as used here: table = rows of S limbs ([K][2^W][S] u32, as uint4*), m, mprime, and
// nm = coef_h (plain, S limbs); R2 / oneR / bases / lohi for the table construction.
template <int TPI>
__device__ __forceinline__ void fbg_row_load(const uint32_t* __restrict__ row, uint32_t (&x)[L], int tig) {
  int t = tig;
  asm volatile("" : "+v"(t));
#pragma unroll
  for (int i = 0; i < L; ++i) x[i] = row[t * L + i];
}

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
    uint32_t a[L];
    fbg_row_load<TPI>(table + (size_t)dg[0] * S, a, tig);            // T_0[d_0] (Montgomery form)
    for (int k = 1; k < K; ++k) {
      // no register prefetch of the next row (37 more VGPRs spill the product): one product is ~40k
      // cycles per wave, the row's HBM latency hides behind the other resident wave of the SIMD
      uint32_t b[L];
      fbg_row_load<TPI>(table + (((size_t)k << W) + dg[(size_t)k * p.n]) * S, b, tig);
      write_limbs_lds<TPI>(slot, b, tig);
      montmul<TPI>(a, a, slot, TPI, m, H->mprime, lane, tig);
    }
    copy_g_to_lds<TPI>(slot, H->nm, tig);                             // coef_h (plain): leaves Montgomery form
    montmul<TPI>(a, a, slot, TPI, m, H->mprime, lane, tig);
    cond_sub<TPI>(a, m, lane, tig);
    if (valid) {
#pragma unroll
      for (int i = 0; i < L; ++i) p.out[((size_t)half * S + tig * L + i) * p.n + ii] = a[i];
    }
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
