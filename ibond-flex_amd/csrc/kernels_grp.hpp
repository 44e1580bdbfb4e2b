// Garner recombination for keys whose CRT squares p^2, q^2 do not fit one lane (nb = 4096: p_h^2 has 4096 bits = 148
// limbs of 28 bits, against the lane engine's 74), on the lane-group engine (bn_group.hpp): k_fbg_garner mod p^2 (TPI 4)
// and k_fbg_fin mod n^2 (TPI 8, the test build's alternative to k_sgp_fin). The pairs come from the 4096-bit samplers
// (kernels_sgp.hpp / kernels_sgs.hpp, or the test build's k_fbgp) through k_sgp_w / k_fbgp_w. (The round-1 group-engine
// sampler k_fbg and its table builders were retired in round 6.)
#pragma once
#include "kernels_crt.hpp"
#include "kernels_fb.hpp"

namespace fpai {

// Garner, step 1 (mod p^2, S = 148): h = (w_p - w_q) (q^2)^-1 mod p^2 = (w_p + 8 p^2 - w_q) coefR R^-1
// (w_q < q^2 < 4 p^2 for balanced primes; the sum < 9 p^2 < R / 4), reduced to < p^2; written over w_p.
struct FbgGarnerParams {
  uint32_t* w;              // [2][S][n]: w_p, w_q; h replaces w_p
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

}  // namespace fpai
