// Public-key encryption for n of up to 1024 bits (the reference protocols' default key, sec_param.json:3; api.py:22)
// on p-adic pairs over the S = 37 limbs of n (bn_pair.hpp: every product mod n^2 as two CIOS rows over n's limbs, a
// square 3.5 S^2 MACs, a product 5 S^2, against 2 (2S)^2 for the group engine's product over the 74 limbs of n^2 that
// k_encrypt<2> runs). n need not be prime: the pair algebra (v = A + n B) uses only R >= 2^12 n. Per element, one lane:
//   k_pe1_words   the obfuscator's words: the caller's r (any stride, 0 for a scalar) or the element's ChaCha20 stream
//   k_dec_pre_pair (kernels_pair.hpp, with n in place of p_h): r~ = r R mod n^2 as a pair, one CIOS over r's digits
//   k_pe1_pow     r^n mod n^2: the lane machine's op list over n on pair tiles, the product by the pair (1, 0) last
//   k_pe1_fin     c = c0 r^n with c0 = 1 + n M (raw_encrypt.py:37-45): (A + n B)(1 + n M) = A + n (B + A M) mod n^2,
//                 A M mod n by two Montgomery products; the words of c out, the exponent and status
#pragma once
#include "kernels_pair.hpp"

namespace fpai {

struct Pe1Params {
  const void* x;
  int dtype, exp_mode, fexp;
  int obf;                  // PAI_OBF_GIVEN (1) or PAI_OBF_RNG (2)
  const uint32_t* r;        // GIVEN: words, element i at r + i * r_stride
  long long r_stride;
  int r_words;              // GIVEN: words of r
  int rng_words;            // RNG: words of the ChaCha20 stream
  uint32_t rng_key[8];
  unsigned long long index_base;
  long long n;              // elements
  const uint32_t* nl;       // n, S limbs
  const uint32_t* one;      // the pair (1, 0), 2S limbs
  const uint32_t* prog;     // op list over n
  int nprog;
  const uint32_t* r2n;      // R^2 mod n, S limbs
  uint32_t mprime;          // -n^-1 mod 2^28
  uint32_t* rw;             // [n][rw_words] obfuscator words
  int rw_words;
  uint32_t* xw;             // [2S][n] pairs
  uint32_t* scratch;        // per-lane tiles
  uint32_t* ct;
  int32_t* exp;
  int32_t* status;
  int ct_words;
};

template <int DUMMY = 0>
__global__ __launch_bounds__(LANE_BLOCK) void k_pe1_words(Pe1Params p) {
  for (long long i = (long long)blockIdx.x * LANE_BLOCK + threadIdx.x; i < p.n; i += (long long)gridDim.x * LANE_BLOCK) {
    uint32_t* o = p.rw + i * p.rw_words;
    if (p.obf == 1) {
      const uint32_t* rg = p.r + i * p.r_stride;
      for (int w = 0; w < p.rw_words; ++w) o[w] = w < p.r_words ? rg[w] : 0u;
    } else {
      const unsigned long long g = p.index_base + (unsigned long long)i;
      for (int b = 0; b * 16 < p.rw_words; ++b) {
        uint32_t blk[16];
        chacha20_block(p.rng_key, (uint32_t)b, (uint32_t)g, (uint32_t)(g >> 32), 0x66786169u, blk);
#pragma unroll
        for (int w = 0; w < 16; ++w)
          if (b * 16 + w < p.rw_words) o[b * 16 + w] = blk[w];
      }
    }
  }
}

template <int S>
__global__ __launch_bounds__(LANE_BLOCK, LANE_OCC) void k_pe1_pow(Pe1Params p) {
  uint32_t m[S];
#pragma unroll
  for (int j = 0; j < S; ++j) m[j] = p.nl[j];
  const LaneScratch tl = lane_scratch(p.scratch);
  const uint32_t* prog = p.prog;
  for (long long base = (long long)blockIdx.x * LANE_BLOCK; base < p.n; base += (long long)gridDim.x * LANE_BLOCK) {
    const long long i = base + threadIdx.x;
    const long long ii = i < p.n ? i : p.n - 1;
    uint32_t A[S], B[S];
#pragma unroll
    for (int j = 0; j < S; ++j) {
      A[j] = p.xw[(size_t)j * p.n + ii];
      B[j] = p.xw[(size_t)(S + j) * p.n + ii];
    }
    ptile_store<S>(tl, 0, A, B, std::make_integer_sequence<int, tile_quads<2 * S>()>{});
    run_pair_program<S>(A, B, tl, prog, p.nprog, p.one, m, p.mprime);   // r^n (the last product by (1, 0))
    pair::canon<S>(A, B, m);
    if (i < p.n) {
#pragma unroll
      for (int j = 0; j < S; ++j) {
        p.xw[(size_t)j * p.n + i] = A[j];
        p.xw[(size_t)(S + j) * p.n + i] = B[j];
      }
    }
  }
}

// word W (bits [32 W, 32 W + 32)) of the value held as N 28-bit limbs X (compile-time limb indices)
template <int N, int W>
__device__ __forceinline__ void pe1_word(const uint32_t (&X)[N], uint32_t* o, int nw) {
  constexpr int bit = 32 * W, k = bit / LB, sh = bit - k * LB;
  uint64_t v = (uint64_t)X[k] >> sh;
  if constexpr (k + 1 < N) v |= (uint64_t)X[k + 1] << (LB - sh);
  if constexpr (k + 2 < N && 2 * LB - sh < 32) v |= (uint64_t)X[k + 2] << (2 * LB - sh);
  if (W < nw) o[W] = (uint32_t)v;
}
template <int N, int... Ws>
__device__ __forceinline__ void pe1_words_out(const uint32_t (&X)[N], uint32_t* o, int nw, std::integer_sequence<int, Ws...>) {
  (pe1_word<N, Ws>(X, o, nw), ...);
}

// the 2S limbs of A + n B (kernels_fbp.hpp fbp_col: product scanning, compile-time columns)
template <int S, int... Ks>
__device__ __forceinline__ void pe1_cols(const uint32_t (&A)[S], const uint32_t (&B)[S], const uint32_t (&m)[S],
                                         uint32_t (&X)[2 * S], std::integer_sequence<int, Ks...>) {
  uint64_t acc = 0;
  ((acc += fbp_col<S, Ks>(A, B, m), X[Ks] = (uint32_t)acc & LMASK, acc >>= LB), ...);
}

template <int S>
__global__ __launch_bounds__(LANE_BLOCK) void k_pe1_fin(Pe1Params p) {
  constexpr int S2 = 2 * S;
  for (long long i = (long long)blockIdx.x * LANE_BLOCK + threadIdx.x; i < p.n; i += (long long)gridDim.x * LANE_BLOCK) {
    int64_t M = 0;
    int e = 0, st;
    const bool fixed = p.exp_mode != 0;
    if (p.dtype == 0) st = encode_float((double)((const float*)p.x)[i], fixed, p.fexp, M, e);
    else if (p.dtype == 1) st = encode_float(((const double*)p.x)[i], fixed, p.fexp, M, e);
    else st = encode_int(((const int64_t*)p.x)[i], fixed, p.fexp, M, e);
    uint32_t m[S], A[S], B[S], t[S], u[S];
#pragma unroll
    for (int j = 0; j < S; ++j) {
      m[j] = p.nl[j];
      A[j] = p.xw[(size_t)j * p.n + i];
      B[j] = p.xw[(size_t)(S + j) * p.n + i];
      t[j] = A[j];
    }
    const bool neg = M < 0;
    const uint64_t mag = neg ? (uint64_t)0 - (uint64_t)M : (uint64_t)M;
#pragma unroll
    for (int j = 0; j < S; ++j) {
      u[j] = j == 0 ? (uint32_t)mag & LMASK : j == 1 ? (uint32_t)(mag >> LB) & LMASK : j == 2 ? (uint32_t)(mag >> (2 * LB)) : 0u;
    }
    lane::mont_mul<S>(t, u, m, p.mprime);          // A |M| R^-1 (< 2n)
#pragma unroll
    for (int j = 0; j < S; ++j) u[j] = p.r2n[j];
    lane::mont_mul<S>(t, u, m, p.mprime);          // A |M| mod n (< 2n)
    lane::cond_sub<S>(t, m);
    {   // B' = B +- A |M| mod n
      uint32_t d[S];
      if (neg) {
        if (lane::sub<S>(B, t, d)) {               // B < A |M|: + n
          uint32_t c = 0;
#pragma unroll
          for (int j = 0; j < S; ++j) {
            const uint32_t v = d[j] + m[j] + c;
            d[j] = v & LMASK;
            c = v >> LB;
          }
        }
      } else {
        uint32_t c = 0;
#pragma unroll
        for (int j = 0; j < S; ++j) {
          const uint32_t v = B[j] + t[j] + c;
          d[j] = v & LMASK;
          c = v >> LB;
        }
        lane::cond_sub<S>(d, m);
      }
#pragma unroll
      for (int j = 0; j < S; ++j) B[j] = d[j];
    }
    // c = A + n B' (< n^2), limbs by product scanning, then 32-bit words
    uint32_t X[S2];
    pe1_cols<S>(A, B, m, X, std::make_integer_sequence<int, S2>{});
    pe1_words_out<S2>(X, p.ct + i * p.ct_words, p.ct_words, std::make_integer_sequence<int, 64>{});
    p.exp[i] = e;
    if (p.status) p.status[i] = st;
  }
}

}  // namespace fpai
