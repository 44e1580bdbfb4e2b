// Fixed-base obfuscation for key holders (device-RNG mode): the per-element factor r^n mod n^2 for a
// uniformly random unit r, sampled through the CRT components instead of through r itself.
//
// With n = p q, r^n mod p^2 depends only on r mod p, and r -> r^n mod p^2 maps the uniform
// distribution on Z_p* onto the uniform distribution on the subgroup H_p = <G_p>, G_p = g_p^n mod
// p^2, for g_p a generator of Z_p* (Z_p* is cyclic, so r = g_p^a with a uniform in [0, p-1)).
// Hence for independent uniform a_p, a_q the pair (G_p^a_p mod p^2, G_q^a_q mod q^2) has exactly the
// distribution of (r^n mod p^2, r^n mod q^2) for r uniform in Z_n* -- the reference's
// SystemRandom().randrange(1, n) (obfuscator.py:35) up to the 2^-1023 mass of non-units -- and the
// ciphertext c0 * CRT(.,.) is a Paillier encryption with the reference's randomizer distribution.
// a_h is taken from 8 (bits(p_h - 1) + 64) / 8 bits of ChaCha20 output (statistical distance 2^-64
// from uniform mod the group order), so the exponent never needs reducing.
//
// G^a = prod_k T_k[d_k] over the 8-bit digits d_k of a, T_k[d] = G^(d 2^(8k)) precomputed per key
// (k_fb_table): ~136 Montgomery products mod p_h^2 per half instead of ~1020 squarings mod p_h
// plus ~1020 mod p_h^2 on the generic-r path (kernels_crt.hpp) -- no squarings at all. The table
// rows stream from HBM/MALL through a double-buffered LDS-DMA prefetch (the next digit's row loads
// while the current product runs); the multiplier is read with ds_read_b128 in inline asm so the
// compiler does not order those reads behind the DMA in flight (it cannot tell the two LDS
// buffers apart).
#pragma once
#include "kernels_crt.hpp"

namespace fpai {

constexpr int FB_W = 8;                  // digit bits
constexpr int FB_ENT = 1 << FB_W;        // table entries per digit position
constexpr uint32_t FB_NONCE = 0x66786230u;   // ChaCha20 nonce word 2 (+ half) of the exponent stream
constexpr int FB_MAX_K = 192;            // digit positions (3 ChaCha blocks)

struct FbHalf {
  const uint4* table;      // [K][FB_ENT][TQ] quads: G^(d 2^(8k)) R mod p_h^2 (rows contiguous)
  const uint32_t* m;       // p_h^2, SB limbs
  const uint32_t* c1;      // CRT coefficient (q^2)^-1 mod p^2 (resp. (p^2)^-1 mod q^2), plain
  const uint32_t* gR;      // G_h R mod p_h^2 (table construction)
  const uint32_t* oneR;    // R mod p_h^2 (table construction)
  uint32_t mprime;
};

struct FbParams {
  const FbHalf* halves;    // [2]
  long long n;             // elements
  int K;                   // digit positions (exponent bits / 8)
  const uint4* digits;     // [2][DQ][n] (k_fb_digits), DQ = ceil(K / 16)
  uint32_t* out;           // u [2][SB][n]
};

struct FbDigitParams {
  long long n;
  uint32_t rng_key[8];
  unsigned long long index_base;
  int K;
  uint4* digits;           // [2][DQ][n]
};

// Exponent digits of both halves: ChaCha20 blocks 0.. of nonce (global index, FB_NONCE + half),
// byte k = digit k (a_h = the little-endian integer of the first K bytes). A kernel of its own:
// the key schedule's registers would otherwise push the modulus out of the SGPRs of k_fb.
template <int W = FB_W>   // (a template only so the header can be included by several units)
__global__ __launch_bounds__(LANE_BLOCK) void k_fb_digits(FbDigitParams p) {
  const int half = blockIdx.y;
  const int DQ = (p.K + 15) / 16;
  for (long long i = (long long)blockIdx.x * LANE_BLOCK + threadIdx.x; i < p.n; i += (long long)gridDim.x * LANE_BLOCK) {
    const unsigned long long g = p.index_base + (unsigned long long)i;
    for (int b = 0; b * 4 < DQ; ++b) {
      uint32_t blk[16];
      chacha20_block(p.rng_key, (uint32_t)b, (uint32_t)g, (uint32_t)(g >> 32), FB_NONCE + (uint32_t)half, blk);
#pragma unroll
      for (int w = 0; w < 4; ++w)
        if (b * 4 + w < DQ)
          p.digits[((size_t)half * DQ + b * 4 + w) * p.n + i] =
              make_uint4(blk[4 * w], blk[4 * w + 1], blk[4 * w + 2], blk[4 * w + 3]);
    }
  }
}

typedef uint32_t fb_v4u __attribute__((ext_vector_type(4)));

// LDS quad read the compiler does not track (see header): 16-bit byte offset per instruction
template <int OFF>
__device__ __forceinline__ fb_v4u lds_read_quad(uint32_t addr) {
  fb_v4u v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF) : "memory");
  return v;
}
__device__ __forceinline__ void lds_quad_wait(fb_v4u& v) { asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v)); }

// a <- a b R^-1 mod m, b = the LDS quad column at byte address `addr` (quad g at addr + g*4096)
template <int S, int J>
__device__ __forceinline__ void fb_step(uint64_t (&P)[S], const uint32_t (&a)[S], fb_v4u& cur, fb_v4u& nxt,
                                        uint32_t addr, const uint32_t (&m)[S], uint32_t mprime) {
  constexpr int TQ = (S + 3) / 4;
  if constexpr (J % 4 == 0) {
    lds_quad_wait(nxt);
    cur = nxt;
    constexpr int g = J / 4 + 1;
    if constexpr (g < TQ) {
      if constexpr (g < 16) nxt = lds_read_quad<g * LANE_BLOCK * 16>(addr);
      else nxt = lds_read_quad<(g - 16) * LANE_BLOCK * 16>(addr + 16 * LANE_BLOCK * 16);
    }
  }
  const uint32_t bj = cur[J % 4];
#pragma unroll
  for (int i = 0; i < S; ++i) P[(i + J) % S] += (uint64_t)a[i] * bj;
  lane::reduce_step<S, J>(P, m, mprime);
}
template <int S, int... Js>
__device__ __forceinline__ void fb_mul_all(uint64_t (&P)[S], const uint32_t (&a)[S], uint32_t addr, const uint32_t (&m)[S],
                                           uint32_t mprime, std::integer_sequence<int, Js...>) {
  fb_v4u cur, nxt = lds_read_quad<0>(addr);
  (fb_step<S, Js>(P, a, cur, nxt, addr, m, mprime), ...);
}
template <int S>
__device__ __forceinline__ void fb_mont_mul(uint32_t (&a)[S], uint32_t addr, const uint32_t (&m)[S], uint32_t mprime) {
  uint64_t P[S];
#pragma unroll
  for (int i = 0; i < S; ++i) P[i] = 0;
  fb_mul_all<S>(P, a, addr, m, mprime, std::make_integer_sequence<int, S>{});
  lane::normalize<S>(P, a);
}

// digit k of the staged exponent (quad k/16 of the lane scratch holds digits 16(k/16) ..)
__device__ __forceinline__ uint32_t fb_digit(const uint4 dq, int k) {
  const int c = (k >> 2) & 3;
  const uint32_t w = c == 0 ? dq.x : c == 1 ? dq.y : c == 2 ? dq.z : dq.w;
  return (w >> (8 * (k & 3))) & 0xFFu;
}

// DMA table row (k, d) -> LDS buffer (the wave's 64-lane slice of each quad row)
template <int S>
__device__ __forceinline__ void fb_row_to_lds(const uint4* __restrict__ table, int k, uint32_t d, uint4* wave_row0) {
  constexpr int TQ = tile_quads<S>();
  const uint4* row = table + ((size_t)k * FB_ENT + d) * TQ;   // quad g at an immediate offset
#pragma unroll
  for (int g = 0; g < TQ; ++g)
    __builtin_amdgcn_global_load_lds((const void*)(row + g),
                                     (__attribute__((address_space(3))) void*)(wave_row0 + g * LANE_BLOCK), 16, 0, 0);
}

template <int SB>
__global__ __launch_bounds__(LANE_BLOCK, 1) void k_fb(FbParams p) {
  constexpr int TQ = tile_quads<SB>();
  __shared__ uint4 lbuf[2 * TQ * LANE_BLOCK];
  const int half = blockIdx.y;
  const FbHalf* H = p.halves + half;
  uint32_t m[SB];
#pragma unroll
  for (int j = 0; j < SB; ++j) m[j] = H->m[j];
  const uint32_t mprime = H->mprime;
  const uint4* table = H->table;
  const int K = p.K;
  const int DQ = (K + 15) / 16;
  uint4* brow[2] = {lbuf + (threadIdx.x & ~63u), lbuf + TQ * LANE_BLOCK + (threadIdx.x & ~63u)};
  typedef __attribute__((address_space(3))) uint4 lds_uint4;
  const uint32_t addr0 = (uint32_t)(size_t)(lds_uint4*)(lbuf + threadIdx.x);                   // LDS byte offsets
  const uint32_t addr1 = (uint32_t)(size_t)(lds_uint4*)(lbuf + TQ * LANE_BLOCK + threadIdx.x);
  for (long long base = (long long)blockIdx.x * LANE_BLOCK; base < p.n; base += (long long)gridDim.x * LANE_BLOCK) {
    const long long i = base + threadIdx.x;
    const long long ii = i < p.n ? i : p.n - 1;
    const uint4* dg = p.digits + (size_t)half * DQ * p.n + ii;   // quad q at dg[q * n]
    uint4 dq = dg[0];
    // a = T_0[d_0] (Montgomery form)
    uint32_t a[SB];
    {
      const uint32_t d0 = fb_digit(dq, 0);
#pragma unroll
      for (int g = 0; g < TQ; ++g) unpack_quad<SB>(table[(size_t)d0 * TQ + g], g, a);
#pragma unroll
      for (int j = 0; j < SB; ++j) asm volatile("" : "+v"(a[j]));   // loads complete before any DMA
    }
    fb_row_to_lds<SB>(table, 1, fb_digit(dq, 1), brow[0]);
    for (int k = 1; k < K; ++k) {
      lds_dma_wait();                                   // row k landed in buffer (k-1)&1
      if (k + 1 < K) {
        if (((k + 1) & 15) == 0) {
          dq = dg[(size_t)((k + 1) >> 4) * p.n];
          asm volatile("" : "+v"(dq.x), "+v"(dq.y), "+v"(dq.z), "+v"(dq.w));
        }
        fb_row_to_lds<SB>(table, k + 1, fb_digit(dq, k + 1), brow[k & 1]);
      }
      fb_mont_mul<SB>(a, (k & 1) ? addr0 : addr1, m, mprime);
    }
    // u_h = G^a * coef (leaves the Montgomery domain); no DMA is in flight and every read of
    // either buffer has completed, so buffer K&1 takes the coefficient
    {
      uint4* col = (K & 1) ? lbuf + TQ * LANE_BLOCK + threadIdx.x : lbuf + threadIdx.x;
      uint32_t cv[SB];
#pragma unroll
      for (int j = 0; j < SB; ++j) cv[j] = H->c1[j];
#pragma unroll
      for (int g = 0; g < TQ; ++g) col[g * LANE_BLOCK] = pack_quad<SB>(cv, g);
      fb_mont_mul<SB>(a, (K & 1) ? addr1 : addr0, m, mprime);
    }
    if (i < p.n) {
#pragma unroll
      for (int j = 0; j < SB; ++j) p.out[((size_t)half * SB + j) * p.n + i] = a[j];
    }
  }
}

// ---------------------------------------------------------------- per-key table: T_k[d] = G^(d 2^(8k)) R
// One block per (digit position k, half); lane d. acc = G~^d (8 steps), then 8k squarings.
template <int SB>
__global__ __launch_bounds__(LANE_BLOCK) void k_fb_table(const FbHalf* halves, uint4* table0, uint4* table1, int K) {
  constexpr int TQ = tile_quads<SB>();
  const int k = blockIdx.x, half = blockIdx.y;
  const FbHalf* H = halves + half;
  uint4* table = half ? table1 : table0;
  const uint32_t d = threadIdx.x;
  uint32_t m[SB], x[SB], acc[SB];
#pragma unroll
  for (int j = 0; j < SB; ++j) {
    m[j] = H->m[j];
    x[j] = H->gR[j];
    acc[j] = H->oneR[j];
  }
  for (int b = FB_W - 1; b >= 0; --b) {
    lane::mont_sqr<SB>(acc, m, H->mprime);
    if ((d >> b) & 1u) lane::mont_mul<SB>(acc, x, m, H->mprime);
  }
  for (int s = 0; s < FB_W * k; ++s) lane::mont_sqr<SB>(acc, m, H->mprime);
  lane::cond_sub<SB>(acc, m);
#pragma unroll
  for (int g = 0; g < TQ; ++g) table[((size_t)k * FB_ENT + d) * TQ + g] = pack_quad<SB>(acc, g);
}

}  // namespace fpai
