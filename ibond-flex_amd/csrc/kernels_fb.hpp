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
// G^a = prod_k T_k[d_k] over the W-bit digits d_k of a, T_k[d] = G^(d 2^(W k)) precomputed per key
// (k_fb_lohi + k_fb_fill): ceil(1088 / W) Montgomery products mod p_h^2 per half for a 2048-bit key
// (136 at W = 8, 68 at W = 16) instead of ~1020 squarings mod p_h plus ~1020 mod p_h^2 on the
// generic-r path (kernels_crt.hpp) -- no squarings at all. W trades table size (K 2^W rows of
// 16 TQ bytes: 21 MB per half at W = 8, 1.35 GB at W = 16, resident in HBM) for products. The table
// rows stream from HBM/MALL through a double-buffered LDS-DMA prefetch (the next digit's row loads
// while the current product runs); the multiplier is read with ds_read_b128 in inline asm so the
// compiler does not order those reads behind the DMA in flight (it cannot tell the two LDS
// buffers apart).
#pragma once
#include "kernels_crt.hpp"

namespace fpai {

constexpr uint32_t FB_NONCE = 0x66786230u;   // ChaCha20 nonce word 2 (+ half) of the exponent stream
constexpr int FB_MAX_WORDS = 48;             // exponent words per element (3 ChaCha blocks): K W <= 1536
constexpr int FB_LO = 1024;                  // entries of the per-position small tables (k_fb_lohi): W <= 20

struct FbHalf {
  const uint4* table;      // [K][2^W][TQ] quads: G^(d 2^(W k)) R mod p_h^2, canonical (rows contiguous)
  const uint32_t* m;       // p_h^2, SB limbs
  const uint32_t* c1;      // CRT coefficient (q^2)^-1 mod p^2 (resp. (p^2)^-1 mod q^2), plain
  const uint32_t* R2;      // R^2 mod p_h^2 (table construction)
  const uint32_t* oneR;    // R mod p_h^2 (table construction)
  const uint32_t* bases;   // [K][SB] B_k = G^(2^(W k)) mod p_h^2, plain (table construction)
  uint32_t* lohi;          // [K][2][FB_LO][SB] scratch of the table construction
  uint32_t mprime;
};

struct FbParams {
  const FbHalf* halves;    // [2]
  long long n;             // elements
  int K, W;                // digit positions, digit bits
  const uint32_t* digits;  // [2][K][n] (k_fb_digits)
  uint32_t* out;           // u [2][SB][n]
};

struct FbDigitParams {
  long long n;
  uint32_t rng_key[8];
  unsigned long long index_base;
  int K, W;
  uint32_t* digits;        // [2][K][n]
};

// Exponent digits of both halves: a_h = the first K W bits (little-endian) of the ChaCha20 stream
// of nonce (global index, FB_NONCE + half), counter 0..; digit k = bits [k W, (k+1) W). A kernel of
// its own: the key schedule's registers would otherwise push the modulus out of the SGPRs of k_fb.
// Each lane stages its stream words in its own LDS row and extracts the digits from there.
template <int DUMMY = 0>   // (a template only so the header can be included by several units)
__global__ __launch_bounds__(LANE_BLOCK) void k_fb_digits(FbDigitParams p) {
  __shared__ uint32_t wb[LANE_BLOCK * (FB_MAX_WORDS + 1)];
  uint32_t* my = wb + threadIdx.x * (FB_MAX_WORDS + 1);
  const int half = blockIdx.y;
  const int nbits = p.K * p.W;
  const int nblk = (nbits + 511) / 512;
  const uint32_t mask = (1u << p.W) - 1u;
  for (long long i = (long long)blockIdx.x * LANE_BLOCK + threadIdx.x; i < p.n; i += (long long)gridDim.x * LANE_BLOCK) {
    const unsigned long long g = p.index_base + (unsigned long long)i;
    for (int b = 0; b < nblk; ++b) {
      uint32_t blk[16];
      chacha20_block(p.rng_key, (uint32_t)b, (uint32_t)g, (uint32_t)(g >> 32), FB_NONCE + (uint32_t)half, blk);
#pragma unroll
      for (int w = 0; w < 16; ++w) my[16 * b + w] = blk[w];
    }
    my[16 * nblk] = 0u;
    for (int k = 0; k < p.K; ++k) {
      const int bit = k * p.W, wi = bit >> 5, sh = bit & 31;
      const uint64_t v = (((uint64_t)my[wi + 1] << 32) | my[wi]) >> sh;
      p.digits[((size_t)half * p.K + k) * p.n + i] = (uint32_t)(v & mask);
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

// DMA table row `row` -> LDS buffer (the wave's 64-lane slice of each quad row)
template <int S>
__device__ __forceinline__ void fb_row_to_lds(const uint4* __restrict__ table, size_t row, uint4* wave_row0) {
  constexpr int TQ = tile_quads<S>();
  const uint4* r = table + row * TQ;   // quad g at an immediate offset
#pragma unroll
  for (int g = 0; g < TQ; ++g)
    __builtin_amdgcn_global_load_lds((const void*)(r + g),
                                     (__attribute__((address_space(3))) void*)(wave_row0 + g * LANE_BLOCK), 16, 0, 0);
}

// One LDS row buffer per wave (78 KB per 4-wave block): two blocks -- two waves per SIMD -- fit a CU,
// so a wave waiting for its next table row is covered by the other wave's product instead of by a
// second buffer (which would hold the CU to one wave per SIMD: measured 18 % wait cycles).
template <int SB>
__global__ __launch_bounds__(LANE_BLOCK, 2) void k_fb(FbParams p) {
  constexpr int TQ = tile_quads<SB>();
  __shared__ uint4 lbuf[TQ * LANE_BLOCK];
  const int half = blockIdx.y;
  const FbHalf* H = p.halves + half;
  uint32_t m[SB];
#pragma unroll
  for (int j = 0; j < SB; ++j) m[j] = H->m[j];
  const uint32_t mprime = H->mprime;
  const uint4* table = H->table;
  const int K = p.K, W = p.W;
  uint4* brow = lbuf + (threadIdx.x & ~63u);
  typedef __attribute__((address_space(3))) uint4 lds_uint4;
  const uint32_t addr0 = (uint32_t)(size_t)(lds_uint4*)(lbuf + threadIdx.x);                   // LDS byte offset
  for (long long base = (long long)blockIdx.x * LANE_BLOCK; base < p.n; base += (long long)gridDim.x * LANE_BLOCK) {
    const long long i = base + threadIdx.x;
    const long long ii = i < p.n ? i : p.n - 1;
    const uint32_t* dg = p.digits + (size_t)half * K * p.n + ii;   // digit k at dg[k * n]
    // a = T_0[d_0] (Montgomery form)
    uint32_t a[SB];
    {
      const uint32_t d0 = dg[0];
#pragma unroll
      for (int g = 0; g < TQ; ++g) unpack_quad<SB>(table[(size_t)d0 * TQ + g], g, a);
#pragma unroll
      for (int j = 0; j < SB; ++j) asm volatile("" : "+v"(a[j]));   // loads complete before any DMA
    }
    uint32_t dn = dg[p.n];                                 // digit 1
    asm volatile("" : "+v"(dn));
    uint32_t dn2 = K > 2 ? dg[2 * p.n] : 0u;               // digit 2, in flight
    fb_row_to_lds<SB>(table, ((size_t)1 << W) + dn, brow);
    for (int k = 1; k < K; ++k) {
      lds_dma_wait();                                   // row k landed, digit k+1 loaded
      fb_mont_mul<SB>(a, addr0, m, mprime);             // every read of the row completes inside
      if (k + 1 < K) {
        const uint32_t dk1 = dn2;
        if (k + 2 < K) dn2 = dg[(size_t)(k + 2) * p.n];
        fb_row_to_lds<SB>(table, ((size_t)(k + 1) << W) + dk1, brow);
      }
    }
    // u_h = G^a * coef (leaves the Montgomery domain); no DMA is in flight and every read of the
    // buffer has completed, so it takes the coefficient
    {
      uint4* col = lbuf + threadIdx.x;
      uint32_t cv[SB];
#pragma unroll
      for (int j = 0; j < SB; ++j) cv[j] = H->c1[j];
#pragma unroll
      for (int g = 0; g < TQ; ++g) col[g * LANE_BLOCK] = pack_quad<SB>(cv, g);
      fb_mont_mul<SB>(a, addr0, m, mprime);
    }
    if (i < p.n) {
#pragma unroll
      for (int j = 0; j < SB; ++j) p.out[((size_t)half * SB + j) * p.n + i] = a[j];
    }
  }
}

// ---------------------------------------------------------------- per-key table: T_k[d] = G^(d 2^(W k)) R
// Two levels: k_fb_lohi builds, per position k, lo[j] = B_k^j (j < 2^LO) and hi[j] = B_k^(2^LO j)
// (j < 2^(W-LO)), LO = W/2, with B_k = G^(2^(W k)) from the host; k_fb_fill forms each of the 2^W
// entries with ONE product hi[d >> LO] * lo[d & (2^LO - 1)]. (~3 ms for both 1.35 GB tables at W = 16.)
template <int SB>
__global__ __launch_bounds__(LANE_BLOCK) void k_fb_lohi(const FbHalf* halves, int K, int W) {
  const int k = blockIdx.x, half = blockIdx.y;
  const FbHalf* H = halves + half;
  const int LO = W / 2, HI = W - LO;
  uint32_t m[SB], x[SB], t[SB], acc[SB];
#pragma unroll
  for (int i = 0; i < SB; ++i) {
    m[i] = H->m[i];
    x[i] = H->bases[(size_t)k * SB + i];
    t[i] = H->R2[i];
  }
  lane::mont_mul<SB>(x, t, m, H->mprime);            // B_k R
  for (int s = 0; s < 2; ++s) {
    const int bits = s ? HI : LO;
    if (s == 1)
      for (int q = 0; q < LO; ++q) lane::mont_sqr<SB>(x, m, H->mprime);   // B_k^(2^LO) R
    for (uint32_t j = threadIdx.x; j < (1u << bits); j += blockDim.x) {
#pragma unroll
      for (int i = 0; i < SB; ++i) acc[i] = H->oneR[i];
      for (int b = bits - 1; b >= 0; --b) {
        lane::mont_sqr<SB>(acc, m, H->mprime);
        if ((j >> b) & 1u) lane::mont_mul<SB>(acc, x, m, H->mprime);
      }
      uint32_t* o = H->lohi + (((size_t)k * 2 + s) * FB_LO + j) * SB;
#pragma unroll
      for (int i = 0; i < SB; ++i) o[i] = acc[i];
    }
  }
}

template <int SB>
__global__ __launch_bounds__(LANE_BLOCK) void k_fb_fill(const FbHalf* halves, int K, int W, uint4* table0, uint4* table1) {
  constexpr int TQ = tile_quads<SB>();
  const int ent = 1 << W;
  const int per = (ent + LANE_BLOCK - 1) / LANE_BLOCK;
  const int k = blockIdx.x / per;
  const int d = (blockIdx.x % per) * LANE_BLOCK + threadIdx.x;
  if (d >= ent) return;
  const int half = blockIdx.y;
  const FbHalf* H = halves + half;
  uint4* table = half ? table1 : table0;
  const int LO = W / 2;
  const uint32_t* lo = H->lohi + (((size_t)k * 2 + 0) * FB_LO + (d & ((1 << LO) - 1))) * SB;
  const uint32_t* hi = H->lohi + (((size_t)k * 2 + 1) * FB_LO + (d >> LO)) * SB;
  uint32_t m[SB], a[SB], b[SB];
#pragma unroll
  for (int i = 0; i < SB; ++i) {
    m[i] = H->m[i];
    a[i] = lo[i];
    b[i] = hi[i];
  }
  lane::mont_mul<SB>(a, b, m, H->mprime);
  lane::cond_sub<SB>(a, m);
#pragma unroll
  for (int g = 0; g < TQ; ++g) table[((size_t)k * ent + d) * TQ + g] = pack_quad<SB>(a, g);
}

}  // namespace fpai
