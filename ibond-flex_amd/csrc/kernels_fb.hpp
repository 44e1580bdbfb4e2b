// Fixed-base obfuscation for key holders (device-RNG mode): the per-element factor r^n mod n^2 for a
// uniformly random unit r, sampled through the CRT components instead of through r itself.
//
// With n = p q, r^n mod p^2 depends only on r mod p, and r -> r^n mod p^2 maps the uniform
// distribution on Z_p* onto the uniform distribution on the subgroup H_p = <G_p>, G_p = g_p^n mod
// p^2, for g_p a generator of Z_p* (Z_p* is cyclic, so r = g_p^a with a uniform mod p - 1).
// Hence for independent uniform a_p, a_q the pair (G_p^a_p mod p^2, G_q^a_q mod q^2) has the
// distribution of (r^n mod p^2, r^n mod q^2) for r uniform in Z_n* -- the reference's
// SystemRandom().randrange(1, n) (obfuscator.py:35) up to the 2^-1023 mass of non-units -- and it IS
// r^n for the explicit obfuscator r = CRT(g_p^a_p mod p, g_q^a_q mod q), so the ciphertext equals the
// reference's pe.encrypt(x, random_value=r) bit for bit (tests/golden/make_golden_fb.py).
//
// a_h = raw_h mod (p_h - 1): raw_h is the first raw_bits = max bits(p_h - 1) + 64 bits of a ChaCha20
// stream (statistical distance 2^-64 from uniform), reduced on the device by Barrett (k_fb_digits),
// then cut into K = ceil(bits(p_h - 1) / W) W-bit digits. G^a = prod_k T_k[d_k] with T_k[d] =
// G^(d 2^(W k)) precomputed once per key (k_fb_lohi + k_fb_fill): for a 2048-bit key 52 Montgomery
// products mod p_h^2 per half at W = 20 (64 at W = 16) and no squarings, against ~1020 squarings mod
// p_h plus ~1020 mod p_h^2 on the generic-r path (kernels_crt.hpp). The tables are resident in HBM
// (2 halves x K 2^W rows x 256 B: 27 GB at W = 20, 2.1 GB at W = 16); rows are 32-bit words of the
// canonical value (256 B = two 128-B lines for a 2048-bit key), converted to 28-bit limbs while the
// product reads them.
//
// Per element and half, k_fb computes c0 G_h^a_h mod p_h^2 with c0 = 1 + n M (raw_encrypt.py:44-45):
// the first product takes the UNREDUCED multiple-of-n sum 1 + sum_c (n 2^(CB c) mod p_h^2) |M|_c
// (< 2^(28 SB - 6), so the CIOS bound a b / R < p_h^2 still holds) as its A operand and row T_0[d_0]
// as B, which leaves the Montgomery domain at once; every later product multiplies by a Montgomery-
// form row and keeps the plain domain. k_fb_fin recombines the halves by Garner:
//   c = w_q + q^2 ((w_p - w_q) (q^2)^-1 mod p^2)     (< n^2; gmpy_math.crt, gmpy_math.py:31-40)
// with one Montgomery product mod p^2 and one plain product, streamed to the ciphertext words.
//
// The table rows stream from HBM into LDS by DMA (global_load_lds) one digit ahead; the product reads
// them with ds_read_b32 in inline asm so the compiler does not order those reads behind the DMA in
// flight (it cannot tell the LDS buffer's two uses apart).
#pragma once
#include "kernels_crt.hpp"
#include "guard.hpp"

namespace fpai {

constexpr uint32_t FB_NONCE = 0x66786230u;   // ChaCha20 nonce word 2 (+ half) of the exponent stream
constexpr int FB_RAW_MAX = 80;               // words of the raw exponent per element (5 ChaCha blocks)
constexpr int FB_DIG_BLOCK = 128;            // threads per block of k_fb_digits
constexpr int FB_LO = 4096;
#ifndef FPAI_FB_NBUF
#define FPAI_FB_NBUF 1                       // k_fb row buffers: 1 (two waves per SIMD) or 2 (one wave, in-wave prefetch)
#endif                  // entries of the per-position small tables (k_fb_lohi): W <= 24

// Compile-time geometry per lane size SB (limbs of p_h^2): TW = 32-bit words per table row (the
// canonical values are < p_h^2 < 2^(32 TW)); c0 = 1 + n M is folded in as NC chunks of CB bits of |M|,
// and negative M through the offset 2^PB p_h^2 (> the chunk sum, < 2^(28 SB - 4)).
template <int SB>
struct FbGeom;
template <>
struct FbGeom<37> {
  static constexpr int TW = 32, CB = 4, NC = 16, PB = 10;
};
template <>
struct FbGeom<74> {
  static constexpr int TW = 64, CB = 16, NC = 4, PB = 20;
};

struct FbRed {             // Barrett reduction of the raw exponent modulo D_h = p_h - 1 (HAC 14.42, b = 2)
  uint32_t D[FB_RAW_MAX];  // D_h, little-endian words
  uint32_t mu[4];          // floor(2^raw_bits / D_h) (< 2^(raw_bits - kbits + 1) <= 2^66)
  int dwords, kbits;       // words and bits of D_h
  int pad[2];
};

struct FbHalf {
  const uint4* table;      // [K][2^W][TW/4] quads: 32-bit words of T_k[d] = G^(d 2^(W k)) R mod p_h^2
  const uint32_t* m;       // p_h^2, SB limbs
  const uint32_t* R2;      // R^2 mod p_h^2 (table construction)
  const uint32_t* oneR;    // R mod p_h^2 (table construction)
  const uint32_t* bases;   // [K][SB] B_k = G^(2^(W k)) mod p_h^2, plain (table construction)
  uint32_t* lohi;          // [K][2][FB_LO][SB] scratch of the table construction
  const uint32_t* nm;      // [NC][SB] n 2^(CB c) mod p_h^2 (c0 folding)
  const uint32_t* pbig;    // [SB] 2^PB p_h^2
  uint32_t mprime;
};

struct FbParams {
  const FbHalf* halves;    // [2]
  long long n;             // elements
  int K, W;                // digit positions, digit bits
  const uint32_t* digits;  // [2][K][n] (k_fb_digits)
  uint32_t* out;           // w [2][SB][n]: c0 G_h^a_h mod p_h^2 (< 2 p_h^2)
  const void* x;           // plaintexts (encode: fixedpoint_number.py:46-90)
  int dtype, exp_mode, fexp;
  int32_t* exp;            // written by the p-half
  int32_t* status;         // nullable
};

struct FbDigitParams {
  long long n;
  uint32_t rng_key[8];
  unsigned long long index_base;
  int K, W, raw_bits;
  const FbRed* red;        // [2]
  uint32_t* digits;        // [2][K][n]
  GuardArgs g;             // test build: digits = 2 K n
};

struct FbFinParams {
  const uint32_t* w;       // [2][SB][n] (k_fb)
  long long n;
  const uint32_t* m;       // p^2 (SB limbs)
  const uint32_t* m8;      // 8 p^2
  const uint32_t* coefR;   // (q^2)^-1 R mod p^2
  const uint32_t* q2;      // q^2
  uint32_t mprime;         // of p^2
  uint32_t* ct;
  int ct_words;
};

// ---------------------------------------------------------------- exponent digits
// Each lane stages its raw stream in its own LDS row (odd stride: conflict-free), reduces it modulo
// D_h in place and extracts the digits. A kernel of its own: the ChaCha key schedule's registers would
// otherwise push the modulus out of the SGPRs of k_fb.
// ROW (odd, >= raw words + 3): LDS words per lane, sized to the key (21 / 37 / 69 at nb = 1024 / 2048 / 4096) so
// that the LDS of a block does not cap the occupancy (the 83-word rows of every key size allowed 1.5 waves per SIMD).
// the per-key constants of the digit extraction, read once per kernel
struct FbDigitKey {
  const FbRed* R;
  int rb, rw, nblk, dw, kb;
  uint32_t mask, mu0, mu1, mu2;
};
__device__ __forceinline__ FbDigitKey fb_digit_key(const FbDigitParams& p, int half) {
  FbDigitKey k;
  k.R = p.red + half;
  k.rb = p.raw_bits;
  k.rw = (k.rb + 31) / 32;
  k.nblk = (k.rw + 15) / 16;
  k.dw = k.R->dwords;
  k.kb = k.R->kbits;
  k.mask = (1u << p.W) - 1u;
  k.mu0 = k.R->mu[0];
  k.mu1 = k.R->mu[1];
  k.mu2 = k.R->mu[2];
  return k;
}

// element i of half `half`: its raw stream staged in the LDS row a (ROW words), reduced modulo D_h in place, cut into
// the K digits (k_fb_digits; and, in a measurement build, k_fbs's prologue, kernels_fbs.hpp FBS_AB & 4)
template <int ROW>
__device__ __forceinline__ void fb_digits_elem(const FbDigitParams& p, const FbDigitKey& dk, int half, long long i, uint32_t* a) {
  const FbRed* R = dk.R;
  const int rb = dk.rb, rw = dk.rw, nblk = dk.nblk, dw = dk.dw, kb = dk.kb;
  const uint32_t mask = dk.mask;
  {
    const unsigned long long g = p.index_base + (unsigned long long)i;
    for (int b = 0; b < nblk; ++b) {
      uint32_t blk[16];
      chacha20_block(p.rng_key, (uint32_t)b, (uint32_t)g, (uint32_t)(g >> 32), FB_NONCE + (uint32_t)half, blk);
#pragma unroll
      for (int w = 0; w < 16; ++w)
        if (16 * b + w < rw) a[16 * b + w] = blk[w];   // (the last block's tail would run into the next lane's row)
    }
    if (rb & 31) a[rw - 1] &= (1u << (rb & 31)) - 1u;
    for (int w = rw; w < ROW; ++w) a[w] = 0u;
    // q^ = floor(floor(a / 2^(k-1)) mu / 2^(raw_bits - k + 1)), q - 2 <= q^ <= q
    uint32_t q1[3];
    {
      const int s = kb - 1, ws = s >> 5, sh = s & 31;
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const uint64_t v = ((uint64_t)a[ws + t + 1] << 32) | a[ws + t];
        q1[t] = (uint32_t)(v >> sh);
      }
    }
    uint32_t q2[7] = {0u, 0u, 0u, 0u, 0u, 0u, 0u};
    {
      const uint32_t mu[3] = {dk.mu0, dk.mu1, dk.mu2};
#pragma unroll
      for (int x = 0; x < 3; ++x) {
        uint64_t c = 0;
#pragma unroll
        for (int y = 0; y < 3; ++y) {
          const uint64_t t = (uint64_t)q1[x] * mu[y] + q2[x + y] + c;
          q2[x + y] = (uint32_t)t;
          c = t >> 32;
        }
        q2[x + 3] = (uint32_t)c;
      }
    }
    uint32_t qh[3];
    {
      const int s = rb - kb + 1, ws = s >> 5, sh = s & 31;
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const uint64_t v = ((uint64_t)q2[ws + t + 1] << 32) | q2[ws + t];
        qh[t] = (uint32_t)(v >> sh);
      }
    }
    // a -= q^ D (word t of q^ at a time; every partial difference stays >= a - q^ D >= 0)
    for (int t = 0; t < 3; ++t) {
      uint64_t mc = 0;
      int64_t br = 0;
      int j = 0;
      for (; j < dw; ++j) {
        const uint64_t pr = (uint64_t)qh[t] * R->D[j] + mc;
        mc = pr >> 32;
        const int64_t v = (int64_t)a[j + t] - (int64_t)(uint32_t)pr + br;
        a[j + t] = (uint32_t)v;
        br = v >> 32;
      }
      for (j += t; j < ROW; ++j) {
        const int64_t v = (int64_t)a[j] - (int64_t)mc + br;
        mc = 0;
        a[j] = (uint32_t)v;
        br = v >> 32;
      }
    }
    // at most two conditional subtractions of D
    for (int rep = 0; rep < 2; ++rep) {
      bool ge = a[dw] != 0u;
      if (!ge) {
        int j = dw - 1;
        while (j > 0 && a[j] == R->D[j]) --j;
        ge = a[j] >= R->D[j];
      }
      if (ge) {
        int64_t br = 0;
        for (int j = 0; j <= dw; ++j) {
          const int64_t v = (int64_t)a[j] - (int64_t)(j < dw ? R->D[j] : 0u) + br;
          a[j] = (uint32_t)v;
          br = v >> 32;
        }
      }
    }
    for (int k = 0; k < p.K; ++k) {
      const int bit = k * p.W, wi = bit >> 5, sh = bit & 31;
      const uint64_t v = (((uint64_t)a[wi + 1] << 32) | a[wi]) >> sh;
      p.digits[FPAI_GUARD_IDX(p.g, GS_DIG_OUT, ((size_t)half * p.K + k) * p.n + i, p.g.digits, i)] = (uint32_t)(v & mask);
    }
  }
}

template <int ROW>
__global__ __launch_bounds__(FB_DIG_BLOCK) void k_fb_digits(FbDigitParams p) {
  static_assert(ROW % 2 == 1 && ROW <= FB_RAW_MAX + 3, "row");
  __shared__ uint32_t wb[FB_DIG_BLOCK * ROW];
  uint32_t* a = wb + threadIdx.x * ROW;
  const int half = blockIdx.y;
  const FbDigitKey dk = fb_digit_key(p, half);
  for (long long i = (long long)blockIdx.x * FB_DIG_BLOCK + threadIdx.x; i < p.n; i += (long long)gridDim.x * FB_DIG_BLOCK)
    fb_digits_elem<ROW>(p, dk, half, i, a);
}

// ---------------------------------------------------------------- products with a word row in LDS
// LDS word read the compiler does not track (see header): 16-bit byte offset per instruction
template <int OFF>
__device__ __forceinline__ uint32_t lds_read_word(uint32_t addr) {
  uint32_t v;
  asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF) : "memory");
  return v;
}
// word WI of this lane's row in the [quad][lane] buffer, 0 past the row
template <int TW, int WI>
__device__ __forceinline__ uint32_t fb_rd(uint32_t addr) {
  if constexpr (WI < TW) return lds_read_word<(WI / 4) * LANE_BLOCK * 16 + (WI % 4) * 4>(addr);
  else return 0u;
}
// limbs 8G .. 8G+7 (224 bits) are exactly words 7G .. 7G+6
template <int TW, int G>
__device__ __forceinline__ void fb_group_read(uint32_t (&w)[7], uint32_t addr) {
  w[0] = fb_rd<TW, 7 * G + 0>(addr);
  w[1] = fb_rd<TW, 7 * G + 1>(addr);
  w[2] = fb_rd<TW, 7 * G + 2>(addr);
  w[3] = fb_rd<TW, 7 * G + 3>(addr);
  w[4] = fb_rd<TW, 7 * G + 4>(addr);
  w[5] = fb_rd<TW, 7 * G + 5>(addr);
  w[6] = fb_rd<TW, 7 * G + 6>(addr);
}
__device__ __forceinline__ void fb_group_wait(uint32_t (&w)[7]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(w[4]), "+v"(w[5]), "+v"(w[6]));
}
// 28-bit limb R (0..7) of a group of 7 words
template <int R>
__device__ __forceinline__ uint32_t fb_limb(const uint32_t (&w)[7]) {
  constexpr int bit = 28 * R, wi = bit >> 5, sh = bit & 31;
  if constexpr (sh == 0) return w[wi] & lane::LMASK;
  else if constexpr (sh + 28 <= 32) return w[wi] >> sh;
  else return __builtin_amdgcn_alignbit(w[wi + 1], w[wi], sh) & lane::LMASK;
}

template <int S, int TW, int J>
__device__ __forceinline__ void fbw_step(uint64_t (&P)[S], const uint32_t (&a)[S], uint32_t (&cur)[7],
                                         uint32_t (&nxt)[7], uint32_t addr, const uint32_t (&m)[S], uint32_t mprime) {
  if constexpr (J % 8 == 0) {
    fb_group_wait(nxt);
#pragma unroll
    for (int t = 0; t < 7; ++t) cur[t] = nxt[t];
    constexpr int G = J / 8 + 1;
    if constexpr (8 * G < S) fb_group_read<TW, G>(nxt, addr);
  }
  const uint32_t bj = fb_limb<J % 8>(cur);
#pragma unroll
  for (int i = 0; i < S; ++i) P[(i + J) % S] += (uint64_t)a[i] * bj;
  lane::reduce_step<S, J>(P, m, mprime);
}
template <int S, int TW, int... Js>
__device__ __forceinline__ void fbw_mul_all(uint64_t (&P)[S], const uint32_t (&a)[S], uint32_t addr,
                                            const uint32_t (&m)[S], uint32_t mprime, std::integer_sequence<int, Js...>) {
  uint32_t cur[7], nxt[7];
  fb_group_read<TW, 0>(nxt, addr);
  (fbw_step<S, TW, Js>(P, a, cur, nxt, addr, m, mprime), ...);
}
// a <- a b R^-1 mod m, b = this lane's word row in LDS (every read completes before the return)
template <int S, int TW>
__device__ __forceinline__ void fbw_mont_mul(uint32_t (&a)[S], uint32_t addr, const uint32_t (&m)[S], uint32_t mprime) {
  uint64_t P[S];
#pragma unroll
  for (int i = 0; i < S; ++i) P[i] = 0;
  fbw_mul_all<S, TW>(P, a, addr, m, mprime, std::make_integer_sequence<int, S>{});
  lane::normalize<S>(P, a);
}

// DMA table row `row` -> LDS buffer (the wave's 64-lane slice of each quad row). The LDS destination of
// each instruction (M0) is formed right here from one scalar base: left to the compiler, the TQ constant
// destinations are precomputed once, spilled under the product's register pressure and reloaded with a
// vmcnt(0) wait before every DMA instruction -- serialising the row stream.
#ifndef FB_DMA_AUX
#define FB_DMA_AUX 0   // cache-policy bits of the row DMA: 0 measured best (nt +5.7 %, sc0 +1 %, sc1 +3.4 % k_fbp time)
#endif
template <int TQ>
__device__ __forceinline__ void fb_row_to_lds(const uint4* __restrict__ table, size_t row, uint4* wave_row0) {
  typedef __attribute__((address_space(3))) uint4 lds_uint4;
  const uint4* r = table + row * TQ;   // quad g at an immediate offset
  const uint32_t lb = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(lds_uint4*)wave_row0);
#pragma unroll
  for (int g = 0; g < TQ; ++g) {
    uint32_t dst = lb + (uint32_t)(g * LANE_BLOCK * 16);
    asm volatile("" : "+s"(dst));
    __builtin_amdgcn_global_load_lds((const void*)(r + g), (__attribute__((address_space(3))) void*)(size_t)dst, 16, 0,
                                     FB_DMA_AUX);
  }
}

// 32-bit word WI of a number held as S canonical 28-bit limbs (4 WI mod 28 <= 24: two limbs suffice)
template <int S, int WI>
__device__ __forceinline__ uint32_t fb_word(const uint32_t (&x)[S]) {
  constexpr int bit = 32 * WI, k = bit / 28, sh = bit - 28 * k;
  uint64_t v = 0;
  if constexpr (k < S) v = (uint64_t)x[k] >> sh;
  if constexpr (k + 1 < S) v |= (uint64_t)x[k + 1] << (28 - sh);
  return (uint32_t)v;
}
template <int S, int... Gs>
__device__ __forceinline__ void fb_store_row(uint4* __restrict__ dst, const uint32_t (&x)[S], std::integer_sequence<int, Gs...>) {
  ((dst[Gs] = make_uint4(fb_word<S, 4 * Gs>(x), fb_word<S, 4 * Gs + 1>(x), fb_word<S, 4 * Gs + 2>(x),
                         fb_word<S, 4 * Gs + 3>(x))),
   ...);
}

// A wave-uniform pointer the optimiser cannot see through (scalar registers): loads through it stay
// where they are written instead of being hoisted out of the element loop.
__device__ __forceinline__ const uint32_t* opaque_uniform(const uint32_t* p) {
  const uint64_t v = (uint64_t)p;
  uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  asm volatile("" : "+s"(lo), "+s"(hi));
  return (const uint32_t*)(((uint64_t)hi << 32) | lo);
}

// A operand of the first product: 1 + n M reduced only partially mod p_h^2 (see header)
template <int SB>
__device__ __forceinline__ void fb_c0(int64_t M, const FbHalf* __restrict__ H, uint32_t (&a)[SB]) {
  using G = FbGeom<SB>;
  const bool neg = M < 0;
  const uint64_t mag = neg ? (uint64_t)0 - (uint64_t)M : (uint64_t)M;
  uint32_t mc[G::NC];
#pragma unroll
  for (int c = 0; c < G::NC; ++c) mc[c] = (uint32_t)((mag >> (G::CB * c)) & ((1ull << G::CB) - 1ull));
  // opaque copies + one scheduling fence per limb: the ~100s of uniform constant loads stay next to
  // their use (hoisted or batched, they pin as many registers for the whole kernel); the latency is
  // irrelevant next to the K products that follow
  const uint32_t* nm = opaque_uniform(H->nm);
  const uint32_t* pb = opaque_uniform(H->pbig);
  int64_t carry = 1;
#pragma unroll
  for (int j = 0; j < SB; ++j) {
    uint64_t s = 0;
#pragma unroll
    for (int c = 0; c < G::NC; ++c) s += (uint64_t)nm[c * SB + j] * mc[c];
    const int64_t v = carry + (neg ? (int64_t)pb[j] - (int64_t)s : (int64_t)s);
    a[j] = (uint32_t)v & lane::LMASK;
    carry = v >> lane::LB;   // arithmetic: the total is positive, partial sums may borrow
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Per element and half, c0 * prod_k T_k[d_k] mod p_h^2 (K products, no squarings).
// One LDS row buffer per wave (64 KB per 4-wave block at SB = 74): two blocks -- two waves per SIMD --
// fit a CU, so a wave waiting for its next table row is covered by the other wave's product.
template <int SB>
__global__ __launch_bounds__(LANE_BLOCK, 3 - FPAI_FB_NBUF) void k_fb(FbParams p) {
  using G = FbGeom<SB>;
  constexpr int TW = G::TW, TQ = TW / 4;
  __shared__ uint4 lbuf[FPAI_FB_NBUF * TQ * LANE_BLOCK];
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
  const uint32_t addr0 = (uint32_t)(size_t)(lds_uint4*)(lbuf + threadIdx.x);   // LDS byte offset
  for (long long base = (long long)blockIdx.x * LANE_BLOCK; base < p.n; base += (long long)gridDim.x * LANE_BLOCK) {
    const long long i = base + threadIdx.x;
    const long long ii = i < p.n ? i : p.n - 1;
    const uint32_t* dg = p.digits + (size_t)half * K * p.n + ii;   // digit k at dg[k * n]
    // loads first (vmcnt counts in order: a wait for x would otherwise also wait for the row DMA)
    uint32_t d0 = dg[0];
    uint32_t dn = K > 1 ? dg[p.n] : 0u;
    double xv;
    int64_t xi = 0;
    if (p.dtype == 0) xv = (double)((const float*)p.x)[ii];
    else if (p.dtype == 1) xv = ((const double*)p.x)[ii];
    else { xi = ((const int64_t*)p.x)[ii]; xv = 0.0; }
    asm volatile("" : "+v"(d0), "+v"(dn), "+v"(xv), "+v"(xi));
    fb_row_to_lds<TQ>(table, d0, brow);                    // row T_0[d_0]
    int64_t M = 0;
    int e = 0, st;
    const bool fixed = p.exp_mode != 0;
    if (p.dtype == 2) st = encode_int(xi, fixed, p.fexp, M, e);
    else st = encode_float(xv, fixed, p.fexp, M, e);
    if (half == 0 && i < p.n) {
      p.exp[i] = e;
      if (p.status) p.status[i] = st;
    }
    uint32_t a[SB];
    fb_c0<SB>(M, H, a);
#if FPAI_FB_NBUF == 2
    // two row buffers, one wave per SIMD: row k+1 streams in while product k runs
    uint4* brow1 = brow + TQ * LANE_BLOCK;
    const uint32_t addr1 = addr0 + TQ * LANE_BLOCK * 16;
    for (int k = 0; k < K; ++k) {
      lds_dma_wait();                                     // row k landed, digit k+1 loaded
      if (k + 1 < K) {
        fb_row_to_lds<TQ>(table, ((size_t)(k + 1) << W) + dn, (k & 1) ? brow : brow1);
        if (k + 2 < K) dn = dg[(size_t)(k + 2) * p.n];
      }
      fbw_mont_mul<SB, TW>(a, (k & 1) ? addr1 : addr0, m, mprime);   // every read of the row completes inside
    }
#else
    uint32_t dn2 = K > 2 ? dg[2 * p.n] : 0u;               // digit 2, in flight
    for (int k = 0; k < K; ++k) {
      lds_dma_wait();                                     // row k landed, digit k+2 loaded
      fbw_mont_mul<SB, TW>(a, addr0, m, mprime);          // every read of the row completes inside
      if (k + 1 < K) {
        const uint32_t dk1 = dn;
        dn = dn2;
        if (k + 3 < K) dn2 = dg[(size_t)(k + 3) * p.n];
        fb_row_to_lds<TQ>(table, ((size_t)(k + 1) << W) + dk1, brow);
      }
    }
#endif
    if (i < p.n) {
#pragma unroll
      for (int j = 0; j < SB; ++j) p.out[((size_t)half * SB + j) * p.n + i] = a[j];
    }
  }
}

// ---------------------------------------------------------------- Garner recombination -> ciphertext words
// column K of the plain product h q^2 (product scanning)
template <int S, int K>
__device__ __forceinline__ uint64_t fb_col(const uint32_t (&h)[S], const uint32_t* __restrict__ q2) {
  uint64_t s = 0;
  constexpr int lo = K < S ? 0 : K - S + 1, hi = K < S ? K : S - 1;
#pragma unroll
  for (int i = lo; i <= hi; ++i) s += (uint64_t)h[i] * q2[K - i];
  return s;
}
template <int S, int CW, int K>
__device__ __forceinline__ void fb_out_step(uint64_t& acc, uint64_t& buf, uint32_t (&o4)[4], const uint32_t (&h)[S],
                                            const uint32_t (&wq)[S], const uint32_t* __restrict__ q2, uint4* dst,
                                            bool valid) {
  if constexpr (K < 2 * S - 1) acc += fb_col<S, K>(h, q2);
  if constexpr (K < S) acc += wq[K];
  const uint32_t limb = (uint32_t)acc & lane::LMASK;
  acc >>= lane::LB;
  constexpr int NB = (28 * K) % 32;           // bits held in buf before this limb
  buf |= (uint64_t)limb << NB;
  if constexpr (NB + 28 >= 32) {
    constexpr int w = (28 * K) / 32;          // word completed by this limb
    o4[w % 4] = (uint32_t)buf;
    buf >>= 32;
    if constexpr (w % 4 == 3 && w < CW) {
      if (valid) dst[w / 4] = make_uint4(o4[0], o4[1], o4[2], o4[3]);
    }
  }
}
template <int S, int CW, int... Ks>
__device__ __forceinline__ void fb_out_all(const uint32_t (&h)[S], const uint32_t (&wq)[S], const uint32_t* __restrict__ q2,
                                           uint4* dst, bool valid, std::integer_sequence<int, Ks...>) {
  uint64_t acc = 0, buf = 0;
  uint32_t o4[4] = {0u, 0u, 0u, 0u};
  (fb_out_step<S, CW, Ks>(acc, buf, o4, h, wq, q2, dst, valid), ...);
}

// c = w_q + q^2 h, h = (w_p - w_q) (q^2)^-1 mod p^2: one element per lane
template <int SB>
__global__ __launch_bounds__(LANE_BLOCK) void k_fb_fin(FbFinParams p) {
  using G = FbGeom<SB>;
  constexpr int CW = 2 * G::TW;   // ciphertext words (n^2 < 2^(64 TW))
  __shared__ uint32_t q2s[SB];
  for (int j = threadIdx.x; j < SB; j += blockDim.x) q2s[j] = p.q2[j];
  __syncthreads();
  uint32_t m[SB];
#pragma unroll
  for (int j = 0; j < SB; ++j) m[j] = p.m[j];
  for (long long base = (long long)blockIdx.x * LANE_BLOCK; base < p.n; base += (long long)gridDim.x * LANE_BLOCK) {
    const long long i = base + threadIdx.x;
    const bool valid = i < p.n;
    const long long ii = valid ? i : p.n - 1;
    uint32_t wp[SB], wq[SB];
#pragma unroll
    for (int j = 0; j < SB; ++j) {
      wp[j] = p.w[(size_t)j * p.n + ii];
      wq[j] = p.w[((size_t)SB + j) * p.n + ii];
    }
    // w_q canonical mod q^2 FIRST: h must be formed from the same representative that c adds
    {
      uint32_t q2[SB];
#pragma unroll
      for (int j = 0; j < SB; ++j) q2[j] = q2s[j];
      lane::cond_sub<SB>(wq, q2);                // w_q < q^2
    }
    // t = w_p + 8 p^2 - w_q in (0, 10 p^2): a valid CIOS input (< 2^(28 SB - 20))
    {
      int64_t c = 0;
#pragma unroll
      for (int j = 0; j < SB; ++j) {
        const int64_t v = (int64_t)wp[j] + (int64_t)p.m8[j] - (int64_t)wq[j] + c;
        wp[j] = (uint32_t)v & lane::LMASK;
        c = v >> lane::LB;
      }
    }
    {
      uint32_t cr[SB];
#pragma unroll
      for (int j = 0; j < SB; ++j) cr[j] = p.coefR[j];
      lane::mont_mul<SB>(wp, cr, m, p.mprime);   // h < 2 p^2
    }
    lane::cond_sub<SB>(wp, m);                   // h < p^2
    fb_out_all<SB, CW>(wp, wq, q2s, reinterpret_cast<uint4*>(p.ct + ii * p.ct_words), valid,
                       std::make_integer_sequence<int, 2 * SB>{});
  }
}

// ---------------------------------------------------------------- per-key table: T_k[d] = G^(d 2^(W k)) R
// Two levels: k_fb_lohi builds, per position k, lo[j] = B_k^j (j < 2^LO) and hi[j] = B_k^(2^LO j)
// (j < 2^(W-LO)), LO = W/2, with B_k = G^(2^(W k)) from the host; k_fb_fill forms each of the 2^W
// entries with ONE product hi[d >> LO] * lo[d & (2^LO - 1)] and stores it as TW 32-bit words.
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
  constexpr int TQ = FbGeom<SB>::TW / 4;
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
  fb_store_row<SB>(table + ((size_t)k * ent + d) * TQ, a, std::make_integer_sequence<int, TQ>{});
}

}  // namespace fpai
