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
// G^(d 2^(W k)) precomputed once per key and resident in HBM; the samplers that multiply the rows are
// kernels_fbs.hpp (1024/2048-bit keys, Shoup rows) and kernels_sgp.hpp / kernels_sgs.hpp (4096-bit keys).
// This header holds what they share: the digit kernel, the row DMA, the table structs and the Garner
// output helpers. (The round-1 sampler k_fb, its Garner k_fb_fin and table builders were retired in
// round 6; the test build keeps k_fbp, kernels_fbp.hpp, as the cross-check of k_fbs.)
#pragma once
#include "kernels_crt.hpp"
#include "guard.hpp"

namespace fpai {

constexpr uint32_t FB_NONCE = 0x66786230u;   // ChaCha20 nonce word 2 (+ half) of the exponent stream
constexpr int FB_RAW_MAX = 80;               // words of the raw exponent per element (5 ChaCha blocks)
constexpr int FB_DIG_BLOCK = 128;            // threads per block of k_fb_digits
constexpr int FB_LO = 4096;
                                             // entries of the per-position small tables (k_fbp_lohi): W <= 24

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
// A wave-uniform pointer the optimiser cannot see through (scalar registers): loads through it stay
// where they are written instead of being hoisted out of the element loop.
__device__ __forceinline__ const uint32_t* opaque_uniform(const uint32_t* p) {
  const uint64_t v = (uint64_t)p;
  uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  asm volatile("" : "+s"(lo), "+s"(hi));
  return (const uint32_t*)(((uint64_t)hi << 32) | lo);
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
}  // namespace fpai
