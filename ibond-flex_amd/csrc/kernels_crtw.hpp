// CRT encryption for protocol-sized calls (a fresh key's first call, HE_SA_FT's per-exchange theta lists,
// he_sa_ft/train.py:38-41): the same two exponentiations as k_crt_a + k_crt_b_pair (kernels_crt.hpp,
// kernels_pair.hpp), with the same constants, op lists and output, but each residue spread over a DPP row of 16
// lanes instead of one lane (or one lane of a pair). On a call of ~1 000 elements those kernels keep ~2 000 lanes of
// the chip's 65 536 busy and take one lane's whole chain -- 1 024 squares of 3.5 S^2 multiply-accumulates in
// sequence (22 ms at nb = 2048, profiles/r06c_fresh_key_1k_trace.log). Here a product is K CIOS digit steps of
// 2 LW multiply-accumulates per lane (K = limbs of the modulus, LW = ceil((K + 1) / 16) limbs per lane), so the
// chain's length is K steps of one digit's dependency (digit, reduction digit q, DPP broadcast, carry) rather than
// K^2 MACs.
//
//   k_crt_w<KA, KB>   per (element, half): x~ = r R mod p_h (kchunks passes over r's KA-limb chunks, as k_crt_a),
//                     y = x~^(q_h mod (p_h - 1)) R^-1 mod p_h (the stage-A op list),
//                     u = (y R)^(p_h) coef R^-1 mod p_h^2 (the stage-B op list of the 2S-limb lane constants,
//                     R = 2^(28 KB)), written as KB 28-bit limbs [2][KB][n] for k_crt_fin.
//   k_dec_w<KA, KB>   decryption's exponentiation the same way (decryptor.py:55-61): c~ = c R mod p_h^2, x =
//                     c~^(p_h - 1) R^-1 mod p_h^2 (the op list over p_h - 1), x made canonical, then the pair of x that
//                     k_dec_fin_pair takes: A = x mod p_h (0 or 1: x == 1 mod p_h unless p_h | c, when x == 0) and
//                     B = (x - A) / p_h, an exact division by REDC's digits (Q = -(x - A) p_h^-1 mod R_A, B = -Q).
//   k_pe_w<K>         a public-key-only party's encryption the same way (encryptor.py:71-114, raw_encrypt.py:37-45,
//                     obfuscator.py:36): c0 = 1 + n M mod n^2 on the row, r R mod n^2, the op list over n with c0 as
//                     the final multiplier, over the K = 74 / 148 limbs of n^2 (k_encrypt's R = 2^(28 K)).
//
// Layout: lane t of a row owns limbs [t LW, t LW + LW) of the accumulator (bn_group.hpp's rotating CIOS with L ->
// LW); every multiplicand sits in LDS as plain limbs (limb j = word j of a slot), read by the row as a broadcast,
// four digits per 16-byte read. The op list's tiles, the squaring operand and the multiplier are LDS slots of the
// row, so a tile never moves: PREFETCH / B_READY / B_SET become pointer updates. One wave per block (four rows);
// blockIdx.y selects the half.
#pragma once
#include "kernels_crt.hpp"

namespace fpai {
namespace crtw {

constexpr int TPI = 16;              // lanes per residue: one DPP row (row_newbcast and row_shl stay inside it)
constexpr int GPW = 64 / TPI;        // residues per wave
constexpr int BLOCK_W = 64;          // one wave per block

template <int K>
struct Geom {
  static constexpr int LW = (K + 1 + TPI - 1) / TPI;   // limbs per lane: room for K + 1 limbs
  static constexpr int W = TPI * LW;                   // limbs per row (a multiple of 16)
};

// one digit step j of a CIOS product with the rotation s = j % LW (bn_group.hpp cios_step)
template <int LW, int J>
__device__ __forceinline__ void step(uint64_t (&P)[LW], const uint32_t (&a)[LW], uint32_t bj, const uint32_t (&m)[LW],
                                     uint32_t mprime) {
  constexpr int s = J % LW;
#pragma unroll
  for (int i = 0; i < LW; ++i) P[(i + s) % LW] += (uint64_t)a[i] * bj;
  const uint32_t q = bcast0<TPI>(((uint32_t)P[s] * mprime) & LMASK);
#pragma unroll
  for (int i = 0; i < LW; ++i) P[(i + s) % LW] += (uint64_t)q * m[i];
  const uint64_t v0 = P[s];
  P[(s + 1) % LW] += v0 >> LB;
  P[s] = (uint64_t)dpp_from_next((uint32_t)v0 & LMASK);
#pragma unroll
  for (int i = 0; i < LW; ++i) asm volatile("" : "+v"(P[i]));
  __builtin_amdgcn_sched_barrier(0);
}

// digits of the multiplicand from its LDS slot, four per 16-byte read, the next quad in flight
template <int K>
struct Digits {
  const uint4* q;
  uint4 c, n;
  __device__ __forceinline__ explicit Digits(const uint32_t* B) : q(reinterpret_cast<const uint4*>(B)) {
    c = q[0];
    if constexpr (K > 4) n = q[1];
  }
  template <int J>
  __device__ __forceinline__ uint32_t get() {
    constexpr int r = J & 3;
    const uint32_t v = r == 0 ? c.x : r == 1 ? c.y : r == 2 ? c.z : c.w;
    if constexpr (r == 3) {
      c = n;
      if constexpr (4 * (J / 4 + 2) < K) n = q[J / 4 + 2];
    }
    return v;
  }
};

// LW consecutive steps from a digit index that is a multiple of LW (so step s has rotation s)
template <int LW, int... Ss>
__device__ __forceinline__ void step_group(uint64_t (&P)[LW], const uint32_t (&a)[LW], const uint32_t* Bg,
                                           const uint32_t (&m)[LW], uint32_t mprime, std::integer_sequence<int, Ss...>) {
  (step<LW, Ss>(P, a, Bg[Ss], m, mprime), ...);
}
// K steps: fully unrolled (the digits four per 16-byte read) up to K = 160; beyond that -- the 296 limbs of a
// 4096-bit key's n^2, whose unrolled product would not fit the instruction cache -- a loop over groups of LW steps
// (compile-time rotations inside a group) and an unrolled tail of K % LW steps
template <int K, int LW, int... Js>
__device__ __forceinline__ void steps(uint64_t (&P)[LW], const uint32_t (&a)[LW], const uint32_t* B,
                                      const uint32_t (&m)[LW], uint32_t mprime, std::integer_sequence<int, Js...>) {
  if constexpr (K <= 160) {
    Digits<K> d(B);
    (step<LW, Js>(P, a, d.template get<Js>(), m, mprime), ...);
  } else {
#pragma unroll 1
    for (int g = 0; g < K / LW; ++g)
      step_group<LW>(P, a, B + g * LW, m, mprime, std::make_integer_sequence<int, LW>{});
    step_group<LW>(P, a, B + (K / LW) * LW, m, mprime, std::make_integer_sequence<int, K % LW>{});
  }
}

// canonical limbs of the accumulator after K steps (rotation K % LW); bn_group.hpp normalize with L -> LW
template <int LW, int S0>
__device__ __forceinline__ void normalize(const uint64_t (&P)[LW], uint32_t (&r)[LW], int lane, int tig) {
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < LW; ++i) {
    const uint64_t v = P[(i + S0) % LW] + c;
    r[i] = (uint32_t)v & LMASK;
    c = v >> LB;
  }
  uint32_t inlo = dpp_from_prev((uint32_t)c);
  uint32_t inhi = dpp_from_prev((uint32_t)(c >> 32));
  if (tig == 0) inlo = inhi = 0;
  c = ((uint64_t)inhi << 32) | inlo;
  // the incoming carry (< 2^40) spreads over the first two limbs; what is left is 0 or 1
#pragma unroll
  for (int i = 0; i < LW; ++i) {
    const uint64_t v = (uint64_t)r[i] + c;
    r[i] = (uint32_t)v & LMASK;
    c = v >> LB;
  }
  const uint32_t c32 = (uint32_t)c;
  if (ballot(c32 != 0) != 0ull) {
    bool all_ones = true;
#pragma unroll
    for (int i = 0; i < LW; ++i) all_ones &= (r[i] == LMASK);
    uint32_t ci = lookahead_carry_in<TPI>(c32 != 0, all_ones, lane);
#pragma unroll
    for (int i = 0; i < LW; ++i) {
      const uint32_t v = r[i] + ci;
      r[i] = v & LMASK;
      ci = v >> LB;
    }
  }
}

// a <- (x + a B) R^-1 mod m with R = 2^(28 K) (x = 0 unless ACC): a < 2m (or a < m with B < R), B < 2m, x < 2m
// -> result < 2m
template <int K, bool ACC = false>
__device__ __forceinline__ void mont(uint32_t (&a)[Geom<K>::LW], const uint32_t* B, const uint32_t (&m)[Geom<K>::LW],
                                     uint32_t mprime, int lane, int tig, const uint32_t (&x)[Geom<K>::LW]) {
  constexpr int LW = Geom<K>::LW;
  uint64_t P[LW];
#pragma unroll
  for (int i = 0; i < LW; ++i) P[i] = ACC ? (uint64_t)x[i] : 0ull;
  steps<K, LW>(P, a, B, m, mprime, std::make_integer_sequence<int, K>{});
  normalize<LW, K % LW>(P, a, lane, tig);
}
template <int K>
__device__ __forceinline__ void mont(uint32_t (&a)[Geom<K>::LW], const uint32_t* B, const uint32_t (&m)[Geom<K>::LW],
                                     uint32_t mprime, int lane, int tig) {
  mont<K, false>(a, B, m, mprime, lane, tig, a);
}

__device__ __forceinline__ const uint32_t* uniform_ptr(const uint32_t* p) {
  const uint64_t v = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (const uint32_t*)(((uint64_t)hi << 32) | lo);
}

// d = a - b over the row's TPI LW limbs (bn_group.hpp sub_limbs with L -> LW); returns true (row-uniform) when a < b
// (d is then the two's-complement wrap)
template <int LW>
__device__ __forceinline__ bool sub(const uint32_t (&a)[LW], const uint32_t (&b)[LW], uint32_t (&d)[LW], int lane, int tig) {
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < LW; ++i) {
    const int32_t v = (int32_t)a[i] - (int32_t)b[i] + c;
    d[i] = (uint32_t)v & LMASK;
    c = v >> LB;
  }
  const int32_t b1 = c;
  int32_t bin = (int32_t)dpp_from_prev((uint32_t)c);
  if (tig == 0) bin = 0;
#pragma unroll
  for (int i = 0; i < LW; ++i) {
    const int32_t v = (int32_t)d[i] + bin;
    d[i] = (uint32_t)v & LMASK;
    bin = v >> LB;
  }
  bool all_zero = true;
#pragma unroll
  for (int i = 0; i < LW; ++i) all_zero &= (d[i] == 0u);
  const bool gen = bin != 0;
  const uint32_t bi = lookahead_carry_in<TPI>(gen, all_zero, lane);
  if (ballot(bi != 0) != 0ull) {
    int32_t b2 = -(int32_t)bi;
#pragma unroll
    for (int i = 0; i < LW; ++i) {
      const int32_t v = (int32_t)d[i] + b2;
      d[i] = (uint32_t)v & LMASK;
      b2 = v >> LB;
    }
  }
  const bool neg_here = (tig == TPI - 1) && (b1 != 0 || gen || (all_zero && bi));
  return ((ballot(neg_here) >> (lane - tig + TPI - 1)) & 1ull) != 0ull;
}

// row-uniform: some limb of the row is nonzero
template <int LW>
__device__ __forceinline__ bool nonzero(const uint32_t (&x)[LW], int lane, int tig) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < LW; ++i) o |= x[i];
  return ((ballot(o != 0u) >> (lane - tig)) & 0xFFFFull) != 0ull;
}

// REDC digit j of an exact division (no product term): q = T_0 mprime, T = (T + q m) / 2^28; q kept by lane j / LW in
// slot j % LW (the slot the rotation frees)
template <int LW, int J>
__device__ __forceinline__ void dstep(uint64_t (&P)[LW], const uint32_t (&m)[LW], uint32_t mprime, uint32_t (&o)[LW], int tig) {
  constexpr int s = J % LW;
  const uint32_t q = bcast0<TPI>(((uint32_t)P[s] * mprime) & LMASK);
  o[s] = tig == J / LW ? q : o[s];
#pragma unroll
  for (int i = 0; i < LW; ++i) P[(i + s) % LW] += (uint64_t)q * m[i];
  const uint64_t v0 = P[s];
  P[(s + 1) % LW] += v0 >> LB;
  P[s] = (uint64_t)dpp_from_next((uint32_t)v0 & LMASK);
#pragma unroll
  for (int i = 0; i < LW; ++i) asm volatile("" : "+v"(P[i]));
  __builtin_amdgcn_sched_barrier(0);
}
template <int LW, int... Js>
__device__ __forceinline__ void dsteps(uint64_t (&P)[LW], const uint32_t (&m)[LW], uint32_t mprime, uint32_t (&o)[LW], int tig,
                                       std::integer_sequence<int, Js...>) {
  (dstep<LW, Js>(P, m, mprime, o, tig), ...);
}

// row slot <- limbs (zero above the row's TPI LW limbs, up to SW words)
template <int LW, int SW>
__device__ __forceinline__ void put(uint32_t* slot, const uint32_t (&x)[LW], int tig) {
  wave_lds_fence();
#pragma unroll
  for (int i = 0; i < LW; ++i) slot[tig * LW + i] = x[i];
  for (int w = TPI * LW + tig; w < SW; w += TPI) slot[w] = 0u;
  wave_lds_fence();
}
template <int LW>
__device__ __forceinline__ void get(const uint32_t* slot, uint32_t (&x)[LW], int tig) {
#pragma unroll
  for (int i = 0; i < LW; ++i) x[i] = slot[tig * LW + i];
}
// modulus-sized constant (nl limbs in global memory) -> this lane's LW limbs
template <int LW>
__device__ __forceinline__ void load_const(const uint32_t* __restrict__ g, int nl, uint32_t (&x)[LW], int tig) {
#pragma unroll
  for (int i = 0; i < LW; ++i) {
    const int k = tig * LW + i;
    x[i] = k < nl ? g[k] : 0u;
  }
}

// The lane machine's op list (kernels_crt.hpp run_lane_program) on a row: a <- ... then the final product with CF.
template <int K, int SW>
__device__ __forceinline__ void run(uint32_t (&a)[Geom<K>::LW], uint32_t* T, uint32_t* SQ, uint32_t* MU, const uint32_t* CF,
                                    const uint32_t* __restrict__ prog, int nprog, const uint32_t (&m)[Geom<K>::LW],
                                    uint32_t mprime, int lane, int tig) {
  constexpr int LW = Geom<K>::LW;
  const uint32_t* ms = MU;
  for (int i = 0; i <= nprog; ++i) {
    const uint32_t op = (i < nprog) ? lane_op(prog, i) : LOP_B_CONST;
    if (op & LOP_A_FROM_T) get<LW>(T + ((op >> 16) & 0xFF) * SW, a, tig);
    const uint32_t* b;
    if (op & LOP_SQR) {
      if (op & LOP_PREFETCH) ms = T + ((op >> 8) & 0xFF) * SW;
      put<LW, SW>(SQ, a, tig);
      b = SQ;
    } else if (op & LOP_B_CONST) {
      b = ms = CF;
    } else if (op & LOP_B_READY) {
      b = ms;
    } else {
      b = ms = T + ((op >> 8) & 0xFF) * SW;
    }
    mont<K>(a, b, m, mprime, lane, tig);
    if (op & LOP_STORE) put<LW, SW>(T + (op >> 24) * SW, a, tig);
    if (op & LOP_B_SET) {
      put<LW, SW>(MU, a, tig);
      ms = MU;
    }
  }
}

struct Params {
  const CrtHalf* ha;            // [2] stage A halves (p_h, R^(K+1) mod p_h, 1, op list)
  const CrtHalf* hb;            // [2] stage B halves, 2S-limb lane constants (p_h^2, R^2, coef, op list; R = 2^(28 KB))
  long long n;
  int obf;                      // PAI_OBF_GIVEN (1) or PAI_OBF_RNG (2)
  const uint32_t* r;            // GIVEN: words, element i at r + i * r_stride
  long long r_stride;
  int r_words;                  // words of r (GIVEN) or of the ChaCha stream (RNG)
  uint32_t rng_key[8];
  unsigned long long index_base;
  int kchunks;                  // ceil(32 r_words / (28 KA)) <= KMAX_CHUNKS
  uint32_t* out;                // u [2][KB][n]
};

constexpr int RW_WORDS = 256;          // staging of r / the ciphertext: up to 8192 bits (a 4096-bit key's ct_words)
template <int KA, int KB>
constexpr int slot_words() { return Geom<KB>::W > Geom<KA>::W ? Geom<KB>::W : Geom<KA>::W; }
constexpr int NSLOT = LANE_NTILE + 2;   // the op list's tiles, the squaring operand, the multiplier
template <int KA, int KB>
constexpr size_t lds_words() { return (size_t)(GPW * NSLOT + 3) * slot_words<KA, KB>(); }

template <int KA, int KB>
__global__ __launch_bounds__(BLOCK_W) void k_crt_w(Params p) {
  constexpr int LA = Geom<KA>::LW, LBW = Geom<KB>::LW;
  constexpr int SW = slot_words<KA, KB>();
  constexpr int CS = (KA + 3) & ~3;                     // stage A: one r chunk per CS words
  static_assert(RW_WORDS + KMAX_CHUNKS * CS <= LANE_NTILE * SW, "r staging must fit the tiles it aliases");
  static_assert(SW % 4 == 0, "16-byte slots");
  __shared__ __attribute__((aligned(16))) uint32_t sm[lds_words<KA, KB>()];
  const int half = blockIdx.y;
  const CrtHalf* HA = p.ha + half;
  const CrtHalf* HB = p.hb + half;
  const int lane = threadIdx.x, tig = lane & (TPI - 1), g = lane / TPI;
  uint32_t* T = sm + g * NSLOT * SW;                    // tile k at T + k SW
  uint32_t* SQ = T + LANE_NTILE * SW;
  uint32_t* MU = SQ + SW;
  uint32_t* CA = sm + GPW * NSLOT * SW;                 // 1 (stage A's last product leaves Montgomery form)
  uint32_t* CR = CA + SW;                               // R^2 mod p_h^2
  uint32_t* CC = CR + SW;                               // (other^2)^-1 mod p_h^2
  for (int w = lane; w < SW; w += BLOCK_W) {
    CA[w] = w < KA ? HA->c1[w] : 0u;
    CR[w] = w < KB ? HB->c0[w] : 0u;
    CC[w] = w < KB ? HB->c1[w] : 0u;
  }
  uint32_t mA[LA], mB[LBW], cK[LA];
  load_const<LA>(HA->m, KA, mA, tig);
  load_const<LBW>(HB->m, KB, mB, tig);
  load_const<LA>(HA->c0 + (size_t)(p.kchunks - 1) * KA, KA, cK, tig);   // R^(kchunks + 1) mod p_h
  const uint32_t mpA = HA->mprime, mpB = HB->mprime;
  // the op lists' addresses and lengths, wave-uniform in SGPRs (lane_op's s_load)
  const uint32_t* progA = uniform_ptr(HA->prog);
  const uint32_t* progB = uniform_ptr(HB->prog);
  const int nA = __builtin_amdgcn_readfirstlane(HA->nprog), nB = __builtin_amdgcn_readfirstlane(HB->nprog);
  const bool given = p.obf == 1;
  for (long long base = (long long)blockIdx.x * GPW; base < p.n; base += (long long)gridDim.x * GPW) {
    const long long i = base + g;
    const long long ii = i < p.n ? i : p.n - 1;
    // r words -> the row's staging words (aliasing the tiles), then r's 28-bit limbs chunk by chunk
    uint32_t* RW = T;
    uint32_t* RL = T + RW_WORDS;
    wave_lds_fence();
    if (given) {
      const uint32_t* rg = p.r + ii * p.r_stride;
      for (int w = tig; w < p.r_words; w += TPI) RW[w] = rg[w];
    } else {
      const unsigned long long gi = p.index_base + (unsigned long long)ii;
      for (int b = tig; b * 16 < p.r_words; b += TPI) {
        uint32_t blk[16];
        chacha20_block(p.rng_key, (uint32_t)b, (uint32_t)gi, (uint32_t)(gi >> 32), 0x66786169u, blk);
#pragma unroll
        for (int w = 0; w < 16; ++w) RW[b * 16 + w] = blk[w];
      }
    }
    wave_lds_fence();
    const int nw = p.r_words;
    for (int j = tig; j < p.kchunks * KA; j += TPI) {
      const int bit = j * LB, wi = bit >> 5, sh = bit & 31;
      const uint64_t lo = wi < nw ? (uint64_t)RW[wi] : 0ull;
      const uint64_t hi = wi + 1 < nw ? (uint64_t)RW[wi + 1] : 0ull;
      RL[(j / KA) * CS + j % KA] = (uint32_t)(((hi << 32) | lo) >> sh) & LMASK;
    }
    wave_lds_fence();
    // stage A: x~ = r R mod p_h = sum_k chunk_k R^(k - kchunks) R^(kchunks + 1), one CIOS pass per chunk
    uint32_t x[LA];
#pragma unroll
    for (int j = 0; j < LA; ++j) x[j] = 0u;
    for (int k = 0; k < p.kchunks; ++k) {
      uint32_t acc[LA];
#pragma unroll
      for (int j = 0; j < LA; ++j) {
        acc[j] = x[j];
        x[j] = cK[j];
      }
      mont<KA, true>(x, RL + k * CS, mA, mpA, lane, tig, acc);
    }
    put<LA, SW>(T, x, tig);                                   // tile 0 (the staging words are consumed)
    run<KA, SW>(x, T, SQ, MU, CA, progA, nA, mA, mpA, lane, tig);   // y = x~^e * 1
    // stage B: (y, R^2) -> y R mod p_h^2, the op list over p_h, then the product with coef
    put<LA, SW>(SQ, x, tig);
    uint32_t a[LBW];
    get<LBW>(SQ, a, tig);
    mont<KB>(a, CR, mB, mpB, lane, tig);
    put<LBW, SW>(T, a, tig);
    run<KB, SW>(a, T, SQ, MU, CC, progB, nB, mB, mpB, lane, tig);
    if (i < p.n) {
#pragma unroll
      for (int j = 0; j < LBW; ++j) {
        const int limb = tig * LBW + j;
        if (limb < KB) p.out[((size_t)half * KB + limb) * p.n + i] = a[j];
      }
    }
  }
}

struct DecParams {
  const CrtHalf* hd;            // [2]: p_h^2 (KB limbs), R^(K+1) mod p_h^2 (R = 2^(28 KB)), 1, op list over p_h - 1
  const CrtHalf* ha;            // [2]: p_h (KA limbs) and its mprime (the exact division)
  long long n;
  const uint32_t* ct;
  int ct_words;
  int kchunks;                  // ceil(32 ct_words / (28 KB)) <= KMAX_CHUNKS
  uint32_t* out;                // [2][2 KA][n]: the pair (A, B) of c^(p_h - 1) mod p_h^2, k_dec_fin_pair's input
};

template <int KA, int KB>
__global__ __launch_bounds__(BLOCK_W) void k_dec_w(DecParams p) {
  constexpr int LBW = Geom<KB>::LW;
  constexpr int SW = slot_words<KA, KB>();
  constexpr int CS = (KB + 3) & ~3;                     // one ciphertext chunk per CS words
  static_assert(RW_WORDS + KMAX_CHUNKS * CS <= LANE_NTILE * SW, "ciphertext staging must fit the tiles it aliases");
  __shared__ __attribute__((aligned(16))) uint32_t sm[lds_words<KA, KB>()];
  const int half = blockIdx.y;
  const CrtHalf* HD = p.hd + half;
  const CrtHalf* HA = p.ha + half;
  const int lane = threadIdx.x, tig = lane & (TPI - 1), g = lane / TPI;
  uint32_t* T = sm + g * NSLOT * SW;
  uint32_t* SQ = T + LANE_NTILE * SW;
  uint32_t* MU = SQ + SW;
  uint32_t* CO = sm + GPW * NSLOT * SW;                 // 1
  for (int w = lane; w < SW; w += BLOCK_W) CO[w] = w < KB ? HD->c1[w] : 0u;
  uint32_t m[LBW], mp[LBW], cK[LBW];
  load_const<LBW>(HD->m, KB, m, tig);
  load_const<LBW>(HA->m, KA, mp, tig);
  load_const<LBW>(HD->c0, KB, cK, tig);                 // R^(kchunks + 1) mod p_h^2
  const uint32_t mpD = HD->mprime, mpA = HA->mprime;
  const uint32_t* prog = uniform_ptr(HD->prog);
  const int nprog = __builtin_amdgcn_readfirstlane(HD->nprog);
  for (long long base = (long long)blockIdx.x * GPW; base < p.n; base += (long long)gridDim.x * GPW) {
    const long long i = base + g;
    const long long ii = i < p.n ? i : p.n - 1;
    uint32_t* RW = T;
    uint32_t* RL = T + RW_WORDS;
    wave_lds_fence();
    {
      const uint32_t* cw = p.ct + ii * p.ct_words;
      for (int w = tig; w < p.ct_words; w += TPI) RW[w] = cw[w];
    }
    wave_lds_fence();
    const int nw = p.ct_words;
    for (int j = tig; j < p.kchunks * KB; j += TPI) {
      const int bit = j * LB, wi = bit >> 5, sh = bit & 31;
      const uint64_t lo = wi < nw ? (uint64_t)RW[wi] : 0ull;
      const uint64_t hi = wi + 1 < nw ? (uint64_t)RW[wi + 1] : 0ull;
      RL[(j / KB) * CS + j % KB] = (uint32_t)(((hi << 32) | lo) >> sh) & LMASK;
    }
    wave_lds_fence();
    // c~ = c R mod p_h^2, one CIOS pass per chunk of the ciphertext's digits (as k_crt_w's x~)
    uint32_t x[LBW];
#pragma unroll
    for (int j = 0; j < LBW; ++j) x[j] = 0u;
    for (int k = 0; k < p.kchunks; ++k) {
      uint32_t acc[LBW];
#pragma unroll
      for (int j = 0; j < LBW; ++j) {
        acc[j] = x[j];
        x[j] = cK[j];
      }
      mont<KB, true>(x, RL + k * CS, m, mpD, lane, tig, acc);
    }
    put<LBW, SW>(T, x, tig);
    run<KB, SW>(x, T, SQ, MU, CO, prog, nprog, m, mpD, lane, tig);   // x = c^(p_h - 1) mod p_h^2, < 2 p_h^2
    {
      uint32_t d[LBW];
      if (!sub<LBW>(x, m, d, lane, tig)) {
#pragma unroll
        for (int j = 0; j < LBW; ++j) x[j] = d[j];
      }
    }
    const uint32_t A = nonzero<LBW>(x, lane, tig) ? 1u : 0u;
    {
      uint32_t av[LBW], d[LBW];
#pragma unroll
      for (int j = 0; j < LBW; ++j) av[j] = (tig == 0 && j == 0) ? A : 0u;
      (void)sub<LBW>(x, av, d, lane, tig);             // x - A (>= 0)
#pragma unroll
      for (int j = 0; j < LBW; ++j) x[j] = d[j];
    }
    uint32_t Bv[LBW];
    {
      uint64_t P[LBW];
      uint32_t q[LBW], z[LBW];
#pragma unroll
      for (int j = 0; j < LBW; ++j) {
        P[j] = x[j];
        q[j] = 0u;
        z[j] = 0u;
      }
      dsteps<LBW>(P, mp, mpA, q, tig, std::make_integer_sequence<int, KA>{});   // q = -(x - A) p_h^-1 mod R_A
      (void)sub<LBW>(z, q, Bv, lane, tig);
#pragma unroll
      for (int j = 0; j < LBW; ++j)
        if (tig * LBW + j >= KA) Bv[j] = 0u;                                   // B = (x - A) / p_h < p_h
    }
    if (i < p.n) {
      uint32_t* o = p.out + (size_t)half * 2 * KA * p.n + i;
#pragma unroll
      for (int j = 0; j < LBW; ++j) {
        const int limb = tig * LBW + j;
        if (limb < KA) {
          o[(size_t)limb * p.n] = limb == 0 ? A : 0u;
          o[(size_t)(KA + limb) * p.n] = Bv[j];
        }
      }
    }
  }
}

template <int K>
__global__ __launch_bounds__(BLOCK_W) void k_pe_w(EncParams p, const uint32_t* prog_, int nprog_) {
  constexpr int LW = Geom<K>::LW, SW = Geom<K>::W;
  constexpr int NS = LANE_NTILE + 3;                    // the tiles, the squaring operand, the multiplier, c0
  static_assert(RW_WORDS <= LANE_NTILE * SW, "r staging must fit the tiles it aliases");
  __shared__ __attribute__((aligned(16))) uint32_t sm[(GPW * NS + 1) * SW];
  const int lane = threadIdx.x, tig = lane & (TPI - 1), g = lane / TPI;
  uint32_t* T = sm + g * NS * SW;
  uint32_t* SQ = T + LANE_NTILE * SW;
  uint32_t* MU = SQ + SW;
  uint32_t* C0 = MU + SW;
  uint32_t* CR = sm + GPW * NS * SW;                    // R^2 mod n^2
  for (int w = lane; w < SW; w += BLOCK_W) CR[w] = w < K ? p.R2[w] : 0u;
  uint32_t m[LW];
  load_const<LW>(p.N, K, m, tig);
  const uint32_t mprime = p.mprime;
  const uint32_t* prog = uniform_ptr(prog_);
  const int nprog = __builtin_amdgcn_readfirstlane(nprog_);
  const bool given = p.obf == 1;
  const int nw = given ? p.r_words : p.rng_words;
  for (long long base = (long long)blockIdx.x * GPW; base < p.n; base += (long long)gridDim.x * GPW) {
    const long long i = base + g;
    const bool valid = i < p.n;
    const long long ii = valid ? i : p.n - 1;
    int64_t M = 0;
    int e = 0, st;
    const bool fixed = p.exp_mode != 0;
    if (p.dtype == 0) st = encode_float((double)((const float*)p.x)[ii], fixed, p.fexp, M, e);
    else if (p.dtype == 1) st = encode_float(((const double*)p.x)[ii], fixed, p.fexp, M, e);
    else st = encode_int(((const int64_t*)p.x)[ii], fixed, p.fexp, M, e);
    {   // c0 = 1 + n M mod n^2 (n^2 - n |M| + 1 for M < 0: raw_encrypt.py's "sneaky inverse" gives the same value)
      const bool neg = M < 0;
      const uint64_t mag = neg ? (uint64_t)0 - (uint64_t)M : (uint64_t)M;
      const uint32_t M0 = (uint32_t)mag & LMASK, M1 = (uint32_t)(mag >> LB) & LMASK, M2 = (uint32_t)(mag >> (2 * LB));
      uint64_t P[LW];
#pragma unroll
      for (int j = 0; j < LW; ++j) {
        const int k = tig * LW + j;
        const uint64_t a0 = k < K ? p.nl[k] : 0u;
        const uint64_t a1 = k >= 1 && k - 1 < K ? p.nl[k - 1] : 0u;
        const uint64_t a2 = k >= 2 && k - 2 < K ? p.nl[k - 2] : 0u;
        P[j] = a0 * M0 + a1 * M1 + a2 * M2;
      }
      uint32_t X[LW], D[LW];
      normalize<LW, 0>(P, X, lane, tig);
      (void)sub<LW>(m, X, D, lane, tig);
#pragma unroll
      for (int j = 0; j < LW; ++j) P[j] = (uint64_t)(neg ? D[j] : X[j]) + ((tig == 0 && j == 0) ? 1u : 0u);
      normalize<LW, 0>(P, X, lane, tig);
      put<LW, SW>(C0, X, tig);
    }
    // r: the caller's words or this element's ChaCha20 stream (k_encrypt's), staged in the tiles
    uint32_t* RW = T;
    wave_lds_fence();
    if (given) {
      const uint32_t* rg = p.r + ii * p.r_stride;
      for (int w = tig; w < nw; w += TPI) RW[w] = rg[w];
    } else {
      const unsigned long long gi = p.index_base + (unsigned long long)ii;
      for (int b = tig; b * 16 < nw; b += TPI) {
        uint32_t blk[16];
        chacha20_block(p.rng_key, (uint32_t)b, (uint32_t)gi, (uint32_t)(gi >> 32), 0x66786169u, blk);
#pragma unroll
        for (int w = 0; w < 16; ++w) RW[b * 16 + w] = blk[w];
      }
    }
    wave_lds_fence();
    uint32_t a[LW];
#pragma unroll
    for (int j = 0; j < LW; ++j) {
      const int bit = (tig * LW + j) * LB, wi = bit >> 5, sh = bit & 31;
      const uint64_t lo = wi < nw ? (uint64_t)RW[wi] : 0ull;
      const uint64_t hi = wi + 1 < nw ? (uint64_t)RW[wi + 1] : 0ull;
      a[j] = (uint32_t)(((hi << 32) | lo) >> sh) & LMASK;
    }
    mont<K>(a, CR, m, mprime, lane, tig);                         // r R (r < 4 n^2, R > 8 n^2)
    put<LW, SW>(T, a, tig);
    run<K, SW>(a, T, SQ, MU, C0, prog, nprog, m, mprime, lane, tig);   // r^n c0 (< 2 n^2)
    {
      uint32_t d[LW];
      if (!sub<LW>(a, m, d, lane, tig)) {
#pragma unroll
        for (int j = 0; j < LW; ++j) a[j] = d[j];
      }
    }
    put<LW, SW>(SQ, a, tig);
    if (valid) {
      for (int w = tig; w < p.ct_words; w += TPI) p.ct[ii * p.ct_words + w] = limbs_word(SQ, SW, w);
      if (tig == 0) {
        p.exp[ii] = e;
        if (p.status) p.status[ii] = st;
      }
    }
  }
}

}  // namespace crtw
}  // namespace fpai
