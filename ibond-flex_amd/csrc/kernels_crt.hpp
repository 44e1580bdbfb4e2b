// CRT encryption for holders of the private key (HE_SA_FT and every other caller that encrypts
// and decrypts with the same keypair, he_sa_ft/train.py:39-46). Same ciphertext bits as the
// public-key path, c = c0 * r^n mod n^2, computed as
//
//   r^n mod p^2 = (r^q mod p)^p mod p^2        (x == x' mod p  =>  x^p == x'^p mod p^2, n = pq)
//   r^q mod p   = (r mod p)^(q mod (p-1)) mod p (Fermat)
//
// and likewise mod q^2, then recombined: u_p = z_p * (q^2)^-1 mod p^2, u_q = z_q * (p^2)^-1 mod q^2,
// r^n == u_p q^2 + u_q p^2 (mod n^2). Per element this is ~4x fewer MACs than the 4096-bit
// modexp of the public path. Three kernels:
//   k_crt_a<SA>   mod p_h, one element per lane (bn_lane.hpp), 1024-bit exponent  -> y_h
//   stage B       mod p_h^2, exponent p_h, times the CRT coefficient -> u_h: k_crt_b_pair (kernels_pair.hpp, on
//                 p-adic pairs; the 2S-limb k_crt_b that first did it was retired in round 6)
//   k_crt_fin<TPI> lane groups mod n^2 (bn_group.hpp): (u_p q^2 + u_q p^2) * c0 with c0 = 1 + n m
// blockIdx.y selects the half (p or q), so modulus, exponent schedule and constants are
// wave-uniform: the modulus limbs live in SGPRs and the sliding window is a scalar op list.
#pragma once
#include "bn_lane.hpp"
#include "kernels.hpp"

namespace fpai {

constexpr int LANE_BLOCK = 256;
#ifndef FPAI_LANE_OCC
#define FPAI_LANE_OCC 1
#endif
constexpr int LANE_OCC = FPAI_LANE_OCC;   // waves per SIMD the exponentiation kernels are built for

// op list of the lane machine (run_lane_program)
enum : uint32_t {
  LOP_SQR = 1u, LOP_A_FROM_T = 2u, LOP_STORE = 4u, LOP_B_CONST = 8u,
  LOP_PREFETCH = 16u,   // SQR op: start the DMA tile[bidx] -> LDS multiplier before squaring (the next
                        // MUL's operand), so the HBM latency of the table row hides behind the squarings
  LOP_B_READY = 32u,    // MUL op: the LDS multiplier already holds the operand (prefetched or kept)
  LOP_B_SET = 64u,      // after the op: LDS multiplier <- a
  LOP_IOTA = 128u,      // k_dec4_pow (factored chain): before the op, the even lane's A goes to the LDS B half
};
constexpr int LANE_NTILE = 16;   // odd powers x^1 .. x^31
constexpr int KMAX_CHUNKS = 5;   // stage A reduces r of up to KMAX_CHUNKS * LB * SA bits
constexpr int RBUF_WORDS = 160;  // per-lane staging of the ChaCha stream (stage A)

struct CrtHalf {
  const uint32_t* m;        // modulus limbs (p_h for stage A, p_h^2 for stage B), S limbs
  const uint32_t* c0;       // stage A: R^(K+1) mod p_h for K = 1..KMAX_CHUNKS ([K-1][S]);
                            // stage B: R^2 mod p_h^2
  const uint32_t* c1;       // stage A: 1; stage B: CRT coefficient (q^2)^-1 mod p^2 (resp. (p^2)^-1 mod q^2)
  const uint32_t* prog;     // op list for x^e
  int nprog;
  uint32_t mprime;
};

struct CrtParams {
  const CrtHalf* halves;    // [2]
  long long n;              // elements
  // stage A inputs: obfuscator r
  int obf;                  // PAI_OBF_GIVEN (1) or PAI_OBF_RNG (2)
  const uint32_t* r;        // GIVEN: words, element i at r + i * r_stride
  long long r_stride;
  int r_words;              // words of r (GIVEN) or of the ChaCha stream (RNG)
  uint32_t rng_key[8];
  unsigned long long index_base;
  int kchunks;              // stage A: ceil(32 r_words / (LB SA)) <= KMAX_CHUNKS
  const uint32_t* yin;      // stage B input  [2][SA][n]
  uint32_t* out;            // stage A: y [2][SA][n]; stage B: u [2][SB][n]
  uint32_t* scratch;        // per-lane tiles
};

// Per-lane scratch, interleaved across the lanes of the grid in 16-byte quads: quad g of lane l
// lives at quad index g * NL + l (NL = lanes in the grid), so every wave access is 1 KiB
// contiguous and the address is a wave-uniform row base plus the lane. Tile k = quads
// [k TQ, (k+1) TQ) (TQ = ceil(S / 4)); stage A's ChaCha staging follows the tiles.
template <int S>
constexpr int tile_quads() { return (S + 3) / 4; }
template <int S>
constexpr size_t lane_scratch_words() {
  return ((size_t)LANE_NTILE * tile_quads<S>() + RBUF_WORDS / 4) * 4;
}
struct LaneScratch {
  uint4* scratch;      // grid scratch base (wave-uniform)
  uint32_t nl;         // lanes in the grid (wave-uniform)
  uint32_t lid;        // this lane
  __device__ __forceinline__ uint4& quad(int g) const { return scratch[(size_t)g * nl + lid]; }
};
__device__ __forceinline__ LaneScratch lane_scratch(uint32_t* scratch) {
  const uint32_t nl = gridDim.x * gridDim.y * blockDim.x;
  const uint32_t lid = (blockIdx.y * gridDim.x + blockIdx.x) * blockDim.x + threadIdx.x;
  return LaneScratch{reinterpret_cast<uint4*>(scratch), nl, lid};
}
template <int S>
__device__ __forceinline__ void unpack_quad(const uint4 v, int g, uint32_t (&x)[S]) {
  if (4 * g + 0 < S) x[4 * g + 0] = v.x;
  if (4 * g + 1 < S) x[4 * g + 1] = v.y;
  if (4 * g + 2 < S) x[4 * g + 2] = v.z;
  if (4 * g + 3 < S) x[4 * g + 3] = v.w;
}
template <int S>
__device__ __forceinline__ uint4 pack_quad(const uint32_t (&x)[S], int g) {
  uint4 v;
  v.x = 4 * g + 0 < S ? x[4 * g + 0] : 0u;
  v.y = 4 * g + 1 < S ? x[4 * g + 1] : 0u;
  v.z = 4 * g + 2 < S ? x[4 * g + 2] : 0u;
  v.w = 4 * g + 3 < S ? x[4 * g + 3] : 0u;
  return v;
}
template <int S>
__device__ __forceinline__ void ltile_load(const LaneScratch& t, int k, uint32_t (&x)[S]) {
  constexpr int TQ = tile_quads<S>();
#pragma unroll
  for (int g = 0; g < TQ; ++g) unpack_quad<S>(t.quad(k * TQ + g), g, x);
}
template <int S>
__device__ __forceinline__ void ltile_store(const LaneScratch& t, int k, const uint32_t (&x)[S]) {
  constexpr int TQ = tile_quads<S>();
#pragma unroll
  for (int g = 0; g < TQ; ++g) t.quad(k * TQ + g) = pack_quad<S>(x, g);
}
// DMA tile k -> the LDS multiplier ([quad][lane] image, 16 bytes per lane per instruction; the
// destination is the wave's 64-lane slice of quad row g). Completion: lds_dma_wait().
template <int S>
__device__ __forceinline__ void ltile_to_lds(const LaneScratch& t, int k, uint4* wave_row0) {
  constexpr int TQ = tile_quads<S>();
#pragma unroll
  for (int g = 0; g < TQ; ++g)
    __builtin_amdgcn_global_load_lds((const void*)&t.quad(k * TQ + g),
                                     (__attribute__((address_space(3))) void*)(wave_row0 + g * LANE_BLOCK), 16, 0, 0);
}
__device__ __forceinline__ void lds_dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// One op of the list through the scalar cache. The compiler will not use s_load here (the kernel
// stores to global memory, so it cannot prove the list invariant) and a vector load - or an LDS
// read, which it orders behind any LDS-DMA in flight - would make every op wait vmcnt(0) and so
// drain the multiplier prefetch. The list is written by the host before the launch and never
// changes, so the scalar cache is coherent for it.
__device__ __forceinline__ uint32_t lane_op(const uint32_t* __restrict__ prog, int i) {
  uint32_t v;
  asm volatile("s_load_dword %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(prog), "s"(i * 4));
  return v;
}

// The lane machine: per op (wave-uniform, scalar-loaded)
//   A_FROM_T : a <- tile[aidx]
//   SQR      : a <- a^2 R^-1   (PREFETCH: first start the DMA tile[bidx] -> LDS multiplier)
//   MUL      : a <- a * b R^-1 with b the LDS multiplier: const c1 (B_CONST), as is (B_READY) or
//              tile[bidx] (DMA now)
//   STORE    : tile[sidx] <- a
//   B_SET    : LDS multiplier <- a
// fields: bidx = op[15:8], aidx = op[23:16], sidx = op[31:24]. The kernel appends the final
// product with c1. The multiplier never occupies VGPRs: MUL reads one limb per CIOS step from LDS.
template <int S>
__device__ __forceinline__ void run_lane_program(uint32_t (&a)[S], const LaneScratch& t,
                                                 const uint32_t* __restrict__ prog, int nprog,
                                                 const uint32_t* __restrict__ c1, const uint32_t (&m)[S],
                                                 uint32_t mprime) {
  constexpr int TQ = tile_quads<S>();
  __shared__ uint4 ldsb[TQ * LANE_BLOCK];
  uint4* bcol = ldsb + threadIdx.x;
  uint4* brow = ldsb + (threadIdx.x & ~63u);
  for (int i = 0; i <= nprog; ++i) {
    const uint32_t op = (i < nprog) ? lane_op(prog, i) : LOP_B_CONST;
    if (op & LOP_A_FROM_T) {
      ltile_load<S>(t, (op >> 16) & 0xFF, a);
      // consume the loads here, inside the branch: otherwise the shared SQR/MUL code below starts
      // with the wait for them, which (vmcnt counts in order) also drains a prefetch DMA
#pragma unroll
      for (int j = 0; j < S; ++j) asm volatile("" : "+v"(a[j]));
    }
    if (op & LOP_SQR) {
      if (op & LOP_PREFETCH) ltile_to_lds<S>(t, (op >> 8) & 0xFF, brow);
      lane::mont_sqr<S>(a, m, mprime);
    } else {
      if (op & LOP_B_CONST) {
        uint32_t cv[S];
#pragma unroll
        for (int j = 0; j < S; ++j) cv[j] = c1[j];
#pragma unroll
        for (int g = 0; g < TQ; ++g) bcol[g * LANE_BLOCK] = pack_quad<S>(cv, g);
      } else if (!(op & LOP_B_READY)) {
        ltile_to_lds<S>(t, (op >> 8) & 0xFF, brow);
      }
      lds_dma_wait();
      lane::mont_mul_lds<S, LANE_BLOCK>(a, bcol, m, mprime);
    }
    if (op & LOP_STORE) ltile_store<S>(t, op >> 24, a);
    if (op & LOP_B_SET) {
#pragma unroll
      for (int g = 0; g < TQ; ++g) bcol[g * LANE_BLOCK] = pack_quad<S>(a, g);
    }
  }
}

// ---------------------------------------------------------------- stage A: y_h = r^(e_h) mod p_h
template <int SA>
__global__ __launch_bounds__(LANE_BLOCK, LANE_OCC) void k_crt_a(CrtParams p) {
  const int half = blockIdx.y;
  const CrtHalf* H = p.halves + half;
  uint32_t m[SA];
#pragma unroll
  for (int j = 0; j < SA; ++j) m[j] = H->m[j];
  const uint32_t mprime = H->mprime;
  const int nprog = H->nprog;
  const uint32_t* prog = H->prog;
  const uint32_t* c1 = H->c1;
  const uint32_t* cK = H->c0 + (size_t)(p.kchunks - 1) * SA;    // R^(K+1) mod p_h
  const LaneScratch tl = lane_scratch(p.scratch);
  for (long long base = (long long)blockIdx.x * LANE_BLOCK; base < p.n; base += (long long)gridDim.x * LANE_BLOCK) {
    const long long i = base + threadIdx.x;
    const long long ii = i < p.n ? i : p.n - 1;
    // r words: the caller's (GIVEN) or this element's ChaCha stream staged in the lane scratch
    const bool given = p.obf == 1;
    const uint32_t* rg = p.r + (given ? ii * p.r_stride : 0);
    if (!given) {
      const unsigned long long g = p.index_base + (unsigned long long)ii;
      for (int b = 0; b * 16 < p.r_words; ++b) {
        uint32_t blk[16];
        chacha20_block(p.rng_key, (uint32_t)b, (uint32_t)g, (uint32_t)(g >> 32), 0x66786169u, blk);
#pragma unroll
        for (int w = 0; w < 4; ++w)
          tl.quad(LANE_NTILE * tile_quads<SA>() + b * 4 + w) =
              make_uint4(blk[4 * w], blk[4 * w + 1], blk[4 * w + 2], blk[4 * w + 3]);
      }
    }
    auto rw = [&](int wi) -> uint32_t {
      if (given) return rg[wi];
      const uint4 v = tl.quad(LANE_NTILE * tile_quads<SA>() + (wi >> 2));
      const int c = wi & 3;
      return c == 0 ? v.x : c == 1 ? v.y : c == 2 ? v.z : v.w;
    };
    // x~ = r R mod p_h: K CIOS passes over the SA-limb chunks of r with a = R^(K+1) mod p_h
    // (invariant T < a + p_h < 2 p_h for any digits < 2^LB)
    uint32_t a[SA];
    {
      uint64_t P[SA];
#pragma unroll
      for (int j = 0; j < SA; ++j) P[j] = 0;
      const int nw = p.r_words;
#pragma unroll 1
      for (int k = 0; k < p.kchunks; ++k) {
        uint32_t b[SA], cst[SA];
#pragma unroll
        for (int j = 0; j < SA; ++j) {
          const int bit = (k * SA + j) * lane::LB, wi = bit >> 5, sh = bit & 31;
          const uint64_t lo = wi < nw ? (uint64_t)rw(wi) : 0ull;
          const uint64_t hi = wi + 1 < nw ? (uint64_t)rw(wi + 1) : 0ull;
          b[j] = (uint32_t)(((hi << 32) | lo) >> sh) & lane::LMASK;
          cst[j] = cK[j];
        }
        lane::mul_pass<SA>(P, cst, b, m, mprime);
      }
      lane::normalize<SA>(P, a);
    }
    ltile_store<SA>(tl, 0, a);
    run_lane_program<SA>(a, tl, prog, nprog, c1, m, mprime);   // ..., then * 1: leaves Montgomery form
    // y_h (< 2 p_h; any representative mod p_h gives the same y^p mod p_h^2 in stage B)
    if (i < p.n) {
#pragma unroll
      for (int j = 0; j < SA; ++j) p.out[((size_t)half * SA + j) * p.n + i] = a[j];
    }
  }
}

// ---------------------------------------------------------------- finish: c = (u_p q^2 + u_q p^2) c0 mod n^2
struct CrtFinParams {
  const void* x;
  int dtype, exp_mode, fexp;
  const uint32_t* u;        // [2][SB][n]
  int sb;
  long long n;
  const uint32_t* N;        // n^2 limbs (group layout, S = TPI*L)
  const uint32_t* nl;       // n limbs
  const uint32_t* kq;       // q^2 R^2 mod n^2
  const uint32_t* kp;       // p^2 R^2 mod n^2
  uint32_t mprime;
  uint32_t* ct;
  int32_t* exp;
  int32_t* status;
  int ct_words;
};

template <int TPI>
__global__ __launch_bounds__(BLOCK, 1) void k_crt_fin(CrtFinParams p) {
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
    int64_t M = 0;
    int e = 0, st;
    const bool fixed = p.exp_mode != 0;
    if (p.dtype == 0) st = encode_float((double)((const float*)p.x)[ii], fixed, p.fexp, M, e);
    else if (p.dtype == 1) st = encode_float(((const double*)p.x)[ii], fixed, p.fexp, M, e);
    else st = encode_int(((const int64_t*)p.x)[ii], fixed, p.fexp, M, e);
    // step 0: acc = u_p * q^2 R ; step 1: acc += u_q * p^2 R ; step 2: acc * c0
    uint32_t acc[L];
    for (int step = 0; step < 3; ++step) {
      uint32_t a[L];
      if (step < 2) {
        int t = tig;
        asm volatile("" : "+v"(t));
#pragma unroll
        for (int j = 0; j < L; ++j) {
          const int limb = t * L + j;
          a[j] = limb < p.sb ? p.u[((size_t)step * p.sb + limb) * p.n + ii] : 0u;
        }
        copy_g_to_lds<TPI>(slot, step == 0 ? p.kq : p.kp, tig);
      } else {
        uint32_t c0[L];
        make_c0<TPI>(M, p.nl, m, c0, lane, tig);
        write_limbs_lds<TPI>(slot, c0, tig);
#pragma unroll
        for (int j = 0; j < L; ++j) a[j] = acc[j];
      }
      montmul<TPI>(a, a, slot, TPI, m, p.mprime, lane, tig);
      if (step == 0) {
#pragma unroll
        for (int j = 0; j < L; ++j) acc[j] = a[j];
      } else if (step == 1) {
        uint64_t P[L];
#pragma unroll
        for (int j = 0; j < L; ++j) P[j] = (uint64_t)acc[j] + a[j];
        normalize<TPI>(P, acc, lane, tig);                       // < 4 n^2: fine as a montmul input
      } else {
#pragma unroll
        for (int j = 0; j < L; ++j) acc[j] = a[j];
      }
    }
    cond_sub<TPI>(acc, m, lane, tig);
    emit_words<TPI>(slot, acc, p.ct + ii * p.ct_words, p.ct_words, valid, tig);
    if (valid && tig == 0) {
      p.exp[ii] = e;
      if (p.status) p.status[ii] = st;
    }
  }
}

}  // namespace fpai
