// Paillier array kernels for gfx950. One element per lane group (encrypt / add) or per
// pair of lane groups (CRT decrypt: p-half and q-half side by side in one wavefront).
#pragma once
#include "bn_group.hpp"
#include "device_ops.hpp"

namespace fpai {

constexpr int BLOCK = 256;
constexpr int TABLE_ODD = 16;   // sliding window k=5: odd powers x^1..x^31
constexpr int TABLE_FIX = 32;   // fixed window k=5: x^0..x^31
constexpr int32_t PAD_EXP = INT32_MIN;   // exponent of a padding operand of k_add (the value 1, skipped)

struct EncParams {
  const void* x;
  int dtype, exp_mode, fexp, obf;
  const uint32_t* r;
  long long r_stride;   // words
  int r_words;
  int rng_words;
  uint32_t rng_key[8];
  unsigned long long index_base;
  uint32_t* ct;
  int32_t* exp;
  int32_t* status;
  long long n;
  const uint32_t* N;    // n^2, LB-bit limbs (S)
  const uint32_t* R2;   // R^2 mod n^2
  const uint32_t* nl;   // n limbs (S, zero padded)
  uint32_t mprime;
  const uint32_t* prog;  // Montgomery program (run_program)
  int nprog;
  uint32_t* scratch;
  int ct_words;
};

constexpr int ADD_KMAX = 64;     // operands per k_add launch (the R^s constants go up to s = ADD_KMAX + 1)
constexpr int ADD_TMAX = 1024;   // step-count buckets of the k_add schedule sort

struct AddParams {
  const uint32_t* cts;    // k x n x ct_words
  const int32_t* exps;    // k x n
  int k;
  uint32_t* out;
  int32_t* out_exp;
  long long n;
  const uint32_t* N;
  const uint32_t* RS;     // [ADD_KMAX + 2][ct_words]: R^s mod n^2, s = 0 .. ADD_KMAX + 1 (32-bit words)
  uint32_t mprime;
  int ct_words;
  // nullable: operand j of instance i is element gidx[i k + j] of the flat cts/exps arrays (-1: padding);
  // segmented sums (pai_segment_add) gather their members this way
  const long long* gidx;
  const int* perm;        // nullable: instance slot t processes instance perm[t] (schedule sort)
};

// Per-half (p: h=0, q: h=1) constants for CRT decryption; all LB-bit limb arrays of S limbs.
// Lives in device memory (indexed per lane by the half a lane works on).
struct DecHalf {
  const uint32_t* m;      // p^2
  const uint32_t* R3;     // R^3 mod p^2
  const uint32_t* one;    // R mod p^2
  const uint32_t* pneg;   // 2^(LB*S) - p
  const uint32_t* ph;     // p
  const uint32_t* hR;     // hp * R mod p
  const uint8_t* digits;  // exponent p-1 in 5-bit windows, most significant first
  uint32_t mprime, dprime, pprime, pad;
};

struct DecParams {
  const uint32_t* ct;
  const int32_t* exp;
  long long n;
  double* val;
  int64_t* mant;
  int32_t* status;
  uint32_t* raw;
  const DecHalf* halves;   // device array [2]
  const uint32_t* qinvR;   // q^-1 * R mod p
  const uint32_t* nlimb;   // n
  const uint32_t* qRn;     // q * R mod n
  const uint32_t* maxint;  // n // 3 - 1
  uint32_t nprime;
  int nwin;
  int ct_words, pt_words;
  int n_limbs;             // limbs actually used by n (<= S)
  uint32_t* scratch;
};

// ---------------------------------------------------------------- small helpers
template <int TPI>
__device__ __forceinline__ void load_limbs_g(const uint32_t* __restrict__ g, uint32_t (&x)[L], int tig) {
#pragma unroll
  for (int i = 0; i < L; ++i) x[i] = g[tig * L + i];
}
template <int TPI>
__device__ __forceinline__ void store_limbs_g(uint32_t* __restrict__ g, const uint32_t (&x)[L], int tig) {
#pragma unroll
  for (int i = 0; i < L; ++i) g[tig * L + i] = x[i];
}
template <int TPI>
__device__ __forceinline__ void copy_g_to_lds(uint32_t* slot, const uint32_t* __restrict__ g, int tig) {
  uint32_t t[L];
  load_limbs_g<TPI>(g, t, tig);
  write_limbs_lds<TPI>(slot, t, tig);
}
template <int TPI>
__device__ __forceinline__ void write_limbs_lds_if(uint32_t* slot, const uint32_t (&x)[L], int tig, bool pred) {
  wave_lds_fence();
  if (pred) {
#pragma unroll
    for (int i = 0; i < L; ++i) slot[tig * L + i] = x[i];
  }
  wave_lds_fence();
}
template <int TPI>
__device__ __forceinline__ void write_one_lds(uint32_t* slot, int tig) {
  uint32_t t[L];
#pragma unroll
  for (int i = 0; i < L; ++i) t[i] = (tig == 0 && i == 0) ? 1u : 0u;
  write_limbs_lds<TPI>(slot, t, tig);
}

// c0 = 1 + n*M mod n^2 (raw_encrypt.py:37-45; the "sneaky inverse" branch yields the same
// value). Branch-free across groups: both signs are computed and selected per group.
template <int TPI>
__device__ __forceinline__ void make_c0(int64_t M, const uint32_t* __restrict__ nl, const uint32_t (&m)[L],
                                        uint32_t (&c0)[L], int lane, int tig) {
  const bool neg = M < 0;
  const uint64_t mag = neg ? (uint64_t)0 - (uint64_t)M : (uint64_t)M;
  const uint32_t M0 = (uint32_t)mag & LMASK, M1 = (uint32_t)(mag >> LB) & LMASK, M2 = (uint32_t)(mag >> (2 * LB));
  uint64_t P[L];
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const int k = tig * L + i;
    const uint64_t a0 = nl[k];
    const uint64_t a1 = k >= 1 ? nl[k - 1] : 0u;
    const uint64_t a2 = k >= 2 ? nl[k - 2] : 0u;
    P[i] = a0 * M0 + a1 * M1 + a2 * M2;
  }
  uint32_t X[L], D[L];
  normalize<TPI>(P, X, lane, tig);
  (void)sub_limbs<TPI>(m, X, D, lane, tig);   // n^2 - n|M| (only used when M < 0)
#pragma unroll
  for (int i = 0; i < L; ++i) P[i] = (uint64_t)(neg ? D[i] : X[i]) + ((tig == 0 && i == 0) ? 1u : 0u);
  normalize<TPI>(P, c0, lane, tig);
}

// ---------------------------------------------------------------- Montgomery program machine
// Every modular product of an encrypt runs through ONE inlined montmul call site, driven by a
// host-built op list (wave-uniform, read with scalar loads). This keeps the kernel's register
// set at the montmul working set (P: 2L, a: L, m: L VGPRs) instead of one copy per call site,
// and the hot loop's code (L unrolled CIOS iterations) resident in the instruction cache.
//   op bit 0  B_FROM_A : LDS slot <- a             (squaring / multiply by the accumulator)
//   op bit 1  B_FROM_T : LDS slot <- tile[bidx]
//   op bit 2  A_FROM_T : a <- tile[aidx]
//   op bit 3  STORE    : tile[sidx] <- a (after the product)
//   fields    bidx = op[15:8], aidx = op[23:16], sidx = op[31:24]
// then a <- a * slot * R^-1 mod m. Tiles are per-lane scratch in global memory laid out
// [lane][tile][limb] (see lane_tiles).
enum : uint32_t { OP_B_FROM_A = 1u, OP_B_FROM_T = 2u, OP_A_FROM_T = 4u, OP_STORE = 8u };
constexpr int T_FINAL = TABLE_ODD;          // tile holding the final multiplier (c0, or 1)
constexpr int NTILE = TABLE_ODD + 1;
constexpr int TROW = (L + 3) & ~3;          // limbs per tile row, padded for 16-byte accesses
constexpr size_t TILE_WORDS_PER_LANE = (size_t)NTILE * TROW;

// Per-lane tiles, [lane][tile][TROW]: one 64-bit base per lane and immediate offsets (< 4 KiB)
// for every limb, 16-byte loads/stores. (A [tile][limb][lane] layout coalesces better but needs
// one 64-bit address per limb row, which the compiler hoists and keeps live: L*2 VGPRs.)
__device__ __forceinline__ uint32_t* lane_tiles(uint32_t* scratch) {
  return scratch + ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * TILE_WORDS_PER_LANE;
}
__device__ __forceinline__ void tile_load(const uint32_t* __restrict__ tl, int k, uint32_t (&x)[L], int /*lane*/) {
  const uint4* q = reinterpret_cast<const uint4*>(tl + k * TROW);
#pragma unroll
  for (int j = 0; j < TROW / 4; ++j) {
    const uint4 v = q[j];
    if (4 * j + 0 < L) x[4 * j + 0] = v.x;
    if (4 * j + 1 < L) x[4 * j + 1] = v.y;
    if (4 * j + 2 < L) x[4 * j + 2] = v.z;
    if (4 * j + 3 < L) x[4 * j + 3] = v.w;
  }
}
__device__ __forceinline__ void tile_store(uint32_t* __restrict__ tl, int k, const uint32_t (&x)[L], int /*lane*/) {
  uint4* q = reinterpret_cast<uint4*>(tl + k * TROW);
#pragma unroll
  for (int j = 0; j < TROW / 4; ++j) {
    uint4 v;
    v.x = 4 * j + 0 < L ? x[4 * j + 0] : 0u;
    v.y = 4 * j + 1 < L ? x[4 * j + 1] : 0u;
    v.z = 4 * j + 2 < L ? x[4 * j + 2] : 0u;
    v.w = 4 * j + 3 < L ? x[4 * j + 3] : 0u;
    q[j] = v;
  }
}

template <int TPI>
__device__ __forceinline__ void run_program(uint32_t (&a)[L], uint32_t* slot, uint32_t* __restrict__ tw,
                                            const uint32_t* __restrict__ prog, int nprog, const uint32_t (&m)[L],
                                            uint32_t mprime, int lane, int tig) {
  for (int i = 0; i <= nprog; ++i) {
    const uint32_t op = (i < nprog) ? __builtin_amdgcn_readfirstlane(prog[i]) : (OP_B_FROM_T | (T_FINAL << 8));
    if (op & OP_B_FROM_A) write_limbs_lds<TPI>(slot, a, tig);
    if (op & OP_B_FROM_T) {
      uint32_t t[L];
      tile_load(tw, (op >> 8) & 0xFF, t, lane);
      write_limbs_lds<TPI>(slot, t, tig);
    }
    if (op & OP_A_FROM_T) tile_load(tw, (op >> 16) & 0xFF, a, lane);
    montmul<TPI>(a, a, slot, TPI, m, mprime, lane, tig);
    if (op & OP_STORE) tile_store(tw, op >> 24, a, lane);
  }
}

// Write canonical limbs (S of them) of the group's result to LDS and emit `nwords` 32-bit
// little-endian words to global memory (lanes of the group interleave -> coalesced).
template <int TPI>
__device__ __forceinline__ void emit_words(uint32_t* slot, const uint32_t (&x)[L], uint32_t* __restrict__ out,
                                           int nwords, bool valid, int tig) {
  constexpr int S = TPI * L;
  write_limbs_lds<TPI>(slot, x, tig);
  if (valid) {
    for (int j = tig; j < nwords; j += TPI) out[j] = limbs_word(slot, S, j);
  }
  wave_lds_fence();
}

// Inverse of emit_words for a ciphertext-sized operand: the group copies `nwords` words (16-byte aligned,
// nwords % 4 == 0, nwords + 2 <= S) into its LDS slot with 16-byte loads, then each lane cuts its L limbs
// out of the slot (two words and one alignbit per limb). Used inside step loops, where the per-limb,
// bounds-checked word loads of words_to_limbs (74 scalar loads, 37 branches) spill registers.
template <int TPI>
__device__ __forceinline__ void stage_words_to_limbs(uint32_t* slot, const uint32_t* __restrict__ src, int nwords,
                                                     uint32_t (&x)[L], int tig) {
  const uint4* s4 = reinterpret_cast<const uint4*>(src);
  uint4* d4 = reinterpret_cast<uint4*>(slot);
  wave_lds_fence();                                   // earlier readers of the slot are done
  for (int q = tig; q < nwords / 4; q += TPI) d4[q] = s4[q];
  if (tig == 0) {
    slot[nwords] = 0u;
    slot[nwords + 1] = 0u;
  }
  wave_lds_fence();
  // opaque copy: stops LICM from hoisting the L per-limb (word index, shift) pairs out of the caller's
  // step loop, which would pin ~2L VGPRs for the whole kernel
  int t = tig;
  asm volatile("" : "+v"(t));
  const int base = t * L * LB;
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const int bit = base + i * LB, j = bit >> 5;
    const uint32_t lo = j < nwords + 2 ? slot[j] : 0u, hi = j + 1 < nwords + 2 ? slot[j + 1] : 0u;
    x[i] = __builtin_amdgcn_alignbit(hi, lo, bit & 31) & LMASK;
  }
  wave_lds_fence();                                   // the slot is rewritten next (write_limbs_lds)
}

// ================================================================= encrypt
// PaillierEncryptor.encrypt over an array (encryptor.py:71-114): encode -> c0 -> c0 * r^n mod n^2.
// The op list (host: build_encrypt_program) computes r~ = r R, the odd powers r~^1..r~^31 into
// tiles 0..15, the sliding-window chain over n, and finally multiplies by tile T_FINAL = c0,
// which also leaves the Montgomery domain: (r^n R) * c0 * R^-1 = c0 r^n.
template <int TPI>
__global__ __launch_bounds__(BLOCK, 2) void k_encrypt(EncParams p) {
  constexpr int S = TPI * L;
  constexpr int GPB = BLOCK / TPI;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int lane = threadIdx.x & 63;
  const int tig = threadIdx.x % TPI;
  const int gib = threadIdx.x / TPI;
  uint32_t* slot = smem + gib * S;
  uint32_t m[L];
  load_limbs_g<TPI>(p.N, m, tig);
  uint32_t* tw = lane_tiles(p.scratch);

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

    uint32_t a[L];
    make_c0<TPI>(M, p.nl, m, a, lane, tig);
    if (p.obf != 0) {
      tile_store(tw, T_FINAL, a, lane);
      if (p.obf == 1) {
        words_to_limbs(p.r + ii * p.r_stride, p.r_words, a, tig);
      } else {
        // ChaCha20 blocks tig, tig+TPI, ... of this element's stream -> LDS words -> limbs
        const unsigned long long gidx = p.index_base + (unsigned long long)ii;
        wave_lds_fence();
        for (int b = tig; b * 16 < p.rng_words; b += TPI) {
          uint32_t blk[16];
          chacha20_block(p.rng_key, (uint32_t)b, (uint32_t)gidx, (uint32_t)(gidx >> 32), 0x66786169u, blk);
#pragma unroll
          for (int w = 0; w < 16; ++w) slot[b * 16 + w] = blk[w];
        }
        wave_lds_fence();
        words_to_limbs(slot, p.rng_words, a, tig);
        wave_lds_fence();
      }
      copy_g_to_lds<TPI>(slot, p.R2, tig);
      run_program<TPI>(a, slot, tw, p.prog, p.nprog, m, p.mprime, lane, tig);
      cond_sub<TPI>(a, m, lane, tig);
    }
    emit_words<TPI>(slot, a, p.ct + ii * p.ct_words, p.ct_words, valid, tig);
    if (valid && tig == 0) {
      p.exp[ii] = e;
      if (p.status) p.status[ii] = st;
    }
  }
}

// ================================================================= k-way homomorphic add
// prod_j c_j^(16^(E - e_j)) mod n^2 (encrypted_number.py:115-137, 166-185), evaluated
// by Horner over the exponent levels instead of operand by operand:
//   acc = prod_{e_j = l0} c_j ;  for each next level l: acc = acc^(16^(l - l_prev)) * prod_{e_j = l} c_j
// so the 4 (E - e_j) alignment squarings of every operand become 4 (E - e_min) squarings of the running
// product (the value is the same integer mod n^2; the reference's sum is order independent). Operands
// enter in plain form; the Montgomery factor is tracked (rho: acc = value R^rho, rho = 1 - m after m plain
// operands of a level) and restored with ONE product by R^s mod n^2 per level change (s = 1 + m) and at
// the end (s = m), instead of one to-Montgomery product per operand.
//
// Every step is one Montgomery product acc * B with a per-group B (acc itself, an operand, or R^s), so
// the groups of a wave run in lock step; a group that is done multiplies by R (leaves acc unchanged).
// k_add_plan / k_add_scan / k_add_scatter sort the elements by their step count, so the 16 groups of a
// wave do (almost) the same number of steps.
__device__ __forceinline__ long long add_src(const AddParams& p, long long e, int j) {
  return p.gidx ? p.gidx[e * p.k + j] : (long long)j * p.n + e;
}
__device__ __forceinline__ int add_exp(const AddParams& p, long long src) { return src < 0 ? PAD_EXP : p.exps[src]; }

// Products the Horner schedule of instance e needs (0 for an all-padding instance).
__device__ __forceinline__ int add_steps(const AddParams& p, long long e, int& E) {
  int emin = INT32_MAX, keff = 0;
  E = PAD_EXP;
  for (int j = 0; j < p.k; ++j) {
    const int ej = add_exp(p, add_src(p, e, j));
    if (ej == PAD_EXP) continue;
    ++keff;
    E = max(E, ej);
    emin = min(emin, ej);
  }
  if (!keff) return 0;
  int levels = 0, cur = emin, last = 0;
  for (;;) {
    int cnt = 0, nl = INT32_MAX;
    for (int j = 0; j < p.k; ++j) {
      const int ej = add_exp(p, add_src(p, e, j));
      if (ej == PAD_EXP) continue;
      cnt += ej == cur;
      if (ej > cur && ej < nl) nl = ej;
    }
    ++levels;
    last = cnt;
    if (nl == INT32_MAX) break;
    cur = nl;
  }
  const long long t = (long long)(keff - 1) + 4ll * ((long long)E - emin) + (levels - 1) + (last >= 2 ? 1 : 0);
  return (int)min(t, (long long)INT32_MAX);
}

template <int DUMMY = 0>
__global__ __launch_bounds__(256) void k_add_plan(AddParams p, uint16_t* bucket, unsigned* hist) {
  __shared__ unsigned h[ADD_TMAX];
  for (int t = threadIdx.x; t < ADD_TMAX; t += blockDim.x) h[t] = 0u;
  __syncthreads();
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < p.n; e += (long long)gridDim.x * blockDim.x) {
    int E;
    const int b = min(add_steps(p, e, E), ADD_TMAX - 1);
    bucket[e] = (uint16_t)b;
    atomicAdd(&h[b], 1u);
  }
  __syncthreads();
  for (int t = threadIdx.x; t < ADD_TMAX; t += blockDim.x)
    if (h[t]) atomicAdd(&hist[t], h[t]);
}

// exclusive prefix sum of the ADD_TMAX bucket counts (one block of ADD_TMAX threads)
template <int DUMMY = 0>
__global__ __launch_bounds__(ADD_TMAX) void k_add_scan(unsigned* hist) {
  __shared__ unsigned v[ADD_TMAX];
  const int t = threadIdx.x;
  v[t] = hist[t];
  __syncthreads();
  for (int o = 1; o < ADD_TMAX; o <<= 1) {
    const unsigned x = t >= o ? v[t - o] : 0u;
    __syncthreads();
    v[t] += x;
    __syncthreads();
  }
  hist[t] = v[t] - hist[t];
}

template <int DUMMY = 0>
__global__ __launch_bounds__(256) void k_add_scatter(long long n, const uint16_t* bucket, unsigned* offs, int* perm) {
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x)
    perm[atomicAdd(&offs[bucket[e]], 1u)] = (int)e;
}

template <int TPI>
__global__ __launch_bounds__(BLOCK, 2) void k_add(AddParams p) {
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
    const long long el = p.perm ? (long long)p.perm[ii] : ii;
    // levels: E = max, cur = min exponent over the non-padding operands (padding counts as 1)
    int E = PAD_EXP, cur = INT32_MAX;
    for (int j = 0; j < p.k; ++j) {
      const int ej = add_exp(p, add_src(p, el, j));
      if (ej == PAD_EXP) continue;
      E = max(E, ej);
      cur = min(cur, ej);
    }
    const bool empty = E == PAD_EXP;
    uint32_t a[L];
    int jc = 0, sq = 0, mcount = 0;
    bool done = empty;
    if (!empty) {
      while (add_exp(p, add_src(p, el, jc)) != cur) ++jc;
      stage_words_to_limbs<TPI>(slot, p.cts + add_src(p, el, jc) * p.ct_words, p.ct_words, a, tig);   // rho = 0
      ++jc;
      mcount = 1;
    } else {
#pragma unroll
      for (int i = 0; i < L; ++i) a[i] = (tig == 0 && i == 0) ? 1u : 0u;
    }
#pragma clang loop unroll(disable)
    for (;;) {
      // this group's next step: 0 square, 1 times operand `osrc`, 2 times R^s, 3 nothing (times R)
      int op = 3, s = 1;
      long long osrc = 0;
      if (!done) {
        if (sq > 0) {
          op = 0;
          --sq;
        } else {
          while (jc < p.k && add_exp(p, add_src(p, el, jc)) != cur) ++jc;
          if (jc < p.k) {
            op = 1;
            osrc = add_src(p, el, jc);
            ++jc;
            ++mcount;                                // rho = 1 - mcount
          } else {
            int nl = INT32_MAX;
            for (int j = 0; j < p.k; ++j) {
              const int ej = add_exp(p, add_src(p, el, j));
              if (ej != PAD_EXP && ej > cur && ej < nl) nl = ej;
            }
            if (nl != INT32_MAX) {
              op = 2;
              s = 1 + mcount;                        // back to rho = 1 for the squarings
              sq = 4 * (nl - cur);
              cur = nl;
              jc = 0;
              mcount = 0;
            } else {
              done = true;
              if (mcount >= 2) {                     // rho = 1 - mcount -> 0
                op = 2;
                s = mcount;
              }
            }
          }
        }
      }
      if (ballot(op != 3) == 0ull) break;
      // branch-free B fill, so the kernel has ONE montmul site (a branch per kind of B makes the
      // compiler duplicate the 11k-instruction product per path)
      {
        const uint32_t* src = op == 1 ? p.cts + osrc * p.ct_words : p.RS + (size_t)s * p.ct_words;
        uint32_t t[L];
        stage_words_to_limbs<TPI>(slot, src, p.ct_words, t, tig);
#pragma unroll
        for (int i = 0; i < L; ++i) t[i] = op == 0 ? a[i] : t[i];
        write_limbs_lds<TPI>(slot, t, tig);
      }
      montmul<TPI>(a, a, slot, TPI, m, p.mprime, lane, tig);
    }
    cond_sub<TPI>(a, m, lane, tig);
    emit_words<TPI>(slot, a, p.out + el * p.ct_words, p.ct_words, valid, tig);
    if (valid && tig == 0) p.out_exp[el] = E;
  }
}

// ================================================================= CRT decrypt + decode
// decryptor.py:33-63 (mp = L(c^(p-1) mod p^2) * hp mod p, mq likewise, gmpy_math.crt :31-40) and
// FixedPointNumber.decode (fixedpoint_number.py:92-107). Lanes [0,TPI) of an element pair run the
// p-half, lanes [TPI,2TPI) the q-half, with identical control flow (fixed-window exponent).
__device__ __forceinline__ void decode_element(const uint32_t* xl, const DecParams& p, long long ii) {
  // xl: canonical limbs of the plaintext x in [0, n), in LDS; one lane.
  const int e = p.exp[ii];
  const int nl = p.n_limbs;
  int cmp_max = 0;   // sign(x - maxint)
  for (int k = nl - 1; k >= 0 && cmp_max == 0; --k) {
    const uint32_t a = xl[k], b = p.maxint[k];
    cmp_max = (a > b) - (a < b);
  }
  bool neg = false;
  int st = ST_OK;
  // |mantissa| is x (x <= maxint) or n - x (x >= n - maxint)
  uint32_t magv[160];
  if (cmp_max <= 0) {
    for (int k = 0; k < nl; ++k) magv[k] = xl[k];
  } else {
    int32_t b = 0;
    for (int k = 0; k < nl; ++k) {
      const int32_t v = (int32_t)p.nlimb[k] - (int32_t)xl[k] + b;
      magv[k] = (uint32_t)v & LMASK;
      b = v >> LB;
    }
    int c2 = 0;
    for (int k = nl - 1; k >= 0 && c2 == 0; --k) c2 = (magv[k] > p.maxint[k]) - (magv[k] < p.maxint[k]);
    if (c2 > 0) st = ST_OVERFLOW;
    neg = true;
  }
  double val = 0.0;
  int64_t mant = 0;
  if (st == ST_OK) {
    int top = nl - 1;
    while (top > 0 && magv[top] == 0) --top;
    const int B = (magv[top] == 0) ? 0 : top * LB + (32 - __clz(magv[top]));   // bit length
    const int lo_bit = B > 64 ? B - 64 : 0;
    uint64_t hi64 = 0;
    bool sticky = false;
    for (int k = top; k >= 0; --k) {
      const uint64_t v = magv[k];
      if (!v) continue;
      const int kb = k * LB;
      if (kb + LB <= lo_bit) { sticky = true; continue; }
      const int sh = kb - lo_bit;
      if (sh >= 0) {
        hi64 |= v << sh;
      } else {
        hi64 |= v >> (-sh);
        if (v & ((1ull << (-sh)) - 1ull)) sticky = true;
      }
    }
    double d;
    if (B <= 53) {
      d = (double)hi64;
    } else {
      const int drop = (B > 64 ? 64 : B) - 53;
      uint64_t keep = hi64 >> drop;
      const uint64_t rem = hi64 & ((1ull << drop) - 1ull);
      const uint64_t half = 1ull << (drop - 1);
      if (rem > half || (rem == half && (sticky || (keep & 1ull)))) keep += 1;
      d = ldexp((double)keep, lo_bit + drop);
    }
    if (e > 0) {
      if (isinf(d) || B > 1024) st = ST_FLOAT_OVF;
      else val = (neg ? -d : d) * ldexp(1.0, -4 * e);
    } else {
      val = ldexp(neg ? -d : d, -4 * e);
      const int sh = -4 * e;
      if (B + sh <= 63) {
        const int64_t mm = (int64_t)(hi64 << sh);
        mant = neg ? -mm : mm;
        st = ST_INT;
      } else {
        st = ST_INT_BIG;
      }
    }
  }
  p.val[ii] = val;
  if (p.mant) p.mant[ii] = mant;
  p.status[ii] = st;
}

template <int TPI>
__global__ __launch_bounds__(BLOCK) void k_decrypt(DecParams p) {
  constexpr int S = TPI * L;
  constexpr int EPB = BLOCK / (2 * TPI);     // elements per block
  constexpr int SLOT = 4 * S;                // [c: 2S limbs][B_p: S][B_q: S]; [0,2S) reused later
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int lane = threadIdx.x & 63;
  const int tig = threadIdx.x % TPI;
  const int h = (threadIdx.x / TPI) & 1;
  const int eib = threadIdx.x / (2 * TPI);
  const int pair_lane = threadIdx.x % (2 * TPI);
  uint32_t* eslot = smem + eib * SLOT;
  uint32_t* bslot = eslot + 2 * S + h * S;   // this half's multiplicand
  const DecHalf* H = p.halves + h;
  const DecHalf* H0 = p.halves;
  uint32_t m[L];
  load_limbs_g<TPI>(H->m, m, tig);
  const uint32_t mprime = H->mprime;
  uint32_t* table = p.scratch + ((size_t)(blockIdx.x * EPB + eib) * 2 + h) * TABLE_FIX * S;

  for (long long base = (long long)blockIdx.x * EPB; base < p.n; base += (long long)gridDim.x * EPB) {
    const long long inst = base + eib;
    const bool valid = inst < p.n;
    const long long ii = valid ? inst : p.n - 1;

    // 1. ciphertext (2*nb bits) -> 2S limbs in the element's shared region
    {
      const uint32_t* cw = p.ct + ii * p.ct_words;
      wave_lds_fence();
      for (int k = pair_lane; k < 2 * S; k += 2 * TPI) {
        const int bit = k * LB, wi = bit >> 5, sh = bit & 31;
        const uint64_t lo = wi < p.ct_words ? (uint64_t)cw[wi] : 0ull;
        const uint64_t hi = wi + 1 < p.ct_words ? (uint64_t)cw[wi + 1] : 0ull;
        eslot[k] = (uint32_t)(((hi << 32) | lo) >> sh) & LMASK;
      }
      wave_lds_fence();
    }
    // 2. x~ = c * R mod p^2: 2S-iteration Montgomery pass with A = R^3 mod p^2, B = c
    uint32_t xt[L], acc[L], t[L];
    load_limbs_g<TPI>(H->R3, t, tig);
    montmul<TPI>(xt, t, eslot, 2 * TPI, m, mprime, lane, tig);
    // 3. fixed-window table x~^0 .. x~^31 (global scratch)
    load_limbs_g<TPI>(H->one, t, tig);
    store_limbs_g<TPI>(table, t, tig);
    store_limbs_g<TPI>(table + S, xt, tig);
    write_limbs_lds<TPI>(bslot, xt, tig);
#pragma unroll
    for (int i = 0; i < L; ++i) t[i] = xt[i];
    for (int k = 2; k < TABLE_FIX; ++k) {
      montmul<TPI>(t, t, bslot, TPI, m, mprime, lane, tig);
      store_limbs_g<TPI>(table + k * S, t, tig);
    }
    // 4. left-to-right fixed windows over p-1 (resp. q-1): identical trip counts in both halves
    load_limbs_g<TPI>(table + H->digits[0] * S, acc, tig);
    for (int w = 1; w < p.nwin; ++w) {
#pragma unroll 1
      for (int s = 0; s < 5; ++s) {
        write_limbs_lds<TPI>(bslot, acc, tig);
        montmul<TPI>(acc, acc, bslot, TPI, m, mprime, lane, tig);
      }
      write_limbs_lds<TPI>(bslot, acc, tig);
      load_limbs_g<TPI>(table + H->digits[w] * S, t, tig);
      montmul<TPI>(acc, t, bslot, TPI, m, mprime, lane, tig);
    }
    // 5. leave the Montgomery domain: x_h = c^(p_h - 1) mod p_h^2, canonical
    write_one_lds<TPI>(bslot, tig);
    montmul<TPI>(acc, acc, bslot, TPI, m, mprime, lane, tig);
    cond_sub<TPI>(acc, m, lane, tig);
    // 6. L_h = (x_h - 1) / p_h exactly: Hensel division digits (x - 1 == x + 2^(27S) - 1 mod 2^(27S))
    uint32_t Ld[L], pl[L];
    {
      uint64_t P[L];
#pragma unroll
      for (int i = 0; i < L; ++i) {
        P[i] = (uint64_t)acc[i] + LMASK;
        Ld[i] = 0;
      }
      load_limbs_g<TPI>(H->pneg, pl, tig);
      uint32_t dummy[L];
      cios<TPI, false, true>(P, dummy, nullptr, TPI, pl, H->dprime, tig, Ld);
    }
    // 7. m_h = L_h * h_h mod p_h (hR = h_h * R mod p_h)
    load_limbs_g<TPI>(H->ph, pl, tig);
    copy_g_to_lds<TPI>(bslot, H->hR, tig);
    uint32_t mh[L];
    montmul<TPI>(mh, Ld, bslot, TPI, pl, H->pprime, lane, tig);
    cond_sub<TPI>(mh, pl, lane, tig);
    // 8. CRT (both halves compute, the p-half's result is kept):
    //    u = (mp*qinv - mq*qinv) mod p ; x = mq + u*q      (gmpy_math.py:31-40)
    write_limbs_lds<TPI>(eslot + h * S, mh, tig);     // region 0: mp, region 1: mq
    uint32_t mp[L], mq[L];
#pragma unroll
    for (int i = 0; i < L; ++i) {
      mp[i] = eslot[tig * L + i];
      mq[i] = eslot[S + tig * L + i];
    }
    wave_lds_fence();
    uint32_t p0[L], a1[L], a2[L], u[L];
    load_limbs_g<TPI>(H0->ph, p0, tig);
    copy_g_to_lds<TPI>(bslot, p.qinvR, tig);
    montmul<TPI>(a1, mp, bslot, TPI, p0, H0->pprime, lane, tig);
    cond_sub<TPI>(a1, p0, lane, tig);
    montmul<TPI>(a2, mq, bslot, TPI, p0, H0->pprime, lane, tig);
    cond_sub<TPI>(a2, p0, lane, tig);
    {
      const bool neg = sub_limbs<TPI>(a1, a2, u, lane, tig);
      uint64_t P[L];
#pragma unroll
      for (int i = 0; i < L; ++i) P[i] = (uint64_t)u[i] + (neg ? p0[i] : 0u);
      normalize<TPI>(P, u, lane, tig);              // (mp - mq) qinv mod p, in [0, p)
    }
    uint32_t nlm[L], uq[L], x[L];
    load_limbs_g<TPI>(p.nlimb, nlm, tig);
    copy_g_to_lds<TPI>(bslot, p.qRn, tig);
    montmul<TPI>(uq, u, bslot, TPI, nlm, p.nprime, lane, tig);   // u * q mod n
    cond_sub<TPI>(uq, nlm, lane, tig);
    {
      uint64_t P[L];
#pragma unroll
      for (int i = 0; i < L; ++i) P[i] = (uint64_t)uq[i] + mq[i];
      normalize<TPI>(P, x, lane, tig);
    }
    // 9. outputs from the p-half: raw plaintext words and the decoded value
    write_limbs_lds_if<TPI>(eslot, x, tig, h == 0);
    if (valid && h == 0 && p.raw) {
      for (int j = tig; j < p.pt_words; j += TPI) p.raw[ii * p.pt_words + j] = limbs_word(eslot, S, j);
    }
    if (valid && h == 0 && tig == 0) decode_element(eslot, p, ii);
    wave_lds_fence();
  }
}

}  // namespace fpai

namespace fpai {
// Debug/unit-test kernel for the group engine (used by tests/test_gpu_engine.py only).
// op 0: a*b*R^-1 mod N (< 2N) | 1: a -> limbs -> words | 2: c0(M = int64 from a[0..1])
// op 3: MontMul(MontMul(a, R2), 1) | 4: a^n mod N via the sliding-window modexp
// op 5: cond_sub(a, N) | 6: sub_limbs(a, b) (wrapped) | 7: normalize(a + b)
struct DbgParams {
  int op;
  const uint32_t* a;
  const uint32_t* b;
  uint32_t* out;
  int32_t* flag;
  long long n;
  int words;
  const uint32_t* N;
  const uint32_t* R2;
  const uint32_t* nl;
  uint32_t mprime;
  const uint32_t* prog;
  int nprog;
  uint32_t* scratch;
};

template <int TPI>
__global__ __launch_bounds__(BLOCK) void k_debug(DbgParams p) {
  constexpr int S = TPI * L;
  constexpr int GPB = BLOCK / TPI;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int lane = threadIdx.x & 63;
  const int tig = threadIdx.x % TPI;
  const int gib = threadIdx.x / TPI;
  uint32_t* slot = smem + gib * S;
  uint32_t m[L];
  load_limbs_g<TPI>(p.N, m, tig);
  const long long inst = (long long)blockIdx.x * GPB + gib;
  const bool valid = inst < p.n;
  const long long ii = valid ? inst : p.n - 1;
  uint32_t a[L], b[L], r[L];
  words_to_limbs(p.a + ii * p.words, p.words, a, tig);
  words_to_limbs(p.b + ii * p.words, p.words, b, tig);
  int flag = 0;
  if (p.op == 0) {
    write_limbs_lds<TPI>(slot, b, tig);
    montmul<TPI>(r, a, slot, TPI, m, p.mprime, lane, tig);
  } else if (p.op == 1) {
#pragma unroll
    for (int i = 0; i < L; ++i) r[i] = a[i];
  } else if (p.op == 2) {
    const int64_t M = (int64_t)(((uint64_t)p.a[ii * p.words + 1] << 32) | p.a[ii * p.words]);
    make_c0<TPI>(M, p.nl, m, r, lane, tig);
  } else if (p.op == 3) {
    uint32_t t[L];
    copy_g_to_lds<TPI>(slot, p.R2, tig);
    montmul<TPI>(t, a, slot, TPI, m, p.mprime, lane, tig);
    write_one_lds<TPI>(slot, tig);
    montmul<TPI>(r, t, slot, TPI, m, p.mprime, lane, tig);
  } else if (p.op == 4) {
    uint32_t* tw = lane_tiles(p.scratch);
    uint32_t one[L];
#pragma unroll
    for (int i = 0; i < L; ++i) one[i] = (tig == 0 && i == 0) ? 1u : 0u;
    tile_store(tw, T_FINAL, one, lane);
#pragma unroll
    for (int i = 0; i < L; ++i) r[i] = a[i];
    copy_g_to_lds<TPI>(slot, p.R2, tig);
    run_program<TPI>(r, slot, tw, p.prog, p.nprog, m, p.mprime, lane, tig);
    cond_sub<TPI>(r, m, lane, tig);
  } else if (p.op == 5) {
#pragma unroll
    for (int i = 0; i < L; ++i) r[i] = a[i];
    cond_sub<TPI>(r, m, lane, tig);
  } else if (p.op == 6) {
    flag = sub_limbs<TPI>(a, b, r, lane, tig) ? 1 : 0;
  } else {
    uint64_t P[L];
#pragma unroll
    for (int i = 0; i < L; ++i) P[i] = (uint64_t)a[i] + b[i];
    normalize<TPI>(P, r, lane, tig);
  }
  emit_words<TPI>(slot, r, p.out + ii * p.words, p.words, valid, tig);
  if (valid && tig == 0) p.flag[ii] = flag;
}
}  // namespace fpai
