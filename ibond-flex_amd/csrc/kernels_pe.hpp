// Public-key encryption on split pairs (kernels_dec4.hpp's device) for 2048-bit keys: c = c0 r^n mod n^2
// (raw_encrypt.py:22-49, obfuscator.py:23-37) with every product mod n^2 a pair product over the 74 limbs
// of n. The pair algebra of bn_pair.hpp needs nothing of the modulus but gcd(R, n) = 1 -- v = A + n B
// (mod n^2) works for n as it does for p_h -- so the parties that hold only the public key get the same
// 5 S^2 against 8 S^2 trade as the key holder:
//
//   k_pe_pre   encode (fixedpoint_number.py:46-90) -> M, exponent, status; r R mod n^2 as a pair: the constant
//              pair of R^3 times r's 2 S digits (explicit r, or the element's ChaCha20 stream exactly as
//              k_encrypt draws it), one split CIOS
//   k_pe_pow   (r R)^n by the lane machine's op list for the exponent n, the final product with the pair of
//              c0 = 1 + n M, i.e. (1, M mod n): the plain pair of c
//   k_pe_fin   the canonical pair -> c = A + n B (< n^2) -> ciphertext words
//
// Round 5, the factored chain (kernels_dec4.hpp d4f_run<S, true>): x^n mod n^2 depends on x mod n
// only, so the base is the B-free (A_r, 0) and the window table its 30 one-pass mm-powers; the chain over n multiplies
// by the entries' A parts (a_t, 0) only (one pass instead of two) and the dropped factors (1 + n b_t), b_t = H_t / a_t,
// are restored at the end by the closing Horner sum in iota = A_r^-1 R^2 mod n. There is no Fermat chain for that
// inverse (n's factors are secret), so it comes from ONE batch inversion per chunk (Montgomery's trick on the group
// engine, kernels_mul.hpp k_inv_up/down, one host inversion mod n^2):
//   k_pe_awords  A_r mod n (the pair's A limbs, reduced) -> words [n][W] for the batch inversion mod n (round 5, later: it
//                had run mod n^2 on the TPI = 4 engine, 4x the work for the same iota)
//   k_pe_iota    iota = REDC(R^3 A_r^-1) = A_r^-1 R^2 mod n -- one split CIOS over the inverse's S digits
//   k_pe_pow_f   the factored chain, then (A_Z, B_Z + A_Z (delta + M)): the plain pair of c, as k_pe_pow's
// A chunk whose A_r has no inverse (probability ~2^-1023) takes k_pe_pow instead (flexpai.hip launch_pe).
#pragma once
#include "kernels_dec4.hpp"

namespace fpai {

struct PeConst {
  const uint32_t* nl;      // n, S limbs
  const uint32_t* X1;      // (1 - R) mod n
  const uint32_t* XK;      // (1 - R^2) mod n
  const uint32_t* cK;      // pair of R^3 mod n^2
  const uint32_t* prog;    // op list for the exponent n
  int nprog;
  uint32_t mprime;         // -n^-1 mod 2^28
  // the factored chain (k_pe_pow_f)
  const uint32_t* progf;   // op list: the table of (A_r, 0), the chain over n with B-free multipliers, (1, 0) -> D4F_G
  int nprogf;
  const uint32_t* kf;      // [16][S] K'_t of the closing Horner sum
  const uint32_t* r2n;     // R^2 mod n
};

struct PeParams {
  const PeConst* k;
  const void* x;
  int dtype, exp_mode, fexp, obf;
  const uint32_t* r;       // GIVEN: words, element i at r + i r_stride
  long long r_stride;
  int r_words, rng_words;
  uint32_t rng_key[8];
  unsigned long long index_base;
  long long n;
  uint32_t* xw;            // [2S][n] pairs
  int64_t* M;              // [n] encodings (k_pe_pre -> k_pe_pow)
  uint32_t* aw;            // [n][aw_words] A_r mod n as words, then its inverse mod n (k_pe_awords -> batch inversion -> k_pe_iota)
  int aw_words;            // words of n
  uint32_t* iota;          // [S][n] A_r^-1 R^2 mod n (k_pe_iota -> k_pe_pow_f)
  const uint32_t* noinv;   // the factored chain's device flag (flexpai.hip batch_invert_async), or null: when set, 1 = no
                           // inverse exists (k_pe_iota / k_pe_pow_f exit, k_pe_pow runs), 0 = k_pe_pow exits
  uint32_t* scratch;
  uint32_t* ct;
  int ct_words;
  int32_t* exp;
  int32_t* status;
};

template <int S>
__global__ __launch_bounds__(LANE_BLOCK, 1) void k_pe_pre(PeParams p) {
  __shared__ uint32_t lds[D4_PAIRS * D4_SLOT];
  const PeConst* K = p.k;
  uint32_t m[S];
#pragma unroll
  for (int j = 0; j < S; ++j) m[j] = (uint32_t)__builtin_amdgcn_readfirstlane(K->nl[j]);   // SGPRs: with 74 VGPRs of modulus the pass kept P in AGPRs (11 k moves, 1.8 k scratch accesses per pass)
  const uint32_t mprime = K->mprime;
  const int tig = threadIdx.x & 1;
  const bool odd = tig != 0;
  const int pib = threadIdx.x >> 1;
  uint32_t* sx = lds + pib * D4_SLOT;
  for (long long base = (long long)blockIdx.x * D4_PAIRS; base < p.n; base += (long long)gridDim.x * D4_PAIRS) {
    const long long e = base + pib;
    const bool valid = e < p.n;
    const long long ee = valid ? e : p.n - 1;
    if (valid && tig == 0) {   // encode (fixedpoint_number.py:46-90): M for k_pe_pow's final product
      int64_t M = 0;
      int ex = 0, stt;
      const bool fixed = p.exp_mode != 0;
      if (p.dtype == 0) stt = encode_float((double)((const float*)p.x)[ee], fixed, p.fexp, M, ex);
      else if (p.dtype == 1) stt = encode_float(((const double*)p.x)[ee], fixed, p.fexp, M, ex);
      else stt = encode_int(((const int64_t*)p.x)[ee], fixed, p.fexp, M, ex);
      p.M[e] = M;
      p.exp[e] = ex;
      if (p.status) p.status[e] = stt;
    }
    // r's words -> sx[2S .. 4S) (staging), its 2S 28-bit digits -> sx[0 .. 2S) (each lane half of them)
    uint32_t* wbuf = sx + 2 * S;
    d4_fence();
    int nw;
    if (p.obf == 1) {
      nw = p.r_words;
      const uint32_t* rg = p.r + ee * p.r_stride;
      for (int w = tig; w < nw; w += 2) wbuf[w] = rg[w];
    } else {
      nw = p.rng_words;
      const unsigned long long g = p.index_base + (unsigned long long)ee;
      for (int b = tig; b * 16 < nw; b += 2) {
        uint32_t blk[16];
        chacha20_block(p.rng_key, (uint32_t)b, (uint32_t)g, (uint32_t)(g >> 32), 0x66786169u, blk);
#pragma unroll
        for (int w = 0; w < 16; ++w)
          if (b * 16 + w < nw) wbuf[b * 16 + w] = blk[w];
      }
    }
    d4_fence();
    for (int k = tig * S; k < (tig + 1) * S; ++k) {
      const int bit = k * lane::LB, wi = bit >> 5, sh = bit & 31;
      const uint64_t lo = wi < nw ? (uint64_t)wbuf[wi] : 0ull;
      const uint64_t hi = wi + 1 < nw ? (uint64_t)wbuf[wi + 1] : 0ull;
      sx[k] = (uint32_t)(((hi << 32) | lo) >> sh) & lane::LMASK;
    }
    d4_fence();
    uint32_t a[S];
#pragma unroll
    for (int i = 0; i < S; ++i) a[i] = K->cK[tig * S + i];
    uint64_t P[S];
#pragma unroll
    for (int i = 0; i < S; ++i) P[i] = 0;
d4_pass<S>(P, a, sx, 0, m, mprime, odd, std::make_integer_sequence<int, S>{});
    d4_pass<S>(P, a, sx + S, 0, m, mprime, odd, std::make_integer_sequence<int, S>{});
    uint32_t y[S];
    lane::normalize<S>(P, y);
    if (valid) {
#pragma unroll
      for (int i = 0; i < S; ++i) p.xw[((size_t)tig * S + i) * p.n + e] = y[i];
    }
  }
}

template <int S>
__global__ __launch_bounds__(LANE_BLOCK, 2) void k_pe_pow(PeParams p) {
  if (p.noinv && *p.noinv == 0u) return;   // the factored chain ran
  constexpr int TQ = tile_quads<S>();
  using Q = std::make_integer_sequence<int, TQ>;
  __shared__ uint32_t lds[D4_PAIRS * D4R_SLOT + S];
  const PeConst* K = p.k;
  uint32_t m[S];
#pragma unroll
  for (int j = 0; j < S; ++j) m[j] = K->nl[j];
  const uint32_t mprime = K->mprime;
  const int nprog = K->nprog;
  const uint32_t* prog = K->prog;
  uint32_t* x1 = lds + D4_PAIRS * D4R_SLOT;   // (1 - R) mod n: the odd row's start in squares
  for (int i = threadIdx.x; i < S; i += blockDim.x) x1[i] = K->X1[i];
  __syncthreads();
  const int tig = threadIdx.x & 1;
  const int pib = threadIdx.x >> 1;
  uint32_t* st = lds + pib * D4R_SLOT;
  const LaneScratch tl = lane_scratch(p.scratch);
  for (long long base = (long long)blockIdx.x * D4_PAIRS; base < p.n; base += (long long)gridDim.x * D4_PAIRS) {
    const long long e = base + pib;
    const bool valid = e < p.n;
    const long long ee = valid ? e : p.n - 1;
    uint32_t a[S];   // this lane's component (kernels_dec4.hpp d4r_run: the even lane A, the odd lane B)
#pragma unroll
    for (int i = 0; i < S; ++i) a[i] = p.xw[((size_t)tig * S + i) * p.n + ee];
    d4r_tile_store<S>(tl, 0, a, Q{});
    // the final multiplier: the pair of c0 = 1 + n M = (1, M mod n) (M < 0: n - |M|)
    // (captures by value: a reference to a register array would force it into scratch)
    const int64_t* Mp = p.M;
    const uint32_t* nlp = K->nl;
    d4r_run<S>(a, st, tl, prog, nprog, x1, m, mprime, tig, [=](uint32_t* dst) {
      if (tig == 0) {
#pragma unroll
        for (int j = 0; j < S; ++j) dst[j] = j == 0 ? 1u : 0u;
      } else {
        const int64_t M = Mp[ee];
        const bool neg = M < 0;
        const uint64_t mag = neg ? (uint64_t)0 - (uint64_t)M : (uint64_t)M;
        int32_t br = 0;
#pragma unroll
        for (int j = 0; j < S; ++j) {
          const uint32_t mj = j < 3 ? (uint32_t)(mag >> (lane::LB * j)) & lane::LMASK : 0u;
          const int32_t v = neg ? (int32_t)nlp[j] - (int32_t)mj + br : (int32_t)mj;
          dst[j] = (uint32_t)v & lane::LMASK;
          br = v >> lane::LB;
        }
      }
    });
    if (valid) {
#pragma unroll
      for (int i = 0; i < S; ++i) p.xw[((size_t)tig * S + i) * p.n + e] = a[i];
    }
  }
}

// A_r -> words [n][ct_words] (the value < 2n zero-extended) for the batch inversion mod n^2
template <int S>
__global__ __launch_bounds__(LANE_BLOCK) void k_pe_awords(PeParams p) {
  for (long long i = (long long)blockIdx.x * LANE_BLOCK + threadIdx.x; i < p.n; i += (long long)gridDim.x * LANE_BLOCK) {
    uint32_t a[S], m[S];
#pragma unroll
    for (int j = 0; j < S; ++j) {
      a[j] = p.xw[(size_t)j * p.n + i];
      m[j] = p.k->nl[j];
    }
    lane::cond_sub<S>(a, m);   // A < 2n -> A mod n (the inverse mod n is what iota needs)
    lane::cond_sub<S>(a, m);
    uint32_t* w = p.aw + (size_t)i * p.aw_words;
#pragma unroll
    for (int k = 0; k < (S * lane::LB + 31) / 32; ++k) {
      const int bit = 32 * k, j = bit / lane::LB, sh = bit - j * lane::LB;
      uint64_t v = (uint64_t)a[j] >> sh;
      if (j + 1 < S) v |= (uint64_t)a[j + 1] << (lane::LB - sh);
      if (j + 2 < S && 2 * lane::LB - sh < 32) v |= (uint64_t)a[j + 2] << (2 * lane::LB - sh);
      if (k < p.aw_words) w[k] = (uint32_t)v;   // (A mod n < n: the words past n's are zero)
    }
    for (int k = (S * lane::LB + 31) / 32; k < p.aw_words; ++k) w[k] = 0u;
  }
}

// iota = REDC(R^3 inv) = inv R^2 mod n, inv = A_r^-1 mod n from p.aw: one split CIOS over the inverse's S digits
// (staged in LDS) by the pair of R^3 (k_pe_pre's constant), the even lane's row (the A component: R^3 mod n)
template <int S>
__global__ __launch_bounds__(LANE_BLOCK, 1) void k_pe_iota(PeParams p) {
  if (p.noinv && *p.noinv != 0u) return;   // no inverse: the general chain (k_pe_pow) instead
  __shared__ uint32_t lds[D4_PAIRS * D4_SLOT];
  const PeConst* K = p.k;
  uint32_t m[S];
#pragma unroll
  for (int j = 0; j < S; ++j) m[j] = K->nl[j];
  const uint32_t mprime = K->mprime;
  const int tig = threadIdx.x & 1;
  const bool odd = tig != 0;
  const int pib = threadIdx.x >> 1;
  uint32_t* sx = lds + pib * D4_SLOT;
  for (long long base = (long long)blockIdx.x * D4_PAIRS; base < p.n; base += (long long)gridDim.x * D4_PAIRS) {
    const long long e = base + pib;
    const bool valid = e < p.n;
    const long long ee = valid ? e : p.n - 1;
    uint32_t* wbuf = sx + 2 * S;
    const int nw = p.aw_words;
    d4_fence();
    for (int w = tig; w < nw; w += 2) wbuf[w] = p.aw[(size_t)ee * nw + w];
    d4_fence();
    for (int k = tig * S; k < (tig + 1) * S; ++k) {
      const int bit = k * lane::LB, wi = bit >> 5, sh = bit & 31;
      const uint64_t lo = wi < nw ? (uint64_t)wbuf[wi] : 0ull;
      const uint64_t hi = wi + 1 < nw ? (uint64_t)wbuf[wi + 1] : 0ull;
      sx[k] = (uint32_t)(((hi << 32) | lo) >> sh) & lane::LMASK;
    }
    d4_fence();
    uint32_t a[S];
#pragma unroll
    for (int i = 0; i < S; ++i) a[i] = K->cK[tig * S + i];
    uint64_t P[S];
#pragma unroll
    for (int i = 0; i < S; ++i) P[i] = 0;
    d4_pass<S>(P, a, sx, 0, m, mprime, odd, std::make_integer_sequence<int, S>{});
    uint32_t y[S];
    lane::normalize<S>(P, y);
    if (valid && !odd) {
#pragma unroll
      for (int i = 0; i < S; ++i) p.iota[(size_t)i * p.n + e] = y[i];
    }
  }
}

// the factored chain (d4f_run<S, true>): the plain pair of c = c0 r^n, as k_pe_pow
template <int S>
__global__ __launch_bounds__(LANE_BLOCK, 2) void k_pe_pow_f(PeParams p) {
  if (p.noinv && *p.noinv != 0u) return;
  __shared__ uint32_t lds[D4_PAIRS * D4R_SLOT + 2 * S];
  const PeConst* K = p.k;
  uint32_t m[S];
#pragma unroll
  for (int j = 0; j < S; ++j) m[j] = K->nl[j];
  const uint32_t mprime = K->mprime;
  uint32_t* x1 = lds + D4_PAIRS * D4R_SLOT;   // (1 - R) mod n: the odd row's start in squares
  uint32_t* kb = x1 + S;                       // K'_t of the current Horner step, then R^2 mod n (block-wide)
  for (int i = threadIdx.x; i < S; i += blockDim.x) x1[i] = K->X1[i];
  __syncthreads();
  const int tig = threadIdx.x & 1;
  const int pib = threadIdx.x >> 1;
  uint32_t* st = lds + pib * D4R_SLOT;
  const LaneScratch tl = lane_scratch(p.scratch);
  for (long long base = (long long)blockIdx.x * D4_PAIRS; base < p.n; base += (long long)gridDim.x * D4_PAIRS) {
    const long long e = base + pib;
    const bool valid = e < p.n;
    const long long ee = valid ? e : p.n - 1;
    uint32_t a[S];
#pragma unroll
    for (int i = 0; i < S; ++i) a[i] = p.xw[((size_t)tig * S + i) * p.n + ee];
    const PefIn pe{p.iota, K->r2n, K->nl, p.n, ee, p.M[ee]};
    d4f_run<S, true>(a, st, kb, tl, opaque_uniform(K->progf), K->nprogf, opaque_uniform(K->kf), x1, m, mprime, tig, pe);
    if (valid) {
#pragma unroll
      for (int i = 0; i < S; ++i) p.xw[((size_t)tig * S + i) * p.n + e] = a[i];
    }
  }
}

// c = A + n B from the plain pair (A < 2n, B < 4n): canonical pair, then the ciphertext words
template <int S>
__global__ __launch_bounds__(LANE_BLOCK) void k_pe_fin(PeParams p) {
  __shared__ uint32_t ns[S];
  for (int i = threadIdx.x; i < S; i += blockDim.x) ns[i] = p.k->nl[i];
  __syncthreads();
  uint32_t m[S];
#pragma unroll
  for (int j = 0; j < S; ++j) m[j] = ns[j];
  for (long long base = (long long)blockIdx.x * LANE_BLOCK; base < p.n; base += (long long)gridDim.x * LANE_BLOCK) {
    const long long i = base + threadIdx.x;
    const bool valid = i < p.n;
    const long long ii = valid ? i : p.n - 1;
    uint32_t a[S], b[S], d[S];
#pragma unroll
    for (int j = 0; j < S; ++j) {
      a[j] = p.xw[(size_t)j * p.n + ii];
      b[j] = p.xw[((size_t)S + j) * p.n + ii];
    }
    const bool lt = lane::sub<S>(a, m, d);
    uint32_t c = lt ? 0u : 1u;
#pragma unroll
    for (int j = 0; j < S; ++j) {
      a[j] = lt ? a[j] : d[j];
      const uint32_t v = b[j] + c;
      b[j] = v & lane::LMASK;
      c = v >> lane::LB;
    }
#pragma unroll 1
    for (int r = 0; r < 4; ++r) lane::cond_sub<S>(b, m);
    fb_out_all<S, 2 * FbGeom<S>::TW>(b, a, ns, reinterpret_cast<uint4*>(p.ct + ii * p.ct_words), valid,
                                     std::make_integer_sequence<int, 2 * S>{});
  }
}

}  // namespace fpai
