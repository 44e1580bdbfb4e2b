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
#pragma unroll 1
    for (int k = 0; k < 2; ++k) d4_pass<S>(P, a, sx + k * S, 0, m, mprime, odd, std::make_integer_sequence<int, S>{});
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
