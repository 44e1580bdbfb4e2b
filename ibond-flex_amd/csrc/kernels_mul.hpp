// Ciphertext x plaintext scalar (PaillierEncryptedNumber.__mul__, encrypted_number.py:86-113) over
// arrays and encrypted-by-plain matrix products (he_otp_lr_ft1/train.py:160 `enc_diff_y.dot(features)`):
//
//   k_mul<TPI>      term t = (k, i, j) (t = (k m + i) d + j): c = ct[i cs_i + k cs_k],
//                   s = x[i xs_i + k xs_k + j xs_j] encoded like the reference (FixedPointNumber.encode,
//                   fixedpoint_number.py:46-90, precision None) to a signed mantissa M and exponent e_s;
//                   out = c^|M| mod n^2, exponent e_c + e_s, flag = (M < 0). The reference computes
//                   invert(c)^|M| for M < 0 (:100-106); that equals invert(c^|M|), so the flagged terms
//                   are finished by ONE batch inversion (k_inv_*) instead of one inversion each.
//   k_inv_up<TPI>   Montgomery's batch inversion, up-sweep: prefix products over segments of INV_SEG
//   k_inv_down<TPI> down-sweep: x_j^-1 = (x_0 .. x_j)^-1 (x_0 .. x_(j-1)), written in place
//
// Lane-group engine (bn_group.hpp), one element per group of TPI lanes, like k_add. A matrix product
// then reduces the terms over k with k_add (padding operands carry exponent PAD_EXP).
#pragma once
#include "kernels.hpp"

namespace fpai {

constexpr int INV_SEG = 64;   // values per segment of the batch inversion

struct MulParams {
  const uint32_t* ct;     // ciphertext words [*][W]
  const int32_t* exp;     // ciphertext exponents
  long long m, d;         // term t = (k m + i) d + j
  long long cs_i, cs_k;   // ciphertext index = i cs_i + k cs_k
  long long xs_i, xs_k, xs_j;   // scalar index = i xs_i + k xs_k + j xs_j
  const void* x;          // scalars
  int dtype;              // PAI_F32 / PAI_F64 / PAI_I64
  long long n;            // terms
  uint32_t* out;          // [n][W]
  int32_t* out_exp;       // [n]
  int32_t* status;        // [n] (nullable): ST_OK or ST_ENC_RANGE
  uint8_t* neg;           // [n]: 1 where the term still needs the inversion
  const uint32_t* N;      // n^2
  const uint32_t* R2;     // R^2 mod n^2
  const uint32_t* oneR;   // R mod n^2
  uint32_t mprime;
  int ct_words;
  uint32_t* scratch;      // per-lane tiles (TILE_WORDS_PER_LANE words per lane)
};

// Left-to-right fixed window 4 over a per-element exponent |M| < 2^63; the window count is the wave
// maximum (groups with shorter exponents run leading zero digits, x^0 = R: harmless).
template <int TPI>
__global__ __launch_bounds__(BLOCK, 2) void k_mul(MulParams p) {
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
    const long long t = valid ? inst : p.n - 1;
    const long long j = t % p.d, r = t / p.d;
    const long long i = r % p.m, k = r / p.m;
    const long long ci = i * p.cs_i + k * p.cs_k;
    const long long xi = i * p.xs_i + k * p.xs_k + j * p.xs_j;
    int64_t M = 0;
    int es = 0, st;
    if (p.dtype == 0) st = encode_float((double)((const float*)p.x)[xi], false, 0, M, es);
    else if (p.dtype == 1) st = encode_float(((const double*)p.x)[xi], false, 0, M, es);
    else st = encode_int(((const int64_t*)p.x)[xi], false, 0, M, es);
    if (st != ST_OK) M = 0;
    const bool negs = M < 0;
    const uint64_t e = negs ? (uint64_t)0 - (uint64_t)M : (uint64_t)M;
    int nw = e ? (67 - __clzll(e)) / 4 : 0;   // 4-bit windows, wave maximum
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) nw = max(nw, __shfl_xor(nw, s));
    uint32_t a[L], tt[L];
    if (nw == 0) {
      load_limbs_g<TPI>(p.oneR, a, tig);                                   // c^0 = 1 (Montgomery R)
    } else {
      // x~ = c R mod n^2; tiles: 0 -> R, d -> x~^d (d = 1..15)
      words_to_limbs(p.ct + ci * p.ct_words, p.ct_words, a, tig);
      copy_g_to_lds<TPI>(slot, p.R2, tig);
      montmul<TPI>(a, a, slot, TPI, m, p.mprime, lane, tig);
      load_limbs_g<TPI>(p.oneR, tt, tig);
      tile_store(tw, 0, tt, lane);
      tile_store(tw, 1, a, lane);
      write_limbs_lds<TPI>(slot, a, tig);
#pragma unroll
      for (int q = 0; q < L; ++q) tt[q] = a[q];
      for (int dd = 2; dd < 16; ++dd) {
        montmul<TPI>(tt, tt, slot, TPI, m, p.mprime, lane, tig);
        tile_store(tw, dd, tt, lane);
      }
      tile_load(tw, (int)((e >> (4 * (nw - 1))) & 0xF), a, lane);
      for (int w = nw - 2; w >= 0; --w) {
#pragma unroll 1
        for (int s = 0; s < 4; ++s) {
          write_limbs_lds<TPI>(slot, a, tig);
          montmul<TPI>(a, a, slot, TPI, m, p.mprime, lane, tig);
        }
        tile_load(tw, (int)((e >> (4 * w)) & 0xF), tt, lane);
        write_limbs_lds<TPI>(slot, tt, tig);
        montmul<TPI>(a, a, slot, TPI, m, p.mprime, lane, tig);
      }
    }
    write_one_lds<TPI>(slot, tig);
    montmul<TPI>(a, a, slot, TPI, m, p.mprime, lane, tig);                 // leave the Montgomery domain
    cond_sub<TPI>(a, m, lane, tig);
    emit_words<TPI>(slot, a, p.out + t * p.ct_words, p.ct_words, valid, tig);
    if (valid && tig == 0) {
      p.out_exp[t] = p.exp[ci] + es;
      p.neg[t] = negs ? 1 : 0;
      if (p.status) p.status[t] = st;
    }
  }
}

// ---------------------------------------------------------------- batch inversion
struct InvParams {
  uint32_t* x;            // [n][W] values; the down-sweep replaces flagged ones by their inverses
  const uint8_t* flag;    // [n] (nullable: all flagged)
  long long n;
  uint32_t* pre;          // [n][S] Montgomery prefix products (limbs, group layout)
  uint32_t* seg;          // [ceil(n / INV_SEG)][W]: up: segment products; down: their inverses
  const uint32_t* N;
  const uint32_t* R2;
  const uint32_t* oneR;
  uint32_t mprime;
  int ct_words;
};

// x~ = (flagged ? x : 1) R mod n^2
template <int TPI>
__device__ __forceinline__ void inv_load(const InvParams& p, long long j, bool use, uint32_t* slot, uint32_t (&xt)[L],
                                         const uint32_t (&m)[L], int lane, int tig) {
  const bool f = use && (p.flag == nullptr || p.flag[j] != 0);
  words_to_limbs(p.x + j * p.ct_words, f ? p.ct_words : 0, xt, tig);   // 0 words -> zero limbs
  if (!f && tig == 0) xt[0] = 1u;                                       // 1
  copy_g_to_lds<TPI>(slot, p.R2, tig);
  montmul<TPI>(xt, xt, slot, TPI, m, p.mprime, lane, tig);
}

template <int TPI>
__global__ __launch_bounds__(BLOCK, 2) void k_inv_up(InvParams p) {
  constexpr int S = TPI * L;
  constexpr int GPB = BLOCK / TPI;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int lane = threadIdx.x & 63;
  const int tig = threadIdx.x % TPI;
  const int gib = threadIdx.x / TPI;
  uint32_t* slot = smem + gib * S;
  uint32_t m[L];
  load_limbs_g<TPI>(p.N, m, tig);
  const long long nseg = (p.n + INV_SEG - 1) / INV_SEG;
  for (long long base = (long long)blockIdx.x * GPB; base < nseg; base += (long long)gridDim.x * GPB) {
    const long long sg = base + gib;
    const bool valid = sg < nseg;
    const long long sv = valid ? sg : nseg - 1;
    const long long s0 = sv * INV_SEG;
    const int cnt = (int)min((long long)INV_SEG, p.n - s0);
    int wcnt = cnt;
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) wcnt = max(wcnt, __shfl_xor(wcnt, s));
    uint32_t acc[L], xt[L];
    load_limbs_g<TPI>(p.oneR, acc, tig);
    for (int j = 0; j < wcnt; ++j) {
      const bool here = j < cnt;
      const long long jj = s0 + (here ? j : cnt - 1);
      inv_load<TPI>(p, jj, here, slot, xt, m, lane, tig);
      write_limbs_lds<TPI>(slot, xt, tig);
      montmul<TPI>(acc, acc, slot, TPI, m, p.mprime, lane, tig);
      if (valid && here) store_limbs_g<TPI>(p.pre + jj * S, acc, tig);
    }
    write_one_lds<TPI>(slot, tig);
    montmul<TPI>(acc, acc, slot, TPI, m, p.mprime, lane, tig);
    cond_sub<TPI>(acc, m, lane, tig);
    emit_words<TPI>(slot, acc, p.seg + sv * p.ct_words, p.ct_words, valid, tig);
  }
}

template <int TPI>
__global__ __launch_bounds__(BLOCK, 2) void k_inv_down(InvParams p) {
  constexpr int S = TPI * L;
  constexpr int GPB = BLOCK / TPI;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int lane = threadIdx.x & 63;
  const int tig = threadIdx.x % TPI;
  const int gib = threadIdx.x / TPI;
  uint32_t* slot = smem + gib * S;
  uint32_t m[L];
  load_limbs_g<TPI>(p.N, m, tig);
  const long long nseg = (p.n + INV_SEG - 1) / INV_SEG;
  for (long long base = (long long)blockIdx.x * GPB; base < nseg; base += (long long)gridDim.x * GPB) {
    const long long sg = base + gib;
    const bool valid = sg < nseg;
    const long long sv = valid ? sg : nseg - 1;
    const long long s0 = sv * INV_SEG;
    const int cnt = (int)min((long long)INV_SEG, p.n - s0);
    int wcnt = cnt;
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) wcnt = max(wcnt, __shfl_xor(wcnt, s));
    // I~ = (x_0 .. x_(cnt-1))^-1 R
    uint32_t I[L], xt[L], r[L];
    words_to_limbs(p.seg + sv * p.ct_words, p.ct_words, I, tig);
    copy_g_to_lds<TPI>(slot, p.R2, tig);
    montmul<TPI>(I, I, slot, TPI, m, p.mprime, lane, tig);
    for (int j = wcnt - 1; j >= 0; --j) {
      const bool here = j < cnt;
      const long long jj = s0 + (here ? j : 0);
      const bool f = here && (p.flag == nullptr || p.flag[jj] != 0);
      // r = I~ prefix(j-1) R^-1 (I~ itself for j = 0), out of the Montgomery domain: x_j^-1
      if (j > 0 && here) {
        uint32_t pv[L];
        load_limbs_g<TPI>(p.pre + (jj - 1) * S, pv, tig);
        write_limbs_lds<TPI>(slot, pv, tig);
      } else {
        copy_g_to_lds<TPI>(slot, p.oneR, tig);
      }
      montmul<TPI>(r, I, slot, TPI, m, p.mprime, lane, tig);
      write_one_lds<TPI>(slot, tig);
      montmul<TPI>(r, r, slot, TPI, m, p.mprime, lane, tig);
      cond_sub<TPI>(r, m, lane, tig);
      // I~ <- I~ x~_j (drops x_j); x_j is read before it is overwritten below
      inv_load<TPI>(p, jj, here, slot, xt, m, lane, tig);
      write_limbs_lds<TPI>(slot, xt, tig);
      montmul<TPI>(I, I, slot, TPI, m, p.mprime, lane, tig);
      emit_words<TPI>(slot, r, p.x + jj * p.ct_words, p.ct_words, valid && f, tig);
    }
  }
}

}  // namespace fpai
