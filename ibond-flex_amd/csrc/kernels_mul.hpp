// Ciphertext x plaintext scalar (PaillierEncryptedNumber.__mul__, encrypted_number.py:86-113) over
// arrays and encrypted-by-plain matrix products (he_otp_lr_ft1/train.py:160 `enc_diff_y.dot(features)`):
//
//   k_mul<TPI>      term t = (k, i, j) (t = (k m + i) d + j): c = ct[i cs_i + k cs_k],
//                   s = x[i xs_i + k xs_k + j xs_j] encoded like the reference (FixedPointNumber.encode,
//                   fixedpoint_number.py:46-90, precision None) to a signed mantissa M and exponent e_s;
//                   out = c^|M| mod n^2, exponent e_c + e_s, flag = (M < 0). The reference computes
//                   invert(c)^|M| for M < 0 (:100-106); that equals invert(c^|M|), so the flagged terms
//                   are finished by ONE batch inversion (k_inv_*) instead of one inversion each.
//   k_inv_up<TPI>   Montgomery's batch inversion, up-sweep: prefix products over segments of p.seg_len values
//   k_inv_down<TPI> down-sweep: x_j^-1 = (x_0 .. x_j)^-1 (x_0 .. x_(j-1)), written in place
//
// Lane-group engine (bn_group.hpp), one element per group of TPI lanes, like k_add. A matrix product
// then reduces the terms over k with k_add (padding operands carry exponent PAD_EXP).
#pragma once
#include "kernels.hpp"

namespace fpai {

constexpr int INV_SEG = 64;   // values per segment of the batch inversion's first level (flexpai.hip batch_invert)

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

// ---------------------------------------------------------------- ciphertext + plaintext
// E(x) + y (PaillierEncryptedNumber.__add_scalar / __add_fixpointnumber, encrypted_number.py:139-164):
// y is encoded with max_exponent = e_x (fixedpoint_number.py:81-84), giving (M, E >= e_x), and
// raw-encrypted with r = 1: c0 = 1 + n M mod n^2 (raw_encrypt.py:37-45). k_plain writes (c0, E) as
// the second operand of a 2-way k_add, whose alignment raises E(x) to E exactly like
// __align_exponent / __increase_exponent_to (:115-137), then multiplies (__raw_add :180-185).
//
// M is exact for any exponent: M = +-mag 2^sh with mag < 2^64, so c0 needs only a shifted 4-limb
// multiplier of n. Elements the device cannot decide bit-exactly get a status instead:
//   ST_FLOAT_OVF  float scalar * 16^E overflows a double (OverflowError in the reference);
//   ST_ENC_RANGE  |M| has more than max_bits (= nb - 3) bits (the reference's exact |M| > max_int test
//                 is then made by the host).
struct PlainParams {
  const int32_t* exp;     // ciphertext exponents [n]: the max_exponent of each element's encode
  const void* x;          // scalars
  int dtype;              // PAI_F32 / PAI_F64 / PAI_I64
  long long xs;           // scalar index = i xs (0: one scalar for every element)
  long long n;
  uint32_t* c0;           // [n][W] out
  int32_t* e0;            // [n] out
  int32_t* status;        // [n] out (nullable)
  const uint32_t* N;      // n^2, limbs (S)
  const uint32_t* nl;     // n, limbs (S, zero padded)
  int ct_words;
  int max_bits;
};

__device__ __forceinline__ int encode_plain_max(int dtype, const void* x, long long xi, int me, uint64_t& mag,
                                                int& sh, bool& neg, int& E, int max_bits) {
  mag = 0;
  sh = 0;
  neg = false;
  if (dtype != 2) {
    const double v = dtype == 0 ? (double)((const float*)x)[xi] : ((const double*)x)[xi];
    if (fabs(v) < 1e-200) {            // scalar = 0, an int: exponent 0 (fixedpoint_number.py:56-57, 67-69)
      E = max(me, 0);
      return ST_OK;
    }
    int fe;
    const double f = frexp(v, &fe);
    const int e0 = floor_div(53 - fe, 4);
    E = max(me, e0);
    neg = v < 0;
    if (E == e0) {
      const double s = rint(ldexp(fabs(v), 4 * E));   // < 2^58: exact scaling, ties-to-even
      mag = (uint64_t)s;
      return ST_OK;
    }
    if (E >= 256 || fe + 4 * E > 1024) return ST_FLOAT_OVF;   // v * 16^E is not a finite double
    mag = (uint64_t)ldexp(fabs(f), 53);                        // v 16^E = (f 2^53) 2^(fe - 53 + 4E)
    sh = fe - 53 + 4 * E;                                      // > 0 since E > e0
  } else {
    const int64_t v = ((const int64_t*)x)[xi];
    E = max(me, 0);
    neg = v < 0;
    mag = neg ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
    if (mag == 0) return ST_OK;
    sh = 4 * E;     // exact: numpy casts int arrays to object (Python ints) for the object add loop
  }
  if (mag != 0 && (64 - __clzll(mag)) + sh > max_bits) return ST_ENC_RANGE;
  return ST_OK;
}

template <int TPI>
__global__ __launch_bounds__(BLOCK) void k_plain(PlainParams p) {
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
    uint64_t mag;
    int sh, E;
    bool neg;
    const int st = encode_plain_max(p.dtype, p.x, ii * p.xs, p.exp[ii], mag, sh, neg, E, p.max_bits);
    if (st != ST_OK) mag = 0;
    // |M| = mag 2^sh as four LB-bit digits starting at limb q
    const int q = sh / LB;
    const unsigned __int128 t = (unsigned __int128)mag << (sh % LB);
    const uint64_t D0 = (uint64_t)t & LMASK, D1 = (uint64_t)(t >> LB) & LMASK, D2 = (uint64_t)(t >> (2 * LB)) & LMASK,
                   D3 = (uint64_t)(t >> (3 * LB));
    uint64_t P[L];
#pragma unroll
    for (int i = 0; i < L; ++i) {
      const int k = tig * L + i - q;
      uint64_t acc = 0;
      if (k >= 0) acc += (uint64_t)p.nl[k] * D0;
      if (k >= 1) acc += (uint64_t)p.nl[k - 1] * D1;
      if (k >= 2) acc += (uint64_t)p.nl[k - 2] * D2;
      if (k >= 3) acc += (uint64_t)p.nl[k - 3] * D3;
      P[i] = acc;
    }
    uint32_t X[L], Dn[L], a[L];
    normalize<TPI>(P, X, lane, tig);                    // n |M| < n^2 / 4
    (void)sub_limbs<TPI>(m, X, Dn, lane, tig);          // n^2 - n |M|
#pragma unroll
    for (int i = 0; i < L; ++i) P[i] = (uint64_t)((neg && mag) ? Dn[i] : X[i]) + ((tig == 0 && i == 0) ? 1u : 0u);
    normalize<TPI>(P, a, lane, tig);
    emit_words<TPI>(slot, a, p.c0 + ii * p.ct_words, p.ct_words, valid, tig);
    if (valid && tig == 0) {
      p.e0[ii] = E;
      if (p.status) p.status[ii] = st;
    }
  }
}

// ---------------------------------------------------------------- batch inversion
struct InvParams {
  uint32_t* x;            // [n][W] values; the down-sweep replaces flagged ones by their inverses
  const uint8_t* flag;    // [n] (nullable: all flagged)
  long long n;
  uint32_t* pre;          // [n][S] Montgomery prefix products (limbs, group layout)
  uint32_t* seg;          // [ceil(n / seg_len)][W]: up: segment products; down: their inverses
  const uint32_t* N;
  const uint32_t* R2;
  const uint32_t* oneR;
  uint32_t mprime;
  int ct_words;
  int seg_len;            // values per segment at this level (<= INV_SEG)
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
  const long long nseg = (p.n + p.seg_len - 1) / p.seg_len;
  for (long long base = (long long)blockIdx.x * GPB; base < nseg; base += (long long)gridDim.x * GPB) {
    const long long sg = base + gib;
    const bool valid = sg < nseg;
    const long long sv = valid ? sg : nseg - 1;
    const long long s0 = sv * p.seg_len;
    const int cnt = (int)min((long long)p.seg_len, p.n - s0);
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
  const long long nseg = (p.n + p.seg_len - 1) / p.seg_len;
  for (long long base = (long long)blockIdx.x * GPB; base < nseg; base += (long long)gridDim.x * GPB) {
    const long long sg = base + gib;
    const bool valid = sg < nseg;
    const long long sv = valid ? sg : nseg - 1;
    const long long s0 = sv * p.seg_len;
    const int cnt = (int)min((long long)p.seg_len, p.n - s0);
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
