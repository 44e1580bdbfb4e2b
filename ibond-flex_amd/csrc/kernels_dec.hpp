// CRT decryption on the lane engine (bn_lane.hpp): one ciphertext per lane, the modulus p_h^2
// wave-uniform in SGPRs, squarings on the triangle. Replaces k_decrypt (lane groups, no squaring
// saving) for keys whose halves fit the lane engine (p^2 <= 74 limbs: 1024- and 2048-bit keys).
//
//   k_dec_pre<SB>    blockIdx.y = half h:  c~ = c R mod p_h^2 (the ciphertext reduced into the
//                                          Montgomery domain, K CIOS passes over its chunks)
//   k_dec_pow<SB>    blockIdx.y = half h:  x_h = c^(p_h - 1) mod p_h^2       (decryptor.py:55-61)
//                                          (the CRT encryption's lane_pow_body, op list for p_h - 1)
//   k_dec_fin<SA,SB> per element:          L_h = (x_h - 1) // p_h            (decryptor.py:29-31)
//                                          m_h = L_h * h_h mod p_h           (keypair.py:81-90)
//                                          u = (m_p - m_q) q^-1 mod p, x = m_q + u q
//                                          (gmpy_math.py:31-40) and FixedPointNumber.decode
//                                          (fixedpoint_number.py:92-107)
// Only the exponentiation is heavy; the split keeps it at k_crt_b's register budget (no spills).
#pragma once
#include "kernels_crt.hpp"

namespace fpai {

struct DecLaneHalf {
  const uint32_t* m2;     // p_h^2, SB limbs
  const uint32_t* cK;     // R_B^(K+1) mod p_h^2, K = ciphertext chunks (SB limbs)
  uint32_t mprime2;       // -p_h^-2 mod 2^LB
  uint32_t pinv;          // p_h^-1 mod 2^LB (exact division)
  uint32_t mprime1;       // -p_h^-1 mod 2^LB
  uint32_t pad;
  const uint32_t* ph;     // p_h, SA limbs
  const uint32_t* hR;     // h_h * R_A mod p_h, SA limbs
  const uint32_t* pm1;    // p_h - 1, SA limbs (L for x == 0: (0 - 1) // p == -1 == p - 1 mod p)
};

struct DecPreParams {
  const DecLaneHalf* halves;   // [2]
  long long n;
  const uint32_t* ct;          // N x ct_words
  int ct_words;
  int kchunks;                 // ceil(32 ct_words / (LB SB))
  uint32_t* out;               // [2][SB][n]
};

// ---------------------------------------------------------------- c~ = c R mod p_h^2
template <int SB>
__global__ __launch_bounds__(LANE_BLOCK) void k_dec_pre(DecPreParams p) {
  const int half = blockIdx.y;
  const DecLaneHalf* H = p.halves + half;
  const uint32_t mprime = H->mprime2;
  for (long long i = (long long)blockIdx.x * LANE_BLOCK + threadIdx.x; i < p.n; i += (long long)gridDim.x * LANE_BLOCK) {
    const uint32_t* cw = p.ct + i * p.ct_words;
    uint32_t m[SB];
#pragma unroll
    for (int j = 0; j < SB; ++j) m[j] = H->m2[j];
    uint64_t P[SB];
#pragma unroll
    for (int j = 0; j < SB; ++j) P[j] = 0;
    const int nw = p.ct_words;
#pragma unroll 1
    for (int k = 0; k < p.kchunks; ++k) {
      uint32_t b[SB], cst[SB];
#pragma unroll
      for (int j = 0; j < SB; ++j) {
        const int bit = (k * SB + j) * lane::LB, wi = bit >> 5, sh = bit & 31;
        const uint64_t lo = wi < nw ? (uint64_t)cw[wi] : 0ull;
        const uint64_t hi = wi + 1 < nw ? (uint64_t)cw[wi + 1] : 0ull;
        b[j] = (uint32_t)(((hi << 32) | lo) >> sh) & lane::LMASK;
        cst[j] = H->cK[j];
      }
      lane::mul_pass<SB>(P, cst, b, m, mprime);   // invariant: T < cst + m < 2 m for digits < 2^LB
    }
    uint32_t a[SB];
    lane::normalize<SB>(P, a);
#pragma unroll
    for (int j = 0; j < SB; ++j) p.out[((size_t)half * SB + j) * p.n + i] = a[j];
  }
}

// ---------------------------------------------------------------- x_h = c~^(p_h - 1) * 1 R^-1
// k_crt_b's loop with an SB-limb input already in the Montgomery domain. (Kept as its own kernel
// body: factoring both into one inlined device function moved the modulus out of the SGPRs and
// spilled ~3.7k VGPRs.)
template <int SB>
__global__ __launch_bounds__(LANE_BLOCK, LANE_OCC) void k_dec_pow(CrtParams p) {
  const int half = blockIdx.y;
  const CrtHalf* H = p.halves + half;
  uint32_t m[SB];
#pragma unroll
  for (int j = 0; j < SB; ++j) m[j] = H->m[j];
  const uint32_t mprime = H->mprime;
  const int nprog = H->nprog;
  const uint32_t* prog = H->prog;
  const uint32_t* c1 = H->c1;
  const LaneScratch tl = lane_scratch(p.scratch);
  for (long long base = (long long)blockIdx.x * LANE_BLOCK; base < p.n; base += (long long)gridDim.x * LANE_BLOCK) {
    const long long i = base + threadIdx.x;
    const long long ii = i < p.n ? i : p.n - 1;
    uint32_t a[SB];
#pragma unroll
    for (int j = 0; j < SB; ++j) a[j] = p.yin[((size_t)half * SB + j) * p.n + ii];
    ltile_store<SB>(tl, 0, a);
    run_lane_program<SB>(a, tl, prog, nprog, c1, m, mprime);     // c~^(p_h - 1) * 1 R^-1
    if (i < p.n) {
#pragma unroll
      for (int j = 0; j < SB; ++j) p.out[((size_t)half * SB + j) * p.n + i] = a[j];
    }
  }
}

// ---------------------------------------------------------------- CRT recombination + decode
struct DecFinParams {
  const DecLaneHalf* halves;  // [2]
  long long n;
  const uint32_t* xh;       // [2][SB][n]: c^(p_h - 1) mod p_h^2 (< 2 p_h^2)
  const int32_t* exp;
  const uint32_t* p;        // SA limbs
  const uint32_t* q;        // SA limbs
  const uint32_t* qinvR;    // q^-1 R_A mod p, SA limbs
  uint32_t pprime;          // -p^-1 mod 2^LB
  const uint32_t* nlimb;    // n, SB limbs
  const uint32_t* maxint;   // n // 3 - 1, SB limbs
  double* val;
  int64_t* mant;
  int32_t* status;
  uint32_t* raw;            // N x pt_words (nullable)
  int pt_words;
};

// m_h = L(x_h, p_h) * h_h mod p_h, canonical (decryptor.py:55-61 with keypair.py:81-90's h_h)
template <int SA, int SB>
__device__ __forceinline__ void dec_half(const DecLaneHalf* __restrict__ H, const uint32_t* __restrict__ xh,
                                         long long n, long long i, uint32_t (&mh)[SA]) {
  uint32_t x[SB], m2[SB];
#pragma unroll
  for (int j = 0; j < SB; ++j) {
    x[j] = xh[(size_t)j * n + i];
    m2[j] = H->m2[j];
  }
  lane::cond_sub<SB>(x, m2);                 // canonical x_h in [0, p_h^2)
  uint32_t zero_acc = 0;
#pragma unroll
  for (int j = 0; j < SB; ++j) zero_acc |= x[j];
  uint32_t pl[SA];
#pragma unroll
  for (int j = 0; j < SA; ++j) pl[j] = H->ph[j];
  // L_h = (x_h - 1) / p_h exactly (x_h == 1 mod p_h): Hensel quotient digits from the low limbs
  {
    const uint32_t pinv = H->pinv;
    int64_t T[SA];
#pragma unroll
    for (int j = 0; j < SA; ++j) T[j] = (int64_t)x[j];
    T[0] -= 1;
#pragma unroll
    for (int d = 0; d < SA; ++d) {
      const uint32_t qd = ((uint32_t)T[d] * pinv) & lane::LMASK;
#pragma unroll
      for (int j = 0; d + j < SA; ++j) T[d + j] -= (int64_t)((uint64_t)qd * pl[j]);
      if (d + 1 < SA) T[d + 1] += T[d] >> lane::LB;   // T[d] == 0 mod 2^LB: exact shift
      mh[d] = qd;
    }
  }
  if (zero_acc == 0) {   // c == 0 mod p_h: the reference's floor division gives L = -1
#pragma unroll
    for (int j = 0; j < SA; ++j) mh[j] = H->pm1[j];
  }
  uint32_t hb[SA];
#pragma unroll
  for (int j = 0; j < SA; ++j) hb[j] = H->hR[j];
  lane::mont_mul<SA>(mh, hb, pl, H->mprime1);   // L_h h_h mod p_h (< 2 p_h)
  lane::cond_sub<SA>(mh, pl);
}

// sign(a - b) over S canonical limbs
template <int S>
__device__ __forceinline__ int cmp_limbs(const uint32_t (&a)[S], const uint32_t (&b)[S]) {
  int c = 0;
#pragma unroll
  for (int k = 0; k < S; ++k) c = (a[k] > b[k]) ? 1 : ((a[k] < b[k]) ? -1 : c);
  return c;
}

// FixedPointNumber.decode (fixedpoint_number.py:92-107) of x in [0, n), x in S canonical limbs:
// float(mantissa) correctly rounded (half even, Python int -> float), times 16^-e.
template <int S>
__device__ __forceinline__ void decode_lane(const uint32_t (&x)[S], const uint32_t (&nl)[S], const uint32_t (&mx)[S],
                                            int e, double& val, int64_t& mant, int& st) {
  uint32_t mag[S];
  bool neg = false;
  st = ST_OK;
  if (cmp_limbs<S>(x, mx) <= 0) {
#pragma unroll
    for (int k = 0; k < S; ++k) mag[k] = x[k];
  } else {
    (void)lane::sub<S>(nl, x, mag);   // n - x (x < n)
    if (cmp_limbs<S>(mag, mx) > 0) st = ST_OVERFLOW;
    neg = true;
  }
  val = 0.0;
  mant = 0;
  if (st != ST_OK) return;
  int top = 0;
  uint32_t xt = 0;
#pragma unroll
  for (int k = 0; k < S; ++k)
    if (mag[k]) {
      top = k;
      xt = mag[k];
    }
  const int B = xt == 0 ? 0 : top * lane::LB + (32 - __clz(xt));   // bit length
  const int lo_bit = B > 64 ? B - 64 : 0;
  uint64_t hi64 = 0;
  bool sticky = false;
#pragma unroll
  for (int k = 0; k < S; ++k) {
    const uint64_t v = mag[k];
    const int sh = k * lane::LB - lo_bit;
    if (sh >= 64) continue;
    if (sh >= 0) {
      hi64 |= v << sh;
    } else if (sh > -lane::LB) {
      hi64 |= v >> (-sh);
      sticky |= (v & ((1ull << (-sh)) - 1ull)) != 0;
    } else {
      sticky |= v != 0;
    }
  }
  double d;
  if (B <= 53) {
    d = (double)hi64;
  } else {
    const int drop = (B > 64 ? 64 : B) - 53;
    uint64_t keep = hi64 >> drop;
    const uint64_t rem = hi64 & ((1ull << drop) - 1ull);
    const uint64_t halfv = 1ull << (drop - 1);
    if (rem > halfv || (rem == halfv && (sticky || (keep & 1ull)))) keep += 1;
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

template <int SA, int SB>
__global__ __launch_bounds__(LANE_BLOCK) void k_dec_fin(DecFinParams p) {
  for (long long i = (long long)blockIdx.x * LANE_BLOCK + threadIdx.x; i < p.n; i += (long long)gridDim.x * LANE_BLOCK) {
    uint32_t mp[SA], mq[SA], pl[SA];
    dec_half<SA, SB>(p.halves, p.xh, p.n, i, mp);
    dec_half<SA, SB>(p.halves + 1, p.xh + (size_t)SB * p.n, p.n, i, mq);
#pragma unroll
    for (int j = 0; j < SA; ++j) pl[j] = p.p[j];
    // u = (mp - mq) q^-1 mod p = mp q^-1 - mq q^-1 (each product < 2p for inputs < R_A)
    uint32_t a1[SA], a2[SA], qi[SA], u[SA];
#pragma unroll
    for (int j = 0; j < SA; ++j) {
      qi[j] = p.qinvR[j];
      a1[j] = mp[j];
      a2[j] = mq[j];
    }
    lane::mont_mul<SA>(a1, qi, pl, p.pprime);
    lane::cond_sub<SA>(a1, pl);
    lane::mont_mul<SA>(a2, qi, pl, p.pprime);
    lane::cond_sub<SA>(a2, pl);
    {
      const bool neg = lane::sub<SA>(a1, a2, u);
      uint64_t c = 0;
#pragma unroll
      for (int j = 0; j < SA; ++j) {
        const uint64_t v = (uint64_t)u[j] + (neg ? pl[j] : 0u) + c;
        u[j] = (uint32_t)v & lane::LMASK;
        c = v >> lane::LB;
      }
    }
    // x = mq + u q  (< n)
    uint32_t x[SB];
    {
      uint64_t X[SB];
#pragma unroll
      for (int k = 0; k < SB; ++k) X[k] = k < SA ? (uint64_t)mq[k] : 0ull;
#pragma unroll
      for (int j = 0; j < SA; ++j) {
        const uint32_t qj = p.q[j];
#pragma unroll
        for (int t = 0; t < SA; ++t)
          if (t + j < SB) X[t + j] += (uint64_t)u[t] * qj;
      }
      lane::normalize<SB>(X, x);
    }
    uint32_t nl[SB], mx[SB];
#pragma unroll
    for (int k = 0; k < SB; ++k) {
      nl[k] = p.nlimb[k];
      mx[k] = p.maxint[k];
    }
    double val;
    int64_t mant;
    int st;
    decode_lane<SB>(x, nl, mx, p.exp[i], val, mant, st);
    p.val[i] = val;
    if (p.mant) p.mant[i] = mant;
    p.status[i] = st;
    if (p.raw) {
      uint32_t* out = p.raw + i * p.pt_words;
#pragma unroll
      for (int w = 0; w < (SB * lane::LB + 31) / 32; ++w) {
        const int bit = 32 * w, k = bit / lane::LB, sh = bit - k * lane::LB;
        uint64_t v = (uint64_t)x[k] >> sh;
        if (k + 1 < SB) v |= (uint64_t)x[k + 1] << (lane::LB - sh);
        if (k + 2 < SB && 2 * lane::LB - sh < 32) v |= (uint64_t)x[k + 2] << (2 * lane::LB - sh);
        if (w < p.pt_words) out[w] = (uint32_t)v;
      }
    }
  }
}

}  // namespace fpai
