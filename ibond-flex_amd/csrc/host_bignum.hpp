// Host-side big integers for the per-key setup (Montgomery constants, CRT constants, exponent schedules, the
// fixed-base tables' bases and generators). Not on any per-element path -- but on the re-keying caller's path
// (HE_SA_FT draws a keypair per exchange, he_sa_ft/train.py:38-39), so the arithmetic is GMP's (round 5: the
// earlier bit-serial division and shift loops cost ~0.25 s per fresh key). HBig stays a little-endian
// word vector; the operations convert through mpz_t.
#pragma once
#include <gmp.h>
#include <stdint.h>

#include <algorithm>
#include <vector>

namespace fpai {

struct HBig {
  std::vector<uint32_t> w;  // little-endian 32-bit words, no trailing zeros

  HBig() = default;
  explicit HBig(uint64_t v) {
    if (v) w.push_back((uint32_t)v);
    if (v >> 32) w.push_back((uint32_t)(v >> 32));
  }
  static HBig from_le_bytes(const uint8_t* b, size_t n) {
    HBig r;
    r.w.assign((n + 3) / 4, 0);
    for (size_t i = 0; i < n; ++i) r.w[i / 4] |= (uint32_t)b[i] << (8 * (i % 4));
    r.trim();
    return r;
  }
  void trim() {
    while (!w.empty() && w.back() == 0) w.pop_back();
  }
  bool is_zero() const { return w.empty(); }
  bool is_odd() const { return !w.empty() && (w[0] & 1); }
  size_t bits() const {
    if (w.empty()) return 0;
    return 32 * (w.size() - 1) + (32 - __builtin_clz(w.back()));
  }
  int bit(size_t i) const {
    size_t k = i / 32;
    return k < w.size() ? (int)((w[k] >> (i % 32)) & 1u) : 0;
  }
  // `lb`-bit limbs (device limb width), zero padded to n limbs
  std::vector<uint32_t> limbs(size_t n, int lb) const {
    std::vector<uint32_t> out(n, 0);
    const uint32_t mask = lb >= 32 ? 0xFFFFFFFFu : (1u << lb) - 1u;
    for (size_t k = 0; k < n; ++k) {
      const size_t b = (size_t)lb * k, i = b / 32, o = b % 32;
      const uint64_t lo = i < w.size() ? w[i] : 0u, hi = i + 1 < w.size() ? w[i + 1] : 0u;
      out[k] = (uint32_t)(((hi << 32) | lo) >> o) & mask;
    }
    return out;
  }
  std::vector<uint32_t> words(size_t n) const {
    std::vector<uint32_t> out(n, 0);
    for (size_t i = 0; i < std::min(n, w.size()); ++i) out[i] = w[i];
    return out;
  }
};

// RAII mpz_t and the conversions HBig <-> mpz
struct Mpz {
  mpz_t v;
  Mpz() { mpz_init(v); }
  explicit Mpz(const HBig& a) {
    mpz_init(v);
    if (!a.w.empty()) mpz_import(v, a.w.size(), -1, sizeof(uint32_t), 0, 0, a.w.data());
  }
  ~Mpz() { mpz_clear(v); }
  Mpz(const Mpz&) = delete;
  Mpz& operator=(const Mpz&) = delete;
  HBig big() const {
    HBig r;
    if (mpz_sgn(v) == 0) return r;
    r.w.assign((mpz_sizeinbase(v, 2) + 31) / 32, 0);
    size_t cnt = 0;
    mpz_export(r.w.data(), &cnt, -1, sizeof(uint32_t), 0, 0, v);
    r.w.resize(cnt);
    r.trim();
    return r;
  }
};

inline int cmp(const HBig& a, const HBig& b) {
  if (a.w.size() != b.w.size()) return a.w.size() < b.w.size() ? -1 : 1;
  for (size_t i = a.w.size(); i-- > 0;)
    if (a.w[i] != b.w[i]) return a.w[i] < b.w[i] ? -1 : 1;
  return 0;
}
inline HBig add(const HBig& a, const HBig& b) {
  HBig r;
  size_t n = std::max(a.w.size(), b.w.size());
  r.w.resize(n + 1);
  uint64_t c = 0;
  for (size_t i = 0; i < n; ++i) {
    c += (uint64_t)(i < a.w.size() ? a.w[i] : 0) + (i < b.w.size() ? b.w[i] : 0);
    r.w[i] = (uint32_t)c;
    c >>= 32;
  }
  r.w[n] = (uint32_t)c;
  r.trim();
  return r;
}
// a - b, requires a >= b
inline HBig sub(const HBig& a, const HBig& b) {
  HBig r;
  r.w.resize(a.w.size());
  int64_t c = 0;
  for (size_t i = 0; i < a.w.size(); ++i) {
    c += (int64_t)a.w[i] - (int64_t)(i < b.w.size() ? b.w[i] : 0);
    r.w[i] = (uint32_t)c;
    c >>= 32;
  }
  r.trim();
  return r;
}
inline HBig mul(const HBig& a, const HBig& b) {
  Mpz x(a), y(b), r;
  mpz_mul(r.v, x.v, y.v);
  return r.big();
}
inline HBig shl1(const HBig& a) {
  HBig r;
  r.w.resize(a.w.size() + 1);
  uint32_t c = 0;
  for (size_t i = 0; i < a.w.size(); ++i) {
    r.w[i] = (a.w[i] << 1) | c;
    c = a.w[i] >> 31;
  }
  r.w[a.w.size()] = c;
  r.trim();
  return r;
}
inline HBig shr1(const HBig& a) {
  HBig r = a;
  for (size_t i = 0; i < r.w.size(); ++i) r.w[i] = (r.w[i] >> 1) | (i + 1 < r.w.size() ? r.w[i + 1] << 31 : 0);
  r.trim();
  return r;
}
// a mod m
inline HBig mod(const HBig& a, const HBig& m) {
  Mpz x(a), y(m), r;
  mpz_mod(r.v, x.v, y.v);
  return r.big();
}
// floor(a / m)
inline HBig div_big(const HBig& a, const HBig& m) {
  Mpz x(a), y(m), r;
  mpz_fdiv_q(r.v, x.v, y.v);
  return r.big();
}
// (a * 2^k) mod m, a < m
inline HBig mul_pow2_mod(HBig a, size_t k, const HBig& m) {
  Mpz x(a), y(m), r;
  mpz_mul_2exp(r.v, x.v, k);
  mpz_mod(r.v, r.v, y.v);
  return r.big();
}
// a^{-1} mod m; returns empty HBig if not invertible
inline HBig inv_mod(const HBig& a0, const HBig& m) {
  Mpz x(a0), y(m), r;
  if (!mpz_invert(r.v, x.v, y.v)) return HBig();
  return r.big();
}
// a^e mod m
inline HBig pow_mod(const HBig& a, const HBig& e, const HBig& m) {
  Mpz x(a), y(e), z(m), r;
  mpz_powm(r.v, x.v, y.v, z.v);
  return r.big();
}
// -m^{-1} mod 2^lb for odd m
inline uint32_t mont_prime(const HBig& m, int lb) {
  uint32_t m0 = m.w.empty() ? 1 : m.w[0];
  uint32_t x = 1;
  for (int i = 0; i < 6; ++i) x *= 2u - m0 * x;   // Newton: x = m0^{-1} mod 2^32
  return (0u - x) & ((1u << lb) - 1u);
}

}  // namespace fpai

namespace fpai {
// a / d for a small divisor d
inline HBig div_small(const HBig& a, uint32_t d) {
  HBig q;
  q.w.assign(a.w.size(), 0);
  uint64_t r = 0;
  for (size_t i = a.w.size(); i-- > 0;) {
    r = (r << 32) | a.w[i];
    q.w[i] = (uint32_t)(r / d);
    r %= d;
  }
  q.trim();
  return q;
}
inline HBig pow2(size_t k) {
  HBig r;
  r.w.assign(k / 32 + 1, 0);
  r.w[k / 32] = 1u << (k % 32);
  return r;
}
}  // namespace fpai

namespace fpai {
// a mod d for a small divisor d
inline uint32_t mod_small(const HBig& a, uint32_t d) {
  uint64_t r = 0;
  for (size_t i = a.w.size(); i-- > 0;) r = ((r << 32) | a.w[i]) % d;
  return (uint32_t)r;
}

// Modular arithmetic modulo m for the one-time host work that needs real exponentiations (fixed-base setup, batch
// inversion). The interface of a Montgomery domain (to / mul / from, r2 the domain's R^2), implemented in the plain
// domain on GMP: to(a) = a mod m, from(a) = a, r2 = 1, mul = a b mod m -- every caller's to/mul/from sequence means
// the same value.
struct HMont {
  HBig m;
  HBig r2{1};
  explicit HMont(const HBig& mod_) : m(mod_) {}
  HBig mul(const HBig& a, const HBig& b) const {
    Mpz x(a), y(b), z(m), r;
    mpz_mul(r.v, x.v, y.v);
    mpz_mod(r.v, r.v, z.v);
    return r.big();
  }
  HBig to(const HBig& a) const { return mod(a, m); }
  HBig from(const HBig& a) const { return a; }
  // a^e mod m (plain in, plain out)
  HBig pow(const HBig& a, const HBig& e) const { return pow_mod(a, e, m); }
  // x^(2^k) mod m
  HBig sqr_k(const HBig& x0, size_t k) const {
    Mpz x(x0), z(m);
    for (size_t i = 0; i < k; ++i) {
      mpz_mul(x.v, x.v, x.v);
      mpz_mod(x.v, x.v, z.v);
    }
    return x.big();
  }
};

// primes below `bound` (sieve)
inline std::vector<uint32_t> small_primes(uint32_t bound) {
  std::vector<uint8_t> comp(bound, 0);
  std::vector<uint32_t> out;
  for (uint32_t i = 2; i < bound; ++i) {
    if (comp[i]) continue;
    out.push_back(i);
    for (uint64_t j = (uint64_t)i * i; j < bound; j += i) comp[j] = 1;
  }
  return out;
}
}  // namespace fpai
