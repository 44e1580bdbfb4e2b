// Minimal host-side big integer helpers for one-time key setup (Montgomery constants,
// CRT constants, exponent schedules). Not on any per-element path.
#pragma once
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
    for (size_t k = 0; k < n; ++k) {
      uint32_t v = 0;
      for (int b = 0; b < lb; ++b) v |= (uint32_t)bit((size_t)lb * k + b) << b;
      out[k] = v;
    }
    return out;
  }
  std::vector<uint32_t> words(size_t n) const {
    std::vector<uint32_t> out(n, 0);
    for (size_t i = 0; i < std::min(n, w.size()); ++i) out[i] = w[i];
    return out;
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
  HBig r;
  if (a.is_zero() || b.is_zero()) return r;
  r.w.assign(a.w.size() + b.w.size(), 0);
  for (size_t i = 0; i < a.w.size(); ++i) {
    uint64_t c = 0;
    for (size_t j = 0; j < b.w.size(); ++j) {
      c += (uint64_t)a.w[i] * b.w[j] + r.w[i + j];
      r.w[i + j] = (uint32_t)c;
      c >>= 32;
    }
    r.w[i + b.w.size()] = (uint32_t)c;
  }
  r.trim();
  return r;
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
// a mod m by binary long division
inline HBig mod(const HBig& a, const HBig& m) {
  HBig r;
  for (size_t i = a.bits(); i-- > 0;) {
    r = shl1(r);
    if (a.bit(i)) {
      if (r.w.empty()) r.w.push_back(0);
      r.w[0] |= 1;
    }
    if (cmp(r, m) >= 0) r = sub(r, m);
  }
  return r;
}
// (a * 2^k) mod m, a < m
inline HBig mul_pow2_mod(HBig a, size_t k, const HBig& m) {
  for (size_t i = 0; i < k; ++i) {
    a = shl1(a);
    if (cmp(a, m) >= 0) a = sub(a, m);
  }
  return a;
}
// a^{-1} mod m for odd m (binary extended Euclid); returns empty HBig if not invertible
inline HBig inv_mod(const HBig& a0, const HBig& m) {
  HBig u = mod(a0, m), v = m, x1(1), x2(0);
  if (u.is_zero()) return HBig();
  auto half = [&](HBig& x) {
    if (x.is_odd()) x = add(x, m);
    x = shr1(x);
  };
  HBig one(1);
  while (cmp(u, one) != 0 && cmp(v, one) != 0) {
    while (!u.is_odd()) { u = shr1(u); half(x1); }
    while (!v.is_odd()) { v = shr1(v); half(x2); }
    if (cmp(u, v) >= 0) {
      u = sub(u, v);
      x1 = cmp(x1, x2) >= 0 ? sub(x1, x2) : sub(add(x1, m), x2);
    } else {
      v = sub(v, u);
      x2 = cmp(x2, x1) >= 0 ? sub(x2, x1) : sub(add(x2, m), x1);
    }
    if (u.is_zero() || v.is_zero()) return HBig();
  }
  return cmp(u, one) == 0 ? mod(x1, m) : mod(x2, m);
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

// Word-level (32-bit) Montgomery arithmetic modulo an odd m, for the one-time host work that needs
// real modular exponentiations (fixed-base obfuscation setup): ~1000x faster than mod().
struct HMont {
  HBig m;
  size_t s = 0;          // words
  uint32_t mp = 0;       // -m^-1 mod 2^32
  HBig r2;               // R^2 mod m, R = 2^(32 s)
  explicit HMont(const HBig& mod_) : m(mod_), s(mod_.w.size()) {
    uint32_t x = 1;
    for (int i = 0; i < 6; ++i) x *= 2u - m.w[0] * x;
    mp = 0u - x;
    r2 = mul_pow2_mod(HBig(1), 64 * s, m);
  }
  // CIOS: a b R^-1 mod m (a, b < m)
  HBig mul(const HBig& a, const HBig& b) const {
    std::vector<uint64_t> t(s + 2, 0);
    for (size_t i = 0; i < s; ++i) {
      const uint64_t ai = i < a.w.size() ? a.w[i] : 0;
      uint64_t c = 0;
      for (size_t j = 0; j < s; ++j) {
        const uint64_t v = t[j] + ai * (j < b.w.size() ? b.w[j] : 0) + c;
        t[j] = (uint32_t)v;
        c = v >> 32;
      }
      uint64_t v = t[s] + c;
      t[s] = (uint32_t)v;
      t[s + 1] = v >> 32;
      const uint64_t q = (uint32_t)((uint32_t)t[0] * mp);
      v = t[0] + q * m.w[0];
      c = v >> 32;
      for (size_t j = 1; j < s; ++j) {
        v = t[j] + q * m.w[j] + c;
        t[j - 1] = (uint32_t)v;
        c = v >> 32;
      }
      v = t[s] + c;
      t[s - 1] = (uint32_t)v;
      t[s] = t[s + 1] + (v >> 32);
    }
    HBig r;
    r.w.assign(s + 1, 0);
    for (size_t i = 0; i <= s; ++i) r.w[i] = (uint32_t)t[i];
    r.trim();
    if (cmp(r, m) >= 0) r = sub(r, m);
    return r;
  }
  HBig to(const HBig& a) const { return mul(mod(a, m), r2); }
  HBig from(const HBig& a) const { return mul(a, HBig(1)); }
  // a^e mod m (plain in, plain out)
  HBig pow(const HBig& a, const HBig& e) const {
    HBig x = to(a), acc = to(HBig(1));
    for (size_t i = e.bits(); i-- > 0;) {
      acc = mul(acc, acc);
      if (e.bit(i)) acc = mul(acc, x);
    }
    return from(acc);
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
