// refcpu_field.h -- host-only F_p arithmetic for the CPU oracle (TEST INFRASTRUCTURE, oracle/).
//
// Restates circom_algebra/src/modular_arithmetic.rs:9-91 (add, mul, sub, div, multi_inv) for
// canonical values with fixed 4x64-bit limbs instead of num-bigint-dig 0.8.4 BigInt.  Every
// result the reference produces is the canonical residue ((a % p) + p) % p, so any exact modular
// arithmetic reproduces it; values are kept in Montgomery form (R = 2^256) internally.
#pragma once
#include <cstdint>
#include <cstring>

namespace refcpu {

typedef unsigned __int128 u128;

struct Fe {
  uint64_t l[4];
  bool is_zero() const { return (l[0] | l[1] | l[2] | l[3]) == 0; }
  bool operator==(const Fe &o) const {
    return l[0] == o.l[0] && l[1] == o.l[1] && l[2] == o.l[2] && l[3] == o.l[3];
  }
  bool operator!=(const Fe &o) const { return !(*this == o); }
};

static inline Fe fe_zero() { Fe z; z.l[0] = z.l[1] = z.l[2] = z.l[3] = 0; return z; }

struct Field {
  uint64_t p[4];
  uint64_t np;  // -p^{-1} mod 2^64
  Fe r2;        // R^2 mod p
  Fe one;       // R mod p (Montgomery one)

  static bool geq(const uint64_t *a, const uint64_t *b) {
    for (int i = 3; i >= 0; --i) {
      if (a[i] != b[i]) return a[i] > b[i];
    }
    return true;
  }
  static uint64_t sub4(uint64_t *r, const uint64_t *a, const uint64_t *b) {
    uint64_t borrow = 0;
    for (int i = 0; i < 4; ++i) {
      u128 d = (u128)a[i] - b[i] - borrow;
      r[i] = (uint64_t)d;
      borrow = (uint64_t)(d >> 64) & 1;
    }
    return borrow;
  }
  static uint64_t add4(uint64_t *r, const uint64_t *a, const uint64_t *b) {
    uint64_t carry = 0;
    for (int i = 0; i < 4; ++i) {
      u128 s = (u128)a[i] + b[i] + carry;
      r[i] = (uint64_t)s;
      carry = (uint64_t)(s >> 64);
    }
    return carry;
  }

  void init(const uint64_t prime[4]) {
    memcpy(p, prime, sizeof(p));
    uint64_t inv = 1;
    for (int i = 0; i < 7; ++i) inv *= 2 - p[0] * inv;
    np = (uint64_t)0 - inv;
    // 2^512 mod p by doubling (p < 2^256).
    uint64_t x[4] = {1, 0, 0, 0};
    for (int i = 0; i < 512; ++i) {
      uint64_t c = add4(x, x, x);
      if (c || geq(x, p)) sub4(x, x, p);
      if (i == 255) memcpy(one.l, x, sizeof(x));
    }
    memcpy(r2.l, x, sizeof(x));
  }

  Fe add(const Fe &a, const Fe &b) const {
    Fe r;
    uint64_t c = add4(r.l, a.l, b.l);
    if (c || geq(r.l, p)) sub4(r.l, r.l, p);
    return r;
  }
  Fe sub(const Fe &a, const Fe &b) const {
    Fe r;
    if (sub4(r.l, a.l, b.l)) add4(r.l, r.l, p);
    return r;
  }
  Fe neg(const Fe &a) const {
    if (a.is_zero()) return a;
    Fe r;
    sub4(r.l, p, a.l);
    return r;
  }
  // CIOS Montgomery product a*b*R^-1 mod p.
  Fe mul(const Fe &a, const Fe &b) const {
    uint64_t t[6] = {0, 0, 0, 0, 0, 0};
    for (int i = 0; i < 4; ++i) {
      uint64_t c = 0;
      for (int j = 0; j < 4; ++j) {
        u128 s = (u128)a.l[j] * b.l[i] + t[j] + c;
        t[j] = (uint64_t)s;
        c = (uint64_t)(s >> 64);
      }
      u128 s = (u128)t[4] + c;
      t[4] = (uint64_t)s;
      t[5] = (uint64_t)(s >> 64);
      uint64_t m = t[0] * np;
      s = (u128)m * p[0] + t[0];
      c = (uint64_t)(s >> 64);
      for (int j = 1; j < 4; ++j) {
        s = (u128)m * p[j] + t[j] + c;
        t[j - 1] = (uint64_t)s;
        c = (uint64_t)(s >> 64);
      }
      s = (u128)t[4] + c;
      t[3] = (uint64_t)s;
      t[4] = t[5] + (uint64_t)(s >> 64);
    }
    Fe r;
    memcpy(r.l, t, 32);
    if (t[4] || geq(r.l, p)) sub4(r.l, r.l, p);
    return r;
  }
  Fe to_mont(const Fe &canon) const { return mul(canon, r2); }
  Fe from_mont(const Fe &a) const {
    Fe o = fe_zero();
    o.l[0] = 1;
    return mul(a, o);
  }
  // a^(p-2): the inverse for a != 0 (modular_arithmetic.rs:41-47 uses mod_inverse; same value).
  Fe inv(const Fe &a) const {
    uint64_t e[4];
    uint64_t two[4] = {2, 0, 0, 0};
    sub4(e, p, two);
    Fe r = one;
    Fe base = a;
    for (int i = 0; i < 256; ++i) {
      if ((e[i >> 6] >> (i & 63)) & 1) r = mul(r, base);
      base = mul(base, base);
    }
    return r;
  }
  bool canonical(const uint64_t v[4]) const { return !geq(v, p); }
};

}  // namespace refcpu
