// field.hpp -- F_p arithmetic for the device (and host helpers), p < 2^256 odd.
//
// Replaces circom_algebra/src/modular_arithmetic.rs:9-91 (num-bigint-dig BigInt + double
// remainder per op) with residues stored as 4 x 64-bit limbs in Montgomery form (R = 2^261): one
// radix-2^29 Montgomery product per field multiplication, carry-propagating add/sub with a single
// conditional correction.  Primes below 2^64 (goldilocks) take a one-word path (two 64-bit
// Montgomery reductions) in the same representation.
// Results are canonical residues, identical to the reference's ((a % p) + p) % p.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace rs {

typedef unsigned __int128 u128;

struct __attribute__((aligned(16))) Fe {
  uint64_t l[4];
};

constexpr int kLimbBits = 29;  // Montgomery radix 2^29, 9 limbs, R = 2^261
constexpr int kLimbs = 9;
constexpr uint32_t kLimbMask = (1u << kLimbBits) - 1;

struct FieldP {
  uint64_t p[4];
  uint32_t pl[kLimbs];  // p in 29-bit limbs
  uint32_t np;          // -p^-1 mod 2^29
  Fe r2;        // R^2 mod p  (R = 2^261)
  Fe one;       // R mod p
  Fe pm2;       // p - 2 (Fermat exponent)
  uint64_t np64;  // -p^-1 mod 2^64 (one-word primes)
  uint64_t k133;  // 2^-133 mod p (one-word primes): folds the 2^64 word radix into R = 2^261
  uint32_t w64;   // p < 2^64 (goldilocks): products take the one-word Montgomery path
};

__host__ __device__ __forceinline__ bool fe_is_zero(const Fe &a) {
  return (a.l[0] | a.l[1] | a.l[2] | a.l[3]) == 0;
}
__host__ __device__ __forceinline__ Fe fe_zero() {
  Fe z;
  z.l[0] = z.l[1] = z.l[2] = z.l[3] = 0;
  return z;
}
__host__ __device__ __forceinline__ bool fe_eq(const Fe &a, const Fe &b) {
  return ((a.l[0] ^ b.l[0]) | (a.l[1] ^ b.l[1]) | (a.l[2] ^ b.l[2]) | (a.l[3] ^ b.l[3])) == 0;
}
__host__ __device__ __forceinline__ bool geq4(const uint64_t *a, const uint64_t *b) {
  if (a[3] != b[3]) return a[3] > b[3];
  if (a[2] != b[2]) return a[2] > b[2];
  if (a[1] != b[1]) return a[1] > b[1];
  return a[0] >= b[0];
}
__host__ __device__ __forceinline__ uint64_t sub4(uint64_t *r, const uint64_t *a, const uint64_t *b) {
  uint64_t br = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    u128 d = (u128)a[i] - b[i] - br;
    r[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1;
  }
  return br;
}
__host__ __device__ __forceinline__ uint64_t add4(uint64_t *r, const uint64_t *a, const uint64_t *b) {
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    u128 s = (u128)a[i] + b[i] + c;
    r[i] = (uint64_t)s;
    c = (uint64_t)(s >> 64);
  }
  return c;
}

__host__ __device__ __forceinline__ Fe fadd(const FieldP &F, const Fe &a, const Fe &b) {
  Fe r;
  uint64_t c = add4(r.l, a.l, b.l);
  if (c || geq4(r.l, F.p)) sub4(r.l, r.l, F.p);
  return r;
}
__host__ __device__ __forceinline__ Fe fsub(const FieldP &F, const Fe &a, const Fe &b) {
  Fe r;
  if (sub4(r.l, a.l, b.l)) add4(r.l, r.l, F.p);
  return r;
}
__host__ __device__ __forceinline__ Fe fneg(const FieldP &F, const Fe &a) {
  if (fe_is_zero(a)) return a;
  Fe r;
  sub4(r.l, F.p, a.l);
  return r;
}
// 256-bit values <-> 9 limbs of 29 bits
__host__ __device__ __forceinline__ void to_limbs(const Fe &x, uint32_t *a) {
#pragma unroll
  for (int i = 0; i < kLimbs; ++i) {
    const int bit = kLimbBits * i, w = bit >> 6, s = bit & 63;
    uint64_t v = x.l[w] >> s;
    if (s > 64 - kLimbBits && w < 3) v |= x.l[w + 1] << (64 - s);
    a[i] = (uint32_t)v & kLimbMask;
  }
}
// One-word Montgomery reduction for p < 2^64 (goldilocks, constants.rs:7): a*b*2^-64 mod p from
// the 128-bit product and one reduction word.  a, b < p, so hi(ab) < p and hi(mp) < p; lo(ab) +
// lo(mp) = 0 mod 2^64 carries iff lo(ab) != 0; the sum < 2p may exceed 2^64 (128-bit compare).
__host__ __device__ __forceinline__ uint64_t mont64(const FieldP &F, uint64_t a, uint64_t b) {
  const u128 t = (u128)a * b;
  const uint64_t lo = (uint64_t)t, m = lo * F.np64;
  const u128 mp = (u128)m * F.p[0];
  u128 u = (t >> 64) + (mp >> 64) + (lo != 0);
  if (u >= F.p[0]) u -= F.p[0];
  return (uint64_t)u;
}
// The same Montgomery product as fmul256 (a*b*2^-261 mod p, so the representation, r2 and one are
// shared and kernels may mix the two paths) in two one-word reductions: mont64(mont64(a, b),
// 2^-133) = a*b*2^-64*2^-133*2^-64.  Eight 32-bit multiply-add pairs instead of 162 limb products.
__host__ __device__ __forceinline__ Fe fmul64(const FieldP &F, uint64_t a, uint64_t b) {
  Fe o;
  o.l[0] = mont64(F, mont64(F, a, b), F.k133);
  o.l[1] = o.l[2] = o.l[3] = 0;
  return o;
}
// Montgomery product a*b*2^-261 mod p, radix 2^29: the 81 limb products of each half go into
// 64-bit column accumulators with independent multiply-adds (no carry chain inside a column; a
// column holds at most 18 products < 2^58), then 9 reduction steps and one carry pass.  44 % lower
// dependent latency than a 8 x 32-bit CIOS on gfx950 (tools/micro/fmul28.hip: 0.60 vs 1.09 us
// per product for one wave), which is what the ordered elimination loop waits on.
__host__ __device__ __forceinline__ Fe fmul256(const FieldP &F, const Fe &A, const Fe &B) {
  uint32_t a[kLimbs], b[kLimbs];
  to_limbs(A, a);
  to_limbs(B, b);
  uint64_t T[2 * kLimbs];
#pragma unroll
  for (int k = 0; k < 2 * kLimbs; ++k) T[k] = 0;
#pragma unroll
  for (int i = 0; i < kLimbs; ++i)
#pragma unroll
    for (int j = 0; j < kLimbs; ++j) T[i + j] += (uint64_t)a[i] * b[j];
#pragma unroll
  for (int i = 0; i < kLimbs; ++i) {
    const uint32_t m = ((uint32_t)T[i] * F.np) & kLimbMask;
#pragma unroll
    for (int j = 0; j < kLimbs; ++j) T[i + j] += (uint64_t)m * F.pl[j];
    T[i + 1] += T[i] >> kLimbBits;
  }
  uint32_t r[kLimbs];
#pragma unroll
  for (int k = kLimbs; k < 2 * kLimbs - 1; ++k) {
    T[k + 1] += T[k] >> kLimbBits;
    r[k - kLimbs] = (uint32_t)T[k] & kLimbMask;
  }
  r[kLimbs - 1] = (uint32_t)T[2 * kLimbs - 1];
  // r < 2p: one conditional subtraction, limb-wise with borrow
  uint32_t d[kLimbs];
  int64_t br = 0;
#pragma unroll
  for (int k = 0; k < kLimbs; ++k) {
    const int64_t x = (int64_t)r[k] - F.pl[k] + br;
    d[k] = (uint32_t)x & kLimbMask;
    br = x >> kLimbBits;
  }
  const bool ge = br >= 0;
  Fe o;
  o.l[0] = o.l[1] = o.l[2] = o.l[3] = 0;
#pragma unroll
  for (int k = 0; k < kLimbs; ++k) {
    const uint64_t v = ge ? d[k] : r[k];
    const int bit = kLimbBits * k, w = bit >> 6, s = bit & 63;
    o.l[w] |= v << s;
    if (s > 64 - kLimbBits && w < 3) o.l[w + 1] |= v >> (64 - s);
  }
  return o;
}
// The field product every kernel uses: the one-word path for p < 2^64 (the prime is uniform over a
// launch, so the branch never diverges a wave), else fmul256.  The tail's ordered loop calls fmul256
// directly, and so does the head's (k_big_spec): the branch cost the tail 18 VGPRs and ~5 % of its
// time on the 256-bit primes, the head ~1.5 %; a goldilocks
// circuit gets the same residues either way.
__host__ __device__ __forceinline__ Fe fmul(const FieldP &F, const Fe &A, const Fe &B) {
  if (F.w64) return fmul64(F, A.l[0], B.l[0]);
  return fmul256(F, A, B);
}
// Montgomery square: the product half is symmetric (45 limb products instead of 81: off-diagonal
// ones doubled; a column still sums below 2^63), the reduction is fmul's.
__host__ __device__ __forceinline__ Fe fsqr(const FieldP &F, const Fe &A) {
  if (F.w64) return fmul64(F, A.l[0], A.l[0]);
  uint32_t a[kLimbs], a2[kLimbs];
  to_limbs(A, a);
#pragma unroll
  for (int i = 0; i < kLimbs; ++i) a2[i] = a[i] << 1;
  uint64_t T[2 * kLimbs];
#pragma unroll
  for (int k = 0; k < 2 * kLimbs; ++k) T[k] = 0;
#pragma unroll
  for (int i = 0; i < kLimbs; ++i) {
    T[2 * i] += (uint64_t)a[i] * a[i];
#pragma unroll
    for (int j = i + 1; j < kLimbs; ++j) T[i + j] += (uint64_t)a2[i] * a[j];
  }
#pragma unroll
  for (int i = 0; i < kLimbs; ++i) {
    const uint32_t m = ((uint32_t)T[i] * F.np) & kLimbMask;
#pragma unroll
    for (int j = 0; j < kLimbs; ++j) T[i + j] += (uint64_t)m * F.pl[j];
    T[i + 1] += T[i] >> kLimbBits;
  }
  uint32_t r[kLimbs];
#pragma unroll
  for (int k = kLimbs; k < 2 * kLimbs - 1; ++k) {
    T[k + 1] += T[k] >> kLimbBits;
    r[k - kLimbs] = (uint32_t)T[k] & kLimbMask;
  }
  r[kLimbs - 1] = (uint32_t)T[2 * kLimbs - 1];
  // r < 2p: one conditional subtraction, limb-wise with borrow
  uint32_t d[kLimbs];
  int64_t br = 0;
#pragma unroll
  for (int k = 0; k < kLimbs; ++k) {
    const int64_t x = (int64_t)r[k] - F.pl[k] + br;
    d[k] = (uint32_t)x & kLimbMask;
    br = x >> kLimbBits;
  }
  const bool ge = br >= 0;
  Fe o;
  o.l[0] = o.l[1] = o.l[2] = o.l[3] = 0;
#pragma unroll
  for (int k = 0; k < kLimbs; ++k) {
    const uint64_t v = ge ? d[k] : r[k];
    const int bit = kLimbBits * k, w = bit >> 6, s = bit & 63;
    o.l[w] |= v << s;
    if (s > 64 - kLimbBits && w < 3) o.l[w + 1] |= v >> (64 - s);
  }
  return o;
}
__host__ __device__ __forceinline__ Fe fto_mont(const FieldP &F, const Fe &c) { return fmul(F, c, F.r2); }
__host__ __device__ __forceinline__ Fe ffrom_mont(const FieldP &F, const Fe &a) {
  Fe o = fe_zero();
  o.l[0] = 1;
  return fmul(F, a, o);
}
// a^(p-2) = a^-1 for a != 0 (Fermat; kept as the reference implementation of finv).
__host__ __device__ inline Fe finv_fermat(const FieldP &F, const Fe &a) {
  Fe r = F.one, base = a;
  for (int w = 0; w < 4; ++w) {
    uint64_t e = F.pm2.l[w];
    for (int i = 0; i < 64; ++i) {
      if (e & 1) r = fmul(F, r, base);
      base = fmul(F, base, base);
      e >>= 1;
    }
  }
  return r;
}
// Inverse in Montgomery form: (aR)^-1 R^2 = (aR)^(p-2) as Montgomery powers, i.e. a^-1 = a^(p-2)
// (Fermat), left to right: ~254 squarings (fsqr) and a product per set bit of p-2.  The control flow
// follows the exponent only, so a wave never diverges.  The same value as num-bigint's mod_inverse
// (the inverse is unique); 3.2x lower latency for one wave than the binary extended GCD this
// replaced (tools/micro/finv_bench.hip).  0 -> 0.
__host__ __device__ inline Fe finv(const FieldP &F, const Fe &a) {
  int top = 3;
  while (top > 0 && F.pm2.l[top] == 0) --top;
  int bit = 63;
  while (bit > 0 && !((F.pm2.l[top] >> bit) & 1)) --bit;
  Fe r = a;  // the leading 1
  for (int w = top; w >= 0; --w) {
    const uint64_t e = F.pm2.l[w];
    for (int i = (w == top ? bit - 1 : 63); i >= 0; --i) {
      r = fsqr(F, r);
      if ((e >> i) & 1) r = fmul(F, r, a);
    }
  }
  return r;
}

inline FieldP make_field(const uint64_t prime[4]) {
  FieldP F;
  for (int i = 0; i < 4; ++i) F.p[i] = prime[i];
  Fe pf;
  for (int i = 0; i < 4; ++i) pf.l[i] = prime[i];
  to_limbs(pf, F.pl);
  uint32_t inv = 1;  // p^-1 mod 2^29 (Newton)
  for (int i = 0; i < 5; ++i) inv *= 2 - F.pl[0] * inv;
  F.np = (0u - inv) & kLimbMask;
  F.w64 = prime[1] == 0 && prime[2] == 0 && prime[3] == 0;
  uint64_t inv64 = 1;  // p^-1 mod 2^64 (Newton: each step doubles the correct bits)
  for (int i = 0; i < 6; ++i) inv64 *= 2 - prime[0] * inv64;
  F.np64 = 0 - inv64;
  u128 h = 1;  // 2^-133 mod p by 133 halvings (p odd)
  for (int i = 0; i < 133 && F.w64; ++i) h = (h & 1) ? (h + prime[0]) >> 1 : h >> 1;
  F.k133 = (uint64_t)h;
  uint64_t x[4] = {1, 0, 0, 0};
  const int rb = kLimbBits * kLimbs;  // R = 2^rb
  for (int i = 0; i < 2 * rb; ++i) {
    uint64_t c = add4(x, x, x);
    if (c || geq4(x, F.p)) sub4(x, x, F.p);
    if (i == rb - 1)
      for (int j = 0; j < 4; ++j) F.one.l[j] = x[j];
  }
  for (int j = 0; j < 4; ++j) F.r2.l[j] = x[j];
  uint64_t two[4] = {2, 0, 0, 0};
  sub4(F.pm2.l, F.p, two);
  return F;
}

}  // namespace rs
