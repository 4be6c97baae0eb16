// field.hpp -- F_p arithmetic for the device (and host helpers), p < 2^256 odd.
//
// Replaces circom_algebra/src/modular_arithmetic.rs:9-91 (num-bigint-dig BigInt + double
// remainder per op) with fixed 4x64-bit limbs in Montgomery form (R = 2^256): one CIOS product
// per field multiplication, carry-propagating add/sub with a single conditional correction.
// Results are canonical residues, identical to the reference's ((a % p) + p) % p.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace rs {

typedef unsigned __int128 u128;

struct __attribute__((aligned(16))) Fe {
  uint64_t l[4];
};

struct FieldP {
  uint64_t p[4];
  uint64_t np;  // -p^-1 mod 2^64
  Fe r2;        // R^2 mod p
  Fe one;       // R mod p
  Fe pm2;       // p - 2 (Fermat exponent)
  Fe r3;        // R^3 mod p (Montgomery-form inverse from a plain binary GCD)
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
// CIOS Montgomery product over 8 x 32-bit limbs: every step is one 32x32+64 multiply-add, which
// gfx950 issues natively (v_mad_u64_u32); 30 % lower dependent latency than 4 x 64-bit limbs
// through unsigned __int128 (tools/micro/fmul_bench.hip: 1.08 vs 1.55 us per product, one wave).
__host__ __device__ __forceinline__ Fe fmul(const FieldP &F, const Fe &A, const Fe &B) {
  uint32_t a[8], b[8], p[8], t[10];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    a[2 * i] = (uint32_t)A.l[i];
    a[2 * i + 1] = (uint32_t)(A.l[i] >> 32);
    b[2 * i] = (uint32_t)B.l[i];
    b[2 * i + 1] = (uint32_t)(B.l[i] >> 32);
    p[2 * i] = (uint32_t)F.p[i];
    p[2 * i + 1] = (uint32_t)(F.p[i] >> 32);
  }
  const uint32_t np = (uint32_t)F.np;  // -p^-1 mod 2^32 (low word of -p^-1 mod 2^64)
#pragma unroll
  for (int i = 0; i < 10; ++i) t[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint64_t c = 0, s;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s = (uint64_t)a[j] * b[i] + t[j] + c;
      t[j] = (uint32_t)s;
      c = s >> 32;
    }
    s = (uint64_t)t[8] + c;
    t[8] = (uint32_t)s;
    t[9] = (uint32_t)(s >> 32);
    const uint32_t m = t[0] * np;
    s = (uint64_t)m * p[0] + t[0];
    c = s >> 32;
#pragma unroll
    for (int j = 1; j < 8; ++j) {
      s = (uint64_t)m * p[j] + t[j] + c;
      t[j - 1] = (uint32_t)s;
      c = s >> 32;
    }
    s = (uint64_t)t[8] + c;
    t[7] = (uint32_t)s;
    t[8] = t[9] + (uint32_t)(s >> 32);
  }
  Fe r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r.l[i] = (uint64_t)t[2 * i] | ((uint64_t)t[2 * i + 1] << 32);
  if (t[8] || geq4(r.l, F.p)) sub4(r.l, r.l, F.p);
  return r;
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
__host__ __device__ __forceinline__ void shr1c(uint64_t *x, uint64_t top) {  // x = (top:x) >> 1
  x[0] = (x[0] >> 1) | (x[1] << 63);
  x[1] = (x[1] >> 1) | (x[2] << 63);
  x[2] = (x[2] >> 1) | (x[3] << 63);
  x[3] = (x[3] >> 1) | (top << 63);
}
__host__ __device__ __forceinline__ bool is_one4(const uint64_t *x) { return x[0] == 1 && (x[1] | x[2] | x[3]) == 0; }
// Inverse in Montgomery form: binary extended Euclid on the residue aR (shifts, adds and
// subtractions only), (aR)^-1 = a^-1 R^-1, then one product by R^3 gives a^-1 R.  The same value
// as num-bigint's mod_inverse (the inverse is unique); about 30x lower latency than Fermat's
// ~384 dependent products (tools/micro/fmul_bench.hip).
__host__ __device__ inline Fe finv(const FieldP &F, const Fe &a) {
  if (fe_is_zero(a)) return a;
  uint64_t u[4], v[4], x1[4] = {1, 0, 0, 0}, x2[4] = {0, 0, 0, 0};
  for (int i = 0; i < 4; ++i) { u[i] = a.l[i]; v[i] = F.p[i]; }
  while (!is_one4(u) && !is_one4(v)) {
    while ((u[0] & 1) == 0) {
      shr1c(u, 0);
      uint64_t c = (x1[0] & 1) ? add4(x1, x1, F.p) : 0;
      shr1c(x1, c);
    }
    while ((v[0] & 1) == 0) {
      shr1c(v, 0);
      uint64_t c = (x2[0] & 1) ? add4(x2, x2, F.p) : 0;
      shr1c(x2, c);
    }
    if (geq4(u, v)) {
      sub4(u, u, v);
      if (sub4(x1, x1, x2)) add4(x1, x1, F.p);
    } else {
      sub4(v, v, u);
      if (sub4(x2, x2, x1)) add4(x2, x2, F.p);
    }
  }
  Fe r;
  const uint64_t *x = is_one4(u) ? x1 : x2;
  for (int i = 0; i < 4; ++i) r.l[i] = x[i];
  return fmul(F, r, F.r3);
}

inline FieldP make_field(const uint64_t prime[4]) {
  FieldP F;
  for (int i = 0; i < 4; ++i) F.p[i] = prime[i];
  uint64_t inv = 1;
  for (int i = 0; i < 7; ++i) inv *= 2 - F.p[0] * inv;
  F.np = (uint64_t)0 - inv;
  uint64_t x[4] = {1, 0, 0, 0};
  for (int i = 0; i < 512; ++i) {
    uint64_t c = add4(x, x, x);
    if (c || geq4(x, F.p)) sub4(x, x, F.p);
    if (i == 255)
      for (int j = 0; j < 4; ++j) F.one.l[j] = x[j];
  }
  for (int j = 0; j < 4; ++j) F.r2.l[j] = x[j];
  uint64_t two[4] = {2, 0, 0, 0};
  sub4(F.pm2.l, F.p, two);
  F.r3 = fmul(F, F.r2, F.r2);
  return F;
}

}  // namespace rs
