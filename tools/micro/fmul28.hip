// Prototype: Montgomery product in radix 2^28 (10 limbs, R = 2^280) with 64-bit column
// accumulators, against the 8x32 CIOS of field.hpp.  Checks canonical equality and measures the
// dependent latency of one wave.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../circom_cvm_amd/csrc/field.hpp"
using namespace rs;

struct F28 { uint32_t p[10]; uint32_t np; uint64_t p64[4]; Fe one, r2; };
constexpr uint32_t M28 = (1u << 28) - 1;

__host__ __device__ __forceinline__ void unpack28(const Fe &x, uint32_t *a) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const int bit = 28 * i, w = bit >> 6, s = bit & 63;
    uint64_t v = x.l[w] >> s;
    if (s > 36 && w < 3) v |= x.l[w + 1] << (64 - s);
    a[i] = (uint32_t)v & M28;
  }
}
__host__ __device__ __forceinline__ Fe fmul28(const F28 &F, const Fe &A, const Fe &B) {
  uint32_t a[10], b[10];
  unpack28(A, a);
  unpack28(B, b);
  uint64_t T[20];
#pragma unroll
  for (int k = 0; k < 20; ++k) T[k] = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i)
#pragma unroll
    for (int j = 0; j < 10; ++j) T[i + j] += (uint64_t)a[i] * b[j];
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t m = ((uint32_t)T[i] * F.np) & M28;
#pragma unroll
    for (int j = 0; j < 10; ++j) T[i + j] += (uint64_t)m * F.p[j];
    T[i + 1] += T[i] >> 28;
  }
  uint32_t r[10];
#pragma unroll
  for (int k = 10; k < 19; ++k) { T[k + 1] += T[k] >> 28; r[k - 10] = (uint32_t)T[k] & M28; }
  r[9] = (uint32_t)T[19];
  // r < 2p: subtract p once if needed (limbwise with borrow)
  uint32_t d[10];
  int64_t br = 0;
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    int64_t x = (int64_t)r[k] - F.p[k] + br;
    d[k] = (uint32_t)x & M28;
    br = x >> 28;
  }
  const bool ge = br >= 0;
  Fe o;
  uint32_t *s = ge ? d : r;
  o.l[0] = (uint64_t)s[0] | ((uint64_t)s[1] << 28) | ((uint64_t)s[2] << 56);
  o.l[1] = ((uint64_t)s[2] >> 8) | ((uint64_t)s[3] << 20) | ((uint64_t)s[4] << 48);
  o.l[2] = ((uint64_t)s[4] >> 16) | ((uint64_t)s[5] << 12) | ((uint64_t)s[6] << 40);
  o.l[3] = ((uint64_t)s[6] >> 24) | ((uint64_t)s[7] << 4) | ((uint64_t)s[8] << 32) | ((uint64_t)s[9] << 60);
  return o;
}

F28 make28(const uint64_t prime[4]) {
  F28 F;
  Fe p; for (int i = 0; i < 4; ++i) { p.l[i] = prime[i]; F.p64[i] = prime[i]; }
  unpack28(p, F.p);
  uint32_t inv = 1;  // p^-1 mod 2^28 by Newton
  for (int i = 0; i < 5; ++i) inv *= 2 - F.p[0] * inv;
  F.np = (0u - inv) & M28;
  uint64_t x[4] = {1, 0, 0, 0};
  for (int i = 0; i < 560; ++i) {
    uint64_t c = add4(x, x, x);
    if (c || geq4(x, F.p64)) sub4(x, x, F.p64);
    if (i == 279) for (int j = 0; j < 4; ++j) F.one.l[j] = x[j];
  }
  for (int j = 0; j < 4; ++j) F.r2.l[j] = x[j];
  return F;
}


template <int W, int N>
struct FR { uint32_t p[N]; uint32_t np; uint64_t p64[4]; Fe one, r2; };
template <int W, int N>
__host__ __device__ __forceinline__ void unpackR(const Fe &x, uint32_t *a) {
  const uint32_t M = (1u << W) - 1;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const int bit = W * i, w = bit >> 6, s = bit & 63;
    uint64_t v = w < 4 ? x.l[w] >> s : 0;
    if (s > 64 - W && w < 3) v |= x.l[w + 1] << (64 - s);
    a[i] = (uint32_t)v & M;
  }
}
template <int W, int N>
__host__ __device__ __forceinline__ Fe fmulR(const FR<W, N> &F, const Fe &A, const Fe &B) {
  const uint32_t M = (1u << W) - 1;
  uint32_t a[N], b[N];
  unpackR<W, N>(A, a);
  unpackR<W, N>(B, b);
  uint64_t T[2 * N];
#pragma unroll
  for (int k = 0; k < 2 * N; ++k) T[k] = 0;
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int j = 0; j < N; ++j) T[i + j] += (uint64_t)a[i] * b[j];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const uint32_t m = ((uint32_t)T[i] * F.np) & M;
#pragma unroll
    for (int j = 0; j < N; ++j) T[i + j] += (uint64_t)m * F.p[j];
    T[i + 1] += T[i] >> W;
  }
  uint32_t r[N];
#pragma unroll
  for (int k = N; k < 2 * N - 1; ++k) { T[k + 1] += T[k] >> W; r[k - N] = (uint32_t)T[k] & M; }
  r[N - 1] = (uint32_t)T[2 * N - 1];
  uint32_t d[N];
  int64_t br = 0;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    int64_t x = (int64_t)r[k] - F.p[k] + br;
    d[k] = (uint32_t)x & M;
    br = x >> W;
  }
  const bool ge = br >= 0;
  Fe o;
  o.l[0] = o.l[1] = o.l[2] = o.l[3] = 0;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    const uint64_t v = ge ? d[k] : r[k];
    const int bit = W * k, w = bit >> 6, s = bit & 63;
    if (w < 4) o.l[w] |= v << s;
    if (s > 64 - W && w < 3) o.l[w + 1] |= v >> (64 - s);
  }
  return o;
}
template <int W, int N>
FR<W, N> makeR(const uint64_t prime[4]) {
  FR<W, N> F;
  Fe p; for (int i = 0; i < 4; ++i) { p.l[i] = prime[i]; F.p64[i] = prime[i]; }
  unpackR<W, N>(p, F.p);
  uint32_t inv = 1;
  for (int i = 0; i < 5; ++i) inv *= 2 - F.p[0] * inv;
  F.np = (0u - inv) & ((1u << W) - 1);
  uint64_t x[4] = {1, 0, 0, 0};
  for (int i = 0; i < 2 * W * N; ++i) {
    uint64_t c = add4(x, x, x);
    if (c || geq4(x, F.p64)) sub4(x, x, F.p64);
    if (i == W * N - 1) for (int j = 0; j < 4; ++j) F.one.l[j] = x[j];
  }
  for (int j = 0; j < 4; ++j) F.r2.l[j] = x[j];
  return F;
}
template <int W, int N>
__global__ void k_chainR(FR<W, N> G, Fe *io, int n, unsigned long long *cyc) {
  Fe x = io[threadIdx.x], y = io[64 + threadIdx.x];
  unsigned long long t0 = wall_clock64();
  for (int i = 0; i < n; ++i) x = fmulR<W, N>(G, x, y);
  unsigned long long t1 = wall_clock64();
  io[threadIdx.x] = x;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
template <int W, int N>
int checkR(const uint64_t (*P)[4], int np_) {
  int bad = 0;
  uint64_t seed = 7;
  auto rnd = [&]() { seed = seed * 6364136223846793005ULL + 1442695040888963407ULL; return seed; };
  for (int q = 0; q < np_; ++q) {
    FieldP F = make_field(P[q]);
    FR<W, N> G = makeR<W, N>(P[q]);
    for (int t = 0; t < 20000; ++t) {
      Fe a, b;
      for (int i = 0; i < 4; ++i) { a.l[i] = rnd(); b.l[i] = rnd(); }
      a = ffrom_mont(F, fto_mont(F, a)); b = ffrom_mont(F, fto_mont(F, b));
      Fe c1 = ffrom_mont(F, fmul(F, fto_mont(F, a), fto_mont(F, b)));
      Fe am = fmulR<W, N>(G, a, G.r2), bm = fmulR<W, N>(G, b, G.r2);
      Fe one; one.l[0] = 1; one.l[1] = one.l[2] = one.l[3] = 0;
      Fe c2 = fmulR<W, N>(G, fmulR<W, N>(G, am, bm), one);
      if (!fe_eq(c1, c2)) ++bad;
    }
  }
  return bad;
}

template <int V>
__global__ void k_chain(FieldP F, F28 G, Fe *io, int n, unsigned long long *cyc) {
  Fe x = io[threadIdx.x], y = io[64 + threadIdx.x];
  unsigned long long t0 = wall_clock64();
  for (int i = 0; i < n; ++i) x = V == 0 ? fmul(F, x, y) : fmul28(G, x, y);
  unsigned long long t1 = wall_clock64();
  io[threadIdx.x] = x;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
  const uint64_t P[3][4] = {{0x43e1f593f0000001ULL, 0x2833e84879b97091ULL, 0xb85045b68181585dULL, 0x30644e72e131a029ULL},
    {0xffffffffffffffffULL, 0x00000000ffffffffULL, 0, 0xffffffff00000001ULL}, {0xffffffff00000001ULL, 0, 0, 0}};
  // host correctness: canonical a*b via both
  int bad = 0;
  uint64_t seed = 1;
  auto rnd = [&]() { seed = seed * 6364136223846793005ULL + 1442695040888963407ULL; return seed; };
  for (auto &pp : P) {
    FieldP F = make_field(pp);
    F28 G = make28(pp);
    for (int t = 0; t < 20000; ++t) {
      Fe a, b;
      for (int i = 0; i < 4; ++i) { a.l[i] = rnd(); b.l[i] = rnd(); }
      a = ffrom_mont(F, fto_mont(F, a)); b = ffrom_mont(F, fto_mont(F, b));  // reduce mod p
      Fe c1 = ffrom_mont(F, fmul(F, fto_mont(F, a), fto_mont(F, b)));
      Fe am = fmul28(G, a, G.r2), bm = fmul28(G, b, G.r2);
      Fe one; one.l[0] = 1; one.l[1] = one.l[2] = one.l[3] = 0;
      Fe c2 = fmul28(G, fmul28(G, am, bm), one);
      if (!fe_eq(c1, c2)) ++bad;
    }
  }
  printf("host mismatches: %d  (29x9: %d, 28x10 generic: %d)\n", bad, checkR<29, 9>(P, 3), checkR<28, 10>(P, 3));
  FieldP F = make_field(P[0]);
  F28 G = make28(P[0]);
  Fe h[128];
  for (int i = 0; i < 128; ++i) for (int j = 0; j < 4; ++j) h[i].l[j] = (0x9e3779b97f4a7c15ULL * (i * 4 + j + 1)) >> 3;
  Fe *d; unsigned long long *c; (void)hipMalloc(&d, sizeof(h)); (void)hipMalloc(&c, 8);
  for (int v = 0; v < 2; ++v)
    for (int rep = 0; rep < 2; ++rep) {
      (void)hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
      int n = 20000;
      if (v == 0) hipLaunchKernelGGL(k_chain<0>, 1, 64, 0, 0, F, G, d, n, c);
      else hipLaunchKernelGGL(k_chain<1>, 1, 64, 0, 0, F, G, d, n, c);
      unsigned long long cy; (void)hipMemcpy(&cy, c, 8, hipMemcpyDeviceToHost);
      if (rep) printf("%s: %.1f ns per dependent product (one wave)\n", v ? "radix 2^28 (10 limbs)" : "8x32 CIOS", cy * 10.0 / n);
    }
  {
    FR<29, 9> G9 = makeR<29, 9>(P[0]);
    FR<28, 10> G10 = makeR<28, 10>(P[0]);
    for (int v = 0; v < 2; ++v)
      for (int rep = 0; rep < 2; ++rep) {
        (void)hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
        int n = 20000;
        if (v == 0) hipLaunchKernelGGL((k_chainR<29, 9>), 1, 64, 0, 0, G9, d, n, c);
        else hipLaunchKernelGGL((k_chainR<28, 10>), 1, 64, 0, 0, G10, d, n, c);
        unsigned long long cy; (void)hipMemcpy(&cy, c, 8, hipMemcpyDeviceToHost);
        if (rep) printf("generic %s: %.1f ns per dependent product (one wave)\n", v ? "28x10" : "29x9", cy * 10.0 / n);
      }
  }
  return 0;
}
