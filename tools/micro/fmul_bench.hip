// Microbenchmark: latency (one wave, dependent chain) and throughput of 256-bit Montgomery products.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include "../../circom_cvm_amd/csrc/field.hpp"
using namespace rs;

// 8x32-bit-limb CIOS (v_mad_u64_u32 does 32x32+64 natively)
__device__ __forceinline__ Fe fmul32(const FieldP &F, const Fe &A, const Fe &B) {
  uint32_t a[8], b[8], p[8], t[10];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    a[2 * i] = (uint32_t)A.l[i]; a[2 * i + 1] = (uint32_t)(A.l[i] >> 32);
    b[2 * i] = (uint32_t)B.l[i]; b[2 * i + 1] = (uint32_t)(B.l[i] >> 32);
    p[2 * i] = (uint32_t)F.p[i]; p[2 * i + 1] = (uint32_t)(F.p[i] >> 32);
  }
  const uint32_t np = (uint32_t)F.np;
#pragma unroll
  for (int i = 0; i < 10; ++i) t[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      uint64_t s = (uint64_t)a[j] * b[i] + t[j] + c;
      t[j] = (uint32_t)s;
      c = s >> 32;
    }
    uint64_t s = (uint64_t)t[8] + c;
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

template <int V>
__global__ void k_chain(FieldP F, Fe *io, int n, unsigned long long *cyc) {
  Fe x = io[threadIdx.x], y = io[64 + threadIdx.x];
  unsigned long long t0 = wall_clock64();
  for (int i = 0; i < n; ++i) x = V == 0 ? fmul(F, x, y) : fmul32(F, x, y);
  unsigned long long t1 = wall_clock64();
  io[threadIdx.x] = x;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

template <int V>
__global__ void k_inv(FieldP F, Fe *io, int n, unsigned long long *cyc) {
  Fe x = io[threadIdx.x];
  unsigned long long t0 = wall_clock64();
  for (int i = 0; i < n; ++i) { x = V == 0 ? finv_fermat(F, x) : finv(F, x); x.l[0] ^= 1; }
  unsigned long long t1 = wall_clock64();
  io[threadIdx.x] = x;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
  const uint64_t bn[4] = {0x43e1f593f0000001ULL, 0x2833e84879b97091ULL, 0xb85045b68181585dULL, 0x30644e72e131a029ULL};
  FieldP F = make_field(bn);
  Fe h[128];
  for (int i = 0; i < 128; ++i) for (int j = 0; j < 4; ++j) h[i].l[j] = (0x9e3779b97f4a7c15ULL * (i * 4 + j + 1)) >> 3;
  Fe *d; unsigned long long *c; hipMalloc(&d, sizeof(h)); hipMalloc(&c, 8);
  Fe out[2][128];
  for (int v = 0; v < 2; ++v) {
    for (int rep = 0; rep < 2; ++rep) {
      hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
      int n = 20000;
      if (v == 0) hipLaunchKernelGGL(k_chain<0>, 1, 64, 0, 0, F, d, n, c);
      else hipLaunchKernelGGL(k_chain<1>, 1, 64, 0, 0, F, d, n, c);
      unsigned long long cy; hipMemcpy(&cy, c, 8, hipMemcpyDeviceToHost);
      hipMemcpy(out[v], d, sizeof(h), hipMemcpyDeviceToHost);
      if (rep) printf("variant %s: %.1f ns per dependent fmul (one wave)\n", v ? "8x32 CIOS" : "4x64 CIOS (u128)", cy * 10.0 / n);
    }
  }
  bool same = true;
  for (int i = 0; i < 64; ++i) for (int j = 0; j < 4; ++j) same &= out[0][i].l[j] == out[1][i].l[j];
  printf("results identical: %s\n", same ? "yes" : "NO");
  for (int v = 0; v < 2; ++v) {
    hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
    int n = v ? 200 : 20;
    if (v == 0) hipLaunchKernelGGL(k_inv<0>, 1, 64, 0, 0, F, d, n, c);
    else hipLaunchKernelGGL(k_inv<1>, 1, 64, 0, 0, F, d, n, c);
    unsigned long long cy; hipMemcpy(&cy, c, 8, hipMemcpyDeviceToHost);
    printf("inverse %s: %.1f us per inversion (one wave, 64 lanes divergent)\n", v ? "binary GCD" : "Fermat", cy * 10.0 / n / 1000.0);
  }
  return 0;
}
