// Dependent latency of one wave's field inversion: binary extended GCD (finv) vs Fermat (finv_fermat).
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../circom_cvm_amd/csrc/field.hpp"
using namespace rs;

template <int V>
__global__ void k_chain(FieldP F, Fe *io, int n, unsigned long long *cyc) {
  Fe x = io[threadIdx.x];
  unsigned long long t0 = wall_clock64();
  for (int i = 0; i < n; ++i) x = V == 0 ? finv(F, x) : finv_fermat(F, x);
  unsigned long long t1 = wall_clock64();
  io[threadIdx.x] = x;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
  const uint64_t P[4] = {0x43e1f593f0000001ULL, 0x2833e84879b97091ULL, 0xb85045b68181585dULL, 0x30644e72e131a029ULL};
  FieldP F = make_field(P);
  Fe h[64];
  for (int i = 0; i < 64; ++i) for (int j = 0; j < 4; ++j) h[i].l[j] = (0x9e3779b97f4a7c15ULL * (i * 4 + j + 1)) >> 4;
  Fe *d; unsigned long long *c; (void)hipMalloc(&d, sizeof(h)); (void)hipMalloc(&c, 8);
  for (int v = 0; v < 2; ++v)
    for (int rep = 0; rep < 2; ++rep) {
      (void)hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
      int n = 50;
      if (v == 0) hipLaunchKernelGGL(k_chain<0>, 1, 64, 0, 0, F, d, n, c);
      else hipLaunchKernelGGL(k_chain<1>, 1, 64, 0, 0, F, d, n, c);
      unsigned long long cy; (void)hipMemcpy(&cy, c, 8, hipMemcpyDeviceToHost);
      if (rep) printf("%s: %.1f us per dependent inversion (one wave)\n", v ? "Fermat" : "binary GCD", cy * 10.0 / n / 1000.0);
    }
  return 0;
}
