// D2H by copy engine vs by a kernel writing pinned host memory, and what each does to the latency of
// a small D2H on another stream meanwhile (the run's scalar read-backs).
// usage: d2h_kernel  (GPU box)
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_to_host(const uint4 *src, uint4 *dst, uint64_t n16) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) dst[i] = src[i];
}
__global__ void k_to_host_nt(const uint4 *src, uint4 *dst, uint64_t n16) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x)
  {
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    const uint4 x = src[i];
    v4u y = {x.x, x.y, x.z, x.w};
    __builtin_nontemporal_store(y, (v4u *)(dst + i));
  }
}

static double now() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main() {
  const size_t n = 512ull << 20;
  void *d, *h, *hsmall, *dsmall;
  CK(hipMalloc(&d, n));
  CK(hipMemset(d, 1, n));
  CK(hipHostMalloc(&h, n, hipHostMallocDefault));
  CK(hipHostMalloc(&hsmall, 64, hipHostMallocDefault));
  CK(hipMalloc(&dsmall, 64));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto small_lat = [&](int reps, bool pageable) {  // small D2H round trips on s2 while s1 is busy
    std::vector<double> t;
    uint64_t v = 0;
    for (int r = 0; r < reps; ++r) {
      const double a = now();
      (void)hipMemcpyAsync(pageable ? (void *)&v : hsmall, dsmall, 8, hipMemcpyDeviceToHost, s2);
      (void)hipStreamSynchronize(s2);
      t.push_back(now() - a);
    }
    double s = 0;
    for (double x : t) s += x;
    return s / reps;
  };
  printf("idle: small D2H %.3f ms pinned, %.3f ms pageable\n", small_lat(20, false), small_lat(20, true));
  // copy engine, 16 MB chunks
  for (int rep = 0; rep < 2; ++rep) {
    CK(hipEventRecord(e0, s1));
    for (size_t o = 0; o < n; o += 16ull << 20) CK(hipMemcpyAsync((char *)h + o, (char *)d + o, 16ull << 20, hipMemcpyDeviceToHost, s1));
    CK(hipEventRecord(e1, s1));
    const double lp = small_lat(10, false), lq = small_lat(10, true);
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (rep) printf("copy engine 16MB chunks: %.1f GB/s; small D2H meanwhile %.3f ms pinned, %.3f ms pageable\n", n / ms / 1e6, lp, lq);
  }
  for (int nt = 0; nt < 2; ++nt)
    for (int g : {8, 16, 32, 64, 128, 256, 1024}) {
      for (int rep = 0; rep < 2; ++rep) {
        CK(hipEventRecord(e0, s1));
        if (nt) hipLaunchKernelGGL(k_to_host_nt, dim3(g), dim3(256), 0, s1, (const uint4 *)d, (uint4 *)h, (uint64_t)(n / 16));
        else hipLaunchKernelGGL(k_to_host, dim3(g), dim3(256), 0, s1, (const uint4 *)d, (uint4 *)h, (uint64_t)(n / 16));
        CK(hipEventRecord(e1, s1));
        const double lp = small_lat(10, false), lq = small_lat(10, true);
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (rep) printf("kernel%s %4d WGs: %.1f GB/s; small D2H meanwhile %.3f ms pinned, %.3f ms pageable\n", nt ? " (nt)" : "", g,
                        n / ms / 1e6, lp, lq);
      }
    }
  // correctness of the kernel path
  CK(hipMemset(d, 7, n));
  hipLaunchKernelGGL(k_to_host, dim3(256), dim3(256), 0, s1, (const uint4 *)d, (uint4 *)h, (uint64_t)(n / 16));
  CK(hipStreamSynchronize(s1));
  size_t bad = 0;
  for (size_t i = 0; i < n; i += 4093) bad += ((unsigned char *)h)[i] != 7;
  printf("kernel copy check: %zu bad samples\n", bad);
  return 0;
}
