// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access patterns of this
// library's kernels (MI355X_MICROARCH.md 'HBM': only 16 B/lane streaming reads and writes are
// calibrated there).  Each kernel moves a known number of bytes over buffers far larger than the
// 256 MiB Infinity Cache; run it under separate `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE`
// passes and divide each dispatch's counter (KiB) by the byte counts printed here.
//   k_stream16   16 B / lane, coalesced (the guide's reference pattern: FETCH_SIZE = 1/2 of the bytes)
//   k_gather36   the frames / elimination pattern: a (u32 key, 32 B value) entry per lane at a random
//                entry index -- keys and values in separate arrays, as in the pool and the heaps
//   k_runs36     the same in runs of 4 consecutive entries at random run starts (short rows)
//   k_emit36     consecutive (key, value) slots written by consecutive lanes (the frames' emit)
// usage: pmc_calib  (prints "kernel read_bytes write_bytes" per dispatch, in launch order)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

struct Fe {
  uint64_t l[4];
};

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

__global__ void k_stream16(const uint4 *src, uint4 *dst, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) dst[i] = src[i];
}
// n entries read at random indices of [0, m), written consecutively
__global__ void k_gather36(const uint32_t *key, const Fe *val, uint64_t m, uint64_t n, uint32_t *okey, Fe *oval) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t j = mix(i + 0x9e3779b97f4a7c15ULL) % m;
    okey[i] = key[j];
    oval[i] = val[j];
  }
}
// runs of 4: entry i reads index start(i / 4) + i % 4
__global__ void k_runs36(const uint32_t *key, const Fe *val, uint64_t m, uint64_t n, uint32_t *okey, Fe *oval) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t j = (mix((i >> 2) + 0x9e3779b97f4a7c15ULL) % (m / 4)) * 4 + (i & 3);
    okey[i] = key[j];
    oval[i] = val[j];
  }
}
// consecutive slots written from registers (the reads are one small broadcast array)
__global__ void k_emit36(const Fe *seed, uint64_t n, uint32_t *okey, Fe *oval) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    Fe v = seed[threadIdx.x & 63];
    v.l[0] ^= i;
    okey[i] = (uint32_t)i;
    oval[i] = v;
  }
}

int main() {
  const uint64_t m = 64ull << 20;  // source entries: 256 MiB of keys + 2 GiB of values
  const uint64_t n = 32ull << 20;  // entries moved per launch
  uint32_t *key, *okey;
  Fe *val, *oval, *seed;
  uint4 *s16, *d16;
  CK(hipMalloc(&key, 4 * m));
  CK(hipMalloc(&val, 32 * m));
  CK(hipMalloc(&okey, 4 * n));
  CK(hipMalloc(&oval, 32 * n));
  CK(hipMalloc(&seed, 32 * 64));
  CK(hipMalloc(&s16, 16 * n * 2));
  CK(hipMalloc(&d16, 16 * n * 2));
  CK(hipMemset(key, 1, 4 * m));
  CK(hipMemset(val, 2, 32 * m));
  CK(hipMemset(seed, 3, 32 * 64));
  CK(hipMemset(s16, 4, 16 * n * 2));
  const dim3 g(4096), b(256);
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(k_stream16, g, b, 0, 0, (const uint4 *)s16, d16, 2 * n);
    printf("k_stream16 %llu %llu\n", (unsigned long long)(32 * n), (unsigned long long)(32 * n));
    hipLaunchKernelGGL(k_gather36, g, b, 0, 0, (const uint32_t *)key, (const Fe *)val, m, n, okey, oval);
    printf("k_gather36 %llu %llu\n", (unsigned long long)(36 * n), (unsigned long long)(36 * n));
    hipLaunchKernelGGL(k_runs36, g, b, 0, 0, (const uint32_t *)key, (const Fe *)val, m, n, okey, oval);
    printf("k_runs36 %llu %llu\n", (unsigned long long)(36 * n), (unsigned long long)(36 * n));
    hipLaunchKernelGGL(k_emit36, g, b, 0, 0, (const Fe *)seed, n, okey, oval);
    printf("k_emit36 %llu %llu\n", 0ull, (unsigned long long)(36 * n));
    CK(hipDeviceSynchronize());
  }
  return 0;
}
