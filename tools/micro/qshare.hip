// Do HIP streams share hardware queues (GPU_MAX_HW_QUEUES) so that a kernel on one stream waits for a
// bulk copy + kernel queued on another?  Streams are created in the engine's order and priorities
// (st, st2 high, stc, stx, str, ste low, stg); the copy stream stc gets 1 GiB of H2D followed by a
// kernel, then an empty kernel + sync on every other stream is timed while the copy is in flight.
// usage: qshare  (GPU box; run with different GPU_MAX_HW_QUEUES)
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_nop(uint64_t *p) { if (threadIdx.x == 0 && blockIdx.x == 0 && p[0] == 12345) p[1] = 1; }

static double now() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main() {
  const char *q = getenv("GPU_MAX_HW_QUEUES");
  printf("GPU_MAX_HW_QUEUES=%s\n", q ? q : "(unset)");
  const size_t n = 1ull << 30;
  void *d, *h;
  uint64_t *dsmall;
  CK(hipMalloc(&d, n));
  CK(hipHostMalloc(&h, n, hipHostMallocDefault));
  memset(h, 2, n);
  CK(hipMalloc((void **)&dsmall, 64));
  CK(hipMemset(dsmall, 0, 64));
  int lo = 0, hi = 0;
  CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  const char *names[7] = {"st", "st2(hi)", "stc", "stx", "str", "ste(lo)", "stg"};
  hipStream_t s[7];
  // QSHARE_CUMASK=1: the normal-priority streams get a full CU mask (hipExtStreamCreateWithCUMask), which
  // gives a stream a hardware queue of its own instead of one from the shared pool
  const bool cumask = getenv("QSHARE_CUMASK") != nullptr;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  uint32_t mask[16] = {};
  for (int c = 0; c < ncu && c < 512; ++c) mask[c / 32] |= 1u << (c % 32);
  const int pre = getenv("QSHARE_PRE") ? atoi(getenv("QSHARE_PRE")) : 0;  // streams some other library made first
  printf("CU mask: %s (%d CUs), %d streams created before\n", cumask ? "full, per stream" : "none", ncu, pre);
  for (int i = 0; i < pre; ++i) {
    hipStream_t x;
    CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
    hipLaunchKernelGGL(k_nop, dim3(1), dim3(64), 0, x, dsmall);
    CK(hipStreamSynchronize(x));
  }
  for (int i = 0; i < 7; ++i) {
    if (i == 1) CK(hipStreamCreateWithPriority(&s[i], hipStreamNonBlocking, hi));
    else if (i == 5) CK(hipStreamCreateWithPriority(&s[i], hipStreamNonBlocking, lo));
    else if (cumask) CK(hipExtStreamCreateWithCUMask(&s[i], (ncu + 31) / 32, mask));
    else CK(hipStreamCreateWithFlags(&s[i], hipStreamNonBlocking));
  }
  const int cs = 2;  // the copy stream
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipDeviceSynchronize());
    const double t0 = now();
    for (size_t o = 0; o < n; o += 32ull << 20) CK(hipMemcpyAsync((char *)d + o, (char *)h + o, 32ull << 20, hipMemcpyHostToDevice, s[cs]));
    hipLaunchKernelGGL(k_nop, dim3(1), dim3(64), 0, s[cs], dsmall);
    printf("rep %d:", rep);
    for (int i = 0; i < 7; ++i) {
      if (i == cs) continue;
      const double a = now();
      hipLaunchKernelGGL(k_nop, dim3(1), dim3(64), 0, s[i], dsmall);
      CK(hipStreamSynchronize(s[i]));
      printf(" %s %.2f ms |", names[i], now() - a);
    }
    CK(hipStreamSynchronize(s[cs]));
    printf(" copy stream done at %.2f ms\n", now() - t0);
  }
  return 0;
}
