// comm.hpp -- the exchange step of the sharded elimination.
//
// One circuit, one rank per GPU.  Every rank holds the whole input and runs the cheap global
// phases itself (eq / const-eq renaming, build_clusters); the clusters are dealt to the ranks and
// each rank eliminates only its own (A7-A12).  The eliminated-signal map -- per slot: `from`, the
// RHS offset/length, the leftovers, per cluster: #subs/#leftovers, and the pool entries those
// offsets point at -- is then exchanged so every rank continues with the full map.
//
// Two transports behind one interface:
//   RcclComm  -- production: RCCL over xGMI, one communicator per engine, collectives on the
//                engine's stream (allgatherv = grouped ncclBroadcast, one per root).
//   LocalComm -- several engines in one process (threads; typically on ONE device): host-staged
//                collectives behind a barrier.  It exists so the sharded path is testable on a
//                one-GPU box, and it is what rs_simplify_multi uses when a device is listed twice.
#pragma once

#include <rccl/rccl.h>

#include <condition_variable>
#include <cstring>
#include <mutex>
#include <vector>

namespace rs {

#define NC(x)                                                                                  \
  do {                                                                                         \
    ncclResult_t r_ = (x);                                                                     \
    if (r_ != ncclSuccess) throw RsError(RS_E_RCCL, std::string(#x) + ": " + ncclGetErrorString(r_)); \
  } while (0)

struct Comm {
  int rank = 0, world = 1;
  virtual ~Comm() {}
  // recv[q-th block] <- rank q's `counts[q]` bytes (send = this rank's block); blocks are packed
  // back to back in rank order.  Every rank passes the same counts.
  virtual void allgatherv(const void *send, void *recv, const std::vector<uint64_t> &counts, hipStream_t st) = 0;
  // in-place element-wise sum over ranks (u32 or u64 elements)
  virtual void allreduce_sum(void *buf, uint64_t n, int elem_bytes, hipStream_t st) = 0;
  // host scalar max over ranks (control decisions every rank must take together)
  virtual uint64_t max_u64(uint64_t v, hipStream_t st) = 0;
  // host vector gather: out[q] = rank q's v
  virtual std::vector<uint64_t> gather_u64(uint64_t v, hipStream_t st) = 0;
};

// ------------------------------------------------------------------ RCCL
struct RcclComm : Comm {
  ncclComm_t c = nullptr;
  uint64_t *d_scalar = nullptr;  // W u64 of device scratch for the scalar collectives
  RcclComm(ncclComm_t comm, int r, int w) : c(comm) {
    rank = r;
    world = w;
    HC(hipMalloc((void **)&d_scalar, 8 * (size_t)w));
  }
  ~RcclComm() override {
    if (d_scalar) (void)hipFree(d_scalar);
    if (c) (void)ncclCommDestroy(c);
  }
  void allgatherv(const void *send, void *recv, const std::vector<uint64_t> &counts, hipStream_t st) override {
    uint64_t off = 0;
    NC(ncclGroupStart());
    for (int q = 0; q < world; ++q) {
      if (counts[q])
        NC(ncclBroadcast(q == rank ? send : (const void *)((uint8_t *)recv + off), (uint8_t *)recv + off, counts[q],
                         ncclUint8, q, c, st));
      off += counts[q];
    }
    NC(ncclGroupEnd());
  }
  void allreduce_sum(void *buf, uint64_t n, int elem_bytes, hipStream_t st) override {
    if (!n) return;
    NC(ncclAllReduce(buf, buf, n, elem_bytes == 8 ? ncclUint64 : ncclUint32, ncclSum, c, st));
  }
  uint64_t max_u64(uint64_t v, hipStream_t st) override {
    HC(hipMemcpyAsync(d_scalar, &v, 8, hipMemcpyHostToDevice, st));
    NC(ncclAllReduce(d_scalar, d_scalar, 1, ncclUint64, ncclMax, c, st));
    uint64_t r = 0;
    HC(hipMemcpyAsync(&r, d_scalar, 8, hipMemcpyDeviceToHost, st));
    HC(hipStreamSynchronize(st));
    return r;
  }
  std::vector<uint64_t> gather_u64(uint64_t v, hipStream_t st) override {
    HC(hipMemcpyAsync(d_scalar + rank, &v, 8, hipMemcpyHostToDevice, st));
    NC(ncclAllGather(d_scalar + rank, d_scalar, 1, ncclUint64, c, st));
    std::vector<uint64_t> r(world);
    HC(hipMemcpyAsync(r.data(), d_scalar, 8 * (size_t)world, hipMemcpyDeviceToHost, st));
    HC(hipStreamSynchronize(st));
    return r;
  }
};

// ------------------------------------------------------------------ in-process (host-staged)
struct LocalGroup {
  int world;
  std::mutex m;
  std::condition_variable cv;
  uint64_t gen = 0;
  int arrived = 0;
  std::vector<std::vector<uint8_t>> slot;
  explicit LocalGroup(int w) : world(w), slot(w) {}
  void barrier() {
    std::unique_lock<std::mutex> lk(m);
    uint64_t g = gen;
    if (++arrived == world) {
      arrived = 0;
      ++gen;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return gen != g; });
    }
  }
};

struct LocalComm : Comm {
  LocalGroup *g;
  LocalComm(LocalGroup *grp, int r) : g(grp) {
    rank = r;
    world = grp->world;
  }
  void post(const void *dev, uint64_t bytes, hipStream_t st) {
    g->slot[rank].resize(bytes);
    if (bytes) HC(hipMemcpyAsync(g->slot[rank].data(), dev, bytes, hipMemcpyDeviceToHost, st));
    HC(hipStreamSynchronize(st));
  }
  void allgatherv(const void *send, void *recv, const std::vector<uint64_t> &counts, hipStream_t st) override {
    post(send, counts[rank], st);
    g->barrier();
    uint64_t off = 0;
    for (int q = 0; q < world; ++q) {
      if (counts[q]) HC(hipMemcpyAsync((uint8_t *)recv + off, g->slot[q].data(), counts[q], hipMemcpyHostToDevice, st));
      off += counts[q];
    }
    HC(hipStreamSynchronize(st));
    g->barrier();  // the slots may be reused only after every rank has read them
  }
  void allreduce_sum(void *buf, uint64_t n, int elem_bytes, hipStream_t st) override {
    if (!n) return;
    post(buf, n * elem_bytes, st);
    g->barrier();
    std::vector<uint8_t> acc(g->slot[0]);
    for (int q = 1; q < world; ++q) {
      if (elem_bytes == 8) {
        uint64_t *a = (uint64_t *)acc.data();
        const uint64_t *b = (const uint64_t *)g->slot[q].data();
        for (uint64_t i = 0; i < n; ++i) a[i] += b[i];
      } else {
        uint32_t *a = (uint32_t *)acc.data();
        const uint32_t *b = (const uint32_t *)g->slot[q].data();
        for (uint64_t i = 0; i < n; ++i) a[i] += b[i];
      }
    }
    HC(hipMemcpyAsync(buf, acc.data(), n * elem_bytes, hipMemcpyHostToDevice, st));
    HC(hipStreamSynchronize(st));
    g->barrier();
  }
  std::vector<uint64_t> gather_u64(uint64_t v, hipStream_t) override {
    g->slot[rank].resize(8);
    memcpy(g->slot[rank].data(), &v, 8);
    g->barrier();
    std::vector<uint64_t> r(world);
    for (int q = 0; q < world; ++q) memcpy(&r[q], g->slot[q].data(), 8);
    g->barrier();
    return r;
  }
  uint64_t max_u64(uint64_t v, hipStream_t st) override {
    uint64_t m = 0;
    for (uint64_t x : gather_u64(v, st)) m = std::max(m, x);
    return m;
  }
};

}  // namespace rs
