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

#include <fcntl.h>
#include <rccl/rccl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <condition_variable>
#include <cstring>
#include <map>
#include <mutex>
#include <set>
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
  // every rank has arrived (and its work on `st` before the call is complete)
  virtual void barrier(hipStream_t st) { (void)gather_u64(0, st); }
  // this rank's call failed: ranks waiting in a collective of an in-process group leave it with an
  // error (RCCL ranks cannot be released this way: a failed rank there ends the job)
  virtual void fail() {}
  // Every entry point that may run collectives brackets itself with begin_call / end_call (every
  // rank makes the same sequence of calls).  A failure belongs to the call it happened in: once
  // every rank has left that call, the group is usable again (in-process groups; no-ops for RCCL).
  virtual void begin_call() {}
  virtual void end_call() {}
  // Collective: host memory every rank of the group sees at the same bytes (page-locked, registered
  // with HIP, so each rank's D2H of its own part of the result lands there directly over its own
  // PCIe link).  Slot `slot` grows only; every rank passes the same size.  nullptr if unavailable.
  virtual void *shared_host(int slot, size_t bytes, hipStream_t st) = 0;
};

// ------------------------------------------------------------------ RCCL
// one process per rank: the shared host region is a POSIX shared-memory segment each rank maps and
// registers; its name carries a tag rank 0 chose (sent with the first gather) and a generation
struct ShmSeg {
  void *p = nullptr;
  size_t cap = 0;
  bool registered = false;
};
struct RcclComm : Comm {
  ncclComm_t c = nullptr;
  uint64_t *d_scalar = nullptr;  // W u64 of device scratch for the scalar collectives
  ShmSeg shm[4];
  uint64_t shm_tag = 0, shm_gen = 0;
  RcclComm(ncclComm_t comm, int r, int w) : c(comm) {
    rank = r;
    world = w;
    HC(hipMalloc((void **)&d_scalar, 8 * (size_t)w));
  }
  ~RcclComm() override {
    for (ShmSeg &g : shm) unmap(g);
    if (d_scalar) (void)hipFree(d_scalar);
    if (c) (void)ncclCommDestroy(c);
  }
  static void unmap(ShmSeg &g) {
    if (!g.p) return;
    if (g.registered) (void)hipHostUnregister(g.p);
    munmap(g.p, g.cap);
    g = ShmSeg{};
  }
  void *shared_host(int slot, size_t bytes, hipStream_t st) override {
    ShmSeg &g = shm[slot];
    if (g.p && g.cap >= bytes) return g.p;
    if (!shm_tag) shm_tag = gather_u64(rank == 0 ? ((uint64_t)getpid() << 20) ^ (uint64_t)(uintptr_t)this : 0, st)[0] | 1;
    const size_t cap = std::max(bytes, g.cap + g.cap / 4);
    unmap(g);
    char name[96];
    snprintf(name, sizeof name, "/rs_simplify_%llx_%d_%llu", (unsigned long long)shm_tag, slot, (unsigned long long)++shm_gen);
    int ok = 1;
    if (rank == 0) {
      const int fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
      ok = fd >= 0 && ftruncate(fd, (off_t)cap) == 0;
      if (fd >= 0) close(fd);
    }
    ok = (int)max_u64(ok ? 0 : 1, st) == 0;  // rank 0 created it (also the barrier before the opens)
    void *p = MAP_FAILED;
    if (ok) {
      const int fd = shm_open(name, O_RDWR, 0600);
      if (fd >= 0) {
        p = mmap(nullptr, cap, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        close(fd);
      }
    }
    const bool mine = p != MAP_FAILED && hipHostRegister(p, cap, hipHostRegisterDefault) == hipSuccess;
    ok = (int)max_u64(mine ? 0 : 1, st) == 0;  // every rank mapped it: the name can go
    if (rank == 0) shm_unlink(name);
    if (p != MAP_FAILED) {
      g.p = p;
      g.cap = cap;
      g.registered = mine;
    }
    if (!ok) {
      unmap(g);
      return nullptr;
    }
    return g.p;
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
  std::vector<std::vector<uint8_t>> slot;
  struct Host {
    void *p = nullptr;
    size_t cap = 0;
  } host[4];  // the group's shared host regions (one process: one pinned allocation each)
  std::vector<const void *> dsend;  // allgatherv: every rank's send buffer (device memory)
  explicit LocalGroup(int w) : world(w), slot(w), dsend(w, nullptr) {}
  ~LocalGroup() {
    for (Host &h : host)
      if (h.p) (void)hipHostFree(h.p);
  }
  // Barriers are counted per call (calls are numbered by each rank's begin_call; every rank makes the
  // same sequence), so ranks one call apart never share a barrier's count.  A failed call releases
  // its waiters with an error; its state is dropped once every rank has ended it, and the ranks'
  // next calls run normally (a persistent group survives an input every rank rejects).
  struct Bar {
    int arrived = 0;
    uint64_t gen = 0;
  };
  std::map<uint64_t, Bar> bars;
  std::set<uint64_t> failed_calls;
  std::map<uint64_t, int> ended;
  void barrier(uint64_t call) {
    std::unique_lock<std::mutex> lk(m);
    if (failed_calls.count(call)) throw RsError(RS_E_RCCL, "another rank of the in-process group failed");
    Bar &b = bars[call];
    const uint64_t g = b.gen;
    if (++b.arrived == world) {
      b.arrived = 0;
      ++b.gen;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return b.gen != g || failed_calls.count(call) != 0; });
      if (b.gen == g) throw RsError(RS_E_RCCL, "another rank of the in-process group failed");
    }
  }
  void fail(uint64_t call) {
    std::lock_guard<std::mutex> lk(m);
    failed_calls.insert(call);
    cv.notify_all();
  }
  void end(uint64_t call) {
    std::lock_guard<std::mutex> lk(m);
    if (++ended[call] == world) {  // nobody is inside this call any more
      ended.erase(call);
      bars.erase(call);
      failed_calls.erase(call);
    }
  }
};

struct LocalComm : Comm {
  LocalGroup *g;
  uint64_t call = 0;     // this rank's current call number (begin_call)
  bool in_call = false;
  LocalComm(LocalGroup *grp, int r) : g(grp) {
    rank = r;
    world = grp->world;
  }
  void post(const void *dev, uint64_t bytes, hipStream_t st) {
    g->slot[rank].resize(bytes);
    if (bytes) HC(hipMemcpyAsync(g->slot[rank].data(), dev, bytes, hipMemcpyDeviceToHost, st));
    HC(hipStreamSynchronize(st));
  }
  // device to device: the ranks of an in-process group are engines of this process (the one-GPU test
  // vehicle), so each reads the others' send buffers where they lie -- through host memory the 20 M-row
  // circuit's blocks (~3 GB, gathered by every rank) took minutes
  void allgatherv(const void *send, void *recv, const std::vector<uint64_t> &counts, hipStream_t st) override {
    HC(hipStreamSynchronize(st));  // the send buffer is complete
    g->dsend[rank] = send;
    g->barrier(call);
    uint64_t off = 0;
    for (int q = 0; q < world; ++q) {
      const bool in_place = g->dsend[q] == (const void *)((uint8_t *)recv + off);  // this rank's own share, already there
      if (counts[q] && !in_place) HC(hipMemcpyAsync((uint8_t *)recv + off, g->dsend[q], counts[q], hipMemcpyDeviceToDevice, st));
      off += counts[q];
    }
    HC(hipStreamSynchronize(st));
    g->barrier(call);  // the send buffers may be reused only after every rank has read them
  }
  void allreduce_sum(void *buf, uint64_t n, int elem_bytes, hipStream_t st) override {
    if (!n) return;
    post(buf, n * elem_bytes, st);
    g->barrier(call);
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
    g->barrier(call);
  }
  std::vector<uint64_t> gather_u64(uint64_t v, hipStream_t) override {
    g->slot[rank].resize(8);
    memcpy(g->slot[rank].data(), &v, 8);
    g->barrier(call);
    std::vector<uint64_t> r(world);
    for (int q = 0; q < world; ++q) memcpy(&r[q], g->slot[q].data(), 8);
    g->barrier(call);
    return r;
  }
  uint64_t max_u64(uint64_t v, hipStream_t st) override {
    uint64_t m = 0;
    for (uint64_t x : gather_u64(v, st)) m = std::max(m, x);
    return m;
  }
  void barrier(hipStream_t st) override {
    HC(hipStreamSynchronize(st));
    g->barrier(call);
  }
  void fail() override { g->fail(call); }
  void begin_call() override {
    ++call;
    in_call = true;
  }
  void end_call() override {
    if (!in_call) return;
    in_call = false;
    g->end(call);
  }
  void *shared_host(int slot, size_t bytes, hipStream_t st) override {
    HC(hipStreamSynchronize(st));
    g->barrier(call);  // nobody still uses the old region
    LocalGroup::Host &h = g->host[slot];
    if (rank == 0 && h.cap < bytes) {
      const size_t cap = std::max(bytes, h.cap + h.cap / 4);
      if (h.p) (void)hipHostFree(h.p);
      h.p = nullptr;
      h.cap = 0;
      if (hipHostMalloc(&h.p, cap, hipHostMallocDefault) == hipSuccess) h.cap = cap;
      else h.p = nullptr;
    }
    g->barrier(call);
    return h.cap >= bytes ? h.p : nullptr;
  }
};

}  // namespace rs
