// comm.hpp -- the exchange step of the sharded elimination.
//
// One circuit, one rank per GPU.  Every rank holds the whole input and runs the cheap global
// phases itself (eq / const-eq renaming, build_clusters); the clusters are dealt to the ranks and
// each rank eliminates only its own (A7-A12).  The eliminated-signal map -- per slot: `from`, the
// RHS offset/length, the leftovers, per cluster: #subs/#leftovers, and the pool entries those
// offsets point at -- is then exchanged so every rank continues with the full map.
//
// Three transports behind one interface:
//   RcclComm  -- production: RCCL over xGMI, one communicator per engine, collectives on the
//                engine's stream (allgatherv = grouped ncclBroadcast, one per root).
//   LocalComm -- several engines in one process (threads; typically on ONE device): host-staged
//                collectives behind a barrier.  It exists so the sharded path is testable on a
//                one-GPU box, and it is what rs_simplify_multi uses when a device is listed twice.
//   HostComm  -- one process per rank on one host (a test vehicle: RCCL refuses two ranks on one
//                device): collectives staged through POSIX shared memory, a spin barrier in a shared
//                control block; the shared result region is made by the same code as RcclComm's
//                (shm_shared_host), so the multi-process result path runs on a one-GPU box.
#pragma once

#include <fcntl.h>
#include <rccl/rccl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
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
static inline void shm_unmap(ShmSeg &g) {
  if (!g.p) return;
  if (g.registered) (void)hipHostUnregister(g.p);
  munmap(g.p, g.cap);
  g = ShmSeg{};
}
// The shared host region of a process-per-rank group (RcclComm, HostComm): collective; segment g grows
// only (every rank passes the same size).  Rank 0 creates a POSIX shm object (name: a tag rank 0 chose,
// sent with the first gather, the slot and a generation), every rank maps it and registers it with
// HIP, and once every rank has it the name is unlinked.  nullptr (every rank alike) if any rank failed.
static inline void *shm_shared_host(Comm &cm, ShmSeg &g, uint64_t &tag, uint64_t &gen, int slot, size_t bytes, hipStream_t st) {
  if (g.p && g.cap >= bytes) return g.p;
  if (!tag) tag = cm.gather_u64(cm.rank == 0 ? ((uint64_t)getpid() << 20) ^ (uint64_t)(uintptr_t)&cm : 0, st)[0] | 1;
  const size_t cap = std::max(bytes, g.cap + g.cap / 4);
  shm_unmap(g);
  char name[96];
  snprintf(name, sizeof name, "/rs_simplify_%llx_%d_%llu", (unsigned long long)tag, slot, (unsigned long long)++gen);
  int ok = 1;
  if (cm.rank == 0) {
    const int fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
    ok = fd >= 0 && ftruncate(fd, (off_t)cap) == 0;
    if (fd >= 0) close(fd);
  }
  ok = (int)cm.max_u64(ok ? 0 : 1, st) == 0;  // rank 0 created it (also the barrier before the opens)
  void *p = MAP_FAILED;
  if (ok) {
    const int fd = shm_open(name, O_RDWR, 0600);
    if (fd >= 0) {
      p = mmap(nullptr, cap, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
      close(fd);
    }
  }
  const bool mine = p != MAP_FAILED && hipHostRegister(p, cap, hipHostRegisterDefault) == hipSuccess;
  ok = (int)cm.max_u64(mine ? 0 : 1, st) == 0;  // every rank mapped it: the name can go
  if (cm.rank == 0) shm_unlink(name);
  if (p != MAP_FAILED) {
    g.p = p;
    g.cap = cap;
    g.registered = mine;
  }
  if (!ok) {
    shm_unmap(g);
    return nullptr;
  }
  return g.p;
}

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
    for (ShmSeg &g : shm) shm_unmap(g);
    if (d_scalar) (void)hipFree(d_scalar);
    if (c) (void)ncclCommDestroy(c);
  }
  void *shared_host(int slot, size_t bytes, hipStream_t st) override {
    return shm_shared_host(*this, shm[slot], shm_tag, shm_gen, slot, bytes, st);
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

// ------------------------------------------------------------------ processes of one host (tests)
// The control block every rank maps: a generation-counting spin barrier, one u64 per rank for the
// scalar collectives, and a failure flag that releases the waiting ranks (RS_E_RCCL).
struct HostCtl {
  std::atomic<uint32_t> joined;
  std::atomic<uint32_t> failed;
  std::atomic<uint64_t> arrived;
  std::atomic<uint64_t> gen;
  uint64_t slot[256];
};
struct HostComm : Comm {
  HostCtl *ctl = nullptr;
  ShmSeg shm[4], stage;  // the result regions (slots) and the collectives' staging region
  uint64_t shm_tag = 0, shm_gen = 0;
  // every rank passes the same tag; rank 0 creates the control block, the others open it (up to 60 s)
  HostComm(int w, int r, const char *tag) {
    rank = r;
    world = w;
    char name[160];
    snprintf(name, sizeof name, "/rs_hostcomm_%.120s", tag);
    int fd = -1;
    if (r == 0) {
      shm_unlink(name);  // a crashed earlier run's object
      fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
      if (fd >= 0 && ftruncate(fd, sizeof(HostCtl)) != 0) { close(fd); fd = -1; }
    } else {
      for (int i = 0; i < 60000 && fd < 0; ++i) {
        fd = shm_open(name, O_RDWR, 0600);
        if (fd < 0) usleep(1000);
        else {
          struct stat sb;
          if (fstat(fd, &sb) != 0 || (size_t)sb.st_size < sizeof(HostCtl)) { close(fd); fd = -1; usleep(1000); }
        }
      }
    }
    if (fd < 0) throw RsError(RS_E_RCCL, std::string("host transport: cannot open ") + name);
    void *p = mmap(nullptr, sizeof(HostCtl), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) throw RsError(RS_E_RCCL, "host transport: mmap");
    ctl = (HostCtl *)p;  // a fresh object is zero-filled: counters at 0
    ctl->joined.fetch_add(1);
    for (int i = 0; i < 600000 && ctl->joined.load() < (uint32_t)w; ++i) usleep(100);
    if (ctl->joined.load() < (uint32_t)w) throw RsError(RS_E_RCCL, "host transport: the other ranks did not join");
    wait_all();
    if (r == 0) shm_unlink(name);  // every rank has it mapped
  }
  ~HostComm() override {
    for (ShmSeg &g : shm) shm_unmap(g);
    shm_unmap(stage);
    if (ctl) munmap(ctl, sizeof(HostCtl));
  }
  // the spin barrier (generation counting); a rank's failure releases the others with an error
  void wait_all() {
    const uint64_t g = ctl->gen.load();
    if (ctl->arrived.fetch_add(1) + 1 == (uint64_t)world) {
      ctl->arrived.store(0);
      ctl->gen.fetch_add(1);
      return;
    }
    for (uint64_t i = 0; ctl->gen.load() == g; ++i) {
      if (ctl->failed.load()) throw RsError(RS_E_RCCL, "another rank of the host group failed");
      if (i > 64) usleep(20);
      if (i > 64 + 10000000ull) throw RsError(RS_E_RCCL, "host transport: barrier timed out");
    }
  }
  void fail() override { if (ctl) ctl->failed.store(1); }
  std::vector<uint64_t> gather_u64(uint64_t v, hipStream_t) override {
    ctl->slot[rank] = v;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    wait_all();
    std::vector<uint64_t> r(world);
    for (int q = 0; q < world; ++q) r[q] = ((volatile uint64_t *)ctl->slot)[q];
    wait_all();  // the slots may be rewritten only after every rank has read them
    return r;
  }
  uint64_t max_u64(uint64_t v, hipStream_t st) override {
    uint64_t m = 0;
    for (uint64_t x : gather_u64(v, st)) m = std::max(m, x);
    return m;
  }
  void barrier(hipStream_t st) override {
    HC(hipStreamSynchronize(st));
    wait_all();
  }
  void *shared_host(int slot, size_t bytes, hipStream_t st) override {
    return shm_shared_host(*this, shm[slot], shm_tag, shm_gen, slot, bytes, st);
  }
  // every rank's block through the staging region: each copies its own in, every rank copies all out
  void allgatherv(const void *send, void *recv, const std::vector<uint64_t> &counts, hipStream_t st) override {
    uint64_t tot = 0, mine = 0;
    for (int q = 0; q < world; ++q) {
      if (q == rank) mine = tot;
      tot += counts[q];
    }
    if (!tot) return;
    uint8_t *h = (uint8_t *)shm_shared_host(*this, stage, shm_tag, shm_gen, 4, tot, st);
    if (!h) throw RsError(RS_E_RCCL, "host transport: no staging region");
    if (counts[rank]) HC(hipMemcpyAsync(h + mine, send, counts[rank], hipMemcpyDeviceToHost, st));
    HC(hipStreamSynchronize(st));
    wait_all();
    uint64_t off = 0;
    for (int q = 0; q < world; ++q) {
      const bool in_place = q == rank && send == (const void *)((uint8_t *)recv + off);
      if (counts[q] && !in_place) HC(hipMemcpyAsync((uint8_t *)recv + off, h + off, counts[q], hipMemcpyHostToDevice, st));
      off += counts[q];
    }
    HC(hipStreamSynchronize(st));
    wait_all();  // the region may be reused only after every rank has read it
  }
  void allreduce_sum(void *buf, uint64_t n, int elem_bytes, hipStream_t st) override {
    if (!n) return;
    const uint64_t nb = n * (uint64_t)elem_bytes;
    uint8_t *h = (uint8_t *)shm_shared_host(*this, stage, shm_tag, shm_gen, 4, nb * (uint64_t)world, st);
    if (!h) throw RsError(RS_E_RCCL, "host transport: no staging region");
    HC(hipMemcpyAsync(h + nb * rank, buf, nb, hipMemcpyDeviceToHost, st));
    HC(hipStreamSynchronize(st));
    wait_all();
    std::vector<uint8_t> acc(h, h + nb);
    for (int q = 1; q < world; ++q) {
      const uint8_t *b = h + nb * q;
      if (elem_bytes == 8)
        for (uint64_t i = 0; i < n; ++i) ((uint64_t *)acc.data())[i] += ((const uint64_t *)b)[i];
      else
        for (uint64_t i = 0; i < n; ++i) ((uint32_t *)acc.data())[i] += ((const uint32_t *)b)[i];
    }
    HC(hipMemcpyAsync(buf, acc.data(), nb, hipMemcpyHostToDevice, st));
    HC(hipStreamSynchronize(st));
    wait_all();
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
