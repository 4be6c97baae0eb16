// engine.hip -- librs_simplify: the MI355X back end of circom's --O1/--O2 simplification.
//
// Host orchestration of constraint_list/src/constraint_simplification.rs:442-730 around the HIP
// kernels of kernels.hpp.  Every step says which part of simplification() it restates.  All
// field arithmetic and every constraint row stay on the GPU; the host keeps the ordered
// bookkeeping the reference keeps in Rust collections (the non-linear signal map of rounds >= 2).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <deque>
#include <mutex>
#include <map>
#include <memory>
#include <stdexcept>
#include <thread>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <functional>
#include <vector>

#include <cstring>
#include <fcntl.h>
#include <pthread.h>
#include <sched.h>
#include <unistd.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "host_common.hpp"
#include "kernels.hpp"
#include "frames_wave.hpp"
#include "spec_loop.hpp"
#include "giant_loop.hpp"
#include "cluster.hpp"
#include "writer.hpp"
#include "maplists.hpp"

namespace rs {


struct RsError : std::runtime_error {
  int code;
  RsError(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};
#define HC(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess)                                                                      \
      throw RsError(e_ == hipErrorOutOfMemory ? RS_E_OOM_DEVICE : RS_E_HIP,                   \
                    std::string(#x) + ": " + hipGetErrorString(e_));                          \
  } while (0)

static bool g_prof_env = getenv("RS_PROF") != nullptr;
static inline double now_ms();
// RS_PROF: host timeline of the round loop (synchronising the stream at each mark)
struct Marks {
  std::vector<std::pair<const char *, double>> m;
  hipStream_t st;
  void mark(const char *what);
  void dump();
};
static inline double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void Marks::mark(const char *what) {
  if (!g_prof_env) return;
  (void)hipStreamSynchronize(st);
  m.push_back({what, now_ms()});
}
void Marks::dump() {
  if (!g_prof_env || m.empty()) return;
  fprintf(stderr, "[rs-prof]");
  for (size_t i = 1; i < m.size(); ++i) fprintf(stderr, " %s %.2f", m[i].first, m[i].second - m[i - 1].second);
  fprintf(stderr, "\n");
}

// ------------------------------------------------------------------ device buffer arena
struct Arena {
  struct B {
    void *p = nullptr;
    size_t cap = 0;
  };
  // named, grow-only device buffers (a few hundred names, each looked up a few times per run):
  // one hash probe per lookup
  std::unordered_map<std::string, B> bufs{512};
  uint64_t gen = 0;  // bumped whenever a buffer moves (raw pointers taken before are then stale)
  // hipFree waits for the whole device: while `defer` is set (the sharded exchange, which runs beside
  // the head's elimination) a moved buffer's old block is kept until flush() instead
  bool defer = false;
  std::vector<void *> graveyard;
  void release(void *p) {
    if (!p) return;
    if (defer) graveyard.push_back(p);
    else HC(hipFree(p));
  }
  void flush() {
    for (void *p : graveyard) (void)hipFree(p);
    graveyard.clear();
  }
  template <class T>
  T *get(const std::string &name, size_t n) {
    size_t bytes = std::max<size_t>(n, 1) * sizeof(T);
    B &b = bufs[name];
    if (b.cap < bytes) {
      ++gen;
      release(b.p);
      size_t cap = std::max(bytes, b.cap + b.cap / 4);
      HC(hipMalloc(&b.p, cap));
      b.cap = cap;
    }
    return (T *)b.p;
  }
  // grows `name` to n elements keeping its first `keep`: the producer stream `ps` is waited for,
  // the kept part copied on `st`
  template <class T>
  void grow_keep(const std::string &name, size_t n, size_t keep, hipStream_t ps, hipStream_t st) {
    const size_t bytes = std::max<size_t>(n, 1) * sizeof(T);
    B &b = bufs[name];
    if (b.cap >= bytes) return;
    const size_t cap = std::max(bytes, b.cap + b.cap / 4);
    void *p = nullptr;
    ++gen;
    HC(hipMalloc(&p, cap));
    if (b.p) {
      HC(hipStreamSynchronize(ps));
      if (keep) HC(hipMemcpyAsync(p, b.p, keep * sizeof(T), hipMemcpyDeviceToDevice, st));
      HC(hipStreamSynchronize(st));
      release(b.p);
    }
    b.p = p;
    b.cap = cap;
  }
  size_t cap_bytes(const std::string &name) {
    auto it = bufs.find(name);
    return it == bufs.end() ? 0 : it->second.cap;
  }
  ~Arena() {
    flush();
    for (auto &kv : bufs)
      if (kv.second.p) (void)hipFree(kv.second.p);
  }
};

// grid of k_frames_wave: one 64-row chunk per wave, at most 16384 workgroups (grid-stride beyond)
constexpr uint64_t kFwBlocks = 16384;

// grid-stride kernels that end in per-wave atomics: a capped grid keeps the atomics few
template <class K, class... Args>
static void launch_capped(hipStream_t st, K kernel, uint64_t n, uint64_t max_blocks, Args... args) {
  uint64_t blocks = std::min<uint64_t>(std::max<uint64_t>((n + 255) / 256, 1), max_blocks);
  hipLaunchKernelGGL(kernel, dim3((unsigned)blocks), dim3(256), 0, st, args...);
  HC(hipGetLastError());
}
template <class K, class... Args>
static void launch(hipStream_t st, K kernel, uint64_t n, Args... args) {
  uint64_t blocks = (n + 255) / 256;
  if (blocks == 0) blocks = 1;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(kernel, dim3((unsigned)blocks), dim3(256), 0, st, args...);
  HC(hipGetLastError());
}

// A kernel group timed by HIP event pairs around each of its launches, on whichever stream they run
// (rs_stats: the input checks, the ragged conversion, the result gathers); `bytes` its algorithmic
// bytes (what the launches must read and write at least), both summed until collect()
struct KGroup {
  std::vector<hipEvent_t> ev;
  size_t n = 0;
  uint64_t bytes = 0;
  void mark(hipStream_t s) {
    if (n == ev.size()) {
      hipEvent_t e;
      HC(hipEventCreate(&e));
      ev.push_back(e);
    }
    HC(hipEventRecord(ev[n++], s));
  }
  template <class F>
  void run(hipStream_t s, uint64_t b, F &&f) {
    mark(s);
    f();
    mark(s);
    bytes += b;
  }
  // ms of the pairs so far (waits for them), launches (0 or 1: one group run per call), bytes; reset
  void collect(double &ms, uint64_t &by, uint64_t &launches) {
    double t = 0;
    for (size_t i = 0; i + 1 < n; i += 2) {
      float m = 0;
      HC(hipEventSynchronize(ev[i + 1]));
      HC(hipEventElapsedTime(&m, ev[i], ev[i + 1]));
      t += m;
    }
    ms += t;
    by += bytes;
    launches += n ? 1 : 0;
    n = 0;
    bytes = 0;
  }
  void destroy() {
    for (hipEvent_t e : ev) (void)hipEventDestroy(e);
    ev.clear();
    n = 0;
  }
};

}  // namespace rs
#include "comm.hpp"
namespace rs {



}  // namespace rs

using namespace rs;

struct rs_engine {
  uint64_t pool_want = 0;  // substitution pool size (entries) that fitted last time
  int device = 0;
  uint32_t n_cu = 256;  // compute units (resident grids)
  hipStream_t st = nullptr;
  hipStream_t srd = nullptr;  // host reads (rd): non-blocking, from the pooled queues
  hipStream_t st2 = nullptr;  // the largest clusters' elimination chain runs here, beside the rest
  hipEvent_t evx[11] = {};    // [0] join-in, [1..4] head chain, [5] after the lane kernel, [6..7] the
                              // largest replays' fork / join, [8..9] the overlapped frames pass
  Arena A;
  bool loaded = false;
  bool have_result = false;
  int fault_at = 0;  // rs_engine_inject_fault: 1 = throw at the start of the first elimination round
  FieldP F;
  uint64_t prime[4];
  uint32_t prime_id = 0;
  uint64_t S = 0, n_pub_out = 0, n_pub_in = 0, n_priv_in = 0;
  std::vector<uint32_t> forbidden;
  // loaded input (canonical, rows sorted)
  struct Blk {
    uint64_t *ptr = nullptr;
    uint32_t *key = nullptr;
    Fe *val = nullptr;
    uint64_t n = 0, nnz = 0;
  } ce, eq, lin, na, nb, nc;
  // result
  uint64_t out_n_dev = 0;  // constraints gathered on device
  uint64_t out_nnz[3] = {0, 0, 0};
  uint64_t n_wires = 0, npiw = 0;
  rs_stats stats{};
  hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr, ev3 = nullptr, ev4 = nullptr, ev5 = nullptr, ev6 = nullptr, ev7 = nullptr;
  // sharded elimination: this engine is rank `comm->rank` of `comm->world`
  std::unique_ptr<rs::Comm> comm;
  // substitution log of the last run (rs_flags.emit_substitution_log), canonical values
  bool log_on = false;
  std::vector<uint32_t> log_from, log_key;
  std::vector<uint64_t> log_ptr, log_val;
  uint32_t *heap_k = nullptr;  // storage-row heap (grows, reused across runs)
  Fe *heap_v = nullptr;
  uint64_t heap_cap = 0;
  // pipelined load: input groups 0 = cons_eq + eq, 1 = linear row pointers + keys, 2 = linear
  // values, 3 = non-linear land on the copy stream, each validated there; the run waits for a group
  // where it first needs it.  rs_engine_simplify stages the linear keys before their values
  // (`staged`): build_clusters can start on the keys while the values are still on the way, and the
  // eq block's values stay on the host (`hin`, valid for the call) -- the device never needs them.
  hipStream_t stc = nullptr;
  hipEvent_t ev_grp[4] = {};
  bool pending[4] = {false, false, false, false};
  int *h_vflag = nullptr;  // pinned: per-group verdicts [2g] row pointers, [2g + 1] rows; [8] linear keys unsorted
  bool staged = false;
  const rs_input *hin = nullptr;
  unsigned long long *h_lvl = nullptr;  // pinned: frontier counts of the head's [0..3] / the tail's [4..7] composition levels
  hipEvent_t ev_lvl[4] = {}, ev_lvlt[4] = {};  // frontier-count events of the head's / the tail's level loops
  double h2d_wait_ms = 0;
  // pinned result buffers of rs_engine_simplify (grow only) and the view handed out
  struct Pin {
    void *p = nullptr;
    size_t cap = 0;
  };
  Pin pin[40];  // a/b/c: ptr, col, val; label_to_wire; spare; rs_engine_write_r1cs's two staging buffers;
                // a/b/c row ends (streamed result); [16..17] the host replay's staging; [18..19] the
                // clustering's read-backs; [20..38]
                // rs_engine_flatten_dag's result (19 arrays)
  rs_input flat_view{};  // rs_engine_flatten_dag's result (views pin[20..38])
  rs_output view{};
  // streamed result (output.hpp; rs_engine_simplify): the storage rows final after round 1 go to
  // pin[3..8] on the copy stream during the later rounds (ev_snap: their D2H is done)
  bool stream_out = false;  // this run streams (set by rs_engine_simplify around engine_run)
  bool snap_on = false;     // the early region was taken in this run
  uint64_t snap_e[3] = {0, 0, 0};  // early-region entries per part
  uint64_t out_ext[3] = {0, 0, 0};  // streamed layout: early + late entries per part
  // Sharded host -> host result: every rank holds the whole result on its device and
  // copies only ITS share -- the storage rows of non-linear rows [nl_lo, nl_hi), the last rank also the
  // linear tail -- into host memory all ranks share (Comm::shared_host), so the D2H leg is split over
  // the ranks' PCIe links.  Entries of part q: rank r's [early | late] at r * sh_cap[q] (capacities
  // agreed over the ranks; gaps allowed by ABI 7); rows: the shared ptr / end arrays at global rows.
  uint64_t nl_lo = 0, nl_hi = UINT64_MAX;
  uint64_t sh_cap[3] = {0, 0, 0};
  void *sh_ent = nullptr;       // shared slot 0: col of a, b, c then val of a, b, c
  bool sh_full = false;         // the region was regrown at the end: the whole [early | late] is copied
  uint64_t sh_klo = 0, sh_khi = 0;  // this rank's run of the keep list (global output rows)
  uint64_t lc_snap_n = 0, lc_snap_base = 0;  // lconst rows in the first early region, where their C part starts
  hipEvent_t ev_snap = nullptr, ev_snap0 = nullptr;  // early gather done / its inputs ready
  uint64_t snap_cap[3] = {0, 0, 0};   // capacity (entries) of the device and host early regions this run
  uint64_t snap_hint[3] = {0, 0, 0};  // the largest early region (both snapshots) of the runs so far
  void *snap_host[6] = {};            // the host early regions: col / val of a, b, c
  // The early region's D2H runs on its own host thread, in chunks, one in flight at a time: the
  // copy engine serves transfers in order, so one large transfer would hold every small D2H the run
  // still issues (scan totals, flags, the head's frontier counts) behind it for ~15 ms.
  struct SnapJob {
    void *dst;
    const void *src;
    size_t bytes;
    hipEvent_t ready;  // its gather is done
  };
  hipEvent_t ev_snapq[6] = {};  // the parts' gathers of the first / second snapshot
  hipEvent_t ev_snaph[3] = {};  // the parts' gathers of the first pass's second half
  hipEvent_t ev_fh[2] = {};     // the first pass in halves: first half done / second half starts
  hipEvent_t ev_nlc = nullptr;  // the non-linear blocks' ragged conversion (copy stream) done
  std::mutex snap_m;
  std::condition_variable snap_cv;
  std::deque<SnapJob> snap_q;  // jobs the D2H thread has not started; closed: no more will come
  bool snap_closed = true;
  std::thread snap_thread;
  cpu_set_t near_cpus;  // the GPU's NUMA-local CPUs the creator's mask allowed (near_gpu_cpus)
  int near_n = 0;
  hipStream_t stx = nullptr;  // the early region's D2H stream
  hipStream_t str = nullptr;  // the host replay's copies (small; never behind the bulk copies)
  hipStream_t ste = nullptr;  // the small clusters' elimination (k_eliminate), beside the tail's chain
  hipStream_t stg = nullptr;  // the giant clusters' component loops (giant_loop.hpp), beside the head's
  hipEvent_t evg[2] = {};     // giant path: fork after the head's preparation / join before its inversion
  // per-kernel timing (rs_stats ABI 8): the tail groups' [prep, after prep + p3_fast, after the loop,
  // after the inversion, after the finish]; build_clusters' device span; the giant path's span
  hipEvent_t evt[2][5] = {};
  hipEvent_t evc[2] = {};
  hipEvent_t evgt[3] = {};
  hipEvent_t ev_sm[3] = {};   // its start / k_eliminate done / its work done (the tail's second group too)
  hipEvent_t ev_chunk[8] = {};
  // rs_stats groups timed launch by launch: [0] input checks (copy stream), [1] ragged conversion and
  // the linear rows' frames, [2] result gathers (snapshots, late rows, the compact CSR)
  KGroup kg[3];
  int snap_rc = 0;
  // the final row views, for the compact CSR built on demand (rs_engine_fetch / the .r1cs writer)
  // when the streamed run skipped it
  bool csr_ready = false;
  // Invariant: these point into arena buffers (sv.*, fin.*, lc.*) and the storage
  // heap as the run left them; nothing between the run and ensure_csr may move them (fin_gen = the
  // arena generation then; ensure_csr refuses a stale view instead of gathering from freed memory).
  DRows fin_parts[3] = {}, fin_xq[2][3] = {};  // storage rows; extras: leftover linear rows, lconst
  uint64_t out_njump[3] = {0, 0, 0};  // ABI 8: rows of the streamed layout that jump, per part
  const uint32_t *fin_keep_ids = nullptr, *fin_x_ids[2] = {nullptr, nullptr};
  uint64_t fin_keep = 0, fin_xn[2] = {0, 0}, fin_gen = 0;
};

namespace rs {

// H2D of one CSR block on the copy stream.  The row pointers are not trusted: the block's
// validation (k_check_ptr) checks ptr[0] = 0, monotonicity and ptr[n] = nnz on the device before
// anything reads a row.
// what of a block to send: everything, the row pointers + keys, or the values alone
enum UpPart { kUpAll = 0, kUpKeys = 1, kUpVals = 2 };

// A sharded engine uploads only its share of every block over its own PCIe link --
// rows [lo[r], lo[r + 1]) and their entries [ptr[lo[r]], ptr[lo[r + 1]]) -- and the ranks complete
// each other's blocks over xGMI: the shares are contiguous in rank order, so one allgatherv per
// array puts every array together in place.  Row bounds balance the entries.  The host reads the
// (still unvalidated) row pointers only at the W + 1 bounds, and every rank computes the same bounds
// from the same input, so a malformed input is rejected by all ranks before any collective.
struct RowSplit {
  std::vector<uint64_t> lo, e;  // W + 1 row bounds, their entry offsets
};
static RowSplit split_rows(const rs_lc &src, int W, const char *name) {
  RowSplit sp;
  const uint64_t n = src.n_rows, nnz = n ? src.nnz : 0;
  sp.lo.assign(W + 1, 0);
  sp.e.assign(W + 1, 0);
  sp.lo[W] = n;
  sp.e[W] = nnz;
  if (n && (src.ptr[0] != 0 || src.ptr[n] != nnz))
    throw RsError(RS_E_INVALID, std::string(name) + " block: bad row pointers (ptr[0] != 0 or ptr[n_rows] != nnz)");
  for (int q = 1; q < W; ++q) {
    const uint64_t want = (unsigned __int128)nnz * q / W;
    uint64_t a = sp.lo[q - 1], b = n;  // first row whose pointer reaches `want`
    while (a < b) {
      const uint64_t m = a + (b - a) / 2;
      if (src.ptr[m] < want) a = m + 1; else b = m;
    }
    sp.lo[q] = a;
    sp.e[q] = src.ptr[a];
    if (sp.e[q] < sp.e[q - 1] || sp.e[q] > nnz)
      throw RsError(RS_E_INVALID, std::string(name) + " block: bad row pointers (decreasing)");
  }
  return sp;
}
static void upload_block(rs_engine *E, const rs_lc &src, rs_engine::Blk &dst, const char *name, int part = kUpAll) {
  if (src.n_rows && !src.ptr) throw RsError(RS_E_INVALID, std::string(name) + ": rows without a ptr array");
  if (src.nnz && (!src.col || !src.val)) throw RsError(RS_E_INVALID, std::string(name) + ": entries without col/val");
  if (src.n_rows > 0xfffffff0ull || src.nnz > (1ull << 40)) throw RsError(RS_E_INVALID, std::string(name) + ": block too large");
  dst.n = src.n_rows;
  dst.nnz = src.n_rows ? src.nnz : 0;
  std::string nm(name);
  dst.ptr = E->A.get<uint64_t>(nm + ".ptr", dst.n + 1);
  dst.key = E->A.get<uint32_t>(nm + ".key", dst.nnz);
  dst.val = E->A.get<Fe>(nm + ".val", dst.nnz);
  hipStream_t s = E->stc;
  Comm *CM = E->comm.get();
  const int W = CM ? CM->world : 1, r = CM ? CM->rank : 0;
  if (W == 1 || !dst.n) {
    if (part != kUpVals) {
      if (dst.n) HC(hipMemcpyAsync(dst.ptr, src.ptr, sizeof(uint64_t) * (dst.n + 1), hipMemcpyHostToDevice, s));
      else HC(hipMemsetAsync(dst.ptr, 0, sizeof(uint64_t), s));
      if (dst.nnz) HC(hipMemcpyAsync(dst.key, src.col, sizeof(uint32_t) * dst.nnz, hipMemcpyHostToDevice, s));
    }
    if (part != kUpKeys && dst.nnz) HC(hipMemcpyAsync(dst.val, src.val, 32 * dst.nnz, hipMemcpyHostToDevice, s));
    return;
  }
  // sharded: this rank's share, then the allgathervs (row pointers: the last share also carries ptr[n])
  const RowSplit sp = split_rows(src, W, name);
  const uint64_t r0 = sp.lo[r], r1 = sp.lo[r + 1] + (r == W - 1 ? 1 : 0), e0 = sp.e[r], e1 = sp.e[r + 1];
  std::vector<uint64_t> cp(W), ck(W), cv(W);
  for (int q = 0; q < W; ++q) {
    cp[q] = 8 * (sp.lo[q + 1] - sp.lo[q] + (q == W - 1 ? 1 : 0));
    ck[q] = 4 * (sp.e[q + 1] - sp.e[q]);
    cv[q] = 32 * (sp.e[q + 1] - sp.e[q]);
  }
  if (part != kUpVals) {
    if (r1 > r0) HC(hipMemcpyAsync(dst.ptr + r0, src.ptr + r0, 8 * (r1 - r0), hipMemcpyHostToDevice, s));
    if (e1 > e0) HC(hipMemcpyAsync(dst.key + e0, src.col + e0, 4 * (e1 - e0), hipMemcpyHostToDevice, s));
    CM->allgatherv(dst.ptr + r0, dst.ptr, cp, s);
    CM->allgatherv(dst.key + e0, dst.key, ck, s);
  }
  if (part != kUpKeys) {
    if (e1 > e0) HC(hipMemcpyAsync(dst.val + e0, src.val + 4 * e0, 32 * (e1 - e0), hipMemcpyHostToDevice, s));
    CM->allgatherv(dst.val + e0, dst.val, cv, s);
  }
}

// ---------------------------------------------------------------- pipelined load
static const char *kGroupName[4] = {"cons_eq/eq", "linear", "linear", "non-linear"};

// Validates the header fields of `in` and enqueues the H2D of every block on the copy stream in
// the order the run consumes them, each group followed by its device checks and the D2H of its
// verdict words into pinned memory:
//   0: cons_eq (k_check_ptr, k_sort_validate, which also sorts rows), eq (staged: row pointers and
//      keys only, k_check_keys -- eq_simplification reads no value; the rows it keeps as they are
//      take their values from the host input);
//   1: linear (staged: row pointers + keys, k_check_keys also flags unsorted rows; else all of it);
//   2: linear values (staged; k_sort_validate, which sorts rows the keys left unsorted);
//   3: nl_a, nl_b, nl_c.
static void load_enqueue(rs_engine *E, const rs_input *in, bool staged) {
  uint64_t p[4];
  if (!prime_of(in, p)) throw RsError(RS_E_INVALID, "unknown prime");
  if (in->max_signal == 0 || in->max_signal > 0x7fffffffull) throw RsError(RS_E_INVALID, "bad max_signal (label_to_wire is int32)");
  if (in->n_forbidden && !in->forbidden) throw RsError(RS_E_INVALID, "forbidden list missing");
  std::vector<uint32_t> forb(in->forbidden, in->forbidden + in->n_forbidden);
  bool has0 = false;
  for (uint32_t f : forb) {
    if (f >= in->max_signal) throw RsError(RS_E_INVALID, "forbidden signal out of range");
    has0 |= f == 0;
  }
  if (!has0) throw RsError(RS_E_INVALID, "signal 0 must be forbidden");
  if (in->nl_a.n_rows != in->nl_b.n_rows || in->nl_a.n_rows != in->nl_c.n_rows)
    throw RsError(RS_E_INVALID, "non-linear blocks differ in row count");
  HC(hipStreamSynchronize(E->stc));  // the previous call's copies are complete
  E->loaded = false;
  E->have_result = false;
  for (bool &pd : E->pending) pd = false;
  memcpy(E->prime, p, 32);
  E->prime_id = in->prime_id;
  E->F = make_field(p);
  E->S = in->max_signal;
  E->n_pub_out = in->n_pub_out;
  E->n_pub_in = in->n_pub_in;
  E->n_priv_in = in->n_priv_in;
  E->forbidden.swap(forb);
  E->h2d_wait_ms = 0;
  E->staged = staged;
  E->hin = staged ? in : nullptr;
  E->nl_lo = 0;
  E->nl_hi = UINT64_MAX;
  if (E->comm && E->comm->world > 1 && in->nl_a.n_rows) {
    // this rank's share of the non-linear rows for the result's D2H: entries of A + B + C balanced
    const int W = E->comm->world, r = E->comm->rank;
    const rs_lc *b3[3] = {&in->nl_a, &in->nl_b, &in->nl_c};
    const uint64_t n = in->nl_a.n_rows;
    for (const rs_lc *L : b3)
      if (!L->ptr) throw RsError(RS_E_INVALID, "non-linear block: rows without a ptr array");
    auto cum = [&](uint64_t row) { return b3[0]->ptr[row] + b3[1]->ptr[row] + b3[2]->ptr[row]; };
    const uint64_t tot = cum(n);
    auto bound = [&](int q) -> uint64_t {
      if (q <= 0) return 0;
      if (q >= W) return n;
      const uint64_t want = (unsigned __int128)tot * q / W;
      uint64_t a = 0, b = n;
      while (a < b) {
        const uint64_t m = a + (b - a) / 2;
        if (cum(m) < want) a = m + 1; else b = m;
      }
      return a;
    };
    E->nl_lo = bound(r);
    E->nl_hi = std::max(E->nl_lo, bound(r + 1));
  }
  int *vf = E->A.get<int>("vflag", 10);
  HC(hipMemsetAsync(vf, 0, 40, E->stc));
  hipStream_t s = E->stc;
  KGroup &kg = E->kg[0];
  kg.n = 0;
  kg.bytes = 0;
  // algorithmic bytes: the row pointers; + the keys (k_check_keys); + keys and values (k_sort_validate)
  auto check = [&](const rs_engine::Blk &B, int g) {
    kg.run(s, 8 * (B.n + 1), [&] { launch(s, k_check_ptr, B.n + 1, (const uint64_t *)B.ptr, B.n, B.nnz, vf + 2 * g); });
  };
  auto check_keys = [&](const rs_engine::Blk &B, int pw, int ew, int *uw) {
    if (B.n)
      kg.run(s, 8 * (B.n + 1) + 4 * B.nnz, [&] {
        launch(s, k_check_keys, B.n, (const uint64_t *)B.ptr, (const uint32_t *)B.key, B.n, E->S, (const int *)(vf + pw), vf + ew, uw);
      });
  };
  // k_sort_validate of block B: skipped when the row pointers' word `pw` is set, verdict into `ew`
  auto sort_validate = [&](const rs_engine::Blk &B, int pw, int ew) {
    if (B.n)
      kg.run(s, 8 * (B.n + 1) + 36 * B.nnz, [&] {
        launch(s, k_sort_validate, B.n, E->F, (const uint64_t *)B.ptr, B.key, B.val, B.n, E->S, (const int *)(vf + pw), vf + ew);
      });
  };
  auto verdict = [&](int g, int words) {
    HC(hipMemcpyAsync(E->h_vflag + 2 * g, vf + 2 * g, 4 * words, hipMemcpyDeviceToHost, s));
    HC(hipEventRecord(E->ev_grp[g], s));
    E->pending[g] = true;
  };
  // group 0
  upload_block(E, in->cons_eq, E->ce, "in.ce");
  upload_block(E, in->eq, E->eq, "in.eq", staged ? kUpKeys : kUpAll);
  check(E->ce, 0);
  check(E->eq, 0);
  sort_validate(E->ce, 0, 1);
  if (staged) {
    check_keys(E->eq, 0, 1, nullptr);
  } else {
    sort_validate(E->eq, 0, 1);
  }
  verdict(0, 2);
  // groups 1 and 2
  upload_block(E, in->linear, E->lin, "in.lin", staged ? kUpKeys : kUpAll);
  check(E->lin, 1);
  if (staged) {
    check_keys(E->lin, 2, 3, vf + 8);
    HC(hipMemcpyAsync(E->h_vflag + 8, vf + 8, 4, hipMemcpyDeviceToHost, s));
    verdict(1, 2);
    upload_block(E, in->linear, E->lin, "in.lin", kUpVals);
    sort_validate(E->lin, 2, 5);
    HC(hipMemcpyAsync(E->h_vflag + 4, vf + 2, 4, hipMemcpyDeviceToHost, s));  // the pointers' verdict
    HC(hipMemcpyAsync(E->h_vflag + 5, vf + 5, 4, hipMemcpyDeviceToHost, s));
    HC(hipEventRecord(E->ev_grp[2], s));
    E->pending[2] = true;
  } else {
    sort_validate(E->lin, 2, 3);
    E->h_vflag[8] = 0;
    verdict(1, 2);
  }
  // group 3
  const rs_lc *nl_src[3] = {&in->nl_a, &in->nl_b, &in->nl_c};
  rs_engine::Blk *nl_dst[3] = {&E->na, &E->nb, &E->nc};
  const char *nl_nm[3] = {"in.na", "in.nb", "in.nc"};
  for (int q = 0; q < 3; ++q) upload_block(E, *nl_src[q], *nl_dst[q], nl_nm[q]);
  for (int q = 0; q < 3; ++q) check(*nl_dst[q], 3);
  for (int q = 0; q < 3; ++q) sort_validate(*nl_dst[q], 6, 7);
  verdict(3, 2);
  E->loaded = true;
}

// Blocks until input group g has landed and passed its checks; the main stream is ordered after it.
static void load_wait(rs_engine *E, int g) {
  if (!E->pending[g]) return;
  const double t0 = now_ms();
  HC(hipEventSynchronize(E->ev_grp[g]));
  E->pending[g] = false;
  E->h2d_wait_ms += now_ms() - t0;
  if (E->h_vflag[2 * g]) {
    E->loaded = false;
    throw RsError(RS_E_INVALID, std::string(kGroupName[g]) + " block: bad row pointers (ptr[0] != 0, decreasing, or ptr[n_rows] != nnz)");
  }
  if (E->h_vflag[2 * g + 1]) {
    E->loaded = false;
    throw RsError(RS_E_INVALID, std::string(kGroupName[g]) +
                                    " block: invalid rows (duplicate key, zero or non-canonical value, signal >= max_signal)");
  }
  HC(hipStreamWaitEvent(E->st, E->ev_grp[g], 0));
}
static void load_wait_all(rs_engine *E) {
  for (int g = 0; g < 4; ++g) load_wait(E, g);
}
// Sharded: the main stream's collectives (the exchange) run after every input group's allgathervs
// on the copy stream have completed on this rank -- so no rank has collectives of both streams of
// one communicator in flight at once.  Device-side ordering only: the verdicts are read later.
static void load_order_collectives(rs_engine *E) {
  for (int g = 0; g < 4; ++g)
    if (E->pending[g]) HC(hipStreamWaitEvent(E->st, E->ev_grp[g], 0));
}
// After a failed call: the copy stream may still be reading the caller's buffers.
static void snap_join(rs_engine *E);
static void *pin_get(rs_engine *E, int slot, size_t bytes);
static void load_abort(rs_engine *E) {
  if (E->stc) (void)hipStreamSynchronize(E->stc);
  snap_join(E);
  for (bool &pd : E->pending) pd = false;
  if (E->comm) E->comm->fail();  // the other ranks leave their collectives with an error instead of waiting
}

// A synchronous device -> host read of data whose producers the caller has already synchronised, on the
// engine's own non-blocking read stream (the engine's dedicated-queue streams block with the null
// stream, which a plain hipMemcpy would use)
static void rd(rs_engine *E, void *dst, const void *src, size_t bytes) {
  if (!bytes) return;
  HC(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, E->srd));
  HC(hipStreamSynchronize(E->srd));
}
// H2D copy whose host buffer may be released right after the call: wait for it.
static void h2d(rs_engine *E, void *dst, const void *src, size_t bytes) {
  if (!bytes) return;
  HC(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, E->st));
  HC(hipStreamSynchronize(E->st));
}

// ---------------------------------------------------------------- scans
static void *pin_get(rs_engine *E, int slot, size_t bytes);
constexpr size_t kPinRb = 128;  // pinned slot 18: small read-backs (one size everywhere: never reallocated)
static uint64_t excl_scan_u64(rs_engine *E, const uint64_t *in, uint64_t *out, uint64_t n, const char *tag,
                              double *waited = nullptr) {
  if (n == 0) return 0;
  size_t tb = 0;
  HC(rocprim::exclusive_scan(nullptr, tb, in, out, (uint64_t)0, (size_t)n, rocprim::plus<uint64_t>(), E->st));
  void *tmp = E->A.get<uint8_t>(std::string("scan.tmp.") + tag, tb);
  HC(rocprim::exclusive_scan(tmp, tb, in, out, (uint64_t)0, (size_t)n, rocprim::plus<uint64_t>(), E->st));
  uint64_t *h = (uint64_t *)pin_get(E, 18, kPinRb) + 4;  // pinned read-back words [4..5] (no staged copy)
  HC(hipMemcpyAsync(h, in + n - 1, 8, hipMemcpyDeviceToHost, E->st));
  HC(hipMemcpyAsync(h + 1, out + n - 1, 8, hipMemcpyDeviceToHost, E->st));
  const double t0 = waited ? now_ms() : 0.0;
  HC(hipStreamSynchronize(E->st));
  if (waited) *waited += now_ms() - t0;
  return h[0] + h[1];
}

// one scan over three capacity columns at once (separate [a..][b..][c..] blocks keep neighbouring
// rows' outputs adjacent, which the fill kernels' writes rely on for coalescing)
struct U3 {
  uint64_t a, b, c;
};
struct U3Plus {
  __host__ __device__ U3 operator()(const U3 &x, const U3 &y) const { return U3{x.a + y.a, x.b + y.b, x.c + y.c}; }
};
// the total through pinned read-back words [8..13]; x (optional): two more device words read in the
// same round trip (an earlier device-only scan's last input and output), their sum into *x_sum
static U3 excl_scan_u3(rs_engine *E, const U3 *in, U3 *out, uint64_t n, const char *tag, const uint64_t *x_in = nullptr,
                       const uint64_t *x_out = nullptr, uint64_t *x_sum = nullptr) {
  if (n == 0 && !x_sum) return U3{0, 0, 0};
  uint64_t *h = (uint64_t *)pin_get(E, 18, kPinRb) + 8;
  if (n) {
    size_t tb = 0;
    const U3 zero{0, 0, 0};
    HC(rocprim::exclusive_scan(nullptr, tb, in, out, zero, (size_t)n, U3Plus(), E->st));
    void *tmp = E->A.get<uint8_t>(std::string("scan3.tmp.") + tag, tb);
    HC(rocprim::exclusive_scan(tmp, tb, in, out, zero, (size_t)n, U3Plus(), E->st));
    HC(hipMemcpyAsync(h, in + n - 1, sizeof(U3), hipMemcpyDeviceToHost, E->st));
    HC(hipMemcpyAsync(h + 3, out + n - 1, sizeof(U3), hipMemcpyDeviceToHost, E->st));
  }
  if (x_sum) {
    HC(hipMemcpyAsync(h + 6, x_in, 8, hipMemcpyDeviceToHost, E->st));
    HC(hipMemcpyAsync(h + 7, x_out, 8, hipMemcpyDeviceToHost, E->st));
  }
  HC(hipStreamSynchronize(E->st));
  if (x_sum) *x_sum = h[6] + h[7];
  return n ? U3{h[0] + h[3], h[1] + h[4], h[2] + h[5]} : U3{0, 0, 0};
}
#include "flatten.hpp"
#include "output.hpp"
__global__ void k_pack3(const uint64_t *a, const uint64_t *b, const uint64_t *c, uint64_t n, U3 *out) {
  for (uint64_t i = gtid(); i < n; i += gstride()) out[i] = U3{a[i], b[i], c[i]};
}
// entry i sets row ids[i] (ids == nullptr: row i); cap (optional): entries with no space
// (cap.a == 0) leave their row's offsets alone
__global__ void k_set_offsets_u3(const U3 *scan, uint64_t ba, uint64_t bb, uint64_t bc, uint64_t n, uint64_t *oa, uint64_t *ob,
                                 uint64_t *oc, const U3 *cap, const uint32_t *ids) {
  for (uint64_t i = gtid(); i < n; i += gstride()) {
    if (cap && cap[i].a == 0) continue;
    const uint64_t r = ids ? ids[i] : i;
    oa[r] = ba + scan[i].a;
    ob[r] = bb + scan[i].b;
    oc[r] = bc + scan[i].c;
  }
}

__global__ void k_mark_u8(const uint32_t *ids, uint64_t n, uint8_t *flag) {
  for (uint64_t i = gtid(); i < n; i += gstride()) flag[ids[i]] = 1;
}

// apply_substitution_to_map (:369-377) appends every key of sub.to to the signal map when
// map[from] is non-empty; only the key set survives the rounds (rebuild_witness), so it is kept as
// bits.  A round's `from` signals never occur in its (non-overlapping) right-hand sides.
__global__ void k_append_marks(const uint32_t *usig, const uint64_t *uoff, const uint32_t *ulen, uint64_t nU,
                               const uint32_t *pk, uint8_t *nlmap) {
  for (uint64_t i = gtid(); i < nU; i += gstride()) {
    if (!nlmap[usig[i]]) continue;
    for (uint32_t t = 0; t < ulen[i]; ++t) nlmap[pk[uoff[i] + t]] = 1;
  }
}

template <class K, class V>
static void sort_pairs(rs_engine *E, const K *kin, K *kout, const V *vin, V *vout, uint64_t n, int end_bit,
                       const char *tag, hipStream_t s = nullptr) {
  if (!n) return;
  if (!s) s = E->st;
  size_t tb = 0;
  HC(rocprim::radix_sort_pairs(nullptr, tb, kin, kout, vin, vout, (size_t)n, 0, end_bit, s));
  void *tmp = E->A.get<uint8_t>(std::string("sort.tmp.") + tag, tb);
  HC(rocprim::radix_sort_pairs(tmp, tb, kin, kout, vin, vout, (size_t)n, 0, end_bit, s));
}
// device-only exclusive scan of u64 on stream s (no read-back)
static void dev_scan_u64(rs_engine *E, const uint64_t *in, uint64_t *out, uint64_t n, hipStream_t s, const char *tag) {
  if (!n) return;
  size_t tb = 0;
  HC(rocprim::exclusive_scan(nullptr, tb, in, out, (uint64_t)0, (size_t)n, rocprim::plus<uint64_t>(), s));
  void *tmp = E->A.get<uint8_t>(std::string("scan.tmp.") + tag, tb);
  HC(rocprim::exclusive_scan(tmp, tb, in, out, (uint64_t)0, (size_t)n, rocprim::plus<uint64_t>(), s));
}
// device-only exclusive scan of u32 on stream s (no read-back; tmp sized on first use)
static void dev_scan_u32(rs_engine *E, const uint32_t *in, uint32_t *out, uint64_t n, hipStream_t s, const char *tag) {
  if (!n) return;
  size_t tb = 0;
  HC(rocprim::exclusive_scan(nullptr, tb, in, out, (uint32_t)0, (size_t)n, rocprim::plus<uint32_t>(), s));
  void *tmp = E->A.get<uint8_t>(std::string("dscan.tmp.") + tag, tb);
  HC(rocprim::exclusive_scan(tmp, tb, in, out, (uint32_t)0, (size_t)n, rocprim::plus<uint32_t>(), s));
}

template <class K>
static void sort_keys(rs_engine *E, const K *kin, K *kout, uint64_t n, int end_bit, const char *tag) {
  if (!n) return;
  size_t tb = 0;
  HC(rocprim::radix_sort_keys(nullptr, tb, kin, kout, (size_t)n, 0, end_bit, E->st));
  void *tmp = E->A.get<uint8_t>(std::string("sortk.tmp.") + tag, tb);
  HC(rocprim::radix_sort_keys(tmp, tb, kin, kout, (size_t)n, 0, end_bit, E->st));
}

__global__ void k_u32_to_u64(const uint32_t *in, uint64_t *out, uint64_t n) {
  for (uint64_t i = gtid(); i < n; i += gstride()) out[i] = in[i];
}
__global__ void k_iota_u32(uint32_t *p, uint64_t n) {
  for (uint64_t i = gtid(); i < n; i += gstride()) p[i] = (uint32_t)i;
}
// copy rows (ptr CSR, canonical) into a ragged layout with `extra` spare slots per row (Montgomery)
__global__ void k_make_ragged(FieldP F, const uint64_t *ptr, const uint32_t *key, const Fe *val, uint64_t n,
                              uint64_t extra, uint64_t *off, uint32_t *len, uint32_t *okey, Fe *oval) {
  for (uint64_t r = gtid(); r < n; r += gstride()) {
    uint64_t b = ptr[r], e = ptr[r + 1];
    uint64_t o = b + extra * r;
    off[r] = o;
    len[r] = (uint32_t)(e - b);
    for (uint64_t i = b; i < e; ++i) {
      okey[o + (i - b)] = key[i];
      oval[o + (i - b)] = fto_mont(F, val[i]);
    }
  }
}
// view of selected rows: off/len gathered from a source view
__global__ void k_view_rows(const uint64_t *soff, const uint32_t *slen, const uint32_t *ids, uint64_t n,
                            uint64_t *off, uint32_t *len) {
  for (uint64_t i = gtid(); i < n; i += gstride()) {
    off[i] = soff[ids[i]];
    len[i] = slen[ids[i]];
  }
}
__global__ void k_set_offsets(const uint64_t *base_scan, uint64_t base, uint64_t *off, uint64_t n) {
  for (uint64_t i = gtid(); i < n; i += gstride()) off[i] = base + base_scan[i];
}
// eq_cluster_simplification's forbidden-pair constraints (:181-187): per forbidden signal f
// {f in an eq cluster, cluster size, min forbidden of the cluster, max row of the cluster}
__global__ void k_eq_forb_info(const uint32_t *fl, uint64_t nf, const uint32_t *root, const uint8_t *in_eq, const uint32_t *cnt,
                               const uint32_t *minf, const int32_t *maxrow, uint32_t *out) {
  for (uint64_t i = gtid(); i < nf; i += gstride()) {
    const uint32_t f = fl[i], r = root[i];
    out[4 * i] = in_eq[f];
    out[4 * i + 1] = cnt[r];
    out[4 * i + 2] = minf[r];
    out[4 * i + 3] = (uint32_t)maxrow[r];
  }
}
// rows whose two signals are forbidden: {row, keys, size of the row's cluster, the two values}
__global__ void k_eq_bf_info(const uint32_t *bf, uint64_t n, const uint64_t *ptr, const uint32_t *key, const Fe *val,
                             const uint32_t *uf, const uint32_t *cnt, uint64_t *rec) {
  for (uint64_t q = gtid(); q < n; q += gstride()) {
    const uint32_t r = bf[q];
    const uint64_t p0 = ptr[r];
    const uint32_t k0 = key[p0], k1 = key[p0 + 1];
    uint32_t x = k0;  // roots are compressed after k_eq_assign; walk to be safe
    while (uf[x] != x) x = uf[x];
    uint64_t *o = rec + 11 * q;
    o[0] = r;
    o[1] = ((uint64_t)k1 << 32) | k0;
    o[2] = cnt[x];
    for (int t = 0; t < 4; ++t) { o[3 + t] = val ? val[p0].l[t] : 0; o[7 + t] = val ? val[p0 + 1].l[t] : 0; }
  }
}
__global__ void k_flag_linear(const uint32_t *la, const uint32_t *lb, uint64_t n, uint64_t *flag_lin, uint64_t *flag_nl) {
  for (uint64_t i = gtid(); i < n; i += gstride()) {
    bool lin = la[i] == 0 && lb[i] == 0;
    flag_lin[i] = lin ? 1 : 0;
    flag_nl[i] = lin ? 0 : 1;
  }
}
__global__ void k_scatter_ids(const uint64_t *flag, const uint64_t *pos, uint64_t n, uint32_t *ids) {
  for (uint64_t i = gtid(); i < n; i += gstride())
    if (flag[i]) ids[pos[i]] = (uint32_t)i;
}
__global__ void k_set_rank(const uint32_t *sig, const int32_t *rank, uint64_t n, int32_t *rank_of) {
  for (uint64_t i = gtid(); i < n; i += gstride()) rank_of[sig[i]] = rank[i];
}
__global__ void k_turn_flags(const int32_t *turn, uint64_t n, uint64_t *flag) {
  for (uint64_t i = gtid(); i < n; i += gstride()) flag[i] = turn[i] >= 0 ? 1 : 0;
}
__global__ void k_commit_round(const uint8_t *touched, const int32_t *turn, uint64_t n, DRows a, DRows b, DRows c,
                               DRows oa, DRows ob, DRows oc) {
  for (uint64_t r = gtid(); r < n; r += gstride()) {
    if (!touched[r]) continue;
    if (turn[r] >= 0) {  // extracted: the linear content is kept in the round's view; storage emptied
      a.len[r] = 0;
      b.len[r] = 0;
      c.off[r] = oc.off[r];
      c.len[r] = oc.len[r];
      continue;
    }
    a.off[r] = oa.off[r]; a.len[r] = oa.len[r];
    b.off[r] = ob.off[r]; b.len[r] = ob.len[r];
    c.off[r] = oc.off[r]; c.len[r] = oc.len[r];
  }
}
__global__ void k_unmark_list(const uint32_t *sig, uint64_t n, uint8_t *bits) {
  for (uint64_t i = gtid(); i < n; i += gstride()) bits[sig[i]] = 0;
}
__global__ void k_zero_c(const uint32_t *ids, uint64_t n, uint32_t *clen) {
  for (uint64_t i = gtid(); i < n; i += gstride()) clen[ids[i]] = 0;
}
__global__ void k_nonempty_flags(const uint32_t *la, const uint32_t *lb, const uint32_t *lc, uint64_t n, uint64_t *flag) {
  for (uint64_t i = gtid(); i < n; i += gstride()) flag[i] = (la[i] | lb[i] | lc[i]) ? 1 : 0;
}

// (signal, row) pairs of the round-1 storage rows for the flagged signals: the initial lists of
// build_non_linear_signal_map (:327-343) restricted to the signals a later round asks for.
__device__ inline bool d_has_key(const uint32_t *k, uint32_t n, uint32_t s) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    if (k[mid] < s) lo = mid + 1; else hi = mid;
  }
  return lo < n && k[lo] == s;
}
__global__ void k_emit_pairs(DRows a, DRows b, DRows c, const uint8_t *flag, uint64_t *pairs, unsigned long long *cnt,
                             uint64_t cap) {
  for (uint64_t r = gtid(); r < a.n; r += gstride()) {
    const uint32_t *ka = a.key + a.off[r], *kb = b.key + b.off[r], *kc = c.key + c.off[r];
    uint32_t na = a.len[r], nb = b.len[r], nc = c.len[r];
    for (int part = 0; part < 3; ++part) {
      const uint32_t *k = part == 0 ? ka : part == 1 ? kb : kc;
      uint32_t n = part == 0 ? na : part == 1 ? nb : nc;
      for (uint32_t i = 0; i < n; ++i) {
        uint32_t s = k[i];
        if (!flag[s]) continue;
        if (part >= 1 && d_has_key(ka, na, s)) continue;
        if (part == 2 && d_has_key(kb, nb, s)) continue;
        unsigned long long o = atomicAdd(cnt, 1ull);
        if (o < cap) pairs[o] = ((uint64_t)s << 32) | (uint32_t)r;
      }
    }
  }
}

// ---------------------------------------------------------------- round ordering (rounds >= 2)
// the valid substitution slots of a round (slot - cluster start < #subs of the cluster)
__global__ void k_sub_valid(const uint32_t *cid, const uint64_t *cl_off, const uint32_t *n_sub, uint64_t n, uint64_t *flag) {
  for (uint64_t s = gtid(); s < n; s += gstride()) {
    const uint32_t c = cid[s];
    flag[s] = s - cl_off[c] < n_sub[c] ? 1 : 0;
  }
}
__global__ void k_sub_keys(const uint32_t *cid, const uint64_t *flag, const uint64_t *pos, const uint32_t *h_sig, uint64_t n,
                           uint64_t *key, uint32_t *val) {
  for (uint64_t s = gtid(); s < n; s += gstride())
    if (flag[s]) {
      key[pos[s]] = ((uint64_t)cid[s] << 32) | h_sig[s];
      val[pos[s]] = (uint32_t)s;
    }
}
// the ordered list: `from`, RHS location, and the dense signal -> rank index
__global__ void k_sub_info(const uint64_t *key, const uint32_t *U, const uint64_t *h_off, const uint32_t *h_len, uint64_t n,
                           uint32_t *usig, uint64_t *uoff, uint32_t *ulen, int32_t *rank_of) {
  for (uint64_t i = gtid(); i < n; i += gstride()) {
    const uint32_t s = (uint32_t)key[i];
    usig[i] = s;
    uoff[i] = h_off[U[i]];
    ulen[i] = h_len[U[i]];
    rank_of[s] = (int32_t)i;
  }
}
__global__ void k_unset_rank(const uint32_t *sig, uint64_t n, int32_t *rank_of) {
  for (uint64_t i = gtid(); i < n; i += gstride()) rank_of[sig[i]] = -1;
}

// ---------------------------------------------------------------- sharded elimination
// The size-ordered cluster lists are dealt to the ranks in snake order (0,1,..,W-1,W-1,..,0, ...),
// so every rank gets a near-equal share of each size class and the largest clusters spread first.
__host__ __device__ inline int snake_rank(uint64_t pos, int W) {
  uint64_t p = pos % (2 * (uint64_t)W);
  return p < (uint64_t)W ? (int)p : (int)(2 * (uint64_t)W - 1 - p);
}
__global__ void k_fill_u8_ids(const uint32_t *ids, uint64_t n, uint8_t v, uint8_t *out) {
  for (uint64_t i = gtid(); i < n; i += gstride()) out[ids[i]] = v;
}
// number of positions < n that rank r owns
static uint64_t snake_count(uint64_t n, int W, int r) {
  uint64_t per = 2 * (uint64_t)W, k = n / per, rem = n % per;
  return 2 * k + (rem > (uint64_t)r ? 1 : 0) + (rem > per - 1 - r ? 1 : 0);
}
// rank r's clusters of a size-ordered list, in list order (closed form: no scan)
__global__ void k_shard_pick(const uint32_t *ids, uint64_t n_out, int W, int r, uint32_t *out) {
  const uint64_t per = 2 * (uint64_t)W;
  for (uint64_t j = gtid(); j < n_out; j += gstride())
    out[j] = ids[(j / 2) * per + ((j & 1) ? per - 1 - r : (uint64_t)r)];
}
__global__ void k_shard_owner(const uint32_t *ids, uint64_t n, int W, uint8_t *owner) {
  for (uint64_t i = gtid(); i < n; i += gstride()) owner[ids[i]] = (uint8_t)snake_rank(i, W);
}
// The exchange, packed: each rank sends only its own clusters' records -- a substitution as
// (slot, from, RHS length, entry offset), its right-hand side only when `from` is needed by some
// row still to be substituted (round 1: the relevant set, build_relevant_set :398-429 -- signals of
// the non-linear rows after the eq renames, minus the constant ones; later rounds: the keys of the
// non-linear signal map, :345-396), a leftover as (slot, length, entry offset) with its entries.
// Every rank unpacks every rank's records into its per-slot arrays (slot = cluster start + index,
// so the counts per cluster follow from the records).
struct XRec {
  uint32_t slot, sig, len, eoff;
};
__global__ void k_xpk_count(const uint32_t *cid, const uint64_t *cl_off, const uint8_t *owner, int r, const uint32_t *n_sub,
                            const uint32_t *n_left, const uint32_t *h_sig, const uint32_t *h_len, const uint32_t *l_len,
                            const uint8_t *need, uint64_t n_slots, uint64_t *sf, uint64_t *lf, uint64_t *se, uint64_t *le) {
  for (uint64_t s = gtid(); s < n_slots; s += gstride()) {
    const uint32_t c = cid[s];
    const uint64_t i = s - cl_off[c];
    const bool own = owner[c] == r;
    const bool is_sub = own && i < n_sub[c], is_left = own && i < n_left[c];
    sf[s] = is_sub;
    se[s] = is_sub && (!need || need[h_sig[s]]) ? h_len[s] : 0;
    lf[s] = is_left;
    le[s] = is_left ? l_len[s] : 0;
  }
}
__global__ void k_xpk_fill(const uint32_t *cid, const uint64_t *cl_off, const uint64_t *sf, const uint64_t *sp,
                           const uint64_t *se, const uint64_t *sep, const uint64_t *lf, const uint64_t *lp, const uint64_t *le,
                           const uint64_t *lep, uint64_t sub_ent, const uint32_t *h_sig, const uint64_t *h_off,
                           const uint64_t *l_off, const uint32_t *pk, const Fe *pv, uint64_t n_slots, XRec *srec, XRec *lrec,
                           uint32_t *ek, Fe *ev) {
  for (uint64_t s = gtid(); s < n_slots; s += gstride()) {
    if (sf[s]) {
      const uint64_t o = sep[s], m = se[s];
      srec[sp[s]] = XRec{(uint32_t)s, h_sig[s], (uint32_t)m, (uint32_t)o};
      for (uint64_t t = 0; t < m; ++t) { ek[o + t] = pk[h_off[s] + t]; ev[o + t] = pv[h_off[s] + t]; }
    }
    if (lf[s]) {
      const uint64_t o = sub_ent + lep[s], m = le[s];
      lrec[lp[s]] = XRec{(uint32_t)s, 0u, (uint32_t)m, (uint32_t)o};
      for (uint64_t t = 0; t < m; ++t) { ek[o + t] = pk[l_off[s] + t]; ev[o + t] = pv[l_off[s] + t]; }
    }
  }
}
// one rank's block of records; `base` = where that rank's entries start in the gathered pool
__global__ void k_xunpack(const XRec *srec, uint64_t ns, const XRec *lrec, uint64_t nl, uint64_t base, const uint32_t *cid,
                          uint32_t *h_sig, uint64_t *h_off, uint32_t *h_len, uint64_t *l_off, uint32_t *l_len, uint32_t *n_sub,
                          uint32_t *n_left, int32_t *sub_of, uint8_t *deleted) {
  for (uint64_t j = gtid(); j < ns + nl; j += gstride()) {
    if (j < ns) {
      const XRec x = srec[j];
      h_sig[x.slot] = x.sig;
      h_len[x.slot] = x.len;
      h_off[x.slot] = base + x.eoff;
      sub_of[x.sig] = (int32_t)x.slot;
      deleted[x.sig] = 1;
      atomicAdd(&n_sub[cid[x.slot]], 1u);
    } else {
      const XRec x = lrec[j - ns];
      l_len[x.slot] = x.len;
      l_off[x.slot] = base + x.eoff;
      atomicAdd(&n_left[cid[x.slot]], 1u);
    }
  }
}
// round 1's relevant set: the signals of the non-linear rows after the eq renames, minus the
// constant ones (build_relevant_set :398-429)
__global__ void k_mark_relevant(DRows R, const int32_t *eq_rep, const uint8_t *ce_has, uint8_t *need) {
  for (uint64_t r = gtid(); r < R.n; r += gstride())
    for (uint32_t i = 0; i < R.len[r]; ++i) {
      const uint32_t k = R.key[R.off[r] + i];
      const int32_t t = eq_rep[k];
      const uint32_t k1 = t >= 0 ? (uint32_t)t : k;
      if (!ce_has[k1]) need[k1] = 1;
    }
}

// ---------------------------------------------------------------- lconst on the device
// The forbidden-only constraints the reference collects in `lconst` -- eq_simplification's pair rows
// (:181-187), constant_eq_simplification's kept rows (:253-273), every round's cluster leftovers
// (:318-323, :629-634) and at --O1 the linear rows themselves (:575-577) -- as C-only rows of one
// device heap, in lconst order.  fix_constraint (algebra.rs:1155-1157; for a row with A = B = empty
// it only removes zero coefficients) is applied as they are copied in; a row it empties stays with
// length 0 and is dropped with the other empty rows at the end (extract_with(is_empty), :697).
// Rows of a source view (ids == nullptr: rows 0..n) -- cnt[i]: its non-zero entries.
__global__ void k_lc_count(DRows src, const uint32_t *ids, uint64_t n, uint64_t *cnt) {
  for (uint64_t i = gtid(); i < n; i += gstride()) {
    const uint64_t r = ids ? ids[i] : i;
    const uint64_t o = src.off[r];
    uint64_t c = 0;
    for (uint32_t t = 0; t < src.len[r]; ++t) c += fe_is_zero(src.val[o + t]) ? 0 : 1;
    cnt[i] = c;
  }
}
// ... copied to the heap: row row0 + i at entry base + pos[i]
__global__ void k_lc_copy(DRows src, const uint32_t *ids, uint64_t n, const uint64_t *pos, uint64_t base, uint64_t row0,
                          DRows lc) {
  for (uint64_t i = gtid(); i < n; i += gstride()) {
    const uint64_t r = ids ? ids[i] : i;
    const uint64_t o = src.off[r], w0 = base + pos[i];
    uint64_t w = w0;
    for (uint32_t t = 0; t < src.len[r]; ++t) {
      const Fe v = src.val[o + t];
      if (fe_is_zero(v)) continue;
      lc.key[w] = src.key[o + t];
      lc.val[w] = v;
      ++w;
    }
    lc.off[row0 + i] = w0;
    lc.len[row0 + i] = (uint32_t)(w - w0);
  }
}
// the leftover slots of a round in lconst order (cluster index, then push order): flag[s] = s is a
// leftover slot of its cluster
__global__ void k_left_flags(const uint32_t *cid, const uint64_t *cl_off, const uint32_t *n_left, uint64_t n, uint64_t *flag) {
  for (uint64_t s = gtid(); s < n; s += gstride()) {
    const uint32_t c = cid[s];
    flag[s] = s - cl_off[c] < n_left[c] ? 1 : 0;
  }
}

// ---------------------------------------------------------------- host clustering
// build_clusters (constraint_simplification.rs:45-99): arena order + dest ++ src lists.
// D2H canonical content of pool maps (leftovers or RHS)
static void fetch_pool_maps(rs_engine *E, const std::vector<uint64_t> &off, const std::vector<uint32_t> &len,
                            const uint32_t *pk, const Fe *pv, std::vector<uint32_t> &keys, std::vector<uint64_t> &vals,
                            std::vector<uint64_t> &optr) {
  uint64_t n = off.size();
  optr.assign(n + 1, 0);
  for (uint64_t i = 0; i < n; ++i) optr[i + 1] = optr[i] + len[i];
  uint64_t tot = optr[n];
  keys.resize(tot);
  vals.resize(4 * tot);
  if (tot == 0) return;
  uint64_t *d_off = E->A.get<uint64_t>("fp.off", n);
  uint32_t *d_len = E->A.get<uint32_t>("fp.len", n);
  uint64_t *d_optr = E->A.get<uint64_t>("fp.optr", n + 1);
  uint32_t *d_k = E->A.get<uint32_t>("fp.k", tot);
  uint64_t *d_v = E->A.get<uint64_t>("fp.v", 4 * tot);
  h2d(E, d_off, off.data(), 8 * n);
  h2d(E, d_len, len.data(), 4 * n);
  h2d(E, d_optr, optr.data(), 8 * (n + 1));
  launch(E->st, k_pool_to_canon, n, E->F, (const uint64_t *)d_off, (const uint32_t *)d_len, (const uint64_t *)d_optr, n,
         pk, pv, d_k, d_v);
  HC(hipMemcpyAsync(keys.data(), d_k, 4 * tot, hipMemcpyDeviceToHost, E->st));
  HC(hipMemcpyAsync(vals.data(), d_v, 32 * tot, hipMemcpyDeviceToHost, E->st));
  HC(hipStreamSynchronize(E->st));
}

// D2H keys of pool maps (no values)
static bool is_zero4(const uint64_t *v) { return (v[0] | v[1] | v[2] | v[3]) == 0; }


// ---------------------------------------------------------------- elimination driver
struct ElimOut {  // what the host keeps of a round's elimination (the rest stays on the device)
  uint64_t n_clusters = 0, n_slots = 0;
  uint64_t n_sub = 0, n_left = 0;  // totals over the clusters
};
__global__ void k_sum_counts(const uint32_t *n_sub, const uint32_t *n_left, uint64_t n, unsigned long long *sums) {
  unsigned long long a = 0, b = 0;
  for (uint64_t c = gtid(); c < n; c += gstride()) {
    a += n_sub[c];
    b += n_left[c];
  }
  wave_atomic_add(sums, a);
  wave_atomic_add(sums + 1, b);
}

struct Pool {
  uint32_t *pk = nullptr;
  Fe *pv = nullptr;
  unsigned long long *top = nullptr;
  uint64_t cap = 0;
};

static Pool get_pool(rs_engine *E, uint64_t want) {
  Pool P;
  P.cap = want;
  P.pk = E->A.get<uint32_t>("pool.k", want);
  P.pv = E->A.get<Fe>("pool.v", want);
  P.top = E->A.get<unsigned long long>("pool.top", 1);
  return P;
}

// Runs linear_simplification (:275-325) for the rows of `view`; on return the per-slot arrays in
// the arena hold the substitutions (h_*) and leftovers (l_*), sub_of/deleted are updated.
// build_clusters (:45-99) on the device (cluster.hpp): cluster offsets and row order in HBM, the
// process_4 / lane split of the clusters (largest first). Only counts and the cluster offsets (for
// the host-side round bookkeeping) come back to the host.
struct DevClusters {
  uint32_t *perm = nullptr, *big = nullptr, *small = nullptr, *cid = nullptr;
  uint64_t *cl_off = nullptr;
  uint64_t n_slots = 0, n_big = 0, n_small = 0, tot_nnz = 0;
  // the largest clusters' row orders are still being replayed on the second stream (evx[7] marks
  // the end); only the head -- ordered after the replay on that stream -- reads them until the join
  bool join_pending = false;
  // host copy of the sorted size keys of the kHeadLimit largest clusters (k_cl_sizekey: size in the
  // high word, inverted; the cluster index in the low word)
  std::vector<uint64_t> top_keys;
  // clusters the host replay found order-free (every row consumed by the uniques phase, d_cl_order_free):
  // no ordered loop at all, so a giant among them skips the giant path (it only sorted empty lists)
  std::unordered_set<uint32_t> order_free;
  bool timed = false;  // evc[0..1] bracket the clustering kernels
  uint64_t alg = 0;    // their algorithmic bytes
};
// Split composition (k_big_finish with ElimArgs.split, then one k_compose_level launch per Kahn
// level of every cluster at once over the whole GPU, k_big_emit at the end).  Level L reads count
// L%3, appends to (L+1)%3 and zeroes (L+2)%3 -- the one level L-1 read and level L+1 appends to --
// and likewise alternates the deferred list's count: no memsets.  Every 4 levels the frontier count
// goes to pinned slot h[b % 4]; with `check` the host reads the slot of two batches back (it never
// waits for the level it just enqueued; launches past an empty frontier return at once).
struct LevelLoop {
  ElimArgs ah;
  const uint32_t *ids = nullptr;
  hipStream_t s = nullptr;
  uint64_t *cur = nullptr, *nxt = nullptr;
  uint64_t n_slots = 0;
  unsigned long long *h = nullptr;
  hipEvent_t *ev = nullptr;
  uint32_t level = 0, levels = 0;
  bool done = false;
  void run(uint32_t upto, bool check) {
    for (; !done && level <= n_slots + 1 && level < upto; ++level) {
      ElimArgs al = ah;
      al.cf_nbig = ah.cf_nbig + (level & 1);
      unsigned long long *nc = ah.cf_n + level % 3, *zc = ah.cf_n + (level + 2) % 3;
      unsigned long long *nn = ah.cf_n + (level + 1) % 3;
      hipLaunchKernelGGL(k_compose_level<8>, dim3(256), dim3(512), 0, s, al, ids, (const uint64_t *)cur, (const unsigned long long *)nc,
                         nxt, nn, level, zc, ah.cf_nbig + ((level + 1) & 1));
      hipLaunchKernelGGL(k_compose_big, dim3(256), dim3(64), 0, s, al, ids, nxt, nn);
      HC(hipGetLastError());
      std::swap(cur, nxt);
      levels = level + 1;
      if (level % 4 == 3) {
        const uint32_t b = level / 4;
        HC(hipMemcpyAsync(h + b % 4, nn, 8, hipMemcpyDeviceToHost, s));
        HC(hipEventRecord(ev[b % 4], s));
        if (check && b >= 2) {
          HC(hipEventSynchronize(ev[(b - 2) % 4]));
          if (!h[(b - 2) % 4]) done = true;
        }
      }
    }
  }
};

// Kahn levels of the head's composition launched over the whole GPU before k_compose_rest takes the
// rest per cluster in one workgroup each (level 0's items need no composition)
constexpr uint32_t kHeadGpuLevels = 8;
// the number of largest clusters eliminated on the second stream by the speculative loop: the tail's
// one-wave loop is bound by its largest clusters (~4.5 us a row), which hold the first frames pass --
// and so the result stream -- back until the tail is done.  On the metric circuit (host -> host,
// best of 5): 48 -> tail loop 7.7 ms, 52.0 ms; 96 -> 5.1 ms, 49.7 ms; 160 -> 5.0 ms, 49.6 ms (device
// time 39.8 / 37.7 / 39.1 ms: the head grows with its cluster count)
constexpr uint64_t kHeadLimit = 96;
// the tail's largest clusters, eliminated on the main stream while the rest runs beside them
// (host -> host on the metric circuit, best of 5: one group 49.6 ms; split at 256 / 1024 / 4096
// clusters 48.6 / 48.4 / 48.7 ms; templated 159.5 vs 162.6 / 161.1 / 159.5 ms)
constexpr uint64_t kTailSplit = 1024;
// The arena replay of one cluster on the host (k_cl_replay_lane's walk): rows in index order, each
// pair's previous row found by path halving and its root's list appended to the row's.  A serial
// union-find of dependent accesses: ~20 ns a pair in a host cache against ~0.3 us in LDS, and the
// largest clusters' replays gate the head's ordered loop.  qo: the cluster's per-row pair offsets
// (n + 1, relative), st: its pairs, srow: its rows; out: the rows in list order.
static void host_replay(uint32_t n, const uint64_t *qo, const uint32_t *st, const uint32_t *srow, uint32_t *out) {
  std::vector<uint32_t> C2(n), T(n), N(n, RS_NONE);
  for (uint32_t t = 0; t < n; ++t) {
    C2[t] = t;
    T[t] = t;
    for (uint64_t q = qo[t]; q < qo[t + 1]; ++q) {
      uint32_t p = st[q] & ~kClRowBit;
      if (p == kClNoPrev) continue;
      while (C2[p] != p) {
        const uint32_t g = C2[C2[p]];
        C2[p] = g;
        p = g;
      }
      if (p == t) continue;
      N[T[t]] = p;
      T[t] = T[p];
      C2[p] = t;
    }
  }
  uint32_t x = n - 1, q = 0;
  while (x != RS_NONE && q < n) {
    out[q++] = srow[x];
    x = N[x];
  }
}

__global__ void k_put_u64(uint64_t *p, uint64_t v) {
  if (gtid() == 0) *p = v;
}
static DevClusters gpu_clusters(rs_engine *E, const DRows &V, int old_heur, const uint8_t *d_forb, ElimOut &eo) {
  Arena &A = E->A;
  hipStream_t st = E->st;
  DevClusters D;
  const uint64_t n = V.n;
  eo = ElimOut{};
  D.cl_off = A.get<uint64_t>("el.cl", 1);
  HC(hipMemsetAsync(D.cl_off, 0, 8, st));
  if (n == 0) return D;
  // the host's share of the span: time blocked in the read-backs' synchronisations and in the host
  // replay (rs_stats.cluster_host_ms); RS_PROF prints the host clock at each step
  double &hw = E->stats.cluster_host_ms;
  std::vector<std::pair<const char *, double>> marks;
  auto mark = [&](const char *w) {
    if (g_prof_env) marks.emplace_back(w, now_ms());
  };
  auto sync = [&](hipStream_t s) {
    const double t = now_ms();
    HC(hipStreamSynchronize(s));
    hw += now_ms() - t;
  };
  struct PrintMarks {
    std::vector<std::pair<const char *, double>> &m;
    ~PrintMarks() {
      if (m.size() < 2) return;
      fprintf(stderr, "[rs-prof] clustering host clock (ms from the start):");
      for (size_t i = 1; i < m.size(); ++i) fprintf(stderr, " %s %.2f", m[i].first, m[i].second - m[0].second);
      fprintf(stderr, "\n");
    }
  } print_marks{marks};
  mark("start");
  HC(hipEventRecord(E->evc[0], st));
  uint64_t *npairs = A.get<uint64_t>("cl.np", n);
  unsigned long long *stat = A.get<unsigned long long>("cl.stat", 8);
  HC(hipMemsetAsync(stat, 0, 64, st));
  launch_capped(st, k_cl_count, n, 1024, V, npairs, stat);
  uint64_t *poff = A.get<uint64_t>("cl.poff", n);
  unsigned long long *hs = (unsigned long long *)pin_get(E, 18, kPinRb);  // pinned: no staged copy
  HC(hipMemcpyAsync(hs, stat, 16, hipMemcpyDeviceToHost, st));
  const uint64_t P = excl_scan_u64(E, npairs, poff, n, "cl1", &hw);  // (its read-back synchronises)
  mark("pairs");
  D.tot_nnz = hs[0];
  const uint64_t n_act = hs[1];
  if (n_act == 0) return D;
  D.timed = true;
  int sbits = 1;
  while (sbits < 32 && (1ull << sbits) <= E->S) ++sbits;
  uint32_t *uf = A.get<uint32_t>("cl.uf", n);
  launch(st, k_iota_u32, n, uf, n);
  uint32_t *prevrow = A.get<uint32_t>("cl.prev", P);
  uint8_t *has_unique = A.get<uint8_t>("cl.uniq", n);
  HC(hipMemsetAsync(has_unique, 0, n, st));
  if (P) {
    uint64_t *pk = A.get<uint64_t>("cl.pk", P), *pk2 = A.get<uint64_t>("cl.pk2", P);
    uint32_t *ps = A.get<uint32_t>("cl.ps", P), *ps2 = A.get<uint32_t>("cl.ps2", P);
    launch(st, k_cl_fill, n, V, (const uint64_t *)poff, pk, ps);
    sort_pairs(E, (const uint64_t *)pk, pk2, (const uint32_t *)ps, ps2, P, 32 + sbits, "cl1");
    launch(st, k_cl_link, P, (const uint64_t *)pk2, (const uint32_t *)ps2, P, prevrow, uf, d_forb, has_unique);
  }
  int32_t *cmax = A.get<int32_t>("cl.cmax", n);
  launch(st, k_fill_i32, n, cmax, (int32_t)-1, n);
  launch(st, k_cl_root, n, (const uint32_t *)V.len, n, uf, cmax);
  uint64_t *rk = A.get<uint64_t>("cl.rk", n), *rk2 = A.get<uint64_t>("cl.rk2", n);
  uint32_t *ri = A.get<uint32_t>("cl.ri", n), *srow = A.get<uint32_t>("cl.srow", n);
  launch(st, k_cl_key, n, (const uint32_t *)V.len, n, uf, (const int32_t *)cmax, rk, ri);
  sort_pairs(E, (const uint64_t *)rk, rk2, (const uint32_t *)ri, srow, n, 64, "cl2");
  uint64_t *flag = A.get<uint64_t>("cl.flag", n_act), *fscan = A.get<uint64_t>("cl.fscan", n_act);
  launch(st, k_cl_flag, n_act, (const uint64_t *)rk2, n_act, flag);
  const uint64_t n_cl = excl_scan_u64(E, flag, fscan, n_act, "cl2", &hw);
  mark("clusters");
  D.cl_off = A.get<uint64_t>("el.cl", n_cl + 1);
  uint32_t *cid = A.get<uint32_t>("cl.cid", n_act), *gpos = A.get<uint32_t>("cl.gpos", n);
  uint64_t *qn = A.get<uint64_t>("cl.qn", n_act), *q_off = A.get<uint64_t>("cl.qoff", n_act + 1);
  uint32_t *n_ordered = A.get<uint32_t>("cl.nord", n_cl);
  HC(hipMemsetAsync(n_ordered, 0, 4 * n_cl, st));
  launch(st, k_cl_starts, n_act, (const uint64_t *)rk2, (const uint64_t *)fscan, (const uint32_t *)srow,
         (const uint64_t *)npairs, n_act, n_cl, D.cl_off, cid, gpos, qn, (const uint8_t *)has_unique, n_ordered);
  // the stream holds every active row's pairs once: Q = P (no read-back, and no host-to-device copy
  // of the total queued behind the input's upload on the copy engine)
  const uint64_t Q = P;
  dev_scan_u64(E, qn, q_off, n_act, st, "cl3");
  hipLaunchKernelGGL(k_put_u64, dim3(1), dim3(64), 0, st, q_off + n_act, Q);
  HC(hipGetLastError());
  uint32_t *stream = A.get<uint32_t>("cl.stream", Q);
  launch(st, k_cl_stream, n_act, (const uint32_t *)srow, (const uint64_t *)poff, (const uint32_t *)prevrow,
         (const uint32_t *)gpos, (const uint32_t *)cid, (const uint64_t *)D.cl_off, (const uint64_t *)q_off, n_act,
         stream);
  // sort order: (workgroup-kernel clusters first, size desc, index asc)
  uint64_t *sk = A.get<uint64_t>("cl.sk", n_cl), *sk2 = A.get<uint64_t>("cl.sk2", n_cl);
  uint32_t *si = A.get<uint32_t>("cl.si", n_cl), *sorted = A.get<uint32_t>("el.big", n_cl);
  unsigned long long *cnt = stat + 2;
  launch_capped(st, k_cl_sizekey, n_cl, 1024, (const uint64_t *)D.cl_off, n_cl, (const uint32_t *)srow, (const uint32_t *)V.len, sk, si, cnt);
  sort_pairs(E, (const uint64_t *)sk, sk2, (const uint32_t *)si, sorted, n_cl, 64, "cl3");
  // the size keys of the largest clusters (the head's; the giant path reads their row counts) and the
  // class counts, into pinned memory in one read-back
  const uint64_t n_top = std::min<uint64_t>(n_cl, kHeadLimit);
  unsigned long long *hcb = (unsigned long long *)pin_get(E, 19, 8 * (8 + kHeadLimit));
  unsigned long long *hc = hcb;
  HC(hipMemcpyAsync(hc, cnt, 40, hipMemcpyDeviceToHost, st));
  if (n_top) HC(hipMemcpyAsync(hcb + 8, sk2, 8 * n_top, hipMemcpyDeviceToHost, st));
  sync(st);
  D.top_keys.assign(hcb + 8, hcb + 8 + n_top);
  mark("sizes");
  const uint64_t first = n_top ? D.top_keys[0] : 0;
  // replay of the arena merges -> row order inside every cluster
  D.perm = A.get<uint32_t>("el.perm", n_act);
  uint32_t *c2c = A.get<uint32_t>("cl.c2c", n_act), *tail = A.get<uint32_t>("cl.tail", n_act);
  uint32_t *next = A.get<uint32_t>("cl.next", n_act);
  launch(st, k_cl_replay_lane, n_cl, (const uint64_t *)D.cl_off, n_cl, (const uint64_t *)q_off,
         (const uint32_t *)stream, (const uint32_t *)srow, c2c, tail, next, D.perm, (const uint32_t *)n_ordered,
         old_heur);
  // (kClMid, kClLds]: the arena replay on the host (host_replay), beside the mid-size replays on the device
  if (hc[4]) {
    // launched first, so the device has the mid-size replays to do while the host replays
    if (hc[2] > hc[4]) {
      const uint64_t nm = hc[2] - hc[4];
      hipLaunchKernelGGL((k_cl_replay_wave<kClMid>), dim3((unsigned)std::min<uint64_t>(nm, 16384)), dim3(64), 0, st,
                         (const uint64_t *)D.cl_off, (const uint32_t *)(sorted + hc[3] + hc[4]), nm,
                         (const uint64_t *)q_off, (const uint32_t *)stream, (const uint32_t *)srow, next, D.perm,
                         (const uint32_t *)n_ordered, old_heur);
      HC(hipGetLastError());
    }
    const double th0 = now_ms();
    // every input of the replays is complete (the stream was synchronised above).  Per cluster (first
    // row, rows, first pair, pairs, ordered rows) into pinned memory; an order-free cluster's list is
    // its row order (d_cl_order_free), copied on the device; the rest are replayed on the host (their
    // offsets, pair streams and rows in one pinned staging block, the orders back from it)
    const uint64_t nh = hc[4];
    uint64_t *d_meta = A.get<uint64_t>("cl.rmeta", kMetaW * nh);
    launch(E->str, k_replay_meta, nh, (const uint64_t *)D.cl_off, (const uint32_t *)(sorted + hc[3]), nh,
           (const uint64_t *)q_off, (const uint32_t *)n_ordered, d_meta);
    uint64_t *meta = (uint64_t *)pin_get(E, 16, 8 * kMetaW * nh);
    HC(hipMemcpyAsync(meta, d_meta, 8 * kMetaW * nh, hipMemcpyDeviceToHost, E->str));
    sync(E->str);
    mark("replay meta");
    HC(hipEventRecord(E->evx[6], st));
    HC(hipStreamWaitEvent(E->st2, E->evx[6], 0));
    std::vector<uint64_t> todo;
    uint64_t tot_q = 0, tot_n = 0;
    for (uint64_t i = 0; i < nh; ++i) {
      const uint64_t rb = meta[kMetaW * i], qn = meta[kMetaW * i + 1];
      if (qn >= 350 && qn < 1000000 && !old_heur && meta[kMetaW * i + 4] == 0) {  // d_cl_order_free
        D.order_free.insert((uint32_t)meta[kMetaW * i + 5]);
        HC(hipMemcpyAsync(D.perm + rb, srow + rb, 4 * qn, hipMemcpyDeviceToDevice, E->st2));
        continue;
      }
      todo.push_back(i);
      tot_n += qn;
      tot_q += meta[kMetaW * i + 3];
    }
    const uint64_t nt = todo.size();
    if (nt) {
      // staging: qo (tot_n + nt u64), pairs (tot_q u32), rows (tot_n u32), orders (tot_n u32)
      uint8_t *stg = (uint8_t *)pin_get(E, 17, 8 * (tot_n + nt) + 4 * (tot_q + 2 * tot_n));
      uint64_t *qo = (uint64_t *)stg;
      uint32_t *hst = (uint32_t *)(qo + tot_n + nt), *hsrow = hst + tot_q, *hperm = hsrow + tot_n;
      std::vector<uint64_t> o_q(nt), o_n(nt), o_o(nt);
      for (uint64_t t = 0, oq = 0, on = 0, o = 0; t < nt; ++t) {
        const uint64_t i = todo[t], rb = meta[kMetaW * i], qn = meta[kMetaW * i + 1], np = meta[kMetaW * i + 3];
        o_q[t] = oq;
        o_n[t] = on;
        o_o[t] = o;
        HC(hipMemcpyAsync(qo + o, q_off + rb, 8 * (qn + 1), hipMemcpyDeviceToHost, E->str));
        if (np) HC(hipMemcpyAsync(hst + oq, stream + meta[kMetaW * i + 2], 4 * np, hipMemcpyDeviceToHost, E->str));
        HC(hipMemcpyAsync(hsrow + on, srow + rb, 4 * qn, hipMemcpyDeviceToHost, E->str));
        oq += np;
        on += qn;
        o += qn + 1;
      }
      sync(E->str);
      mark("replay staged");
      std::atomic<uint64_t> next_t{0};
      auto work = [&] {  // a few host threads, largest cluster first (the list is size-ordered)
        for (uint64_t t; (t = next_t.fetch_add(1)) < nt;) {
          const uint64_t *qoi = qo + o_o[t], q0 = qoi[0];
          const uint32_t n_i = (uint32_t)meta[kMetaW * todo[t] + 1];
          std::vector<uint64_t> rel(n_i + 1);
          for (uint32_t k = 0; k <= n_i; ++k) rel[k] = qoi[k] - q0;
          host_replay(n_i, rel.data(), hst + o_q[t], hsrow + o_n[t], hperm + o_n[t]);
        }
      };
      const unsigned hwc = std::max(1u, std::thread::hardware_concurrency());
      const uint64_t n_th = std::min<uint64_t>({nt, (uint64_t)hwc, 16});
      const double tr0 = now_ms();
      std::vector<std::thread> th;
      for (uint64_t k = 1; k < n_th; ++k) th.emplace_back(work);
      work();
      for (auto &t : th) t.join();
      hw += now_ms() - tr0;
      mark("replayed");
      for (uint64_t t = 0; t < nt; ++t) {
        const uint64_t i = todo[t];
        HC(hipMemcpyAsync(D.perm + meta[kMetaW * i], hperm + o_n[t], 4 * meta[kMetaW * i + 1], hipMemcpyHostToDevice, E->st2));
      }
      sync(E->st2);  // the staging block is reused by the next round's replay
      mark("orders back");
    }
    if (g_prof_env)
      fprintf(stderr, "[rs-prof] host replay: %llu clusters (%llu order-free), %llu rows, %llu pairs, %.2f ms\n", (unsigned long long)nh,
              (unsigned long long)(nh - nt), (unsigned long long)tot_n, (unsigned long long)tot_q, now_ms() - th0);
  }
  if (hc[2] && !hc[4]) {  // (kClSmall, kClMid] (launched above when there is a host replay)
    const uint64_t nm = hc[2] - hc[4];
    hipLaunchKernelGGL((k_cl_replay_wave<kClMid>), dim3((unsigned)std::min<uint64_t>(nm, 16384)), dim3(64), 0, st,
                       (const uint64_t *)D.cl_off, (const uint32_t *)(sorted + hc[3] + hc[4]), nm,
                       (const uint64_t *)q_off, (const uint32_t *)stream, (const uint32_t *)srow, next, D.perm,
                       (const uint32_t *)n_ordered, old_heur);
    HC(hipGetLastError());
  }
  if (hc[4]) {  // join: the elimination reads every cluster's order -- deferred when every cluster
                // replayed there is a head cluster (single rank: the head is this rank's largest)
    HC(hipEventRecord(E->evx[7], E->st2));
    const bool sharded = E->comm && E->comm->world > 1;
    if (!sharded && hc[3] + hc[4] <= kHeadLimit) D.join_pending = true;
    else HC(hipStreamWaitEvent(st, E->evx[7], 0));
  }
  // elimination split: clusters of kWaveMin rows or more and the heavy small ones (a prefix of the
  // sort order, k_cl_sizekey) go to the workgroup kernels (process_3 or process_4 per cluster), the
  // rest one lane each
  const uint64_t h = 0, nb = hc[1];
  D.big = sorted + h;
  D.n_big = nb;
  D.n_small = n_cl - nb;
  D.small = A.get<uint32_t>("el.small", D.n_small);
  if (D.n_small) launch(st, k_cl_small_ids, D.n_small, (const uint32_t *)sorted, n_cl, h, nb, D.small);
  D.n_slots = n_act;
  D.cid = cid;
  eo.n_clusters = n_cl;
  eo.n_slots = n_act;
  HC(hipEventRecord(E->evc[1], st));
  // its algorithmic bytes: the rows' keys read twice (count, fill), each (signal, row) pair written,
  // sorted (one read and one write) and linked (read, prev written), ~8 words per row over the
  // union-find / root / key / order passes, the replay stream written and read
  D.alg = 8 * D.tot_nnz + 52 * P + 32 * n + 8 * Q;
  E->stats.n_clusters += n_cl;
  E->stats.max_cluster = std::max<uint64_t>(E->stats.max_cluster, (0xffffffffull - (first >> 32)) & 0x7fffffffull);
  return D;
}

// The exchange step of the sharded elimination: after it every rank holds the complete
// eliminated-signal map of the round -- every substitution's `from` (sub_of, deleted), the
// right-hand sides some later substitution step will read (`need`; null = all, e.g. for the
// substitution log), every leftover -- in a pool made of every rank's packed entries.  Four
// allgathervs of packed records and entries replace the round-1 design's zero-padded per-slot
// sum-allreduce and whole-pool gather.
// Replicated clusters (owner == W: the head, which every rank eliminates itself) are not exchanged
// and keep their counts; the received records land in a pool of their own (G), since the head may
// still be allocating from the local one.
__global__ void k_zero_owned(const uint8_t *owner, int W, uint64_t n, uint32_t *n_sub, uint32_t *n_left) {
  for (uint64_t c = gtid(); c < n; c += gstride())
    if (owner[c] < W) {
      n_sub[c] = 0;
      n_left[c] = 0;
    }
}
// shift the pool offsets of the replicated clusters' slots by `by` (their entries moved into G)
__global__ void k_shift_owned(const uint32_t *cid, const uint8_t *owner, int W, uint64_t n_slots, uint64_t by, uint64_t *h_off,
                              uint64_t *l_off) {
  for (uint64_t s = gtid(); s < n_slots; s += gstride())
    if (owner[cid[s]] == W) {
      h_off[s] += by;
      l_off[s] += by;
    }
}
static void shard_exchange(rs_engine *E, const ElimArgs &a, const DevClusters &D, const uint8_t *owner, const Pool &P,
                           const uint8_t *need, Pool &G) {
  Comm &CM = *E->comm;
  Arena &A = E->A;
  hipStream_t st = E->st;
  const double t0 = now_ms();
  A.defer = true;  // the head is still running on st2: no device-wide hipFree while its buffers grow
  const uint64_t n_slots = D.n_slots, n_cl = a.n_clusters;
  uint64_t *sf = A.get<uint64_t>("x.sf", n_slots), *sp = A.get<uint64_t>("x.sp", n_slots);
  uint64_t *se = A.get<uint64_t>("x.se", n_slots), *sep = A.get<uint64_t>("x.sep", n_slots);
  uint64_t *lf = A.get<uint64_t>("x.lf", n_slots), *lp = A.get<uint64_t>("x.lp", n_slots);
  uint64_t *le = A.get<uint64_t>("x.le", n_slots), *lep = A.get<uint64_t>("x.lep", n_slots);
  launch(st, k_xpk_count, n_slots, (const uint32_t *)D.cid, (const uint64_t *)D.cl_off, owner, CM.rank,
         (const uint32_t *)a.n_sub, (const uint32_t *)a.n_left, (const uint32_t *)a.h_sig, (const uint32_t *)a.h_len,
         (const uint32_t *)a.l_len, need, n_slots, sf, lf, se, le);
  const uint64_t n_s = excl_scan_u64(E, sf, sp, n_slots, "xs");
  const uint64_t n_l = excl_scan_u64(E, lf, lp, n_slots, "xl");
  const uint64_t e_s = excl_scan_u64(E, se, sep, n_slots, "xse");
  const uint64_t e_l = excl_scan_u64(E, le, lep, n_slots, "xle");
  XRec *srec = A.get<XRec>("x.srec", n_s + 1), *lrec = A.get<XRec>("x.lrec", n_l + 1);
  uint32_t *ek = A.get<uint32_t>("x.ek", e_s + e_l + 1);
  Fe *ev = A.get<Fe>("x.ev", e_s + e_l + 1);
  launch(st, k_xpk_fill, n_slots, (const uint32_t *)D.cid, (const uint64_t *)D.cl_off, (const uint64_t *)sf,
         (const uint64_t *)sp, (const uint64_t *)se, (const uint64_t *)sep, (const uint64_t *)lf, (const uint64_t *)lp,
         (const uint64_t *)le, (const uint64_t *)lep, e_s, (const uint32_t *)a.h_sig, (const uint64_t *)a.h_off,
         (const uint64_t *)a.l_off, (const uint32_t *)P.pk, (const Fe *)P.pv, n_slots, srec, lrec, ek, ev);
  const std::vector<uint64_t> ns = CM.gather_u64(n_s, st), nl = CM.gather_u64(n_l, st), ne = CM.gather_u64(e_s + e_l, st);
  uint64_t ts = 0, tl = 0, te = 0;
  std::vector<uint64_t> cs(CM.world), cl(CM.world), ck(CM.world), cv(CM.world);
  for (int q = 0; q < CM.world; ++q) {
    ts += ns[q]; tl += nl[q]; te += ne[q];
    cs[q] = sizeof(XRec) * ns[q]; cl[q] = sizeof(XRec) * nl[q]; ck[q] = 4 * ne[q]; cv[q] = 32 * ne[q];
  }
  XRec *gs = A.get<XRec>("x.gs", ts + 1), *gl = A.get<XRec>("x.gl", tl + 1);
  uint32_t *gk = A.get<uint32_t>("pool.gk", te + 1);
  Fe *gv = A.get<Fe>("pool.gv", te + 1);
  CM.allgatherv(srec, gs, cs, st);
  CM.allgatherv(lrec, gl, cl, st);
  CM.allgatherv(ek, gk, ck, st);
  CM.allgatherv(ev, gv, cv, st);
  launch(st, k_zero_owned, n_cl, owner, CM.world, n_cl, a.n_sub, a.n_left);
  uint64_t os = 0, ol = 0, oe = 0;
  for (int q = 0; q < CM.world; ++q) {
    if (ns[q] + nl[q])
      launch(st, k_xunpack, ns[q] + nl[q], (const XRec *)(gs + os), ns[q], (const XRec *)(gl + ol), nl[q], oe,
             (const uint32_t *)D.cid, a.h_sig, a.h_off, a.h_len, a.l_off, a.l_len, a.n_sub, a.n_left, a.sub_of, a.deleted);
    os += ns[q]; ol += nl[q]; oe += ne[q];
  }
  HC(hipStreamSynchronize(st));
  A.defer = false;
  G.pk = gk;
  G.pv = gv;
  G.top = nullptr;
  G.cap = te;  // entries in use
  E->stats.exchange_ms += now_ms() - t0;
  E->stats.exchange_bytes += sizeof(XRec) * (ts + tl) + 36 * te + 24 * CM.world;
}

// ---- the giant path (giant_loop.hpp): head clusters of kGiantRows rows or more
// Buffers for a giant cluster of n rows (allocated before any launch of the round: a growing arena
// buffer is freed with hipFree, which waits for the whole device).
static GiantArgs giant_buffers(rs_engine *E, uint64_t n) {
  Arena &A = E->A;
  GiantArgs G{};
  G.n = n;
  G.uf = A.get<uint32_t>("gi.uf", E->S);
  G.gst = A.get<uint64_t>("gi.gst", E->S);
  G.rkey = A.get<uint64_t>("gi.rkey", n);
  G.rkey2 = A.get<uint64_t>("gi.rkey2", n);
  G.rval = A.get<uint32_t>("gi.rval", n);
  G.rval2 = A.get<uint32_t>("gi.rval2", n);
  G.comp_of = A.get<uint32_t>("gi.comp_of", n);
  G.c_start = A.get<uint32_t>("gi.c_start", n);
  G.c_size = A.get<uint32_t>("gi.c_size", n);
  G.ckey = A.get<uint64_t>("gi.ckey", n);
  G.ckey2 = A.get<uint64_t>("gi.ckey2", n);
  G.cidx = A.get<uint32_t>("gi.cidx", n);
  G.cidx2 = A.get<uint32_t>("gi.cidx2", n);
  G.c_nsub = A.get<uint32_t>("gi.c_nsub", n);
  G.c_nleft = A.get<uint32_t>("gi.c_nleft", n);
  G.c_dsub = A.get<uint32_t>("gi.c_dsub", n);
  G.scal = A.get<uint32_t>("gi.scal", 8);
  G.t_sig = A.get<uint32_t>("gi.t_sig", n);
  G.t_coef = A.get<Fe>("gi.t_coef", n);
  G.t_off = A.get<uint64_t>("gi.t_off", n);
  G.t_len = A.get<uint32_t>("gi.t_len", n);
  G.lmark = A.get<uint32_t>("gi.lmark", n);
  G.lscan = A.get<uint32_t>("gi.lscan", n);
  G.tl_off = A.get<uint64_t>("gi.tl_off", n);
  G.tl_len = A.get<uint32_t>("gi.tl_len", n);
  if (g_prof_env) {
    G.c_merges = A.get<uint32_t>("gi.c_merges", n);
    G.c_clk = A.get<uint64_t>("gi.c_clk", n);
    G.sec = A.get<unsigned long long>("gi.sec", 32);
  }
  size_t tb = 0;  // the sorts' and scans' temporaries at their final size
  HC(rocprim::radix_sort_pairs(nullptr, tb, G.rkey, G.rkey2, G.rval, G.rval2, (size_t)n, 0, 64, E->stg));
  (void)A.get<uint8_t>("sort.tmp.gi", tb);
  tb = 0;
  HC(rocprim::exclusive_scan(nullptr, tb, G.c_nsub, G.c_dsub, (uint32_t)0, (size_t)n, rocprim::plus<uint32_t>(), E->stg));
  (void)A.get<uint8_t>("dscan.tmp.gi", tb);
  return G;
}
// The giant path of head cluster c (position ci in the head list) on E->stg: components, the
// component loops, the results back into the cluster's slots (n_sub / n_left set at the end).
static void giant_launch(rs_engine *E, const ElimArgs &a, GiantArgs G, uint64_t c, uint64_t ci) {
  hipStream_t s = E->stg;
  G.ci = ci;
  const uint64_t n = G.n;
  const unsigned gb = (unsigned)std::min<uint64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_gi_state, dim3(gb), dim3(256), 0, s, a, G, c);
  hipLaunchKernelGGL(k_gi_union, dim3(gb), dim3(256), 0, s, a, G, c);
  hipLaunchKernelGGL(k_gi_rowkey, dim3(gb), dim3(256), 0, s, a, G, c);
  HC(hipGetLastError());
  sort_pairs(E, (const uint64_t *)G.rkey, G.rkey2, (const uint32_t *)G.rval, G.rval2, n, 64, "gi", s);
  hipLaunchKernelGGL(k_gi_segment, dim3(1), dim3(1024), 0, s, a, G);
  HC(hipGetLastError());
  sort_pairs(E, (const uint64_t *)G.ckey, G.ckey2, (const uint32_t *)G.cidx, G.cidx2, n, 64, "gi", s);
  if (g_prof_env) {
    HC(hipMemsetAsync(G.sec, 0, 256, s));
    HC(hipStreamSynchronize(s));
  }
  const double tl0 = g_prof_env ? now_ms() : 0.0;
  hipLaunchKernelGGL(k_gi_loop, dim3((unsigned)std::min<uint64_t>(n, 512)), dim3(kGhThreads), 0, s, a, G, c);
  HC(hipGetLastError());
  if (g_prof_env) {  // the components' loops: count, the largest by time, merges per microsecond
    HC(hipStreamSynchronize(s));
    const double tl1 = now_ms();
    uint32_t nc = 0;
    HC(hipMemcpy(&nc, G.scal, 4, hipMemcpyDeviceToHost));
    std::vector<uint32_t> sz(nc), mg(nc);
    std::vector<uint64_t> ck(nc);
    if (nc) {
      HC(hipMemcpy(sz.data(), G.c_size, 4 * nc, hipMemcpyDeviceToHost));
      HC(hipMemcpy(mg.data(), G.c_merges, 4 * nc, hipMemcpyDeviceToHost));
      HC(hipMemcpy(ck.data(), G.c_clk, 8 * nc, hipMemcpyDeviceToHost));
    }
    std::vector<uint32_t> ord(nc);
    for (uint32_t i = 0; i < nc; ++i) ord[i] = i;
    std::sort(ord.begin(), ord.end(), [&](uint32_t x, uint32_t y) { return ck[x] > ck[y]; });
    uint64_t tm = 0, tc = 0;
    for (uint32_t i = 0; i < nc; ++i) { tm += mg[i]; tc += ck[i]; }
    fprintf(stderr, "[rs-prof] giant %llu rows: %u components, %llu merges, loop %.1f ms (sum of component times %.1f ms)\n",
            (unsigned long long)n, nc, (unsigned long long)tm, tl1 - tl0, tc / 1e5);
    for (uint32_t i = 0; i < nc && i < 8; ++i)
      fprintf(stderr, "[rs-prof]   component rows %u merges %u: %.1f ms (%.2f us/merge)\n", sz[ord[i]], mg[ord[i]], ck[ord[i]] / 1e5,
              mg[ord[i]] ? ck[ord[i]] / 1e2 / mg[ord[i]] : 0.0);
    unsigned long long sec[32];
    HC(hipMemcpy(sec, G.sec, 256, hipMemcpyDeviceToHost));
    const double nm = (double)std::max<uint64_t>(tm, 1);
    fprintf(stderr, "[rs-prof]   loop clocks per merge, slot side: decide %.0f | to B' %.0f | combine+B %.0f | rebuild %.0f | row start %.0f | "
            "row end %.0f | serial %.0f\n", sec[0] / nm, sec[1] / nm, sec[2] / nm, sec[3] / nm, sec[4] / nm, sec[5] / nm, sec[6] / nm);
    fprintf(stderr, "[rs-prof]   loop clocks per merge, RHS side: decide %.0f | loads %.0f | find %.0f | product %.0f | insert %.0f | B' %.0f | "
            "B %.0f\n", sec[16] / nm, sec[24] / nm, sec[25] / nm, sec[26] / nm, sec[27] / nm, sec[17] / nm, sec[18] / nm);
  }
  dev_scan_u32(E, G.c_nsub, G.c_dsub, n, s, "gi");
  hipLaunchKernelGGL(k_gi_gather, dim3(gb), dim3(256), 0, s, a, G, c);
  HC(hipGetLastError());
  dev_scan_u32(E, G.lmark, G.lscan, n, s, "gi");
  hipLaunchKernelGGL(k_gi_scatter, dim3(gb), dim3(256), 0, s, a, G, c);
  hipLaunchKernelGGL(k_gi_fin, dim3(1), dim3(64), 0, s, a, G, c);
  HC(hipGetLastError());
}

// Runs linear_simplification (:275-325) for the rows of `view`; on return the per-slot arrays in
// the arena hold the substitutions (h_*) and leftovers (l_*), sub_of/deleted are updated.
// Work enqueued on the main stream while the head clusters are still being eliminated (given the
// head's cluster ids and the elimination arguments; the tail's substitutions are complete by then).
using HeadOverlap = std::function<void(const uint32_t *head_ids, uint64_t n_head, const ElimArgs &a)>;

static void run_linear_simplification(rs_engine *E, const DRows &view, int old_heur, ElimOut &eo, Pool &P,
                                      int *d_err, uint8_t *d_forb, int32_t *sub_of, uint8_t *deleted,
                                      const HeadOverlap *overlap = nullptr,
                                      const std::function<void()> *before_elim = nullptr,
                                      const uint8_t *need = nullptr) {
  double t0 = now_ms();
  if (E->fault_at == 1) {
    E->fault_at = 0;
    throw RsError(RS_E_INTERNAL, "injected fault (rs_engine_inject_fault)");
  }
  DevClusters D = gpu_clusters(E, view, old_heur, d_forb, eo);
  // keys-first rows: their values now (main stream; every elimination kernel is ordered after it)
  if (before_elim) (*before_elim)();
  double t1 = now_ms();
  E->stats.cluster_ms += t1 - t0;
  const uint64_t n_slots = D.n_slots, tot_nnz = D.tot_nnz;
  uint64_t n_big = D.n_big, n_small = D.n_small;
  uint32_t *d_perm = D.perm, *d_big = D.big, *d_small = D.small, *d_cid = D.cid;
  uint64_t *d_cl = D.cl_off;
  // sharded: this rank eliminates its snake share of each size-ordered list
  Comm *CM = E->comm.get();
  const int W = CM ? CM->world : 1, RK = CM ? CM->rank : 0;
  uint8_t *d_owner = nullptr;
  // Sharded: the head -- the kHeadLimit largest clusters, the critical path no exchange can shorten --
  // is eliminated by every rank (owner W, nothing exchanged); every other cluster belongs to one rank
  // (snake order over the size-ordered lists) and reaches the others through the exchange, which runs
  // as soon as the tail is done, while the head is still going.
  const uint64_t n_rep = std::min<uint64_t>(n_big, kHeadLimit);
  if (W > 1 && eo.n_clusters) {
    d_owner = E->A.get<uint8_t>("sh.owner", eo.n_clusters);
    const uint64_t n_tb = n_big - n_rep;
    if (n_rep) launch(E->st, k_fill_u8_ids, n_rep, (const uint32_t *)d_big, n_rep, (uint8_t)W, d_owner);
    if (n_tb) launch(E->st, k_shard_owner, n_tb, (const uint32_t *)(d_big + n_rep), n_tb, W, d_owner);
    if (n_small) launch(E->st, k_shard_owner, n_small, (const uint32_t *)d_small, n_small, W, d_owner);
    const uint64_t nb = snake_count(n_tb, W, RK), ns = snake_count(n_small, W, RK);
    uint32_t *bb = E->A.get<uint32_t>("sh.big", n_rep + nb), *ss = E->A.get<uint32_t>("sh.small", ns);
    if (n_rep) HC(hipMemcpyAsync(bb, d_big, 4 * n_rep, hipMemcpyDeviceToDevice, E->st));
    if (nb) launch(E->st, k_shard_pick, nb, (const uint32_t *)(d_big + n_rep), nb, W, RK, bb + n_rep);
    if (ns) launch(E->st, k_shard_pick, ns, (const uint32_t *)d_small, ns, W, RK, ss);
    d_big = bb;
    d_small = ss;
    n_big = n_rep + nb;
    n_small = ns;
  }
  // the substitution pool: 8x the cluster entries (an exhausted pool retries larger, and the size that
  // fitted is remembered) -- the pool is the engine's largest buffer: 24x took 20.8 GB on the 20 M-row
  // circuit, and eight in-process ranks did not fit one GPU
  uint64_t want = std::max<uint64_t>(std::max<uint64_t>(1 << 20, 8 * (tot_nnz + n_slots)), E->pool_want);
  {  // a giant cluster's fill-in: configs[1]'s 559 k-row cluster writes ~170 pool entries a row (its
     // substitutions' right-hand sides grow along its chains); reserve for it so the first attempt fits
    uint64_t giant_rows_sum = 0;
    for (uint64_t i = 0; i < std::min<uint64_t>(n_big, kHeadLimit) && i < D.top_keys.size(); ++i) {
      const uint64_t r = (0xffffffffull - (D.top_keys[i] >> 32)) & 0x7fffffffull;
      if (r >= kGiantRows && !D.order_free.count((uint32_t)(D.top_keys[i] & 0xffffffffull))) giant_rows_sum += r;
    }
    if (!getenv("RS_GI_NOPOOL")) want = std::max<uint64_t>(want, 192 * giant_rows_sum);
  }
  for (int attempt = 0; attempt < 8; ++attempt) {
    P = get_pool(E, want);
    Pool G{};  // sharded: every rank's exchanged entries (shard_exchange)
    bool exchanged = false;
    HC(hipMemsetAsync(P.top, 0, 8, E->st));
    HC(hipMemsetAsync(d_err, 0, 4, E->st));
    ElimArgs a;
    a.F = E->F;
    a.rows = view;
    a.perm = d_perm;
    a.cl_off = d_cl;
    a.n_clusters = eo.n_clusters;
    a.forb = d_forb;
    a.old_heur = old_heur;
    a.holder_idx = E->A.get<int32_t>("el.holder_idx", E->S);
    a.occ = E->A.get<int32_t>("el.occ", E->S);
    a.rep_pos = E->A.get<int32_t>("el.rep_pos", E->S);
    a.noov = E->A.get<int32_t>("el.noov", E->S);
    a.del = E->A.get<uint8_t>("el.del", E->S);
    a.h_sig = E->A.get<uint32_t>("el.h_sig", n_slots);
    a.h_coef = E->A.get<Fe>("el.h_coef", n_slots);
    a.h_off = E->A.get<uint64_t>("el.h_off", n_slots);
    a.h_len = E->A.get<uint32_t>("el.h_len", n_slots);
    a.tmp = E->A.get<uint32_t>("el.tmp", n_slots);
    a.ftmp = E->A.get<Fe>("el.ftmp", n_slots);
    a.dead = E->A.get<uint8_t>("el.dead", n_slots);
    a.order = E->A.get<uint32_t>("el.order", n_slots);
    a.l_off = E->A.get<uint64_t>("el.l_off", n_slots);
    a.l_len = E->A.get<uint32_t>("el.l_len", n_slots);
    a.n_sub = E->A.get<uint32_t>("el.n_sub", eo.n_clusters);
    a.n_left = E->A.get<uint32_t>("el.n_left", eo.n_clusters);
    a.sub_of = sub_of;
    a.deleted = deleted;
    a.pk = P.pk;
    a.pv = P.pv;
    a.pool_top = P.top;
    a.pool_cap = P.cap;
    a.err = d_err;
    // compositions sort unless the sort cannot take them (merging the short ones too was 45 % slower
    // on the metric circuit's tail, equal on templated)
    a.compose_sort = 1;
    // in-kernel algorithmic-byte counters: [0] k_eliminate, [1] / [2] the head's ordered loop /
    // inversion + normalisation + composition + emit, [3] / [4] the tail's, [7] the giant path
    a.bytes = E->A.get<unsigned long long>("el.bytes", 8);
    a.big_touch_off = E->A.get<uint64_t>("el.bt_off", std::max<uint64_t>(n_big, 1));
    a.big_touch_n = E->A.get<uint32_t>("el.bt_n", std::max<uint64_t>(n_big, 1));
    a.big_alive = E->A.get<uint32_t>("el.alive", std::max<uint64_t>(n_big, 1));
    a.row_off = E->A.get<uint64_t>("el.row_off", n_slots);
    a.row_len = E->A.get<uint32_t>("el.row_len", n_slots);

    a.prof = (getenv("RS_DEBUG") || getenv("RS_PROF")) && n_big ? E->A.get<unsigned long long>("el.prof", kProfWords * n_big) : nullptr;
    if (a.prof) HC(hipMemsetAsync(a.prof, 0, 8 * kProfWords * n_big, E->st));
    a.fclk = nullptr;
#ifdef RS_FINCLK
    a.fclk = E->A.get<unsigned long long>("el.fclk", 32);
    HC(hipMemsetAsync(a.fclk, 0, 8 * 32, E->st));
#endif
    a.bytes_main = a.bytes + 1;
    a.bytes_fin = a.bytes + 2;
    HC(hipMemsetAsync(a.bytes, 0, 64, E->st));
    // The largest clusters' prep -> main -> finish chain runs on a second stream: the elimination
    // time is the critical path of the largest cluster, and everything else overlaps it.
    const uint64_t n_head = std::min<uint64_t>(n_big, kHeadLimit), n_tail = n_big - n_head;
    a.wide = 1;       // the head's largest process_4 clusters go through the k_wide_* grid
    a.skip = nullptr;
    ElimArgs at = a;  // the tail's per-cluster side arrays follow the head's
    at.wide = 0;
    at.bytes_main = a.bytes + 3;
    at.bytes_fin = a.bytes + 4;
    at.big_touch_off += n_head;
    at.big_touch_n += n_head;
    at.big_alive += n_head;
    if (at.prof) at.prof += kProfWords * n_head;
    at.split = 0;
    // the head's giant clusters (rows >= kGiantRows, from the size keys the clustering read back): the
    // component loops of giant_loop.hpp on their own stream; k_big_spec skips them
    std::vector<uint64_t> giants;  // head positions
    for (uint64_t i = 0; i < n_head && i < D.top_keys.size(); ++i)
      if (((0xffffffffull - (D.top_keys[i] >> 32)) & 0x7fffffffull) >= kGiantRows &&
          !D.order_free.count((uint32_t)(D.top_keys[i] & 0xffffffffull)))  // (an order-free one has no loop rows)
        giants.push_back(i);
    uint64_t giant_rows = 0;
    for (uint64_t i : giants) giant_rows = std::max<uint64_t>(giant_rows, (0xffffffffull - (D.top_keys[i] >> 32)) & 0x7fffffffull);
    GiantArgs GA{};
    ElimArgs aspec = a;  // the speculative loop's arguments: the giants flagged in skip
    if (!giants.empty()) {
      GA = giant_buffers(E, giant_rows);
      uint8_t *gskip = E->A.get<uint8_t>("gi.skip", n_head);
      HC(hipMemsetAsync(gskip, 0, n_head, E->st));
      for (uint64_t i : giants) HC(hipMemsetAsync(gskip + i, 1, 1, E->st));
      aspec.skip = gskip;
    }
    ElimArgs ah = a;  // the head: split composition (k_big_finish -> k_compose_level per level -> k_big_emit)
    uint64_t *cf_next = nullptr;
    if (n_head) {
      const uint64_t cap_items = n_head * std::max<uint64_t>(E->stats.max_cluster, 1);
      ah.split = 1;
      ah.cf_items = E->A.get<uint64_t>("cf.items0", cap_items);
      cf_next = E->A.get<uint64_t>("cf.items1", cap_items);
      ah.cf_n = E->A.get<unsigned long long>("cf.cnt", 3);  // frontier counts, rotating over the levels
      ah.cf_deg = E->A.get<uint64_t>("cf.deg", n_head);
      ah.cf_dl = E->A.get<uint64_t>("cf.dl", n_head);
      ah.cf_done = E->A.get<uint32_t>("cf.done", n_head);
      ah.cf_big = E->A.get<uint64_t>("cf.big", cap_items);
      ah.cf_nbig = E->A.get<unsigned long long>("cf.nbig", 2);  // deferred counts, alternating
      HC(hipMemsetAsync(ah.cf_n, 0, 24, E->st));
      HC(hipMemsetAsync(ah.cf_nbig, 0, 16, E->st));
    }
    // the tail's composition: inside k_big_finish, one workgroup per cluster (level by level over the
    // GPU like the head's was slower on the metric circuit, 15 vs 6.6 ms)
    constexpr uint32_t kHeadLevels = 36;
    LevelLoop hl;
    int n_tgroups = 0;  // tail groups launched (their evt events are recorded)
    if (eo.n_clusters) {
      HC(hipEventRecord(E->ev2, E->st));
      if (n_head) {
        HC(hipStreamWaitEvent(E->st2, E->ev2, 0));
        const unsigned g = (unsigned)n_head;
        HC(hipEventRecord(E->evx[1], E->st2));
        {  // the largest process_4 clusters: occurrences / uniques over a 2-D grid first
          const dim3 g2(kWideX, g);
          const uint32_t *ids = d_big;
          hipLaunchKernelGGL(k_wide_alloc, dim3(g), dim3(256), 0, E->st2, a, ids, n_head);
          hipLaunchKernelGGL(k_wide_count, g2, dim3(256), 0, E->st2, a, ids, n_head);
          hipLaunchKernelGGL(k_wide_conv, g2, dim3(256), 0, E->st2, a, ids, n_head);
          hipLaunchKernelGGL(k_wide_uniq, g2, dim3(256), 0, E->st2, a, ids, n_head);
          hipLaunchKernelGGL(k_wide_remove, g2, dim3(256), 0, E->st2, a, ids, n_head);
          hipLaunchKernelGGL(k_wide_clear, g2, dim3(256), 0, E->st2, a, ids, n_head);
          HC(hipGetLastError());
        }
        hipLaunchKernelGGL(k_big_prep, dim3(g), dim3(256), 0, E->st2, a, (const uint32_t *)d_big, n_head);
        HC(hipGetLastError());
        HC(hipEventRecord(E->evx[2], E->st2));
        HC(hipEventRecord(E->evx[10], E->st2));
        if (!giants.empty()) {  // beside the speculative loop, joined before the head's inversion
          HC(hipStreamWaitEvent(E->stg, E->evx[10], 0));
          HC(hipMemsetAsync(GA.scal + 5, 0, 4, E->stg));  // the merge count over this run's giants
          HC(hipEventRecord(E->evgt[0], E->stg));
          ElimArgs ag = a;
          ag.bytes_main = a.bytes + 7;
          for (uint64_t i : giants) {
            GiantArgs G = GA;
            G.n = (0xffffffffull - (D.top_keys[i] >> 32)) & 0x7fffffffull;
            giant_launch(E, ag, G, D.top_keys[i] & 0xffffffffull, i);
          }
          HC(hipEventRecord(E->evgt[1], E->stg));
          HC(hipEventRecord(E->evg[1], E->stg));
        }
        // the ordered loop: twelve waves reduce rows speculatively against the LDS signal table and
        // commit in pop order (spec_loop.hpp).  12 vs 8 waves (three per SIMD at <= 168 VGPRs, 152 B of
        // spills): the metric circuit's largest cluster 12.9 -> 12.0 ms (the turns that wait for a row
        // still reducing: 4.5 -> 3.0 ms), templated 26.7 -> 28.1 ms (its chains conflict at distance 1)
        hipLaunchKernelGGL(k_big_spec<12>, dim3(g), dim3(768), 0, E->st2, aspec, (const uint32_t *)d_big, n_head);
        HC(hipGetLastError());
        HC(hipEventRecord(E->evx[3], E->st2));
        if (!giants.empty()) HC(hipStreamWaitEvent(E->st2, E->evg[1], 0));
        HC(hipEventRecord(E->evgt[2], E->st2));  // the head's composition chain starts (after the giants)
        // one inversion per head cluster
        hipLaunchKernelGGL(k_batch_inv_tree, dim3(g), dim3(256), 0, E->st2, a, (const uint32_t *)d_big, n_head);
        HC(hipGetLastError());
        hipLaunchKernelGGL(k_normalize, dim3(16, g), dim3(256), 0, E->st2, ah, (const uint32_t *)d_big, n_head);
        HC(hipGetLastError());
        hipLaunchKernelGGL(k_big_finish<8>, dim3(g), dim3(512), 0, E->st2, ah, (const uint32_t *)d_big, n_head, 0u);
        HC(hipGetLastError());
        // the Kahn levels and the emission follow once the rest is enqueued (the level loop waits)
      }
      // the main stream starts once the head's preparation is done: its short workgroups come after
      // the head's large-LDS ones have found CUs.  The small clusters first (k_eliminate, one lane
      // each), then the tail: the frames pass that follows waits for both.
      if (n_head) HC(hipStreamWaitEvent(E->st, E->evx[10], 0));
      // the small clusters (one lane each) on their own stream: nothing of the tail's chain reads them
      // (disjoint signals; the pool allocation is atomic), so the chain -- the first frames pass's and
      // hence the result stream's critical path -- starts at once; the main stream joins after it
      HC(hipEventRecord(E->ev4, E->st));
      HC(hipStreamWaitEvent(E->ste, E->ev4, 0));
      HC(hipEventRecord(E->ev_sm[0], E->ste));
      if (n_small) {
        uint64_t blocks = (n_small + 63) / 64;
        hipLaunchKernelGGL(k_eliminate, dim3((unsigned)std::min<uint64_t>(blocks, 1u << 20)), dim3(64), 0, E->ste, a,
                           (const uint32_t *)d_small, (uint64_t)n_small);
        HC(hipGetLastError());
      }
      HC(hipEventRecord(E->ev_sm[1], E->ste));
      HC(hipEventRecord(E->evx[5], E->st));
      n_tgroups = 0;
      if (n_tail) {
        // The tail in two groups on two streams: its kTailSplit largest clusters on the main stream
        // (their ordered loops are the tail's latency), the rest -- most of the composition work,
        // which fills the GPU -- beside them on the small clusters' stream, after k_eliminate.  One
        // launch per kernel over all of them made every finish wait for the largest loops.
        static const uint64_t split = getenv("RS_TAIL_SPLIT") ? strtoull(getenv("RS_TAIL_SPLIT"), nullptr, 10) : kTailSplit;
        const uint64_t n_t1 = n_tail > split + split / 4 ? split : n_tail, n_t2 = n_tail - n_t1;
        n_tgroups = n_t2 ? 2 : 1;
        auto tail_group = [&](hipStream_t s, ElimArgs g, const uint32_t *ids, uint64_t n, const char *cls_name, int grp) {
          const bool timed = grp == 0;
          hipEvent_t *ev = E->evt[grp];
          // grids: a few workgroups per CU, grid-stride over the clusters (largest first); the
          // per-lane pool chunks are bounded by the grid size
          const unsigned gb = (unsigned)std::min<uint64_t>(n, 2048), gm = (unsigned)std::min<uint64_t>(n, 8192);
          HC(hipEventRecord(ev[0], s));
          hipLaunchKernelGGL(k_big_prep, dim3(gb), dim3(256), 0, s, g, ids, n);
          HC(hipGetLastError());
          // process_3 clusters whose rows' pivots are all distinct: every row at once (k_p3_fast); the
          // ordered loop skips the clusters it took
          HC(hipMemsetAsync(g.skip, 0, n, s));
          hipLaunchKernelGGL(k_p3_fast, dim3(gb), dim3(256), 0, s, g, ids, n);
          HC(hipGetLastError());
          if (timed) HC(hipEventRecord(E->ev5, s));
          HC(hipEventRecord(ev[1], s));
          hipLaunchKernelGGL(k_big_main<256>, dim3(gm), dim3(64), 0, s, g, ids, n);
          HC(hipGetLastError());
          if (timed) HC(hipEventRecord(E->ev6, s));
          HC(hipEventRecord(ev[2], s));
          {  // the group's clusters flagged in cls, then one inversion per 64 slots across clusters
            uint8_t *cls = E->A.get<uint8_t>(cls_name, eo.n_clusters);
            HC(hipMemsetAsync(cls, 0, eo.n_clusters, s));
            launch(s, k_mark_u8, n, ids, n, cls);
            launch(s, k_batch_inv_flat, (n_slots + 63) / 64, g, (const uint32_t *)d_cid, (const uint8_t *)cls, n_slots);
          }
          HC(hipEventRecord(ev[3], s));
          // clusters of kFinWaveBelow rows and more by the workgroup, the rest one wave each (most
          // compose chains: the level latency, not the lanes, is their cost)
          hipLaunchKernelGGL(k_big_finish<4>, dim3(gb), dim3(256), 0, s, g, ids, n, kFinWaveBelow);
          HC(hipGetLastError());
          HC(hipEventRecord(ev[4], s));
        };
        uint8_t *skip = E->A.get<uint8_t>("el.skip", n_tail);
        at.skip = skip;
        tail_group(E->st, at, d_big + n_head, n_t1, "el.cls", 0);
        if (n_t2) {
          ElimArgs a2 = at;  // per-cluster side arrays indexed by the position in the launch's list
          a2.big_touch_off += n_t1;
          a2.big_touch_n += n_t1;
          a2.big_alive += n_t1;
          a2.skip = skip + n_t1;
          if (a2.prof) a2.prof += kProfWords * n_t1;
          tail_group(E->ste, a2, d_big + n_head + n_t1, n_t2, "el.cls2", 1);
        }
      }
      HC(hipEventRecord(E->ev_sm[2], E->ste));  // the main stream joins after the tail's second group
      // the head's first levels go in before the host waits for the tail's
      if (n_head) {
        hl.ah = ah;
        hl.ids = d_big;
        hl.s = E->st2;
        hl.cur = ah.cf_items;
        hl.nxt = cf_next;
        hl.n_slots = n_slots;
        hl.h = E->h_lvl;
        hl.ev = E->ev_lvl;
        if (overlap) hl.run(std::min(kHeadGpuLevels, kHeadLevels), false);
      }
      HC(hipEventRecord(E->ev7, E->st));
      HC(hipStreamWaitEvent(E->st, E->ev_sm[2], 0));  // the small clusters' and the tail's second group's, from here on
      if (D.join_pending) {  // the main stream reads the head clusters' orders from here on
        HC(hipStreamWaitEvent(E->st, E->evx[7], 0));
        D.join_pending = false;
      }
      // the head's composition: the first (wide) Kahn levels over the whole GPU, the rest in one
      // workgroup per cluster.  With a fixed level count nothing waits on the host, so all of it is
      // enqueued before the first frames pass (whose set-up synchronises with the main stream).
      auto finish_head = [&] {
        hl.run(kHeadGpuLevels, false);
        if (!hl.done) {
          hipLaunchKernelGGL(k_compose_rest<8>, dim3((unsigned)n_head), dim3(512), 0, E->st2, ah, (const uint32_t *)d_big,
                             (const uint64_t *)hl.cur, (const unsigned long long *)(ah.cf_n + hl.level % 3), n_head);
          HC(hipGetLastError());
        }
        hipLaunchKernelGGL(k_big_emit<8>, dim3((unsigned)n_head), dim3(512), 0, E->st2, ah, (const uint32_t *)d_big, n_head);
        HC(hipGetLastError());
        HC(hipEventRecord(E->evx[4], E->st2));
        if (g_prof_env) fprintf(stderr, "[rs-prof] head composition: %u level launches\n", hl.levels);
      };
      if (n_head) finish_head();
      // sharded: the clusters this rank owns are done (the main stream is past the tail): the exchange,
      // while the head -- every rank's own -- is still being eliminated
      if (W > 1) {
        int e0 = 0;
        HC(hipMemcpyAsync(&e0, d_err, 4, hipMemcpyDeviceToHost, E->st));
        HC(hipStreamSynchronize(E->st));
        exchanged = CM->max_u64((uint32_t)e0, E->st) == 0;  // else the attempt fails below, every rank alike
        if (exchanged) shard_exchange(E, a, D, d_owner, P, need, G);
      }
      if (n_head && overlap && (W == 1 || exchanged)) {
        ElimArgs ao = a;  // the frames read the substitutions of the clusters done: the gathered pool
        if (W > 1) {
          ao.pk = G.pk;
          ao.pv = G.pv;
        }
        (*overlap)(d_big, n_head, ao);
      }
      if (n_head) HC(hipStreamWaitEvent(E->st, E->evx[4], 0));
      HC(hipEventRecord(E->ev3, E->st));
    }
    // the verdict and the substitution / leftover totals in one read-back
    unsigned long long *d_sums = E->A.get<unsigned long long>("el.sums", 2);
    auto sum_counts = [&](unsigned long long *h) {
      HC(hipMemsetAsync(d_sums, 0, 16, E->st));
      if (eo.n_clusters) launch_capped(E->st, k_sum_counts, eo.n_clusters, 256, (const uint32_t *)a.n_sub, (const uint32_t *)a.n_left,
                                       eo.n_clusters, d_sums);
      HC(hipMemcpyAsync(h, d_sums, 16, hipMemcpyDeviceToHost, E->st));
    };
    unsigned long long sums[2] = {0, 0};
    int err = 0;
    sum_counts(sums);
    HC(hipMemcpyAsync(&err, d_err, 4, hipMemcpyDeviceToHost, E->st));
    HC(hipStreamSynchronize(E->st));
    if (W > 1) {  // every rank takes the same retry / failure decision
      const uint64_t mine = (uint32_t)err;
      err = 0;
      for (uint64_t x : CM->gather_u64(mine, E->st)) err |= (int)x;
    }
    if ((err & 8) && !(err & kGiErrBounds)) {  // pool exhausted (a bounds violation fails below instead)
      size_t fr_ = 0, tot_ = 0;
      (void)hipMemGetInfo(&fr_, &tot_);
      if (getenv("RS_PROF")) {
        unsigned long long used = 0;
        HC(hipMemcpy(&used, P.top, 8, hipMemcpyDeviceToHost));
        fprintf(stderr, "[rs-debug] pool exhausted: cap %llu entries, top %llu, attempt %d\n",
                (unsigned long long)want, used, attempt);
      }
      want = std::min<uint64_t>(want * 2, (uint64_t)(fr_ * 0.8) / 36 + want / 2);
      continue;
    }
    if (err) throw RsError(RS_E_INTERNAL, "elimination invariant violated (code " + std::to_string(err) + ")");
    E->pool_want = std::max(E->pool_want, want);  // the next run starts from a size that fitted
    if (g_prof_env) {
      unsigned long long used = 0;
      HC(hipMemcpy(&used, P.top, 8, hipMemcpyDeviceToHost));
      fprintf(stderr, "[rs-prof] pool: %llu of %llu entries (%.2f per cluster entry)\n", used, (unsigned long long)want,
                (double)used / (double)std::max<uint64_t>(1, tot_nnz + n_slots));
    }
    if (W > 1 && eo.n_clusters) {
      // the head's entries (this rank's local pool, with its own share's) go behind the gathered ones;
      // the replicated clusters' slots follow them, and the gathered pool is the round's pool from here
      unsigned long long top = 0;
      HC(hipMemcpyAsync(&top, P.top, 8, hipMemcpyDeviceToHost, E->st));
      HC(hipStreamSynchronize(E->st));
      const uint64_t base = G.cap;
      E->A.grow_keep<uint32_t>("pool.gk", base + top + 1, base, E->st, E->st);
      E->A.grow_keep<Fe>("pool.gv", base + top + 1, base, E->st, E->st);
      uint32_t *gk = E->A.get<uint32_t>("pool.gk", 1);
      Fe *gv = E->A.get<Fe>("pool.gv", 1);
      if (top) {
        HC(hipMemcpyAsync(gk + base, P.pk, 4 * top, hipMemcpyDeviceToDevice, E->st));
        HC(hipMemcpyAsync(gv + base, P.pv, 32 * top, hipMemcpyDeviceToDevice, E->st));
      }
      launch(E->st, k_shift_owned, n_slots, (const uint32_t *)D.cid, (const uint8_t *)d_owner, W, n_slots, base, a.h_off, a.l_off);
      P.pk = gk;
      P.pv = gv;
    }
    if (eo.n_clusters) {
      float ms = 0;
      unsigned long long by = 0;
      HC(hipEventElapsedTime(&ms, E->ev2, E->ev3));
      float msm = 0;
      HC(hipEventElapsedTime(&msm, E->ev_sm[0], E->ev_sm[1]));
      E->stats.elim_big_ms += ms;  // wall of the workgroup kernels (both streams; the small ones run beside)
      E->stats.elim_small_ms += msm;
      unsigned long long b5[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      rd(E, b5, a.bytes, 64);
      by = b5[0];
      E->stats.elim_kernel_ms += ms;
      E->stats.elim_kernel_launches++;
      E->stats.elim_bytes += by;
      E->stats.big_main_bytes += b5[1] + b5[3] + b5[7];
      E->stats.big_finish_bytes += b5[2] + b5[4];
      E->stats.head_main_bytes += b5[1];
      E->stats.tail_main_bytes += b5[3];
      E->stats.tail_fin_bytes += b5[4];
      E->stats.head_fin_bytes += b5[2];
      E->stats.small_bytes += b5[0];
      E->stats.giant_bytes += b5[7];
      if (D.timed) {
        float mc = 0;
        HC(hipEventElapsedTime(&mc, E->evc[0], E->evc[1]));
        E->stats.cluster_dev_ms += mc;
        E->stats.cluster_bytes += D.alg;
        E->stats.cluster_launches++;
      }
      if (n_small) {
        E->stats.small_ms += msm;
        E->stats.small_launches++;
      }
      if (!giants.empty()) {
        float mg = 0;
        HC(hipEventElapsedTime(&mg, E->evgt[0], E->evgt[1]));
        E->stats.giant_ms += mg;
        E->stats.giant_launches++;
        uint32_t nmg = 0;
        rd(E, &nmg, GA.scal + 5, 4);
        E->stats.giant_merges += nmg;
      }
      if (n_tail) {
        float m0 = 0, m1 = 0, m2 = 0;
        HC(hipEventElapsedTime(&m0, E->evx[5], E->ev5));
        HC(hipEventElapsedTime(&m1, E->ev5, E->ev6));
        HC(hipEventElapsedTime(&m2, E->ev6, E->ev7));
        E->stats.big_prep_ms += m0;
        E->stats.big_main_ms += m1;
        E->stats.big_finish_ms += m2;
        E->stats.big_launches++;
        for (int g = 0; g < n_tgroups; ++g) {  // each group on its own stream: kernel times add up
          float p0 = 0, p1 = 0, p2 = 0;
          HC(hipEventElapsedTime(&p0, E->evt[g][0], E->evt[g][1]));
          HC(hipEventElapsedTime(&p1, E->evt[g][1], E->evt[g][2]));
          HC(hipEventElapsedTime(&p2, E->evt[g][2], E->evt[g][4]));
          E->stats.prep_ms += p0;
          E->stats.tail_main_ms += p1;
          E->stats.tail_fin_ms += p2;
        }
        E->stats.prep_launches += n_tgroups;
        E->stats.tail_launches += n_tgroups;
        E->stats.tail_fin_launches += n_tgroups;
      }
      if (g_prof_env) {
        float t0 = 0, t1 = 0, t2 = 0, t3 = 0;
        if (n_tail) {
          HC(hipEventElapsedTime(&t0, E->evx[5], E->ev5));
          HC(hipEventElapsedTime(&t1, E->ev5, E->ev6));
          HC(hipEventElapsedTime(&t2, E->ev6, E->ev7));
        }
        HC(hipEventElapsedTime(&t3, E->ev_sm[0], E->ev_sm[1]));
        fprintf(stderr, "[rs-prof] tail(%llu): prep %.2f main %.2f inv+finish %.2f small %.2f", (unsigned long long)n_tail, t0, t1, t2, t3);
        if (n_head) {
          float h0 = 0, h1 = 0, h2 = 0;
          HC(hipEventElapsedTime(&h0, E->evx[1], E->evx[2]));
          HC(hipEventElapsedTime(&h1, E->evx[2], E->evx[3]));
          HC(hipEventElapsedTime(&h2, E->evx[3], E->evx[4]));
          fprintf(stderr, " | head(%llu): prep %.2f main %.2f inv+finish %.2f", (unsigned long long)n_head, h0, h1, h2);
        }
        fprintf(stderr, " | wall %.2f\n", ms);
      }
      if (n_head) {
        float m0 = 0, m1 = 0, m2 = 0;
        HC(hipEventElapsedTime(&m0, E->evx[1], E->evx[2]));
        HC(hipEventElapsedTime(&m1, E->evx[2], E->evx[3]));
        HC(hipEventElapsedTime(&m2, E->evx[3], E->evx[4]));
        E->stats.big_prep_ms += m0;
        E->stats.big_main_ms += m1;
        E->stats.big_finish_ms += m2;
        E->stats.big_launches++;
        E->stats.head_main_ms += m1;
        E->stats.head_launches++;
        float mf = 0;
        HC(hipEventElapsedTime(&mf, E->evgt[2], E->evx[4]));
        E->stats.head_fin_ms += mf;
        E->stats.head_fin_launches++;
      }
    }
    if (a.prof) {
      std::vector<unsigned long long> pf(kProfWords * n_big);
      HC(hipMemcpy(pf.data(), a.prof, 8 * pf.size(), hipMemcpyDeviceToHost));
      {  // head workgroups' start offsets (k_big_spec)
        unsigned long long t0m = ~0ull;
        for (uint64_t q = 0; q < std::min<uint64_t>(n_big, 16); ++q)
          if (pf[kProfWords * q + 22]) t0m = std::min(t0m, pf[kProfWords * q + 22]);
        fprintf(stderr, "[rs-prof] head starts (us after the first):");
        for (uint64_t q = 0; q < std::min<uint64_t>(n_big, 16); ++q)
          fprintf(stderr, " %llu:%.0f/%.0f", (unsigned long long)pf[kProfWords * q],
                  pf[kProfWords * q + 22] ? (pf[kProfWords * q + 22] - t0m) / 100.0 : -1.0, pf[kProfWords * q + 5] / 100.0);
        fprintf(stderr, "\n");
        // k_big_spec counters (spec_loop.hpp): rows, conflicts, rows on lane 0, merges kept / thrown
        // away, turn time (of it: exact passes), turns that waited for their row's speculation
        fprintf(stderr, "[rs-prof] head spec (rows conf serial merges redo | turn us exact us | late n us | wall us):");
        for (uint64_t q = 0; q < std::min<uint64_t>(n_big, 16); ++q) {
          const unsigned long long *P = &pf[kProfWords * q];
          fprintf(stderr, " [%llu %llu %llu %llu %llu | %.0f %.0f | %llu %.0f | %.0f]", P[2], P[8], P[9], P[10], P[11],
                  P[12] / 100.0, P[13] / 100.0, P[14], P[15] / 100.0, P[5] / 100.0);
        }
        fprintf(stderr, "\n");
      }
#ifdef RS_FINCLK
      if (a.fclk) {
        unsigned long long c[32];
        HC(hipMemcpy(c, a.fclk, sizeof c, hipMemcpyDeviceToHost));
        for (int t = 0; t < 2; ++t) {
          const unsigned long long *d = c + 16 * t;
          fprintf(stderr, "[rs-prof] tail finish clocks (%s, ms summed over waves): dag %.1f release %.1f | groups %.1f over %llu "
                  "substitutions (%llu sent on) | whole wave %.1f over %llu (rhs entries %llu, serial %llu) | levels %llu\n",
                  t ? "workgroup teams" : "wave teams", d[0] / 1e5, d[1] / 1e5, d[2] / 1e5, d[3], d[9], d[4] / 1e5, d[5], d[7],
                  d[6], d[10]);
        }
      }
#endif
      if (n_tail) {  // the tail's k_big_finish: per-cluster compose time, Kahn levels
        double tn = 0, tc = 0;
        std::map<int, uint64_t> lh;
        std::vector<uint64_t> tq;
        for (uint64_t q = n_head; q < n_big; ++q) {
          const unsigned long long *P = &pf[kProfWords * q];
          tn += P[6] / 100.0;
          tc += P[7] / 100.0;
          int b = 0;
          while ((1ull << b) < P[20] + 1) ++b;
          lh[b]++;
          tq.push_back(q);
        }
        std::sort(tq.begin(), tq.end(), [&](uint64_t x, uint64_t y) { return pf[kProfWords * x + 7] > pf[kProfWords * y + 7]; });
        fprintf(stderr, "[rs-prof] tail finish: summed normalize %.0f us compose %.0f us; levels (log2):", tn, tc);
        for (auto &kv : lh) fprintf(stderr, " %d:%llu", kv.first, (unsigned long long)kv.second);
        fprintf(stderr, "; slowest (rows subs levels us):");
        for (size_t i = 0; i < std::min<size_t>(tq.size(), 6); ++i) {
          const unsigned long long *P = &pf[kProfWords * tq[i]];
          fprintf(stderr, " [%llu %llu %llu %.0f]", P[0], P[1], P[20], P[7] / 100.0);
        }
        fprintf(stderr, "\n");
      }
      std::vector<uint64_t> ix(n_big);
      for (uint64_t i = 0; i < n_big; ++i) ix[i] = i;
      std::sort(ix.begin(), ix.end(), [&](uint64_t x, uint64_t y) {
        return pf[kProfWords * x + 4] + pf[kProfWords * x + 5] + pf[kProfWords * x + 6] + pf[kProfWords * x + 7] > pf[kProfWords * y + 4] + pf[kProfWords * y + 5] + pf[kProfWords * y + 6] + pf[kProfWords * y + 7];
      });
      double sum[4] = {0, 0, 0, 0};
      unsigned long long rows_all = 0, rows_main = 0, subs_all = 0, it_max = 0;
      for (uint64_t q = 0; q < n_big; ++q) {
        for (int j = 0; j < 4; ++j) sum[j] += pf[kProfWords * q + 4 + j] / 100.0;
        rows_all += pf[kProfWords * q]; subs_all += pf[kProfWords * q + 1]; rows_main += pf[kProfWords * q + 2];
        it_max = std::max(it_max, pf[kProfWords * q + 3]);
      }
      fprintf(stderr, "[rs-debug] big clusters: %llu rows %llu subs %llu sequential rows %llu max iters %llu; "
              "summed us: %.0f / %.0f / %.0f / %.0f\n", (unsigned long long)n_big, rows_all, subs_all, rows_main, it_max,
              sum[0], sum[1], sum[2], sum[3]);
      fprintf(stderr, "[rs-debug] big clusters: %llu (times in us: count+uniques / main / normalize / compose)\n", (unsigned long long)n_big);
      for (uint64_t q = 0; q < std::min<uint64_t>(n_big, 8); ++q) {
        unsigned long long *p = &pf[kProfWords * ix[q]];
        fprintf(stderr, "[rs-debug]   n=%llu m=%llu main_rows=%llu  prep %.1f / main %.1f / normalize %.1f / compose %.1f us"
                "  [kclocks: merges packed %llu (lanes %.1f) reg %llu lds %llu | row starts %.1f pivot %.1f holder %.1f "
                "merge %.1f (packed: loads %.1f search+product %.1f hand-off %.1f combine %.1f) new-sub %.1f us] levels %llu touched %llu\n",
                p[0], p[1], p[2], p[4] / 100.0, p[5] / 100.0, p[6] / 100.0, p[7] / 100.0,
                p[8], p[8] ? (double)p[12] / p[8] : 0.0, p[9], p[10], p[3] / 100.0, p[13] / 100.0, p[14] / 100.0,
                p[15] / 100.0, p[16] / 100.0, p[17] / 100.0, p[18] / 100.0, p[19] / 100.0, p[11] / 100.0, p[20], p[21]);
      }
    }
    if (W > 1 && eo.n_clusters) {  // the exchange rebuilt the per-cluster counts from every rank's records
      sum_counts(sums);
      HC(hipStreamSynchronize(E->st));
    }
    eo.n_sub = sums[0];
    eo.n_left = sums[1];
    E->stats.n_substitutions += eo.n_sub;
    E->stats.elim_ms += now_ms() - t1;
    E->A.defer = false;
    E->A.flush();  // every stream that could read an old block was synchronised above
    return;
  }
  throw RsError(RS_E_OOM_DEVICE, "substitution pool exhausted");
}

// The device lconst heap (see k_lc_count): rows appended in lconst order, C-only, Montgomery form.
struct LcHeap {
  uint64_t n = 0, top = 0;  // rows, entries
  DRows view(Arena &A) {
    DRows v{};
    v.n = n;
    v.off = A.get<uint64_t>("lc.off", 1);
    v.len = A.get<uint32_t>("lc.len", 1);
    v.key = A.get<uint32_t>("lc.key", 1);
    v.val = A.get<Fe>("lc.val", 1);
    return v;
  }
  // rows ids[0..m) (ids == nullptr: 0..m) of `src`, fixed (zeros dropped)
  void append(rs_engine *E, const DRows &src, const uint32_t *ids, uint64_t m) {
    if (!m) return;
    Arena &A = E->A;
    hipStream_t st = E->st;
    uint64_t *cnt = A.get<uint64_t>("lc.cnt", m), *pos = A.get<uint64_t>("lc.pos", m);
    launch(st, k_lc_count, m, src, ids, m, cnt);
    const uint64_t tot = excl_scan_u64(E, cnt, pos, m, "lc");
    // (a move waits for the copy stream too: a snapshot may be reading the heap there)
    A.grow_keep<uint64_t>("lc.off", n + m, n, E->stc, st);
    A.grow_keep<uint32_t>("lc.len", n + m, n, E->stc, st);
    A.grow_keep<uint32_t>("lc.key", top + tot, top, E->stc, st);
    A.grow_keep<Fe>("lc.val", top + tot, top, E->stc, st);
    launch(st, k_lc_copy, m, src, ids, m, (const uint64_t *)pos, top, n, view(A));
    n += m;
    top += tot;
  }
};

// a round's leftovers (cluster order, then push order) -> the lconst heap
static void collect_leftovers(rs_engine *E, const ElimOut &eo, const Pool &P, LcHeap &lc) {
  const uint64_t n_slots = eo.n_slots, nl = eo.n_left;
  if (!nl || !n_slots) return;
  Arena &A = E->A;
  uint64_t *f = A.get<uint64_t>("lc.lf", n_slots), *fp = A.get<uint64_t>("lc.lp", n_slots);
  uint32_t *slots = A.get<uint32_t>("lc.slots", nl);
  launch(E->st, k_left_flags, n_slots, (const uint32_t *)A.get<uint32_t>("cl.cid", 1), (const uint64_t *)A.get<uint64_t>("el.cl", 1),
         (const uint32_t *)A.get<uint32_t>("el.n_left", 1), n_slots, f);
  const uint64_t m = excl_scan_u64(E, f, fp, n_slots, "lcl");
  if (m != nl) throw RsError(RS_E_INTERNAL, "leftover count mismatch");
  launch(E->st, k_scatter_ids, n_slots, (const uint64_t *)f, (const uint64_t *)fp, n_slots, slots);
  DRows src{};
  src.n = n_slots;
  src.off = A.get<uint64_t>("el.l_off", 1);
  src.len = A.get<uint32_t>("el.l_len", 1);
  src.key = P.pk;
  src.val = P.pv;
  lc.append(E, src, slots, m);
}

// ---------------------------------------------------------------- substitution log
static void log_push(rs_engine *E, uint32_t from, const uint32_t *k, const uint64_t *v, uint64_t n) {
  E->log_from.push_back(from);
  E->log_key.insert(E->log_key.end(), k, k + n);
  E->log_val.insert(E->log_val.end(), v, v + 4 * n);
  E->log_ptr.push_back(E->log_key.size());
}
// linear_simplification's log_substitutions (:318-320) for the round just eliminated: the valid
// slots in cluster order, ascending `from` inside a cluster (one sort of (cluster, from) keys),
// then the canonical content of each normalised, non-overlapping right-hand side.
static void log_linear_round(rs_engine *E, const ElimOut &eo, const Pool &P) {
  Arena &A = E->A;
  hipStream_t st = E->st;
  const uint64_t n_slots = eo.n_slots;
  if (!n_slots) return;
  uint64_t *vf = A.get<uint64_t>("lg.vf", n_slots), *vp = A.get<uint64_t>("lg.vp", n_slots);
  const uint32_t *cid = A.get<uint32_t>("cl.cid", 1);
  launch(st, k_sub_valid, n_slots, cid, (const uint64_t *)A.get<uint64_t>("el.cl", 1),
         (const uint32_t *)A.get<uint32_t>("el.n_sub", 1), n_slots, vf);
  const uint64_t nU = excl_scan_u64(E, vf, vp, n_slots, "lgvf");
  if (!nU) return;
  uint64_t *uk = A.get<uint64_t>("lg.uk", nU), *uk2 = A.get<uint64_t>("lg.uk2", nU);
  uint32_t *uv = A.get<uint32_t>("lg.uv", nU), *U = A.get<uint32_t>("lg.U", nU);
  launch(st, k_sub_keys, n_slots, cid, (const uint64_t *)vf, (const uint64_t *)vp,
         (const uint32_t *)A.get<uint32_t>("el.h_sig", 1), n_slots, uk, uv);
  int cbits = 1;
  while (cbits < 32 && (1ull << cbits) <= eo.n_clusters) ++cbits;
  sort_pairs(E, (const uint64_t *)uk, uk2, (const uint32_t *)uv, U, nU, 32 + cbits, "lgus");
  std::vector<uint64_t> keys(nU), hoff(nU);
  std::vector<uint32_t> slots(nU), hlen(nU);
  uint64_t *d_off = A.get<uint64_t>("lg.off", nU);
  uint32_t *d_len = A.get<uint32_t>("lg.len", nU);
  launch(st, k_gather_u64, nU, (const uint64_t *)A.get<uint64_t>("el.h_off", 1), (const uint32_t *)U, d_off, nU);
  launch(st, k_gather_u32, nU, (const uint32_t *)A.get<uint32_t>("el.h_len", 1), (const uint32_t *)U, d_len, nU);
  HC(hipMemcpyAsync(keys.data(), uk2, 8 * nU, hipMemcpyDeviceToHost, st));
  HC(hipMemcpyAsync(hoff.data(), d_off, 8 * nU, hipMemcpyDeviceToHost, st));
  HC(hipMemcpyAsync(hlen.data(), d_len, 4 * nU, hipMemcpyDeviceToHost, st));
  HC(hipStreamSynchronize(st));
  std::vector<uint32_t> rk;
  std::vector<uint64_t> rv, rptr;
  fetch_pool_maps(E, hoff, hlen, P.pk, P.pv, rk, rv, rptr);
  for (uint64_t i = 0; i < nU; ++i)
    log_push(E, (uint32_t)keys[i], rk.data() + rptr[i], rv.data() + 4 * rptr[i], rptr[i + 1] - rptr[i]);
}

// ---------------------------------------------------------------- debug: host re-check of a round
static void d2h_row(rs_engine *E, const DRows &R, uint64_t r, std::vector<uint32_t> &k, std::vector<Fe> &v) {
  uint64_t off = 0;
  uint32_t len = 0;
  HC(hipMemcpy(&off, R.off + r, 8, hipMemcpyDeviceToHost));
  HC(hipMemcpy(&len, R.len + r, 4, hipMemcpyDeviceToHost));
  k.resize(len);
  v.resize(len);
  if (len) {
    HC(hipMemcpy(k.data(), R.key + off, 4 * len, hipMemcpyDeviceToHost));
    HC(hipMemcpy(v.data(), R.val + off, 32 * len, hipMemcpyDeviceToHost));
  }
}
static void debug_check_round(rs_engine *E, const RoundArgs &ra, uint64_t n, uint64_t) {
  HC(hipStreamSynchronize(E->st));
  const FieldP &F = E->F;
  std::vector<uint8_t> touched(n);
  HC(hipMemcpy(touched.data(), ra.touched, n, hipMemcpyDeviceToHost));
  int shown = 0;
  for (uint64_t r = 0; r < n && shown < 3; ++r) {
    if (!touched[r]) continue;
    std::vector<uint32_t> ik[3], ok[3];
    std::vector<Fe> iv[3], ov[3];
    const DRows *in[3] = {&ra.a, &ra.b, &ra.c}, *out[3] = {&ra.oa, &ra.ob, &ra.oc};
    std::map<uint32_t, Fe> exp[3];
    for (int q = 0; q < 3; ++q) {
      d2h_row(E, *in[q], r, ik[q], iv[q]);
      d2h_row(E, *out[q], r, ok[q], ov[q]);
      for (size_t i = 0; i < ik[q].size(); ++i) {
        int32_t s = -1;
        HC(hipMemcpy(&s, ra.sub_of + ik[q][i], 4, hipMemcpyDeviceToHost));
        if (s < 0) {
          Fe &x = exp[q][ik[q][i]];
          if (!exp[q].count(ik[q][i])) x = fe_zero();
          x = fadd(F, x, iv[q][i]);
          continue;
        }
        uint64_t ho = 0;
        uint32_t hl = 0;
        HC(hipMemcpy(&ho, ra.h_off + s, 8, hipMemcpyDeviceToHost));
        HC(hipMemcpy(&hl, ra.h_len + s, 4, hipMemcpyDeviceToHost));
        std::vector<uint32_t> hk(hl);
        std::vector<Fe> hv(hl);
        HC(hipMemcpy(hk.data(), ra.pk + ho, 4 * hl, hipMemcpyDeviceToHost));
        HC(hipMemcpy(hv.data(), ra.pv + ho, 32 * hl, hipMemcpyDeviceToHost));
        for (uint32_t j = 0; j < hl; ++j) {
          auto it = exp[q].find(hk[j]);
          Fe add = fmul(F, iv[q][i], hv[j]);
          if (it == exp[q].end()) exp[q][hk[j]] = add;
          else it->second = fadd(F, it->second, add);
        }
      }
    }
    // drop zeros (no fix re-check: report A/B/C expansions)
    bool bad = false;
    for (int q = 0; q < 3; ++q) {
      std::vector<std::pair<uint32_t, Fe>> e;
      for (auto &kv : exp[q])
        if (!fe_is_zero(kv.second)) e.push_back(kv);
      bool same = e.size() == ok[q].size();
      for (size_t i = 0; same && i < e.size(); ++i) same = e[i].first == ok[q][i] && fe_eq(e[i].second, ov[q][i]);
      if (!same) {
        bad = true;
        fprintf(stderr, "[rs-debug] row %llu part %d: in=%zu out=%zu expected=%zu\n", (unsigned long long)r, q,
                ik[q].size(), ok[q].size(), e.size());
        for (size_t i = 0; i < ik[q].size(); ++i) {
          Fe c = ffrom_mont(F, iv[q][i]);
          fprintf(stderr, "   in  %u:%llu\n", ik[q][i], (unsigned long long)c.l[0]);
        }
        for (size_t i = 0; i < ok[q].size(); ++i) {
          Fe c = ffrom_mont(F, ov[q][i]);
          fprintf(stderr, "   out %u:%llu\n", ok[q][i], (unsigned long long)c.l[0]);
        }
        for (auto &kv : e) {
          Fe c = ffrom_mont(F, kv.second);
          fprintf(stderr, "   exp %u:%llu\n", kv.first, (unsigned long long)c.l[0]);
        }
      }
    }
    if (bad) ++shown;
  }
}

// ---------------------------------------------------------------- the run
// the early region's D2H (see rs_engine::SnapJob) on its own thread, fed with jobs as snapshots are
// taken: each job waits for its gather, then goes in 32 MB chunks, two in flight (16 / 32 / 64 MB,
// best of 7, two rounds each: metric circuit 48.0-48.4 / 47.8 / 47.6-48.0 ms host -> host, templated
// 159.8-160.3 / 155.5-156.0 / 158.4 ms; chunks alternating over two streams -- two copy engines --
// 49.0 vs 49.6 ms on the metric circuit but 164.9 vs 157.6 ms templated: the run's own copies wait
// behind both engines)
static void snap_join(rs_engine *E) {
  {
    std::lock_guard<std::mutex> lk(E->snap_m);
    E->snap_closed = true;
  }
  E->snap_cv.notify_all();
  if (E->snap_thread.joinable()) E->snap_thread.join();
  E->snap_q.clear();
}
static void snap_start(rs_engine *E);
// queues a job, starting the thread when none runs (a run whose first snapshot was empty takes its
// first rows at a later one)
static void snap_push(rs_engine *E, const rs_engine::SnapJob &j) {
  snap_start(E);
  {
    std::lock_guard<std::mutex> lk(E->snap_m);
    E->snap_q.push_back(j);
  }
  E->snap_cv.notify_all();
}
static void snap_start(rs_engine *E) {
  if (E->snap_thread.joinable()) return;  // running: jobs are pushed to it
  E->snap_rc = 0;
  E->snap_closed = false;
  E->snap_thread = std::thread([E]() {
    // 128 MiB chunks, two in flight (host -> host medians 44.1-44.3 ms against 44.5-45.6 with 32 MiB
    // chunks, tools/r6_snap_ab.sh): small copies on the other streams are not held behind them
    // (tools/micro/copyq.hip), and fewer chunks leave fewer gaps between them on the link
    static const size_t chunk = (getenv("RS_SNAP_CHUNK_MB") ? strtoull(getenv("RS_SNAP_CHUNK_MB"), nullptr, 10) : 128ull) << 20;
    static const int depth = std::max(1, std::min(8, getenv("RS_SNAP_DEPTH") ? atoi(getenv("RS_SNAP_DEPTH")) : 2));
    if (hipSetDevice(E->device) != hipSuccess) { E->snap_rc = RS_E_HIP; return; }
    int k = 0;
    double prof_ms = 0.0, prof_b = 0.0;
    for (;;) {
      rs_engine::SnapJob j;
      {
        std::unique_lock<std::mutex> lk(E->snap_m);
        E->snap_cv.wait(lk, [E] { return E->snap_closed || !E->snap_q.empty(); });
        if (E->snap_q.empty()) break;  // closed and drained
        j = E->snap_q.front();
        E->snap_q.pop_front();
      }
      if (E->snap_rc) continue;
      // (an event a later snapshot records again is waited for at its newer point: still after this gather)
      if (hipEventSynchronize(j.ready) != hipSuccess) { E->snap_rc = RS_E_HIP; continue; }
      const double tj = g_prof_env ? now_ms() : 0.0;
      for (size_t o = 0; o < j.bytes; o += chunk, ++k) {
        const size_t n = std::min(chunk, j.bytes - o);
        if (k >= depth && hipEventSynchronize(E->ev_chunk[k % depth]) != hipSuccess) { E->snap_rc = RS_E_HIP; break; }
        if (hipMemcpyAsync((uint8_t *)j.dst + o, (const uint8_t *)j.src + o, n, hipMemcpyDeviceToHost, E->stx) != hipSuccess ||
            hipEventRecord(E->ev_chunk[k % depth], E->stx) != hipSuccess) {
          E->snap_rc = RS_E_HIP;
          break;
        }
      }
      if (g_prof_env) {  // RS_PROF: the link's rate while this job copies (the job is waited for)
        if (hipStreamSynchronize(E->stx) != hipSuccess) E->snap_rc = RS_E_HIP;
        prof_ms += now_ms() - tj;
        prof_b += j.bytes;
      }
    }
    if (hipStreamSynchronize(E->stx) != hipSuccess) E->snap_rc = RS_E_HIP;
    if (g_prof_env && prof_b)
      fprintf(stderr, "[rs-prof] result stream: %.1f MB in %.2f ms of copying (%.1f GB/s)\n", prof_b / 1e6, prof_ms,
              prof_b / 1e6 / prof_ms);
  });
}

static void *pin_get(rs_engine *E, int slot, size_t bytes) {
  rs_engine::Pin &b = E->pin[slot];
  if (b.cap < bytes) {
    const size_t cap = std::max(bytes, b.cap + b.cap / 4);
    if (b.p) HC(hipHostFree(b.p));
    b.p = nullptr;
    b.cap = 0;
    HC(hipHostMalloc(&b.p, cap, hipHostMallocDefault));
    b.cap = cap;
  }
  return b.p;
}

// the shared entry region of a sharded result: col of a, b, c (W x sh_cap[q] each), then val of a, b, c
static uint64_t sh_ent_bytes(rs_engine *E) {
  const uint64_t W = E->comm->world;
  return 36 * W * (E->sh_cap[0] + E->sh_cap[1] + E->sh_cap[2]);
}
static uint32_t *sh_col(rs_engine *E, int q) {
  const uint64_t W = E->comm->world;
  uint64_t off = 0;
  for (int p = 0; p < q; ++p) off += 4 * W * E->sh_cap[p];
  return (uint32_t *)((uint8_t *)E->sh_ent + off);
}
static uint64_t *sh_val(rs_engine *E, int q) {
  const uint64_t W = E->comm->world;
  uint64_t off = 4 * W * (E->sh_cap[0] + E->sh_cap[1] + E->sh_cap[2]);
  for (int p = 0; p < q; ++p) off += 32 * W * E->sh_cap[p];
  return (uint64_t *)((uint8_t *)E->sh_ent + off);
}

// The compact CSR of the result on the device (out.{a,b,c}.{ptr,col,val}): built by every run that
// does not stream, and on demand (rs_engine_fetch, the .r1cs writer) after one that does.
static void ensure_csr(rs_engine *E) {
  if (E->csr_ready) return;
  Arena &A = E->A;
  if (A.gen != E->fin_gen) throw RsError(RS_E_INTERNAL, "result views are stale: a buffer moved after the run");
  hipStream_t st = E->st;
  const char *nm[3] = {"out.a", "out.b", "out.c"};
  const uint64_t n_keep = E->fin_keep, n_out = E->out_n_dev;
  for (int q = 0; q < 3; ++q) {
    const uint64_t tot = E->out_nnz[q];
    const uint64_t *ptr = A.get<uint64_t>(std::string(nm[q]) + ".ptr", n_out + 1);
    uint32_t *col = A.get<uint32_t>(std::string(nm[q]) + ".col", tot);
    uint64_t *val = A.get<uint64_t>(std::string(nm[q]) + ".val", 4 * tot);
    E->kg[2].run(st, 24 * n_out + 72 * tot, [&] {  // kg[2]: 72 B an entry, the row's id / extent / ptr
      if (n_keep) launch(st, k_gather_rows, n_keep, E->F, E->fin_parts[q], E->fin_keep_ids, n_keep, ptr, col, val);
      for (int x = 0; x < 2; ++x) {
        const uint64_t o = n_keep + (x ? E->fin_xn[0] : 0);
        if (E->fin_xn[x]) launch(st, k_gather_rows, E->fin_xn[x], E->F, E->fin_xq[x][q], E->fin_x_ids[x], E->fin_xn[x], ptr + o, col, val);
      }
    });
  }
  E->csr_ready = true;
}

static void engine_run(rs_engine *E, const rs_flags *fl) {
  const uint64_t S = E->S;
  hipStream_t st = E->st;
  E->stats = rs_stats{};
  E->stats.world = E->comm ? (uint64_t)E->comm->world : 1;
  for (int g = 1; g < 3; ++g) {  // (kg[0]: the load's checks, recorded before the run)
    E->kg[g].n = 0;
    E->kg[g].bytes = 0;
  }
  if (E->A.defer || !E->A.graveyard.empty()) {  // an exchange a failed run left mid-way: its deferred frees
    for (hipStream_t q : {E->st, E->st2, E->stc, E->ste, E->stg})  // (nothing still reads them)
      if (q) (void)hipStreamSynchronize(q);
    E->A.defer = false;
    E->A.flush();
  }
  double T0 = now_ms();
  bool apply_linear = !fl->flag_s;
  uint64_t no_rounds = fl->no_rounds;
  Arena &A = E->A;
  int *d_err = A.get<int>("err", 1);
  HC(hipMemsetAsync(d_err, 0, 4, st));

  // forbidden bitmap, deleted, scratch defaults
  uint8_t *d_forb = A.get<uint8_t>("forb", S);
  uint8_t *d_deleted = A.get<uint8_t>("deleted", S);
  HC(hipMemsetAsync(d_forb, 0, S, st));
  HC(hipMemsetAsync(d_deleted, 0, S, st));
  {
    uint32_t *d_fl = A.get<uint32_t>("forb.list", E->forbidden.size());
    h2d(E, d_fl, E->forbidden.data(), 4 * E->forbidden.size());
    launch(st, k_mark_list, E->forbidden.size(), (const uint32_t *)d_fl, (uint64_t)E->forbidden.size(), d_forb);
  }
  for (const char *nm : {"el.holder_idx", "el.occ", "el.noov", "el.rep_pos"})
    HC(hipMemsetAsync(A.get<int32_t>(nm, S), 0xff, 4 * S, st));
  HC(hipMemsetAsync(A.get<uint8_t>("el.del", S), 0, S, st));
  int32_t *sub_of = A.get<int32_t>("sub_of", S);
  HC(hipMemsetAsync(sub_of, 0xff, 4 * S, st));

  LcHeap lc;  // lconst (device)
  snap_join(E);
  E->snap_on = false;
  E->lc_snap_n = 0;
  E->csr_ready = false;
  E->log_on = fl->emit_substitution_log != 0;
  E->log_from.clear();
  E->log_key.clear();
  E->log_val.clear();
  E->log_ptr.assign(1, 0);

  // ======================= eq_simplification (:198-251) + renaming of linear / cons_eq rows
  load_wait(E, 0);
  int32_t *eq_rep = A.get<int32_t>("eq_rep", S);
  HC(hipMemsetAsync(eq_rep, 0xff, 4 * S, st));
  {
    uint32_t *uf = A.get<uint32_t>("uf", S);
    uint32_t *cnt = A.get<uint32_t>("eq.cnt", S);
    int32_t *maxrow = A.get<int32_t>("eq.maxrow", S);
    uint32_t *minf = A.get<uint32_t>("eq.minf", S);
    uint32_t *minr = A.get<uint32_t>("eq.minr", S);
    uint8_t *in_eq = A.get<uint8_t>("eq.in", S);
    uint32_t *bf = A.get<uint32_t>("eq.bf", E->eq.n);
    uint32_t *bfn = A.get<uint32_t>("eq.bfn", 1);
    launch(st, k_iota_u32, S, uf, S);
    HC(hipMemsetAsync(cnt, 0, 4 * S, st));
    HC(hipMemsetAsync(maxrow, 0xff, 4 * S, st));
    HC(hipMemsetAsync(minf, 0xff, 4 * S, st));
    HC(hipMemsetAsync(minr, 0xff, 4 * S, st));
    HC(hipMemsetAsync(in_eq, 0, S, st));
    HC(hipMemsetAsync(bfn, 0, 4, st));
    if (E->eq.n) {
      launch(st, k_eq_union, E->eq.n, (const uint64_t *)E->eq.ptr, (const uint32_t *)E->eq.key, E->eq.n, uf, d_err);
      launch(st, k_eq_stats, E->eq.n, (const uint64_t *)E->eq.ptr, (const uint32_t *)E->eq.key, E->eq.n, uf,
             (const uint8_t *)d_forb, cnt, maxrow, minf, minr, in_eq);
      launch(st, k_eq_assign, E->eq.n, (const uint64_t *)E->eq.ptr, (const uint32_t *)E->eq.key, E->eq.n, uf,
             (const uint8_t *)d_forb, (const uint32_t *)minf, (const uint32_t *)minr, eq_rep, d_deleted, bf, bfn);
    }
    if (E->log_on && E->eq.n) {  // log_substitutions (:249)
      uint64_t *lk = A.get<uint64_t>("lg.eqk", S), *lk2 = A.get<uint64_t>("lg.eqk2", S);
      uint32_t *lr = A.get<uint32_t>("lg.eqr", S), *lr2 = A.get<uint32_t>("lg.eqr2", S);
      unsigned long long *ln = A.get<unsigned long long>("lg.eqn", 1);
      HC(hipMemsetAsync(ln, 0, 8, st));
      launch(st, k_eq_log_keys, S, (const int32_t *)eq_rep, uf, (const uint32_t *)cnt, (const int32_t *)maxrow, S, lk, lr, ln);
      unsigned long long nlog = 0;
      HC(hipMemcpyAsync(&nlog, ln, 8, hipMemcpyDeviceToHost, st));
      HC(hipStreamSynchronize(st));
      sort_pairs(E, (const uint64_t *)lk, lk2, (const uint32_t *)lr, lr2, nlog, 64, "lgeq");
      std::vector<uint64_t> hk(nlog);
      std::vector<uint32_t> hr(nlog);
      if (nlog) {
        HC(hipMemcpyAsync(hk.data(), lk2, 8 * nlog, hipMemcpyDeviceToHost, st));
        HC(hipMemcpyAsync(hr.data(), lr2, 4 * nlog, hipMemcpyDeviceToHost, st));
        HC(hipStreamSynchronize(st));
      }
      const uint64_t one[4] = {1, 0, 0, 0};
      for (uint64_t i = 0; i < nlog; ++i) log_push(E, (uint32_t)hk[i], &hr[i], one, 1);  // Substitution::new(Signal)
    }
    // eq cons (forbidden-only constraints), ordered by cluster index (= max row) then signal
    uint64_t nf = E->forbidden.size();
    uint32_t *fl_d = A.get<uint32_t>("forb.list", nf);
    uint32_t *g_root = A.get<uint32_t>("eq.g_root", nf);
    HC(hipMemsetAsync(g_root, 0, 4 * nf, st));
    launch(st, k_uf_roots, nf, uf, (const uint32_t *)fl_d, g_root, nf);
    uint32_t nbf = 0;
    HC(hipMemcpyAsync(&nbf, bfn, 4, hipMemcpyDeviceToHost, st));
    HC(hipStreamSynchronize(st));
    struct EqCon {  // a row of C: keys ascending, canonical values
      int64_t order;
      uint32_t f;
      std::vector<uint32_t> k;
      std::vector<uint64_t> v;
    };
    std::vector<EqCon> eqc;
    // per forbidden signal: in an eq cluster?  cluster size, min forbidden, max row (one gather)
    std::vector<uint32_t> finfo(4 * nf);
    if (nf) {
      uint32_t *d_fi = A.get<uint32_t>("eq.finfo", 4 * nf);
      launch(st, k_eq_forb_info, nf, (const uint32_t *)fl_d, nf, (const uint32_t *)g_root, (const uint8_t *)in_eq,
             (const uint32_t *)cnt, (const uint32_t *)minf, (const int32_t *)maxrow, d_fi);
      HC(hipMemcpyAsync(finfo.data(), d_fi, 16 * nf, hipMemcpyDeviceToHost, st));
      HC(hipStreamSynchronize(st));
    }
    for (uint64_t i = 0; i < nf; ++i) {
      uint32_t f = E->forbidden[i];
      if (!finfo[4 * i]) continue;
      uint32_t c = finfo[4 * i + 1], mf = finfo[4 * i + 2];
      int32_t mr = (int32_t)finfo[4 * i + 3];
      if (c <= 1 || f == mf) continue;
      // transform(sub(Signal f, Signal rh)) = {0: 0, rh: 1, f: -1}
      EqCon e;
      e.order = mr;
      e.f = f;
      uint64_t one[4] = {1, 0, 0, 0}, m1[4];
      memcpy(m1, E->prime, 32);
      m1[0] -= 1;
      e.k = {0};
      e.v = {0, 0, 0, 0};
      if (mf < f) {
        e.k.push_back(mf); e.v.insert(e.v.end(), one, one + 4);
        e.k.push_back(f); e.v.insert(e.v.end(), m1, m1 + 4);
      } else {
        e.k.push_back(f); e.v.insert(e.v.end(), m1, m1 + 4);
        e.k.push_back(mf); e.v.insert(e.v.end(), one, one + 4);
      }
      eqc.push_back(std::move(e));
    }
    if (nbf) {  // rows with both ends forbidden: kept as is when they are a cluster of their own
      std::vector<uint64_t> rec(11 * (uint64_t)nbf);
      uint64_t *d_rec = A.get<uint64_t>("eq.bfrec", 11 * (uint64_t)nbf);
      // staged load: the eq values were never uploaded; these rows take theirs from the host input
      launch(st, k_eq_bf_info, nbf, (const uint32_t *)bf, (uint64_t)nbf, (const uint64_t *)E->eq.ptr,
             (const uint32_t *)E->eq.key, E->hin ? (const Fe *)nullptr : (const Fe *)E->eq.val, (const uint32_t *)uf,
             (const uint32_t *)cnt, d_rec);
      HC(hipMemcpyAsync(rec.data(), d_rec, 88 * (uint64_t)nbf, hipMemcpyDeviceToHost, st));
      HC(hipStreamSynchronize(st));
      for (uint32_t q = 0; q < nbf; ++q) {
        uint64_t *x = &rec[11 * (uint64_t)q];
        if (x[2] != 1) continue;  // a single-constraint cluster with both ends forbidden: kept as is
        if (E->hin) {
          const rs_lc &H = E->hin->eq;
          const uint64_t p0 = H.ptr[x[0]];
          for (int t = 0; t < 4; ++t) { x[3 + t] = H.val[4 * p0 + t]; x[7 + t] = H.val[4 * (p0 + 1) + t]; }
          for (int e2 = 0; e2 < 2; ++e2) {
            const uint64_t *v = x + 3 + 4 * e2;
            if ((v[0] | v[1] | v[2] | v[3]) == 0 || geq4(v, E->prime))
              throw RsError(RS_E_INVALID, "eq block: zero or non-canonical value");
          }
          if ((uint32_t)x[1] > (uint32_t)(x[1] >> 32)) {  // the device sorted rows; these are as given
            x[1] = (x[1] << 32) | (x[1] >> 32);
            for (int t = 0; t < 4; ++t) std::swap(x[3 + t], x[7 + t]);
          }
        }
        EqCon e;
        e.order = (int64_t)x[0];
        e.f = 0;
        e.k = {(uint32_t)x[1], (uint32_t)(x[1] >> 32)};
        e.v.assign(x + 3, x + 11);
        eqc.push_back(std::move(e));
      }
    }
    std::sort(eqc.begin(), eqc.end(), [](const EqCon &x, const EqCon &y) {
      return x.order != y.order ? x.order < y.order : x.f < y.f;
    });
    if (!eqc.empty()) {  // to the device (canonical -> Montgomery), then into the lconst heap
      const uint64_t ne = eqc.size();
      std::vector<uint64_t> ho(ne);
      std::vector<uint32_t> hl(ne), hk;
      std::vector<uint64_t> hv;
      for (uint64_t i = 0; i < ne; ++i) {
        ho[i] = hk.size();
        hl[i] = (uint32_t)eqc[i].k.size();
        hk.insert(hk.end(), eqc[i].k.begin(), eqc[i].k.end());
        hv.insert(hv.end(), eqc[i].v.begin(), eqc[i].v.end());
      }
      DRows src{};
      src.n = ne;
      src.off = A.get<uint64_t>("lc.eo", ne);
      src.len = A.get<uint32_t>("lc.el", ne);
      src.key = A.get<uint32_t>("lc.ek", hk.size());
      src.val = A.get<Fe>("lc.ev", hk.size());
      h2d(E, src.off, ho.data(), 8 * ne);
      h2d(E, src.len, hl.data(), 4 * ne);
      h2d(E, src.key, hk.data(), 4 * hk.size());
      h2d(E, src.val, hv.data(), 8 * hv.size());
      launch(st, k_to_mont, hk.size(), E->F, (const Fe *)src.val, src.val, (uint64_t)hk.size());
      lc.append(E, src, nullptr, ne);
    }
  }

  // working copies (Montgomery): cons_eq (C), linear (C, one spare slot per row)
  DRows ce{}, lin{};
  ce.n = E->ce.n;
  ce.off = A.get<uint64_t>("ce.off", ce.n);
  ce.len = A.get<uint32_t>("ce.len", ce.n);
  ce.key = A.get<uint32_t>("ce.key", E->ce.nnz);
  ce.val = A.get<Fe>("ce.val", E->ce.nnz);
  // kg[1]'s algorithmic bytes: k_make_ragged reads the CSR and writes the ragged copy, 72 B an entry
  // and 20 a row; the linear rows' frames read what they rewrite (+ eq_rep / ce_has per entry)
  KGroup &kg1 = E->kg[1];
  if (ce.n)
    kg1.run(st, 72 * E->ce.nnz + 20 * ce.n + 8, [&] {
      launch(st, k_make_ragged, ce.n, E->F, (const uint64_t *)E->ce.ptr, (const uint32_t *)E->ce.key, (const Fe *)E->ce.val, ce.n,
             (uint64_t)0, ce.off, ce.len, ce.key, ce.val);
    });
  lin.n = E->lin.n;
  lin.off = A.get<uint64_t>("lin.off", lin.n);
  lin.len = A.get<uint32_t>("lin.len", lin.n);
  lin.key = A.get<uint32_t>("lin.key", E->lin.nnz + lin.n);
  lin.val = A.get<Fe>("lin.val", E->lin.nnz + lin.n);
  if (ce.n) launch(st, k_rename_rows, ce.n, E->F, ce, (const int32_t *)eq_rep);
  if (E->log_on && ce.n) {  // log_substitutions (:271), row order
    uint32_t *lsig = A.get<uint32_t>("lg.cesig", ce.n);
    uint64_t *lval = A.get<uint64_t>("lg.ceval", 4 * ce.n);
    launch(st, k_const_log, ce.n, E->F, ce, (const uint8_t *)d_forb, lsig, lval);
    std::vector<uint32_t> hs(ce.n);
    std::vector<uint64_t> hv(4 * ce.n);
    HC(hipMemcpyAsync(hs.data(), lsig, 4 * ce.n, hipMemcpyDeviceToHost, st));
    HC(hipMemcpyAsync(hv.data(), lval, 32 * ce.n, hipMemcpyDeviceToHost, st));
    HC(hipStreamSynchronize(st));
    const uint32_t k0 = 0;
    for (uint64_t r = 0; r < ce.n; ++r)
      if (hs[r] != RS_NONE) log_push(E, hs[r], &k0, &hv[4 * r], is_zero4(&hv[4 * r]) ? 0 : 1);
  }

  // ======================= constant_eq_simplification (:253-273)
  int32_t *ce_last = A.get<int32_t>("ce.last", S);
  uint8_t *ce_has = A.get<uint8_t>("ce.has", S);
  Fe *ce_val = A.get<Fe>("ce.val_s", S);
  HC(hipMemsetAsync(ce_last, 0xff, 4 * S, st));
  HC(hipMemsetAsync(ce_has, 0, S, st));
  {
    uint32_t *cl = A.get<uint32_t>("ce.cons", ce.n);
    uint32_t *cn = A.get<uint32_t>("ce.consn", 1);
    HC(hipMemsetAsync(cn, 0, 4, st));
    if (ce.n) {
      launch(st, k_const_pick, ce.n, ce, (const uint8_t *)d_forb, ce_last, d_deleted, cl, cn, d_err);
      launch(st, k_const_value, ce.n, E->F, ce, (const uint8_t *)d_forb, (const int32_t *)ce_last, ce_val, ce_has);
    }
    uint32_t ncons = 0;
    HC(hipMemcpyAsync(&ncons, cn, 4, hipMemcpyDeviceToHost, st));
    HC(hipStreamSynchronize(st));
    if (ncons) {  // the kept rows in row order (k_const_pick listed them in any order)
      uint32_t *sorted = A.get<uint32_t>("ce.cons_sorted", ncons);
      sort_keys(E, (const uint32_t *)cl, sorted, ncons, 32, "ce");
      lc.append(E, ce, sorted, ncons);
    }
  }
  // the linear rows: keys first when their values are still on the way (staged load, sorted rows,
  // no renaming collision) -- build_clusters needs keys only; the values follow in
  // `linear_values`, run just before the elimination reads them
  bool keys_first = false;
  load_wait(E, 1);
  uint8_t *lin_fixed = nullptr;
  if (E->staged && apply_linear && lin.n && !E->h_vflag[8]) {
    // rows that keys alone cannot settle (a renaming collision, or no non-constant key left) take
    // their values from the host input now (hundreds of rows out of millions, typically); the rest
    // wait for their values
    const uint64_t unc_cap = std::max<uint64_t>(1024, lin.n / 16);
    int *unc = A.get<int>("lin.unc", 1);
    uint32_t *unc_list = A.get<uint32_t>("lin.unc_list", unc_cap);
    lin_fixed = A.get<uint8_t>("lin.fixed", lin.n);
    HC(hipMemsetAsync(unc, 0, 4, st));
    HC(hipMemsetAsync(lin_fixed, 0, lin.n, st));
    kg1.run(st, 13 * E->lin.nnz + 20 * lin.n + 8, [&] {
      launch(st, k_lin_keyframes, lin.n, (const uint64_t *)E->lin.ptr, (const uint32_t *)E->lin.key, lin.n, lin,
             (const int32_t *)eq_rep, (const uint8_t *)ce_has, unc, unc_list, unc_cap);
    });
    int hu = 0;
    HC(hipMemcpyAsync(&hu, unc, 4, hipMemcpyDeviceToHost, st));
    HC(hipStreamSynchronize(st));
    keys_first = (uint64_t)hu <= unc_cap;
    if (keys_first && hu) {
      std::vector<uint32_t> rows(hu);
      HC(hipMemcpyAsync(rows.data(), unc_list, 4 * (uint64_t)hu, hipMemcpyDeviceToHost, st));
      HC(hipStreamSynchronize(st));
      const rs_lc &H = E->hin->linear;
      std::vector<uint64_t> hp(1, 0);
      std::vector<uint32_t> hk;
      std::vector<uint64_t> hv;
      for (uint32_t r : rows) {
        const uint64_t b = H.ptr[r], e = H.ptr[r + 1];
        hk.insert(hk.end(), H.col + b, H.col + e);
        hv.insert(hv.end(), H.val + 4 * b, H.val + 4 * e);
        hp.push_back(hk.size());
      }
      uint64_t *d_hp = A.get<uint64_t>("lin.fx_ptr", hp.size());
      uint32_t *d_hk = A.get<uint32_t>("lin.fx_key", std::max<size_t>(hk.size(), 1));
      Fe *d_hv = A.get<Fe>("lin.fx_val", std::max<size_t>(hk.size(), 1));
      uint32_t *d_rows = A.get<uint32_t>("lin.fx_rows", hu);
      h2d(E, d_hp, hp.data(), 8 * hp.size());
      h2d(E, d_hk, hk.data(), 4 * hk.size());
      h2d(E, d_hv, hv.data(), 8 * hv.size());
      h2d(E, d_rows, rows.data(), 4 * rows.size());
      launch(st, k_lin_fixrows, (uint64_t)hu, E->F, (const uint64_t *)d_hp, (const uint32_t *)d_hk, (const Fe *)d_hv,
             (const uint32_t *)d_rows, (uint64_t)hu, lin, (const int32_t *)eq_rep, (const uint8_t *)ce_has,
             (const Fe *)ce_val, lin_fixed);
    }
    if (g_prof_env) fprintf(stderr, "[rs-prof] keys-first: %d rows settled from host values\n", hu);
  }
  if (!keys_first) {
    load_wait(E, 2);
    if (lin.n) {
      kg1.run(st, 72 * E->lin.nnz + 20 * lin.n + 8 + 77 * E->lin.nnz + 16 * lin.n, [&] {
        launch(st, k_make_ragged, lin.n, E->F, (const uint64_t *)E->lin.ptr, (const uint32_t *)E->lin.key, (const Fe *)E->lin.val,
               lin.n, (uint64_t)1, lin.off, lin.len, lin.key, lin.val);
        launch(st, k_linear_frames12, lin.n, E->F, lin, (const int32_t *)eq_rep, (const uint8_t *)ce_has, (const Fe *)ce_val);
      });
    }
  }
  const std::function<void()> linear_values = [&]() {
    load_wait(E, 2);
    kg1.run(st, 77 * E->lin.nnz + 20 * lin.n + 8, [&] {
      launch(st, k_lin_valframes, lin.n, E->F, (const uint64_t *)E->lin.ptr, (const uint32_t *)E->lin.key, (const Fe *)E->lin.val,
             lin.n, lin, (const int32_t *)eq_rep, (const uint8_t *)ce_has, (const Fe *)ce_val, (const uint8_t *)lin_fixed);
    });
  };
  if (g_prof_env) fprintf(stderr, "[rs-prof] linear rows: %s\n", keys_first ? "keys first" : "keys + values");
  HC(hipStreamSynchronize(st));
  E->stats.eq_ms = now_ms() - T0;

  // ======================= obtain_and_simplify_non_linear (non_linear_utils.rs:6-31): setup
  const uint64_t n_nl = E->na.n;
  DRows ia{}, ib{}, ic{};
  auto mk_in = [&](rs_engine::Blk &B, DRows &R, const char *nm, hipStream_t ms) {
    R.n = B.n;
    R.off = A.get<uint64_t>(std::string(nm) + ".off", R.n);
    R.len = A.get<uint32_t>(std::string(nm) + ".len", R.n);
    R.key = A.get<uint32_t>(std::string(nm) + ".key", B.nnz);
    R.val = A.get<Fe>(std::string(nm) + ".val", B.nnz);
    if (R.n)
      kg1.run(ms, 72 * B.nnz + 20 * R.n + 8, [&] {
        launch(ms, k_make_ragged, R.n, E->F, (const uint64_t *)B.ptr, (const uint32_t *)B.key, (const Fe *)B.val, R.n, (uint64_t)0,
               R.off, R.len, R.key, R.val);
      });
  };
  // the non-linear blocks are staged where the frames first need them: their upload (group 2)
  // overlaps the clustering and elimination
  bool nl_staged = false;
  auto stage_nl = [&]() {
    if (nl_staged) return;
    load_wait(E, 3);
    // the conversion on the copy stream (in order after the blocks' upload and checks), beside what
    // the main stream still runs (the tail's finish): the frames wait for it there
    static const bool on_main = getenv("RS_NLC_MAIN") != nullptr;
    hipStream_t cs = on_main ? st : E->stc;
    mk_in(E->na, ia, "nla", cs);
    mk_in(E->nb, ib, "nlb", cs);
    mk_in(E->nc, ic, "nlc", cs);
    HC(hipEventRecord(E->ev_nlc, cs));
    HC(hipStreamWaitEvent(st, E->ev_nlc, 0));
    nl_staged = true;
  };
  // storage rows live in one growable heap of (key, value) entries, owned by the engine
  DRows sa{}, sb{}, sc{};
  uint64_t heap_top = 0;
  uint32_t *heap_k = E->heap_k;
  Fe *heap_v = E->heap_v;
  auto heap_reserve = [&](uint64_t need) {
    if (heap_top + need <= E->heap_cap && E->heap_k) return;
    // grows by a quarter (doubling left the 20 M-row circuit's heap at 12 GB for 6 GB of rows; eight
    // in-process ranks on one GPU did not fit)
    uint64_t ncap = std::max<uint64_t>(heap_top + need + (heap_top + need) / 16, E->heap_cap + E->heap_cap / 4);
    ncap = std::max<uint64_t>(ncap, 1 << 16);
    uint32_t *nk = nullptr;
    Fe *nv = nullptr;
    HC(hipStreamSynchronize(st));
    HC(hipMalloc((void **)&nk, 4 * ncap));
    HC(hipMalloc((void **)&nv, 32 * ncap));
    if (heap_top) {
      HC(hipMemcpyAsync(nk, E->heap_k, 4 * heap_top, hipMemcpyDeviceToDevice, st));
      HC(hipMemcpyAsync(nv, E->heap_v, 32 * heap_top, hipMemcpyDeviceToDevice, st));
      HC(hipStreamSynchronize(st));
    }
    if (E->snap_on) HC(hipStreamSynchronize(E->stc));  // the early gather reads the old heap
    if (E->heap_k) { HC(hipFree(E->heap_k)); HC(hipFree(E->heap_v)); }
    E->heap_k = heap_k = nk;
    E->heap_v = heap_v = nv;
    E->heap_cap = ncap;
  };
  unsigned long long *d_bytes = A.get<unsigned long long>("nl.bytes", 1);
  HC(hipMemsetAsync(d_bytes, 0, 8, st));
  int *d_fw_err = A.get<int>("fw.err", 1);  // k_frames_wave batch bounds (checked with the input checks)
  HC(hipMemsetAsync(d_fw_err, 0, 4, st));
  FrameArgs fr;
  fr.F = E->F;
  fr.eq_rep = eq_rep;
  fr.ce_has = ce_has;
  fr.ce_val = ce_val;
  fr.sub_of = sub_of;
  for (DRows *R : {&sa, &sb, &sc}) {
    R->n = n_nl;
  }
  sa.off = A.get<uint64_t>("st.a.off", n_nl);
  sa.len = A.get<uint32_t>("st.a.len", n_nl);
  sb.off = A.get<uint64_t>("st.b.off", n_nl);
  sb.len = A.get<uint32_t>("st.b.len", n_nl);
  sc.off = A.get<uint64_t>("st.c.off", n_nl);
  sc.len = A.get<uint32_t>("st.c.len", n_nl);
  uint64_t *ca = nullptr, *cb = nullptr, *cc = nullptr;
  U3 *cap3 = nullptr, *sc3 = nullptr;
  uint64_t *nl_late = nullptr, *nl_lpos = nullptr;
  uint8_t *hmark = nullptr;
  uint32_t *nl_lids = nullptr;
  uint64_t n_late = 0;
  if (n_nl) {
    ca = A.get<uint64_t>("nl.capa", n_nl); cb = A.get<uint64_t>("nl.capb", n_nl); cc = A.get<uint64_t>("nl.capc", n_nl);
    cap3 = A.get<U3>("nl.c3", n_nl); sc3 = A.get<U3>("nl.s3", n_nl);
  }
  // one pass of the frames over the non-linear rows ids[0, n) (phase: see NLArgs); the fill's
  // kernel time is read from (e0, e1) once the caller synchronises
  // streamed result (output.hpp): the non-linear rows round 1's substitution has finished and left
  // non-linear (storage rows) are gathered to the early region and copied to the host on the copy
  // stream while the run goes on.  late: rows a second frames pass still has to do (nullptr: none).
  uint8_t *so_early = nullptr;
  U3 *so_eoff = nullptr;
  bool fh_split = false;  // the last nl_phase ran in two halves (ev_fh)
  // hi_rows < n_nl: the first pass's first half only (snap_take_h2 takes the rest once it is done)
  auto snap_take = [&](const uint64_t *late, uint64_t hi_rows) {
    if (!E->stream_out || !n_nl) return;
    so_early = A.get<uint8_t>("so.early", n_nl);
    so_eoff = A.get<U3>("so.eoff", n_nl);
    U3 *elen = A.get<U3>("so.elen", n_nl);
    Comm *CM = E->comm.get();
    const bool shard = CM && CM->world > 1;
    // the gather reads copies of the selected rows' views: the second pass and later rounds re-point rows
    const DRows *src[3] = {&sa, &sb, &sc};
    const char *nm[3] = {"so.a", "so.b", "so.c"};
    DRows cp[3];
    ViewCopy vc;
    for (int q = 0; q < 3; ++q) {
      cp[q] = *src[q];
      cp[q].off = vc.off[q] = A.get<uint64_t>(std::string(nm[q]) + ".off", n_nl);
      cp[q].len = vc.len[q] = A.get<uint32_t>(std::string(nm[q]) + ".len", n_nl);
    }
    launch(st, k_snap_flags, n_nl, sa, sb, sc, late, n_nl, shard ? E->nl_lo : (uint64_t)0, shard ? E->nl_hi : hi_rows, so_early, elen,
           vc);
    const U3 et = excl_scan_u3(E, elen, so_eoff, n_nl, "so");
    // single engine: the lconst rows so far (final as they enter the heap) go behind the C part
    E->lc_snap_n = shard ? 0 : lc.n;
    E->lc_snap_base = et.c;
    const uint64_t lc_e = shard ? 0 : lc.top;
    const uint64_t ev[3] = {et.a, et.b, et.c + lc_e};
    E->sh_full = false;
    if (shard) {  // every rank's share of each part gets the same capacity in the shared region
      for (int q = 0; q < 3; ++q) E->sh_cap[q] = CM->max_u64(std::max<uint64_t>(ev[q] + ev[q] / 4 + 65536, E->sh_cap[q]), st);
      E->sh_ent = CM->shared_host(0, sh_ent_bytes(E), st);
      if (!E->sh_ent) {  // every rank alike (shared_host agrees): no stream; each rank fetches the whole result
        if (g_prof_env) fprintf(stderr, "[rs-prof] no shared host memory: unstreamed per-rank result\n");
        E->stream_out = false;
        return;
      }
    }
    HC(hipEventRecord(E->ev_snap0, st));
    HC(hipStreamWaitEvent(E->stc, E->ev_snap0, 0));
    for (int q = 0; q < 3; ++q) {
      E->snap_e[q] = ev[q];
      E->snap_hint[q] = std::max(E->snap_hint[q], ev[q]);
      // the device early region = the head of the layout's arrays; the late rows follow it
      // room for the second snapshot's rows too (the largest early region so far, else a margin)
      // (a first half: room for the whole pass, scaled by rows)
      const uint64_t est = hi_rows < n_nl && hi_rows ? (uint64_t)((double)ev[q] * n_nl / hi_rows) : ev[q];
      const uint64_t cap = std::max<uint64_t>(est + std::max<uint64_t>(est / 4, 1 << 16), E->snap_hint[q]);
      const std::string xn = std::string("out.") + "abc"[q];
      uint32_t *col = A.get<uint32_t>(xn + ".xcol", cap);
      uint64_t *val = A.get<uint64_t>(xn + ".xval", 4 * cap);
      // kg[2]'s algorithmic bytes: 72 an entry (key + value read, canonical key + value written) and
      // what a row's selection reads (its flag; its extent when selected)
      if (ev[q])
        E->kg[2].run(E->stc, 13 * n_nl + 72 * ev[q], [&] {
          launch(E->stc, k_snap_gather, n_nl, E->F, cp[q], (const uint8_t *)so_early, (const U3 *)so_eoff, q, n_nl, col, val,
                 (const uint64_t *)nullptr, (uint64_t)0);
        });
      if (q == 2 && lc_e) {
        const DRows lcv = lc.view(A);
        E->kg[2].run(E->stc, 72 * lc_e, [&] {
          launch(E->stc, k_lc_snap, lc_e, E->F, (const uint32_t *)lcv.key, (const Fe *)lcv.val, lc_e, col + et.c, val + 4 * et.c);
        });
      }
      void *hc = shard ? (void *)(sh_col(E, q) + CM->rank * E->sh_cap[q]) : pin_get(E, 3 + q, 4 * cap);
      void *hv = shard ? (void *)(sh_val(E, q) + 4 * CM->rank * E->sh_cap[q]) : pin_get(E, 6 + q, 32 * cap);
      E->snap_cap[q] = cap;
      E->snap_host[2 * q] = hc;
      E->snap_host[2 * q + 1] = hv;
      if (ev[q]) {  // a part's copies start once its own gather is done
        HC(hipEventRecord(E->ev_snapq[q], E->stc));
        snap_push(E, {hc, col, 4 * ev[q], E->ev_snapq[q]});
        snap_push(E, {hv, val, 32 * ev[q], E->ev_snapq[q]});
      }
    }
    HC(hipEventRecord(E->ev_snap, E->stc));
    E->snap_on = true;
    if (g_prof_env)
      fprintf(stderr, "[rs-prof] stream: early region %llu / %llu / %llu entries (%.1f MB)%s\n", (unsigned long long)ev[0],
              (unsigned long long)ev[1], (unsigned long long)ev[2], 36e-6 * (ev[0] + ev[1] + ev[2]), late ? " after the first pass" : "");
  };
  // The second snapshot (single engine): the rows of the second frames pass -- those touching the head
  // clusters -- that stayed storage rows go behind the first snapshot's, when they fit the regions
  // sized at the first (else they stay late), so they stream during the later rounds too.
  auto snap_take2 = [&]() {
    if (!E->snap_on || !nl_late || !n_late || (E->comm && E->comm->world > 1)) return;
    HC(hipStreamWaitEvent(st, E->ev_snap, 0));  // the first snapshot's gathers read the flags rewritten here
    U3 *elen = A.get<U3>("so.elen", n_nl), *eoff2 = A.get<U3>("so.eoff2", n_nl);
    const DRows *src[3] = {&sa, &sb, &sc};
    const char *nm[3] = {"so2.a", "so2.b", "so2.c"};
    DRows cp[3];  // copies of the selected rows' views (the rounds re-point rows)
    ViewCopy vc;
    for (int q = 0; q < 3; ++q) {
      cp[q] = *src[q];
      cp[q].off = vc.off[q] = A.get<uint64_t>(std::string(nm[q]) + ".off", n_nl);
      cp[q].len = vc.len[q] = A.get<uint32_t>(std::string(nm[q]) + ".len", n_nl);
    }
    launch(st, k_snap_lens2, n_nl, sa, sb, sc, (const uint64_t *)nl_late, n_nl, elen, vc);
    const U3 et = excl_scan_u3(E, elen, eoff2, n_nl, "so2");
    const uint64_t e2[3] = {et.a, et.b, et.c};
    for (int q = 0; q < 3; ++q) E->snap_hint[q] = std::max(E->snap_hint[q], E->snap_e[q] + e2[q]);
    for (int q = 0; q < 3; ++q)
      if (E->snap_e[q] + e2[q] > E->snap_cap[q]) return;  // no room this time (the hint grows the next run's)
    launch(st, k_snap_mark2, n_nl, (const uint64_t *)nl_late, (const U3 *)elen, (const U3 *)eoff2,
           U3{E->snap_e[0], E->snap_e[1], E->snap_e[2]}, n_nl, so_early, so_eoff);
    HC(hipEventRecord(E->ev_snap0, st));
    HC(hipStreamWaitEvent(E->stc, E->ev_snap0, 0));
    for (int q = 0; q < 3; ++q) {
      const uint64_t b = E->snap_e[q];
      const std::string xn = std::string("out.") + "abc"[q];
      uint32_t *col = A.get<uint32_t>(xn + ".xcol", 1);
      uint64_t *val = A.get<uint64_t>(xn + ".xval", 1);
      if (!e2[q]) continue;
      E->kg[2].run(E->stc, 21 * n_nl + 72 * e2[q], [&] {
        launch(E->stc, k_snap_gather, n_nl, E->F, cp[q], (const uint8_t *)so_early, (const U3 *)so_eoff, q, n_nl, col, val,
               (const uint64_t *)nl_late, (uint64_t)0);
      });
      HC(hipEventRecord(E->ev_snapq[3 + q], E->stc));
      snap_push(E, {(uint32_t *)E->snap_host[2 * q] + b, col + b, 4 * e2[q], E->ev_snapq[3 + q]});
      snap_push(E, {(uint64_t *)E->snap_host[2 * q + 1] + 4 * b, val + 4 * b, 32 * e2[q], E->ev_snapq[3 + q]});
      E->snap_e[q] = b + e2[q];
    }
    HC(hipEventRecord(E->ev_snap, E->stc));
    if (g_prof_env)
      fprintf(stderr, "[rs-prof] stream: second snapshot %llu / %llu / %llu entries (%.1f MB)\n", (unsigned long long)e2[0],
              (unsigned long long)e2[1], (unsigned long long)e2[2], 36e-6 * (e2[0] + e2[1] + e2[2]));
  };
  // split < n (phase 1): the frames of rows [0, split), `between` (the first half's snapshot), then the
  // rest; the kernel time excludes what runs between
  // The first pass's second half (single engine): its rows [h, n_nl) that are done and stayed storage
  // rows go behind the first half's in the regions sized at the first snapshot, when they fit (else
  // they stay late and the capacity hint grows).
  auto snap_take_h2 = [&](uint64_t h) {
    if (!E->snap_on || (E->comm && E->comm->world > 1)) return;
    HC(hipStreamWaitEvent(st, E->ev_snap, 0));  // the first half's gathers read the flags rewritten here
    U3 *elen = A.get<U3>("so.elenh", n_nl), *eoffh = A.get<U3>("so.eoffh", n_nl);
    const DRows *src[3] = {&sa, &sb, &sc};
    const char *nm[3] = {"soh.a", "soh.b", "soh.c"};
    DRows cp[3];  // copies of the selected rows' views (the second pass and the rounds re-point rows)
    ViewCopy vc;
    for (int q = 0; q < 3; ++q) {
      cp[q] = *src[q];
      cp[q].off = vc.off[q] = A.get<uint64_t>(std::string(nm[q]) + ".off", n_nl);
      cp[q].len = vc.len[q] = A.get<uint32_t>(std::string(nm[q]) + ".len", n_nl);
    }
    launch(st, k_snap_lens_rng, n_nl, sa, sb, sc, (const uint64_t *)nl_late, h, n_nl, n_nl, elen, vc);
    const U3 et = excl_scan_u3(E, elen, eoffh, n_nl, "soh");
    const uint64_t e2[3] = {et.a, et.b, et.c};
    for (int q = 0; q < 3; ++q) E->snap_hint[q] = std::max(E->snap_hint[q], E->snap_e[q] + e2[q]);
    for (int q = 0; q < 3; ++q)
      if (E->snap_e[q] + e2[q] > E->snap_cap[q]) return;
    launch(st, k_snap_mark_sel, n_nl, (const U3 *)elen, (const U3 *)eoffh, U3{E->snap_e[0], E->snap_e[1], E->snap_e[2]}, n_nl,
           so_early, so_eoff);
    HC(hipEventRecord(E->ev_snap0, st));
    HC(hipStreamWaitEvent(E->stc, E->ev_snap0, 0));
    for (int q = 0; q < 3; ++q) {
      const uint64_t b = E->snap_e[q];
      const std::string xn = std::string("out.") + "abc"[q];
      uint32_t *col = A.get<uint32_t>(xn + ".xcol", 1);
      uint64_t *val = A.get<uint64_t>(xn + ".xval", 1);
      if (!e2[q]) continue;
      E->kg[2].run(E->stc, 13 * (n_nl - h) + 72 * e2[q], [&] {
        launch(E->stc, k_snap_gather, n_nl - h, E->F, cp[q], (const uint8_t *)so_early, (const U3 *)so_eoff, q, n_nl, col, val,
               (const uint64_t *)nullptr, h);
      });
      HC(hipEventRecord(E->ev_snaph[q], E->stc));
      snap_push(E, {(uint32_t *)E->snap_host[2 * q] + b, col + b, 4 * e2[q], E->ev_snaph[q]});
      snap_push(E, {(uint64_t *)E->snap_host[2 * q + 1] + 4 * b, val + 4 * b, 32 * e2[q], E->ev_snaph[q]});
      E->snap_e[q] = b + e2[q];
    }
    HC(hipEventRecord(E->ev_snap, E->stc));
    if (g_prof_env)
      fprintf(stderr, "[rs-prof] stream: the first pass's second half %llu / %llu / %llu entries (%.1f MB)\n", (unsigned long long)e2[0],
              (unsigned long long)e2[1], (unsigned long long)e2[2], 36e-6 * (e2[0] + e2[1] + e2[2]));
  };
  auto nl_phase = [&](int phase, const uint32_t *ids, uint64_t n, hipEvent_t e0, hipEvent_t e1, uint64_t split = ~0ull,
                      const std::function<void()> &between = {}) {
    stage_nl();
    NLArgs a{};
    a.fr = fr;
    a.a = ia; a.b = ib; a.c = ic;
    a.cap_a = ca; a.cap_b = cb; a.cap_c = cc;
    a.bytes = d_bytes;
    a.ids = ids;
    a.n = n;
    a.phase = phase;
    a.hmark = hmark;
    a.late = nl_late;
    launch(st, k_nl_count, n, a);
    const bool lists = phase == 1 && n_nl;
    if (lists) {  // the skipped rows, listed for the second pass (their count comes back with the heap's)
      dev_scan_u64(E, nl_late, nl_lpos, n_nl, st, "nll");
      launch(st, k_scatter_ids, n_nl, (const uint64_t *)nl_late, (const uint64_t *)nl_lpos, n_nl, nl_lids);
    }
    launch(st, k_pack3, n, (const uint64_t *)ca, (const uint64_t *)cb, (const uint64_t *)cc, n, cap3);
    const U3 t3 = lists ? excl_scan_u3(E, cap3, sc3, n, "nl", nl_late + n_nl - 1, nl_lpos + n_nl - 1, &n_late)
                        : excl_scan_u3(E, cap3, sc3, n, "nl");
    if (g_prof_env) fprintf(stderr, "[rs-prof] nl phase %d: %llu rows, %llu heap entries\n", phase, (unsigned long long)n,
                            (unsigned long long)(t3.a + t3.b + t3.c));
    heap_reserve(t3.a + t3.b + t3.c);
    launch(st, k_set_offsets_u3, n, (const U3 *)sc3, heap_top, heap_top + t3.a, heap_top + t3.a + t3.b, n, sa.off, sb.off,
           sc.off, phase == 1 ? (const U3 *)cap3 : nullptr, ids);
    heap_top += t3.a + t3.b + t3.c;
    sa.key = sb.key = sc.key = heap_k;
    sa.val = sb.val = sc.val = heap_v;
    a.oa = sa; a.ob = sb; a.oc = sc;
    // whole waves on batches of rows (frames_wave.hpp); the rows too large for a batch, one lane each
    FrameWaveArgs w{};
    w.fr = fr;
    w.in[0] = ia; w.in[1] = ib; w.in[2] = ic;
    w.out[0] = sa; w.out[1] = sb; w.out[2] = sc;
    w.cap[0] = ca; w.cap[1] = cb; w.cap[2] = cc;
    w.ids = ids;
    w.n = n;
    w.late = phase == 1 ? nl_late : nullptr;
    w.big = A.get<uint32_t>(phase == 1 ? "nl.big1" : "nl.big2", n);
    w.n_big = A.get<unsigned>(phase == 1 ? "nl.nbig1" : "nl.nbig2", 1);
    w.err = d_fw_err;
    w.bytes = d_bytes;
    HC(hipMemsetAsync(w.n_big, 0, 4, st));
#ifdef RS_FWCLK
    w.clk = A.get<unsigned long long>(phase == 1 ? "fw.clk1" : "fw.clk2", 32 + 8 * 64);
    HC(hipMemsetAsync(w.clk, 0, 8 * (32 + 8 * 64), st));
#endif
    a.xlist = w.big;
    a.n_xlist = w.n_big;
    HC(hipEventRecord(e0, st));
    fh_split = split < n;
    if (fh_split) {
      w.n = split;
      launch_capped(st, k_frames_wave<0>, split, kFwBlocks, w);
      launch(st, k_nl_fill, n, a);  // the rows over a batch listed so far
      HC(hipEventRecord(E->ev_fh[0], st));
      between();
      HC(hipMemsetAsync(w.n_big, 0, 4, st));
      HC(hipEventRecord(E->ev_fh[1], st));
      w.x0 = split;
      w.n = n;
      launch_capped(st, k_frames_wave<0>, n - split, kFwBlocks, w);
    } else {
      launch_capped(st, k_frames_wave<0>, n, kFwBlocks, w);
    }
    launch(st, k_nl_fill, n, a);  // a grid for every row: the list may be long, idle lanes leave at once
    HC(hipEventRecord(e1, st));
    if (g_prof_env) {
      unsigned nb = 0;
      HC(hipMemcpyAsync(&nb, w.n_big, 4, hipMemcpyDeviceToHost, st));
      HC(hipStreamSynchronize(st));
      fprintf(stderr, "[rs-prof] nl phase %d: %u rows over a wave batch\n", phase, nb);
      if (w.clk) {
        unsigned long long c[32 + 8 * 64];
        HC(hipMemcpy(c, w.clk, sizeof c, hipMemcpyDeviceToHost));
        for (int q = 0; q < 0; ++q) {
          const unsigned long long *d = c + 32 + q * 64;
          fprintf(stderr, "[rs-prof] zero A row %llu: %llu entries:", d[0], d[1]);
          for (unsigned i = 0; i < d[1] && i < 6; ++i)
            fprintf(stderr, " (key/slot %llu kind %llu w %llu)", d[2 + i] >> 32, (d[2 + i] >> 16) & 0xff, d[2 + i] & 0xffff);
          fprintf(stderr, " | %llu terms:", d[8]);
          for (unsigned i = 0; i < d[8] && i < 24; ++i) fprintf(stderr, " %llu:%llx", d[9 + 2 * i] >> 32, d[10 + 2 * i]);
          fprintf(stderr, "\n");
        }
        fprintf(stderr, "[rs-prof] frames clocks (Mcycles summed over waves): groups %.1f entries %.1f terms %.1f rank %.1f "
                "heads %.1f emit %.1f rows %.1f plan %.1f | batches %llu, wave total %.1f over %llu waves\n",
                c[0] / 1e6, c[1] / 1e6, c[2] / 1e6, c[3] / 1e6, c[4] / 1e6, c[5] / 1e6, c[6] / 1e6, c[7] / 1e6, c[8],
                c[9] / 1e6, c[10]);
        fprintf(stderr, "[rs-prof] frames fallbacks: A const %llu, B const %llu | emit: loads %.1f values %.1f sync %.1f stores %.1f\n",
                c[12], c[13], c[16] / 1e6, c[17] / 1e6, c[18] / 1e6, c[19] / 1e6);
      }
    }
    E->stats.apply_kernel_launches++;
  };
  auto nl_ms = [&](hipEvent_t e0, hipEvent_t e1) {
    float ms = 0;
    HC(hipEventSynchronize(e1));
    if (fh_split) {  // the two halves, without the snapshot between them
      float m2 = 0;
      HC(hipEventElapsedTime(&ms, e0, E->ev_fh[0]));
      HC(hipEventElapsedTime(&m2, E->ev_fh[1], e1));
      ms += m2;
      fh_split = false;
    } else {
      HC(hipEventElapsedTime(&ms, e0, e1));
    }
    E->stats.apply_kernel_ms += ms;
  };
  // rows that touch none of the largest clusters go through the frames while those clusters are
  // still being eliminated (sharded: after the exchange of the clusters other than the head, which every
  // rank eliminates itself)
  bool nl_split = false;
  HeadOverlap overlap = [&](const uint32_t *ids, uint64_t n_head, const ElimArgs &ea) {
    hmark = A.get<uint8_t>("nl.hmark", E->S);
    nl_late = A.get<uint64_t>("nl.late", n_nl);
    nl_lpos = A.get<uint64_t>("nl.lpos", n_nl);
    nl_lids = A.get<uint32_t>("nl.lids", n_nl);
    HC(hipMemsetAsync(hmark, 0, E->S, st));
    hipLaunchKernelGGL(k_mark_head_keys, dim3(16, (unsigned)n_head), dim3(256), 0, st, ea.rows, (const uint32_t *)ea.perm,
                       (const uint64_t *)ea.cl_off, ids, hmark);
    HC(hipGetLastError());
    fr.h_off = ea.h_off; fr.h_len = ea.h_len; fr.pk = ea.pk; fr.pv = ea.pv;
    // the first pass in two halves with a snapshot after each (single engine, streamed): the result
    // stream starts after half the pass
    const bool halves = E->stream_out && !(E->comm && E->comm->world > 1) && n_nl >= (getenv("RS_HALVES_MIN") ? strtoull(getenv("RS_HALVES_MIN"), nullptr, 10) : (1ull << 20)) &&
                       !getenv("RS_NO_HALVES");
    const double frac = getenv("RS_HALF_FRAC") ? atof(getenv("RS_HALF_FRAC")) : 0.5;
    const uint64_t h = halves ? std::max<uint64_t>(1, std::min<uint64_t>(n_nl - 1, (uint64_t)(n_nl * frac))) : n_nl;
    nl_phase(1, nullptr, n_nl, E->evx[8], E->evx[9], h, [&] { snap_take(nl_late, h); });
    if (!halves) snap_take(nl_late, n_nl);
    else snap_take_h2(h);
    nl_split = true;
  };

  // ======================= linear round 1 (:544-578)
  ElimOut eo;
  Pool P = get_pool(E, 1 << 20);
  if (apply_linear) {
    // sharded: only the relevant substitutions' right-hand sides travel (the log needs them all)
    uint8_t *relevant = nullptr;
    if (E->comm && E->comm->world > 1 && !E->log_on) {
      relevant = A.get<uint8_t>("x.relevant", S);
      HC(hipMemsetAsync(relevant, 0, S, st));
      if (n_nl) {
        stage_nl();
        for (const DRows *R : {&ia, &ib, &ic})
          launch(st, k_mark_relevant, R->n, *R, (const int32_t *)eq_rep, (const uint8_t *)ce_has, relevant);
      }
    }
    if (E->comm && E->comm->world > 1) load_order_collectives(E);
    run_linear_simplification(E, lin, fl->use_old_heuristics, eo, P, d_err, d_forb, sub_of, d_deleted,
                              n_nl ? &overlap : nullptr, keys_first ? &linear_values : nullptr, relevant);
    if (E->log_on) log_linear_round(E, eo, P);
    collect_leftovers(E, eo, P, lc);
    E->stats.rounds++;
  } else {
    // --O1: the linear rows join lconst as they are after the eq / constant frames (:575-577)
    if (!keys_first) lc.append(E, lin, nullptr, lin.n);
    else throw RsError(RS_E_INTERNAL, "--O1 with keys-first linear rows");
  }

  // ======================= obtain_and_simplify_non_linear (non_linear_utils.rs:6-31)
  double Ts = now_ms();
  fr.h_off = A.get<uint64_t>("el.h_off", 1);
  fr.h_len = A.get<uint32_t>("el.h_len", 1);
  fr.pk = P.pk;
  fr.pv = P.pv;
  if (n_nl) {
    if (nl_split) nl_ms(E->evx[8], E->evx[9]);
    if (!nl_split) {
      nl_phase(0, nullptr, n_nl, E->ev0, E->ev1);
      snap_take(nullptr, n_nl);
      nl_ms(E->ev0, E->ev1);
    } else if (n_late) {
      nl_phase(2, nl_lids, n_late, E->ev0, E->ev1);
      snap_take2();
      nl_ms(E->ev0, E->ev1);
    }
  }
  unsigned long long bytes = 0;
  HC(hipMemcpyAsync(&bytes, d_bytes, 8, hipMemcpyDeviceToHost, st));
  // split: storage (still non-linear) vs with_linear, both in DFS order
  uint64_t n_st = 0, n_wl = 0;
  uint32_t *st_ids = A.get<uint32_t>("st.ids", n_nl), *wl_ids = A.get<uint32_t>("wl.ids", n_nl);
  if (n_nl) {
    uint64_t *fl_lin = A.get<uint64_t>("fl.lin", n_nl), *fl_nl = A.get<uint64_t>("fl.nl", n_nl);
    uint64_t *p_lin = A.get<uint64_t>("fl.plin", n_nl), *p_nl = A.get<uint64_t>("fl.pnl", n_nl);
    launch(st, k_flag_linear, n_nl, (const uint32_t *)sa.len, (const uint32_t *)sb.len, n_nl, fl_lin, fl_nl);
    n_wl = excl_scan_u64(E, fl_lin, p_lin, n_nl, "fl");
    n_st = excl_scan_u64(E, fl_nl, p_nl, n_nl, "fn");
    launch(st, k_scatter_ids, n_nl, (const uint64_t *)fl_lin, (const uint64_t *)p_lin, n_nl, wl_ids);
    launch(st, k_scatter_ids, n_nl, (const uint64_t *)fl_nl, (const uint64_t *)p_nl, n_nl, st_ids);
  }
  HC(hipStreamSynchronize(st));
  E->stats.apply_bytes += bytes;
  if (no_rounds > 0) no_rounds--;

  // storage view (compacted) and the non-linear signal map bitmap (:599-612)
  DRows ta_{}, tb_{}, tc_{};
  for (DRows *R : {&ta_, &tb_, &tc_}) { R->n = n_st; R->key = heap_k; R->val = heap_v; }
  ta_.off = A.get<uint64_t>("sv.a.off", n_st); ta_.len = A.get<uint32_t>("sv.a.len", n_st);
  tb_.off = A.get<uint64_t>("sv.b.off", n_st); tb_.len = A.get<uint32_t>("sv.b.len", n_st);
  tc_.off = A.get<uint64_t>("sv.c.off", n_st); tc_.len = A.get<uint32_t>("sv.c.len", n_st);
  if (n_st) {
    launch(st, k_view_rows, n_st, (const uint64_t *)sa.off, (const uint32_t *)sa.len, (const uint32_t *)st_ids, n_st, ta_.off, ta_.len);
    launch(st, k_view_rows, n_st, (const uint64_t *)sb.off, (const uint32_t *)sb.len, (const uint32_t *)st_ids, n_st, tb_.off, tb_.len);
    launch(st, k_view_rows, n_st, (const uint64_t *)sc.off, (const uint32_t *)sc.len, (const uint32_t *)st_ids, n_st, tc_.off, tc_.len);
  }
  uint8_t *nlmap = A.get<uint8_t>("nlmap", S);
  HC(hipMemsetAsync(nlmap, 0, S, st));
  if (n_st) {
    launch(st, k_mark_keys, n_st, ta_, nlmap);
    launch(st, k_mark_keys, n_st, tb_, nlmap);
    launch(st, k_mark_keys, n_st, tc_, nlmap);
  }
  // the current linear list: a C-only view
  DRows lv{};
  lv.n = n_wl;
  lv.key = heap_k;
  lv.val = heap_v;
  lv.off = A.get<uint64_t>("lv.off", n_wl);
  lv.len = A.get<uint32_t>("lv.len", n_wl);
  if (n_wl) launch(st, k_view_rows, n_wl, (const uint64_t *)sc.off, (const uint32_t *)sc.len, (const uint32_t *)wl_ids, n_wl, lv.off, lv.len);
  HC(hipStreamSynchronize(st));
  E->stats.subst_ms += now_ms() - Ts;
  E->stats.nl_ms += now_ms() - Ts;

  // ======================= rounds >= 2 (:613-646)
  bool apply_round = apply_linear && no_rounds > 0 && n_wl > 0;
  // streamed result: rows a later round touches are taken from the late region
  uint8_t *so_dirty = nullptr;
  if (so_early) {
    so_dirty = A.get<uint8_t>("so.dirty", n_st ? n_st : 1);
    if (n_st) HC(hipMemsetAsync(so_dirty, 0, n_st, st));
  }
  // A round's snapshot (single engine): the storage rows the round rewrote that stay storage rows go
  // behind the early region right away -- final unless a later round rewrites them again (dirty once
  // more: late at the end) -- so a round that rewrites most rows (the templated circuit's round 2)
  // streams them while the run goes on instead of after it.  Skipped when the regions sized at the first
  // snapshot cannot take them (the capacity hint grows for the next run).
  auto snap_round = [&](const uint8_t *touched, const int32_t *turn, const DRows &pa, const DRows &pb, const DRows &pc) {
    if (!so_dirty || !n_st || (E->comm && E->comm->world > 1)) return;
    // the earlier snapshots' gathers read the early flags / offsets this one rewrites, and its own buffers
    HC(hipStreamWaitEvent(st, E->ev_snap, 0));
    U3 *elen = A.get<U3>("so.rlen", n_st), *eoff3 = A.get<U3>("so.roff", n_st);
    const DRows *src[3] = {&pa, &pb, &pc};
    const char *nm[3] = {"sor.a", "sor.b", "sor.c"};
    DRows cp[3];  // copies of the selected rows' views (a later round re-points rows)
    ViewCopy vc;
    for (int q = 0; q < 3; ++q) {
      cp[q] = *src[q];
      cp[q].off = vc.off[q] = A.get<uint64_t>(std::string(nm[q]) + ".off", n_st);
      cp[q].len = vc.len[q] = A.get<uint32_t>(std::string(nm[q]) + ".len", n_st);
    }
    launch(st, k_snap_lens_round, n_st, pa, pb, pc, touched, turn, (const uint32_t *)st_ids, (const uint8_t *)so_early, n_st, elen, vc);
    const U3 et = excl_scan_u3(E, elen, eoff3, n_st, "sor");
    const uint64_t e3[3] = {et.a, et.b, et.c};
    if (!(e3[0] | e3[1] | e3[2])) return;
    for (int q = 0; q < 3; ++q) E->snap_hint[q] = std::max(E->snap_hint[q], E->snap_e[q] + e3[q]);
    for (int q = 0; q < 3; ++q)
      if (E->snap_e[q] + e3[q] > E->snap_cap[q]) return;
    launch(st, k_snap_mark_round, n_st, (const uint32_t *)st_ids, (const U3 *)elen, (const U3 *)eoff3,
           U3{E->snap_e[0], E->snap_e[1], E->snap_e[2]}, n_st, so_early, so_eoff, so_dirty);
    // the previous snapshot's gathers still read their view copies and elen / offsets (stc is in order)
    HC(hipEventRecord(E->ev_snap0, st));
    HC(hipStreamWaitEvent(E->stc, E->ev_snap0, 0));
    for (int q = 0; q < 3; ++q) {
      const uint64_t b = E->snap_e[q];
      const std::string xn = std::string("out.") + "abc"[q];
      uint32_t *col = A.get<uint32_t>(xn + ".xcol", 1);
      uint64_t *val = A.get<uint64_t>(xn + ".xval", 1);
      if (!e3[q]) continue;
      E->kg[2].run(E->stc, 24 * n_st + 72 * e3[q], [&] {
        launch(E->stc, k_snap_gather_st, n_st, E->F, cp[q], (const U3 *)elen, (const U3 *)eoff3, b, q, n_st, col, val);
      });
      HC(hipEventRecord(E->ev_snapq[3 + q], E->stc));
      snap_push(E, {(uint32_t *)E->snap_host[2 * q] + b, col + b, 4 * e3[q], E->ev_snapq[3 + q]});
      snap_push(E, {(uint64_t *)E->snap_host[2 * q + 1] + 4 * b, val + 4 * b, 32 * e3[q], E->ev_snapq[3 + q]});
      E->snap_e[q] = b + e3[q];
    }
    HC(hipEventRecord(E->ev_snap, E->stc));
    if (g_prof_env)
      fprintf(stderr, "[rs-prof] stream: round snapshot %llu / %llu / %llu entries (%.1f MB)\n", (unsigned long long)e3[0],
              (unsigned long long)e3[1], (unsigned long long)e3[2], 36e-6 * (e3[0] + e3[1] + e3[2]));
  };
  if (getenv("RS_DEBUG")) {
    HC(hipStreamSynchronize(st));
    fprintf(stderr, "[rs-debug] heap %p cap %llu top %llu n_st %llu n_wl %llu\n", (void *)heap_k,
            (unsigned long long)E->heap_cap, (unsigned long long)heap_top, (unsigned long long)n_st, (unsigned long long)n_wl);
    for (uint64_t r = 0; r < std::min<uint64_t>(n_st, 3); ++r) {
      uint64_t o = 0; uint32_t l = 0;
      HC(hipMemcpy(&o, tc_.off + r, 8, hipMemcpyDeviceToHost));
      HC(hipMemcpy(&l, tc_.len + r, 4, hipMemcpyDeviceToHost));
      std::vector<uint32_t> kk; std::vector<Fe> vv;
      d2h_row(E, tc_, r, kk, vv);
      fprintf(stderr, "[rs-debug]  st %llu C off %llu len %u:", (unsigned long long)r, (unsigned long long)o, l);
      for (size_t i = 0; i < kk.size(); ++i) fprintf(stderr, " %u:%llu", kk[i], (unsigned long long)ffrom_mont(E->F, vv[i]).l[0]);
      fprintf(stderr, "\n");
    }
  }
  if (apply_round) {
    // the non-linear signal map, kept on the host only for the signals a round substitutes:
    // initial lists (round-1 storage rows, ascending ids; built on the GPU on demand) + appends
    double Tm = now_ms();
    DRows ia0 = ta_, ib0 = tb_, ic0 = tc_;  // snapshot of the round-1 storage rows
    ia0.off = A.get<uint64_t>("m0.a.off", n_st); ia0.len = A.get<uint32_t>("m0.a.len", n_st);
    ib0.off = A.get<uint64_t>("m0.b.off", n_st); ib0.len = A.get<uint32_t>("m0.b.len", n_st);
    ic0.off = A.get<uint64_t>("m0.c.off", n_st); ic0.len = A.get<uint32_t>("m0.c.len", n_st);
    if (n_st) {
      HC(hipMemcpyAsync(ia0.off, ta_.off, 8 * n_st, hipMemcpyDeviceToDevice, st));
      HC(hipMemcpyAsync(ia0.len, ta_.len, 4 * n_st, hipMemcpyDeviceToDevice, st));
      HC(hipMemcpyAsync(ib0.off, tb_.off, 8 * n_st, hipMemcpyDeviceToDevice, st));
      HC(hipMemcpyAsync(ib0.len, tb_.len, 4 * n_st, hipMemcpyDeviceToDevice, st));
      HC(hipMemcpyAsync(ic0.off, tc_.off, 8 * n_st, hipMemcpyDeviceToDevice, st));
      HC(hipMemcpyAsync(ic0.len, tc_.len, 4 * n_st, hipMemcpyDeviceToDevice, st));
    }
    // the appended lists of the non-linear signal map, lazily (maplists.hpp)
    MapLists ML;
    auto &minit = ML.minit;  // initial lists, queried signals only
    uint8_t *qflag = A.get<uint8_t>("m.qflag", S);
    HC(hipMemsetAsync(qflag, 0, S, st));
    auto query_initial = [&](const std::vector<uint32_t> &sigs) {
      std::vector<uint32_t> q;
      for (uint32_t s : sigs)
        if (!minit.count(s)) { minit[s]; q.push_back(s); }
      if (q.empty() || n_st == 0) return;
      uint32_t *d_q = A.get<uint32_t>("m.q", q.size());
      h2d(E, d_q, q.data(), 4 * q.size());
      launch(st, k_mark_list, q.size(), (const uint32_t *)d_q, (uint64_t)q.size(), qflag);
      unsigned long long *d_cnt = A.get<unsigned long long>("m.cnt", 1);
      uint64_t cap = std::max<uint64_t>(4 * q.size(), 1 << 16);
      for (;;) {
        uint64_t *d_pairs = A.get<uint64_t>("m.pairs", cap);
        HC(hipMemsetAsync(d_cnt, 0, 8, st));
        for (DRows *R : {&ia0, &ib0, &ic0}) { R->key = heap_k; R->val = heap_v; }
        launch(st, k_emit_pairs, n_st, ia0, ib0, ic0, (const uint8_t *)qflag, d_pairs, d_cnt, cap);
        unsigned long long cnt = 0;
        HC(hipMemcpyAsync(&cnt, d_cnt, 8, hipMemcpyDeviceToHost, st));
        HC(hipStreamSynchronize(st));
        if (cnt > cap) { cap = cnt; continue; }
        std::vector<uint64_t> pairs(cnt);
        if (cnt) {
          HC(hipMemcpyAsync(pairs.data(), d_pairs, 8 * cnt, hipMemcpyDeviceToHost, st));
          HC(hipStreamSynchronize(st));
        }
        std::sort(pairs.begin(), pairs.end());
        for (uint64_t x : pairs) minit[(uint32_t)(x >> 32)].push_back((uint32_t)x);
        break;
      }
      launch(st, k_unmark_list, q.size(), (const uint32_t *)d_q, (uint64_t)q.size(), qflag);
    };
    E->stats.subst_ms += now_ms() - Tm;
    E->stats.map_ms += now_ms() - Tm;
    int32_t *rank_of = A.get<int32_t>("rank_of", S);
    HC(hipMemsetAsync(rank_of, 0xff, 4 * S, st));
    int32_t *r_sub_of = A.get<int32_t>("r.sub_of", S);
    HC(hipMemsetAsync(r_sub_of, 0xff, 4 * S, st));
    while (apply_round) {
      // linear_simplification over the current list
      ElimOut er;
      HC(hipMemsetAsync(r_sub_of, 0xff, 4 * S, st));
      run_linear_simplification(E, lv, fl->use_old_heuristics, er, P, d_err, d_forb, r_sub_of, d_deleted, nullptr, nullptr,
                                E->comm && E->comm->world > 1 && !E->log_on ? nlmap : nullptr);
      if (E->log_on) log_linear_round(E, er, P);
      E->stats.rounds++;
      Marks MK;
      MK.st = st;
      MK.mark("start");
      collect_leftovers(E, er, P, lc);
      MK.mark("leftovers");
      double Tr = now_ms();
      // ordered substitutions of the round: cluster order, ascending `from` -- one sort of the
      // (cluster, from) keys of the valid slots on the device; the host fetches the list only when
      // a row turned linear or another round follows
      const uint64_t n_slots = er.n_slots;
      uint64_t nU = 0;
      uint32_t *d_us = A.get<uint32_t>("r.us", 1), *d_U = A.get<uint32_t>("r.U", 1), *d_ulen = A.get<uint32_t>("r.ulen", 1);
      uint64_t *d_uoff = A.get<uint64_t>("r.uoff", 1);
      if (n_slots) {
        uint64_t *vf = A.get<uint64_t>("r.vf", n_slots), *vp = A.get<uint64_t>("r.vp", n_slots);
        launch(st, k_sub_valid, n_slots, (const uint32_t *)A.get<uint32_t>("cl.cid", 1), (const uint64_t *)A.get<uint64_t>("el.cl", 1),
               (const uint32_t *)A.get<uint32_t>("el.n_sub", 1), n_slots, vf);
        nU = excl_scan_u64(E, vf, vp, n_slots, "vf");
        if (nU) {
          uint64_t *uk = A.get<uint64_t>("r.uk", nU), *uk2 = A.get<uint64_t>("r.uk2", nU);
          uint32_t *uv = A.get<uint32_t>("r.uv", nU);
          d_U = A.get<uint32_t>("r.U", nU);
          d_us = A.get<uint32_t>("r.us", nU);
          d_uoff = A.get<uint64_t>("r.uoff", nU);
          d_ulen = A.get<uint32_t>("r.ulen", nU);
          launch(st, k_sub_keys, n_slots, (const uint32_t *)A.get<uint32_t>("cl.cid", 1), (const uint64_t *)vf,
                 (const uint64_t *)vp, (const uint32_t *)A.get<uint32_t>("el.h_sig", 1), n_slots, uk, uv);
          int cbits = 1;
          while (cbits < 32 && (1ull << cbits) <= er.n_clusters) ++cbits;
          sort_pairs(E, (const uint64_t *)uk, uk2, (const uint32_t *)uv, d_U, nU, 32 + cbits, "us");
          launch(st, k_sub_info, nU, (const uint64_t *)uk2, (const uint32_t *)d_U, (const uint64_t *)A.get<uint64_t>("el.h_off", 1),
                 (const uint32_t *)A.get<uint32_t>("el.h_len", 1), nU, d_us, d_uoff, d_ulen, rank_of);
        }
      }
      std::vector<uint32_t> usig;  // host copy of the ordered `from` list, fetched on demand
      auto need_usig = [&]() {
        if (usig.size() == nU) return;
        usig.resize(nU);
        HC(hipMemcpyAsync(usig.data(), d_us, 4 * nU, hipMemcpyDeviceToHost, st));
        HC(hipStreamSynchronize(st));
      };
      MK.mark("order");
      // apply to every storage row (apply_substitution_to_map, :345-396)
      std::vector<std::pair<uint64_t, uint32_t>> turned;  // (order key, storage id)
      if (n_st && nU) {
        RoundArgs ra{};
        ra.F = E->F;
        ra.a = ta_; ra.b = tb_; ra.c = tc_;
        uint64_t *ca = A.get<uint64_t>("r.capa", n_st), *cb = A.get<uint64_t>("r.capb", n_st), *cc = A.get<uint64_t>("r.capc", n_st);
        ra.cap_a = ca; ra.cap_b = cb; ra.cap_c = cc;
        ra.sub_of = r_sub_of;
        ra.rank_of = rank_of;
        ra.h_off = A.get<uint64_t>("el.h_off", 1);
        ra.h_len = A.get<uint32_t>("el.h_len", 1);
        ra.pk = P.pk;
        ra.pv = P.pv;
        ra.turn = A.get<int32_t>("r.turn", n_st);
        ra.touched = A.get<uint8_t>("r.touched", n_st);
        launch(st, k_round_count, n_st, ra);
        U3 *cap3 = A.get<U3>("r.c3", n_st), *sc3 = A.get<U3>("r.s3", n_st);
        launch(st, k_pack3, n_st, (const uint64_t *)ca, (const uint64_t *)cb, (const uint64_t *)cc, n_st, cap3);
        const U3 q3 = excl_scan_u3(E, cap3, sc3, n_st, "r");
        const uint64_t qt = q3.a + q3.b + q3.c;
        heap_reserve(qt);
        for (DRows *R : {&ta_, &tb_, &tc_, &lv}) { R->key = heap_k; R->val = heap_v; }
        ra.a = ta_; ra.b = tb_; ra.c = tc_;
        DRows oa = ta_, ob = tb_, oc = tc_;
        oa.off = A.get<uint64_t>("r.oa.off", n_st); oa.len = A.get<uint32_t>("r.oa.len", n_st);
        ob.off = A.get<uint64_t>("r.ob.off", n_st); ob.len = A.get<uint32_t>("r.ob.len", n_st);
        oc.off = A.get<uint64_t>("r.oc.off", n_st); oc.len = A.get<uint32_t>("r.oc.len", n_st);
        launch(st, k_set_offsets_u3, n_st, (const U3 *)sc3, heap_top, heap_top + q3.a, heap_top + q3.a + q3.b, n_st, oa.off,
               ob.off, oc.off, (const U3 *)nullptr, (const uint32_t *)nullptr);
        heap_top += qt;
        ra.c_base = heap_top - q3.c;  // row scratch = 2 * (its C offset - c_base)
        ra.oa = oa; ra.ob = ob; ra.oc = oc;
        ra.tmpk = A.get<uint32_t>("r.tmpk", 2 * (q3.c + 1));
        ra.tmpv = A.get<Fe>("r.tmpv", 2 * (q3.c + 1));
        MK.mark("count");
        {  // compact the touched rows: the fill's lanes all have work
          uint64_t *tfl = A.get<uint64_t>("r.tfl", n_st), *tfp = A.get<uint64_t>("r.tfp", n_st);
          uint32_t *tids = A.get<uint32_t>("r.touch_ids", n_st);
          launch(st, k_touch_flags, n_st, (const uint64_t *)cc, n_st, tfl);
          ra.n_ids = excl_scan_u64(E, tfl, tfp, n_st, "tfl");
          if (ra.n_ids) launch(st, k_scatter_ids, n_st, (const uint64_t *)tfl, (const uint64_t *)tfp, n_st, tids);
          ra.ids = tids;
          HC(hipMemsetAsync(ra.turn, 0xff, 4 * n_st, st));
          HC(hipMemsetAsync(ra.touched, 0, n_st, st));
        }
        ra.bytes = A.get<unsigned long long>("r.bytes", 1);
        HC(hipMemsetAsync(ra.bytes, 0, 8, st));
        if (ra.n_ids) {
          FrameWaveArgs w{};
          w.fr.F = E->F;
          w.fr.sub_of = r_sub_of;
          w.fr.h_off = ra.h_off; w.fr.h_len = ra.h_len; w.fr.pk = ra.pk; w.fr.pv = ra.pv;
          w.in[0] = ta_; w.in[1] = tb_; w.in[2] = tc_;
          w.out[0] = oa; w.out[1] = ob; w.out[2] = oc;
          w.cap[0] = ca; w.cap[1] = cb; w.cap[2] = cc;
          w.cap_by_row = 1;
          w.ids = ra.ids;
          w.n = ra.n_ids;
          w.big = A.get<uint32_t>("r.big", ra.n_ids);
          w.n_big = A.get<unsigned>("r.nbig", 2);
          w.round = 1;
          w.touched = ra.touched;
          w.turn_list = A.get<uint32_t>("r.turnlist", ra.n_ids);
          w.n_turn = w.n_big + 1;
          w.err = d_fw_err;
          w.bytes = ra.bytes;
          HC(hipMemsetAsync(w.n_big, 0, 8, st));
#ifdef RS_FWCLK
          w.clk = A.get<unsigned long long>("fw.clkr", 32);
          HC(hipMemsetAsync(w.clk, 0, 8 * 32, st));
#endif
          RoundArgs rb = ra, rt = ra;
          rb.rlist = w.big; rb.n_rlist = w.n_big;
          rt.rlist = w.turn_list; rt.n_rlist = w.n_turn;
          HC(hipEventRecord(E->ev0, st));
          launch_capped(st, k_frames_wave<1>, ra.n_ids, kFwBlocks, w);
          {  // the rows too long for a wave's LDS batch: A / B / C expanded by one device-wide sort
            unsigned nbig = 0;
            HC(hipMemcpyAsync(&nbig, w.n_big, 4, hipMemcpyDeviceToHost, st));
            HC(hipStreamSynchronize(st));
#ifdef RS_FWCLK
            if (g_prof_env) {
              unsigned long long c[32];
              HC(hipMemcpy(c, w.clk, sizeof c, hipMemcpyDeviceToHost));
              fprintf(stderr, "[rs-prof] round frames clocks (Mcycles summed over waves): groups %.1f entries %.1f terms %.1f "
                      "rank %.1f emit %.1f rows %.1f plan %.1f | batches %llu, wave total %.1f over %llu waves | emit: loads %.1f "
                      "values %.1f sync %.1f stores %.1f | %u rows over a batch of %llu\n", c[0] / 1e6, c[1] / 1e6, c[2] / 1e6,
                      c[3] / 1e6, c[5] / 1e6, c[6] / 1e6, c[7] / 1e6, c[8], c[9] / 1e6, c[10], c[16] / 1e6, c[17] / 1e6,
                      c[18] / 1e6, c[19] / 1e6, nbig, (unsigned long long)ra.n_ids);
            }
#endif
            if (nbig) {
              const uint64_t nseg = 3ull * nbig;
              uint64_t *xc = A.get<uint64_t>("x.cnt", nseg), *xo = A.get<uint64_t>("x.off", nseg + 1);
              launch(st, k_xrow_count, nseg, rb, nseg, xc);
              const uint64_t T = excl_scan_u64(E, xc, xo, nseg, "xrow");
              h2d(E, xo + nseg, &T, 8);
              if (T) {
                uint64_t *xk = A.get<uint64_t>("x.k", T), *xk2 = A.get<uint64_t>("x.k2", T);
                uint32_t *xi = A.get<uint32_t>("x.i", T), *xi2 = A.get<uint32_t>("x.i2", T);
                Fe *xv = A.get<Fe>("x.v", T);
                launch(st, k_xrow_expand, 64 * nseg, rb, nseg, (const uint64_t *)xo, xk, xv, xi);
                int sb = 1;
                while (sb < 32 && (1ull << sb) <= nseg) ++sb;
                sort_pairs(E, (const uint64_t *)xk, xk2, (const uint32_t *)xi, xi2, T, 32 + sb, "xrow");
                launch(st, k_xrow_combine, 64 * nseg, rb, nseg, (const uint64_t *)xo, (const uint64_t *)xk2,
                       (const uint32_t *)xi2, (const Fe *)xv);
              } else {
                launch(st, k_xrow_combine, 64 * nseg, rb, nseg, (const uint64_t *)xo, (const uint64_t *)nullptr,
                       (const uint32_t *)nullptr, (const Fe *)nullptr);
              }
              rb.pre_expanded = 1;
            }
          }
          launch(st, k_round_fill, ra.n_ids, rb);
          launch(st, k_round_turn, ra.n_ids, rt);
          HC(hipEventRecord(E->ev1, st));
          if (g_prof_env) {
            unsigned nb[2] = {0, 0};
            HC(hipMemcpyAsync(nb, w.n_big, 8, hipMemcpyDeviceToHost, st));
            HC(hipStreamSynchronize(st));
            fprintf(stderr, "[rs-prof] round: %llu rows, %u over a wave batch, %u turn\n", (unsigned long long)ra.n_ids, nb[0], nb[1]);
          }
          float fm = 0;
          unsigned long long fb = 0;
          HC(hipMemcpyAsync(&fb, ra.bytes, 8, hipMemcpyDeviceToHost, st));
          HC(hipEventSynchronize(E->ev1));
          HC(hipStreamSynchronize(st));
          HC(hipEventElapsedTime(&fm, E->ev0, E->ev1));
          E->stats.round_fill_ms += fm;
          E->stats.round_fill_bytes += fb;
          E->stats.round_fill_launches++;
        }
        MK.mark("fill");
        if (getenv("RS_DEBUG")) debug_check_round(E, ra, n_st, qt);
        launch(st, k_commit_round, n_st, (const uint8_t *)ra.touched, (const int32_t *)ra.turn, n_st, ta_, tb_, tc_, oa, ob, oc);
        if (so_dirty) launch(st, k_or_u8, n_st, (const uint8_t *)ra.touched, n_st, so_dirty);
        snap_round(ra.touched, ra.turn, ta_, tb_, tc_);
        // turned rows
        uint64_t *tf = A.get<uint64_t>("r.tf", n_st), *tp = A.get<uint64_t>("r.tp", n_st);
        launch(st, k_turn_flags, n_st, (const int32_t *)ra.turn, n_st, tf);
        uint64_t n_turn = excl_scan_u64(E, tf, tp, n_st, "tf");
        uint32_t *tids = A.get<uint32_t>("r.tids", n_turn);
        launch(st, k_scatter_ids, n_st, (const uint64_t *)tf, (const uint64_t *)tp, n_st, tids);
        std::vector<uint32_t> htids(n_turn);
        std::vector<int32_t> hturn(n_turn);  // turn value of each turned row (aligned with htids)
        if (n_turn) {
          int32_t *d_tt = A.get<int32_t>("r.tturn", n_turn);
          launch(st, k_gather_u32, n_turn, (const uint32_t *)ra.turn, (const uint32_t *)tids, (uint32_t *)d_tt, n_turn);
          HC(hipMemcpyAsync(htids.data(), tids, 4 * n_turn, hipMemcpyDeviceToHost, st));
          HC(hipMemcpyAsync(hturn.data(), d_tt, 4 * n_turn, hipMemcpyDeviceToHost, st));
          HC(hipStreamSynchronize(st));
          need_usig();
        }
        std::unordered_map<uint32_t, std::vector<uint32_t>> ext;  // appended lists of those signals
        {  // initial map lists of the turning substitutions' signals only
          double Tq = now_ms();
          std::vector<uint32_t> qs;
          for (uint64_t i = 0; i < n_turn; ++i) qs.push_back(usig[hturn[i]]);
          std::sort(qs.begin(), qs.end());
          qs.erase(std::unique(qs.begin(), qs.end()), qs.end());
          query_initial(qs);
          ext = ML.resolve(qs, query_initial);
          E->stats.map_ms += now_ms() - Tq;
        }
        // order key: (rank of the turning substitution, first position in map[from])
        for (uint64_t ti = 0; ti < n_turn; ++ti) {
          const uint32_t r = htids[ti];
          int32_t q = hturn[ti];
          uint32_t from = usig[q];
          uint64_t pos = UINT64_MAX;
          const std::vector<uint32_t> &L0 = minit[from];
          auto lb = std::lower_bound(L0.begin(), L0.end(), r);  // initial lists are ascending
          if (lb != L0.end() && *lb == r) pos = lb - L0.begin();
          if (pos == UINT64_MAX) {
            auto it = ext.find(from);
            if (it != ext.end())
              for (uint64_t t = 0; t < it->second.size(); ++t)
                if (it->second[t] == r) { pos = L0.size() + t; break; }
          }
          if (pos == UINT64_MAX) throw RsError(RS_E_INTERNAL, "substituted row missing from the signal map");
          turned.push_back({((uint64_t)q << 32) | (pos & 0xffffffffu), r});
        }
        std::sort(turned.begin(), turned.end());
        MK.mark("turned");
        if (getenv("RS_DEBUG")) {
          std::vector<uint8_t> tch(n_st);
          HC(hipMemcpy(tch.data(), ra.touched, n_st, hipMemcpyDeviceToHost));
          uint64_t nt = 0;
          for (auto x : tch) nt += x;
          fprintf(stderr, "[rs-debug] round: nU=%llu touched=%llu turned=%llu:", (unsigned long long)nU,
                  (unsigned long long)nt, (unsigned long long)n_turn);
          for (auto &t : turned) fprintf(stderr, " %u(q%llu)", t.second, (unsigned long long)(t.first >> 32));
          fprintf(stderr, "\n");
        }
      }
      MK.mark("appends");
      if (nU) launch(st, k_unset_rank, nU, (const uint32_t *)d_us, nU, rank_of);  // reset the dense rank index
      // next linear list: the turned rows, non-empty, in linear_id order
      std::vector<uint32_t> next_ids;
      {
        if (!turned.empty()) {  // C lengths of the turned rows only
          std::vector<uint32_t> tid_(turned.size()), tlen(turned.size());
          for (size_t i = 0; i < turned.size(); ++i) tid_[i] = turned[i].second;
          uint32_t *d_t = A.get<uint32_t>("r.tid", tid_.size()), *d_tl = A.get<uint32_t>("r.tlen", tid_.size());
          h2d(E, d_t, tid_.data(), 4 * tid_.size());
          launch(st, k_gather_u32, tid_.size(), (const uint32_t *)tc_.len, (const uint32_t *)d_t, d_tl, (uint64_t)tid_.size());
          HC(hipMemcpyAsync(tlen.data(), d_tl, 4 * tlen.size(), hipMemcpyDeviceToHost, st));
          HC(hipStreamSynchronize(st));
          for (size_t i = 0; i < turned.size(); ++i)
            if (tlen[i]) next_ids.push_back(turned[i].second);
        }
      }
      uint64_t nn = next_ids.size();
      // map appends (:369-377): the key set on the device; the row lists (positions for a later
      // round's ordering) only when another round follows
      if (nU) {
        launch(st, k_append_marks, nU, (const uint32_t *)d_us, (const uint64_t *)d_uoff, (const uint32_t *)d_ulen, nU,
               (const uint32_t *)P.pk, nlmap);
      }
      const bool another = nn > 0 && (no_rounds > 0 ? no_rounds - 1 : 0) > 0;
      if (another) {
        double Tq = now_ms();
        need_usig();
        // this round's batch of appends: every substitution's `from` and RHS keys (no values).  The
        // keys are copied on the device now (the next round's elimination reuses the pool) and come to
        // the host only if a later round resolves a list through this batch -- most never do (the
        // templated circuit's round 2: 9.8 ms of D2H and host copies saved per call)
        MapLists::Batch B;
        B.from = usig;
        const size_t bi = ML.batches.size();
        const std::string bn = "ml." + std::to_string(bi);
        uint64_t *d_optr = A.get<uint64_t>(bn + ".ptr", nU + 1);
        uint64_t *d_len64 = A.get<uint64_t>(bn + ".len", nU + 1);
        launch(st, k_u32_to_u64, nU, (const uint32_t *)d_ulen, d_len64, nU);
        HC(hipMemsetAsync(d_len64 + nU, 0, 8, st));
        const uint64_t tot = excl_scan_u64(E, d_len64, d_optr, nU + 1, "mlb");
        uint32_t *d_keys = A.get<uint32_t>(bn + ".keys", std::max<uint64_t>(tot, 1));
        if (tot)
          launch(st, k_pool_keys, 64 * nU, (const uint64_t *)d_uoff, (const uint32_t *)d_ulen, (const uint64_t *)d_optr, nU,
                 (const uint32_t *)P.pk, d_keys);
        B.load = [E, d_optr, d_keys, nU, tot](MapLists::Batch &Bt) {
          Bt.ptr.resize(nU + 1);
          Bt.keys.resize(tot);
          HC(hipMemcpyAsync(Bt.ptr.data(), d_optr, 8 * (nU + 1), hipMemcpyDeviceToHost, E->st));
          if (tot) HC(hipMemcpyAsync(Bt.keys.data(), d_keys, 4 * tot, hipMemcpyDeviceToHost, E->st));
          HC(hipStreamSynchronize(E->st));
        };
        ML.add_batch(std::move(B));
        E->stats.map_ms += now_ms() - Tq;
      }
      MK.mark("appends2");
      lv.n = nn;
      lv.off = A.get<uint64_t>("lv.off", nn);
      lv.len = A.get<uint32_t>("lv.len", nn);
      lv.key = heap_k;
      lv.val = heap_v;
      if (nn) {
        uint32_t *d_ids = A.get<uint32_t>("lv.ids", nn);
        h2d(E, d_ids, next_ids.data(), 4 * nn);
        launch(st, k_view_rows, nn, (const uint64_t *)tc_.off, (const uint32_t *)tc_.len, (const uint32_t *)d_ids, nn, lv.off, lv.len);
      }
      // emptied storage rows (storage.replace(c_id, C::empty()))
      if (!turned.empty()) {
        std::vector<uint32_t> all;
        for (auto &t : turned) all.push_back(t.second);
        uint32_t *d_all = A.get<uint32_t>("r.all", all.size());
        h2d(E, d_all, all.data(), 4 * all.size());
        launch(st, k_zero_c, all.size(), (const uint32_t *)d_all, (uint64_t)all.size(), tc_.len);
      }
      HC(hipStreamSynchronize(st));
      if (getenv("RS_DEBUG")) {
        for (uint64_t r = 0; r < std::min<uint64_t>(n_st, 24); ++r) {
          uint32_t la = 0, lb = 0, lc = 0;
          HC(hipMemcpy(&la, ta_.len + r, 4, hipMemcpyDeviceToHost));
          HC(hipMemcpy(&lb, tb_.len + r, 4, hipMemcpyDeviceToHost));
          HC(hipMemcpy(&lc, tc_.len + r, 4, hipMemcpyDeviceToHost));
          std::vector<uint32_t> kk;
          std::vector<Fe> vv;
          d2h_row(E, tc_, r, kk, vv);
          fprintf(stderr, "[rs-debug] storage %llu lens %u %u %u C:", (unsigned long long)r, la, lb, lc);
          for (size_t i = 0; i < kk.size(); ++i) fprintf(stderr, " %u:%llu", kk[i], (unsigned long long)ffrom_mont(E->F, vv[i]).l[0]);
          fprintf(stderr, "\n");
        }
      }
      MK.mark("next");
      MK.dump();
      if (g_prof_env) fprintf(stderr, "[rs-prof] round: nU %llu n_st %llu next %llu\n", (unsigned long long)nU, (unsigned long long)n_st, (unsigned long long)nn);
      E->stats.subst_ms += now_ms() - Tr;
      E->stats.rounds_ms += now_ms() - Tr;
      if (no_rounds > 0) no_rounds--;
      apply_round = nn > 0 && no_rounds > 0;
    }
  }
  // ======================= final assembly (:648-729)
  double Tf = now_ms();
  // leftover linear rows (rounds exhausted) and lconst: appended after the storage rows; their
  // signals join the non-linear map (:648-686)
  const DRows lcv = lc.view(A);
  if (lv.n) launch(st, k_mark_keys, lv.n, lv, nlmap);
  if (lcv.n) launch(st, k_mark_keys, lcv.n, lcv, nlmap);
  HC(hipMemsetAsync(nlmap, 0, 1, st));  // the constant key is not a signal
  uint32_t *kept = A.get<uint32_t>("fin.kept", S);
  uint64_t *kept64 = A.get<uint64_t>("fin.kept64", S);
  uint64_t *rank = A.get<uint64_t>("fin.rank", S);
  int32_t *l2w = A.get<int32_t>("fin.l2w", S);
  launch(st, k_kept, S, (const uint8_t *)d_deleted, (const uint8_t *)d_forb, (const uint8_t *)nlmap, kept, S);
  launch(st, k_u32_to_u64, S, (const uint32_t *)kept, kept64, S);
  E->n_wires = excl_scan_u64(E, kept64, rank, S, "kept");
  launch(st, k_l2w, S, (const uint32_t *)kept, (const uint64_t *)rank, l2w, S);
  {
    uint64_t lo = E->n_pub_out + 1, hi = E->n_pub_out + E->n_pub_in + E->n_priv_in;
    uint64_t del_in = 0;
    if (hi >= lo && lo < S) {
      uint64_t cnt = std::min<uint64_t>(hi, S - 1) - lo + 1;
      std::vector<uint32_t> k(cnt);
      HC(hipMemcpyAsync(k.data(), kept + lo, 4 * cnt, hipMemcpyDeviceToHost, st));
      HC(hipStreamSynchronize(st));
      for (uint32_t x : k) del_in += x ? 0 : 1;
    }
    E->npiw = E->n_priv_in - del_in;
  }
  // output rows: storage (non-empty) ++ leftover linear ++ lconst, empty rows dropped
  // (extract_with(is_empty), :697); the last two are C-only ("extras")
  {
    uint64_t *nef = A.get<uint64_t>("fin.nef", n_st), *nep = A.get<uint64_t>("fin.nep", n_st);
    uint64_t n_keep = 0;
    if (n_st) {
      launch(st, k_nonempty_flags, n_st, (const uint32_t *)ta_.len, (const uint32_t *)tb_.len, (const uint32_t *)tc_.len, n_st, nef);
      n_keep = excl_scan_u64(E, nef, nep, n_st, "ne");
    }
    uint32_t *keep_ids = A.get<uint32_t>("fin.keep", n_keep);
    if (n_keep) launch(st, k_scatter_ids, n_st, (const uint64_t *)nef, (const uint64_t *)nep, n_st, keep_ids);
    const DRows xsrc[2] = {lv, lcv};
    const uint64_t zn = std::max<uint64_t>(lv.n, lcv.n);
    uint32_t *zero_len = A.get<uint32_t>("fin.zlen", zn);
    if (zn) HC(hipMemsetAsync(zero_len, 0, 4 * zn, st));
    uint32_t *x_ids[2];
    uint64_t n_x[2] = {0, 0}, x_at[2];
    for (int x = 0; x < 2; ++x) {
      const DRows &V = xsrc[x];
      x_ids[x] = A.get<uint32_t>(x ? "fin.lcids" : "fin.lvids", V.n);
      if (!V.n) continue;
      uint64_t *lf = A.get<uint64_t>("fin.xf", V.n), *lp = A.get<uint64_t>("fin.xp", V.n);
      launch(st, k_nonempty_flags, V.n, (const uint32_t *)zero_len, (const uint32_t *)zero_len, (const uint32_t *)V.len, V.n, lf);
      n_x[x] = excl_scan_u64(E, lf, lp, V.n, "xf");
      launch(st, k_scatter_ids, V.n, (const uint64_t *)lf, (const uint64_t *)lp, V.n, x_ids[x]);
    }
    x_at[0] = n_keep;
    x_at[1] = n_keep + n_x[0];
    const uint64_t n_out = n_keep + n_x[0] + n_x[1];
    if (n_keep > n_st || n_x[0] > lv.n || n_x[1] > lcv.n) throw RsError(RS_E_INTERNAL, "final assembly: row counts out of range");
    E->out_n_dev = n_out;
    const DRows *parts[3] = {&ta_, &tb_, &tc_};
    const char *nm[3] = {"out.a", "out.b", "out.c"};
    // the streamed layout covers this engine's rows: all of them, or sharded its share -- the kept
    // storage rows of its non-linear rows (a run [k_lo, k_hi) of the keep list), the last rank also
    // the two C-only tails
    Comm *CMf = E->comm.get();
    const bool shard = E->snap_on && CMf && CMf->world > 1;
    uint64_t k_lo = 0, k_hi = n_keep;
    bool with_x = true;
    if (shard) {
      uint64_t kr[2] = {0, 0};
      if (n_keep) {
        uint64_t *d_kr = A.get<uint64_t>("fin.krange", 2);
        launch(st, k_keep_range, 2, (const uint32_t *)keep_ids, n_keep, (const uint32_t *)st_ids, E->nl_lo, E->nl_hi, d_kr);
        HC(hipMemcpyAsync(kr, d_kr, 16, hipMemcpyDeviceToHost, st));
        HC(hipStreamSynchronize(st));
      }
      k_lo = kr[0];
      k_hi = std::max(kr[0], kr[1]);
      with_x = CMf->rank == CMf->world - 1;
    }
    E->sh_klo = k_lo;
    E->sh_khi = k_hi;
    const uint64_t own = k_hi - k_lo;
    const uint32_t *own_ids = keep_ids + k_lo;
    const uint64_t xl_at[2] = {own, own + (with_x ? n_x[0] : 0)};
    const uint64_t xl_n[2] = {with_x ? n_x[0] : 0, with_x ? n_x[1] : 0};
    const uint64_t m_loc = own + xl_n[0] + xl_n[1];
    for (int q = 0; q < 3; ++q) {
      uint64_t *lens = A.get<uint64_t>(std::string(nm[q]) + ".lens", n_out + 1);
      uint64_t *ptr = A.get<uint64_t>(std::string(nm[q]) + ".ptr", n_out + 1);
      if (n_keep) launch(st, k_row_lens, n_keep, *parts[q], (const uint32_t *)keep_ids, n_keep, lens);
      DRows xq[2];
      for (int x = 0; x < 2; ++x) {
        xq[x] = xsrc[x];
        if (q < 2) xq[x].len = zero_len;
        if (n_x[x]) launch(st, k_row_lens, n_x[x], xq[x], (const uint32_t *)x_ids[x], n_x[x], lens + x_at[x]);
        E->fin_xq[x][q] = xq[x];
      }
      HC(hipMemsetAsync(lens + n_out, 0, 8, st));
      uint64_t tot = excl_scan_u64(E, lens, ptr, n_out + 1, nm[q]);
      E->out_nnz[q] = tot;
      E->fin_parts[q] = *parts[q];
      if (!E->snap_on) continue;
      // streamed layout: the rows not reused from the early region, after it
      uint64_t *late = A.get<uint64_t>(std::string(nm[q]) + ".late", m_loc + 1);
      uint64_t *lptr = A.get<uint64_t>(std::string(nm[q]) + ".lptr", m_loc + 1);
      if (own) launch(st, k_out_late_lens, own, *parts[q], own_ids, own, (const uint32_t *)st_ids, (const uint8_t *)so_early,
                      (const uint8_t *)so_dirty, late);
      if (xl_n[0]) launch(st, k_row_lens, xl_n[0], xq[0], (const uint32_t *)x_ids[0], xl_n[0], late + xl_at[0]);
      if (xl_n[1]) launch(st, k_lc_late_lens, xl_n[1], xq[1], (const uint32_t *)x_ids[1], xl_n[1], E->lc_snap_n, late + xl_at[1]);
      HC(hipMemsetAsync(late + m_loc, 0, 8, st));
      const uint64_t L = excl_scan_u64(E, late, lptr, m_loc + 1, "late");
      const uint64_t base = E->snap_e[q], ext = base + L;
      E->out_ext[q] = ext;
      uint64_t *beg = A.get<uint64_t>(std::string(nm[q]) + ".beg", m_loc + 1);
      uint64_t *end = A.get<uint64_t>(std::string(nm[q]) + ".end", m_loc + 1);

      if (own) launch(st, k_out_extent, own, *parts[q], own_ids, own, (const uint32_t *)st_ids, (const uint8_t *)so_early,
                      (const uint8_t *)so_dirty, (const U3 *)so_eoff, q, base, (const uint64_t *)lptr, beg, end);
      if (xl_n[0])
        launch(st, k_out_extent, xl_n[0], xq[0], (const uint32_t *)x_ids[0], xl_n[0], (const uint32_t *)nullptr, (const uint8_t *)nullptr,
               (const uint8_t *)nullptr, (const U3 *)nullptr, q, base, (const uint64_t *)(lptr + xl_at[0]), beg + xl_at[0], end + xl_at[0]);
      if (xl_n[1])
        launch(st, k_lc_extent, xl_n[1], xq[1], (const uint32_t *)x_ids[1], xl_n[1], E->lc_snap_n, E->lc_snap_base, q, base,
               (const uint64_t *)(lptr + xl_at[1]), beg + xl_at[1], end + xl_at[1]);
      launch(st, k_set_u64, 1, beg + m_loc, ext);
      {  // ABI 8: per row its length (+ RS_ROW_JUMP) and the jump table -- what crosses the link
        uint32_t *len32 = A.get<uint32_t>(std::string(nm[q]) + ".len32", m_loc + 1);
        uint64_t *jf = A.get<uint64_t>(std::string(nm[q]) + ".jf", m_loc + 1);
        uint64_t *jpos = A.get<uint64_t>(std::string(nm[q]) + ".jpos", m_loc + 1);
        uint64_t nj = 0;
        if (m_loc) {
          launch(st, k_out_jumps, m_loc, (const uint64_t *)beg, (const uint64_t *)end, m_loc, shard ? 1 : 0, len32, jf);
          nj = excl_scan_u64(E, jf, jpos, m_loc, "jump");
        }
        uint64_t *jtab = A.get<uint64_t>(std::string(nm[q]) + ".jtab", nj + 1);
        if (nj) launch(st, k_out_jtab, m_loc, (const uint64_t *)beg, (const uint64_t *)jf, (const uint64_t *)jpos, m_loc, (uint64_t)0, jtab);
        E->out_njump[q] = nj;
        if (shard) (void)A.get<uint64_t>(std::string(nm[q]) + ".jtabx", nj + 1);  // fetch_result_shared's rebased copy
      }
      // the device copy of the whole layout grows past the early region when it must (the
      // early region is copied along once its gather is done)
      const std::string xc = std::string(nm[q]) + ".xcol", xv = std::string(nm[q]) + ".xval";
      if (A.cap_bytes(xc) < 4 * ext || A.cap_bytes(xv) < 32 * ext) snap_join(E);  // its D2H reads them
      A.grow_keep<uint32_t>(xc, ext, base, E->stc, st);
      A.grow_keep<uint64_t>(xv, 4 * ext, 4 * base, E->stc, st);
      uint32_t *col = A.get<uint32_t>(xc, ext);
      uint64_t *val = A.get<uint64_t>(xv, 4 * ext);
      E->kg[2].run(st, 30 * (own + xl_n[0] + xl_n[1]) + 72 * L, [&] {
        if (own) launch(st, k_gather_late, own, E->F, *parts[q], own_ids, own, (const uint32_t *)st_ids, (const uint8_t *)so_early,
                        (const uint8_t *)so_dirty, (const uint64_t *)lptr, col + base, val + 4 * base);
        if (xl_n[0])
          launch(st, k_gather_late, xl_n[0], E->F, xq[0], (const uint32_t *)x_ids[0], xl_n[0], (const uint32_t *)nullptr,
                 (const uint8_t *)nullptr, (const uint8_t *)nullptr, (const uint64_t *)(lptr + xl_at[0]), col + base, val + 4 * base);
        if (xl_n[1])
          launch(st, k_lc_gather_late, xl_n[1], E->F, xq[1], (const uint32_t *)x_ids[1], xl_n[1], E->lc_snap_n,
                 (const uint64_t *)(lptr + xl_at[1]), col + base, val + 4 * base);
      });
    }
    if (shard) {  // a share past its capacity: the region regrows and every rank copies its whole layout
      uint64_t over = 0;
      for (int q = 0; q < 3; ++q) over |= E->out_ext[q] > E->sh_cap[q];
      if (CMf->max_u64(over, st)) {
        snap_join(E);  // the early copies into the old region are done (they are redone below)
        for (int q = 0; q < 3; ++q) E->sh_cap[q] = CMf->max_u64(E->out_ext[q] + E->out_ext[q] / 4 + 65536, st);
        E->sh_ent = CMf->shared_host(0, sh_ent_bytes(E), st);
        // (the first snapshot's shared_host already fell back when the host had no room; a regrow
        // that fails here is an error every rank reports alike)
        if (!E->sh_ent) throw RsError(RS_E_RCCL, "no shared host memory for the sharded result");
        E->sh_full = true;
      }
    }
    E->fin_keep = n_keep;
    E->fin_keep_ids = keep_ids;
    for (int x = 0; x < 2; ++x) {
      E->fin_xn[x] = n_x[x];
      E->fin_x_ids[x] = x_ids[x];
    }
    E->fin_gen = A.gen;
    if (!E->snap_on) ensure_csr(E);
  }
  load_wait_all(E);  // a group the path never needed (e.g. no non-linear rows) is still checked
  int err = 0, fw_err = 0;
  HC(hipMemcpyAsync(&err, d_err, 4, hipMemcpyDeviceToHost, st));
  HC(hipMemcpyAsync(&fw_err, d_fw_err, 4, hipMemcpyDeviceToHost, st));
  HC(hipStreamSynchronize(st));
  if (err) throw RsError(RS_E_INVALID, "input rejected by the device checks (code " + std::to_string(err) + ")");
  if (fw_err) throw RsError(RS_E_INTERNAL, "frames batch over its bounds (code " + std::to_string(fw_err) + ")");
  E->stats.final_ms = now_ms() - Tf;
  E->stats.total_ms = now_ms() - T0;
  if (g_prof_env) {
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess)
      fprintf(stderr, "[rs-prof] device memory in use after the run: %.1f of %.1f GB (heap %.1f GB)\n", (tot - fr) / 1e9, tot / 1e9,
              36e-9 * E->heap_cap);
    std::vector<std::pair<size_t, std::string>> big;
    size_t sum = 0;
    for (auto &kv : A.bufs) {
      big.push_back({kv.second.cap, kv.first});
      sum += kv.second.cap;
    }
    std::sort(big.rbegin(), big.rend());
    fprintf(stderr, "[rs-prof] arena %.1f GB in %zu buffers; largest:", sum / 1e9, big.size());
    for (size_t i = 0; i < big.size() && i < 16; ++i) fprintf(stderr, " %s %.2f", big[i].second.c_str(), big[i].first / 1e9);
    fprintf(stderr, "\n");
  }
  E->stats.h2d_wait_ms = E->h2d_wait_ms;
  E->kg[0].collect(E->stats.check_ms, E->stats.check_bytes, E->stats.check_launches);
  E->kg[1].collect(E->stats.ragged_ms, E->stats.ragged_bytes, E->stats.ragged_launches);
  E->kg[2].collect(E->stats.gather_ms, E->stats.gather_bytes, E->stats.gather_launches);
  {  // B_alg: the in-kernel counters + input / output entries and rows + the label map
    const uint64_t z_in = E->ce.nnz + E->eq.nnz + E->lin.nnz + E->na.nnz + E->nb.nnz + E->nc.nnz;
    const uint64_t r_in = E->ce.n + E->eq.n + E->lin.n + E->na.n;
    const uint64_t z_out = E->out_nnz[0] + E->out_nnz[1] + E->out_nnz[2], r_out = E->out_n_dev;
    const rs_stats &s = E->stats;
    E->stats.alg_bytes = s.elim_bytes + s.big_main_bytes + s.big_finish_bytes + s.apply_bytes + s.round_fill_bytes +
                         s.cluster_bytes + 36 * (z_in + z_out) + 8 * (r_in + r_out) + 8 * S;
  }
  E->have_result = true;
}

}  // namespace rs

namespace rs {
// One entry point's bracket around its collectives (Comm::begin_call / end_call): a call that does not
// end in RS_OK marks the call failed, which releases the ranks of an in-process group waiting in its
// collectives (rs_engine_run's failures left them waiting); the group itself stays usable.
struct CallScope {
  rs_engine *E;
  bool ok = false;
  explicit CallScope(rs_engine *e) : E(e) {
    if (E->comm) E->comm->begin_call();
  }
  ~CallScope() {
    if (!E->comm) return;
    if (!ok) E->comm->fail();
    E->comm->end_call();
  }
};
}  // namespace rs

// ==================================================================== C API
extern "C" {

int rs_abi_version(void) { return RS_ABI_VERSION; }

namespace rs {
// The host side of a call (synchronisations, the clustering's host replay, the result stream's thread)
// is latency-bound; on a multi-socket host a thread placed on the far socket from the GPU ran every
// call ~5 ms slower (the metric circuit, 42 vs 47-49 ms, process to process).  So for the duration of
// each engine call the calling thread -- and the threads the call starts (host replay, result stream,
// writer), which inherit it -- runs on the CPUs of the GPU's own NUMA node (sysfs local_cpulist of its
// PCI function) that the caller's affinity allows; the caller's own mask is restored when the call
// returns (CpuNear), so a host thread pool created later, or an engine on the other socket, is not
// narrowed by an earlier one.  near_gpu_cpus: that node's CPU set among the creator's allowed CPUs
// (the count; 0: no binding, e.g. RS_NO_CPU_BIND=1, one node, or no sysfs entry).
static int near_gpu_cpus(int device, cpu_set_t *want_out) {
  if (getenv("RS_NO_CPU_BIND")) return 0;
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof bus, device) != hipSuccess) return 0;
  for (char *c = bus; *c; ++c) *c = (char)tolower(*c);
  const std::string path = std::string("/sys/bus/pci/devices/") + bus + "/local_cpulist";
  FILE *f = fopen(path.c_str(), "r");
  if (!f) return 0;
  char buf[4096] = {0};
  const size_t got = fread(buf, 1, sizeof buf - 1, f);
  fclose(f);
  buf[got] = 0;
  cpu_set_t allowed, want;
  CPU_ZERO(&want);
  if (sched_getaffinity(0, sizeof allowed, &allowed) != 0) return 0;
  int n = 0;
  for (char *p = buf; *p && *p != '\n';) {  // "a-b,c,d-e"
    char *e = nullptr;
    const long a = strtol(p, &e, 10);
    if (e == p) break;
    long b = a;
    p = e;
    if (*p == '-') b = strtol(p + 1, &p, 10);
    for (long c = a; c <= b && c < CPU_SETSIZE; ++c)
      if (c >= 0 && CPU_ISSET(c, &allowed)) { CPU_SET(c, &want); ++n; }
    if (*p == ',') ++p;
  }
  if (n == 0 || n == CPU_COUNT(&allowed)) return 0;
  *want_out = want;
  return n;
}
// RAII: the calling thread on the engine's GPU-near CPUs for one call (those its own mask allows),
// its mask restored on return
struct CpuNear {
  cpu_set_t old;
  bool set = false;
  explicit CpuNear(const rs_engine *E);
  ~CpuNear() {
    if (set) (void)pthread_setaffinity_np(pthread_self(), sizeof old, &old);
  }
};
CpuNear::CpuNear(const rs_engine *E) {
  if (!E || !E->near_n || pthread_getaffinity_np(pthread_self(), sizeof old, &old) != 0) return;
  cpu_set_t want;
  CPU_AND(&want, &old, &E->near_cpus);
  if (CPU_COUNT(&want) == 0 || CPU_EQUAL(&want, &old)) return;
  set = pthread_setaffinity_np(pthread_self(), sizeof want, &want) == 0;
}
}  // namespace rs

int rs_engine_create(int device, rs_engine **eng) {
  try {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
      set_error("no HIP device visible: librs_simplify runs only on a gfx950 GPU");
      return RS_E_NODEVICE;
    }
    if (device < 0 || device >= n) { set_error("bad device ordinal"); return RS_E_INVALID; }
    HC(hipSetDevice(device));
    hipDeviceProp_t prop;
    HC(hipGetDeviceProperties(&prop, device));
    if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos) {
      set_error(std::string("device is ") + prop.gcnArchName + ", this build targets gfx950 only");
      return RS_E_NODEVICE;
    }
    std::unique_ptr<rs_engine> E(new rs_engine());
    E->device = device;
    CPU_ZERO(&E->near_cpus);
    E->near_n = near_gpu_cpus(device, &E->near_cpus);
    if (g_prof_env && E->near_n) fprintf(stderr, "[rs-prof] engine calls run on the GPU's %d local CPUs\n", E->near_n);
    E->n_cu = (uint32_t)prop.multiProcessorCount;
    // Streams and hardware queues.  HIP maps the normal-priority streams of a process round-robin onto
    // a pool of GPU_MAX_HW_QUEUES (4) hardware queues, and two streams that share a queue execute in
    // one order: a kernel on one waits for a barrier the other queued behind a copy.  Which engine
    // stream shares the copy stream's queue depended on how many streams the process had created
    // before the engine (tools/micro/qshare.hip on MI355X: none -> stg, one -> stx, two -> st), and with
    // st there the whole clustering waits for the input's upload (the stc queue holds its check kernels
    // behind the linear values' and the non-linear blocks' copies).  A stream with a CU mask gets a
    // hardware queue of its own, so the copy stream -- the one stream whose kernels wait behind long
    // copies -- is made with the full mask and shares its queue with nothing (RS_POOLED_STREAMS=1: a
    // pooled one; RS_CUMASK_STREAMS=1: every normal-priority stream dedicated, measured no better).
    // A CU-mask stream blocks with the null stream: nothing in a run uses it (E->srd takes host reads).
    const bool pooled = getenv("RS_POOLED_STREAMS") != nullptr, all_masked = getenv("RS_CUMASK_STREAMS") != nullptr;
    std::vector<uint32_t> cu_mask((E->n_cu + 31) / 32, 0u);
    for (uint32_t c = 0; c < E->n_cu; ++c) cu_mask[c / 32] |= 1u << (c % 32);
    auto mk_stream = [&](hipStream_t *sp, bool dedicated) {
      if (pooled || !dedicated || hipExtStreamCreateWithCUMask(sp, (uint32_t)cu_mask.size(), cu_mask.data()) != hipSuccess)
        HC(hipStreamCreateWithFlags(sp, hipStreamNonBlocking));
    };
    mk_stream(&E->st, all_masked);
    HC(hipStreamCreateWithFlags(&E->srd, hipStreamNonBlocking));
    {  // the second stream carries the critical path (the largest clusters' chain): high priority
      int lo = 0, hi = 0;
      if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess ||
          hipStreamCreateWithPriority(&E->st2, hipStreamNonBlocking, hi) != hipSuccess)
        HC(hipStreamCreateWithFlags(&E->st2, hipStreamNonBlocking));
    }
    mk_stream(&E->stc, true);
    mk_stream(&E->stx, all_masked);
    mk_stream(&E->str, all_masked);
    {  // the small clusters and the tail's second group: least priority, so the tail's first group (the
       // first frames pass's critical path) finds CUs before their wide finish does
      int lo = 0, hi = 0;
      if (getenv("RS_STE_DEFAULT") || hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess ||
          hipStreamCreateWithPriority(&E->ste, hipStreamNonBlocking, lo) != hipSuccess)
        HC(hipStreamCreateWithFlags(&E->ste, hipStreamNonBlocking));
      if (g_prof_env) fprintf(stderr, "[rs-prof] stream priorities: least %d greatest %d\n", lo, hi);
    }
    mk_stream(&E->stg, all_masked);
    for (auto &ev : E->evg) HC(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    for (auto &g : E->evt)
      for (auto &ev : g) HC(hipEventCreate(&ev));
    for (auto &ev : E->evc) HC(hipEventCreate(&ev));
    for (auto &ev : E->evgt) HC(hipEventCreate(&ev));
    for (auto &ev : E->ev_sm) HC(hipEventCreate(&ev));
    for (auto &ev : E->evx) HC(hipEventCreate(&ev));
    for (auto &ev : E->ev_grp) HC(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    HC(hipHostMalloc((void **)&E->h_vflag, 10 * sizeof(int), hipHostMallocDefault));
    memset(E->h_vflag, 0, 10 * sizeof(int));
    HC(hipHostMalloc((void **)&E->h_lvl, 8 * sizeof(unsigned long long), hipHostMallocDefault));
    for (auto &ev : E->ev_lvl) HC(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    for (auto &ev : E->ev_lvlt) HC(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    HC(hipEventCreate(&E->ev0));
    HC(hipEventCreate(&E->ev1));
    HC(hipEventCreate(&E->ev2));
    HC(hipEventCreate(&E->ev3));
    HC(hipEventCreate(&E->ev4));
    HC(hipEventCreate(&E->ev5));
    HC(hipEventCreate(&E->ev6));
    HC(hipEventCreate(&E->ev7));
    HC(hipEventCreateWithFlags(&E->ev_snap, hipEventDisableTiming));
    HC(hipEventCreateWithFlags(&E->ev_snap0, hipEventDisableTiming));
    for (auto &ev : E->ev_chunk) HC(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    for (auto &ev : E->ev_snapq) HC(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    for (auto &ev : E->ev_snaph) HC(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    for (auto &ev : E->ev_fh) HC(hipEventCreate(&ev));
    HC(hipEventCreateWithFlags(&E->ev_nlc, hipEventDisableTiming));
    *eng = E.release();
    return RS_OK;
  } catch (const RsError &e) {
    set_error(e.what());
    return e.code;
  } catch (const std::exception &e) {
    set_error(e.what());
    return RS_E_INTERNAL;
  }
}

void rs_engine_destroy(rs_engine *E) {
  if (!E) return;
  (void)hipSetDevice(E->device);
  if (E->st) (void)hipStreamSynchronize(E->st);
  if (E->st2) (void)hipStreamSynchronize(E->st2);
  if (E->stc) (void)hipStreamSynchronize(E->stc);
  if (E->ste) (void)hipStreamSynchronize(E->ste);
  if (E->stg) (void)hipStreamSynchronize(E->stg);
  snap_join(E);
  E->comm.reset();
  for (auto &pb : E->pin)
    if (pb.p) (void)hipHostFree(pb.p);
  if (E->h_vflag) (void)hipHostFree(E->h_vflag);
  if (E->h_lvl) (void)hipHostFree(E->h_lvl);
  for (auto &ev : E->ev_lvl)
    if (ev) (void)hipEventDestroy(ev);
  for (auto &ev : E->ev_lvlt)
    if (ev) (void)hipEventDestroy(ev);
  for (auto &ev : E->ev_grp)
    if (ev) (void)hipEventDestroy(ev);
  for (auto &g : E->kg) g.destroy();
  if (E->stc) (void)hipStreamDestroy(E->stc);
  if (E->stx) (void)hipStreamDestroy(E->stx);
  if (E->str) (void)hipStreamDestroy(E->str);
  if (E->ste) (void)hipStreamDestroy(E->ste);
  if (E->stg) (void)hipStreamDestroy(E->stg);
  if (E->srd) (void)hipStreamDestroy(E->srd);
  for (auto &ev : E->evg)
    if (ev) (void)hipEventDestroy(ev);
  for (auto &g : E->evt)
    for (auto &ev : g)
      if (ev) (void)hipEventDestroy(ev);
  for (auto &ev : E->evc)
    if (ev) (void)hipEventDestroy(ev);
  for (auto &ev : E->evgt)
    if (ev) (void)hipEventDestroy(ev);
  for (auto &ev : E->ev_sm)
    if (ev) (void)hipEventDestroy(ev);
  if (E->ev0) (void)hipEventDestroy(E->ev0);
  if (E->ev1) (void)hipEventDestroy(E->ev1);
  if (E->ev2) (void)hipEventDestroy(E->ev2);
  if (E->ev3) (void)hipEventDestroy(E->ev3);
  if (E->ev4) (void)hipEventDestroy(E->ev4);
  if (E->ev5) (void)hipEventDestroy(E->ev5);
  if (E->ev6) (void)hipEventDestroy(E->ev6);
  if (E->ev7) (void)hipEventDestroy(E->ev7);
  if (E->ev_snap) (void)hipEventDestroy(E->ev_snap);
  if (E->ev_snap0) (void)hipEventDestroy(E->ev_snap0);
  for (auto &ev : E->ev_chunk)
    if (ev) (void)hipEventDestroy(ev);
  for (auto &ev : E->ev_snapq)
    if (ev) (void)hipEventDestroy(ev);
  if (E->heap_k) (void)hipFree(E->heap_k);
  if (E->heap_v) (void)hipFree(E->heap_v);
  if (E->st) (void)hipStreamDestroy(E->st);
  if (E->st2) (void)hipStreamDestroy(E->st2);
  for (auto &ev : E->evx)
    if (ev) (void)hipEventDestroy(ev);
  delete E;
}

int rs_engine_load(rs_engine *E, const rs_input *in) {
  CpuNear cpu_near_(E);  // the caller's affinity is restored on return
  CallScope cs(E);
  try {
    HC(hipSetDevice(E->device));
    load_enqueue(E, in, false);
    load_wait_all(E);
    cs.ok = true;
    return RS_OK;
  } catch (const RsError &e) {
    load_abort(E);
    E->loaded = false;
    set_error(e.what());
    return e.code;
  } catch (const std::exception &e) {
    load_abort(E);
    E->loaded = false;
    set_error(e.what());
    return RS_E_INTERNAL;
  }
}

int rs_engine_run(rs_engine *E, const rs_flags *fl) {
  CpuNear cpu_near_(E);  // the caller's affinity is restored on return
  CallScope cs(E);
  try {
    if (!E->loaded) { set_error("engine has no input"); return RS_E_INVALID; }
    HC(hipSetDevice(E->device));
    engine_run(E, fl);
    cs.ok = true;
    return RS_OK;
  } catch (const RsError &e) {
    set_error(e.what());
    return e.code;
  } catch (const std::exception &e) {
    set_error(e.what());
    return RS_E_INTERNAL;
  }
}

int rs_engine_stats(rs_engine *E, rs_stats *s) {
  *s = E->stats;
  return RS_OK;
}

namespace rs {
// The result in host memory.  buf(slot, bytes) supplies the destination of each array -- slots
// 0-2 ptr of a/b/c, 3-5 col, 6-8 val, 9 label_to_wire -- (malloc for rs_engine_fetch, the engine's
// pinned buffers for rs_engine_simplify).  Every D2H is enqueued first and waited for once.  The
// substitution log is copied
// (own = true) or pointed at (the engine's vectors, rs_engine_simplify's view).
// grows pinned slot `slot` keeping its first `keep` bytes (the early region, once its D2H is done)
static void *pin_grow_keep(rs_engine *E, int slot, size_t bytes, size_t keep) {
  rs_engine::Pin &b = E->pin[slot];
  if (b.cap >= bytes) return b.p;
  snap_join(E);
  const size_t cap = std::max(bytes, b.cap + b.cap / 4);
  void *p = nullptr;
  HC(hipHostMalloc(&p, cap, hipHostMallocDefault));
  if (keep) memcpy(p, b.p, keep);
  if (b.p) HC(hipHostFree(b.p));
  b.p = p;
  b.cap = cap;
  return p;
}

// D2H of the last result.  streamed (rs_engine_simplify after a run that took the early region):
// the early region is already on its way into pin[3..8]; the late rows land after it and every
// row gets [beg, end) (rs_output.{a,b,c}_end).  Otherwise the compact CSR.
static void fetch_result(rs_engine *E, rs_output *o, const std::function<void *(int, size_t)> &buf, bool own_log, bool streamed) {
  const uint64_t nd = E->out_n_dev;
  o->n_constraints = nd;
  const char *nm[3] = {"out.a", "out.b", "out.c"};
  rs_lc *dst[3] = {&o->a, &o->b, &o->c};
  uint32_t **lens[3] = {&o->a_len, &o->b_len, &o->c_len};
  uint64_t **jumps[3] = {&o->a_jump, &o->b_jump, &o->c_jump};
  uint64_t *njs[3] = {&o->a_njump, &o->b_njump, &o->c_njump};
  if (!streamed) ensure_csr(E);
  for (int q = 0; q < 3; ++q) {
    rs_lc &L = *dst[q];
    const std::string n(nm[q]);
    L.n_rows = nd;
    if (!streamed) {
      const uint64_t tot = E->out_nnz[q];
      L.nnz = tot;
      L.ptr = (uint64_t *)buf(q, 8 * (nd + 1));
      L.col = (uint32_t *)buf(3 + q, 4 * (tot ? tot : 1));
      L.val = (uint64_t *)buf(6 + q, 32 * (tot ? tot : 1));
      *lens[q] = nullptr;
      *jumps[q] = nullptr;
      *njs[q] = 0;
      if (nd) HC(hipMemcpyAsync(L.ptr, E->A.get<uint64_t>(n + ".ptr", 1), 8 * (nd + 1), hipMemcpyDeviceToHost, E->st));
      else L.ptr[0] = 0;
      if (tot) {
        HC(hipMemcpyAsync(L.col, E->A.get<uint32_t>(n + ".col", 1), 4 * tot, hipMemcpyDeviceToHost, E->st));
        HC(hipMemcpyAsync(L.val, E->A.get<uint64_t>(n + ".val", 1), 32 * tot, hipMemcpyDeviceToHost, E->st));
      }
      continue;
    }
    const uint64_t early = E->snap_e[q], ext = E->out_ext[q], nj = E->out_njump[q];
    L.nnz = ext;
    L.ptr = nullptr;  // ABI 8: lengths + jumps (rs_rows_next)
    *lens[q] = (uint32_t *)pin_get(E, 13 + q, 4 * (nd ? nd : 1));
    *jumps[q] = (uint64_t *)pin_get(E, q, 8 * (nj ? nj : 1));
    *njs[q] = nj;
    L.col = (uint32_t *)pin_grow_keep(E, 3 + q, 4 * (ext ? ext : 1), 4 * early);
    L.val = (uint64_t *)pin_grow_keep(E, 6 + q, 32 * (ext ? ext : 1), 32 * early);
    if (nd) HC(hipMemcpyAsync(*lens[q], E->A.get<uint32_t>(n + ".len32", 1), 4 * nd, hipMemcpyDeviceToHost, E->st));
    if (nj) HC(hipMemcpyAsync(*jumps[q], E->A.get<uint64_t>(n + ".jtab", 1), 8 * nj, hipMemcpyDeviceToHost, E->st));
    if (ext > early) {
      HC(hipMemcpyAsync(L.col + early, E->A.get<uint32_t>(n + ".xcol", 1) + early, 4 * (ext - early), hipMemcpyDeviceToHost, E->st));
      HC(hipMemcpyAsync(L.val + 4 * early, E->A.get<uint64_t>(n + ".xval", 1) + 4 * early, 32 * (ext - early),
                        hipMemcpyDeviceToHost, E->st));
    }
  }
  o->n_labels = E->S;
  o->label_to_wire = (int32_t *)buf(9, 4 * E->S);
  HC(hipMemcpyAsync(o->label_to_wire, E->A.get<int32_t>("fin.l2w", 1), 4 * E->S, hipMemcpyDeviceToHost, E->st));
  const double tf0 = g_prof_env ? now_ms() : 0.0;
  HC(hipStreamSynchronize(E->st));
  if (g_prof_env && streamed) {
    double late = 4.0 * E->S;
    for (int q = 0; q < 3; ++q) late += 4.0 * nd + 8.0 * E->out_njump[q] + 36.0 * (E->out_ext[q] - E->snap_e[q]);
    fprintf(stderr, "[rs-prof] fetch: row extents, late rows and label_to_wire %.1f MB, waited %.2f ms\n", late / 1e6, now_ms() - tf0);
  }
  if (streamed) {
    snap_join(E);
    if (E->snap_rc) throw RsError(RS_E_HIP, "D2H of the streamed rows failed");
  }
  o->n_wires = E->n_wires;
  o->no_private_inputs_witness = E->npiw;
  o->n_log = 0;
  o->log_from = nullptr;
  o->log_to = rs_lc{};
  if (E->log_on) {
    const uint64_t n = E->log_from.size(), nnz = E->log_key.size();
    o->n_log = n;
    o->log_to.n_rows = n;
    o->log_to.nnz = nnz;
    if (own_log) {
      o->log_from = (uint32_t *)malloc(4 * (n ? n : 1));
      o->log_to.ptr = (uint64_t *)malloc(8 * (n + 1));
      o->log_to.col = (uint32_t *)malloc(4 * (nnz ? nnz : 1));
      o->log_to.val = (uint64_t *)malloc(32 * (nnz ? nnz : 1));
      if (n) memcpy(o->log_from, E->log_from.data(), 4 * n);
      memcpy(o->log_to.ptr, E->log_ptr.data(), 8 * (n + 1));
      if (nnz) {
        memcpy(o->log_to.col, E->log_key.data(), 4 * nnz);
        memcpy(o->log_to.val, E->log_val.data(), 32 * nnz);
      }
    } else {
      o->log_from = E->log_from.data();
      o->log_to.ptr = E->log_ptr.data();
      o->log_to.col = E->log_key.data();
      o->log_to.val = E->log_val.data();
    }
  }
}

// The sharded host -> host result: every rank copies its share (its rows' extents at their global
// row numbers, its late entries after its early ones, its slice of label_to_wire) into the shared
// host regions; after a barrier each rank's *o describes the whole result there (the view is the
// same on every rank).  Row extents of part q are rank-based: rank r's entries start at r * sh_cap[q].
static void fetch_result_shared(rs_engine *E, rs_output *o, bool own_log) {
  Comm &CM = *E->comm;
  Arena &A = E->A;
  hipStream_t st = E->st;
  const uint64_t W = CM.world, r = CM.rank, nd = E->out_n_dev, S = E->S;
  const uint64_t k_lo = E->sh_klo, own = E->sh_khi - E->sh_klo, n_keep = E->fin_keep;
  const bool with_x = r == W - 1;
  const uint64_t m_loc = own + (with_x ? nd - n_keep : 0);
  // rows region (ABI 8): the row lengths of a, b, c (u32, nd each), the jump tables of a, b, c (every
  // rank's, in rank order -- the ranks' rows are consecutive in storage order, each rank's first row
  // jumps to its base), then label_to_wire
  uint64_t nj_tot[3], nj_before[3];
  for (int q = 0; q < 3; ++q) {
    const std::vector<uint64_t> g = CM.gather_u64(E->out_njump[q], st);
    nj_tot[q] = nj_before[q] = 0;
    for (uint64_t x = 0; x < W; ++x) {
      if (x < r) nj_before[q] += g[x];
      nj_tot[q] += g[x];
    }
  }
  const uint64_t len_bytes = (12 * nd + 7) / 8 * 8, jump_bytes = 8 * (nj_tot[0] + nj_tot[1] + nj_tot[2]);
  const uint64_t rows_bytes = len_bytes + jump_bytes + 4 * S;
  uint8_t *rb = (uint8_t *)CM.shared_host(1, rows_bytes, st);
  if (!rb) throw RsError(RS_E_RCCL, "no shared host memory for the sharded result");
  const char *nm[3] = {"out.a", "out.b", "out.c"};
  rs_lc *dst[3] = {&o->a, &o->b, &o->c};
  uint32_t **lens[3] = {&o->a_len, &o->b_len, &o->c_len};
  uint64_t **jumps[3] = {&o->a_jump, &o->b_jump, &o->c_jump};
  uint64_t *njs[3] = {&o->a_njump, &o->b_njump, &o->c_njump};
  o->n_constraints = nd;
  uint64_t *jbase = (uint64_t *)(rb + len_bytes);
  for (int q = 0; q < 3; ++q) {
    uint32_t *len = (uint32_t *)(rb + 4 * nd * q);
    uint64_t *jtab = jbase + (q > 0 ? nj_tot[0] : 0) + (q > 1 ? nj_tot[1] : 0);
    const std::string n(nm[q]);
    const uint64_t rbase = r * E->sh_cap[q], early = E->snap_e[q], ext = E->out_ext[q], nj = E->out_njump[q];
    if (own) HC(hipMemcpyAsync(len + k_lo, A.get<uint32_t>(n + ".len32", 1), 4 * own, hipMemcpyDeviceToHost, st));
    if (m_loc > own)
      HC(hipMemcpyAsync(len + n_keep, A.get<uint32_t>(n + ".len32", 1) + own, 4 * (m_loc - own), hipMemcpyDeviceToHost, st));
    if (nj) {  // this rank's jumps, moved to its base
      uint64_t *jx = A.get<uint64_t>(n + ".jtabx", 1);  // sized by the run
      launch(st, k_add_u64, nj, (const uint64_t *)A.get<uint64_t>(n + ".jtab", 1), nj, rbase, jx);
      HC(hipMemcpyAsync(jtab + nj_before[q], jx, 8 * nj, hipMemcpyDeviceToHost, st));
    }
    const uint64_t from = E->sh_full ? 0 : early;  // the early entries are on their way (snap thread)
    if (ext > from) {
      HC(hipMemcpyAsync(sh_col(E, q) + rbase + from, A.get<uint32_t>(n + ".xcol", 1) + from, 4 * (ext - from), hipMemcpyDeviceToHost, st));
      HC(hipMemcpyAsync(sh_val(E, q) + 4 * (rbase + from), A.get<uint64_t>(n + ".xval", 1) + 4 * from, 32 * (ext - from),
                        hipMemcpyDeviceToHost, st));
    }
    rs_lc &L = *dst[q];
    L.n_rows = nd;
    L.nnz = W * E->sh_cap[q];
    L.ptr = nullptr;
    L.col = sh_col(E, q);
    L.val = sh_val(E, q);
    *lens[q] = len;
    *jumps[q] = jtab;
    *njs[q] = nj_tot[q];
  }
  int32_t *l2w = (int32_t *)(rb + len_bytes + jump_bytes);
  const uint64_t s0 = S * r / W, s1 = S * (r + 1) / W;
  if (s1 > s0) HC(hipMemcpyAsync(l2w + s0, A.get<int32_t>("fin.l2w", 1) + s0, 4 * (s1 - s0), hipMemcpyDeviceToHost, st));
  HC(hipStreamSynchronize(st));
  snap_join(E);
  const uint64_t bad = CM.max_u64(E->snap_rc ? 1 : 0, st);  // also the barrier: every share has landed
  if (bad) throw RsError(RS_E_HIP, "D2H of the streamed rows failed");
  o->n_labels = S;
  o->label_to_wire = l2w;
  o->n_wires = E->n_wires;
  o->no_private_inputs_witness = E->npiw;
  o->n_log = 0;
  o->log_from = nullptr;
  o->log_to = rs_lc{};
  if (E->log_on) {
    const uint64_t n = E->log_from.size(), nnz = E->log_key.size();
    o->n_log = n;
    o->log_to.n_rows = n;
    o->log_to.nnz = nnz;
    (void)own_log;
    o->log_from = E->log_from.data();
    o->log_to.ptr = E->log_ptr.data();
    o->log_to.col = E->log_key.data();
    o->log_to.val = E->log_val.data();
  }
}

}  // namespace rs

int rs_engine_fetch(rs_engine *E, rs_output **out) {
  CpuNear cpu_near_(E);  // the caller's affinity is restored on return
  try {
    if (!E->have_result) { set_error("no result"); return RS_E_INVALID; }
    HC(hipSetDevice(E->device));
    rs_output *o = (rs_output *)calloc(1, sizeof(rs_output));
    try {
      fetch_result(E, o, [](int, size_t bytes) { void *p = malloc(bytes ? bytes : 1); if (!p) throw std::bad_alloc(); return p; }, true,
                   false);
    } catch (...) {
      rs_output_free(o);
      throw;
    }
    *out = o;
    return RS_OK;
  } catch (const RsError &e) {
    set_error(e.what());
    return e.code;
  } catch (const std::exception &e) {
    set_error(e.what());
    return RS_E_INTERNAL;
  }
}

int rs_engine_simplify(rs_engine *E, const rs_input *in, const rs_flags *fl, const rs_output **out) {
  CpuNear cpu_near_(E);  // the caller's affinity is restored on return
  CallScope cs(E);
  try {
    const double t0 = now_ms();
    HC(hipSetDevice(E->device));
    load_enqueue(E, in, true);
    E->stream_out = true;
    try {
      engine_run(E, fl);
    } catch (...) {
      E->stream_out = false;
      throw;
    }
    E->stream_out = false;
    E->hin = nullptr;
    const double t1 = now_ms();
    E->view = rs_output{};
    if (E->snap_on && E->comm && E->comm->world > 1) fetch_result_shared(E, &E->view, false);
    else fetch_result(E, &E->view, [E](int slot, size_t bytes) { return pin_get(E, slot, bytes); }, false, E->snap_on);
    const double t2 = now_ms();
    E->stats.d2h_ms = t2 - t1;
    E->stats.host_total_ms = t2 - t0;
    *out = &E->view;
    cs.ok = true;
    return RS_OK;
  } catch (const RsError &e) {
    load_abort(E);
    E->loaded = false;
    set_error(e.what());
    return e.code;
  } catch (const std::exception &e) {
    load_abort(E);
    E->loaded = false;
    set_error(e.what());
    return RS_E_INTERNAL;
  }
}

// The last result as a .r1cs file (constraint_list/src/r1cs_porting.rs:4-124, the same bytes as
// rs_write_r1cs on the fetched output): the constraint section is built on the device (writer.hpp)
// and streamed to the file through two pinned staging buffers; the small sections follow.  o0_r1cs (optional): custom-gate sections as rs_write_r1cs_gates.
int rs_engine_write_r1cs(rs_engine *E, const char *path, const char *o0_r1cs) {
  CpuNear cpu_near_(E);  // the caller's affinity is restored on return
  try {
    if (!E->have_result) { set_error("no result"); return RS_E_INVALID; }
    HC(hipSetDevice(E->device));
    const double t0 = now_ms();
    Arena &A = E->A;
    hipStream_t st = E->st;
    const uint32_t fs = (uint32_t)field_size_bytes(E->prime);
    const uint64_t n = E->out_n_dev, S = E->S;
    if (getenv("RS_WRITER_HOST") || n >= (1ull << (64 - kLeKeyBits)) || E->out_nnz[0] >> 32 || E->out_nnz[1] >> 32 || E->out_nnz[2] >> 32) {
      // the device sort key holds the row in 64 - 36 = 28 bits and the entry index in 32: beyond
      // that, the host writer over the fetched result (same bytes, no such limits)
      rs_output *o = nullptr;
      int rc = rs_engine_fetch(E, &o);
      if (rc != RS_OK) return rc;
      rs_input hin{};
      hin.prime_id = RS_PRIME_CUSTOM;
      memcpy(hin.prime, E->prime, sizeof(hin.prime));
      hin.max_signal = S;
      hin.n_pub_out = E->n_pub_out;
      hin.n_pub_in = E->n_pub_in;
      hin.n_priv_in = E->n_priv_in;
      rc = o0_r1cs ? rs_write_r1cs_gates(path, &hin, o, o0_r1cs) : rs_write_r1cs(path, &hin, o);
      rs_output_free(o);
      E->stats.write_ms = now_ms() - t0;
      return rc;
    }
    ensure_csr(E);
    const char *nm[3] = {"out.a", "out.b", "out.c"};
    const uint64_t *pq[3];
    for (int q = 0; q < 3; ++q) pq[q] = A.get<uint64_t>(std::string(nm[q]) + ".ptr", 1);
    const int32_t *l2w = A.get<int32_t>("fin.l2w", 1);
    int *d_err = A.get<int>("w.err", 1);
    HC(hipMemsetAsync(d_err, 0, 4, st));
    // record offsets
    uint64_t *sz = A.get<uint64_t>("w.sz", n + 1), *roff = A.get<uint64_t>("w.roff", n + 1);
    if (n) launch(st, k_w_rowbytes, n, pq[0], pq[1], pq[2], n, fs, sz);
    HC(hipMemsetAsync(sz + n, 0, 8, st));
    const uint64_t dev_bytes = excl_scan_u64(E, sz, roff, n + 1, "wsz");
    uint32_t *img = A.get<uint32_t>("w.img", dev_bytes / 4 + 1);
    if (n) launch(st, k_w_counts, n, pq[0], pq[1], pq[2], (const uint64_t *)roff, n, fs, img);
    int rbits = 1;
    while (rbits < 28 && (1ull << rbits) <= n) ++rbits;
    for (int q = 0; q < 3; ++q) {
      const uint64_t nnz = E->out_nnz[q];
      if (!nnz) continue;
      uint64_t *k1 = A.get<uint64_t>("w.k1", nnz), *k2 = A.get<uint64_t>("w.k2", nnz);
      uint32_t *i1 = A.get<uint32_t>("w.i1", nnz), *i2 = A.get<uint32_t>("w.i2", nnz);
      const uint32_t *col = A.get<uint32_t>(std::string(nm[q]) + ".col", 1);
      const uint64_t *val = A.get<uint64_t>(std::string(nm[q]) + ".val", 1);
      launch(st, k_w_keys, n, pq[q], n, col, l2w, k1, i1, d_err);
      sort_pairs(E, (const uint64_t *)k1, k2, (const uint32_t *)i1, i2, nnz, kLeKeyBits + rbits, "w");
      launch(st, k_w_entries, nnz, (const uint64_t *)k2, (const uint32_t *)i2, nnz, q, pq[0], pq[1], pq[2],
             (const uint64_t *)roff, col, val, l2w, fs, img);
    }
    uint64_t *w2l = A.get<uint64_t>("w.w2l", E->n_wires + 1);
    launch(st, k_w_w2l, S, l2w, S, w2l);
    std::vector<int32_t> hl2w(S);
    HC(hipMemcpyAsync(hl2w.data(), l2w, 4 * S, hipMemcpyDeviceToHost, st));
    std::vector<uint64_t> hw2l(E->n_wires);
    if (E->n_wires) HC(hipMemcpyAsync(hw2l.data(), w2l, 8 * E->n_wires, hipMemcpyDeviceToHost, st));
    int err = 0;
    HC(hipMemcpyAsync(&err, d_err, 4, hipMemcpyDeviceToHost, st));
    HC(hipStreamSynchronize(st));
    if (err) throw RsError(RS_E_INTERNAL, "constraint mentions a removed signal (apply_raw_correspondence panics)");
    std::vector<uint8_t> gates;
    bool with_gates = false;
    if (o0_r1cs && !r1cs_gate_sections(o0_r1cs, hl2w.data(), S, gates, with_gates)) return RS_E_INVALID;
    const double t_built = now_ms();
    // the file: magic + section 2's header, the device image, then sections 1 and 3 (+ the gates'
    // sections).  The image goes out in 32 MB chunks that four threads pwrite at their offsets while
    // the next chunks' D2H run.  The page cache bounds it: on the GPU box's overlay file system a fresh
    // 0.92 GB file takes 130-160 ms with one or four writers (a shared mapping with four copiers:
    // ~400 ms of page faults); the device build is 10-23 ms of it, the D2H ~18 ms at link speed
    std::vector<uint8_t> head, tail;
    auto put32 = [](std::vector<uint8_t> &v, uint32_t x) { const uint8_t *b = (const uint8_t *)&x; v.insert(v.end(), b, b + 4); };
    auto put64 = [](std::vector<uint8_t> &v, uint64_t x) { const uint8_t *b = (const uint8_t *)&x; v.insert(v.end(), b, b + 8); };
    {
      const char *magic = with_gates ? "r1cs\x01\x00\x00\x00\x05\x00\x00\x00" : "r1cs\x01\x00\x00\x00\x03\x00\x00\x00";
      head.insert(head.end(), (const uint8_t *)magic, (const uint8_t *)magic + 12);
      put32(head, 2);
      put64(head, dev_bytes);
      // header (r1cs_writer.rs:246-269)
      put32(tail, 1);
      put64(tail, 4 + fs + 4 * 4 + 8 + 4);
      put32(tail, fs);
      tail.insert(tail.end(), (const uint8_t *)E->prime, (const uint8_t *)E->prime + fs);
      put32(tail, (uint32_t)E->n_wires);
      put32(tail, (uint32_t)E->n_pub_out);
      put32(tail, (uint32_t)E->n_pub_in);
      put32(tail, (uint32_t)E->n_priv_in);
      put64(tail, S);
      put32(tail, (uint32_t)n);
      // wire -> label
      put32(tail, 3);
      put64(tail, 8 * E->n_wires);
      if (E->n_wires) tail.insert(tail.end(), (const uint8_t *)hw2l.data(), (const uint8_t *)(hw2l.data() + E->n_wires));
      if (with_gates) tail.insert(tail.end(), gates.begin(), gates.end());
    }
    constexpr uint64_t kChunk = 32ull << 20;
    constexpr int kBufs = 8, kThreads = 4;
    const uint64_t nch = (dev_bytes + kChunk - 1) / kChunk;
    // everything that can throw before the file exists: the pinned buffers, the events (a
    // throw between open() and the guarded block leaked the fd or destroyed joinable threads)
    uint8_t *pool = nch ? (uint8_t *)pin_get(E, 11, kBufs * kChunk) : nullptr;
    struct Events {
      hipEvent_t e[kBufs] = {};
      ~Events() {
        for (hipEvent_t x : e)
          if (x) (void)hipEventDestroy(x);
      }
    } evs;
    hipEvent_t *evb = evs.e;
    for (int b = 0; b < kBufs; ++b) HC(hipEventCreateWithFlags(&evb[b], hipEventDisableTiming));
    struct Fd {
      int fd;
      ~Fd() {
        if (fd >= 0) close(fd);
      }
    } file{open(path, O_WRONLY | O_CREAT | O_TRUNC, 0644)};
    if (file.fd < 0) throw RsError(RS_E_INVALID, std::string("cannot write ") + path);
    const int fd = file.fd;
    std::atomic<bool> io_err{false};
    auto pwrite_all = [&](const uint8_t *p, uint64_t len, uint64_t off) {
      while (len) {
        const ssize_t w = pwrite(fd, p, len, (off_t)off);
        if (w <= 0) { io_err = true; return; }
        p += w;
        len -= (uint64_t)w;
        off += (uint64_t)w;
      }
    };
    const uint64_t img_off = head.size(), fsize = img_off + dev_bytes + tail.size();
    // the file's blocks up front (a fresh 0.92 GB file: 10.0 -> 11.4 GB/s from host memory on the GPU box's
    // /tmp, tools/writer_bench.py); a file system without fallocate gets the size by ftruncate
    if (posix_fallocate(fd, 0, (off_t)fsize) != 0 && ftruncate(fd, (off_t)fsize) != 0) io_err = true;
    pwrite_all(head.data(), head.size(), 0);
    pwrite_all(tail.data(), tail.size(), img_off + dev_bytes);
    std::mutex mu;
    std::condition_variable cv;
    std::deque<uint64_t> work;       // chunks whose D2H is enqueued
    std::vector<char> written(nch, 0);
    bool closing = false;
    // the writer threads are joined on every way out of this scope (a throw included): closing drains
    // them, and the guard lives after everything they reference
    struct Writers {
      std::vector<std::thread> th;
      std::mutex &mu;
      std::condition_variable &cv;
      bool &closing;
      std::deque<uint64_t> &work;
      void stop(bool drop) {
        {
          std::lock_guard<std::mutex> lk(mu);
          closing = true;
          if (drop) work.clear();
        }
        cv.notify_all();
        for (auto &x : th)
          if (x.joinable()) x.join();
      }
      ~Writers() { stop(true); }
    } writers{{}, mu, cv, closing, work};
    for (int t = 0; t < kThreads && (uint64_t)t < nch; ++t)
      writers.th.emplace_back([&]() {
        for (;;) {
          uint64_t i;
          {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return closing || !work.empty(); });
            if (work.empty()) return;
            i = work.front();
            work.pop_front();
          }
          const uint64_t off = i * kChunk, len = std::min(kChunk, dev_bytes - off);
          if (hipEventSynchronize(evb[i % kBufs]) != hipSuccess) io_err = true;
          else pwrite_all(pool + (i % kBufs) * kChunk, len, img_off + off);
          {
            std::lock_guard<std::mutex> lk(mu);
            written[i] = 1;
          }
          cv.notify_all();
        }
      });
    const uint8_t *src = (const uint8_t *)img;
    for (uint64_t i = 0; i < nch; ++i) {
      if (i >= (uint64_t)kBufs) {  // the buffer's previous chunk is on disk
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return written[i - kBufs] != 0; });
      }
      const uint64_t off = i * kChunk, len = std::min(kChunk, dev_bytes - off);
      HC(hipMemcpyAsync(pool + (i % kBufs) * kChunk, src + off, len, hipMemcpyDeviceToHost, st));
      HC(hipEventRecord(evb[i % kBufs], st));
      {
        std::lock_guard<std::mutex> lk(mu);
        work.push_back(i);
      }
      cv.notify_all();
    }
    writers.stop(false);  // every chunk written
    file.fd = -1;
    if (close(fd) != 0) io_err = true;
    if (io_err) throw RsError(RS_E_INVALID, "write error");
    if (g_prof_env)
      fprintf(stderr, "[rs-prof] write_r1cs: device image %.1f MB built in %.2f ms, D2H + %d writers %.2f ms\n", dev_bytes / 1e6,
              t_built - t0, kThreads, now_ms() - t_built);
    E->stats.write_ms = now_ms() - t0;
    return RS_OK;
  } catch (const RsError &e) {
    set_error(e.what());
    return e.code;
  } catch (const std::exception &e) {
    set_error(e.what());
    return RS_E_INTERNAL;
  }
}

void *rs_host_alloc(uint64_t bytes) {
  void *p = nullptr;
  if (hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) return nullptr;
  return p;
}
void rs_host_free(void *p) {
  if (p) (void)hipHostFree(p);
}

void rs_output_free(rs_output *o) {
  if (!o) return;
  free_lc(o->a);
  free_lc(o->b);
  free_lc(o->c);
  free(o->label_to_wire);
  free(o->log_from);
  free_lc(o->log_to);
  free(o->a_len);
  free(o->b_len);
  free(o->c_len);
  free(o->a_jump);
  free(o->b_jump);
  free(o->c_jump);
  free(o);
}

// ------------------------------------------------------------------ multi-GPU (sharded elimination)
struct rs_group {
  rs::LocalGroup g;
  explicit rs_group(int w) : g(w) {}
};

int rs_comm_unique_id(uint8_t id[RS_COMM_ID_BYTES]) {
  static_assert(sizeof(ncclUniqueId) == RS_COMM_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId u;
  ncclResult_t r = ncclGetUniqueId(&u);
  if (r != ncclSuccess) { set_error(std::string("ncclGetUniqueId: ") + ncclGetErrorString(r)); return RS_E_RCCL; }
  memcpy(id, &u, RS_COMM_ID_BYTES);
  return RS_OK;
}

int rs_engine_join_rccl(rs_engine *E, int world, int rank, const uint8_t id[RS_COMM_ID_BYTES]) {
  try {
    if (world < 1 || world > 255 || rank < 0 || rank >= world) { set_error("bad world/rank"); return RS_E_INVALID; }
    HC(hipSetDevice(E->device));
    ncclUniqueId u;
    memcpy(&u, id, RS_COMM_ID_BYTES);
    ncclComm_t c = nullptr;
    NC(ncclCommInitRank(&c, world, u, rank));
    E->comm.reset(new RcclComm(c, rank, world));
    return RS_OK;
  } catch (const RsError &e) {
    set_error(e.what());
    return e.code;
  } catch (const std::exception &e) {
    set_error(e.what());
    return RS_E_INTERNAL;
  }
}

int rs_engine_join_host(rs_engine *E, int world, int rank, const char *tag) {
  try {
    if (!E || !tag || world < 1 || world > 255 || rank < 0 || rank >= world) { set_error("bad world/rank/tag"); return RS_E_INVALID; }
    HC(hipSetDevice(E->device));
    E->comm.reset(new HostComm(world, rank, tag));
    return RS_OK;
  } catch (const RsError &e) {
    set_error(e.what());
    return e.code;
  } catch (const std::exception &e) {
    set_error(e.what());
    return RS_E_INTERNAL;
  }
}

int rs_engine_inject_fault(rs_engine *E, int where) {
  if (!E || where < 0 || where > 1) { set_error("rs_engine_inject_fault: bad argument"); return RS_E_INVALID; }
  E->fault_at = where;
  return RS_OK;
}

rs_group *rs_group_create(int world) {
  if (world < 1 || world > 255) return nullptr;
  return new rs_group(world);
}
void rs_group_destroy(rs_group *g) { delete g; }

int rs_engine_join_group(rs_engine *E, rs_group *g, int rank) {
  if (!g || rank < 0 || rank >= g->g.world) { set_error("bad group/rank"); return RS_E_INVALID; }
  E->comm.reset(new LocalComm(&g->g, rank));
  return RS_OK;
}

int rs_simplify_multi(const rs_input *in, const rs_flags *fl, int n_dev, const int *devices, rs_output **out) {
  if (n_dev < 1 || n_dev > 255 || !devices) { set_error("bad device list"); return RS_E_INVALID; }
  if (n_dev == 1) {
    rs_flags f = *fl;
    f.device = devices[0];
    return rs_simplify(in, &f, out);
  }
  std::vector<rs_engine *> eng(n_dev, nullptr);
  int rc = RS_OK;
  for (int r = 0; r < n_dev && !rc; ++r) rc = rs_engine_create(devices[r], &eng[r]);
  bool distinct = true;
  for (int r = 0; r < n_dev; ++r)
    for (int q = 0; q < r; ++q) distinct &= devices[q] != devices[r];
  std::unique_ptr<rs_group> grp;
  if (!rc) {
    if (distinct) {  // RCCL: one communicator per device, created together
      try {
        std::vector<ncclComm_t> comms(n_dev);
        NC(ncclCommInitAll(comms.data(), n_dev, devices));
        for (int r = 0; r < n_dev; ++r) eng[r]->comm.reset(new RcclComm(comms[r], r, n_dev));
      } catch (const RsError &e) {
        set_error(e.what());
        rc = e.code;
      }
    } else {
      grp.reset(new rs_group(n_dev));
      for (int r = 0; r < n_dev; ++r) eng[r]->comm.reset(new LocalComm(&grp->g, r));
    }
  }
  std::vector<int> rcs(n_dev, RS_OK);
  std::vector<std::string> errs(n_dev);
  if (!rc) {
    std::vector<std::thread> th;
    for (int r = 0; r < n_dev; ++r)
      th.emplace_back([&, r] {
        rs_flags f = *fl;
        f.device = devices[r];
        int x = rs_engine_load(eng[r], in);
        if (!x) x = rs_engine_run(eng[r], &f);
        if (!x && r == 0) x = rs_engine_fetch(eng[r], out);
        rcs[r] = x;
        if (x) errs[r] = rs_last_error();
      });
    for (auto &t : th) t.join();
    for (int r = 0; r < n_dev && !rc; ++r)
      if (rcs[r]) { rc = rcs[r]; set_error("rank " + std::to_string(r) + ": " + errs[r]); }
  }
  for (auto *E : eng) rs_engine_destroy(E);
  return rc;
}

int rs_flatten_dag(int device, const rs_dag *dag, rs_input **in) {
  if (!dag || !in) { set_error("rs_flatten_dag: null argument"); return RS_E_INVALID; }
  *in = nullptr;
  rs_engine *E = nullptr;
  int rc = rs_engine_create(device, &E);
  if (rc) return rc;
  rs_input *o = (rs_input *)calloc(1, sizeof(rs_input));
  try {
    HC(hipSetDevice(E->device));
    flatten_dag(E, dag, o, [](int, size_t bytes) {  // malloc'ed like rs_read_r1cs_o0's (rs_input_free)
      void *p = malloc(bytes ? bytes : 1);
      if (!p) throw std::bad_alloc();
      return p;
    });
    *in = o;
    o = nullptr;
    rc = RS_OK;
  } catch (const RsError &e) {
    set_error(e.what());
    rc = e.code;
  } catch (const std::exception &e) {
    set_error(e.what());
    rc = RS_E_INTERNAL;
  }
  if (o) rs_input_free(o);  // a failed call: the arrays made so far (calloc'ed struct: NULL elsewhere)
  rs_engine_destroy(E);
  return rc;
}

int rs_engine_flatten_dag(rs_engine *E, const rs_dag *dag, const rs_input **in) {
  CpuNear cpu_near_(E);  // the caller's affinity is restored on return
  if (!E || !dag || !in) { set_error("rs_engine_flatten_dag: null argument"); return RS_E_INVALID; }
  *in = nullptr;
  try {
    HC(hipSetDevice(E->device));
    snap_join(E);  // no D2H of an earlier result still reads the engine's buffers
    E->flat_view = rs_input{};
    flatten_dag(E, dag, &E->flat_view, [E](int slot, size_t bytes) { return pin_get(E, 20 + slot, bytes); });
    *in = &E->flat_view;
    return RS_OK;
  } catch (const RsError &e) {
    set_error(e.what());
    return e.code;
  } catch (const std::exception &e) {
    set_error(e.what());
    return RS_E_INTERNAL;
  }
}

int rs_simplify(const rs_input *in, const rs_flags *fl, rs_output **out) {
  rs_engine *E = nullptr;
  int rc = rs_engine_create(fl->device, &E);
  if (rc) return rc;
  rc = rs_engine_load(E, in);
  if (!rc) rc = rs_engine_run(E, fl);
  if (!rc) rc = rs_engine_fetch(E, out);
  rs_engine_destroy(E);
  return rc;
}

}  // extern "C"
