// giant_loop.hpp -- the ordered loop of process_3 / process_4 for clusters too large for the head's
// speculative loop (kGiantRows rows or more: BASELINE configs[1]'s 559 k-row cluster, the templated
// circuit's 2e5-row chain), split into independent components and run with 256-lane merges.
//
// Exactness of the split.  The loop (substitution_process_3/4 -> treat_constraint_3/4,
// simplification_utils.rs:143-185, 259-349, 368-411) keeps per-signal state only for TAKEABLE
// signals: deleted_symbols, the occurrence counts (SignalsInformation, :60-113) and the holders
// (SHNotNormalized, keyed by the deleted signal).  A row reads the state of its own takeable keys and
// of the keys its merges bring in -- a holder's right-hand side is a row of the same cluster -- so
// the rows of a cluster that share no takeable signal, directly or through other rows, never read
// each other's state: forbidden signals (public inputs, the constant) are passengers that are never
// counted, deleted or taken (take_signal_3/4 skip them).  build_clusters (constraint_simplification.rs
// :45-99) unions over every signal, forbidden ones included, so one public input touched by rows of
// many otherwise independent chains makes them one cluster (configs[1]: 1/64 of the rows touch one of
// 32 public inputs; its 559 k-row cluster is 63 k takeable components, the largest 100 k rows).
// Each component therefore runs the reference's loop on its own rows in the cluster's pop order
// (descending position), with the cluster's process_3 / process_4 decision (:548-553, made on the
// whole cluster's size), and produces exactly the substitutions and leftovers the whole loop produces
// for those rows.  The results merge back: substitutions are keyed by signal (the holder BTreeMap;
// every later step orders them by signal or by their dependency DAG, never by creation), and a
// leftover is pushed when its row is popped, so the cluster's leftover list is all components'
// leftovers by descending position (k_gi_compact*).
//
// The loop of one component runs in one workgroup: the work row in an LDS hash table (k_gi_loop
// below), a merge one 256-bit product latency and two barriers.  Per-signal state is one u64 word in
// HBM (gst: forbidden / occurrence count / deleted + the holder's pool header offset), so a holder
// is one round trip (its header and right-hand side are contiguous in the pool, k_big_prep and
// d_clear_nn write them so), and the states of a right-hand side's keys are loaded as they arrive
// and land under the product.  The official per-signal arrays (occ, del, holder_idx, the slot
// arrays) are kept current as well: rows or merges past the table's capacity finish on one lane over
// them (d_gi_serial, d_treat_scalar's logic), and the composition kernels read them afterwards.
//
// Included by engine.hip after kernels.hpp, inside namespace rs.
#pragma once
#include "kernels.hpp"

namespace rs {

constexpr uint64_t kGiantRows = 11800;   // head clusters with this many rows take the giant path
constexpr uint64_t kGiForb = ~0ull;      // gst: a forbidden signal
constexpr uint64_t kGiDel = 1ull << 63;  // gst: deleted; low bits = its holder's pool header offset (else: occurrences)
// err bit of a giant-path bounds violation (a table probe that finds no free slot, a slot / position /
// pool offset outside its cluster or the pool): the run fails with RS_E_INTERNAL instead of touching
// memory out of range.  None is reachable when the invariants hold; the guards keep a broken one from
// becoming an illegal access (round 5's scratch run s5i faulted in this path).
constexpr int kGiErrBounds = 128;

struct GiantArgs {
  uint64_t ci;                 // the cluster's position in the head list (A.big_alive / touch arrays)
  uint64_t n;                  // its rows (cl_off[c + 1] - cl_off[c])
  uint32_t *uf;                // per signal: union-find over takeable signals
  uint64_t *gst;               // per signal: state word
  uint64_t *rkey;              // per loop row: (component root << 32) | position, sorted into rkey2
  uint32_t *rval, *rval2;      // loop-row positions, sorted by rkey
  uint64_t *rkey2;
  uint32_t *comp_of;           // per sorted position: its component
  uint32_t *c_start, *c_size;  // per component: range in the sorted list
  uint64_t *ckey, *ckey2;      // components by size (largest first)
  uint32_t *cidx, *cidx2;
  uint32_t *c_nsub, *c_nleft;  // per component: substitutions / leftovers it made
  uint32_t *c_dsub;            // exclusive scan of c_nsub
  uint32_t *scal;              // [0] components, [1] next component, [3] substitutions, [4] leftovers, [5] merges
  uint32_t *t_sig;             // compaction temporaries (per substitution / per position)
  Fe *t_coef;
  uint64_t *t_off;
  uint32_t *t_len;
  uint32_t *lmark, *lscan;     // per position: a leftover popped there, its exclusive scan
  uint64_t *tl_off;
  uint32_t *tl_len;
  uint32_t *c_merges;          // RS_PROF: per component, merges and wall-clock ticks (100 MHz), else null
  uint64_t *c_clk;
  unsigned long long *sec;     // RS_PROF: shader clocks per loop section, summed over the workgroups
};
// Section clocks of k_gi_loop (-DRS_GICLK builds, tools/kclk_build.sh RS_GICLK giclk): thread 0's
// view (the slots) and thread 129's (the right-hand side); the barriers line the workgroup up with them
#ifdef RS_GICLK
#define GI_SEC(i)                                    \
  do {                                               \
    if (G.sec && (tid == 0 || tid == 129)) {         \
      const unsigned long long now_ = clock64();     \
      sec_acc[i] += now_ - sec_t;                    \
      sec_t = now_;                                  \
    }                                                \
  } while (0)
#else
#define GI_SEC(i) \
  do {            \
  } while (0)
#endif

// ---- components: union-find over the takeable signals of every row of the cluster (dead rows
// included: a unique's holder carries its row's other keys into the rows that merge with it)
__global__ void k_gi_state(ElimArgs A, GiantArgs G, uint64_t c) {
  const uint64_t b = A.cl_off[c];
  for (uint64_t pos = gtid(); pos < G.n; pos += gstride()) {
    const uint32_t r = A.perm[b + pos];
    const uint32_t *k = A.rows.key + A.rows.off[r];
    const uint32_t len = A.rows.len[r];
    for (uint32_t i = 0; i < len; ++i) {
      const uint32_t s = k[i];
      if (A.forb[s]) { G.gst[s] = kGiForb; continue; }
      G.uf[s] = s;
      uint64_t st;
      if (A.del[s]) {  // k_big_prep / d_clear_nn: header before the RHS
        const int32_t hi = A.holder_idx[s];
        const uint64_t ho = hi >= 0 ? A.h_off[hi] : 0;
        if (hi < 0 || ho == 0 || ho > A.pool_cap) { atomicOr(A.err, kGiErrBounds); G.gst[s] = kGiForb; continue; }
        st = kGiDel | (ho - 1);
      } else st = A.occ[s] < 0 ? 0ull : (uint64_t)A.occ[s];         // process_3 keeps no counts
      G.gst[s] = st;
    }
  }
}

__global__ void k_gi_union(ElimArgs A, GiantArgs G, uint64_t c) {
  const uint64_t b = A.cl_off[c];
  for (uint64_t pos = gtid(); pos < G.n; pos += gstride()) {
    const uint32_t r = A.perm[b + pos];
    const uint32_t *k = A.rows.key + A.rows.off[r];
    const uint32_t len = A.rows.len[r];
    uint32_t first = RS_NONE;
    for (uint32_t i = 0; i < len; ++i) {
      const uint32_t s = k[i];
      if (A.forb[s]) continue;
      if (first == RS_NONE) { first = s; continue; }
      uint32_t x = first, y = s;
      for (;;) {  // k_eq_union's lock-free link: the larger root hooks under the smaller
        x = uf_find(G.uf, x);
        y = uf_find(G.uf, y);
        if (x == y) break;
        if (x > y) { const uint32_t t = x; x = y; y = t; }
        const uint32_t old = atomicCAS(&G.uf[y], y, x);
        if (old == y) break;
        y = old;
      }
    }
  }
}

// loop rows (positions [0, n_loop) of k_big_prep's row list) keyed by (component root, position);
// rows without a takeable key pop as leftovers and form one group of their own (root RS_NONE)
__global__ void k_gi_rowkey(ElimArgs A, GiantArgs G, uint64_t c) {
  const uint64_t b = A.cl_off[c];
  const uint32_t n_loop = A.big_alive[G.ci];
  for (uint64_t q = gtid(); q < G.n; q += gstride()) {
    uint64_t key = ~0ull;
    if (q < n_loop) {
      const uint32_t *k = A.rows.key + A.row_off[b + q];
      const uint32_t len = A.row_len[b + q];
      uint32_t root = RS_NONE;
      for (uint32_t i = 0; i < len; ++i)
        if (!A.forb[k[i]]) { root = uf_find(G.uf, k[i]); break; }
      key = ((uint64_t)root << 32) | q;
    }
    G.rkey[q] = key;
    G.rval[q] = (uint32_t)q;
  }
}

// component boundaries of the sorted row list (one workgroup): start / size / the position -> component
// map, the size-ordered keys of the components (padding sorts last), the per-component counters zeroed
__global__ __launch_bounds__(1024) void k_gi_segment(ElimArgs A, GiantArgs G) {
  __shared__ uint32_t part[1024];
  const uint32_t tid = threadIdx.x, nt = blockDim.x;
  const uint32_t n_loop = A.big_alive[G.ci];
  const uint32_t per = (n_loop + nt - 1) / nt, lo = min(n_loop, tid * per), hi = min(n_loop, lo + per);
  uint32_t cnt = 0;
  for (uint32_t i = lo; i < hi; ++i) cnt += (i == 0 || (G.rkey2[i] >> 32) != (G.rkey2[i - 1] >> 32)) ? 1u : 0u;
  part[tid] = cnt;
  __syncthreads();
  if (tid == 0) {
    uint32_t acc = 0;
    for (uint32_t t = 0; t < nt; ++t) { const uint32_t x = part[t]; part[t] = acc; acc += x; }
    G.scal[0] = acc;
    G.scal[1] = 0;
  }
  __syncthreads();
  uint32_t k = part[tid];
  for (uint32_t i = lo; i < hi; ++i) {
    if (i == 0 || (G.rkey2[i] >> 32) != (G.rkey2[i - 1] >> 32)) G.c_start[k++] = i;
    G.comp_of[i] = k - 1;
  }
  __syncthreads();
  const uint32_t n_comp = G.scal[0];
  for (uint64_t q = tid; q < G.n; q += nt) {
    if (q < n_comp) {
      const uint32_t e = q + 1 < n_comp ? G.c_start[q + 1] : n_loop;
      const uint32_t sz = e - G.c_start[q];
      G.c_size[q] = sz;
      G.ckey[q] = ((uint64_t)(0xffffffffu - sz) << 32) | q;
    } else {
      G.ckey[q] = ~0ull;
    }
    G.cidx[q] = (uint32_t)q;
    G.c_nsub[q] = 0;
    G.c_nleft[q] = 0;
    G.lmark[q] = 0;
  }
}

// ---- the serial continuation of a row past the LDS capacity (d_treat_scalar with the giant path's
// slot bases and the state word kept current)
__device__ inline bool d_gi_serial(const ElimArgs &A, const GiantArgs &G, Alloc &al, uint64_t sub_base, uint64_t left_base,
                                   uint32_t qi, const uint32_t *k, const Fe *v, uint32_t len, uint32_t &m, uint32_t &nl, bool p4,
                                   unsigned long long &by, uint64_t slot_end) {
  const FieldP &F = A.F;
  for (;;) {
    if (len == 0) return true;
    if (left_base + nl >= slot_end || sub_base + m >= slot_end) { atomicOr(A.err, kGiErrBounds); return false; }
    uint32_t oi = RS_NONE;
    int32_t occ_ret = -1;
    for (uint32_t i = 0; i < len; ++i) {
      const uint32_t s = k[i];
      if (A.forb[s]) continue;
      if (!p4) { oi = i; continue; }  // take_signal_3: the max takeable key (keys ascending)
      if (A.del[s]) { oi = i; break; }
      int32_t c2 = A.occ[s];
      if (c2 < 0) { atomicOr(A.err, 16); c2 = 0; }
      if (occ_ret < 0 || c2 < occ_ret) { oi = i; occ_ret = c2; }
      else if (c2 == occ_ret && k[oi] < s) oi = i;
    }
    if (oi == RS_NONE) {
      const uint64_t o = pool_alloc(A, al, len);
      if (o == RS_NONE) return false;
      for (uint32_t i = 0; i < len; ++i) { A.pk[o + i] = k[i]; A.pv[o + i] = v[i]; }
      A.l_off[left_base + nl] = o;
      A.l_len[left_base + nl] = len;
      A.tmp[left_base + nl] = qi;
      ++nl;
      by += 36ull * len;
      return true;
    }
    const uint32_t out = k[oi];
    const int32_t hi = A.holder_idx[out];
    if (!A.del[out] || hi < 0) {
      Fe coef;
      uint64_t to_off;
      uint32_t to_len;
      if (!d_clear_nn(A, al, k, v, len, oi, coef, to_off, to_len)) return false;
      d_set_holder(A, out, sub_base + m, coef, to_off, to_len);
      ++m;
      A.occ[out] = -1;
      A.del[out] = 1;
      G.gst[out] = kGiDel | (to_off - 1);
      by += 36ull * to_len;
      return true;
    }
    uint64_t w_off;
    uint32_t w_len;
    if (A.h_off[hi] + A.h_len[hi] > A.pool_cap) { atomicOr(A.err, kGiErrBounds); return false; }
    by += 36ull * (len + A.h_len[hi]);
    if (!d_merge(A, al, k, v, len, oi, fneg(F, v[oi]), A.h_coef[hi], A.h_off[hi], A.h_len[hi], w_off, w_len)) return false;
    k = A.pk + w_off;
    v = A.pv + w_off;
    len = w_len;
    by += 36ull * len;
  }
}

// ---- the component loop.  The work row lives in a kGhSlots-slot open-addressing table in LDS, one
// slot per lane of waves 0-1 (which keep their slot's key / value / state in registers).  A merge
// work = c2*work - c*R (:338-347) is two barriers: waves 2-3 load the holder's header and
// right-hand side (one entry per lane, one round trip: header and RHS are contiguous in the pool),
// multiply c*R and look each key up in the table -- a hit leaves its product in the slot's add
// cell, a miss claims a free slot -- while waves 0-1 multiply c2*work (one 256-bit product latency
// for the whole merge, no branch between the two products); after the first barrier every slot
// combines (hit ? c*R - c2*w : -c2*w, the reference's order of operations), drops the pivot and the
// cancelled keys (tombstones) and takes part in the next pivot's reduction (LDS atomics over
// key << 8 | slot: take_signal_4's first deleted key, take_signal_3's largest takeable key); the
// second barrier publishes it.  No scan and no sort inside the row: it is sorted once, by rank,
// when it leaves the loop (a new substitution's right-hand side, a leftover).  Rows longer than
// kGhRowMax and merges that could overflow the table finish on one lane (d_gi_serial) over the
// official per-signal arrays, which this path keeps current.
constexpr uint32_t kGhSlots = 128;
constexpr uint32_t kGhEmpty = 0xffffffffu, kGhTomb = 0xfffffffeu;  // above every signal id (< 2^31)
constexpr uint32_t kGhRowMax = 96;    // live entries the table takes (load <= 3/4)
constexpr uint32_t kGhRhsMax = 127;   // right-hand-side entries: lanes 1..127 of waves 2-3 (lane 0: the header)
constexpr uint32_t kGhUsedMax = 124;  // keys + tombstones before a merge's inserts; above it the table is rebuilt
constexpr uint32_t kGhThreads = 2 * kGhSlots;
static_assert(kGhUsedMax + 1 < kGhSlots && kGhRowMax + kGhRhsMax <= 2 * kGhSlots, "the table keeps an empty slot");

struct __attribute__((aligned(16))) GhSmem {
  uint32_t tk[kGhSlots];  // slot keys: kGhEmpty / kGhTomb / a signal
  Fe tv[kGhSlots];        // slot values (row start and rebuilds; the merges keep them in registers)
  uint64_t ts[kGhSlots];  // the key's state word (gst)
  Fe rv[kGhSlots];        // c*R of right-hand-side entry j (wave 3)
  uint32_t sj[kGhSlots];  // per slot: j + 1 of the right-hand-side entry that hit or claimed it (wave 2), else 0
  // per-wave reduction records of the two slot waves, by parity: the wave's pivot candidate
  // (key << 8 | slot, ~0 if none), its state word and value, live / used counts, key 0 present
  unsigned long long w_key[2][2];
  uint64_t w_st[2][2];
  Fe w_val[2][2];
  uint32_t w_live[2][2], w_used[2][2], w_has0[2][2];
  unsigned long long r_best;  // take_signal_4 without a deleted key: occurrences << 32 | ~key
  Fe s_pv;                    // that pivot's value
  uint64_t s_o;
  uint32_t s_ps, s_comp, s_ok, s_m, s_nl;
};

// values every lane holds alike (read from one LDS or global address) into scalar registers: the
// branches on them become scalar branches and the products take them as scalar operands
__device__ __forceinline__ uint32_t uni32(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ uint64_t uni64(uint64_t x) { return ((uint64_t)uni32((uint32_t)(x >> 32)) << 32) | uni32((uint32_t)x); }
__device__ __forceinline__ Fe uniFe(const Fe &a) {
  Fe r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r.l[i] = uni64(a.l[i]);
  return r;
}
__device__ __forceinline__ uint32_t gh_hash(uint32_t k) { return (k * 0x9E3779B1u) >> 25; }
__device__ __forceinline__ uint32_t gh_ld(const uint32_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// claims the first free (empty or tombstone) slot of K's probe sequence (the table always has one
// when the loads are bounded as below; a full table returns kGhEmpty and the caller flags the run)
__device__ __forceinline__ uint32_t gh_claim(GhSmem &S, uint32_t K) {
  uint32_t s = gh_hash(K);
  for (uint32_t i = 0; i < 4 * kGhSlots; ++i) {  // each failed CAS means another lane took a slot
    const uint32_t t = gh_ld(&S.tk[s]);
    if (t >= kGhTomb) {
      if (atomicCAS(&S.tk[s], t, K) == t) return s;
      continue;  // taken meanwhile: look at the slot again
    }
    s = (s + 1) & (kGhSlots - 1);
  }
  return kGhEmpty;
}
// the slot holding K, or kGhEmpty.  Keys are placed at the first free slot of their sequence and
// slots never become empty inside a row (only tombstones), so the first empty slot ends the search;
// concurrent claims only turn free slots into other keys.
__device__ __forceinline__ uint32_t gh_find(const GhSmem &S, uint32_t K) {
  uint32_t s = gh_hash(K);
  for (uint32_t i = 0; i < kGhSlots; ++i) {
    const uint32_t t = gh_ld(&S.tk[s]);
    if (t == K) return s;
    if (t == kGhEmpty) break;
    s = (s + 1) & (kGhSlots - 1);
  }
  return kGhEmpty;
}
// rank of `key` among the table's keys (empty / tombstone slots compare above every signal)
__device__ __forceinline__ uint32_t gh_rank(const GhSmem &S, uint32_t key) {
  uint32_t r = 0;
#pragma unroll 8
  for (uint32_t i = 0; i < kGhSlots; i += 4) {
    const uint4 k4 = *reinterpret_cast<const uint4 *>(&S.tk[i]);
    r += (k4.x < key ? 1u : 0u) + (k4.y < key ? 1u : 0u) + (k4.z < key ? 1u : 0u) + (k4.w < key ? 1u : 0u);
  }
  return r;
}
// a slot wave's share of a pivot reduction into set q: the wave's candidate by DPP (take_signal_4:
// the smallest deleted key; take_signal_3: the largest takeable key), written with its state and
// value by the lane that holds it, so the decision needs one LDS round trip and no atomics
__device__ __forceinline__ void gh_reduce(GhSmem &S, uint32_t q, bool p4, uint32_t slot, uint32_t wk, uint64_t wst, const Fe &wv) {
  const uint32_t w = slot >> 6;
  const bool live = wk < kGhTomb;
  const bool tk = live && wst != kGiForb;
  const uint32_t cand = p4 ? (tk && (wst & kGiDel) ? wk : kGhEmpty) : (tk ? ~wk : kGhEmpty);
  const uint32_t m = wave_min_u32(cand);
  if (m != kGhEmpty && cand == m) {
    S.w_key[q][w] = ((unsigned long long)wk << 8) | slot;
    S.w_st[q][w] = wst;
    S.w_val[q][w] = wv;
  }
  const uint64_t bl = __ballot(live), bu = __ballot(wk != kGhEmpty), b0 = __ballot(live && wk == 0);
  if ((slot & 63) == 0) {
    if (m == kGhEmpty) S.w_key[q][w] = ~0ull;
    S.w_live[q][w] = (uint32_t)__popcll(bl);
    S.w_used[q][w] = (uint32_t)__popcll(bu);
    S.w_has0[q][w] = b0 ? 1u : 0u;
  }
}

// A barrier over LDS only: the merge's two barriers publish LDS writes (slots, products, the
// reductions), never global stores, and __syncthreads()'s workgroup fence would also wait for every
// outstanding global load.
__device__ __forceinline__ void gh_lds_barrier() { __asm__ volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// thread 0's pool allocation in the loop: RS_NONE (and the run flagged) past the pool
__device__ __forceinline__ uint64_t gi_alloc(const ElimArgs &A, Alloc &al, uint64_t n) {
  const uint64_t o = pool_alloc(A, al, n);
  if (o != RS_NONE && o + n > A.pool_cap) { atomicOr(A.err, kGiErrBounds); return RS_NONE; }
  return o;
}

__global__ __launch_bounds__(kGhThreads) void k_gi_loop(ElimArgs A, GiantArgs G, uint64_t c) {
  __shared__ GhSmem S;
  const FieldP &F = A.F;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool wsd = tid < kGhSlots;  // waves 0-1: the table's slots; wave 2: lookups / claims; wave 3: c*R
  const uint32_t slot = tid;
  const uint64_t b = A.cl_off[c], e = A.cl_off[c + 1];
  const bool p4 = d_is_p4(A, (uint32_t)(e - b));
  const uint32_t n_uniq = A.n_sub[c];  // the uniques phase's substitutions (k_big_prep); the loop's follow
  Alloc al0;  // thread 0's pool chunk
  al0.chunk = 4096;
  unsigned long long by = 0;
#ifdef RS_GICLK
  unsigned long long sec_acc[16] = {}, sec_t = G.sec ? clock64() : 0ull;
#endif
  uint32_t q = 0;  // the reduction set the next decision reads
  uint32_t wk = kGhEmpty;  // (waves 0-1) the slot's key, value, state
  Fe wv = fe_zero();
  uint64_t wst = 0;
  if (tid == 0) S.s_ok = 1;
  if (wsd) S.sj[slot] = 0;
  for (;;) {
    __syncthreads();
    if (tid == 0) S.s_comp = atomicAdd(&G.scal[1], 1u);
    __syncthreads();
    const uint32_t kc = S.s_comp, n_comp = G.scal[0];
    if (kc >= n_comp || !S.s_ok) break;
    const uint32_t comp = G.cidx2[kc];
    const uint32_t n_loop = A.big_alive[G.ci];
    // the component's range of the sorted row list (uniform: every thread reads the same words)
    const uint32_t start = comp < n_comp ? G.c_start[comp] : 0u, size = comp < n_comp ? G.c_size[comp] : 0u;
    if (comp >= n_comp || (uint64_t)start + size > n_loop || (uint64_t)n_uniq + n_loop > e - b) {
      if (tid == 0) { S.s_ok = 0; atomicOr(A.err, kGiErrBounds); }
      break;
    }
    const uint64_t sub_base = b + n_uniq + start, left_base = b + start;
    if (tid == 0) { S.s_m = 0; S.s_nl = 0; }
    const uint64_t clk0 = G.c_clk ? wall_clock64() : 0;
    uint32_t n_merge = 0;
    __syncthreads();
    for (uint32_t ii = start + size; ii-- > start;) {  // pop order: descending position (Vec::pop)
      if (!S.s_ok) break;
      const uint32_t qi = G.rval2[ii];
      if (qi >= n_loop) {  // uniform
        if (tid == 0) { S.s_ok = 0; atomicOr(A.err, kGiErrBounds); }
        __syncthreads();
        break;
      }
      const uint64_t r_off = A.row_off[b + qi];
      const uint32_t len = A.row_len[b + qi];
      const uint32_t *rk0 = A.rows.key + r_off;
      const Fe *rv0 = A.rows.val + r_off;
      by += 36ull * len;
      if (len > kGhRowMax) {  // remove_constraint on the global state, then one lane
        for (uint32_t i = tid; i < len; i += kGhThreads) {
          const uint32_t s = rk0[i];
          const uint64_t st = G.gst[s];
          if (p4 && st != kGiForb && !(st & kGiDel) && st > 0) { G.gst[s] = st - 1; A.occ[s] = (int32_t)(st - 1); }
        }
        __syncthreads();
        if (tid == 0) {
          uint32_t m = S.s_m, nl = S.s_nl;
          if (!d_gi_serial(A, G, al0, sub_base, left_base, qi, rk0, rv0, len, m, nl, p4, by, e)) S.s_ok = 0;
          S.s_m = m;
          S.s_nl = nl;
        }
        __syncthreads();  // thread 0's stores (state words, holders) before the next row reads them
        GI_SEC(6);
        continue;
      }
      // ---- the row into the table; remove_constraint (:94-106): occurrences - 1
      if (wsd) S.tk[slot] = kGhEmpty;
      if (tid == 0) S.r_best = ~0ull;
      __syncthreads();
      if (tid < len) {
        const uint32_t s = rk0[tid];
        uint64_t st = G.gst[s];
        if (p4 && st != kGiForb && !(st & kGiDel) && st > 0) {
          st -= 1;
          G.gst[s] = st;
          A.occ[s] = (int32_t)st;
        }
        const uint32_t at = gh_claim(S, s);
        if (at != kGhEmpty) {
          S.tv[at] = rv0[tid];
          S.ts[at] = st;
        } else {
          atomicOr(A.err, kGiErrBounds);
        }
      }
      __syncthreads();
      if (wsd) {
        wk = S.tk[slot];
        if (wk < kGhTomb) { wv = S.tv[slot]; wst = S.ts[slot]; }
        gh_reduce(S, q, p4, slot, wk, wst, wv);
      }
      __syncthreads();
      GI_SEC(4);
      uint32_t pend_live = 0, pend_rl = 0;  // the merge whose bytes are counted once its result is known
      bool pend = false;
      for (;;) {
        // ---- the decision: set q's two wave records (one LDS round trip), into scalars
        const unsigned long long k0 = uni64(S.w_key[q][0]), k1 = uni64(S.w_key[q][1]);
        const uint64_t st0 = uni64(S.w_st[q][0]), st1 = uni64(S.w_st[q][1]);
        const Fe v0 = S.w_val[q][0], v1 = S.w_val[q][1];  // values stay per lane (vector registers): scalars are scarce
        const uint32_t live = uni32(S.w_live[q][0] + S.w_live[q][1]);
        const uint32_t used = uni32(S.w_used[q][0] + S.w_used[q][1]);
        const uint32_t has0 = uni32(S.w_has0[q][0] | S.w_has0[q][1]);
        q ^= 1;
        if (pend) by += 36ull * (pend_live + pend_rl + live);
        pend = false;
        if (live == 0) break;  // reduced to nothing: no substitution, no leftover
        // p4: the smaller key (~0: none); p3: the larger valid key
        const bool w1 = p4 ? k1 < k0 : (k0 == ~0ull || (k1 != ~0ull && k1 > k0));
        const unsigned long long kw = w1 ? k1 : k0;
        const uint64_t pst = w1 ? st1 : st0;
        const Fe pval = w1 ? v1 : v0;
        const bool any = kw != ~0ull;
        uint32_t ps = any ? (uint32_t)(kw & 255) : kGhEmpty;
        const bool merge = any && (pst & kGiDel) != 0;  // p4's candidates are deleted keys
        GI_SEC(0);
        if (merge) {
          // ---- conflict with holder(p): work = c2*work - c*R (:338-347), c = -v_p
          const uint64_t hdr = pst & ~kGiDel;
          if (hdr >= A.pool_cap) {  // uniform: a state word that points past the pool
            if (tid == 0) { S.s_ok = 0; atomicOr(A.err, kGiErrBounds); }
            __syncthreads();
            break;
          }
          // header and right-hand side in one round trip: waves 2-3 load before the length is known
          const bool rlane = !wsd && lane >= 1 && hdr + lane < A.pool_cap;
          uint32_t K = 0;
          Fe R = fe_zero();
          if (rlane) {
            if (wave == 2) K = A.pk[hdr + lane];
            R = A.pv[hdr + lane];
          }
          const uint32_t rl = uni32(A.pk[hdr]);
          if (hdr + 1 + (uint64_t)rl > A.pool_cap) {  // uniform
            if (tid == 0) { S.s_ok = 0; atomicOr(A.err, kGiErrBounds); }
            __syncthreads();
            break;
          }
          if (rl > kGhRhsMax || live - 1 + rl > kGhRowMax) {  // could pass the table: the rest on one lane
            if (tid == 0) { S.s_o = gi_alloc(A, al0, live); if (S.s_o == RS_NONE) S.s_ok = 0; }
            __syncthreads();
            if (S.s_ok) {
              const uint64_t o = S.s_o;
              if (wsd && wk < kGhTomb) {
                const uint32_t r = gh_rank(S, wk);
                if (r < live) {
                  A.pk[o + r] = wk;
                  A.pv[o + r] = wv;
                } else {
                  atomicOr(A.err, kGiErrBounds);
                }
              }
              __syncthreads();
              if (tid == 0) {
                uint32_t m = S.s_m, nl = S.s_nl;
                if (!d_gi_serial(A, G, al0, sub_base, left_base, qi, A.pk + o, A.pv + o, live, m, nl, p4, by, e)) S.s_ok = 0;
                S.s_m = m;
                S.s_nl = nl;
              }
            }
            __syncthreads();
            GI_SEC(6);
            break;
          }
          if (used + rl > kGhUsedMax) {  // tombstones: rebuild the table from the live slots
            const uint32_t kp = (uint32_t)(kw >> 8);
            if (wsd) S.tk[slot] = kGhEmpty;
            __syncthreads();
            if (wsd && wk < kGhTomb) {
              const uint32_t at = gh_claim(S, wk);
              if (at != kGhEmpty) {
                S.tv[at] = wv;
                S.ts[at] = wst;
              } else {
                atomicOr(A.err, kGiErrBounds);
              }
            }
            __syncthreads();
            if (wsd) {
              wk = S.tk[slot];
              if (wk < kGhTomb) { wv = S.tv[slot]; wst = S.ts[slot]; }
              if (wk == kp) S.s_ps = slot;
            }
            __syncthreads();
            ps = uni32(S.s_ps);
            GI_SEC(3);
          }
          Fe c2w;
          if (wave == 3) {  // c*R, entry j = lane (+ 64)
            const Fe coef = fneg(F, pval);
            for (uint32_t jj = lane; jj <= rl; jj += 64) {
              if (jj == 0) continue;
              const Fe Rj = jj == lane ? R : A.pv[hdr + jj];
              S.rv[jj] = fmul256(F, coef, Rj);
            }
          } else if (wave == 2) {  // each key into the table: a hit marks its slot, a miss claims one
            for (uint32_t jj = lane; jj <= rl; jj += 64) {
              if (jj == 0) continue;
              const uint32_t Kj = jj == lane ? K : A.pk[hdr + jj];
              const Fe Rj = jj == lane ? R : A.pv[hdr + jj];
              const uint64_t st_r = G.gst[Kj];
              const uint32_t at = gh_find(S, Kj);
              if (at != kGhEmpty) {
                S.sj[at] = jj + 1;
              } else if (!fe_is_zero(Rj)) {  // a zero-valued RHS key ({0: 0}) only ever adds into the row
                const uint32_t f = gh_claim(S, Kj);
                if (f != kGhEmpty) {
                  S.ts[f] = st_r;
                  S.sj[f] = jj + 1;
                } else {
                  atomicOr(A.err, kGiErrBounds);
                }
              }
            }
          } else if (wk < kGhTomb && slot != ps) {
            c2w = fmul256(F, A.pv[hdr], wv);
          }
          gh_lds_barrier();
          GI_SEC(1);
          if (wsd) {
            const uint32_t sjv = S.sj[slot];
            if (sjv) S.sj[slot] = 0;
            if (wk < kGhTomb) {
              bool drop = slot == ps;
              if (!drop) {
                const Fe x = sjv ? fsub(F, S.rv[sjv - 1], c2w) : fneg(F, c2w);
                drop = fe_is_zero(x);
                wv = x;
              }
              if (drop) {
                S.tk[slot] = kGhTomb;
                wk = kGhTomb;
              }
            } else if (sjv) {  // a key the right-hand side brought in
              wk = S.tk[slot];
              wst = S.ts[slot];
              wv = S.rv[sjv - 1];
            }
            gh_reduce(S, q, p4, slot, wk, wst, wv);
          }
          ++n_merge;
          pend = true;
          pend_live = live;
          pend_rl = rl;
          gh_lds_barrier();
          GI_SEC(2);
          continue;
        }
        // ---- the row leaves the loop
        uint32_t kp = any ? (uint32_t)(kw >> 8) : 0u;
        Fe wpv = pval;
        if (p4) {  // take_signal_4 without a deleted key: fewest occurrences, ties -> the largest id
          if (wsd && wk < kGhTomb && wst != kGiForb)
            atomicMin(&S.r_best, ((wst & 0xffffffffull) << 32) | (0xffffffffu - wk));
          __syncthreads();
          const unsigned long long best = uni64(S.r_best);
          if (best != ~0ull) {
            kp = 0xffffffffu - (uint32_t)(best & 0xffffffffull);
            if (wsd && wk == kp) { S.s_ps = slot; S.s_pv = wv; }
            __syncthreads();
            ps = uni32(S.s_ps);
            wpv = uniFe(S.s_pv);
          }
        }
        if (ps == kGhEmpty) {  // no takeable key: a leftover, unnormalised (:325-327)
          by += 36ull * live;
          if (tid == 0) {
            S.s_o = left_base + S.s_nl < e ? gi_alloc(A, al0, live) : RS_NONE;
            if (S.s_o == RS_NONE) S.s_ok = 0;
            if (left_base + S.s_nl >= e) atomicOr(A.err, kGiErrBounds);
          }
          __syncthreads();
          if (S.s_ok) {
            const uint64_t o = S.s_o;
            if (wsd && wk < kGhTomb) {
              const uint32_t r = gh_rank(S, wk);
              if (r < live) {
                A.pk[o + r] = wk;
                A.pv[o + r] = wv;
              } else {
                atomicOr(A.err, kGiErrBounds);
              }
            }
            if (tid == 0) {
              A.l_off[left_base + S.s_nl] = o;
              A.l_len[left_base + S.s_nl] = live;
              A.tmp[left_base + S.s_nl] = qi;
              S.s_nl = S.s_nl + 1;
            }
          }
        } else {  // a new substitution: (coefficient, p := rest) (clear_signal_not_normalized)
          const uint32_t sh = has0 ? 0u : 1u;  // {0: 0} is inserted when absent
          const uint32_t mm = live - 1 + sh;
          by += 36ull * mm;
          if (tid == 0) {
            S.s_o = sub_base + S.s_m < e ? gi_alloc(A, al0, (uint64_t)mm + 1) : RS_NONE;
            if (S.s_o == RS_NONE) S.s_ok = 0;
            if (sub_base + S.s_m >= e) atomicOr(A.err, kGiErrBounds);
          }
          __syncthreads();
          if (S.s_ok) {
            const uint64_t o = S.s_o;
            if (wsd && wk < kGhTomb && slot != ps) {
              const uint32_t r = gh_rank(S, wk) - (kp < wk ? 1u : 0u);
              if (sh + r < mm) {
                A.pk[o + 1 + sh + r] = wk;
                A.pv[o + 1 + sh + r] = wv;
              } else {
                atomicOr(A.err, kGiErrBounds);
              }
            }
            if (tid == 0) {
              const Fe cf = fneg(F, wpv);
              if (sh) { A.pk[o + 1] = 0; A.pv[o + 1] = fe_zero(); }
              A.pk[o] = mm;  // the header: RHS length, coefficient
              A.pv[o] = cf;
              d_set_holder(A, kp, sub_base + S.s_m, cf, o + 1, mm);
              S.s_m = S.s_m + 1;
              A.occ[kp] = -1;
              A.del[kp] = 1;
              G.gst[kp] = kGiDel | o;
            }
          }
        }
        __syncthreads();
        GI_SEC(5);
        break;
      }
    }
    __syncthreads();
    if (tid == 0) {
      G.c_nsub[comp] = S.s_m;
      G.c_nleft[comp] = S.s_nl;
      if (n_merge) atomicAdd(&G.scal[5], n_merge);
      if (G.c_clk) {
        G.c_clk[comp] = wall_clock64() - clk0;
        G.c_merges[comp] = n_merge;
      }
    }
  }
  __syncthreads();
  if (tid == 0) {
    if (!S.s_ok) atomicOr(A.err, 8);
  }
  // algorithmic bytes: one atomic per workgroup (thread 0 counted the lane-serial rows)
  by = tid == 0 ? by : 0ull;
  if (tid == 0 && by) atomicAdd(A.bytes_main, by);
#ifdef RS_GICLK
  if (G.sec && (tid == 0 || tid == 129)) {
    GI_SEC(7);
    for (int i = 0; i < 16; ++i) atomicAdd(G.sec + (tid ? 16 : 0) + i, sec_acc[i]);
  }
#endif
}

// ---- results back to the cluster's slots: substitutions contiguous after the uniques' (any order:
// holders are keyed by signal), leftovers by descending position (the order they were pushed)
__global__ void k_gi_gather(ElimArgs A, GiantArgs G, uint64_t c) {
  const uint64_t b = A.cl_off[c];
  const uint32_t n_loop = A.big_alive[G.ci], n_uniq = A.n_sub[c];
  for (uint64_t i = gtid(); i < n_loop; i += gstride()) {
    const uint32_t k = G.comp_of[i];
    const uint32_t li = (uint32_t)i - G.c_start[k];
    if (li < G.c_nsub[k]) {
      const uint64_t src = b + n_uniq + i, d = G.c_dsub[k] + li;
      G.t_sig[d] = A.h_sig[src];
      G.t_coef[d] = A.h_coef[src];
      G.t_off[d] = A.h_off[src];
      G.t_len[d] = A.h_len[src];
    }
    if (li < G.c_nleft[k]) {
      const uint32_t qi = A.tmp[b + i];
      if (qi >= n_loop) { atomicOr(A.err, kGiErrBounds); continue; }
      G.tl_off[qi] = A.l_off[b + i];
      G.tl_len[qi] = A.l_len[b + i];
      G.lmark[qi] = 1;
    }
  }
}
__global__ void k_gi_scatter(ElimArgs A, GiantArgs G, uint64_t c) {
  const uint64_t b = A.cl_off[c];
  const uint32_t n_loop = A.big_alive[G.ci], n_uniq = A.n_sub[c];
  const uint32_t n_comp = G.scal[0];
  const uint32_t n_subs = n_comp ? G.c_dsub[n_comp - 1] + G.c_nsub[n_comp - 1] : 0u;
  const uint32_t n_left = n_loop ? G.lscan[n_loop - 1] + G.lmark[n_loop - 1] : 0u;
  for (uint64_t j = gtid(); j < n_loop; j += gstride()) {
    if (j < n_subs) {
      const uint64_t d = b + n_uniq + j;
      const uint32_t s = G.t_sig[j];
      A.h_sig[d] = s;
      A.h_coef[d] = G.t_coef[j];
      A.h_off[d] = G.t_off[j];
      A.h_len[d] = G.t_len[j];
      A.holder_idx[s] = (int32_t)d;
    }
    if (G.lmark[j]) {  // position j: its leftover goes after those of the higher positions
      const uint64_t d = b + (n_left - 1 - G.lscan[j]);
      A.l_off[d] = G.tl_off[j];
      A.l_len[d] = G.tl_len[j];
    }
  }
  if (gtid() == 0) {
    G.scal[3] = n_subs;
    G.scal[4] = n_left;
  }
}
__global__ void k_gi_fin(ElimArgs A, GiantArgs G, uint64_t c) {
  if (gtid() != 0) return;
  A.n_sub[c] = A.n_sub[c] + G.scal[3];
  A.n_left[c] = G.scal[4];
}

}  // namespace rs
