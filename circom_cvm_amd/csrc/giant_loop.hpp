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
// The loop of one component runs in one workgroup of kGiNW waves.  A merge `work = c2*work - c*R`
// packs the work list (positions [0, len)) and the holder's right-hand side ([len, len + rl)) one
// entry per lane -- a 72-entry merge of the configs[1] component costs one 256-bit product latency
// instead of two per lane (the one-wave loop's register merge) -- each side binary-searches the
// other in LDS, and a block scan of the keep flags places the survivors.  Per-signal state is one
// u64 word in HBM (gst: forbidden / occurrence count / deleted + the holder's pool header offset), so
// a holder is one round trip (its header and right-hand side are contiguous in the pool, k_big_prep
// and d_clear_nn write them so), and the states of a right-hand side's keys are loaded as they arrive
// and land under the product.  The official per-signal arrays (occ, del, holder_idx, the slot
// arrays) are kept current as well: rows or merges past the LDS capacity finish on one lane over them
// (d_gi_serial, d_treat_scalar's logic), and the composition kernels read them afterwards.
//
// Included by engine.hip after kernels.hpp, inside namespace rs.
#pragma once
#include "kernels.hpp"

namespace rs {

constexpr uint64_t kGiantRows = 11800;   // head clusters with this many rows take the giant path
constexpr uint32_t kGiCap = 256;         // LDS work-list capacity (entries); beyond it: one lane
constexpr int kGiNW = 4;                 // waves per workgroup (kGiT lanes)
constexpr uint32_t kGiT = 64 * kGiNW;
constexpr uint64_t kGiForb = ~0ull;      // gst: a forbidden signal
constexpr uint64_t kGiDel = 1ull << 63;  // gst: deleted; low bits = its holder's pool header offset (else: occurrences)
static_assert(kGiCap == kGiT, "one work position and one right-hand-side position per lane in the packed merge");

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
  uint32_t *scal;              // [0] components, [1] next component, [3] substitutions, [4] leftovers
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
// RS_PROF section clocks of k_gi_loop (thread 0's view; the barriers line the workgroup up with it)
#define GI_SEC(i)                                    \
  do {                                               \
    if (G.sec && tid == 0) {                         \
      const unsigned long long now_ = clock64();     \
      sec_acc[i] += now_ - sec_t;                    \
      sec_t = now_;                                  \
    }                                                \
  } while (0)

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
      if (A.del[s]) st = kGiDel | (A.h_off[A.holder_idx[s]] - 1);  // k_big_prep / d_clear_nn: header before the RHS
      else st = A.occ[s] < 0 ? 0ull : (uint64_t)A.occ[s];         // process_3 keeps no counts
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
                                   unsigned long long &by) {
  const FieldP &F = A.F;
  for (;;) {
    if (len == 0) return true;
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
    by += 36ull * (len + A.h_len[hi]);
    if (!d_merge(A, al, k, v, len, oi, fneg(F, v[oi]), A.h_coef[hi], A.h_off[hi], A.h_len[hi], w_off, w_len)) return false;
    k = A.pk + w_off;
    v = A.pv + w_off;
    len = w_len;
    by += 36ull * len;
  }
}

struct GiSmem {
  uint32_t wk[2][kGiCap];
  uint64_t ws[2][kGiCap];
  Fe wv[2][kGiCap];
  uint32_t rk[kGiCap];
  uint64_t rs[kGiCap];
  Fe rv[kGiCap];
  uint32_t sc[2 * kGiCap + 1];  // exclusive scan of the packed positions' keep flags
  uint32_t lb[2 * kGiCap];      // per packed position: lower bound in the other list
  uint32_t wsum[2][kGiNW];
  uint32_t s_fdel[2], s_p3[2];
  unsigned long long s_best[2];
  uint32_t s_comp, s_ok, s_m, s_nl;
  uint64_t s_o;
};

// block exclusive scan of the flags of positions [0, 2 * kGiT) (f0: position tid, f1: tid + kGiT);
// writes sc[] and returns the total
__device__ __forceinline__ uint32_t gi_scan2(GiSmem &S, bool f0, bool f1, uint32_t tid) {
  const uint32_t lane = tid & 63, w = tid >> 6;
  const uint64_t lt = lane ? ((1ull << lane) - 1ull) : 0ull;
  const uint64_t b0 = __ballot(f0), b1 = __ballot(f1);
  if (lane == 0) { S.wsum[0][w] = (uint32_t)__popcll(b0); S.wsum[1][w] = (uint32_t)__popcll(b1); }
  __syncthreads();
  uint32_t base0 = 0, tot0 = 0, base1 = 0, tot1 = 0;
#pragma unroll
  for (int q = 0; q < kGiNW; ++q) {
    const uint32_t x0 = S.wsum[0][q], x1 = S.wsum[1][q];
    if (q < (int)w) { base0 += x0; base1 += x1; }
    tot0 += x0;
    tot1 += x1;
  }
  S.sc[tid] = base0 + (uint32_t)__popcll(b0 & lt);
  S.sc[kGiT + tid] = tot0 + base1 + (uint32_t)__popcll(b1 & lt);
  if (tid == 0) S.sc[2 * kGiT] = tot0 + tot1;
  __syncthreads();
  return tot0 + tot1;
}

template <int NW>
__global__ __launch_bounds__(64 * NW) void k_gi_loop(ElimArgs A, GiantArgs G, uint64_t c) {
  static_assert(NW == kGiNW, "GiSmem is sized for kGiNW waves");
  __shared__ GiSmem S;
  const FieldP &F = A.F;
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint64_t b = A.cl_off[c], e = A.cl_off[c + 1];
  const bool p4 = d_is_p4(A, (uint32_t)(e - b));
  const uint32_t n_uniq = A.n_sub[c];  // the uniques phase's substitutions (k_big_prep); the loop's follow
  Alloc al0;  // thread 0's pool chunk
  al0.chunk = 4096;
  unsigned long long by = 0;
  unsigned long long sec_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sec_t = G.sec ? clock64() : 0ull;
  uint32_t step = 0;  // reduction-slot parity
  if (tid == 0) { S.s_ok = 1; S.s_fdel[0] = S.s_fdel[1] = RS_NONE; S.s_best[0] = S.s_best[1] = ~0ull; S.s_p3[0] = S.s_p3[1] = 0; }
  for (;;) {
    __syncthreads();
    if (tid == 0) S.s_comp = atomicAdd(&G.scal[1], 1u);
    __syncthreads();
    const uint32_t kc = S.s_comp;
    if (kc >= G.scal[0] || !S.s_ok) break;
    const uint32_t comp = G.cidx2[kc];
    const uint32_t start = G.c_start[comp], size = G.c_size[comp];
    const uint64_t sub_base = b + n_uniq + start, left_base = b + start;
    if (tid == 0) { S.s_m = 0; S.s_nl = 0; }
    const uint64_t clk0 = G.c_clk ? wall_clock64() : 0;
    uint32_t n_merge = 0;
    __syncthreads();
    for (uint32_t ii = start + size; ii-- > start;) {  // pop order: descending position (Vec::pop)
      if (!S.s_ok) break;
      const uint32_t qi = G.rval2[ii];
      const uint64_t r_off = A.row_off[b + qi];
      uint32_t len = A.row_len[b + qi];
      const uint32_t *rk0 = A.rows.key + r_off;
      const Fe *rv0 = A.rows.val + r_off;
      by += 36ull * len;
      if (len > kGiCap) {  // remove_constraint on the global state, then one lane
        for (uint32_t i = tid; i < len; i += kGiT) {
          const uint32_t s = rk0[i];
          const uint64_t st = G.gst[s];
          if (p4 && st != kGiForb && !(st & kGiDel) && st > 0) { G.gst[s] = st - 1; A.occ[s] = (int32_t)(st - 1); }
        }
        __syncthreads();
        if (tid == 0) {
          uint32_t m = S.s_m, nl = S.s_nl;
          if (!d_gi_serial(A, G, al0, sub_base, left_base, qi, rk0, rv0, len, m, nl, p4, by)) S.s_ok = 0;
          S.s_m = m;
          S.s_nl = nl;
        }
        __syncthreads();  // thread 0's stores (state words, holders) before the next row reads them
        continue;
      }
      uint32_t cur = 0;
      if (tid < len) {  // the row and its keys' states; remove_constraint (:94-106): occurrences - 1
        const uint32_t s = rk0[tid];
        uint64_t st = G.gst[s];
        if (p4 && st != kGiForb && !(st & kGiDel) && st > 0) {
          st -= 1;
          G.gst[s] = st;
          A.occ[s] = (int32_t)st;
        }
        S.wk[0][tid] = s;
        S.wv[0][tid] = rv0[tid];
        S.ws[0][tid] = st;
      }
      __syncthreads();
      GI_SEC(6);
      while (len > 0) {
        // ---- the pivot: p4 take_signal_4 (:379-411) first deleted key (ascending), else fewest
        // occurrences, ties -> the largest id; p3 take_signal_3 (:368-377) the largest takeable key
        const uint32_t sl = step & 1, sn = sl ^ 1;
        ++step;
        {
          const uint64_t st = tid < len ? S.ws[cur][tid] : kGiForb;
          const bool tk = st != kGiForb, dl = tk && (st & kGiDel);
          const uint64_t dm = __ballot(dl), tm = __ballot(tk);
          const uint32_t w = tid >> 6;
          if (p4) {
            if (dm && lane == 0) atomicMin(&S.s_fdel[sl], 64u * w + (uint32_t)(__ffsll((long long)dm) - 1));
            unsigned long long v = (tk && !dl) ? ((st & 0xffffffffull) << 32) | (0xffffffffu - tid) : ~0ull;
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) {
              const unsigned long long x = __shfl_xor(v, d);
              v = x < v ? x : v;
            }
            if (lane == 0 && v != ~0ull) atomicMin(&S.s_best[sl], v);
          } else if (tm && lane == 0) {
            atomicMax(&S.s_p3[sl], 64u * w + (uint32_t)(64 - __clzll(tm)));  // 1 + the largest index
          }
          if (tid == 0) { S.s_fdel[sn] = RS_NONE; S.s_best[sn] = ~0ull; S.s_p3[sn] = 0; }
        }
        __syncthreads();
        GI_SEC(0);
        uint32_t oi = RS_NONE;
        if (p4) {
          const uint32_t fd = S.s_fdel[sl];
          const unsigned long long bs = S.s_best[sl];
          oi = fd != RS_NONE ? fd : (bs != ~0ull ? 0xffffffffu - (uint32_t)(bs & 0xffffffffull) : RS_NONE);
        } else {
          oi = S.s_p3[sl] ? S.s_p3[sl] - 1 : RS_NONE;
        }
        if (oi == RS_NONE) {  // no takeable key: a leftover, unnormalised (:325-327)
          if (tid == 0) { S.s_o = pool_alloc(A, al0, len); if (S.s_o == RS_NONE) S.s_ok = 0; }
          __syncthreads();
          by += 36ull * len;
          if (S.s_ok) {
            const uint64_t o = S.s_o;
            if (tid < len) { A.pk[o + tid] = S.wk[cur][tid]; A.pv[o + tid] = S.wv[cur][tid]; }
            if (tid == 0) {
              A.l_off[left_base + S.s_nl] = o;
              A.l_len[left_base + S.s_nl] = len;
              A.tmp[left_base + S.s_nl] = qi;
              S.s_nl = S.s_nl + 1;
            }
          }
          break;
        }
        const uint32_t p = S.wk[cur][oi];
        const uint64_t stp = S.ws[cur][oi];
        if (!(stp & kGiDel)) {  // a new substitution: (coefficient, p := rest) (clear_signal_not_normalized)
          const uint32_t sh = S.wk[cur][0] == 0 ? 0 : 1;  // {0: 0} is inserted when absent
          const uint32_t mm = len - 1 + sh;
          by += 36ull * mm;
          if (tid == 0) { S.s_o = pool_alloc(A, al0, (uint64_t)mm + 1); if (S.s_o == RS_NONE) S.s_ok = 0; }
          __syncthreads();
          if (S.s_ok) {
            const uint64_t o = S.s_o;
            if (tid < len && tid != oi) {
              const uint32_t q = (tid < oi ? tid : tid - 1) + sh;
              A.pk[o + 1 + q] = S.wk[cur][tid];
              A.pv[o + 1 + q] = S.wv[cur][tid];
            }
            if (tid == 0) {
              const Fe cf = fneg(F, S.wv[cur][oi]);
              if (sh) { A.pk[o + 1] = 0; A.pv[o + 1] = fe_zero(); }
              A.pk[o] = mm;  // the header: RHS length, coefficient
              A.pv[o] = cf;
              d_set_holder(A, p, sub_base + S.s_m, cf, o + 1, mm);
              S.s_m = S.s_m + 1;
              A.occ[p] = -1;
              A.del[p] = 1;
              G.gst[p] = kGiDel | o;
            }
          }
          break;
        }
        // ---- conflict with holder(p): work = c2*work - c*R (:338-347), c = -v_p
        const uint64_t hdr = stp & ~kGiDel;
        const uint32_t rl = A.pk[hdr];
        const Fe c2 = A.pv[hdr];
        if (rl > kGiCap || len + rl > kGiCap + 1) {  // the merged list could pass the LDS lists: one lane
          if (tid == 0) { S.s_o = pool_alloc(A, al0, len); if (S.s_o == RS_NONE) S.s_ok = 0; }
          __syncthreads();
          if (S.s_ok) {
            const uint64_t o = S.s_o;
            if (tid < len) { A.pk[o + tid] = S.wk[cur][tid]; A.pv[o + tid] = S.wv[cur][tid]; }
            __syncthreads();
            if (tid == 0) {
              uint32_t m = S.s_m, nl = S.s_nl;
              if (!d_gi_serial(A, G, al0, sub_base, left_base, qi, A.pk + o, A.pv + o, len, m, nl, p4, by)) S.s_ok = 0;
              S.s_m = m;
              S.s_nl = nl;
            }
          }
          break;
        }
        GI_SEC(1);
        // the right-hand side, one entry per lane, and its keys' states (they land under the product)
        uint64_t st_r = kGiForb;
        if (tid < rl) {
          const uint32_t key = A.pk[hdr + 1 + tid];
          S.rk[tid] = key;
          S.rv[tid] = A.pv[hdr + 1 + tid];
          st_r = G.gst[key];
        }
        const Fe coef = fneg(F, S.wv[cur][oi]);
        __syncthreads();
        GI_SEC(2);
        // packed positions: q < len the work entry q, else the RHS entry q - len; each searches the
        // other list and takes its one product
        bool hit0 = false, hit1 = false;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const uint32_t q = tid + h * kGiT;
          if (q >= len + rl) continue;
          bool hit;
          uint32_t lbq;
          if (q < len) {
            lbq = lds_lb_e<kGiCap / 64>(S.rk, rl, S.wk[cur][q], hit);
            S.wv[cur][q] = fmul256(F, c2, S.wv[cur][q]);
          } else {
            const uint32_t j = q - len;
            lbq = lds_lb_e<kGiCap / 64>(S.wk[cur], len, S.rk[j], hit);
            S.rv[j] = fmul256(F, coef, S.rv[j]);
          }
          S.lb[q] = lbq;
          if (h == 0) hit0 = hit; else hit1 = hit;
        }
        if (tid < rl) S.rs[tid] = st_r;
        __syncthreads();
        GI_SEC(3);
        bool keep0 = false, keep1 = false;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const uint32_t q = tid + h * kGiT;
          if (q >= len + rl) continue;
          const bool hit = h == 0 ? hit0 : hit1;
          bool keep;
          if (q < len) {  // -c2*v (+ c*rv when the RHS has the key)
            keep = false;
            if (q != oi) {
              const Fe pv = S.wv[cur][q];
              const Fe x = hit ? fsub(F, S.rv[S.lb[q]], pv) : fneg(F, pv);
              S.wv[cur][q] = x;
              keep = !fe_is_zero(x);
            }
          } else {  // RHS-only keys: c*rv
            keep = !hit && !fe_is_zero(S.rv[q - len]);
          }
          if (h == 0) keep0 = keep; else keep1 = keep;
        }
        const uint32_t nlen = gi_scan2(S, keep0, keep1, tid);
        GI_SEC(4);
        uint32_t tot_w = 0;
        {  // kept work entries = the scan at position len
          tot_w = S.sc[len];
        }
        const uint32_t nx = cur ^ 1;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const uint32_t q = tid + h * kGiT;
          const bool keep = h == 0 ? keep0 : keep1;
          if (!keep) continue;
          uint32_t pos;
          if (q < len) {
            const uint32_t l = S.lb[q];
            pos = S.sc[q] + (l < rl ? S.sc[len + l] - tot_w : nlen - tot_w);
            S.wk[nx][pos] = S.wk[cur][q];
            S.wv[nx][pos] = S.wv[cur][q];
            S.ws[nx][pos] = S.ws[cur][q];
          } else {
            const uint32_t j = q - len, l = S.lb[q];
            pos = (S.sc[q] - tot_w) + (l < len ? S.sc[l] : tot_w);
            S.wk[nx][pos] = S.rk[j];
            S.wv[nx][pos] = S.rv[j];
            S.ws[nx][pos] = S.rs[j];
          }
        }
        by += 36ull * (len + rl + nlen);
        ++n_merge;
        __syncthreads();
        GI_SEC(5);
        cur = nx;
        len = nlen;
      }
      __syncthreads();
    }
    __syncthreads();
    if (tid == 0) {
      G.c_nsub[comp] = S.s_m;
      G.c_nleft[comp] = S.s_nl;
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
  if (G.sec && tid == 0) {
    GI_SEC(7);
    for (int i = 0; i < 8; ++i) atomicAdd(G.sec + i, sec_acc[i]);
  }
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
