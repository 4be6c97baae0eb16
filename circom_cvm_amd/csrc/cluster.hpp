// cluster.hpp -- build_clusters (constraint_list/src/constraint_simplification.rs:45-99) on the device.
//
// The reference walks the linear rows in list order; row j gets arena slot j and, for each of its
// signals s (canonical order: ascending), merges the cluster of prev(s) -- the last earlier row
// holding s -- into its own: merged = [j's list] ++ [that cluster's list] (Cluster::merge, :32-38).
// Because the destination is always the newest row, the root of every cluster is its maximum row
// index, which gives the device formulation:
//   1. pairs (s, j) sorted by (s, j)            -> prev(s, j) and a union-find over rows;
//   2. cluster of a row = max row of its component; clusters are emitted in ascending max row
//      (arena order, :90-97) and a cluster's rows are first listed by ascending index;
//   3. the list order inside a cluster is the replay of the arena merges restricted to that cluster
//      (clusters are independent): one lane per small cluster, one workgroup with LDS-resident u16
//      state per large cluster, the lane-serial global-memory replay beyond the LDS capacity.
#pragma once
#include "kernels.hpp"

namespace rs {

constexpr uint32_t kClRowBit = 0x80000000u;  // stream entry: first pair of a row
constexpr uint32_t kClNoPrev = 0x7fffffffu;
constexpr uint32_t kClSmall = 64;     // clusters up to this size: one lane each
constexpr uint32_t kClLds = 32768;    // clusters up to this size: LDS replay (u16 local ids)
constexpr uint32_t kClChunk = 4096;   // stream entries staged per LDS chunk
constexpr uint32_t kClMid = 2048;     // mid-size clusters: replay with a small LDS footprint
constexpr uint32_t kWaveMin = 32;     // clusters from this size on are eliminated by the workgroup kernels

// pairs per row (non-constant keys) and the active-row statistics
__global__ void k_cl_count(DRows V, uint64_t *npairs, unsigned long long *stat /* [0] nnz, [1] active */) {
  unsigned long long nnz = 0, act = 0;
  for (uint64_t r = gtid(); r < V.n; r += gstride()) {
    uint32_t len = V.len[r];
    npairs[r] = len - (len && V.key[V.off[r]] == 0 ? 1 : 0);
    nnz += len;
    act += len ? 1 : 0;
  }
  wave_atomic_add(&stat[0], nnz);  // launched on a capped grid: few waves, few atomics
  wave_atomic_add(&stat[1], act);
}
__global__ void k_cl_fill(DRows V, const uint64_t *poff, uint64_t *pkey, uint32_t *pslot) {
  for (uint64_t r = gtid(); r < V.n; r += gstride()) {
    uint64_t o = poff[r];
    const uint32_t *k = V.key + V.off[r];
    for (uint32_t i = 0; i < V.len[r]; ++i) {
      if (k[i] == 0) continue;
      pkey[o] = ((uint64_t)k[i] << 32) | r;
      pslot[o] = (uint32_t)o;
      ++o;
    }
  }
}
__device__ inline void uf_union(uint32_t *uf, uint32_t a, uint32_t b) {
  for (;;) {
    a = uf_find(uf, a);
    b = uf_find(uf, b);
    if (a == b) return;
    if (a > b) { uint32_t t = a; a = b; b = t; }
    uint32_t old = atomicCAS(&uf[b], b, a);
    if (old == b) return;
    b = old;
  }
}
// prev(s, j) from the sorted pairs; rows sharing a signal are joined.  A row holding a non-forbidden
// signal that no other row of the list holds is marked: process_4 consumes such rows in its uniques
// phase, independently of their order (simplification_utils.rs:166-172).
__global__ void k_cl_link(const uint64_t *pk, const uint32_t *ps, uint64_t P, uint32_t *prevrow, uint32_t *uf,
                          const uint8_t *forb, uint8_t *has_unique) {
  for (uint64_t i = gtid(); i < P; i += gstride()) {
    uint64_t x = pk[i];
    if ((i == 0 || (pk[i - 1] >> 32) != (x >> 32)) && (i + 1 == P || (pk[i + 1] >> 32) != (x >> 32)) &&
        !forb[x >> 32])
      has_unique[(uint32_t)x] = 1;
    if (i > 0 && (pk[i - 1] >> 32) == (x >> 32)) {
      uint32_t p = (uint32_t)pk[i - 1];
      prevrow[ps[i]] = p;
      uf_union(uf, p, (uint32_t)x);
    } else {
      prevrow[ps[i]] = RS_NONE;
    }
  }
}
__global__ void k_cl_root(const uint32_t *len, uint64_t n, uint32_t *uf, int32_t *cmax) {
  for (uint64_t r = gtid(); r < n; r += gstride())
    if (len[r]) atomicMax(&cmax[uf_find(uf, (uint32_t)r)], (int32_t)r);
}
__global__ void k_cl_key(const uint32_t *len, uint64_t n, uint32_t *uf, const int32_t *cmax, uint64_t *rkey,
                         uint32_t *ridx) {
  for (uint64_t r = gtid(); r < n; r += gstride()) {
    rkey[r] = len[r] ? ((uint64_t)(uint32_t)cmax[uf_find(uf, (uint32_t)r)] << 32) | r : ~0ull;
    ridx[r] = (uint32_t)r;
  }
}
__global__ void k_cl_flag(const uint64_t *rkey, uint64_t n_act, uint64_t *flag) {
  for (uint64_t i = gtid(); i < n_act; i += gstride())
    flag[i] = (i == 0 || (rkey[i] >> 32) != (rkey[i - 1] >> 32)) ? 1 : 0;
}
// cluster starts, cluster of each position, position of each row, pair counts in cluster order
__global__ void k_cl_starts(const uint64_t *rkey, const uint64_t *fscan, const uint32_t *srow, const uint64_t *npairs,
                            uint64_t n_act, uint64_t n_cl, uint64_t *cl_off, uint32_t *cid, uint32_t *gpos, uint64_t *qn,
                            const uint8_t *has_unique, uint32_t *n_ordered) {
  for (uint64_t i = gtid(); i < n_act; i += gstride()) {
    bool st = i == 0 || (rkey[i] >> 32) != (rkey[i - 1] >> 32);
    uint64_t c = fscan[i] + (st ? 1 : 0) - 1;
    if (st) cl_off[c] = i;
    if (i == 0) cl_off[n_cl] = n_act;
    cid[i] = (uint32_t)c;
    uint32_t j = srow[i];
    gpos[j] = (uint32_t)i;
    qn[i] = npairs[j];
    if (!has_unique[j]) atomicAdd(&n_ordered[c], 1u);  // rows whose order matters to process_4
  }
}
// process_4 cluster (:548-553) whose every row is consumed by the uniques phase: any order is exact
__device__ __forceinline__ bool d_cl_order_free(uint32_t n, int old_heur, const uint32_t *n_ordered, uint64_t c) {
  return n >= 350 && n < 1000000 && !old_heur && n_ordered[c] == 0;
}
// the per-cluster replay stream: local id of prev(s, j) for each pair, rows in ascending index
__global__ void k_cl_stream(const uint32_t *srow, const uint64_t *poff, const uint32_t *prevrow, const uint32_t *gpos,
                            const uint32_t *cid, const uint64_t *cl_off, const uint64_t *q_off, uint64_t n_act,
                            uint32_t *stream) {
  for (uint64_t i = gtid(); i < n_act; i += gstride()) {
    uint32_t j = srow[i];
    uint64_t base = cl_off[cid[i]], q = q_off[i], np = q_off[i + 1] - q, o = poff[j];
    for (uint64_t t = 0; t < np; ++t) {
      uint32_t p = prevrow[o + t];
      uint32_t loc = p == RS_NONE ? kClNoPrev : (uint32_t)(gpos[p] - base);
      stream[q + t] = loc | (t == 0 ? kClRowBit : 0u);
    }
  }
}

// lane replay (small clusters, and the global-memory path beyond the LDS capacity)
__global__ void k_cl_replay_lane(const uint64_t *cl_off, uint64_t n_cl, const uint64_t *q_off, const uint32_t *stream,
                                 const uint32_t *srow, uint32_t *c2c, uint32_t *tail, uint32_t *next, uint32_t *perm,
                                 const uint32_t *n_ordered, int old_heur) {
  for (uint64_t c = gtid(); c < n_cl; c += gstride()) {
    const uint64_t b = cl_off[c];
    const uint32_t n = (uint32_t)(cl_off[c + 1] - b);
    if (n > kClSmall && n <= kClLds) continue;
    if (d_cl_order_free(n, old_heur, n_ordered, c)) {
      for (uint32_t t = 0; t < n; ++t) perm[b + t] = srow[b + t];
      continue;
    }
    uint32_t *C2 = c2c + b, *T = tail + b, *N = next + b;
    for (uint32_t t = 0; t < n; ++t) {
      C2[t] = t;
      T[t] = t;
      N[t] = RS_NONE;
      for (uint64_t q = q_off[b + t]; q < q_off[b + t + 1]; ++q) {
        uint32_t p = stream[q] & ~kClRowBit;
        if (p == kClNoPrev) continue;
        while (C2[p] != p) { uint32_t g = C2[C2[p]]; C2[p] = g; p = g; }  // path halving
        if (p == t) continue;
        N[T[t]] = p;
        T[t] = T[p];
        C2[p] = t;
      }
    }
    uint32_t x = n - 1, q = 0;
    while (x != RS_NONE) { perm[b + q++] = srow[b + x]; x = N[x]; }
  }
}

// workgroup replay with the union-find state in LDS (kClSmall < n <= CAP); `ids` lists them.  Two
// instantiations: CAP = kClLds (150 KB of LDS, one workgroup per CU) for the large clusters and
// CAP = kClMid (small LDS footprint, many workgroups per CU) for the many mid-size ones.
template <uint32_t CAP, uint32_t CHUNK>
__global__ __launch_bounds__(256) void k_cl_replay_lds(const uint64_t *cl_off, const uint32_t *ids, uint64_t n_ids,
                                                       const uint64_t *q_off, const uint32_t *stream,
                                                       const uint32_t *srow, uint32_t *next, uint32_t *perm,
                                                       const uint32_t *n_ordered, int old_heur,
                                                       unsigned long long *prof = nullptr) {
  constexpr uint32_t kClChunk = CHUNK;
  __shared__ uint16_t C2[CAP], T[CAP];
  __shared__ uint32_t S[kClChunk];
  const uint32_t tid = threadIdx.x, nt = blockDim.x;
  for (uint64_t ci = blockIdx.x; ci < n_ids; ci += gridDim.x) {
    const uint64_t c = ids[ci];
    const uint64_t b = cl_off[c];
    const uint32_t n = (uint32_t)(cl_off[c + 1] - b);
    if (d_cl_order_free(n, old_heur, n_ordered, c)) {
      for (uint32_t i = tid; i < n; i += nt) perm[b + i] = srow[b + i];
      continue;
    }
    const uint64_t q0 = q_off[b], q1 = q_off[b + n];
    const unsigned long long t_0 = prof ? wall_clock64() : 0ull;
    uint32_t *N = next + b;
    int32_t t = -1;  // lane 0: current row
    uint32_t tail = 0;
    for (uint64_t qc = q0; qc < q1; qc += kClChunk) {
      const uint32_t m = (uint32_t)min<uint64_t>(kClChunk, q1 - qc);
      __syncthreads();
      for (uint32_t i = tid; i < m; i += nt) S[i] = stream[qc + i];
      __syncthreads();
      if (tid == 0) {
        // the current row's list tail lives in a register; T[] holds the tails of earlier roots
        for (uint32_t i = 0; i < m; ++i) {
          const uint32_t e = S[i];
          if (e & kClRowBit) {
            if (t >= 0) T[t] = (uint16_t)tail;
            ++t;
            C2[t] = (uint16_t)t;
            N[t] = RS_NONE;
            tail = (uint32_t)t;
          }
          uint32_t p = e & ~kClRowBit;
          if (p == kClNoPrev) continue;
          uint32_t q = C2[p];
          while (q != p) {  // path halving
            const uint32_t g = C2[q];
            C2[p] = (uint16_t)g;
            p = q == g ? q : g;
            q = C2[p];
          }
          if (p == (uint32_t)t) continue;
          N[tail] = p;
          tail = T[p];
          C2[p] = (uint16_t)t;
        }
      }
    }
    if (tid == 0 && t >= 0) T[t] = (uint16_t)tail;
    __syncthreads();
    // next -> LDS (C2 is free now), walk from the root (the last row), gather the rows
    for (uint32_t i = tid; i < n; i += nt) { uint32_t x = N[i]; C2[i] = (uint16_t)(x == RS_NONE ? 0xffffu : x); }
    __syncthreads();
    if (tid == 0) {
      uint32_t x = n - 1, q = 0;
      while (x != 0xffffu) { T[q++] = (uint16_t)x; x = C2[x]; }
    }
    __syncthreads();
    for (uint32_t i = tid; i < n; i += nt) perm[b + i] = srow[b + T[i]];
    if (prof && tid == 0) {  // RS_PROF: (cluster, rows, pairs, 100 MHz ticks)
      prof[4 * ci] = c;
      prof[4 * ci + 1] = n;
      prof[4 * ci + 2] = q1 - q0;
      prof[4 * ci + 3] = wall_clock64() - t_0;
    }
    __syncthreads();
  }
}

// One-wave replay (kClSmall < n <= CAP), the same arena merges as k_cl_replay_lds with the finds of a
// row done in parallel: the stream is read 64 entries at a time (one per lane, the next window
// prefetched), each row's entries in the window find their roots together (path halving; concurrent
// halving writes only ever store ancestors), then the row's links run in entry order -- one LDS
// read pair per entry instead of a whole dependent find chain.  Finds of a row see every link of
// the earlier rows; a root linked earlier in the same row is recognised by C2[root] != root, a root
// equal to the current row by r == t.
template <uint32_t CAP>
__global__ __launch_bounds__(64) void k_cl_replay_wave(const uint64_t *cl_off, const uint32_t *ids, uint64_t n_ids,
                                                       const uint64_t *q_off, const uint32_t *stream,
                                                       const uint32_t *srow, uint32_t *next, uint32_t *perm,
                                                       const uint32_t *n_ordered, int old_heur,
                                                       unsigned long long *prof = nullptr) {
  __shared__ uint16_t C2[CAP], T[CAP];
  const uint32_t lane = threadIdx.x;
  for (uint64_t ci = blockIdx.x; ci < n_ids; ci += gridDim.x) {
    const uint64_t c = ids[ci];
    const uint64_t b = cl_off[c];
    const uint32_t n = (uint32_t)(cl_off[c + 1] - b);
    if (d_cl_order_free(n, old_heur, n_ordered, c)) {
      for (uint32_t i = lane; i < n; i += 64) perm[b + i] = srow[b + i];
      continue;
    }
    const uint64_t q0 = q_off[b], q1 = q_off[b + n];
    const unsigned long long t_0 = prof ? wall_clock64() : 0ull;
    uint32_t *N = next + b;
    int32_t t = -1;     // current row (uniform)
    uint32_t tail = 0;  // its list tail (uniform)
    uint32_t e_nx = q0 + lane < q1 ? stream[q0 + lane] : 0u;
    for (uint64_t q = q0; q < q1; q += 64) {
      const uint32_t e = e_nx;
      const bool valid = q + lane < q1;
      e_nx = q + 64 + lane < q1 ? stream[q + 64 + lane] : 0u;
      const uint64_t starts = __ballot(valid && (e & kClRowBit));
      const uint32_t cnt = (uint32_t)min<uint64_t>(64, q1 - q);
      uint32_t a = 0;
      while (a < cnt) {
        const uint64_t later = a >= 63 ? 0ull : (starts & ~((2ull << a) - 1ull));
        const uint32_t bnd = later ? (uint32_t)(__ffsll((long long)later) - 1) : cnt;
        if ((starts >> a) & 1ull) {  // a new row
          if (t >= 0 && lane == 0) T[t] = (uint16_t)tail;
          ++t;
          if (lane == 0) { C2[t] = (uint16_t)t; N[t] = RS_NONE; }
          tail = (uint32_t)t;
          wave_sync();
        }
        uint32_t r = e & ~kClRowBit;
        const bool mine = lane >= a && lane < bnd && r != kClNoPrev;
        if (mine) {
          uint32_t p2 = C2[r];
          while (p2 != r) {  // path halving
            const uint32_t g = C2[p2];
            C2[r] = (uint16_t)g;
            r = p2 == g ? p2 : g;
            p2 = C2[r];
          }
        }
        wave_sync();
        uint64_t mm = __ballot(mine);
        while (mm) {
          const int l = __ffsll((long long)mm) - 1;
          mm &= mm - 1;
          const uint32_t rr = (uint32_t)__shfl((int)r, l);
          const uint32_t cr = C2[rr], tr = T[rr];
          if (rr == (uint32_t)t || cr != rr) continue;  // already in this row's list
          if (lane == 0) {
            N[tail] = rr;
            C2[rr] = (uint16_t)t;
          }
          tail = tr;
          wave_sync();
        }
        a = bnd;
      }
    }
    if (lane == 0 && t >= 0) T[t] = (uint16_t)tail;
    __syncthreads();  // N (global) complete
    for (uint32_t i = lane; i < n; i += 64) { const uint32_t x = N[i]; C2[i] = (uint16_t)(x == RS_NONE ? 0xffffu : x); }
    __syncthreads();
    if (lane == 0) {
      uint32_t x = n - 1, qq = 0;
      while (x != 0xffffu) { T[qq++] = (uint16_t)x; x = C2[x]; }
    }
    __syncthreads();
    for (uint32_t i = lane; i < n; i += 64) perm[b + i] = srow[b + T[i]];
    if (prof && lane == 0) {  // RS_PROF: (cluster, rows, pairs, 100 MHz ticks)
      prof[4 * ci] = c;
      prof[4 * ci + 1] = n;
      prof[4 * ci + 2] = q1 - q0;
      prof[4 * ci + 3] = wall_clock64() - t_0;
    }
    __syncthreads();
  }
}

// what the host replay of clusters ids[0..n) needs to fetch their pair streams: (first row, rows,
// first pair, pairs, rows whose order matters, the cluster) per cluster
constexpr int kMetaW = 6;
__global__ void k_replay_meta(const uint64_t *cl_off, const uint32_t *ids, uint64_t n, const uint64_t *q_off,
                              const uint32_t *n_ordered, uint64_t *meta) {
  for (uint64_t i = gtid(); i < n; i += gstride()) {
    const uint32_t c = ids[i];
    const uint64_t b = cl_off[c], e = cl_off[c + 1];
    meta[kMetaW * i] = b;
    meta[kMetaW * i + 1] = e - b;
    meta[kMetaW * i + 2] = q_off[b];
    meta[kMetaW * i + 3] = q_off[e] - q_off[b];
    meta[kMetaW * i + 4] = n_ordered[c];
    meta[kMetaW * i + 5] = c;
  }
}

// cluster-size classes for the elimination kernels, sorted by (workgroup kernels first, size desc,
// index).  The workgroup kernels take every cluster of kWaveMin rows or more, and also the smaller
// ones holding kHeavyNnz entries or more: rounds >= 2 cluster rows that substitution made long (a
// chain's composed right-hand sides), which one lane would merge serially for tens of ms.  Both
// kernels run the same process_3 / process_4 rules, and results are collected by cluster index, so
// the routing changes no output.
constexpr uint32_t kHeavyNnz = 128;  // MI355X sweep: templated round-2 small clusters 21.8 -> 7.4 ms vs 256, metric device time unchanged
__global__ void k_cl_sizekey(const uint64_t *cl_off, uint64_t n_cl, const uint32_t *srow, const uint32_t *len,
                             uint64_t *skey, uint32_t *sidx,
                             unsigned long long *cnt /* [0] >= 1e6, [1] workgroup kernels, [2] LDS replay, [3] > LDS, [4] large LDS replay */) {
  unsigned long long k[5] = {0, 0, 0, 0, 0};
  for (uint64_t c = gtid(); c < n_cl; c += gstride()) {
    const uint64_t b = cl_off[c], sz = cl_off[c + 1] - b;
    bool wg = sz >= kWaveMin;
    if (!wg) {
      uint64_t nnz = 0;
      for (uint64_t i = b; i < b + sz; ++i) nnz += len[srow[i]];
      wg = nnz >= kHeavyNnz;
    }
    const uint64_t rank = wg ? (1ull << 31) + sz : sz;  // sz < 2^31
    skey[c] = ((0xffffffffull - rank) << 32) | c;
    sidx[c] = (uint32_t)c;
    k[0] += sz >= 1000000;
    k[1] += wg;
    k[2] += sz > kClSmall && sz <= kClLds;
    k[3] += sz > kClLds;
    k[4] += sz > kClMid && sz <= kClLds;
  }
#pragma unroll
  for (int i = 0; i < 5; ++i) wave_atomic_add(&cnt[i], k[i]);
}
// small list = sorted[0, h) ++ sorted[h + nb, n_cl)
__global__ void k_cl_small_ids(const uint32_t *sorted, uint64_t n_cl, uint64_t h, uint64_t nb, uint32_t *small) {
  for (uint64_t i = gtid(); i < n_cl - nb; i += gstride()) small[i] = sorted[i < h ? i : i + nb];
}

}  // namespace rs
