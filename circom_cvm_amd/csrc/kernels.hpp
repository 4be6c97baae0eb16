// kernels.hpp -- HIP kernels of the simplification path (gfx950).
//
// Rows live in HBM as ragged CSR: row r = entries [off[r], off[r] + len[r]) of (key u32, Fe
// value 32 B, Montgomery form); keys sorted ascending, unique.  Substitution right-hand sides
// (RHS) live in a bump-allocated pool with the same (key, value) SoA layout.
//
// Every kernel names the reference function it restates (file:line in /root/reference).
#pragma once
#include <hip/hip_runtime.h>

#include "field.hpp"

namespace rs {

#define RS_NONE 0xffffffffu
constexpr uint64_t kProfWords = 24;  // RS_PROF words per workgroup cluster

struct DRows {
  uint64_t *off;
  uint32_t *len;
  uint32_t *key;
  Fe *val;
  uint64_t n;
};

__device__ __forceinline__ uint64_t gtid() { return (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; }
__device__ __forceinline__ uint64_t gstride() { return (uint64_t)gridDim.x * blockDim.x; }
// One atomic per wave for a counter every lane contributes to (all lanes of the wave must call it):
// per-lane atomics on one address serialise in the L2 (a million of them cost milliseconds).
__device__ __forceinline__ void wave_atomic_add(unsigned long long *p, unsigned long long x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d);
  if ((threadIdx.x & 63) == 0 && x) atomicAdd(p, x);
}

// ---------------------------------------------------------------- small sequential helpers
// insertion sort by key + combine duplicate keys (sum); zeros are kept (HashMap semantics).
__device__ inline uint32_t d_sort_combine(const FieldP &F, uint32_t *k, Fe *v, uint32_t n) {
  if (n <= 32) {  // short lists: insertion sort
    for (uint32_t i = 1; i < n; ++i) {
      uint32_t kk = k[i];
      Fe vv = v[i];
      uint32_t j = i;
      while (j > 0 && k[j - 1] > kk) {
        k[j] = k[j - 1];
        v[j] = v[j - 1];
        --j;
      }
      k[j] = kk;
      v[j] = vv;
    }
  } else {  // in-place heap sort: n log n moves (a frame-3 expansion of a long row is thousands of
            // entries; insertion sort moved O(n^2) 36-byte entries on one lane)
    auto sift = [&](uint32_t i, uint32_t m) {
      const uint32_t kk = k[i];
      const Fe vv = v[i];
      for (;;) {
        uint32_t c = 2 * i + 1;
        if (c >= m) break;
        if (c + 1 < m && k[c + 1] > k[c]) ++c;
        if (k[c] <= kk) break;
        k[i] = k[c];
        v[i] = v[c];
        i = c;
      }
      k[i] = kk;
      v[i] = vv;
    };
    for (uint32_t i = n / 2; i-- > 0;) sift(i, n);
    for (uint32_t m = n; m-- > 1;) {
      const uint32_t tk = k[0];
      const Fe tv = v[0];
      k[0] = k[m];
      v[0] = v[m];
      k[m] = tk;
      v[m] = tv;
      sift(0, m);
    }
  }
  // equal keys are summed (field addition is commutative: the order among them does not matter)
  uint32_t w = 0;
  for (uint32_t i = 0; i < n; ++i) {
    if (w > 0 && k[w - 1] == k[i]) v[w - 1] = fadd(F, v[w - 1], v[i]);
    else { k[w] = k[i]; v[w] = v[i]; ++w; }
  }
  return w;
}
__device__ inline uint32_t d_drop_zeros(uint32_t *k, Fe *v, uint32_t n) {
  uint32_t w = 0;
  for (uint32_t i = 0; i < n; ++i)
    if (!fe_is_zero(v[i])) { k[w] = k[i]; v[w] = v[i]; ++w; }
  return w;
}
// out = c - s*b over sorted maps, zeros dropped (constant_linear_linear_reduction, algebra.rs:1326-1344)
__device__ inline uint32_t d_axpy_merge(const FieldP &F, const uint32_t *ck, const Fe *cv, uint32_t cn,
                                        const uint32_t *bk, const Fe *bv, uint32_t bn, const Fe &s,
                                        uint32_t *ok, Fe *ov) {
  uint32_t i = 0, j = 0, w = 0;
  while (i < cn || j < bn) {
    uint32_t kk;
    Fe x;
    if (j >= bn || (i < cn && ck[i] < bk[j])) { kk = ck[i]; x = cv[i]; ++i; }
    else if (i >= cn || bk[j] < ck[i]) { kk = bk[j]; x = fneg(F, fmul(F, s, bv[j])); ++j; }
    else { kk = ck[i]; x = fsub(F, cv[i], fmul(F, s, bv[j])); ++i; ++j; }
    if (!fe_is_zero(x)) { ok[w] = kk; ov[w] = x; ++w; }
  }
  return w;
}

// fix_raw_constraint (algebra.rs:1309-1324) on zero-free sorted maps a, b, c (in place).
// c must have room for |c| + max(|a|, |b|) entries plus scratch of the same size after it.
__device__ inline void d_fix(const FieldP &F, uint32_t *ak, Fe *av, uint32_t &an, uint32_t *bk, Fe *bv,
                             uint32_t &bn, uint32_t *ck, Fe *cv, uint32_t &cn, uint32_t *tk, Fe *tv) {
  if (an == 0 || bn == 0) { an = 0; bn = 0; return; }
  const uint32_t *ok_;
  const Fe *ov_;
  uint32_t on;
  Fe s;
  if (an == 1 && ak[0] == 0) { s = av[0]; ok_ = bk; ov_ = bv; on = bn; }
  else if (bn == 1 && bk[0] == 0) { s = bv[0]; ok_ = ak; ov_ = av; on = an; }
  else return;
  uint32_t w = d_axpy_merge(F, ck, cv, cn, ok_, ov_, on, s, tk, tv);
  for (uint32_t i = 0; i < w; ++i) { ck[i] = tk[i]; cv[i] = tv[i]; }
  cn = w;
  an = 0;
  bn = 0;
}

// ---------------------------------------------------------------- load / convert / validate
// Row pointers of an uploaded block: ptr[0] = 0, non-decreasing, ptr[n] = nnz.  Runs before any
// kernel reads a row of the block (a decreasing ptr would make a row length wrap).
__global__ void k_check_ptr(const uint64_t *ptr, uint64_t n, uint64_t nnz, int *flag) {
  for (uint64_t r = gtid(); r <= n; r += gstride()) {
    const uint64_t v = ptr[r];
    bool bad = r == 0 ? v != 0 : v < ptr[r - 1];
    if (r == n) bad |= v != nnz;
    if (bad) atomicOr(flag, 1);
  }
}
// Keys of a block whose values are still on the way (rs_engine_simplify's staged load): every key
// < S; a row not strictly ascending sets `unsorted` (its values will be sorted with it once they
// land), or, without `unsorted` (2-key eq rows), is invalid unless its keys are distinct.
__global__ void k_check_keys(const uint64_t *ptr, const uint32_t *key, uint64_t n, uint64_t S, const int *ptr_bad, int *err,
                             int *unsorted) {
  if (*ptr_bad) return;
  for (uint64_t r = gtid(); r < n; r += gstride()) {
    const uint64_t b = ptr[r], e = ptr[r + 1];
    bool asc = true;
    for (uint64_t i = b; i < e; ++i) {
      if (key[i] >= S) atomicOr(err, 1);
      if (i > b && key[i - 1] >= key[i]) asc = false;
    }
    if (asc) continue;
    if (unsorted) { atomicOr(unsorted, 1); continue; }
    for (uint64_t i = b; i < e; ++i)
      for (uint64_t j = i + 1; j < e && j < b + 64; ++j)
        if (key[i] == key[j]) atomicOr(err, 1);
  }
}
// heap sort of (key, value) pairs by key (rows too long for an insertion sort)
__device__ inline void d_heap_sort_pairs(uint32_t *k, Fe *v, uint32_t n) {
  auto sift = [&](uint32_t i, uint32_t m) {
    for (;;) {
      uint32_t c = 2 * i + 1;
      if (c >= m) return;
      if (c + 1 < m && k[c + 1] > k[c]) ++c;
      if (k[i] >= k[c]) return;
      uint32_t tk = k[i]; k[i] = k[c]; k[c] = tk;
      Fe tv = v[i]; v[i] = v[c]; v[c] = tv;
      i = c;
    }
  };
  for (uint32_t i = n / 2; i-- > 0;) sift(i, n);
  for (uint32_t m = n; m-- > 1;) {
    uint32_t tk = k[0]; k[0] = k[m]; k[m] = tk;
    Fe tv = v[0]; v[0] = v[m]; v[m] = tv;
    sift(0, m);
  }
}
// Sorts every row by key and validates it (distinct keys < S, canonical nonzero values).  Skipped
// when the block's row pointers failed k_check_ptr (`ptr_bad`, stream-ordered before this kernel).
__global__ void k_sort_validate(FieldP F, const uint64_t *ptr, uint32_t *key, Fe *val, uint64_t n,
                                uint64_t S, const int *ptr_bad, int *err) {
  if (*ptr_bad) return;
  for (uint64_t r = gtid(); r < n; r += gstride()) {
    uint64_t b = ptr[r], e = ptr[r + 1];
    uint32_t *k = key + b;
    Fe *v = val + b;
    uint32_t m = (uint32_t)(e - b);
    bool sorted = true;
    for (uint32_t i = 1; i < m && sorted; ++i) sorted = k[i - 1] < k[i];
    if (!sorted && m <= 32) {
      for (uint32_t i = 1; i < m; ++i) {
        uint32_t kk = k[i];
        Fe vv = v[i];
        uint32_t j = i;
        while (j > 0 && k[j - 1] > kk) { k[j] = k[j - 1]; v[j] = v[j - 1]; --j; }
        k[j] = kk;
        v[j] = vv;
      }
    } else if (!sorted) {
      d_heap_sort_pairs(k, v, m);
    }
    for (uint32_t i = 0; i < m; ++i) {
      if (k[i] >= S || (i > 0 && k[i] == k[i - 1]) || fe_is_zero(v[i]) || geq4(v[i].l, F.p)) atomicOr(err, 1);
    }
  }
}
// canonical -> Montgomery copy (working buffers), plus len/off for ragged rows.
__global__ void k_to_mont(FieldP F, const Fe *src, Fe *dst, uint64_t n) {
  for (uint64_t i = gtid(); i < n; i += gstride()) dst[i] = fto_mont(F, src[i]);
}
__global__ void k_ptr_to_ragged(const uint64_t *ptr, uint64_t *off, uint32_t *len, uint64_t n, uint64_t extra) {
  for (uint64_t r = gtid(); r < n; r += gstride()) {
    off[r] = ptr[r] + extra * r;
    len[r] = (uint32_t)(ptr[r + 1] - ptr[r]);
  }
}
__global__ void k_fill_i32(int32_t *p, int32_t v, uint64_t n) {
  for (uint64_t i = gtid(); i < n; i += gstride()) p[i] = v;
}

// ---------------------------------------------------------------- eq_simplification (:126-251)
__device__ __forceinline__ uint32_t uf_load(uint32_t *uf, uint32_t x) {
  return __hip_atomic_load(&uf[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline uint32_t uf_find(uint32_t *uf, uint32_t x) {
  uint32_t p = uf_load(uf, x);
  while (p != x) {
    uint32_t gp = uf_load(uf, p);
    if (gp != p) __hip_atomic_store(&uf[x], gp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    x = p;
    p = gp;
  }
  return x;
}
// build_clusters over the equalities: connected components of the 2-signal rows.
__global__ void k_eq_union(const uint64_t *ptr, const uint32_t *key, uint64_t n, uint32_t *uf, int *err) {
  for (uint64_t r = gtid(); r < n; r += gstride()) {
    if (ptr[r + 1] - ptr[r] != 2 || key[ptr[r]] == 0) { atomicOr(err, 2); continue; }
    uint32_t a = key[ptr[r]], b = key[ptr[r] + 1];
    for (;;) {
      a = uf_find(uf, a);
      b = uf_find(uf, b);
      if (a == b) break;
      if (a > b) { uint32_t t = a; a = b; b = t; }
      uint32_t old = atomicCAS(&uf[b], b, a);
      if (old == b) break;
      b = old;
    }
  }
}
// per-component statistics: #rows, max row index (= arena index, i.e. cluster order),
// min forbidden and min removable signal (eq_cluster_simplification :158-179).
__global__ void k_eq_stats(const uint64_t *ptr, const uint32_t *key, uint64_t n, uint32_t *uf,
                           const uint8_t *forb, uint32_t *cnt, int32_t *maxrow, uint32_t *minf,
                           uint32_t *minr, uint8_t *in_eq) {
  for (uint64_t r = gtid(); r < n; r += gstride()) {
    uint32_t a = key[ptr[r]], b = key[ptr[r] + 1];
    uint32_t root = uf_find(uf, a);
    atomicAdd(&cnt[root], 1u);
    atomicMax(&maxrow[root], (int32_t)r);
    for (int t = 0; t < 2; ++t) {
      uint32_t s = t ? b : a;
      in_eq[s] = 1;
      if (forb[s]) atomicMin(&minf[root], s);
      else atomicMin(&minr[root], s);
    }
  }
}
// every removable signal := representative (min forbidden, else min removable).
__global__ void k_eq_assign(const uint64_t *ptr, const uint32_t *key, uint64_t n, uint32_t *uf,
                            const uint8_t *forb, const uint32_t *minf, const uint32_t *minr,
                            int32_t *eq_rep, uint8_t *deleted, uint32_t *bf_list, uint32_t *bf_n) {
  for (uint64_t r = gtid(); r < n; r += gstride()) {
    uint32_t a = key[ptr[r]], b = key[ptr[r] + 1];
    uint32_t root = uf_find(uf, a);
    uint32_t rh = minf[root] != RS_NONE ? minf[root] : minr[root];
    for (int t = 0; t < 2; ++t) {
      uint32_t s = t ? b : a;
      if (!forb[s] && s != rh) { eq_rep[s] = (int32_t)rh; deleted[s] = 1; }
    }
    if (forb[a] && forb[b]) bf_list[atomicAdd(bf_n, 1u)] = (uint32_t)r;
  }
}
// the union-find roots of signals idx[i] (k_eq_stats / k_eq_assign compress only the paths from a
// row's first key, so a signal met only as a second key may sit several links below its root)
__global__ void k_uf_roots(uint32_t *uf, const uint32_t *idx, uint32_t *dst, uint64_t n) {
  for (uint64_t i = gtid(); i < n; i += gstride()) dst[i] = uf_find(uf, idx[i]);
}
__global__ void k_gather_u32(const uint32_t *src, const uint32_t *idx, uint32_t *dst, uint64_t n) {
  for (uint64_t i = gtid(); i < n; i += gstride()) dst[i] = src[idx[i]];
}
__global__ void k_gather_u64(const uint64_t *src, const uint32_t *idx, uint64_t *dst, uint64_t n) {
  for (uint64_t i = gtid(); i < n; i += gstride()) dst[i] = src[idx[i]];
}

// ---------------------------------------------------------------- constant equalities (:253-273)
// Applies the eq frame (fast_encoded_constraint_substitution + fix) to a C-only row in place;
// renaming never grows a row.
__device__ inline uint32_t d_rename_row(const FieldP &F, uint32_t *k, Fe *v, uint32_t n, const int32_t *eq_rep) {
  bool any = false;
  for (uint32_t i = 0; i < n; ++i) {
    int32_t t = eq_rep[k[i]];
    if (t >= 0) { k[i] = (uint32_t)t; any = true; }
  }
  if (!any) return n;
  n = d_sort_combine(F, k, v, n);
  return d_drop_zeros(k, v, n);
}
__global__ void k_rename_rows(FieldP F, DRows R, const int32_t *eq_rep) {
  for (uint64_t r = gtid(); r < R.n; r += gstride())
    R.len[r] = d_rename_row(F, R.key + R.off[r], R.val + R.off[r], R.len[r], eq_rep);
}
// picks, per signal, the last constant equality (HashMap insert: last wins) and lists the
// forbidden ones, which stay as constraints.
__global__ void k_const_pick(DRows R, const uint8_t *forb, int32_t *ce_last, uint8_t *deleted,
                             uint32_t *cons_list, uint32_t *cons_n, int *err) {
  for (uint64_t r = gtid(); r < R.n; r += gstride()) {
    const uint32_t *k = R.key + R.off[r];
    uint32_t n = R.len[r];
    uint32_t s = n ? k[n - 1] : 0;
    if (s == 0) { atomicOr(err, 4); continue; }
    if (forb[s]) { cons_list[atomicAdd(cons_n, 1u)] = (uint32_t)r; continue; }
    atomicMax(&ce_last[s], (int32_t)r);
    deleted[s] = 1;
  }
}
// clear_signal (algebra.rs:1108-1124): s := c / (-k)   (an empty map when c == 0 -> value 0)
// One inversion per 8 rows (Montgomery's trick over the rows that define their signal's value;
// exact inverses, so the batching is invisible): the inversion is the costly part of a row.
__global__ void k_const_value(FieldP F, DRows R, const uint8_t *forb, const int32_t *ce_last, Fe *ce_val,
                              uint8_t *ce_has) {
  constexpr uint32_t C = 8;
  for (uint64_t r0 = gtid() * C; r0 < R.n; r0 += gstride() * C) {
    const uint32_t m = (uint32_t)min<uint64_t>(C, R.n - r0);
    Fe pre[C];  // prefix products of the pivots -k (1 for rows that define nothing)
    Fe acc = F.one;
#pragma unroll
    for (uint32_t i = 0; i < C; ++i) {
      if (i < m) {
        const uint64_t r = r0 + i;
        const uint32_t n = R.len[r];
        if (n) {
          const uint32_t *k = R.key + R.off[r];
          const uint32_t s = k[n - 1];
          if (!forb[s] && ce_last[s] == (int32_t)r) acc = fmul(F, acc, fneg(F, R.val[R.off[r] + n - 1]));
        }
      }
      pre[i] = acc;
    }
    Fe inv = finv(F, acc);
#pragma unroll
    for (int i = C - 1; i >= 0; --i) {
      if ((uint32_t)i >= m) continue;
      const uint64_t r = r0 + i;
      const uint32_t n = R.len[r];
      if (!n) continue;
      const uint32_t *k = R.key + R.off[r];
      const Fe *v = R.val + R.off[r];
      const uint32_t s = k[n - 1];
      if (forb[s] || ce_last[s] != (int32_t)r) continue;
      const Fe inv_i = i ? fmul(F, pre[i - 1], inv) : inv;  // 1 / (-k) of this row
      inv = fmul(F, inv, fneg(F, v[n - 1]));
      const Fe c = (n == 2 && k[0] == 0) ? v[0] : fe_zero();
      ce_val[s] = fmul(F, c, inv_i);
      ce_has[s] = 1;
    }
  }
}
// eq frame then constant frame on one linear row (each frame + fix, :493-527); capacity n+1.
__device__ inline uint32_t d_linear_frames12(const FieldP &F, uint32_t *k, Fe *v, uint32_t n0, const int32_t *eq_rep,
                                             const uint8_t *ce_has, const Fe *ce_val) {
  {
    uint32_t n = d_rename_row(F, k, v, n0, eq_rep);
    bool any = false;
    for (uint32_t i = 0; i < n; ++i)
      if (ce_has[k[i]]) any = true;
    if (any) {
      Fe c0 = fe_zero();
      uint32_t w = 0;
      for (uint32_t i = 0; i < n; ++i) {
        if (ce_has[k[i]]) c0 = fadd(F, c0, fmul(F, v[i], ce_val[k[i]]));
        else if (k[i] == 0) c0 = fadd(F, c0, v[i]);
        else { k[w] = k[i]; v[w] = v[i]; ++w; }
      }
      // key 0 goes first (smallest key)
      for (uint32_t i = w; i > 0; --i) { k[i] = k[i - 1]; v[i] = v[i - 1]; }
      k[0] = 0;
      v[0] = c0;
      n = d_drop_zeros(k, v, w + 1);
    }
    return n;
  }
}
__global__ void k_linear_frames12(FieldP F, DRows R, const int32_t *eq_rep, const uint8_t *ce_has, const Fe *ce_val) {
  for (uint64_t r = gtid(); r < R.n; r += gstride())
    R.len[r] = d_linear_frames12(F, R.key + R.off[r], R.val + R.off[r], R.len[r], eq_rep, ce_has, ce_val);
}

// Keys-first linear rows (rs_engine_simplify): the eq and constant frames applied to the keys
// alone, so build_clusters runs before the values land.  Row r of the upload (sorted, distinct keys)
// becomes [0 if any constant or key 0] ++ sorted renamed non-constant keys in the ragged copy R
// (off = ptr + r, room for len + 1).  Exact when no two keys of a row rename to the same signal
// (their coefficients could cancel) and a row keeps a non-constant key (else whether it is empty
// depends on its constant term): a row that breaks either sets `uncertain`, and the caller falls
// back to the frames on values (k_make_ragged + k_linear_frames12) before clustering.
__global__ void k_lin_keyframes(const uint64_t *ptr, const uint32_t *key, uint64_t n, DRows R, const int32_t *eq_rep,
                                const uint8_t *ce_has, int *uncertain, uint32_t *unc_list, uint64_t unc_cap) {
  for (uint64_t r = gtid(); r < n; r += gstride()) {
    const uint64_t b = ptr[r];
    const uint32_t m = (uint32_t)(ptr[r + 1] - b);
    const uint64_t o = b + r;
    R.off[r] = o;
    uint32_t *out = R.key + o + 1;  // slot 0 is reserved for key 0
    bool has0 = false;
    uint32_t w = 0;
    for (uint32_t i = 0; i < m; ++i) {
      const uint32_t k = key[b + i];
      const int32_t t = eq_rep[k];
      const uint32_t k1 = t >= 0 ? (uint32_t)t : k;
      if (k1 == 0 || ce_has[k1]) { has0 = true; continue; }
      uint32_t j = w++;  // insertion into the sorted prefix
      while (j > 0 && out[j - 1] > k1) { out[j] = out[j - 1]; --j; }
      out[j] = k1;
    }
    uint32_t u = 0;  // distinct
    bool dup = false;
    for (uint32_t i = 0; i < w; ++i) {
      if (u > 0 && out[u - 1] == out[i]) { dup = true; continue; }
      out[u++] = out[i];
    }
    if (dup || u == 0) {
      const int q = atomicAdd(uncertain, 1);
      if ((uint64_t)q < unc_cap) unc_list[q] = (uint32_t)r;
    }
    if (has0) {
      R.key[o] = 0;
      R.len[r] = u + 1;
    } else {
      for (uint32_t i = 0; i < u; ++i) R.key[o + i] = out[i];
      R.len[r] = u;
    }
  }
}
// The values of the keys-first rows once they land: each renamed non-constant entry fills its key's
// slot (one contribution: no two keys of the row met), constant entries and key 0 sum into the
// constant term c0 (Montgomery), which is dropped when zero -- the result of k_make_ragged +
// k_linear_frames12 on the same row.
__global__ void k_lin_valframes(FieldP F, const uint64_t *ptr, const uint32_t *key, const Fe *val, uint64_t n, DRows R,
                                const int32_t *eq_rep, const uint8_t *ce_has, const Fe *ce_val, const uint8_t *fixed) {
  for (uint64_t r = gtid(); r < n; r += gstride()) {
    if (fixed[r]) continue;  // done by k_lin_fixrows
    const uint64_t b = ptr[r];
    const uint32_t m = (uint32_t)(ptr[r + 1] - b);
    const uint64_t o = R.off[r];
    uint32_t len = R.len[r];
    uint32_t *ok = R.key + o;
    Fe *ov = R.val + o;
    const bool has0 = len > 0 && ok[0] == 0;
    const uint32_t s0 = has0 ? 1 : 0;
    Fe c0 = fe_zero();
    for (uint32_t i = 0; i < m; ++i) {
      const uint32_t k = key[b + i];
      const Fe v = fto_mont(F, val[b + i]);
      const int32_t t = eq_rep[k];
      const uint32_t k1 = t >= 0 ? (uint32_t)t : k;
      if (k1 == 0) { c0 = fadd(F, c0, v); continue; }
      if (ce_has[k1]) { c0 = fadd(F, c0, fmul(F, v, ce_val[k1])); continue; }
      uint32_t lo = s0, hi = len;  // lower bound of k1 among the non-constant keys
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (ok[mid] < k1) lo = mid + 1; else hi = mid;
      }
      ov[lo] = v;
    }
    if (has0) {
      if (fe_is_zero(c0)) {
        for (uint32_t i = 1; i < len; ++i) { ok[i - 1] = ok[i]; ov[i - 1] = ov[i]; }
        R.len[r] = len - 1;
      } else {
        ov[0] = c0;
      }
    }
  }
}

// The rows k_lin_keyframes could not settle from keys, with their values (copied from the host
// input, canonical, as given): the frames on values, exactly as k_make_ragged + k_linear_frames12.
__global__ void k_lin_fixrows(FieldP F, const uint64_t *hptr, const uint32_t *hkey, const Fe *hval, const uint32_t *rows,
                              uint64_t m, DRows R, const int32_t *eq_rep, const uint8_t *ce_has, const Fe *ce_val,
                              uint8_t *fixed) {
  for (uint64_t q = gtid(); q < m; q += gstride()) {
    const uint32_t r = rows[q];
    const uint64_t b = hptr[q];
    const uint32_t len = (uint32_t)(hptr[q + 1] - b);
    uint32_t *k = R.key + R.off[r];
    Fe *v = R.val + R.off[r];
    for (uint32_t i = 0; i < len; ++i) { k[i] = hkey[b + i]; v[i] = fto_mont(F, hval[b + i]); }
    R.len[r] = d_linear_frames12(F, k, v, len, eq_rep, ce_has, ce_val);
    fixed[r] = 1;
  }
}

// ---------------------------------------------------------------- per-cluster elimination
// full_simplification (simplification_utils.rs:543-581): one thread per cluster.
struct ElimArgs {
  FieldP F;
  DRows rows;               // linear rows of this round
  const uint32_t *perm;     // rows in cluster order (clusters concatenated)
  const uint64_t *cl_off;   // cluster c = perm[cl_off[c] .. cl_off[c+1])
  uint64_t n_clusters;
  const uint8_t *forb;
  int old_heur;
  // dense per-signal scratch (clusters are signal-disjoint); reset by the kernel
  int32_t *holder_idx, *occ, *rep_pos, *noov;
  uint8_t *del;
  // per-slot arrays (slot = position in perm)
  uint32_t *h_sig;
  Fe *h_coef;
  uint64_t *h_off;
  uint32_t *h_len;
  uint32_t *tmp;            // scratch u32 per slot
  Fe *ftmp;                 // scratch Fe per slot
  uint8_t *dead;            // p4 rows emptied by the uniques phase
  uint32_t *order;          // p4 deletion order
  uint64_t *l_off;          // leftovers
  uint32_t *l_len;
  uint32_t *n_sub, *n_left; // per cluster
  // outputs
  int32_t *sub_of;          // dense: signal -> slot of its substitution
  uint8_t *deleted;
  // pool
  uint32_t *pk;
  Fe *pv;
  unsigned long long *pool_top;
  uint64_t pool_cap;
  int *err;
  unsigned long long *bytes;  // algorithmic bytes (SURVEY 8(d) B_alg terms of this kernel)
  unsigned long long *bytes_main, *bytes_fin;  // the same, for k_big_main and k_big_finish
  unsigned long long *prof;   // debug: 16 words per big cluster (see run_linear_simplification), or null
  unsigned long long *fclk;   // RS_FINCLK builds: the tail finish's section clocks (wall_clock64 ticks), or null
  uint64_t *big_touch_off;    // per big cluster: touched-signal list in the pool (k_big_prep)
  uint32_t *big_touch_n;
  uint32_t *big_alive;        // per big cluster: #rows left for the ordered loop
  uint64_t *row_off;          // per slot: (offset, length) of those rows in loop order (k_big_prep)
  uint32_t *row_len;
  int wide;                   // the k_wide_* kernels prepared this launch's largest p4 clusters
  uint8_t *skip = nullptr;    // per cluster (launch order): k_p3_fast finished it, the ordered loop skips it
  // split composition (the head's clusters): k_big_finish only normalises and builds each cluster's
  // dependency DAG, k_compose_level composes one Kahn level of every cluster at a time over the
  // whole GPU, k_big_emit finishes
  int split;
  int compose_sort;         // 1: compositions merge only where the sort cannot (0: every composition merges)
  uint64_t *cf_items;         // the first frontier (cluster position << 32 | local slot)
  unsigned long long *cf_n;   // its length
  uint64_t *cf_deg, *cf_dl;   // per cluster: pool offsets of deg[m] (+ dcnt[m+1]) and of the dependents
  uint32_t *cf_done;          // per cluster: substitutions that reached a frontier
  uint64_t *cf_big;           // a level's compositions too long for k_compose_level's waves
  unsigned long long *cf_nbig;

};

// Registers substitution `slot` for signal p (holder.insert): slot arrays + the dense per-signal copy
__device__ __forceinline__ void d_set_holder(const ElimArgs &A, uint32_t p, uint64_t slot, const Fe &coef, uint64_t off,
                                             uint32_t len) {
  A.holder_idx[p] = (int32_t)slot;
  A.h_sig[slot] = p;
  A.h_coef[slot] = coef;
  A.h_off[slot] = off;
  A.h_len[slot] = len;
}
__device__ __forceinline__ uint64_t pool_alloc_global(const ElimArgs &A, uint64_t n) {
  unsigned long long o = atomicAdd(A.pool_top, (unsigned long long)n);
  if (o + n > A.pool_cap) { atomicOr(A.err, 8); return RS_NONE; }
  return (uint64_t)o;
}
// Per-thread bump allocator over chunks of the pool: one global atomic per chunk instead of one per
// allocation (the global counter is shared by every lane of every cluster).
struct Alloc {
  uint64_t cur = 0, end = 0;
  uint32_t chunk = 512;
};
__device__ __forceinline__ uint64_t pool_alloc(const ElimArgs &A, Alloc &al, uint64_t n) {
  if (al.cur + n <= al.end) { uint64_t o = al.cur; al.cur += n; return o; }
  if (n >= al.chunk / 4) return pool_alloc_global(A, n);
  uint64_t c = pool_alloc_global(A, al.chunk);
  if (c == RS_NONE) return RS_NONE;
  al.cur = c + n;
  al.end = c + al.chunk;
  return c;
}

// clear_signal_not_normalized (algebra.rs:1126-1136): to = row minus key, {0: 0} ensured.
// Every substitution created before or inside the ordered loop is preceded in the pool by a header
// entry (key = RHS length, value = the coefficient): k_big_spec reads a holder's header and its
// right-hand side in one round trip.
__device__ __forceinline__ uint32_t d_clear_nn_len(const uint32_t *k, uint32_t n, uint32_t oi) {  // RHS entries
  const bool has0 = n > 0 && k[0] == 0 && oi != 0;
  return n - 1 + (has0 ? 0 : 1);
}
__device__ inline void d_clear_nn_at(const ElimArgs &A, const uint32_t *k, const Fe *v, uint32_t n, uint32_t oi,
                                     uint64_t o, Fe &coef, uint64_t &to_off, uint32_t &to_len);
__device__ inline bool d_clear_nn(const ElimArgs &A, Alloc &al, const uint32_t *k, const Fe *v, uint32_t n, uint32_t oi,
                                  Fe &coef, uint64_t &to_off, uint32_t &to_len) {
  const uint64_t o = pool_alloc(A, al, (uint64_t)d_clear_nn_len(k, n, oi) + 1);
  if (o == RS_NONE) return false;
  d_clear_nn_at(A, k, v, n, oi, o, coef, to_off, to_len);
  return true;
}
// the same at a given pool offset o (header at o, the RHS from o + 1)
__device__ inline void d_clear_nn_at(const ElimArgs &A, const uint32_t *k, const Fe *v, uint32_t n, uint32_t oi,
                                     uint64_t o, Fe &coef, uint64_t &to_off, uint32_t &to_len) {
  coef = fneg(A.F, v[oi]);
  const bool has0 = n > 0 && k[0] == 0 && oi != 0;
  const uint32_t m = n - 1 + (has0 ? 0 : 1);
  A.pk[o] = m;
  A.pv[o] = coef;
  ++o;
  uint32_t w = 0;
  if (!has0) { A.pk[o] = 0; A.pv[o] = fe_zero(); w = 1; }
  for (uint32_t i = 0; i < n; ++i)
    if (i != oi) { A.pk[o + w] = k[i]; A.pv[o + w] = v[i]; ++w; }
  to_off = o;
  to_len = m;
}
// treat_constraint_3/4 conflict: work = coef*R - c2*L, zeros dropped; L = row minus key (+{0:0}).
__device__ inline bool d_merge(const ElimArgs &A, Alloc &al, const uint32_t *k, const Fe *v, uint32_t n, uint32_t oi,
                               const Fe &coef, const Fe &c2, uint64_t r_off, uint32_t r_len,
                               uint64_t &w_off, uint32_t &w_len) {
  const FieldP &F = A.F;
  uint64_t o = pool_alloc(A, al, (uint64_t)n + r_len + 1);
  if (o == RS_NONE) return false;
  const uint32_t *rk = A.pk + r_off;
  const Fe *rv = A.pv + r_off;
  uint32_t i = 0, j = 0, w = 0;
  while (i < n || j < r_len) {
    if (i == oi) { ++i; continue; }
    uint32_t kk;
    Fe x;
    if (j >= r_len || (i < n && k[i] < rk[j])) { kk = k[i]; x = fneg(F, fmul(F, c2, v[i])); ++i; }
    else if (i >= n || rk[j] < k[i]) { kk = rk[j]; x = fmul(F, coef, rv[j]); ++j; }
    else { kk = k[i]; x = fsub(F, fmul(F, coef, rv[j]), fmul(F, c2, v[i])); ++i; ++j; }
    if (!fe_is_zero(x)) { A.pk[o + w] = kk; A.pv[o + w] = x; ++w; }
  }
  w_off = o;
  w_len = w;
  return true;
}
// Substitution::apply_substitution with a single change (raw_substitution, algebra.rs:1279-1294):
// out = src[from := val*rhs]; every rhs key is inserted, zeros kept; both maps hold key 0.
__device__ inline bool d_raw_sub(const ElimArgs &A, Alloc &al, uint64_t s_off, uint32_t s_len, uint32_t from, uint64_t r_off,
                                 uint32_t r_len, uint64_t &o_off, uint32_t &o_len) {
  const FieldP &F = A.F;
  const uint32_t *sk = A.pk + s_off;
  const Fe *sv = A.pv + s_off;
  const uint32_t *rk = A.pk + r_off;
  const Fe *rv = A.pv + r_off;
  Fe val = fe_zero();
  uint32_t fi = RS_NONE;
  for (uint32_t i = 0; i < s_len; ++i)
    if (sk[i] == from) { val = sv[i]; fi = i; break; }
  if (fi == RS_NONE) { o_off = s_off; o_len = s_len; return true; }
  uint64_t o = pool_alloc(A, al, (uint64_t)s_len + r_len);
  if (o == RS_NONE) return false;
  uint32_t i = 0, j = 0, w = 0;
  while (i < s_len || j < r_len) {
    if (i == fi) { ++i; continue; }
    if (j >= r_len || (i < s_len && sk[i] < rk[j])) { A.pk[o + w] = sk[i]; A.pv[o + w] = sv[i]; ++i; }
    else if (i >= s_len || rk[j] < sk[i]) { A.pk[o + w] = rk[j]; A.pv[o + w] = fmul(F, val, rv[j]); ++j; }
    else { A.pk[o + w] = sk[i]; A.pv[o + w] = fadd(F, sv[i], fmul(F, val, rv[j])); ++i; ++j; }
    ++w;
  }
  o_off = o;
  o_len = w;
  return true;
}

// raw_substitution into a caller-provided buffer (no allocation)
__device__ inline void d_raw_sub_into(const ElimArgs &A, uint64_t s_off, uint32_t s_len, uint32_t from, uint64_t r_off,
                                      uint32_t r_len, uint64_t o, uint32_t &o_len) {
  const FieldP &F = A.F;
  const uint32_t *sk = A.pk + s_off;
  const Fe *sv = A.pv + s_off;
  const uint32_t *rk = A.pk + r_off;
  const Fe *rv = A.pv + r_off;
  Fe val = fe_zero();
  uint32_t fi = RS_NONE;
  for (uint32_t i = 0; i < s_len; ++i)
    if (sk[i] == from) { val = sv[i]; fi = i; break; }
  uint32_t i = 0, j = 0, w = 0;
  if (fi == RS_NONE) {
    for (; i < s_len; ++i) { A.pk[o + i] = sk[i]; A.pv[o + i] = sv[i]; }
    o_len = s_len;
    return;
  }
  while (i < s_len || j < r_len) {
    if (i == fi) { ++i; continue; }
    if (j >= r_len || (i < s_len && sk[i] < rk[j])) { A.pk[o + w] = sk[i]; A.pv[o + w] = sv[i]; ++i; }
    else if (i >= s_len || rk[j] < sk[i]) { A.pk[o + w] = rk[j]; A.pv[o + w] = fmul(F, val, rv[j]); ++j; }
    else { A.pk[o + w] = sk[i]; A.pv[o + w] = fadd(F, sv[i], fmul(F, val, rv[j])); ++i; ++j; }
    ++w;
  }
  o_len = w;
}

__device__ inline void d_heap_sort_u32(uint32_t *a, uint32_t n) {
  if (n < 2) return;
  for (uint32_t start = n / 2; start-- > 0;) {
    uint32_t root = start;
    for (;;) {
      uint32_t child = 2 * root + 1;
      if (child >= n) break;
      if (child + 1 < n && a[child] < a[child + 1]) ++child;
      if (a[root] < a[child]) { uint32_t t = a[root]; a[root] = a[child]; a[child] = t; root = child; }
      else break;
    }
  }
  for (uint32_t end = n - 1; end > 0; --end) {
    uint32_t t = a[0]; a[0] = a[end]; a[end] = t;
    uint32_t root = 0;
    for (;;) {
      uint32_t child = 2 * root + 1;
      if (child >= end) break;
      if (child + 1 < end && a[child] < a[child + 1]) ++child;
      if (a[root] < a[child]) { uint32_t tt = a[root]; a[root] = a[child]; a[child] = tt; root = child; }
      else break;
    }
  }
}

// normalize_substitutions (:414-437) + create_nonoverlapping_substitutions(_4) (:451-479).
// Slots [b, b+m) hold the holder; `seq` lists the signals in composition order.
__device__ inline bool d_normalize_compose(const ElimArgs &A, Alloc &al, uint64_t b, uint32_t m, const uint32_t *seq) {
  const FieldP &F = A.F;
  if (m == 0) return true;
  // batch inversion (Montgomery's trick; exact inverses, so order-free)
  Fe acc = A.h_coef[b];
  A.ftmp[b] = acc;
  for (uint32_t i = 1; i < m; ++i) { acc = fmul(F, acc, A.h_coef[b + i]); A.ftmp[b + i] = acc; }
  Fe inv = finv(F, acc);
  for (uint32_t i = m; i-- > 0;) {
    Fe inv_i = i ? fmul(F, A.ftmp[b + i - 1], inv) : inv;
    inv = fmul(F, inv, A.h_coef[b + i]);
    Fe *v = A.pv + A.h_off[b + i];
    for (uint32_t t = 0; t < A.h_len[b + i]; ++t) v[t] = fmul(F, v[t], inv_i);
  }
  for (uint32_t q = 0; q < m; ++q) {
    uint32_t s = seq[q];
    int32_t slot = A.holder_idx[s];
    uint64_t off = A.h_off[slot];
    uint32_t len = A.h_len[slot];
    // collect the keys to apply first (take_substitutions_to_be_applied, :439-448)
    const uint32_t *kk = A.pk + off;
    uint32_t n_app = 0;
    for (uint32_t t = 0; t < len; ++t)
      if (A.noov[kk[t]] >= 0) ++n_app;
    if (n_app) {
      // one output bound for all applications, two ping-pong buffers (raw_substitution applied
      // key by key in ascending order; applying one never removes another applicable key)
      uint64_t bound = len;
      for (uint32_t t = 0; t < len; ++t) {
        int32_t ns = A.noov[kk[t]];
        if (ns >= 0) bound += A.h_len[ns];
      }
      uint64_t buf0 = pool_alloc(A, al, bound), buf1 = pool_alloc(A, al, bound);
      if (buf0 == RS_NONE || buf1 == RS_NONE) return false;
      uint64_t orig_off = off;
      uint32_t orig_len = len;
      uint64_t dst = buf0;
      for (uint32_t t = 0; t < orig_len; ++t) {
        uint32_t key = A.pk[orig_off + t];
        int32_t ns = A.noov[key];
        if (ns < 0) continue;
        uint32_t nl;
        d_raw_sub_into(A, off, len, key, A.h_off[ns], A.h_len[ns], dst, nl);
        off = dst;
        len = nl;
        dst = dst == buf0 ? buf1 : buf0;
      }
      A.h_off[slot] = off;
      A.h_len[slot] = len;
    }
    A.noov[s] = slot;
  }
  return true;
}

__global__ __launch_bounds__(64) void k_eliminate(ElimArgs A, const uint32_t *ids, uint64_t n_ids) {
  const FieldP &F = A.F;
  Alloc al;
  unsigned long long by_all = 0;  // algorithmic bytes of this lane's clusters
  for (uint64_t ci = gtid(); ci < n_ids; ci += gstride()) {
    const uint64_t c = ids[ci];
    const uint64_t b = A.cl_off[c], e = A.cl_off[c + 1];
    const uint32_t n = (uint32_t)(e - b);
    const bool use4 = n >= 350 && n < 1000000 && !A.old_heur;
    uint32_t m = 0, nl = 0, nd = 0;
    bool ok = true;
    if (!use4) {
      // ---- substitution_process_3 + treat_constraint_3 + take_signal_3 (:143-154, :259-294, :368-377)
      for (uint64_t idx = e; idx-- > b && ok;) {
        uint32_t r = A.perm[idx];
        const uint32_t *k = A.rows.key + A.rows.off[r];
        const Fe *v = A.rows.val + A.rows.off[r];
        uint32_t len = A.rows.len[r];
        for (;;) {
          if (len == 0) break;
          uint32_t oi = RS_NONE;
          for (uint32_t i = len; i-- > 0;)
            if (!A.forb[k[i]]) { oi = i; break; }
          if (oi == RS_NONE) {  // no takeable signal: leftover
            uint64_t o = pool_alloc(A, al, len);
            if (o == RS_NONE) { ok = false; break; }
            for (uint32_t i = 0; i < len; ++i) { A.pk[o + i] = k[i]; A.pv[o + i] = v[i]; }
            A.l_off[b + nl] = o;
            A.l_len[b + nl] = len;
            ++nl;
            break;
          }
          uint32_t out = k[oi];
          int32_t hi = A.holder_idx[out];
          if (hi < 0) {
            Fe coef;
            uint64_t to_off;
            uint32_t to_len;
            if (!d_clear_nn(A, al, k, v, len, oi, coef, to_off, to_len)) { ok = false; break; }
            A.holder_idx[out] = (int32_t)(b + m);
            A.h_sig[b + m] = out;
            A.h_coef[b + m] = coef;
            A.h_off[b + m] = to_off;
            A.h_len[b + m] = to_len;
            ++m;
            break;
          }
          uint64_t w_off;
          uint32_t w_len;
          if (!d_merge(A, al, k, v, len, oi, fneg(F, v[oi]), A.h_coef[hi], A.h_off[hi], A.h_len[hi], w_off, w_len)) {
            ok = false;
            break;
          }
          k = A.pk + w_off;
          v = A.pv + w_off;
          len = w_len;
        }
      }
      // BTreeMap order: ascending signal
      for (uint32_t i = 0; i < m; ++i) A.tmp[b + i] = A.h_sig[b + i];
      d_heap_sort_u32(A.tmp + b, m);
      if (ok) ok = d_normalize_compose(A, al, b, m, A.tmp + b);
    } else {
      // ---- substitution_process_4 (:156-185), SignalsInformation (:60-113)
      uint32_t n_touch = 0;
      uint64_t touch_off = 0;
      {
        uint64_t tot = 0;
        for (uint64_t idx = b; idx < e; ++idx) tot += A.rows.len[A.perm[idx]];
        touch_off = pool_alloc(A, al, tot + 1);
        if (touch_off == RS_NONE) ok = false;
      }
      uint32_t *touch = A.pk + touch_off;
      for (uint64_t idx = b; idx < e && ok; ++idx) {
        uint32_t r = A.perm[idx];
        const uint32_t *k = A.rows.key + A.rows.off[r];
        uint32_t len = A.rows.len[r];
        A.dead[idx] = 0;
        for (uint32_t i = 0; i < len; ++i) {
          uint32_t s = k[i];
          if (A.forb[s]) continue;
          if (A.occ[s] < 0) { A.occ[s] = 1; A.rep_pos[s] = (int32_t)(idx - b); touch[n_touch++] = s; }
          else A.occ[s]++;
        }
      }
      // uniques in ascending signal order (scratch after the touched list; can exceed n)
      uint32_t n_u = 0;
      uint64_t uniq_off = ok ? pool_alloc(A, al, (uint64_t)n_touch + 1) : RS_NONE;
      if (uniq_off == RS_NONE) ok = false;
      uint32_t *uniq = A.pk + (ok ? uniq_off : 0);
      if (ok) {
        for (uint32_t t = 0; t < n_touch; ++t)
          if (A.occ[touch[t]] == 1) uniq[n_u++] = touch[t];
        d_heap_sort_u32(uniq, n_u);
      }
      auto remove_constraint = [&](const uint32_t *k, uint32_t len) {
        for (uint32_t i = 0; i < len; ++i)
          if (!A.forb[k[i]] && A.occ[k[i]] >= 0) A.occ[k[i]]--;
      };
      for (uint32_t u = 0; u < n_u && ok; ++u) {
        uint32_t s = uniq[u];
        uint64_t idx = b + (uint64_t)A.rep_pos[s];
        if (A.dead[idx]) continue;
        A.dead[idx] = 1;
        uint32_t r = A.perm[idx];
        const uint32_t *k = A.rows.key + A.rows.off[r];
        const Fe *v = A.rows.val + A.rows.off[r];
        uint32_t len = A.rows.len[r];
        remove_constraint(k, len);
        uint32_t oi = 0;
        while (k[oi] != s) ++oi;
        Fe coef;
        uint64_t to_off;
        uint32_t to_len;
        if (!d_clear_nn(A, al, k, v, len, oi, coef, to_off, to_len)) { ok = false; break; }
        A.holder_idx[s] = (int32_t)(b + m);
        A.h_sig[b + m] = s;
        A.h_coef[b + m] = coef;
        A.h_off[b + m] = to_off;
        A.h_len[b + m] = to_len;
        ++m;
        A.occ[s] = -1;
        A.del[s] = 1;
        A.order[b + nd++] = s;
      }
      for (uint64_t idx = e; idx-- > b && ok;) {
        if (A.dead[idx]) continue;
        uint32_t r = A.perm[idx];
        const uint32_t *k = A.rows.key + A.rows.off[r];
        const Fe *v = A.rows.val + A.rows.off[r];
        uint32_t len = A.rows.len[r];
        remove_constraint(k, len);
        for (;;) {
          if (len == 0) break;
          // take_signal_4 (:379-411), HashMap order := ascending
          uint32_t oi = RS_NONE;
          int32_t occ_ret = -1;
          for (uint32_t i = 0; i < len; ++i) {
            uint32_t s = k[i];
            if (A.forb[s]) continue;
            if (A.del[s]) { oi = i; break; }
            int32_t c2 = A.occ[s];
            if (c2 < 0) { atomicOr(A.err, 16); c2 = 0; }
            if (occ_ret < 0 || c2 < occ_ret) { oi = i; occ_ret = c2; }
            else if (c2 == occ_ret && k[oi] < s) oi = i;
          }
          if (oi == RS_NONE) {
            uint64_t o = pool_alloc(A, al, len);
            if (o == RS_NONE) { ok = false; break; }
            for (uint32_t i = 0; i < len; ++i) { A.pk[o + i] = k[i]; A.pv[o + i] = v[i]; }
            A.l_off[b + nl] = o;
            A.l_len[b + nl] = len;
            ++nl;
            break;
          }
          uint32_t out = k[oi];
          int32_t hi = A.holder_idx[out];
          if (hi < 0) {
            Fe coef;
            uint64_t to_off;
            uint32_t to_len;
            if (!d_clear_nn(A, al, k, v, len, oi, coef, to_off, to_len)) { ok = false; break; }
            A.holder_idx[out] = (int32_t)(b + m);
            A.h_sig[b + m] = out;
            A.h_coef[b + m] = coef;
            A.h_off[b + m] = to_off;
            A.h_len[b + m] = to_len;
            ++m;
            A.occ[out] = -1;
            A.del[out] = 1;
            A.order[b + nd++] = out;
            break;
          }
          uint64_t w_off;
          uint32_t w_len;
          if (!d_merge(A, al, k, v, len, oi, fneg(F, v[oi]), A.h_coef[hi], A.h_off[hi], A.h_len[hi], w_off, w_len)) {
            ok = false;
            break;
          }
          k = A.pk + w_off;
          v = A.pv + w_off;
          len = w_len;
        }
      }
      for (uint32_t t = 0; t < n_touch; ++t) A.occ[touch[t]] = -1;
      for (uint32_t t = 0; t < nd; ++t) A.del[A.order[b + t]] = 0;
      // composition order: deletion order, newest first
      uint32_t *seq = A.tmp + b;
      for (uint32_t t = 0; t < nd; ++t) seq[t] = A.order[b + nd - 1 - t];
      if (ok) ok = d_normalize_compose(A, al, b, m, seq);
    }
    for (uint32_t i = 0; i < m; ++i) {
      uint32_t s = A.h_sig[b + i];
      A.holder_idx[s] = -1;
      A.noov[s] = -1;
      A.sub_of[s] = (int32_t)(b + i);
      A.deleted[s] = 1;
    }
    A.n_sub[c] = m;
    A.n_left[c] = nl;
    if (!ok) atomicOr(A.err, 8);
    // B_alg of the cluster: its rows read once (36 B per entry + 8 B row pointer), every
    // substitution read and written by normalisation and written once more by composition
    uint64_t rows_e = 0, subs_e = 0;
    for (uint64_t idx = b; idx < e; ++idx) rows_e += A.rows.len[A.perm[idx]];
    for (uint32_t i = 0; i < m; ++i) subs_e += A.h_len[b + i];
    by_all += 36ull * (rows_e + 3 * subs_e) + 8ull * n;
  }
  wave_atomic_add(A.bytes, by_all);
}



// ================================================================ large clusters (process_4)
// Three launches per round, one workgroup per cluster (largest first):
//   k_big_prep   (256 lanes) SignalsInformation::new + the uniques pass           (:296-316)
//   k_big_main   ( 64 lanes) the ordered main loop (treat_constraint_4 + take_signal_4, :317-366):
//                the row walk is inherently sequential, so one wave runs it cooperatively -- the work
//                list lives in LDS, the pivot is a wave reduction, and each conflict is a merge-path
//                merge whose 256-bit products are spread over the lanes.
//   k_big_finish (256 lanes) normalize_substitutions + create_nonoverlapping_substitutions_4
//                (:414-479) as a dependency worklist (Kahn order), emit and scratch reset.
// full_simplification (:543-581): process_4 for 350 <= rows < 1e6 unless the old heuristics are
// requested, process_3 otherwise.
__device__ __forceinline__ bool d_is_p4(const ElimArgs &A, uint32_t n) {
  return n >= 350 && n < 1000000 && !A.old_heur;
}

// ---- wide preparation of the largest process_4 clusters (SignalsInformation::new, the uniques
// phase and remove_constraint of substitution_process_4, :156-185): the same work as k_big_prep's
// first phases, spread over a 2-D grid (x: 64 workgroups per cluster, y: the cluster) so a cluster
// of tens of thousands of long rows is not serialised on one CU.  Phase boundaries are kernel
// boundaries; k_big_prep then finishes (remove_signal, rows left for the ordered loop).
constexpr uint32_t kWideMin = 2048;  // rows
constexpr uint32_t kWideX = 64;      // workgroups per cluster
__device__ __forceinline__ bool d_is_wide(const ElimArgs &A, uint32_t n) { return A.wide && d_is_p4(A, n) && n >= kWideMin; }

// per cluster: #entries -> touched-signal list capacity in the pool, counters reset
__global__ __launch_bounds__(256) void k_wide_alloc(ElimArgs A, const uint32_t *ids, uint64_t n_ids) {
  __shared__ unsigned long long s_tot;
  const uint64_t ci = blockIdx.x;
  if (ci >= n_ids) return;
  const uint64_t c = ids[ci], b = A.cl_off[c];
  const uint32_t n = (uint32_t)(A.cl_off[c + 1] - b);
  if (!d_is_wide(A, n)) return;
  if (threadIdx.x == 0) s_tot = 0;
  __syncthreads();
  unsigned long long tot = 0;
  for (uint32_t pos = threadIdx.x; pos < n; pos += blockDim.x) {
    tot += A.rows.len[A.perm[b + pos]];
    A.dead[b + pos] = 0;
  }
  atomicAdd(&s_tot, tot);
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t o = pool_alloc_global(A, s_tot + 1);
    A.big_touch_off[ci] = o == RS_NONE ? 0 : o;
    A.big_touch_n[ci] = 0;
    A.n_sub[c] = 0;
    A.big_alive[ci] = o == RS_NONE ? RS_NONE : 0;  // RS_NONE: failure marker, see k_big_prep
  }
}
// occurrences (init -1 = absent) over non-forbidden signals + the touched list
__global__ __launch_bounds__(256) void k_wide_count(ElimArgs A, const uint32_t *ids, uint64_t n_ids) {
  const uint64_t ci = blockIdx.y;
  const uint64_t c = ids[ci], b = A.cl_off[c];
  const uint32_t n = (uint32_t)(A.cl_off[c + 1] - b);
  if (!d_is_wide(A, n) || A.big_alive[ci] == RS_NONE) return;
  uint32_t *touch = A.pk + A.big_touch_off[ci];
  for (uint32_t pos = blockIdx.x * blockDim.x + threadIdx.x; pos < n; pos += gridDim.x * blockDim.x) {
    const uint32_t r = A.perm[b + pos];
    const uint32_t *k = A.rows.key + A.rows.off[r];
    const uint32_t len = A.rows.len[r];
    for (uint32_t i = 0; i < len; ++i) {
      const uint32_t s = k[i];
      if (A.forb[s]) continue;
      if (atomicAdd(&A.occ[s], 1) == -1) touch[atomicAdd(&A.big_touch_n[ci], 1u)] = s;
    }
  }
}
// -1 based -> counts
__global__ __launch_bounds__(256) void k_wide_conv(ElimArgs A, const uint32_t *ids, uint64_t n_ids) {
  const uint64_t ci = blockIdx.y;
  const uint64_t c = ids[ci], b = A.cl_off[c];
  const uint32_t n = (uint32_t)(A.cl_off[c + 1] - b);
  if (!d_is_wide(A, n) || A.big_alive[ci] == RS_NONE) return;
  const uint32_t *touch = A.pk + A.big_touch_off[ci];
  const uint32_t nt = A.big_touch_n[ci];
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < nt; t += gridDim.x * blockDim.x) A.occ[touch[t]] += 1;
}
// uniques: each row is consumed by its smallest unique signal
__global__ __launch_bounds__(256) void k_wide_uniq(ElimArgs A, const uint32_t *ids, uint64_t n_ids) {
  const uint64_t ci = blockIdx.y;
  const uint64_t c = ids[ci], b = A.cl_off[c];
  const uint32_t n = (uint32_t)(A.cl_off[c + 1] - b);
  if (!d_is_wide(A, n) || A.big_alive[ci] == RS_NONE) return;
  for (uint32_t pos = blockIdx.x * blockDim.x + threadIdx.x; pos < n; pos += gridDim.x * blockDim.x) {
    const uint32_t r = A.perm[b + pos];
    const uint32_t *k = A.rows.key + A.rows.off[r];
    const uint32_t len = A.rows.len[r];
    for (uint32_t i = 0; i < len; ++i)
      if (!A.forb[k[i]] && A.occ[k[i]] == 1) { A.dead[b + pos] = 1; A.order[b + pos] = i; break; }
  }
}
// remove_constraint of the consumed rows
__global__ __launch_bounds__(256) void k_wide_remove(ElimArgs A, const uint32_t *ids, uint64_t n_ids) {
  const uint64_t ci = blockIdx.y;
  const uint64_t c = ids[ci], b = A.cl_off[c];
  const uint32_t n = (uint32_t)(A.cl_off[c + 1] - b);
  if (!d_is_wide(A, n) || A.big_alive[ci] == RS_NONE) return;
  for (uint32_t pos = blockIdx.x * blockDim.x + threadIdx.x; pos < n; pos += gridDim.x * blockDim.x) {
    if (!A.dead[b + pos]) continue;
    const uint32_t r = A.perm[b + pos];
    const uint32_t *k = A.rows.key + A.rows.off[r];
    const uint32_t len = A.rows.len[r];
    for (uint32_t i = 0; i < len; ++i)
      if (!A.forb[k[i]]) atomicSub(&A.occ[k[i]], 1);
  }
}
// the substitutions of the consumed rows (clear_signal_not_normalized; slot order is normalised
// later, like k_big_prep's atomic slots)
__global__ __launch_bounds__(256) void k_wide_clear(ElimArgs A, const uint32_t *ids, uint64_t n_ids) {
  const uint64_t ci = blockIdx.y;
  const uint64_t c = ids[ci], b = A.cl_off[c];
  const uint32_t n = (uint32_t)(A.cl_off[c + 1] - b);
  if (!d_is_wide(A, n) || A.big_alive[ci] == RS_NONE) return;
  Alloc al;
  al.chunk = 256;
  for (uint32_t pos = blockIdx.x * blockDim.x + threadIdx.x; pos < n; pos += gridDim.x * blockDim.x) {
    if (!A.dead[b + pos]) continue;
    const uint32_t r = A.perm[b + pos];
    const uint32_t *k = A.rows.key + A.rows.off[r];
    const Fe *v = A.rows.val + A.rows.off[r];
    const uint32_t oi = A.order[b + pos];
    Fe coef;
    uint64_t to_off;
    uint32_t to_len;
    if (!d_clear_nn(A, al, k, v, A.rows.len[r], oi, coef, to_off, to_len)) { atomicOr(A.err, 8); continue; }
    const uint32_t slot = atomicAdd(&A.n_sub[c], 1u);
    const uint32_t s = k[oi];
    d_set_holder(A, s, b + slot, coef, to_off, to_len);
    A.del[s] = 1;
  }
}

__global__ __launch_bounds__(256) void k_big_prep(ElimArgs A, const uint32_t *ids, uint64_t n_ids) {
  __shared__ uint32_t s_m, s_touch, s_ok, s_alive_part[256];
  __shared__ unsigned long long s_tot;
  __shared__ uint64_t s_touch_off;
  const uint32_t tid = threadIdx.x, nt = blockDim.x;
  Alloc al;
  al.chunk = 64;
  for (uint64_t ci = blockIdx.x; ci < n_ids; ci += gridDim.x) {
    const uint64_t c = ids[ci];
    const uint64_t b = A.cl_off[c], e = A.cl_off[c + 1];
    const uint32_t n = (uint32_t)(e - b);
    unsigned long long t_0 = wall_clock64();
    if (!d_is_p4(A, n)) {  // process_3: no occurrence bookkeeping, every row goes to the loop
      for (uint32_t pos = tid; pos < n; pos += nt) {
        const uint32_t r = A.perm[b + pos];
        A.row_off[b + pos] = A.rows.off[r];
        A.row_len[b + pos] = A.rows.len[r];
      }
      if (tid == 0) { A.n_sub[c] = 0; A.big_touch_n[ci] = 0; A.big_alive[ci] = n; }
      continue;
    }
    if (d_is_wide(A, n)) {  // counted, uniques and their substitutions done by the k_wide_* grid
      __syncthreads();
      if (tid == 0) {
        s_m = A.n_sub[c];
        s_ok = A.big_alive[ci] != RS_NONE;
        s_touch_off = A.big_touch_off[ci];
        s_touch = A.big_touch_n[ci];
      }
      __syncthreads();
      if (!s_ok) {
        if (tid == 0) { A.n_sub[c] = 0; A.big_touch_n[ci] = 0; A.big_alive[ci] = 0; atomicOr(A.err, 8); }
        __syncthreads();
        continue;
      }
    } else {
    uint64_t tot = 0;
    if (tid == 0) { s_m = 0; s_touch = 0; s_ok = 1; s_tot = 0; }
    for (uint32_t pos = tid; pos < n; pos += nt) tot += A.rows.len[A.perm[b + pos]];
    __syncthreads();
    atomicAdd(&s_tot, (unsigned long long)tot);
    __syncthreads();
    if (tid == 0) {
      s_touch_off = pool_alloc_global(A, s_tot + 1);
      if (s_touch_off == RS_NONE) s_ok = 0;
    }
    __syncthreads();
    if (!s_ok) {
      if (tid == 0) { A.n_sub[c] = 0; A.big_touch_n[ci] = 0; A.big_alive[ci] = 0; atomicOr(A.err, 8); }
      __syncthreads();
      continue;
    }
    uint32_t *touch = A.pk + s_touch_off;
    // SignalsInformation::new: occurrences (init -1 = absent) over non-forbidden signals
    for (uint32_t pos = tid; pos < n; pos += nt) {
      uint32_t r = A.perm[b + pos];
      const uint32_t *k = A.rows.key + A.rows.off[r];
      uint32_t len = A.rows.len[r];
      A.dead[b + pos] = 0;
      for (uint32_t i = 0; i < len; ++i) {
        uint32_t s = k[i];
        if (A.forb[s]) continue;
        int32_t old = atomicAdd(&A.occ[s], 1);
        if (old == -1) touch[atomicAdd(&s_touch, 1u)] = s;
      }
    }
    __syncthreads();
    const uint32_t n_touch = s_touch;
    for (uint32_t t = tid; t < n_touch; t += nt) A.occ[touch[t]] += 1;  // -1 based -> count
    __syncthreads();
    // uniques: each row is consumed by its smallest unique signal
    for (uint32_t pos = tid; pos < n; pos += nt) {
      uint32_t r = A.perm[b + pos];
      const uint32_t *k = A.rows.key + A.rows.off[r];
      uint32_t len = A.rows.len[r];
      for (uint32_t i = 0; i < len; ++i)
        if (!A.forb[k[i]] && A.occ[k[i]] == 1) { A.dead[b + pos] = 1; A.order[b + pos] = i; break; }
    }
    __syncthreads();
    for (uint32_t pos = tid; pos < n; pos += nt) {
      if (!A.dead[b + pos]) continue;
      uint32_t r = A.perm[b + pos];
      const uint32_t *k = A.rows.key + A.rows.off[r];
      for (uint32_t i = 0; i < A.rows.len[r]; ++i)
        if (!A.forb[k[i]]) atomicSub(&A.occ[k[i]], 1);  // remove_constraint
    }
    __syncthreads();
    for (uint32_t pos = tid; pos < n; pos += nt) {
      if (!A.dead[b + pos]) continue;
      uint32_t r = A.perm[b + pos];
      const uint32_t *k = A.rows.key + A.rows.off[r];
      const Fe *v = A.rows.val + A.rows.off[r];
      uint32_t oi = A.order[b + pos];
      Fe coef;
      uint64_t to_off;
      uint32_t to_len;
      if (!d_clear_nn(A, al, k, v, A.rows.len[r], oi, coef, to_off, to_len)) { s_ok = 0; continue; }
      uint32_t slot = atomicAdd(&s_m, 1u);
      uint32_t s = k[oi];
      d_set_holder(A, s, b + slot, coef, to_off, to_len);
      A.del[s] = 1;
    }
    }  // not wide
    __syncthreads();
    const uint32_t n_touch = s_touch;
    for (uint32_t i = tid; i < s_m; i += nt) A.occ[A.h_sig[b + i]] = -1;  // remove_signal
    {  // the rows left for the ordered loop, ascending (tmp[b ..]); order kept by a block scan
      const uint32_t per = (n + nt - 1) / nt, lo = min(n, tid * per), hi = min(n, lo + per);
      uint32_t cnt = 0;
      for (uint32_t pos = lo; pos < hi; ++pos) cnt += A.dead[b + pos] ? 0 : 1;
      s_alive_part[tid] = cnt;
      __syncthreads();
      if (tid == 0) {
        uint32_t acc = 0;
        for (uint32_t q = 0; q < nt; ++q) { uint32_t x = s_alive_part[q]; s_alive_part[q] = acc; acc += x; }
        A.big_alive[ci] = acc;
      }
      __syncthreads();
      uint32_t w = s_alive_part[tid];
      for (uint32_t pos = lo; pos < hi; ++pos)
        if (!A.dead[b + pos]) {
          const uint32_t r = A.perm[b + pos];
          A.row_off[b + w] = A.rows.off[r];
          A.row_len[b + w] = A.rows.len[r];
          ++w;
        }
    }
    if (tid == 0) {
      A.n_sub[c] = s_m;
      A.big_touch_off[ci] = s_touch_off;
      A.big_touch_n[ci] = n_touch;
      if (!s_ok) atomicOr(A.err, 8);
      if (A.prof) {
        unsigned long long *P = A.prof + kProfWords * ci;
        P[0] = n; P[4] = wall_clock64() - t_0; P[21] = n_touch;
      }
    }
    __syncthreads();
  }
}

// ---- process_3 without a merge, row-parallel (substitution_process_3 / treat_constraint_3 /
// take_signal_3, simplification_utils.rs:143-154, 259-294, 368-377).  A process_3 row's pivot is its
// largest takeable key; it merges only if that key was already deleted, i.e. only if an earlier-popped
// row has the same pivot.  When no two rows of a cluster share a pivot (checked here with one atomic
// per row), the sequential loop makes every row with a takeable key a new substitution for its pivot
// and every other row a leftover, in pop order -- which this kernel writes directly, every row at
// once: slot = its rank among the pivot rows popped before it, leftover index likewise.  A cluster
// with a shared pivot is left to the ordered loop (skip stays 0).  One workgroup per cluster, grid-
// stride over the tail; the per-signal occurrence slots (unused by process_3, -1) count the pivots
// and are reset.
__global__ __launch_bounds__(256) void k_p3_fast(ElimArgs A, const uint32_t *ids, uint64_t n_ids) {
  __shared__ uint32_t s_dirty, s_ph[256], s_pl[256];
  __shared__ uint64_t s_pz[256], s_base;
  __shared__ unsigned long long s_by;
  const uint32_t tid = threadIdx.x, nt = blockDim.x;
  for (uint64_t ci = blockIdx.x; ci < n_ids; ci += gridDim.x) {
    const uint64_t c = ids[ci];
    const uint64_t b = A.cl_off[c], e = A.cl_off[c + 1];
    const uint32_t n = (uint32_t)(e - b);
    if (d_is_p4(A, n)) continue;
    if (tid == 0) { s_dirty = 0; s_by = 0; }
    __syncthreads();
    for (uint32_t pos = tid; pos < n; pos += nt) {  // take_signal_3 of every row; shared pivots?
      const uint64_t ro = A.row_off[b + pos];
      const uint32_t rl = A.row_len[b + pos];
      uint32_t mi = RS_NONE;
      for (uint32_t i = rl; i-- > 0;)
        if (!A.forb[A.rows.key[ro + i]]) { mi = i; break; }
      A.tmp[b + pos] = mi;
      if (mi != RS_NONE && atomicAdd(&A.occ[A.rows.key[ro + mi]], 1) != -1) s_dirty = 1;
    }
    __syncthreads();
    for (uint32_t pos = tid; pos < n; pos += nt) {
      const uint32_t mi = A.tmp[b + pos];
      if (mi != RS_NONE) A.occ[A.rows.key[A.row_off[b + pos] + mi]] = -1;
    }
    const bool dirty = s_dirty != 0;
    __syncthreads();
    if (dirty) continue;
    // ranks in pop order (descending position) and the pool space of every row: per thread a
    // contiguous segment, segments counted from the last thread down; one allocation per cluster
    const uint32_t per = (n + nt - 1) / nt, lo = min(n, tid * per), hi = min(n, lo + per);
    uint32_t ch = 0, cl = 0;
    uint64_t cz = 0;
    for (uint32_t pos = lo; pos < hi; ++pos) {
      const uint32_t mi = A.tmp[b + pos], len = A.row_len[b + pos];
      if (mi != RS_NONE) {
        ++ch;
        cz += 1 + d_clear_nn_len(A.rows.key + A.row_off[b + pos], len, mi);
      } else if (len) {
        ++cl;
        cz += len;
      }
    }
    s_ph[tid] = ch;
    s_pl[tid] = cl;
    s_pz[tid] = cz;
    __syncthreads();
    uint32_t rh = 0, rlft = 0, th = 0, tl = 0;
    uint64_t oz = 0, tz = 0;
    for (uint32_t q = 0; q < nt; ++q) {
      if (q > tid) { rh += s_ph[q]; rlft += s_pl[q]; oz += s_pz[q]; }
      th += s_ph[q];
      tl += s_pl[q];
      tz += s_pz[q];
    }
    if (tid == 0) s_base = pool_alloc_global(A, tz);
    __syncthreads();
    const uint64_t base = s_base;
    if (base == RS_NONE) continue;  // pool exhausted (err 8 set, the run is retried): left to the loop
    uint64_t o = base + oz;
    unsigned long long by = 0;
    for (uint32_t pos = hi; pos-- > lo;) {
      const uint64_t ro = A.row_off[b + pos];
      const uint32_t len = A.row_len[b + pos];
      const uint32_t *k = A.rows.key + ro;
      const Fe *v = A.rows.val + ro;
      const uint32_t mi = A.tmp[b + pos];
      by += 36ull * len;
      if (mi != RS_NONE) {  // clear_signal_not_normalized: a new substitution, slot = its pop rank
        Fe coef;
        uint64_t to_off;
        uint32_t to_len;
        d_clear_nn_at(A, k, v, len, mi, o, coef, to_off, to_len);
        d_set_holder(A, k[mi], b + rh, coef, to_off, to_len);
        A.del[k[mi]] = 1;
        by += 36ull * to_len;
        o += 1 + to_len;
        ++rh;
      } else if (len) {  // nothing takeable: leftover, as popped (an empty row is dropped, :267)
        for (uint32_t i = 0; i < len; ++i) { A.pk[o + i] = k[i]; A.pv[o + i] = v[i]; }
        A.l_off[b + rlft] = o;
        A.l_len[b + rlft] = len;
        by += 36ull * len;
        o += len;
        ++rlft;
      }
    }
    atomicAdd(&s_by, by);
    __syncthreads();
    if (tid == 0) {
      A.n_sub[c] = th;
      A.n_left[c] = tl;
      A.skip[ci] = 1;
      atomicAdd(A.bytes_main, s_by);
    }
    __syncthreads();
  }
}
// The rest of one row's treat_constraint_3/4 loop on a work list in the pool (single lane; used
// when a list does not fit the LDS buffers of k_big_main).
__device__ inline bool d_treat_scalar(const ElimArgs &A, Alloc &al, uint64_t b, const uint32_t *k, const Fe *v,
                                      uint32_t len, uint32_t &m, uint32_t &nl, bool p4) {
  const FieldP &F = A.F;
  for (;;) {
    if (len == 0) return true;
    uint32_t oi = RS_NONE;
    int32_t occ_ret = -1;
    for (uint32_t i = 0; i < len; ++i) {
      uint32_t s = k[i];
      if (A.forb[s]) continue;
      if (!p4) { oi = i; continue; }  // take_signal_3: the max takeable key (keys ascending)
      if (A.del[s]) { oi = i; break; }
      int32_t c2 = A.occ[s];
      if (c2 < 0) { atomicOr(A.err, 16); c2 = 0; }
      if (occ_ret < 0 || c2 < occ_ret) { oi = i; occ_ret = c2; }
      else if (c2 == occ_ret && k[oi] < s) oi = i;
    }
    if (oi == RS_NONE) {
      uint64_t o = pool_alloc(A, al, len);
      if (o == RS_NONE) return false;
      for (uint32_t i = 0; i < len; ++i) { A.pk[o + i] = k[i]; A.pv[o + i] = v[i]; }
      A.l_off[b + nl] = o;
      A.l_len[b + nl] = len;
      ++nl;
      return true;
    }
    uint32_t out = k[oi];
    int32_t hi = A.holder_idx[out];
    if (hi < 0) {
      Fe coef;
      uint64_t to_off;
      uint32_t to_len;
      if (!d_clear_nn(A, al, k, v, len, oi, coef, to_off, to_len)) return false;
      d_set_holder(A, out, b + m, coef, to_off, to_len);
      ++m;
      A.occ[out] = -1;
      A.del[out] = 1;
      return true;
    }
    uint64_t w_off;
    uint32_t w_len;
    if (!d_merge(A, al, k, v, len, oi, fneg(F, v[oi]), A.h_coef[hi], A.h_off[hi], A.h_len[hi], w_off, w_len)) return false;
    k = A.pk + w_off;
    v = A.pv + w_off;
    len = w_len;
  }
}

// LDS barrier of ONE wave (the workgroup barrier of a 64-lane workgroup, and what a single wave of a
// larger workgroup runs the same code with: d_big_main_cluster, wave_excl_scan)
__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
// exclusive scan of a[0..n) (LDS) by one 64-lane wave; returns the total
__device__ inline uint32_t wave_excl_scan(uint32_t *a, uint32_t n) {
  const uint32_t lane = threadIdx.x;
  uint32_t per = (n + 63) / 64, lo = min(n, lane * per), hi = min(n, lo + per);
  uint32_t sum = 0;
  for (uint32_t i = lo; i < hi; ++i) sum += a[i];
  uint32_t x = sum;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t y = __shfl_up(x, d);
    if ((int)lane >= d) x += y;
  }
  uint32_t acc = x - sum;
  for (uint32_t i = lo; i < hi; ++i) { uint32_t t = a[i]; a[i] = acc; acc += t; }
  uint32_t total = __shfl(x, 63);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  return total;
}
// Per-signal state of a work-list entry, loaded once when the entry enters the list: a row's
// merges never change it (deletions happen only when the row ends in a new substitution).
constexpr uint32_t kStForb = 0xffffffffu, kStTake = 0xfffffffeu;  // else: the holder slot (deleted)
__device__ __forceinline__ uint32_t d_sig_state(const uint8_t *forb, const uint8_t *del, const int32_t *holder, uint32_t s) {
  const uint8_t f = forb[s], d = del[s];
  const int32_t h = holder[s];
  return f ? kStForb : (d ? (uint32_t)h : kStTake);
}
// LDS hand-off between the lanes of one wave (in-order LDS: no workgroup barrier needed)
// min over the wave (every lane active), by DPP: quad swaps, half-row and row mirrors, then the row
// broadcasts; lane 63 ends with the minimum.  The compiler's own lowering of a divergent LDS atomic
// (one iteration per active lane) cost hundreds of cycles per merge.
template <int ctrl, int rmask>
__device__ __forceinline__ uint32_t dpp_min_step(uint32_t v) {
  const uint32_t o = (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, ctrl, rmask, 0xf, false);
  return o < v ? o : v;
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
  v = dpp_min_step<0xB1, 0xf>(v);   // quad_perm [1,0,3,2]
  v = dpp_min_step<0x4E, 0xf>(v);   // quad_perm [2,3,0,1]
  v = dpp_min_step<0x141, 0xf>(v);  // row_half_mirror
  v = dpp_min_step<0x140, 0xf>(v);  // row_mirror
  v = dpp_min_step<0x142, 0xa>(v);  // row_bcast:15 into rows 1, 3
  v = dpp_min_step<0x143, 0xc>(v);  // row_bcast:31 into rows 2, 3
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// lower_bound over a sorted LDS list of n <= 64 keys, branch-free (straight-line code the scheduler
// can interleave with independent work); a[] must be readable up to index 63.  hit: a[pos] == key.
__device__ __forceinline__ uint32_t lds_lb64(const uint32_t *a, uint32_t n, uint32_t key, bool &hit) {
  uint32_t pos = 0;
#pragma unroll
  for (uint32_t step = 32; step >= 1; step >>= 1) {
    const uint32_t q = pos + step;
    const uint32_t v = a[q - 1];
    pos = ((q <= n) & (v < key)) ? q : pos;  // non-short-circuit: the load stays unconditional
  }
  const uint32_t v = a[pos < 63 ? pos : 63];
  const bool lt = (pos < n) & (v < key);  // only when all 64 keys are below key
  hit = (pos < n) & (v == key);
  return pos + (lt ? 1u : 0u);
}
__device__ __forceinline__ uint32_t lds_lower_bound(const uint32_t *a, uint32_t n, uint32_t key) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    if (a[mid] < key) lo = mid + 1; else hi = mid;
  }
  return lo;
}


// CAP: LDS work-list capacity (longer lists take the lane-serial spill path).  512 for the head's
// largest clusters; 256 for the tail, whose many clusters are throughput-bound: 34 KB of LDS lets
// four single-wave workgroups share a CU, as many as the kernel's VGPR budget allows.
template <uint32_t CAP>
struct BigSmem {
  uint32_t wk[2][CAP];
  uint32_t ws[2][CAP];  // per work entry: its signal's state (kStForb / kStTake / holder slot)
  Fe wv[2][CAP];
  uint32_t rk[CAP];
  Fe rv[CAP];
  uint32_t fw[CAP], fr[CAP], lbw[CAP], lbr[CAP];
  uint32_t s_fdel, s_m, s_nl, s_ok;
  unsigned long long s_best;
  uint64_t s_o;
};
// One cluster's ordered loop (the body of k_big_main; k_big_spec also runs it, on wave 0, for
// the clusters whose signals do not fit its table).
template <uint32_t CAP>
__device__ __forceinline__ void d_big_main_cluster(const ElimArgs &A, const uint32_t *ids, uint64_t ci, BigSmem<CAP> &S,
                                                   Alloc &al0) {
  constexpr uint32_t kBigCap = CAP;
  const FieldP &F = A.F;
  auto &wk = S.wk;
  auto &ws = S.ws;
  auto &wv = S.wv;
  auto &rk = S.rk;
  auto &rv = S.rv;
  auto &fw = S.fw;
  auto &fr = S.fr;
  auto &lbw = S.lbw;
  auto &lbr = S.lbr;
  uint32_t &s_fdel = S.s_fdel, &s_m = S.s_m, &s_nl = S.s_nl, &s_ok = S.s_ok;
  unsigned long long &s_best = S.s_best;
  uint64_t &s_o = S.s_o;
  const uint32_t tid = threadIdx.x, nt = 64;
  {
    const uint64_t c = ids[ci];
    const uint64_t b = A.cl_off[c], e = A.cl_off[c + 1];
    unsigned long long t_1 = 0;
    unsigned long long merges = 0, mwork = 0, rows = 0, by = 0;  // by: algorithmic bytes (lane 0)
    unsigned long long tp_piv = 0, tp_hold = 0, tp_merge = 0, tp_x, tp_row = 0, tp_new = 0, tp_r0;  // debug clocks
    unsigned long long tp_q[4] = {0, 0, 0, 0};
    unsigned long long n_packed = 0, n_reg = 0, n_lds = 0, w_packed = 0;  // RS_KCLOCKS path counts
    const bool p4 = d_is_p4(A, (uint32_t)(e - b));
    const bool prof = A.prof != nullptr;
#ifdef RS_KCLOCKS  // per-phase debug clocks inside the loop (each read splits the schedule)
    auto clk = [prof]() -> unsigned long long { return prof ? wall_clock64() : 0ull; };
#else
    auto clk = []() -> unsigned long long { return 0ull; };
#endif
    if (A.skip && A.skip[ci]) return;  // k_p3_fast did this cluster's loop
    t_1 = prof ? wall_clock64() : 0ull;
    if (tid == 0) { s_m = A.n_sub[c]; s_nl = 0; s_ok = 1; }
    wave_sync_lds();
    const uint32_t n_loop = A.big_alive[ci];
    uint64_t nx_off = n_loop ? A.row_off[b + n_loop - 1] : 0;  // descriptor of the next row, one ahead
    uint32_t nx_len = n_loop ? A.row_len[b + n_loop - 1] : 0;
    for (uint32_t qi = n_loop; qi-- > 0;) {  // rows from the back (Vec::pop)
      if (!s_ok) break;
      ++rows;
      tp_r0 = clk();
      const uint64_t r_off = nx_off;
      uint32_t len = nx_len;
      if (qi) { nx_off = A.row_off[b + qi - 1]; nx_len = A.row_len[b + qi - 1]; }
      const uint32_t *k = A.rows.key + r_off;
      const Fe *v = A.rows.val + r_off;
      by += 36ull * len;
      for (uint32_t i = tid; i < len; i += nt) {  // remove_constraint (keys of a row are distinct)
        uint32_t s = k[i];
        if (!A.forb[s] && A.occ[s] >= 0) A.occ[s]--;
      }
      if (len > kBigCap) {
        wave_sync_lds();
        if (tid == 0) {
          uint32_t m = s_m, nl = s_nl;
          if (!d_treat_scalar(A, al0, b, k, v, len, m, nl, p4)) s_ok = 0;
          s_m = m;
          s_nl = nl;
        }
        wave_sync_lds();
        continue;
      }
      for (uint32_t i = tid; i < len; i += nt) {
        const uint32_t kk = k[i];
        wk[0][i] = kk;
        wv[0][i] = v[i];
        ws[0][i] = d_sig_state(A.forb, A.del, A.holder_idx, kk);
      }
      uint32_t cur = 0;
      bool st_ok = true;  // ws[cur] holds the states of wk[cur]
      wave_sync_lds();
      tp_row += clk() - tp_r0;
      while (len > 0) {
        tp_x = clk();
        // take_signal_4 (:379-409): the first deleted key (ascending), else min occurrences, ties
        // -> max id.  take_signal_3 (:368-377): the max takeable key; a conflict iff it is deleted.
        uint32_t oi = RS_NONE;
        bool conflict = false;
        int32_t hs = -1;
        if (len <= 64) {  // one entry per lane: ballots and a butterfly instead of LDS atomics
          const uint32_t key = tid < len ? wk[cur][tid] : 0u;
          const uint32_t stv = tid >= len ? kStForb : (st_ok ? ws[cur][tid] : d_sig_state(A.forb, A.del, A.holder_idx, key));
          const bool tk = stv != kStForb, dl = stv < kStTake;
          const int32_t hsl = dl ? (int32_t)stv : -1;
          const uint64_t tm = __ballot(tk), dm = __ballot(tk && dl);
          int32_t oc = 0;
          if (p4 && tm && !dm && tk) {  // no deleted key: min occurrences (the row's last step)
            oc = A.occ[key];
            if (oc < 0) { atomicOr(A.err, 16); oc = 0; }
          }
          if (tm) {
            if (!p4) {
              oi = 63 - __clzll(tm);
            } else if (dm) {
              oi = __ffsll((long long)dm) - 1;
            } else {
              // min of (occurrences << 32 | ~index): the high words' DPP minimum, then the low words' among it
              const uint32_t vh = tk ? (uint32_t)oc : 0xffffffffu, vl = tk ? 0xffffffffu - tid : 0xffffffffu;
              const uint32_t mh = wave_min_u32(vh);
              oi = 0xffffffffu - wave_min_u32(vh == mh ? vl : 0xffffffffu);
            }
            conflict = (dm >> oi) & 1ull;
            hs = __shfl(hsl, (int)oi);
          }
        } else {
          if (tid == 0) { s_fdel = RS_NONE; s_best = ~0ull; }
          wave_sync_lds();
          for (uint32_t i = tid; i < len; i += nt) {
            uint32_t s = wk[cur][i];
            if (A.forb[s]) continue;
            if (!p4) { atomicMin(&s_best, 0xffffffffull - i); continue; }
            if (A.del[s]) { atomicMin(&s_fdel, i); continue; }
            int32_t o = A.occ[s];
            if (o < 0) { atomicOr(A.err, 16); o = 0; }
            atomicMin(&s_best, ((unsigned long long)(uint32_t)o << 32) | (0xffffffffu - i));  // sorted keys
          }
          wave_sync_lds();
          const uint32_t fdel = s_fdel;
          const unsigned long long best = s_best;
          if (fdel != RS_NONE || best != ~0ull) {
            oi = fdel != RS_NONE ? fdel : 0xffffffffu - (uint32_t)(best & 0xffffffffu);
            conflict = fdel != RS_NONE || (!p4 && A.del[wk[cur][oi]]);
            if (conflict) hs = A.holder_idx[wk[cur][oi]];
          }
        }
        if (oi == RS_NONE) {  // nothing takeable: leftover
          if (tid == 0) { s_o = pool_alloc(A, al0, len); if (s_o == RS_NONE) s_ok = 0; }
          wave_sync_lds();
          by += 36ull * len;
          if (s_ok) {
            const uint64_t o = s_o;
            for (uint32_t i = tid; i < len; i += nt) { A.pk[o + i] = wk[cur][i]; A.pv[o + i] = wv[cur][i]; }
            if (tid == 0) { A.l_off[b + s_nl] = o; A.l_len[b + s_nl] = len; s_nl = s_nl + 1; }
          }
          wave_sync_lds();
          break;
        }
        const uint32_t p = wk[cur][oi];
        if (!conflict) {  // new substitution p = -(work - v_p p) / v_p (clear_signal_not_normalized)
          const unsigned long long tn0 = clk();
          const uint32_t sh = wk[cur][0] == 0 ? 0 : 1;  // {0: 0} is inserted when absent
          const uint32_t mm = len - 1 + sh;
          by += 36ull * mm;
          if (tid == 0) { s_o = pool_alloc(A, al0, mm); if (s_o == RS_NONE) s_ok = 0; }
          wave_sync_lds();
          if (s_ok) {
            const uint64_t o = s_o;
            for (uint32_t i = tid; i < len; i += nt) {
              if (i == oi) continue;
              uint32_t q = (i < oi ? i : i - 1) + sh;
              A.pk[o + q] = wk[cur][i];
              A.pv[o + q] = wv[cur][i];
            }
            if (tid == 0) {
              if (sh) { A.pk[o] = 0; A.pv[o] = fe_zero(); }
              d_set_holder(A, p, b + s_m, fneg(F, wv[cur][oi]), o, mm);
              s_m = s_m + 1;
              A.occ[p] = -1;
              A.del[p] = 1;
            }
          }
          wave_sync_lds();
          tp_new += clk() - tn0;
          break;
        }
        { unsigned long long t = clk(); tp_piv += t - tp_x; tp_x = t; }
        // conflict with holder(p): work = -v_p * R - c2 * (work - v_p p); every lane reads the
        // holder's words itself (same addresses: one request per wave)
        const uint64_t roff = A.h_off[hs];
        const uint32_t rl = A.h_len[hs];
        const Fe c2 = A.h_coef[hs];
        ++merges;
        mwork += len + rl;
        if (rl > kBigCap || len + rl > kBigCap + 1) {  // spill, finish the row on lane 0
          if (tid == 0) { s_o = pool_alloc(A, al0, len); if (s_o == RS_NONE) s_ok = 0; }
          wave_sync_lds();
          if (s_ok) {
            const uint64_t o = s_o;
            for (uint32_t i = tid; i < len; i += nt) { A.pk[o + i] = wk[cur][i]; A.pv[o + i] = wv[cur][i]; }
            wave_sync_lds();
            if (tid == 0) {
              uint32_t m = s_m, nl = s_nl;
              if (!d_treat_scalar(A, al0, b, A.pk + o, A.pv + o, len, m, nl, p4)) s_ok = 0;
              s_m = m;
              s_nl = nl;
            }
          }
          wave_sync_lds();
          break;
        }
        { unsigned long long t = clk(); tp_hold += t - tp_x; tp_x = t; }
        const Fe coef = fneg(F, wv[cur][oi]);
        const uint32_t nx = cur ^ 1;
#ifdef RS_KCLOCKS
        if (len + rl <= 64) { ++n_packed; w_packed += len + rl; } else if (len <= 64 && rl <= 64) ++n_reg; else ++n_lds;
#endif
        if (len + rl <= 64) {
          // ---- packed register merge: lanes [0, len) hold the work, lanes [len, len + rl) the
          // RHS, so the whole step costs one product latency; positions by ballots
          const uint32_t l = tid;
          const bool isw = l < len, isr = !isw && l < len + rl;
          const uint32_t j = l - len;
          uint32_t key = 0;
          Fe val = fe_zero();
          if (isw) { key = wk[cur][l]; val = wv[cur][l]; }
          uint32_t stv = !isw ? kStForb : (st_ok ? ws[cur][l] : d_sig_state(A.forb, A.del, A.holder_idx, key));
          if (isr) {
            key = A.pk[roff + j];
            val = A.pv[roff + j];
            rk[j] = key;
            stv = d_sig_state(A.forb, A.del, A.holder_idx, key);  // in flight under the product
          }
          const unsigned long long tq0 = clk();
          wave_sync();  // the RHS keys are in LDS (one wave: no workgroup barrier needed)
          // one search per lane in the other list (work lanes in the RHS, RHS lanes in the work) on
          // the keys alone, and the product on the value: two independent chains in one basic block,
          // so the LDS reads of the search hide under the product's latency
          const uint32_t *ok = isw ? rk : wk[cur];
          const uint32_t on = isw ? rl : (isr ? len : 0u);
          bool hit;
          const uint32_t lb = lds_lb64(ok, on, key, hit);
          val = fmul256(F, isw ? c2 : coef, val);
          const unsigned long long tq1 = clk();
          if (isr) rv[j] = val;
          wave_sync();
          const unsigned long long tq2 = clk();
          tp_q[0] += tq0 - tp_x;  // loads
          tp_q[1] += tq1 - tq0;   // search + product
          tp_q[2] += tq2 - tq1;   // barrier
          bool keep = false;
          if (isw) {  // -c2*v (+ coef*rv when the RHS has the key)
            if (l != oi) {
              val = hit ? fsub(F, rv[lb], val) : fneg(F, val);
              keep = !fe_is_zero(val);
            }
          } else if (isr) {  // RHS-only keys: coef*rv
            keep = !hit && !fe_is_zero(val);
          }
          const unsigned long long tq3 = clk();
          tp_q[3] += tq3 - tq2;  // combine (the scatter is in tp_merge - sum)
          const uint64_t km = __ballot(keep);
          const uint64_t wmk = len >= 64 ? km : (km & ((1ull << len) - 1ull)), rmk = km >> len;
          auto below = [](uint64_t m, uint32_t k) -> uint32_t {
            return (uint32_t)__popcll(k >= 64 ? m : (m & ((1ull << k) - 1ull)));
          };
          if (keep) {
            const uint32_t q = isw ? below(wmk, l) + below(rmk, lb) : below(rmk, j) + below(wmk, lb);
            wk[nx][q] = key;
            wv[nx][q] = val;
            ws[nx][q] = stv;
          }
          wave_sync();  // LDS-only hand-off inside the wave
          st_ok = true;
          const uint32_t nlen = (uint32_t)__popcll(km);
          cur = nx;
          by += 36ull * (len + rl + nlen);
          tp_merge += clk() - tp_x;
          len = nlen;
          continue;
        }
        if (len <= 64 && rl <= 64) {
          // ---- register merge: lane l holds work entry l and RHS entry l; positions by ballots
          const uint32_t l = tid;
          uint32_t wkey = 0, rkey = RS_NONE;
          Fe wval = fe_zero(), rval = fe_zero();
          if (l < rl) { rkey = A.pk[roff + l]; rval = A.pv[roff + l]; }
          if (l < len) { wkey = wk[cur][l]; wval = wv[cur][l]; }
          if (l < len) wval = fmul256(F, c2, wval);   // one product per entry, both lists at once
          if (l < rl) rval = fmul256(F, coef, rval);
          if (l < rl) { rk[l] = rkey; rv[l] = rval; }
          wave_sync_lds();
          bool keep_w = false, keep_r = false;
          uint32_t lb_w = 0, lb_r = 0;
          if (l < len && l != oi) {  // -c2*v (+ coef*rv when the RHS has the key)
            lb_w = lds_lower_bound(rk, rl, wkey);
            wval = fneg(F, wval);
            if (lb_w < rl && rk[lb_w] == wkey) wval = fadd(F, rv[lb_w], wval);
            keep_w = !fe_is_zero(wval);
          }
          if (l < rl) {  // RHS-only keys: coef*rv
            lb_r = lds_lower_bound(wk[cur], len, rkey);
            keep_r = !(lb_r < len && wk[cur][lb_r] == rkey) && !fe_is_zero(rval);
          }
          const uint64_t wmk = __ballot(keep_w), rmk = __ballot(keep_r);
          auto below = [](uint64_t m, uint32_t k) -> uint32_t {
            return (uint32_t)__popcll(k >= 64 ? m : (m & ((1ull << k) - 1ull)));
          };
          if (keep_w) {
            const uint32_t q = below(wmk, l) + below(rmk, lb_w);
            wk[nx][q] = wkey;
            wv[nx][q] = wval;
          }
          if (keep_r) {
            const uint32_t q = below(rmk, l) + below(wmk, lb_r);
            wk[nx][q] = rkey;
            wv[nx][q] = rval;
          }
          wave_sync_lds();
          const uint32_t nlen = (uint32_t)(__popcll(wmk) + __popcll(rmk));
          cur = nx;
          st_ok = false;
          by += 36ull * (len + rl + nlen);
          tp_merge += clk() - tp_x;
          len = nlen;
          continue;
        }
        for (uint32_t j = tid; j < rl; j += nt) { rk[j] = A.pk[roff + j]; rv[j] = A.pv[roff + j]; }
        wave_sync_lds();
        // one product per entry, all lanes at once: work entries c2*v, RHS entries coef*rv
        for (uint32_t q = tid; q < len + rl; q += nt) {
          if (q < len) wv[cur][q] = fmul256(F, c2, wv[cur][q]);
          else rv[q - len] = fmul256(F, coef, rv[q - len]);
        }
        wave_sync_lds();
        for (uint32_t i = tid; i < len; i += nt) {  // work keys: -c2*v (+ coef*rv when the RHS has the key)
          if (i == oi) { fw[i] = 0; continue; }
          const uint32_t key = wk[cur][i];
          const uint32_t lb = lds_lower_bound(rk, rl, key);
          Fe x = fneg(F, wv[cur][i]);
          if (lb < rl && rk[lb] == key) x = fadd(F, rv[lb], x);
          wv[cur][i] = x;
          lbw[i] = lb;
          fw[i] = fe_is_zero(x) ? 0 : 1;
        }
        for (uint32_t j = tid; j < rl; j += nt) {  // RHS-only keys: coef*rv
          const uint32_t key = rk[j];
          const uint32_t lb = lds_lower_bound(wk[cur], len, key);
          if (lb < len && wk[cur][lb] == key) { fr[j] = 0; lbr[j] = RS_NONE; continue; }
          lbr[j] = lb;
          fr[j] = fe_is_zero(rv[j]) ? 0 : 1;
        }
        wave_sync_lds();
        const uint32_t tw = wave_excl_scan(fw, len);
        const uint32_t tr = wave_excl_scan(fr, rl);
        for (uint32_t i = tid; i < len; i += nt) {
          if (i == oi || fe_is_zero(wv[cur][i])) continue;
          const uint32_t lb = lbw[i];
          const uint32_t q = fw[i] + (lb < rl ? fr[lb] : tr);
          wk[nx][q] = wk[cur][i];
          wv[nx][q] = wv[cur][i];
        }
        for (uint32_t j = tid; j < rl; j += nt) {
          const uint32_t lb = lbr[j];
          if (lb == RS_NONE || fe_is_zero(rv[j])) continue;
          const uint32_t q = fr[j] + (lb < len ? fw[lb] : tw);
          wk[nx][q] = rk[j];
          wv[nx][q] = rv[j];
        }
        wave_sync_lds();
        cur = nx;
        st_ok = false;
        by += 36ull * (len + rl + tw + tr);
        tp_merge += clk() - tp_x;
        len = tw + tr;
      }
    }
    if (tid == 0) {
      A.n_sub[c] = s_m;
      A.n_left[c] = s_nl;
      atomicAdd(A.bytes_main, by);
      if (!s_ok) atomicOr(A.err, 8);
      if (A.prof) {
        unsigned long long *P = A.prof + kProfWords * ci;
        // [2] rows, [5] wall; RS_KCLOCKS builds: [3] row starts, [8..10] packed / register / LDS
        // merges, [11] new substitutions, [12] lanes used by packed merges, [13..15] pivot / holder /
        // merge time (100 MHz ticks)
        P[2] = rows; P[5] = wall_clock64() - t_1;
        P[3] = tp_row; P[8] = n_packed; P[9] = n_reg; P[10] = n_lds; P[11] = tp_new; P[12] = w_packed;
        P[13] = tp_piv; P[14] = tp_hold; P[15] = tp_merge;
        P[16] = tp_q[0]; P[17] = tp_q[1]; P[18] = tp_q[2]; P[19] = tp_q[3];  // packed merge: loads / search+product / hand-off / combine+scatter
        (void)merges; (void)mwork;
      }
    }
    wave_sync_lds();
  }
}
template <uint32_t CAP>
__global__ __launch_bounds__(64) void k_big_main(ElimArgs A, const uint32_t *ids, uint64_t n_ids) {
  __shared__ BigSmem<CAP> S;
  Alloc al0;  // lane 0's allocator
  al0.chunk = 4096;
  for (uint64_t ci = blockIdx.x; ci < n_ids; ci += gridDim.x) d_big_main_cluster<CAP>(A, ids, ci, S, al0);
}

// LDS signal-table encoding of the head's speculative loop (spec_loop.hpp): empty slot / deleted bit
constexpr uint32_t kTabEmpty = 0xffffffffu, kStDel = 0x80000000u;

// multi_inv (modular_arithmetic.rs:71-91) of the pivot coefficients, before normalisation (exact
// inverses, so the chunking is free).
// The same inverses with one Fermat inversion per cluster (one workgroup each): thread t takes a
// contiguous chunk of the pivots, the chunks' products are scanned across the workgroup both ways
// (prefix X_t, suffix S_t) in LDS, and the inverse of the whole product -- the only inversion --
// gives every chunk the inverse of its running product (inv_T * S_{t+1}), from which the chunk walks
// back as Montgomery's trick does.  A chain-per-lane k_batch_inv needs one inversion per 16 pivots
// (hundreds of waves for the head's clusters, queued behind the tail's workgroups for CUs); this is
// one inversion's latency per cluster.  ftmp[slot] <- h_coef[slot]^-1.
__global__ __launch_bounds__(256) void k_batch_inv_tree(ElimArgs A, const uint32_t *ids, uint64_t n_ids) {
  const FieldP &F = A.F;
  __shared__ Fe s_x[256], s_y[256];
  __shared__ Fe s_inv;
  const uint32_t t = threadIdx.x;
  for (uint64_t ci = blockIdx.x; ci < n_ids; ci += gridDim.x) {
    const uint64_t c = ids[ci];
    const uint64_t b = A.cl_off[c];
    const uint32_t m = A.n_sub[c];
    if (m == 0) continue;
    if (t == 0) atomicAdd(A.bytes_fin, 96ull * m);  // per pivot: its coefficient, the prefix written and read back
    const uint32_t per = (m + 255) / 256, c0 = min(m, t * per), c1 = min(m, c0 + per);
    Fe acc = F.one;  // the chunk's running product, kept in ftmp
    for (uint32_t i = c0; i < c1; ++i) {
      acc = i == c0 ? A.h_coef[b + i] : fmul(F, acc, A.h_coef[b + i]);
      A.ftmp[b + i] = acc;
    }
    // inclusive prefix (s_x) and suffix (s_y) products of the chunk totals
    s_x[t] = acc;
    s_y[t] = acc;
    __syncthreads();
    for (uint32_t d = 1; d < 256; d <<= 1) {
      const Fe px = t >= d ? s_x[t - d] : F.one, py = t + d < 256 ? s_y[t + d] : F.one;
      __syncthreads();
      if (t >= d) s_x[t] = fmul(F, s_x[t], px);
      if (t + d < 256) s_y[t] = fmul(F, s_y[t], py);
      __syncthreads();
    }
    if (t == 0) s_inv = finv(F, s_x[255]);
    __syncthreads();
    if (c0 < c1) {
      const Fe X = t ? s_x[t - 1] : F.one;                          // product before the chunk
      Fe inv = t < 255 ? fmul(F, s_inv, s_y[t + 1]) : s_inv;            // (X * chunk product)^-1
      for (uint32_t i = c1 - 1; i > c0; --i) {
        const Fe h = A.h_coef[b + i];
        A.ftmp[b + i] = fmul(F, fmul(F, X, A.ftmp[b + i - 1]), inv);  // prefix through i-1, over prefix through i
        inv = fmul(F, inv, h);
      }
      A.ftmp[b + c0] = fmul(F, X, inv);
    }
    __syncthreads();
  }
}
// normalize_substitutions (:414-437) of the split clusters: every RHS times its pivot's inverse,
// one lane per substitution over a 2-D grid like k_batch_inv's
__global__ __launch_bounds__(256) void k_normalize(ElimArgs A, const uint32_t *ids, uint64_t n_ids) {
  const FieldP &F = A.F;
  unsigned long long by = 0;
  for (uint64_t ci = blockIdx.y; ci < n_ids; ci += gridDim.y) {
    const uint64_t c = ids[ci];
    const uint64_t b = A.cl_off[c];
    const uint32_t m = A.n_sub[c];
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
      const Fe inv_i = A.ftmp[b + i];
      Fe *vv = A.pv + A.h_off[b + i];
      const uint32_t l = A.h_len[b + i];
      for (uint32_t t = 0; t < l; ++t) vv[t] = fmul(F, vv[t], inv_i);
      by += 64ull * (l + 1);
    }
  }
  wave_atomic_add(A.bytes_fin, by);
}

// The same over the slot space of many clusters at once (the tail stream's clusters, cls == 1):
// chunks of 64 slots cross cluster boundaries, so tens of thousands of small clusters share a few
// thousand inversions instead of waiting on one each.
__device__ __forceinline__ bool d_inv_slot(const ElimArgs &A, const uint32_t *cid, const uint8_t *cls, uint64_t sl) {
  const uint32_t c = cid[sl];
  return cls[c] == 1 && sl - A.cl_off[c] < A.n_sub[c];
}
__global__ void k_batch_inv_flat(ElimArgs A, const uint32_t *cid, const uint8_t *cls, uint64_t n_slots) {
  const FieldP &F = A.F;
  unsigned long long by = 0;  // per pivot: its coefficient, the prefix written and read back
  for (uint64_t t = gtid(); t * 64 < n_slots; t += gstride()) {
    const uint64_t s0 = t * 64, s1 = min<uint64_t>(n_slots, s0 + 64);
    Fe acc = F.one;
    uint64_t last = RS_NONE;
    for (uint64_t sl = s0; sl < s1; ++sl) {
      if (!d_inv_slot(A, cid, cls, sl)) continue;
      acc = fmul(F, acc, A.h_coef[sl]);
      A.ftmp[sl] = acc;  // prefix product up to sl
      last = sl;
      by += 96;
    }
    if (last == RS_NONE) continue;
    Fe inv = finv(F, acc);
    uint64_t cur = last;  // valid slot whose predecessor is being looked for
    for (uint64_t sl = last; sl-- > s0;) {
      if (!d_inv_slot(A, cid, cls, sl)) continue;
      const Fe inv_cur = fmul(F, A.ftmp[sl], inv);
      inv = fmul(F, inv, A.h_coef[cur]);
      A.ftmp[cur] = inv_cur;
      cur = sl;
    }
    A.ftmp[cur] = inv;
  }
  wave_atomic_add(A.bytes_fin, by);
}

// Lane-serial composition of slot `sl` (raw_substitution key by key, ascending): the fallback for
// lists the wave path does not hold.
__device__ inline bool d_compose_serial(const ElimArgs &A, Alloc &al, uint64_t sl, unsigned long long &by) {
  uint64_t off = A.h_off[sl];
  uint32_t len = A.h_len[sl];
  const uint32_t *kk = A.pk + off;
  uint64_t bound = len;
  for (uint32_t t = 0; t < len; ++t) {
    int32_t hs = A.holder_idx[kk[t]];
    if (hs >= 0) bound += A.h_len[hs];
  }
  uint64_t buf0 = pool_alloc(A, al, bound), buf1 = pool_alloc(A, al, bound);
  if (buf0 == RS_NONE || buf1 == RS_NONE) return false;
  const uint64_t orig_off = off;
  const uint32_t orig_len = len;
  uint64_t dst = buf0;
  for (uint32_t t = 0; t < orig_len; ++t) {
    uint32_t key = A.pk[orig_off + t];
    int32_t hs = A.holder_idx[key];
    if (hs < 0) continue;
    uint32_t nl2;
    d_raw_sub_into(A, off, len, key, A.h_off[hs], A.h_len[hs], dst, nl2);
    off = dst;
    len = nl2;
    dst = dst == buf0 ? buf1 : buf0;
  }
  A.h_off[sl] = off;
  A.h_len[sl] = len;
  by += 36ull * (bound + len);
  return true;
}


constexpr uint32_t kComposeCap = 256;  // entries one wave composes in LDS
constexpr uint32_t kFinWaveBelow = 512;  // tail clusters under this many rows finish on one wave (k_big_finish)
#ifndef RS_FIN_G
#define RS_FIN_G 8
#endif
constexpr uint32_t kFinG = RS_FIN_G, kFinPer = 64 / kFinG;  // k_big_finish: lanes per composition group, groups per wave

// Composition of slot `sl` by one wave as a k-way merge of sorted runs (every dependency already
// final; the same result as d_compose_wave): run 0 = the slot's own (non-deleted) entries, run 1 + j =
// R(t_j) of its j-th deleted key, scaled by c_j at read time.  Each run is sorted by key, so an
// element's place in the sorted union is its index in its run plus, per other run, a binary search
// of its key (ties: the earlier run first); the first run holding a key is its head and sums the
// equal keys of the later runs.  Only the keys live in LDS (values are read where they lie), so the
// cost per element is D searches, not a sort: a chain link (D = 1, a long R(t)) composes in
// O(E / 64) instead of bitonic passes or a lane-serial merge.
// Scratch: K[KCAP] keys, OI[OCAP] own entry -> RHS index, RS[DCAP + 2] run starts, DOF[DCAP] /
// DMU[DCAP] dependency offsets / coefficients, HB[KCAP / 64] head bits, HP[KCAP / 64 + 1] prefixes.
// Returns 0 on success, 1 when the lists do not fit (caller falls back), 2 on pool exhaustion.
struct MergeScratch {
  uint32_t *K;
  uint16_t *OI;
  uint32_t *RS;
  uint64_t *DOF;
  Fe *DMU;
  uint64_t *HB;
  uint32_t *HP;
};
template <uint32_t KCAP, uint32_t OCAP, uint32_t DCAP>
__device__ inline int d_compose_merge(const ElimArgs &A, Alloc &al, uint64_t sl, const MergeScratch &M,
                                      unsigned long long &by, uint32_t sort_runs = ~0u, uint32_t sort_cap = 0) {
  static_assert(KCAP % 64 == 0 && KCAP / 64 <= 4096, "merge scratch");
  const FieldP &F = A.F;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t lt = lane ? ((1ull << lane) - 1ull) : 0ull;
  const uint64_t off = A.h_off[sl];
  const uint32_t len = A.h_len[sl];
  if (len > OCAP + DCAP) return 1;
  // pass 1: own entries (their RHS index) and dependencies (offset, length prefix, coefficient)
  uint32_t n_own = 0, D = 0, tot = 0;
  for (uint32_t c0 = 0; c0 < len; c0 += 64) {
    const uint32_t i = c0 + lane;
    int32_t hs = -1;
    uint32_t dl = 0;
    if (i < len) {
      hs = A.holder_idx[A.pk[off + i]];
      if (hs >= 0) dl = A.h_len[hs];
    }
    const uint64_t dm = __ballot(hs >= 0), om = __ballot(i < len && hs < 0);
    uint32_t x = dl;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(x, d);
      if ((int)lane >= d) x += y;
    }
    const uint32_t ctot = __shfl(x, 63), nd = (uint32_t)__popcll(dm), no = (uint32_t)__popcll(om);
    if (n_own + no > OCAP || D + nd > DCAP || n_own + no + tot + ctot > KCAP) return 1;
    if (hs >= 0) {
      const uint32_t r = D + (uint32_t)__popcll(dm & lt);
      M.RS[1 + r] = tot + x - dl;  // made absolute below
      M.DOF[r] = A.h_off[hs];
      M.DMU[r] = A.pv[off + i];
    } else if (i < len) {
      M.OI[n_own + (uint32_t)__popcll(om & lt)] = (uint16_t)i;
    }
    n_own += no;
    D += nd;
    tot += ctot;
  }
  const uint32_t E = n_own + tot, W = (E + 63) / 64;
  if (D > sort_runs && E <= sort_cap) return 1;  // the caller's sort is cheaper for many short runs
  wave_sync();
  for (uint32_t j = lane; j < D; j += 64) M.RS[1 + j] += n_own;
  if (lane == 0) {
    M.RS[0] = 0;
    M.RS[D + 1] = E;
  }
  for (uint32_t w = lane; w < W; w += 64) M.HB[w] = 0;
  wave_sync();
  // the keys of every run, concatenated (consecutive lanes on consecutive entries of a run)
  for (uint32_t x = lane; x < E; x += 64) {
    if (x < n_own) {
      M.K[x] = A.pk[off + M.OI[x]];
    } else {
      uint32_t lo = 1, hi = D + 1;  // the run: last j with RS[j] <= x
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (M.RS[mid] <= x) lo = mid; else hi = mid;
      }
      M.K[x] = A.pk[M.DOF[lo - 1] + (x - M.RS[lo])];
    }
  }
  wave_sync();
  // an element's run, its sorted rank, and whether it heads its key (pass 2: head bits; pass 3: output)
  auto locate = [&](uint32_t x, uint32_t &a, uint32_t &rank, bool &head) {
    uint32_t lo = 0, hi = D + 1;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (M.RS[mid] <= x) lo = mid; else hi = mid;
    }
    a = lo;
    const uint32_t k = M.K[x];
    rank = x - M.RS[a];
    head = true;
    for (uint32_t b = 0; b <= D; ++b) {
      if (b == a) continue;
      uint32_t s = M.RS[b], e = M.RS[b + 1];
      const uint32_t s0 = s;
      if (b < a) {  // elements <= k
        while (s < e) {
          const uint32_t m = (s + e) >> 1;
          if (M.K[m] <= k) s = m + 1; else e = m;
        }
        if (s > s0 && M.K[s - 1] == k) head = false;
      } else {  // elements < k
        while (s < e) {
          const uint32_t m = (s + e) >> 1;
          if (M.K[m] < k) s = m + 1; else e = m;
        }
      }
      rank += s - s0;
    }
  };
  for (uint32_t x = lane; x < E; x += 64) {
    uint32_t a, rank;
    bool head;
    locate(x, a, rank, head);
    if (head) atomicOr((unsigned long long *)&M.HB[rank >> 6], 1ull << (rank & 63));
  }
  wave_sync();
  uint32_t run_tot = 0;
  for (uint32_t w0 = 0; w0 < W; w0 += 64) {  // word prefixes of the head bits
    const uint32_t w = w0 + lane;
    const uint32_t c = w < W ? (uint32_t)__popcll(M.HB[w]) : 0u;
    uint32_t x = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(x, d);
      if ((int)lane >= d) x += y;
    }
    if (w < W) M.HP[w] = run_tot + x - c;
    run_tot += __shfl(x, 63);
  }
  uint64_t o = 0;
  if (lane == 0) o = pool_alloc(A, al, run_tot ? run_tot : 1);
  o = __shfl(o, 0);
  if (o == RS_NONE) return 2;
  wave_sync();
  auto value = [&](uint32_t run, uint32_t x) -> Fe {
    if (run == 0) return A.pv[off + M.OI[x]];
    return fmul(F, M.DMU[run - 1], A.pv[M.DOF[run - 1] + (x - M.RS[run])]);
  };
  for (uint32_t x = lane; x < E; x += 64) {
    uint32_t a, rank;
    bool head;
    locate(x, a, rank, head);
    if (!head) continue;
    const uint32_t k = M.K[x];
    Fe v = value(a, x);
    for (uint32_t b = a + 1; b <= D; ++b) {  // the equal keys of the later runs
      uint32_t s = M.RS[b], e = M.RS[b + 1];
      while (s < e) {
        const uint32_t m = (s + e) >> 1;
        if (M.K[m] < k) s = m + 1; else e = m;
      }
      if (s < M.RS[b + 1] && M.K[s] == k) v = fadd(F, v, value(b, s));
    }
    const uint32_t slot = M.HP[rank >> 6] + (uint32_t)__popcll(M.HB[rank >> 6] & ((1ull << (rank & 63)) - 1ull));
    A.pk[o + slot] = k;
    A.pv[o + slot] = v;
  }
  if (lane == 0) {
    A.h_off[sl] = o;
    A.h_len[sl] = run_tot;
    by += 36ull * (len + tot + run_tot);
  }
  return 0;
}

// Composition of slot `sl` by one wave (every dependency already final): the result is the sum of
// the slot's non-deleted entries and c_t * R(t) for each deleted key t (coefficient c_t), with
// every key kept even when its sum is zero -- the value raw_substitution applied key by key gives
// (algebra.rs:1279-1294), in any order.  Entries are gathered into LDS (one product per
// dependency entry, spread over the lanes), bitonic-sorted by key, summed per key and written out.
// Returns 0 on success, 1 when the lists do not fit (caller falls back), 2 on pool exhaustion.
__device__ inline int d_compose_wave(const ElimArgs &A, Alloc &al, uint64_t sl, uint64_t *S, Fe *V,
                                     uint32_t *dex, uint64_t *dof, Fe *dmu, unsigned long long &by,
                                     bool merge_few = false) {
  const FieldP &F = A.F;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t off = A.h_off[sl];
  const uint32_t len = A.h_len[sl];
  if (len > 64) return 1;
  uint32_t key = 0;
  Fe val = fe_zero();
  int32_t hs = -1;
  uint32_t dl = 0;
  uint64_t doff = 0;
  if (lane < len) {
    key = A.pk[off + lane];
    val = A.pv[off + lane];
    hs = A.holder_idx[key];
    if (hs >= 0) { dl = A.h_len[hs]; doff = A.h_off[hs]; }
  }
  const uint64_t dm = __ballot(hs >= 0), om = __ballot(lane < len && hs < 0);
  const uint64_t lt = lane ? ((1ull << lane) - 1ull) : 0ull;
  const uint32_t n_own = (uint32_t)__popcll(om);
  // exclusive prefix of the dependency lengths
  uint32_t x = dl;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t y = __shfl_up(x, d);
    if ((int)lane >= d) x += y;
  }
  const uint32_t tot = __shfl(x, 63), ex = x - dl;
  const uint32_t E = n_own + tot;
  if (E > kComposeCap) return 1;
  if (merge_few && __popcll(dm) <= 4) return 3;  // few runs: d_compose_merge is cheaper
  if (hs >= 0) {
    const uint32_t r = (uint32_t)__popcll(dm & lt);
    dex[r] = ex;
    dof[r] = doff;
    dmu[r] = val;
  }
  if (lane < len && hs < 0) {
    const uint32_t q = (uint32_t)__popcll(om & lt);
    S[q] = ((uint64_t)key << 32) | q;
    V[q] = val;
  }
  wave_sync();
  const uint32_t D = (uint32_t)__popcll(dm);
  for (uint32_t e = lane; e < tot; e += 64) {  // c_t * R(t), one product per entry
    uint32_t lo = 0, hi = D;                     // last dependency with dex <= e
    while (hi - lo > 1) {
      uint32_t mid = (lo + hi) >> 1;
      if (dex[mid] <= e) lo = mid; else hi = mid;
    }
    const uint64_t src = dof[lo] + (e - dex[lo]);
    const uint32_t q = n_own + e;
    S[q] = ((uint64_t)A.pk[src] << 32) | q;
    V[q] = fmul(F, dmu[lo], A.pv[src]);
  }
  uint32_t np2 = 1;
  while (np2 < E) np2 <<= 1;
  for (uint32_t q = E + lane; q < np2; q += 64) S[q] = ~0ull;
  wave_sync();
  for (uint32_t k = 2; k <= np2; k <<= 1) {  // bitonic sort of (key, position)
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t t = lane; t < np2 / 2; t += 64) {
        const uint32_t i = (t / j) * 2 * j + (t % j), pr = i + j;
        const uint64_t a = S[i], c = S[pr];
        if ((a > c) == ((i & k) == 0)) { S[i] = c; S[pr] = a; }
      }
      wave_sync();
    }
  }
  uint64_t o = 0;
  if (lane == 0) o = pool_alloc(A, al, E ? E : 1);
  o = __shfl(o, 0);
  if (o == RS_NONE) return 2;
  uint32_t run = 0;
  for (uint32_t cb = 0; cb < E; cb += 64) {  // one output entry per distinct key, values summed
    const uint32_t p = cb + lane;
    const uint32_t k0 = p < E ? (uint32_t)(S[p] >> 32) : 0u;
    const bool head = p < E && (p == 0 || (uint32_t)(S[p - 1] >> 32) != k0);
    const uint64_t hm = __ballot(head);
    if (head) {
      Fe v = V[(uint32_t)S[p]];
      for (uint32_t q = p + 1; q < E && (uint32_t)(S[q] >> 32) == k0; ++q) v = fadd(F, v, V[(uint32_t)S[q]]);
      const uint64_t w = o + run + (uint32_t)__popcll(hm & lt);
      A.pk[w] = k0;
      A.pv[w] = v;
    }
    run += (uint32_t)__popcll(hm);
  }
  if (lane == 0) {
    A.h_off[sl] = o;
    A.h_len[sl] = run;
    by += 36ull * (len + tot + run);
  }
  return 0;
}

// Up to 64 / G compositions at once by one wave, G lanes each -- the same result as d_compose_wave.
// Most substitutions of the tail's clusters are short (the metric circuit's: 2.6 right-hand-side
// entries composing to 3.7), so one composition by a whole wave is a chain of dependent loads with
// the wave idle; G-lane groups overlap 64 / G of those chains.  Group g = lane / G composes slot `sl`
// (group-uniform; ~0: none) in its share of the wave's buffers (4G entries of S / V, G of dex / dof /
// dmu).  Returns the ballot of the group leaders (lane % G == 0) whose composition does not fit (right-
// hand side over G entries, or over 4G composed): the caller composes those with the whole wave.
// oom: the pool is exhausted (group-uniform).
template <uint32_t G>
__device__ inline uint64_t d_compose_groups(const ElimArgs &A, Alloc &al, uint64_t sl, uint64_t *S, Fe *V, uint32_t *dex,
                                            uint64_t *dof, Fe *dmu, unsigned long long &by, bool &oom) {
  static_assert(G >= 2 && G <= 32 && (G & (G - 1)) == 0, "group size");
  constexpr uint32_t CAP = 4 * G;
  const FieldP &F = A.F;
  const uint32_t lane = threadIdx.x & 63, g = lane / G, li = lane % G, g0 = g * G;
  uint64_t *gS = S + g * CAP;
  Fe *gV = V + g * CAP;
  uint32_t *gdex = dex + g0;
  uint64_t *gdof = dof + g0;
  Fe *gdmu = dmu + g0;
  const uint64_t gmask = ((1ull << G) - 1ull) << g0;
  const uint64_t ltg = (lane ? ((1ull << lane) - 1ull) : 0ull) & gmask;
  const bool has = sl != ~0ull;
  uint64_t off = 0;
  uint32_t len = 0;
  if (has) {
    off = A.h_off[sl];
    len = A.h_len[sl];
  }
  bool fit = has && len <= G;
  uint32_t key = 0, dl = 0;
  Fe val = fe_zero();
  int32_t hs = -1;
  uint64_t doff = 0;
  if (fit && li < len) {
    key = A.pk[off + li];
    val = A.pv[off + li];
    hs = A.holder_idx[key];
    if (hs >= 0) { dl = A.h_len[hs]; doff = A.h_off[hs]; }
  }
  const uint64_t dm = __ballot(hs >= 0) & gmask, om = __ballot(fit && li < len && hs < 0) & gmask;
  uint32_t x = dl;  // inclusive prefix of the dependency lengths over the group
#pragma unroll
  for (uint32_t d = 1; d < G; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, G);
    if (li >= d) x += y;
  }
  const uint32_t tot = __shfl(x, g0 + G - 1), n_own = (uint32_t)__popcll(om), D = (uint32_t)__popcll(dm);
  const uint32_t E = n_own + tot;
  fit = fit && E <= CAP;
  if (fit && hs >= 0) {
    const uint32_t r = (uint32_t)__popcll(dm & ltg);
    gdex[r] = x - dl;
    gdof[r] = doff;
    gdmu[r] = val;
  }
  if (fit && li < len && hs < 0) {
    const uint32_t q = (uint32_t)__popcll(om & ltg);
    gS[q] = ((uint64_t)key << 32) | q;
    gV[q] = val;
  }
  const uint32_t Ef = fit ? E : 0u;
  for (uint32_t q = Ef + li; q < CAP; q += G) gS[q] = ~0ull;  // (the gather below writes [n_own, E))
  wave_sync();
  for (uint32_t e = li; e < (fit ? tot : 0u); e += G) {  // c_t * R(t), one product per entry
    uint32_t lo = 0, hi = D;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (gdex[mid] <= e) lo = mid; else hi = mid;
    }
    const uint64_t src = gdof[lo] + (e - gdex[lo]);
    const uint32_t q = n_own + e;
    gS[q] = ((uint64_t)A.pk[src] << 32) | q;
    gV[q] = fmul(F, gdmu[lo], A.pv[src]);
  }
  uint32_t np2 = 1;  // wave-uniform: the largest group's power of two
  while (np2 < Ef) np2 <<= 1;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) np2 = max(np2, (uint32_t)__shfl_xor(np2, d));
  wave_sync();
  for (uint32_t k = 2; k <= np2; k <<= 1) {  // bitonic sort of (key, position), every group at once
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t t = li; t < np2 / 2; t += G) {
        const uint32_t i = (t / j) * 2 * j + (t % j), pr = i + j;
        const uint64_t a = gS[i], c = gS[pr];
        if ((a > c) == ((i & k) == 0)) { gS[i] = c; gS[pr] = a; }
      }
      wave_sync();
    }
  }
  uint64_t o = 0;
  if (fit && li == 0) o = pool_alloc(A, al, Ef ? Ef : 1);
  o = __shfl(o, g0);
  oom = fit && o == RS_NONE;
  const bool go = fit && !oom;
  uint32_t run = 0;
  for (uint32_t cb = 0; cb < (go ? Ef : 0u); cb += G) {  // one output entry per distinct key, values summed
    const uint32_t p = cb + li;
    const uint32_t k0 = p < Ef ? (uint32_t)(gS[p] >> 32) : 0u;
    const bool head = p < Ef && (p == 0 || (uint32_t)(gS[p - 1] >> 32) != k0);
    const uint64_t hm = __ballot(head) & gmask;
    if (head) {
      Fe v = gV[(uint32_t)gS[p]];
      for (uint32_t q = p + 1; q < Ef && (uint32_t)(gS[q] >> 32) == k0; ++q) v = fadd(F, v, gV[(uint32_t)gS[q]]);
      const uint64_t w = o + run + (uint32_t)__popcll(hm & ltg);
      A.pk[w] = k0;
      A.pv[w] = v;
    }
    run += (uint32_t)__popcll(hm);
  }
  if (go && li == 0) {
    A.h_off[sl] = o;
    A.h_len[sl] = run;
    by += 36ull * (len + tot + run);
  }
  wave_sync();
  return __ballot(has && !fit && li == 0);
}

// the per-wave composition buffers of k_big_finish / k_compose_level, seen as d_compose_merge scratch
__device__ __forceinline__ MergeScratch merge_scratch_small(uint64_t *S, Fe *V, uint32_t *dex, uint64_t *dof, Fe *dmu) {
  MergeScratch M;
  M.K = (uint32_t *)V;                     // 256 Fe = 2,048 keys
  M.OI = (uint16_t *)S;                    // 512 own entries (1 KB)
  M.HB = S + 128;                          // 32 words
  M.HP = (uint32_t *)(S + 160);            // 33 prefixes
  M.RS = dex;                              // 64 run starts
  M.DOF = dof;
  M.DMU = dmu;
  return M;
}
constexpr uint32_t kMergeK = 2048, kMergeO = 512, kMergeD = 62;
// one composition by one wave: the k-way merge, else the bitonic sort; 1 = neither fits (the caller
// falls back), 2 = pool exhausted
// (a right-hand side of <= 64 entries composing to <= 256 sorts -- with compose_sort = 0 only when it
// has more than four dependencies; the lists the sort cannot hold merge)
__device__ inline int d_compose_wave_any(const ElimArgs &A, Alloc &al, uint64_t sl, uint64_t *S, Fe *V, uint32_t *dex,
                                         uint64_t *dof, Fe *dmu, unsigned long long &by) {
  if (A.h_len[sl] <= 64) {
    const int rc = d_compose_wave(A, al, sl, S, V, dex, dof, dmu, by, !A.compose_sort);
    if (rc != 1 && rc != 3) return rc;
    wave_sync();
  }
  return d_compose_merge<kMergeK, kMergeO, kMergeD>(A, al, sl, merge_scratch_small(S, V, dex, dof, dmu), by);
}

// d_compose_wave for right-hand sides of up to LCAP entries composing to up to ECAP entries: the
// RHS is read 64 entries at a time (running counts for the own entries and the dependencies), the
// rest is the same gather / bitonic sort / sum.  A single wave with a large LDS budget: the long
// compositions of the largest clusters, which d_compose_wave sends back.
template <uint32_t ECAP, uint32_t LCAP>
__device__ inline int d_compose_wave_big(const ElimArgs &A, Alloc &al, uint64_t sl, uint64_t *S, Fe *V,
                                         uint32_t *dex, uint64_t *dof, Fe *dmu, unsigned long long &by) {
  const FieldP &F = A.F;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t off = A.h_off[sl];
  const uint32_t len = A.h_len[sl];
  if (len > LCAP) return 1;
  const uint64_t lt = lane ? ((1ull << lane) - 1ull) : 0ull;
  uint32_t n_own = 0, D = 0, tot = 0;  // wave-uniform running counts
  for (uint32_t c0 = 0; c0 < len; c0 += 64) {
    const uint32_t i = c0 + lane;
    uint32_t key = 0, dl = 0;
    Fe val = fe_zero();
    int32_t hs = -1;
    uint64_t doff = 0;
    if (i < len) {
      key = A.pk[off + i];
      val = A.pv[off + i];
      hs = A.holder_idx[key];
      if (hs >= 0) { dl = A.h_len[hs]; doff = A.h_off[hs]; }
    }
    const uint64_t dm = __ballot(hs >= 0), om = __ballot(i < len && hs < 0);
    uint32_t x = dl;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      uint32_t y = __shfl_up(x, d);
      if ((int)lane >= d) x += y;
    }
    const uint32_t ctot = __shfl(x, 63);
    if (n_own + (uint32_t)__popcll(om) + tot + ctot > ECAP) return 1;
    if (hs >= 0) {
      const uint32_t r = D + (uint32_t)__popcll(dm & lt);
      dex[r] = tot + x - dl;
      dof[r] = doff;
      dmu[r] = val;
    }
    if (i < len && hs < 0) {
      const uint32_t q = n_own + (uint32_t)__popcll(om & lt);
      S[q] = ((uint64_t)key << 32) | q;
      V[q] = val;
    }
    n_own += (uint32_t)__popcll(om);
    D += (uint32_t)__popcll(dm);
    tot += ctot;
  }
  const uint32_t E = n_own + tot;
  wave_sync();
  for (uint32_t e = lane; e < tot; e += 64) {  // c_t * R(t), one product per entry
    uint32_t lo = 0, hi = D;
    while (hi - lo > 1) {
      uint32_t mid = (lo + hi) >> 1;
      if (dex[mid] <= e) lo = mid; else hi = mid;
    }
    const uint64_t src = dof[lo] + (e - dex[lo]);
    const uint32_t q = n_own + e;
    S[q] = ((uint64_t)A.pk[src] << 32) | q;
    V[q] = fmul(F, dmu[lo], A.pv[src]);
  }
  uint32_t np2 = 1;
  while (np2 < E) np2 <<= 1;
  for (uint32_t q = E + lane; q < np2; q += 64) S[q] = ~0ull;
  wave_sync();
  for (uint32_t k = 2; k <= np2; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t t = lane; t < np2 / 2; t += 64) {
        const uint32_t i = (t / j) * 2 * j + (t % j), pr = i + j;
        const uint64_t a = S[i], c = S[pr];
        if ((a > c) == ((i & k) == 0)) { S[i] = c; S[pr] = a; }
      }
      wave_sync();
    }
  }
  uint64_t o = 0;
  if (lane == 0) o = pool_alloc(A, al, E ? E : 1);
  o = __shfl(o, 0);
  if (o == RS_NONE) return 2;
  uint32_t run = 0;
  for (uint32_t cb = 0; cb < E; cb += 64) {
    const uint32_t p = cb + lane;
    const uint32_t k0 = p < E ? (uint32_t)(S[p] >> 32) : 0u;
    const bool head = p < E && (p == 0 || (uint32_t)(S[p - 1] >> 32) != k0);
    const uint64_t hm = __ballot(head);
    if (head) {
      Fe v = V[(uint32_t)S[p]];
      for (uint32_t q = p + 1; q < E && (uint32_t)(S[q] >> 32) == k0; ++q) v = fadd(F, v, V[(uint32_t)S[q]]);
      const uint64_t w = o + run + (uint32_t)__popcll(hm & lt);
      A.pk[w] = k0;
      A.pv[w] = v;
    }
    run += (uint32_t)__popcll(hm);
  }
  if (lane == 0) {
    A.h_off[sl] = o;
    A.h_len[sl] = run;
    by += 36ull * (len + tot + run);
  }
  return 0;
}

// k_big_finish's per-cluster work, by a team of NT threads (a workgroup, or one wave: NT = 64):
// team-scoped barriers and scans, the team's scalars in `T`, one composition buffer set per wave.
struct FinTeam {
  uint32_t ok, nf, part[16];
  uint64_t scr;
  unsigned long long hsum, hmax;
};
template <uint32_t NT>
__device__ __forceinline__ void team_sync() {
  if constexpr (NT == 64) wave_sync();
  else __syncthreads();
}
// exclusive scan of a[0..n) in place by the team; returns the total
template <uint32_t NT>
__device__ inline uint32_t team_excl_scan(uint32_t *a, uint32_t n, FinTeam &T, uint32_t tid) {
  const uint32_t lane = tid & 63, w = tid >> 6;
  const uint32_t per = (n + NT - 1) / NT, lo = min(n, tid * per), hi = min(n, lo + per);
  uint32_t sum = 0;
  for (uint32_t i = lo; i < hi; ++i) sum += a[i];
  uint32_t x = sum;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d);
    if ((int)lane >= d) x += y;
  }
  if (lane == 63) T.part[w] = x;
  team_sync<NT>();
  uint32_t base = 0, total = 0;
  for (uint32_t q = 0; q < NT / 64; ++q) { if (q < w) base += T.part[q]; total += T.part[q]; }
  uint32_t acc = base + x - sum;
  for (uint32_t i = lo; i < hi; ++i) { const uint32_t t = a[i]; a[i] = acc; acc += t; }
  team_sync<NT>();
  return total;
}
struct FinBufs {  // the composition buffers of wave 0 of the workgroup; wave w's are w strides on
  uint64_t *S;    // kComposeCap per wave
  Fe *V;          // kComposeCap
  uint32_t *dex;  // 64
  uint64_t *dof;  // 64
  Fe *dmu;        // 64
};
template <uint32_t NT>
__device__ inline void d_finish_cluster(const ElimArgs &A, Alloc &al, uint64_t ci, uint64_t c, uint32_t tid, FinTeam &T,
                                        const FinBufs &bufs, uint32_t wave0, unsigned long long &by_el,
                                        unsigned long long &by_fin) {
  const FieldP &F = A.F;
  constexpr uint32_t nt = NT;
  const uint64_t b = A.cl_off[c], e = A.cl_off[c + 1];
  const uint32_t n = (uint32_t)(e - b);
  const uint32_t m = A.n_sub[c];
  unsigned long long t_2 = wall_clock64();
  unsigned long long by = 0;  // algorithmic bytes of this lane
  if (tid == 0) T.ok = 1;
  // ---- normalize_substitutions (:414-437): the inverses come from k_batch_inv (split clusters:
  // k_normalize did it over the whole GPU)
  for (uint32_t i = tid; i < (A.split ? 0u : m); i += nt) {
    const Fe inv_i = A.ftmp[b + i];
    Fe *vv = A.pv + A.h_off[b + i];
    for (uint32_t t = 0; t < A.h_len[b + i]; ++t) vv[t] = fmul(F, vv[t], inv_i);
    by += 64ull * (A.h_len[b + i] + 1);
  }
  team_sync<NT>();
  unsigned long long t_3 = wall_clock64();
  // ---- composition over the dependency DAG in Kahn order: a substitution is composed once every
  // deleted key of its right-hand side is final (the result does not depend on the order).
  // scratch (u32): deg[m], dcnt[m+1], dfill[m], frontier[2][m], dependents[sum deg]
  if (tid == 0) {
    T.scr = pool_alloc_global(A, 6ull * m + 8);
    if (T.scr == RS_NONE) T.ok = 0;
    if (A.split) A.cf_done[ci] = 0;
  }
  team_sync<NT>();
  uint32_t levels = 0;
  if (A.split && !(T.ok && m)) {  // nothing to compose: k_big_emit still finishes the cluster
    if (tid == 0 && !T.ok) atomicOr(A.err, 8);
    by_fin += by;
    team_sync<NT>();
    return;
  }
  if (T.ok && m) {
    uint32_t *deg = A.pk + T.scr, *dcnt = deg + m, *dfill = dcnt + m + 1, *fr0 = dfill + m, *fr1 = fr0 + m;
    for (uint32_t i = tid; i < m; i += nt) { deg[i] = 0; dcnt[i] = 0; dfill[i] = 0; }
    if (tid == 0) { dcnt[m] = 0; T.nf = 0; }
    team_sync<NT>();
    for (uint32_t i = tid; i < m; i += nt) {
      const uint32_t *kk = A.pk + A.h_off[b + i];
      uint32_t len = A.h_len[b + i], d = 0;
      for (uint32_t t = 0; t < len; ++t) {
        int32_t hs = A.holder_idx[kk[t]];
        if (hs >= 0) { ++d; atomicAdd(&dcnt[hs - b], 1u); }
      }
      deg[i] = d;
      if (!d) fr0[atomicAdd(&T.nf, 1u)] = i;
    }
    team_sync<NT>();
    const uint32_t n_edges = team_excl_scan<NT>(dcnt, m + 1, T, tid);
    if (tid == 0) {
      T.scr = pool_alloc_global(A, (uint64_t)n_edges + 1);
      if (T.scr == RS_NONE) T.ok = 0;
    }
    team_sync<NT>();
    if (T.ok) {
      uint32_t *dl = A.pk + T.scr;
      for (uint32_t i = tid; i < m; i += nt) {
        if (!deg[i]) continue;
        const uint32_t *kk = A.pk + A.h_off[b + i];
        uint32_t len = A.h_len[b + i];
        for (uint32_t t = 0; t < len; ++t) {
          int32_t hs = A.holder_idx[kk[t]];
          if (hs >= 0) { uint32_t q = (uint32_t)(hs - b); dl[dcnt[q] + atomicAdd(&dfill[q], 1u)] = i; }
        }
      }
      team_sync<NT>();
      if (A.split) {  // hand the DAG and the first frontier to k_compose_level
        const uint32_t nf0 = T.nf;
        if (tid == 0) {
          A.cf_deg[ci] = (uint64_t)(deg - A.pk);
          A.cf_dl[ci] = T.scr;
          A.cf_done[ci] = nf0;
          T.scr = atomicAdd(A.cf_n, (unsigned long long)nf0);
        }
        team_sync<NT>();
        for (uint32_t f = tid; f < nf0; f += nt) A.cf_items[T.scr + f] = ((uint64_t)ci << 32) | fr0[f];
        by_fin += by;
        team_sync<NT>();
        return;  // team-uniform: k_big_emit finishes the cluster
      }
      uint32_t nf = T.nf, done = nf;
      uint32_t *cur = fr0, *nxt = fr1;
#ifdef RS_FINCLK
      unsigned long long fc[10] = {wall_clock64() - t_3, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#endif
      while (nf && T.ok) {
#ifdef RS_FINCLK
        unsigned long long tl0 = wall_clock64();
#endif
        team_sync<NT>();
        if (tid == 0) T.nf = 0;
        team_sync<NT>();
        for (uint32_t f = tid; f < nf; f += nt) {
          uint32_t q = cur[f];
          for (uint32_t t = dcnt[q]; t < dcnt[q + 1]; ++t) {
            uint32_t d = dl[t];
            if (atomicSub(&deg[d], 1u) == 1u) nxt[atomicAdd(&T.nf, 1u)] = d;
          }
        }
        team_sync<NT>();
        nf = T.nf;
#ifdef RS_FINCLK
        fc[1] += wall_clock64() - tl0;
#endif
        {  // one wave per substitution of the frontier
          const uint32_t wv_ = tid >> 6, nw = nt >> 6;
          const uint32_t bw = wave0 + wv_;  // this wave's buffers
          uint64_t *bS = bufs.S + bw * kComposeCap, *bdof = bufs.dof + bw * 64;
          Fe *bV = bufs.V + bw * kComposeCap, *bdmu = bufs.dmu + bw * 64;
          uint32_t *bdex = bufs.dex + bw * 64;
          // kFinG-lane groups take kFinPer substitutions at once; the ones too long for a group
          // follow one by one on the whole wave
          for (uint32_t f0 = wv_ * kFinPer; f0 < nf; f0 += nw * kFinPer) {
            const uint32_t f = f0 + (tid & 63) / kFinG;
            const uint64_t sl = f < nf ? b + nxt[f] : ~0ull;
            bool oom = false;
#ifdef RS_FINCLK
            const unsigned long long tc0 = wall_clock64();
#endif
            uint64_t fbk = d_compose_groups<kFinG>(A, al, sl, bS, bV, bdex, bdof, bdmu, by, oom);
#ifdef RS_FINCLK
            fc[2] += wall_clock64() - tc0;
            fc[3] += min(nf - f0, kFinPer);
            fc[9] += __popcll(fbk);
#endif
            if (__ballot(oom) && (tid & 63) == 0) T.ok = 0;
            while (fbk) {
              const uint32_t l = (uint32_t)__ffsll((unsigned long long)fbk) - 1;
              fbk &= fbk - 1;
              const uint64_t sl2 = __shfl(sl, l);
#ifdef RS_FINCLK
              const unsigned long long tc1 = wall_clock64();
              fc[7] += A.h_len[sl2];
#endif
              const int rc = d_compose_wave_any(A, al, sl2, bS, bV, bdex, bdof, bdmu, by);
#ifdef RS_FINCLK
              fc[4] += wall_clock64() - tc1;
              fc[5]++;
              if (rc == 1) fc[6]++;
#endif
              if (rc == 2) { if ((tid & 63) == 0) T.ok = 0; continue; }
              if (rc == 1 && (tid & 63) == 0 && !d_compose_serial(A, al, sl2, by)) T.ok = 0;
              wave_sync();
            }
          }
        }
        done += nf;
        ++levels;
        uint32_t *t = cur; cur = nxt; nxt = t;
        team_sync<NT>();  // T.ok is read by every lane in the loop condition
      }
      team_sync<NT>();
#ifdef RS_FINCLK
      if (A.fclk && (tid & 63) == 0)
        for (int j = 0; j < 10; ++j) atomicAdd(&A.fclk[(NT == 64 ? 0 : 16) + j], fc[j]);
      if (A.fclk && tid == 0) atomicAdd(&A.fclk[NT == 64 ? 10 : 26], (unsigned long long)levels);
#endif
      if (T.ok && done != m) { if (tid == 0) { T.ok = 0; atomicOr(A.err, 32); } }
    }
  }
  team_sync<NT>();
  // ---- emit, reset the dense scratch
  for (uint32_t i = tid; i < m; i += nt) {
    uint32_t s = A.h_sig[b + i];
    A.holder_idx[s] = -1;
    A.del[s] = 0;
    A.sub_of[s] = (int32_t)(b + i);
    A.deleted[s] = 1;
  }
  const uint32_t *touch = A.pk + A.big_touch_off[ci];
  for (uint32_t t = tid; t < A.big_touch_n[ci]; t += nt) A.occ[touch[t]] = -1;
  uint64_t rows_e = 0, subs_e = 0;
  uint32_t hmax = 0;
  for (uint32_t pos = tid; pos < n; pos += nt) rows_e += A.rows.len[A.perm[b + pos]];
  for (uint32_t i = tid; i < m; i += nt) { subs_e += A.h_len[b + i]; hmax = max(hmax, A.h_len[b + i]); }
  by_el += 36ull * (rows_e + 3 * subs_e) + 8ull * (tid == 0 ? n : 0);
  by_fin += by;
  if (A.prof) {
    if (tid == 0) { T.hsum = 0; T.hmax = 0; }
    team_sync<NT>();
    atomicAdd(&T.hsum, (unsigned long long)subs_e);
    atomicMax(&T.hmax, (unsigned long long)hmax);
    team_sync<NT>();
  }
  if (tid == 0) {
    if (!T.ok) atomicOr(A.err, 8);
    if (A.prof) {
      unsigned long long *P = A.prof + kProfWords * ci;
      P[1] = m; P[6] = t_3 - t_2; P[7] = wall_clock64() - t_3; P[20] = levels;
    }
  }
  team_sync<NT>();
}

// normalize + compose + emit of every listed cluster.  Clusters of at least `wave_below` rows (a prefix
// of the size-ordered list) take a whole workgroup each; the rest one wave each -- most of them compose
// chains (one substitution per Kahn level), where the level latency, not the lanes, is the cost, so
// NW clusters of a workgroup advance at once.  wave_below = 0: every cluster by the workgroup.
template <int NW>  // waves per workgroup
__global__ __launch_bounds__(64 * NW, 3) void k_big_finish(ElimArgs A, const uint32_t *ids, uint64_t n_ids,
                                                        uint32_t wave_below = 0) {
  static_assert(NW <= 16, "FinTeam.part");
  __shared__ FinTeam s_team[NW];
  __shared__ uint64_t cw_S[NW][kComposeCap];  // per-wave composition buffers
  __shared__ Fe cw_V[NW][kComposeCap];
  __shared__ uint32_t cw_dex[NW][64];
  __shared__ uint64_t cw_dof[NW][64];
  __shared__ Fe cw_dmu[NW][64];
  const uint32_t tid = threadIdx.x, wv = tid >> 6;
  const FinBufs bufs{cw_S[0], cw_V[0], cw_dex[0], cw_dof[0], cw_dmu[0]};
  Alloc al;
  al.chunk = 128;
  unsigned long long by_el = 0, by_fin = 0;  // this lane's algorithmic bytes (one atomic per wave at the end)
  // the list is ordered largest first: the workgroup part is the prefix of clusters >= wave_below rows
  uint64_t split = n_ids;
  if (wave_below) {
    uint64_t lo = 0, hi = n_ids;
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1, c = ids[mid];
      if (A.cl_off[c + 1] - A.cl_off[c] >= wave_below) lo = mid + 1; else hi = mid;
    }
    split = lo;
  }
  for (uint64_t ci = blockIdx.x; ci < split; ci += gridDim.x)
    d_finish_cluster<64 * NW>(A, al, ci, ids[ci], tid, s_team[0], bufs, 0, by_el, by_fin);
  for (uint64_t ci = split + (uint64_t)blockIdx.x * NW + wv; ci < n_ids; ci += (uint64_t)gridDim.x * NW)
    d_finish_cluster<64>(A, al, ci, ids[ci], tid & 63, s_team[wv], bufs, wv, by_el, by_fin);
  wave_atomic_add(A.bytes_fin, by_el + by_fin);  // the emit's reads count with the finish (A.bytes: k_eliminate)
}

// One Kahn level of the split composition, over every head cluster at once and the whole GPU: each
// wave takes a frontier substitution, composes it (its dependencies were final one launch ago;
// level 0 holds the substitutions without deleted keys, which need no composition), then releases
// its dependents -- the ones whose last dependency this was form the next frontier.
template <int NW>
__global__ __launch_bounds__(64 * NW) void k_compose_level(ElimArgs A, const uint32_t *ids, const uint64_t *cur,
                                                          const unsigned long long *n_cur, uint64_t *nxt,
                                                          unsigned long long *n_nxt, uint32_t level,
                                                          unsigned long long *zero_cnt, unsigned long long *zero_big) {
  __shared__ uint64_t cw_S[NW][kComposeCap];
  __shared__ Fe cw_V[NW][kComposeCap];
  __shared__ uint32_t cw_dex[NW][64];
  __shared__ uint64_t cw_dof[NW][64];
  __shared__ Fe cw_dmu[NW][64];
  const uint32_t wv_ = threadIdx.x >> 6, lane = threadIdx.x & 63;
  Alloc al;
  al.chunk = 128;
  unsigned long long by = 0;
  const uint64_t n = *n_cur, total = (uint64_t)gridDim.x * NW;
  if (blockIdx.x == 0 && threadIdx.x == 0) {  // the counters the next level starts from (see the host loop)
    *zero_cnt = 0;
    *zero_big = 0;
  }
  // each wave takes kFinPer frontier substitutions at once, one per kFinG-lane group (d_compose_groups);
  // the ones too long for a group follow on the whole wave, and the ones too long for its buffers go to
  // k_compose_big, which releases their dependents itself
  const uint32_t li = lane % kFinG;
  for (uint64_t f0 = ((uint64_t)blockIdx.x * NW + wv_) * kFinPer; f0 < n; f0 += total * kFinPer) {
    const uint64_t f = f0 + lane / kFinG;
    const bool valid = f < n;
    const uint64_t item = valid ? cur[f] : 0ull;
    const uint32_t ci = (uint32_t)(item >> 32), q = (uint32_t)item;
    const uint32_t c = valid ? ids[ci] : 0u;
    const uint64_t b = valid ? A.cl_off[c] : 0ull;
    const uint32_t m = valid ? A.n_sub[c] : 0u;
    uint64_t bigm = 0;  // groups whose substitution went to k_compose_big
    if (level > 0) {
      bool oom = false;
      const uint64_t sl = valid ? b + q : ~0ull;
      uint64_t fbk = d_compose_groups<kFinG>(A, al, sl, cw_S[wv_], cw_V[wv_], cw_dex[wv_], cw_dof[wv_], cw_dmu[wv_], by, oom);
      if (oom && li == 0) atomicOr(A.err, 8);
      while (fbk) {
        const uint32_t l = (uint32_t)__ffsll((unsigned long long)fbk) - 1;
        fbk &= fbk - 1;
        const uint64_t sl2 = __shfl(sl, l);
        const int rc = d_compose_wave_any(A, al, sl2, cw_S[wv_], cw_V[wv_], cw_dex[wv_], cw_dof[wv_], cw_dmu[wv_], by);
        if (rc == 2 && lane == 0) atomicOr(A.err, 8);
        if (rc == 1) {  // too long for this wave's LDS
          const uint64_t it2 = __shfl(item, l);
          if (lane == 0) A.cf_big[atomicAdd(A.cf_nbig, 1ull)] = it2;
          bigm |= 1ull << (l / kFinG);
        }
        wave_sync();
      }
    }
    if (!valid || ((bigm >> (lane / kFinG)) & 1)) continue;
    uint32_t *deg = A.pk + A.cf_deg[ci], *dcnt = deg + m;
    const uint32_t *dl = A.pk + A.cf_dl[ci];
    for (uint32_t t = dcnt[q] + li; t < dcnt[q + 1]; t += kFinG) {
      const uint32_t d = dl[t];
      if (atomicSub(&deg[d], 1u) == 1u) {
        nxt[atomicAdd(n_nxt, 1ull)] = ((uint64_t)ci << 32) | d;
        atomicAdd(&A.cf_done[ci], 1u);
      }
    }
  }
  wave_atomic_add(A.bytes_fin, by);
}

// The level's long compositions (deferred by k_compose_level): one wave per workgroup with room for
// 2,048 composed entries; longer ones are composed lane-serially.  Then their dependents are
// released like k_compose_level's.
__global__ __launch_bounds__(64) void k_compose_big(ElimArgs A, const uint32_t *ids, uint64_t *nxt,
                                                   unsigned long long *n_nxt) {
  constexpr uint32_t ECAP = 2048, LCAP = 512;
  __shared__ uint64_t S[ECAP];
  __shared__ Fe V[ECAP];
  __shared__ uint32_t dex[LCAP];
  __shared__ uint64_t dof[LCAP];
  __shared__ Fe dmu[LCAP];
  const uint32_t lane = threadIdx.x & 63;
  Alloc al;
  al.chunk = 256;
  unsigned long long by = 0;
  const uint64_t n = *A.cf_nbig;
  for (uint64_t f = blockIdx.x; f < n; f += gridDim.x) {
    const uint64_t item = A.cf_big[f];
    const uint32_t ci = (uint32_t)(item >> 32), q = (uint32_t)item;
    const uint32_t c = ids[ci];
    const uint64_t b = A.cl_off[c];
    const uint32_t m = A.n_sub[c];
    MergeScratch ms;
    ms.K = (uint32_t *)V;                  // 16,384 keys
    ms.OI = (uint16_t *)S;                 // 4,096 own entries
    ms.HB = S + 1024;                      // 256 words
    ms.HP = (uint32_t *)(S + 1280);        // 257 prefixes
    ms.RS = dex;
    ms.DOF = dof;
    ms.DMU = dmu;
    int rc = d_compose_merge<16 * ECAP / 2, 4096, LCAP - 2>(A, al, b + q, ms, by, 16, ECAP);
    if (rc == 1) {
      wave_sync();
      rc = d_compose_wave_big<ECAP, LCAP>(A, al, b + q, S, V, dex, dof, dmu, by);
    }
    if (rc == 2 && lane == 0) atomicOr(A.err, 8);
    if (rc == 1 && lane == 0 && !d_compose_serial(A, al, b + q, by)) atomicOr(A.err, 8);
    wave_sync();
    uint32_t *deg = A.pk + A.cf_deg[ci], *dcnt = deg + m;
    const uint32_t *dl = A.pk + A.cf_dl[ci];
    for (uint32_t t = dcnt[q] + lane; t < dcnt[q + 1]; t += 64) {
      const uint32_t d = dl[t];
      if (atomicSub(&deg[d], 1u) == 1u) {
        nxt[atomicAdd(n_nxt, 1ull)] = ((uint64_t)ci << 32) | d;
        atomicAdd(&A.cf_done[ci], 1u);
      }
    }
  }
  wave_atomic_add(A.bytes_fin, by);
}

// The head's composition after its first (wide) Kahn levels: one workgroup per cluster continues the
// levels in-kernel from the frontier k_compose_level left (its items for this cluster gathered from
// `cur`), one wave per substitution, a workgroup barrier between levels -- the narrow deep levels
// cost a barrier each instead of a launch.  Compositions too long for a wave's buffers fall back to
// the lane-serial composition.
template <int NW>
__global__ __launch_bounds__(64 * NW) void k_compose_rest(ElimArgs A, const uint32_t *ids, const uint64_t *cur,
                                                         const unsigned long long *n_cur, uint64_t n_ids) {
  __shared__ uint64_t cw_S[NW][kComposeCap];
  __shared__ Fe cw_V[NW][kComposeCap];
  __shared__ uint32_t cw_dex[NW][64];
  __shared__ uint64_t cw_dof[NW][64];
  __shared__ Fe cw_dmu[NW][64];
  __shared__ uint32_t s_nf;
  const uint32_t tid = threadIdx.x, nt = 64 * NW, wv = tid >> 6, lane = tid & 63;
  Alloc al;
  al.chunk = 128;
  unsigned long long by = 0;
  const uint64_t n = *n_cur;
  for (uint64_t ci = blockIdx.x; ci < n_ids; ci += gridDim.x) {
    const uint64_t c = ids[ci];
    const uint64_t b = A.cl_off[c];
    const uint32_t m = A.n_sub[c];
    if (m == 0) continue;  // block-uniform
    uint32_t *deg = A.pk + A.cf_deg[ci], *dcnt = deg + m, *fr0 = dcnt + m + 1 + m, *fr1 = fr0 + m;
    const uint32_t *dl = A.pk + A.cf_dl[ci];
    if (tid == 0) s_nf = 0;
    __syncthreads();
    for (uint64_t f = tid; f < n; f += nt) {
      const uint64_t item = cur[f];
      if ((item >> 32) == ci) fr0[atomicAdd(&s_nf, 1u)] = (uint32_t)item;
    }
    __syncthreads();
    uint32_t nf = s_nf;
    uint32_t *cu = fr0, *nx = fr1;
    while (nf) {
      for (uint32_t f0 = wv * kFinPer; f0 < nf; f0 += NW * kFinPer) {  // kFinPer at once (d_compose_groups)
        const uint32_t f = f0 + lane / kFinG;
        const uint64_t sl = f < nf ? b + cu[f] : ~0ull;
        bool oom = false;
        uint64_t fbk = d_compose_groups<kFinG>(A, al, sl, cw_S[wv], cw_V[wv], cw_dex[wv], cw_dof[wv], cw_dmu[wv], by, oom);
        if (oom && lane % kFinG == 0) atomicOr(A.err, 8);
        while (fbk) {
          const uint32_t l = (uint32_t)__ffsll((unsigned long long)fbk) - 1;
          fbk &= fbk - 1;
          const uint64_t sl2 = __shfl(sl, l);
          const int rc = d_compose_wave_any(A, al, sl2, cw_S[wv], cw_V[wv], cw_dex[wv], cw_dof[wv], cw_dmu[wv], by);
          if (rc == 2 && lane == 0) atomicOr(A.err, 8);
          if (rc == 1 && lane == 0 && !d_compose_serial(A, al, sl2, by)) atomicOr(A.err, 8);
          wave_sync();
        }
      }
      __syncthreads();
      if (tid == 0) s_nf = 0;
      __syncthreads();
      for (uint32_t f = tid; f < nf; f += nt) {
        const uint32_t q = cu[f];
        for (uint32_t t = dcnt[q]; t < dcnt[q + 1]; ++t) {
          const uint32_t d = dl[t];
          if (atomicSub(&deg[d], 1u) == 1u) nx[atomicAdd(&s_nf, 1u)] = d;
        }
      }
      __syncthreads();
      nf = s_nf;
      if (tid == 0) atomicAdd(&A.cf_done[ci], nf);
      uint32_t *t = cu; cu = nx; nx = t;
      __syncthreads();
    }
  }
  wave_atomic_add(A.bytes_fin, by);
}

// The end of k_big_finish for split clusters: every substitution composed?  Emit, reset the dense
// scratch, count the algorithmic bytes.
template <int NW>
__global__ __launch_bounds__(64 * NW) void k_big_emit(ElimArgs A, const uint32_t *ids, uint64_t n_ids) {
  const uint32_t tid = threadIdx.x, nt = blockDim.x;
  unsigned long long by_el = 0;
  for (uint64_t ci = blockIdx.x; ci < n_ids; ci += gridDim.x) {
    const uint64_t c = ids[ci];
    const uint64_t b = A.cl_off[c], e = A.cl_off[c + 1];
    const uint32_t n = (uint32_t)(e - b);
    const uint32_t m = A.n_sub[c];
    if (tid == 0 && m && A.cf_done[ci] != m) atomicOr(A.err, 32);
    for (uint32_t i = tid; i < m; i += nt) {
      uint32_t s = A.h_sig[b + i];
      A.holder_idx[s] = -1;
      A.del[s] = 0;
      A.sub_of[s] = (int32_t)(b + i);
      A.deleted[s] = 1;
    }
    const uint32_t *touch = A.pk + A.big_touch_off[ci];
    for (uint32_t t = tid; t < A.big_touch_n[ci]; t += nt) A.occ[touch[t]] = -1;
    uint64_t rows_e = 0, subs_e = 0;
    for (uint32_t pos = tid; pos < n; pos += nt) rows_e += A.rows.len[A.perm[b + pos]];
    for (uint32_t i = tid; i < m; i += nt) subs_e += A.h_len[b + i];
    by_el += 36ull * (rows_e + 3 * subs_e) + 8ull * (tid == 0 ? n : 0);
    if (tid == 0 && A.prof) A.prof[kProfWords * ci + 1] = m;
  }
  wave_atomic_add(A.bytes_fin, by_el);
}

// ---------------------------------------------------------------- substitution frames
// obtain_and_simplify_non_linear (non_linear_utils.rs:6-31): frames [eq, const, linear], then fix.
struct FrameArgs {
  FieldP F;
  const int32_t *eq_rep;   // frame 1: signal -> representative (Signal substitution)
  const uint8_t *ce_has;   // frame 2: signal -> constant
  const Fe *ce_val;
  const int32_t *sub_of;   // frame 3: signal -> slot of its RHS in the pool
  const uint64_t *h_off;
  const uint32_t *h_len;
  const uint32_t *pk;
  const Fe *pv;
};

__device__ __forceinline__ uint32_t d_frame_weight(const FrameArgs &A, uint32_t k) {
  int32_t t = A.eq_rep ? A.eq_rep[k] : -1;
  uint32_t k1 = t >= 0 ? (uint32_t)t : k;
  if (A.ce_has && A.ce_has[k1]) return 1;
  int32_t s = A.sub_of[k1];
  return s >= 0 ? A.h_len[s] : 1;
}

// Frame 3 (the linear substitutions) as a merge of sorted lists: list 0 is the tail entries whose
// signal is not substituted (in place, skipping the others), lists 1..K the right-hand sides of the
// substituted ones scaled by their coefficients.  One list is consumed per step (the smallest head
// key; duplicates across lists meet consecutively and are summed on emit), zero sums are dropped --
// the result of expanding, sorting, summing and dropping zeros (fast_encoded_constraint_substitution
// + fix), in O(w * K) for rows of any length with at most K substituted entries (false otherwise:
// the caller sorts).  Output from k[0]; the tail [rb, rb + n) must lie beyond every output position.
template <int K>
__device__ inline bool d_frame3_merge(const FrameArgs &A, uint32_t *k, Fe *v, uint32_t rb, uint32_t n, uint32_t &w_out) {
  const FieldP &F = A.F;
  uint32_t si[K], hk[K], hr[K];
  uint64_t hb[K];
#pragma unroll
  for (int j = 0; j < K; ++j) { si[j] = RS_NONE; hk[j] = RS_NONE; hr[j] = 0; hb[j] = 0; }
  uint32_t ns = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const int32_t s = A.sub_of[k[rb + i]];
    if (s < 0) continue;
    if (ns == (uint32_t)K) return false;
    const uint64_t off = A.h_off[s];
    const uint32_t len = A.h_len[s];
    const uint32_t k0 = len ? A.pk[off] : RS_NONE;
#pragma unroll
    for (int j = 0; j < K; ++j)
      if ((uint32_t)j == ns) { si[j] = i; hb[j] = off; hr[j] = len; hk[j] = k0; }
    ++ns;
  }
  auto is_sub = [&](uint32_t i) -> bool {
    bool r = false;
#pragma unroll
    for (int j = 0; j < K; ++j) r |= si[j] == i;
    return r;
  };
  uint32_t c0 = 0;
  while (c0 < n && is_sub(c0)) ++c0;
  uint32_t key0 = c0 < n ? k[rb + c0] : RS_NONE;
  uint32_t w = 0, lk = RS_NONE;
  Fe lv = fe_zero();
  for (;;) {
    uint32_t mk = key0, mi = K;  // K: list 0
#pragma unroll
    for (int j = 0; j < K; ++j)
      if (hk[j] < mk) { mk = hk[j]; mi = (uint32_t)j; }
    if (mk == RS_NONE) break;
    Fe c;
    if (mi == (uint32_t)K) {
      c = v[rb + c0];
      ++c0;
      while (c0 < n && is_sub(c0)) ++c0;
      key0 = c0 < n ? k[rb + c0] : RS_NONE;
    } else {
      uint64_t b = 0;
      uint32_t rem = 0, ix = 0;
#pragma unroll
      for (int j = 0; j < K; ++j)
        if ((uint32_t)j == mi) { b = hb[j]; rem = hr[j]; ix = si[j]; }
      c = fmul(F, v[rb + ix], A.pv[b]);
      const uint32_t nk = rem > 1 ? A.pk[b + 1] : RS_NONE;
#pragma unroll
      for (int j = 0; j < K; ++j)
        if ((uint32_t)j == mi) { hk[j] = nk; hr[j] = rem - 1; hb[j] = b + 1; }
    }
    if (mk == lk) {
      lv = fadd(F, lv, c);
    } else {
      if (lk != RS_NONE && !fe_is_zero(lv)) { k[w] = lk; v[w] = lv; ++w; }
      lk = mk;
      lv = c;
    }
  }
  if (lk != RS_NONE && !fe_is_zero(lv)) { k[w] = lk; v[w] = lv; ++w; }
  w_out = w;
  return true;
}

// Expands one linear combination through the frames into [k, v).  The region holds
// 1 + sum(d_frame_weight) + n entries (n = input length): the input is staged in its last n slots.
__device__ inline uint32_t d_apply_frames(const FrameArgs &A, const uint32_t *ik, const Fe *iv, uint32_t n,
                                          uint32_t *k, Fe *v, uint32_t cap) {
  const FieldP &F = A.F;
  // place the input at the tail of the region, frames 1-2 in place there
  uint32_t base = cap - n;
  for (uint32_t i = 0; i < n; ++i) { k[base + i] = ik[i]; v[base + i] = iv[i]; }
  uint32_t *tk = k + base;
  Fe *tv = v + base;
  bool any = false;
  if (A.eq_rep)
    for (uint32_t i = 0; i < n; ++i) {
      int32_t t = A.eq_rep[tk[i]];
      if (t >= 0) { tk[i] = (uint32_t)t; any = true; }
    }
  if (any) n = d_sort_combine(F, tk, tv, n);
  if (A.ce_has) {
    any = false;
    for (uint32_t i = 0; i < n; ++i)
      if (A.ce_has[tk[i]]) { tv[i] = fmul(F, tv[i], A.ce_val[tk[i]]); tk[i] = 0; any = true; }
    if (any) n = d_sort_combine(F, tk, tv, n);
  }
  {
    uint32_t w;
    if (d_frame3_merge<8>(A, k, v, base, n, w)) return w;
  }
  // frame 3 expands (more than 8 substituted entries): write from the front, reading from the
  // (shrunk) tail copy, then sort
  uint32_t rb = cap - n;
  if (rb != base)
    for (uint32_t i = n; i-- > 0;) { k[rb + i] = tk[i]; v[rb + i] = tv[i]; }  // overlapping: copy backwards
  uint32_t w = 0;
  any = false;
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t kk = k[rb + i];
    Fe vv = v[rb + i];
    int32_t s = A.sub_of[kk];
    if (s >= 0) {
      any = true;
      const uint32_t *rk = A.pk + A.h_off[s];
      const Fe *rv = A.pv + A.h_off[s];
      uint32_t rl = A.h_len[s];
      for (uint32_t j = 0; j < rl; ++j) { k[w] = rk[j]; v[w] = fmul(F, vv, rv[j]); ++w; }
    } else {
      k[w] = kk;
      v[w] = vv;
      ++w;
    }
  }
  if (any) w = d_sort_combine(F, k, v, w);
  return d_drop_zeros(k, v, w);
}

struct NLArgs {
  FrameArgs fr;
  DRows a, b, c;       // input rows
  DRows oa, ob, oc;    // output rows (off/cap computed by the count pass)
  uint64_t *cap_a, *cap_b, *cap_c;
  unsigned long long *bytes;  // algorithmic bytes counter
  // rows processed: ids[0, n) (ids == nullptr: rows 0..n-1); cap_* are indexed by position in that list.
  // phase 1 (while the largest clusters are still being eliminated) skips the rows one of whose
  // signals (after frames 1-2) occurs in those clusters, flagging them in `late`; the caller runs
  // them once every substitution is known.
  const uint32_t *ids;
  uint64_t n;
  int phase;
  const uint8_t *hmark;  // signal -> occurs in a row of a head cluster
  uint64_t *late;
  // k_nl_fill only: the positions k_frames_wave left to it (rows too large for a wave's LDS batch)
  const uint32_t *xlist;
  const unsigned *n_xlist;
};

// Marks the signals of the head clusters' rows (signal 0 is never substituted).
__global__ void k_mark_head_keys(DRows rows, const uint32_t *perm, const uint64_t *cl_off, const uint32_t *ids,
                                 uint8_t *hmark) {
  const uint32_t c = ids[blockIdx.y];
  const uint64_t b = cl_off[c], e = cl_off[c + 1];
  for (uint64_t i = b + blockIdx.x * blockDim.x + threadIdx.x; i < e; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t r = perm[i];
    const uint64_t o = rows.off[r];
    for (uint32_t j = 0; j < rows.len[r]; ++j) {
      const uint32_t k = rows.key[o + j];
      if (k) hmark[k] = 1;
    }
  }
}

__device__ inline bool d_touches_head(const FrameArgs &F, const uint8_t *hmark, const DRows &R, uint64_t r) {
  const uint64_t o = R.off[r];
  for (uint32_t i = 0; i < R.len[r]; ++i) {
    const uint32_t k = R.key[o + i];
    const int32_t t = F.eq_rep ? F.eq_rep[k] : -1;
    const uint32_t k1 = t >= 0 ? (uint32_t)t : k;
    if (F.ce_has && F.ce_has[k1]) continue;
    if (hmark[k1]) return true;
  }
  return false;
}

__global__ void k_nl_count(NLArgs A) {
  for (uint64_t x = gtid(); x < A.n; x += gstride()) {
    const uint64_t r = A.ids ? A.ids[x] : x;
    if (A.phase == 1) {
      const bool lt = d_touches_head(A.fr, A.hmark, A.a, r) || d_touches_head(A.fr, A.hmark, A.b, r) ||
                      d_touches_head(A.fr, A.hmark, A.c, r);
      A.late[r] = lt;
      if (lt) {  // a later pass's row: no space now
        A.cap_a[x] = A.cap_b[x] = A.cap_c[x] = 0;
        continue;
      }
    }
    // expansion bound + 1, plus the staged input (d_apply_frames)
    uint64_t ca = 1 + A.a.len[r], cb = 1 + A.b.len[r], cc = 1 + A.c.len[r];
    for (uint32_t i = 0; i < A.a.len[r]; ++i) ca += d_frame_weight(A.fr, A.a.key[A.a.off[r] + i]);
    for (uint32_t i = 0; i < A.b.len[r]; ++i) cb += d_frame_weight(A.fr, A.b.key[A.b.off[r] + i]);
    for (uint32_t i = 0; i < A.c.len[r]; ++i) cc += d_frame_weight(A.fr, A.c.key[A.c.off[r] + i]);
    A.cap_a[x] = ca;
    A.cap_b[x] = cb;
    A.cap_c[x] = 2 * cc + (ca > cb ? ca : cb);  // expansion + scratch for c - a0*b
  }
}

// One lane per row: the rows k_frames_wave hands over (xlist), or every row when xlist is null.
__global__ void k_nl_fill(NLArgs A) {
  unsigned long long bytes = 0;
  const uint64_t nx = A.xlist ? *A.n_xlist : A.n;
  for (uint64_t xi = gtid(); xi < nx; xi += gstride()) {
    const uint64_t x = A.xlist ? A.xlist[xi] : xi;
    const uint64_t r = A.ids ? A.ids[x] : x;
    if (A.phase == 1 && A.late[r]) continue;
    uint64_t oa = A.oa.off[r], ob = A.ob.off[r], oc = A.oc.off[r];
    uint32_t capa = (uint32_t)A.cap_a[x], capb = (uint32_t)A.cap_b[x];
    uint32_t capc = (uint32_t)A.cap_c[x];
    uint32_t mx = capa > capb ? capa : capb;
    uint32_t cc = (capc - mx) / 2;
    uint32_t na = d_apply_frames(A.fr, A.a.key + A.a.off[r], A.a.val + A.a.off[r], A.a.len[r], A.oa.key + oa, A.oa.val + oa, capa);
    uint32_t nb = d_apply_frames(A.fr, A.b.key + A.b.off[r], A.b.val + A.b.off[r], A.b.len[r], A.ob.key + ob, A.ob.val + ob, capb);
    uint32_t nc = d_apply_frames(A.fr, A.c.key + A.c.off[r], A.c.val + A.c.off[r], A.c.len[r], A.oc.key + oc, A.oc.val + oc, cc);
    d_fix(A.fr.F, A.oa.key + oa, A.oa.val + oa, na, A.ob.key + ob, A.ob.val + ob, nb, A.oc.key + oc, A.oc.val + oc,
          nc, A.oc.key + oc + cc, A.oc.val + oc + cc);
    A.oa.len[r] = na;
    A.ob.len[r] = nb;
    A.oc.len[r] = nc;
    bytes += 36ull * (A.a.len[r] + A.b.len[r] + A.c.len[r] + na + nb + nc) + 24;
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) bytes += __shfl_xor(bytes, d);  // one atomic per wave
  if ((threadIdx.x & 63) == 0 && bytes) atomicAdd(A.bytes, bytes);
}

// ---------------------------------------------------------------- rounds >= 2 on the storage
// apply_substitution_to_map (:345-396) restated per row: the final content is
// fix(all of this round's substitutions applied) and `turn` is the rank (in the round's
// substitution order) of the first substitution after which the row is linear.
struct RoundArgs {
  FieldP F;
  DRows a, b, c;        // storage rows (updated in place into oa/ob/oc)
  DRows oa, ob, oc;
  uint64_t *cap_a, *cap_b, *cap_c;
  const int32_t *sub_of;   // signal -> slot (this round)
  const int32_t *rank_of;  // signal -> position in this round's ordered list
  const uint64_t *h_off;
  const uint32_t *h_len;
  const uint32_t *pk;
  const Fe *pv;
  int32_t *turn;           // out: rank or -1
  uint8_t *touched;        // out: row contained a substituted signal
  uint32_t *tmpk;          // per-row scratch: 2 * cap_c entries at 2 * (C offset - c_base)
  Fe *tmpv;
  uint64_t c_base;
  const uint32_t *ids;     // the rows a substitution touches (cap_c != 0), compacted
  uint64_t n_ids;
  // k_round_fill / k_round_turn: the rows k_frames_wave left (rlist), or every id when null
  const uint32_t *rlist;
  const unsigned *n_rlist;
  unsigned long long *bytes;  // algorithmic bytes: 36 per entry read (row + right-hand sides) or written
  // k_round_fill: A / B / C were already expanded into oa / ob / oc (lengths in their len arrays) by
  // k_xrow_count / k_xrow_expand / k_xrow_combine -- the rows too long for a wave's LDS batch
  int pre_expanded;
};
__global__ void k_touch_flags(const uint64_t *cap_c, uint64_t n, uint64_t *flag) {
  for (uint64_t r = gtid(); r < n; r += gstride()) flag[r] = cap_c[r] != 0;
}

__global__ void k_round_count(RoundArgs A) {
  for (uint64_t r = gtid(); r < A.a.n; r += gstride()) {
    uint64_t ca = 1 + A.a.len[r], cb = 1 + A.b.len[r], cc = 1 + A.c.len[r];  // + the staged input
    bool hit = false;
    for (uint32_t i = 0; i < A.a.len[r]; ++i) { int32_t s = A.sub_of[A.a.key[A.a.off[r] + i]]; ca += s >= 0 ? A.h_len[s] : 1; hit |= s >= 0; }
    for (uint32_t i = 0; i < A.b.len[r]; ++i) { int32_t s = A.sub_of[A.b.key[A.b.off[r] + i]]; cb += s >= 0 ? A.h_len[s] : 1; hit |= s >= 0; }
    for (uint32_t i = 0; i < A.c.len[r]; ++i) { int32_t s = A.sub_of[A.c.key[A.c.off[r] + i]]; cc += s >= 0 ? A.h_len[s] : 1; hit |= s >= 0; }
    if (!hit) ca = cb = cc = 0;
    A.cap_a[r] = ca;
    A.cap_b[r] = cb;
    A.cap_c[r] = hit ? 2 * cc + (ca > cb ? ca : cb) : 0;
  }
}

// is the (zero-free, sorted) map empty or constant-only?
__device__ __forceinline__ bool d_const_or_empty(const uint32_t *k, uint32_t n) { return n == 0 || (n == 1 && k[0] == 0); }

// The rank (in the round's substitution order) of the first substitution after which the row's
// A or B is constant or empty -- for a row whose final A or B is (the caller checked).  Replays the
// substitutions one by one on copies of A and B held in the row's A / B output regions (their final
// content is dropped anyway: fix_constraint clears A and B of such a row) with the row's scratch
// [2 * (oc - c_base), + 2 * capc) for the ranks and merges.  Writes turn[r] (-2: linear on input).
__device__ inline void d_round_turn(const RoundArgs &A, uint64_t r) {
  const FieldP &F = A.F;
  const uint64_t oa = A.oa.off[r], ob = A.ob.off[r], oc = A.oc.off[r];
  const uint32_t capc = (uint32_t)A.cap_c[r];
  // applicable ranks from A u B, ascending
  uint32_t *rk_ = A.tmpk + 2 * (oc - A.c_base);
  uint32_t nr = 0;
  for (int part = 0; part < 2; ++part) {
    const DRows &P = part ? A.b : A.a;
    for (uint32_t i = 0; i < P.len[r]; ++i) {
      int32_t q = A.rank_of[P.key[P.off[r] + i]];
      if (q >= 0) rk_[nr++] = (uint32_t)q;
    }
  }
  d_heap_sort_u32(rk_, nr);
  uint32_t na = A.a.len[r], nb = A.b.len[r];
  uint32_t *ak = A.oa.key + oa, *bk = A.ob.key + ob;
  Fe *av = A.oa.val + oa, *bv = A.ob.val + ob;
  for (uint32_t i = 0; i < na; ++i) { ak[i] = A.a.key[A.a.off[r] + i]; av[i] = A.a.val[A.a.off[r] + i]; }
  for (uint32_t i = 0; i < nb; ++i) { bk[i] = A.b.key[A.b.off[r] + i]; bv[i] = A.b.val[A.b.off[r] + i]; }
  if (d_const_or_empty(ak, na) || d_const_or_empty(bk, nb)) A.turn[r] = -2;  // already linear
  for (uint32_t q = 0; q < nr && A.turn[r] == -1; ++q) {
    if (q > 0 && rk_[q] == rk_[q - 1]) continue;
    for (int part = 0; part < 2; ++part) {
      uint32_t *pk_ = part ? bk : ak;
      Fe *pv_ = part ? bv : av;
      uint32_t &pn = part ? nb : na;
      // find the signal with this rank in the part
      uint32_t fi = RS_NONE;
      for (uint32_t i = 0; i < pn; ++i)
        if (A.rank_of[pk_[i]] == (int32_t)rk_[q]) { fi = i; break; }
      if (fi == RS_NONE) continue;
      int32_t s = A.sub_of[pk_[fi]];
      Fe val = pv_[fi];
      const uint32_t *hk = A.pk + A.h_off[s];
      const Fe *hv = A.pv + A.h_off[s];
      uint32_t hl = A.h_len[s];
      // merge (pn - 1 + hl <= the part's capacity) via the scratch after the ranks
      uint32_t *mk = A.tmpk + 2 * (oc - A.c_base) + capc;
      Fe *mv = A.tmpv + 2 * (oc - A.c_base) + capc;
      uint32_t i = 0, j = 0, w = 0;
      while (i < pn || j < hl) {
        if (i == fi) { ++i; continue; }
        if (j >= hl || (i < pn && pk_[i] < hk[j])) { mk[w] = pk_[i]; mv[w] = pv_[i]; ++i; }
        else if (i >= pn || hk[j] < pk_[i]) { mk[w] = hk[j]; mv[w] = fmul(F, val, hv[j]); ++j; }
        else { mk[w] = pk_[i]; mv[w] = fadd(F, pv_[i], fmul(F, val, hv[j])); ++i; ++j; }
        ++w;
      }
      w = d_drop_zeros(mk, mv, w);
      for (uint32_t t = 0; t < w; ++t) { pk_[t] = mk[t]; pv_[t] = mv[t]; }
      pn = w;
    }
    if (d_const_or_empty(ak, na) || d_const_or_empty(bk, nb)) A.turn[r] = (int32_t)rk_[q];
  }
}

__device__ __forceinline__ FrameArgs d_round_frames(const RoundArgs &A) {
  FrameArgs fr;
  fr.F = A.F;
  fr.eq_rep = nullptr;
  fr.ce_has = nullptr;
  fr.ce_val = nullptr;
  fr.sub_of = A.sub_of;
  fr.h_off = A.h_off;
  fr.h_len = A.h_len;
  fr.pk = A.pk;
  fr.pv = A.pv;
  return fr;
}

// One lane per touched row: the rows k_frames_wave left (rlist), or every id when rlist is null
// (turn = -1 and touched = 0 were set for every row beforehand).
__global__ void k_round_fill(RoundArgs A) {
  const FieldP &F = A.F;
  unsigned long long bytes = 0;
  const uint64_t n = A.rlist ? *A.n_rlist : A.n_ids;
  for (uint64_t i = gtid(); i < n; i += gstride()) {
    const uint64_t r = A.rlist ? A.rlist[i] : A.ids[i];
    A.touched[r] = 1;
    const FrameArgs fr = d_round_frames(A);
    uint64_t oa = A.oa.off[r], ob = A.ob.off[r], oc = A.oc.off[r];
    uint32_t capa = (uint32_t)A.cap_a[r], capb = (uint32_t)A.cap_b[r], capc = (uint32_t)A.cap_c[r];
    uint32_t mx = capa > capb ? capa : capb;
    uint32_t cc = (capc - mx) / 2;
    // A row that turns linear stays linear (fix_constraint clears A and B; later substitutions only
    // touch C), so it turns iff its final A or B -- all of the round's substitutions applied -- is
    // constant or empty.  The final A and B come first; only the rows that turn (few) replay the
    // substitutions one by one to find the rank at which they turn.
    uint32_t na, nb;
    if (A.pre_expanded) {
      na = A.oa.len[r];
      nb = A.ob.len[r];
    } else {
      na = d_apply_frames(fr, A.a.key + A.a.off[r], A.a.val + A.a.off[r], A.a.len[r], A.oa.key + oa, A.oa.val + oa, capa);
      nb = d_apply_frames(fr, A.b.key + A.b.off[r], A.b.val + A.b.off[r], A.b.len[r], A.ob.key + ob, A.ob.val + ob, capb);
    }
    if (d_const_or_empty(A.oa.key + oa, na) || d_const_or_empty(A.ob.key + ob, nb)) {
      d_round_turn(A, r);
      // the replay used the A / B regions as scratch: final A and B again
      na = d_apply_frames(fr, A.a.key + A.a.off[r], A.a.val + A.a.off[r], A.a.len[r], A.oa.key + oa, A.oa.val + oa, capa);
      nb = d_apply_frames(fr, A.b.key + A.b.off[r], A.b.val + A.b.off[r], A.b.len[r], A.ob.key + ob, A.ob.val + ob, capb);
    }
    // ---- final content: fix(all substitutions applied)
    uint32_t nc = A.pre_expanded ? A.oc.len[r]
                                       : d_apply_frames(fr, A.c.key + A.c.off[r], A.c.val + A.c.off[r], A.c.len[r], A.oc.key + oc,
                                                        A.oc.val + oc, cc);
    d_fix(F, A.oa.key + oa, A.oa.val + oa, na, A.ob.key + ob, A.ob.val + ob, nb, A.oc.key + oc, A.oc.val + oc, nc,
          A.oc.key + oc + cc, A.oc.val + oc + cc);
    A.oa.len[r] = na;
    A.ob.len[r] = nb;
    A.oc.len[r] = nc;
    // read: the row and, per entry, its right-hand side (the capacity bound minus the staging slots)
    bytes += 36ull * ((capa - 1) + (capb - 1) + (cc - 1) - A.a.len[r] - A.b.len[r] - A.c.len[r]) +
             36ull * (na + nb + nc);
  }
  wave_atomic_add(A.bytes, bytes);
}

// ---- rows too long for a wave's LDS batch (k_frames_wave lists them in rlist): their A, B and C
// through the round's substitutions as a device-wide sort instead of one lane per row.  Segment
// s = 3 * i + part (part 0 / 1 / 2 = A / B / C of rlist[i]):
//   k_xrow_count   entries after expansion (a substituted entry -> its right-hand side),
//   k_xrow_expand  (s, key) keys + coefficient x RHS values, one wave per segment,
//   one radix sort of (s, key), then
//   k_xrow_combine equal keys summed, zero sums dropped, written in key order into the row's output
//                  region -- what d_apply_frames (frame 3: sort_combine + drop_zeros) produces.
__device__ __forceinline__ const DRows &d_part(const RoundArgs &A, uint32_t p) { return p == 0 ? A.a : (p == 1 ? A.b : A.c); }
__global__ void k_xrow_count(RoundArgs A, uint64_t nseg, uint64_t *cnt) {
  for (uint64_t sg = gtid(); sg < nseg; sg += gstride()) {
    const uint64_t r = A.rlist[sg / 3];
    const DRows &P = d_part(A, (uint32_t)(sg % 3));
    uint64_t c = 0;
    for (uint32_t i = 0; i < P.len[r]; ++i) {
      const int32_t s = A.sub_of[P.key[P.off[r] + i]];
      c += s >= 0 ? A.h_len[s] : 1;
    }
    cnt[sg] = c;
  }
}
__global__ __launch_bounds__(256) void k_xrow_expand(RoundArgs A, uint64_t nseg, const uint64_t *soff, uint64_t *xk, Fe *xv,
                                                     uint32_t *xi) {
  const FieldP &F = A.F;
  const uint32_t lane = threadIdx.x & 63;
  for (uint64_t sg = gtid() >> 6; sg < nseg; sg += gstride() >> 6) {
    const uint64_t r = A.rlist[sg / 3];
    const DRows &P = d_part(A, (uint32_t)(sg % 3));
    const uint64_t ro = P.off[r];
    const uint32_t n = P.len[r];
    uint64_t base = soff[sg];
    for (uint32_t c0 = 0; c0 < n; c0 += 64) {
      const uint32_t i = c0 + lane;
      uint32_t k = 0, m = 0;
      int32_t s = -1;
      if (i < n) {
        k = P.key[ro + i];
        s = A.sub_of[k];
        m = s >= 0 ? A.h_len[s] : 1;
      }
      uint32_t x = m;  // inclusive scan of the counts over the wave
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d);
        if (lane >= (uint32_t)d) x += y;
      }
      const uint64_t o = base + x - m;
      if (i < n) {
        const Fe vv = P.val[ro + i];
        if (s < 0) {
          xk[o] = ((uint64_t)sg << 32) | k;
          xv[o] = vv;
          xi[o] = (uint32_t)(o - soff[sg]);
        } else {
          const uint64_t hb = A.h_off[s];
          for (uint32_t t = 0; t < m; ++t) {
            xk[o + t] = ((uint64_t)sg << 32) | A.pk[hb + t];
            xv[o + t] = fmul(F, vv, A.pv[hb + t]);
            xi[o + t] = (uint32_t)(o + t - soff[sg]);
          }
        }
      }
      base += __shfl(x, 63);
    }
  }
}
__global__ __launch_bounds__(256) void k_xrow_combine(RoundArgs A, uint64_t nseg, const uint64_t *soff, const uint64_t *xk,
                                                      const uint32_t *xi, const Fe *xv) {
  const FieldP &F = A.F;
  const uint32_t lane = threadIdx.x & 63;
  for (uint64_t sg = gtid() >> 6; sg < nseg; sg += gstride() >> 6) {
    const uint64_t r = A.rlist[sg / 3];
    const uint32_t p = (uint32_t)(sg % 3);
    const DRows &O = p == 0 ? A.oa : (p == 1 ? A.ob : A.oc);
    uint32_t *ok = O.key + O.off[r];
    Fe *ov = O.val + O.off[r];
    const uint64_t b = soff[sg], e = soff[sg + 1];
    uint32_t w = 0;
    for (uint64_t q0 = b; q0 < e; q0 += 64) {
      const uint64_t q = q0 + lane;
      bool keep = false;
      uint32_t key = 0;
      Fe sum = fe_zero();
      if (q < e) {
        key = (uint32_t)xk[q];
        if (q == b || (uint32_t)xk[q - 1] != key) {  // the head of a run of equal keys sums it
          sum = xv[b + xi[q]];
          for (uint64_t t = q + 1; t < e && (uint32_t)xk[t] == key; ++t) sum = fadd(F, sum, xv[b + xi[t]]);
          keep = !fe_is_zero(sum);
        }
      }
      const uint64_t km = __ballot(keep);
      if (keep) {
        const uint32_t at = w + (uint32_t)__popcll(km & ((1ull << lane) - 1ull));
        ok[at] = key;
        ov[at] = sum;
      }
      w += (uint32_t)__popcll(km);
    }
    if (lane == 0) {
      if (p == 0) A.oa.len[r] = w;
      else if (p == 1) A.ob.len[r] = w;
      else A.oc.len[r] = w;
    }
  }
}

// The turn ranks of the rows k_frames_wave listed (their final content is already written).
__global__ void k_round_turn(RoundArgs A) {
  const uint64_t n = *A.n_rlist;
  for (uint64_t i = gtid(); i < n; i += gstride()) d_round_turn(A, A.rlist[i]);
}

// ---------------------------------------------------------------- final assembly
__global__ void k_mark_keys(DRows R, uint8_t *bits) {
  for (uint64_t r = gtid(); r < R.n; r += gstride())
    for (uint32_t i = 0; i < R.len[r]; ++i) bits[R.key[R.off[r] + i]] = 1;
}
__global__ void k_mark_list(const uint32_t *sig, uint64_t n, uint8_t *bits) {
  for (uint64_t i = gtid(); i < n; i += gstride()) bits[sig[i]] = 1;
}
// rebuild_witness (:101-124): kept = !deleted && (forbidden || key of non_linear_map)
__global__ void k_kept(const uint8_t *deleted, const uint8_t *forb, const uint8_t *nlmap, uint32_t *kept, uint64_t S) {
  for (uint64_t s = gtid(); s < S; s += gstride()) kept[s] = (!deleted[s] && (forb[s] || nlmap[s])) ? 1u : 0u;
}
__global__ void k_l2w(const uint32_t *kept, const uint64_t *rank, int32_t *l2w, uint64_t S) {
  for (uint64_t s = gtid(); s < S; s += gstride()) l2w[s] = kept[s] ? (int32_t)rank[s] : -1;
}
// gathers ragged rows (selected ids) into a compact CSR with canonical values
__global__ void k_gather_rows(FieldP F, DRows R, const uint32_t *ids, uint64_t n, const uint64_t *optr,
                              uint32_t *ocol, uint64_t *oval) {
  for (uint64_t i = gtid(); i < n; i += gstride()) {
    uint32_t r = ids[i];
    uint64_t o = optr[i];
    for (uint32_t t = 0; t < R.len[r]; ++t) {
      ocol[o + t] = R.key[R.off[r] + t];
      Fe c = ffrom_mont(F, R.val[R.off[r] + t]);
      oval[4 * (o + t) + 0] = c.l[0];
      oval[4 * (o + t) + 1] = c.l[1];
      oval[4 * (o + t) + 2] = c.l[2];
      oval[4 * (o + t) + 3] = c.l[3];
    }
  }
}
__global__ void k_row_lens(DRows R, const uint32_t *ids, uint64_t n, uint64_t *lens) {
  for (uint64_t i = gtid(); i < n; i += gstride()) lens[i] = R.len[ids[i]];
}
// pool RHS / leftover copy-out (canonical) for the host bookkeeping of rounds >= 2
__global__ void k_pool_to_canon(FieldP F, const uint64_t *off, const uint32_t *len, const uint64_t *optr, uint64_t n,
                                const uint32_t *pk, const Fe *pv, uint32_t *ok, uint64_t *ov) {
  for (uint64_t i = gtid(); i < n; i += gstride()) {
    uint64_t o = optr[i];
    for (uint32_t t = 0; t < len[i]; ++t) {
      ok[o + t] = pk[off[i] + t];
      Fe c = ffrom_mont(F, pv[off[i] + t]);
      for (int q = 0; q < 4; ++q) ov[4 * (o + t) + q] = c.l[q];
    }
  }
}

// keys only (the rounds' map appends read no value): one wave per map, consecutive lanes copy
// consecutive keys
__global__ __launch_bounds__(256) void k_pool_keys(const uint64_t *off, const uint32_t *len, const uint64_t *optr, uint64_t n,
                                                   const uint32_t *pk, uint32_t *ok) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint64_t i = gtid() >> 6; i < n; i += gstride() >> 6) {
    const uint64_t o = optr[i], b = off[i];
    for (uint32_t t = lane; t < len[i]; t += 64) ok[o + t] = pk[b + t];
  }
}

// ---------------------------------------------------------------- substitution log
// eq_simplification's substitutions (constraint_simplification.rs:198-251) in log order: every
// renamed signal s (eq_rep[s] = its representative) keyed by (cluster of more than one row,
// cluster index = max row, s) -- size-1 clusters are logged first (:219-223), the others by
// cluster id (:240-244), each cluster's removable signals ascending (:188-192, canonical).
__global__ void k_eq_log_keys(const int32_t *eq_rep, uint32_t *uf, const uint32_t *cnt, const int32_t *maxrow, uint64_t S,
                              uint64_t *key, uint32_t *rep, unsigned long long *n) {
  for (uint64_t s = gtid(); s < S; s += gstride()) {
    const int32_t r = eq_rep[s];
    if (r < 0) continue;
    const uint32_t root = uf_find(uf, (uint32_t)s);
    const unsigned long long i = atomicAdd(n, 1ull);
    key[i] = ((uint64_t)(cnt[root] > 1) << 63) | ((uint64_t)(uint32_t)maxrow[root] << 32) | s;
    rep[i] = (uint32_t)r;
  }
}
// constant_eq_simplification's substitutions (:253-273) per cons_eq row, in row order: the row's
// largest signal s (take_cloned_signals_ordered().pop()) := clear_signal (algebra.rs:1108-1124)
// = c / (-k) with zeros removed; sig = RS_NONE when s is forbidden (the row stays a constraint).
__global__ void k_const_log(FieldP F, DRows R, const uint8_t *forb, uint32_t *sig, uint64_t *val) {
  for (uint64_t r = gtid(); r < R.n; r += gstride()) {
    const uint32_t *k = R.key + R.off[r];
    const Fe *v = R.val + R.off[r];
    const uint32_t n = R.len[r];
    const uint32_t s = n ? k[n - 1] : 0;
    sig[r] = (n == 0 || forb[s]) ? RS_NONE : s;
    Fe x = fe_zero();
    if (n && !forb[s] && n == 2 && k[0] == 0) x = ffrom_mont(F, fmul(F, v[0], finv(F, fneg(F, v[n - 1]))));
    for (int q = 0; q < 4; ++q) val[4 * r + q] = x.l[q];
  }
}

}  // namespace rs
