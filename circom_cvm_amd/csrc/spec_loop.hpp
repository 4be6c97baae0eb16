// spec_loop.hpp -- the ordered loop of process_3 / process_4 for the largest clusters, run by NW waves
// of one workgroup that reduce the next rows speculatively and commit them in the reference's order.
//
// The loop (substitution_process_3/4 -> treat_constraint_3/4, take_signal_3/4,
// simplification_utils.rs:143-185, 259-349, 368-411) pops the cluster's rows from the back.  A row
// is reduced against the substitutions (holders) of the rows popped before it -- p4: eliminate the
// first deleted key, ascending, until none is left; p3: eliminate the largest takeable key while it
// is deleted -- and then becomes a new holder for a fresh pivot (p4: fewest occurrences, ties -> the
// largest id; p3: the largest takeable key) or a leftover.  Each merge is `work = c2*work - c*R`
// (the holder's pivot coefficient against the work's), zeros dropped.
//
// Rows depend on each other only through the holders they merge with and the pivots that later rows
// see as deleted.  On the 10M metric circuit 46 % of the largest cluster's rows depend on no earlier
// loop row at all, and fewer than 5 % on one of the 8 rows before them (tools/elim_trace.cpp).  So:
//   dispatch   rows in pop order to the waves (an LDS counter); a wave reduces its row against the
//              state as it is (the LDS table below) and records every key its work lists held;
//   commit     in pop order (an LDS turn counter): the wave whose turn it is checks the pivots
//              committed since it started (an LDS ring) against its recorded keys -- one of them among
//              them means a status it read has changed, and the row is reduced again now, when the
//              state is final for it.  Otherwise its reduction IS the reference's: every choice of the
//              merge sequence depended only on statuses that are still the same, and holders never
//              change.  Then, in order: remove_constraint (the occurrence counts of the original row's
//              keys), the pivot on the fresh counts, the holder (or leftover) written, the pivot's
//              state published, the turn passed on.
// Waves validate the commits that land while they wait, so at its turn a wave usually checks one.
// The speculative part keeps the work list in registers (one entry per lane, <= 64); a row or merge
// beyond that finishes at its turn on lane 0 (d_treat_scalar over the global state, kept current).
//
// LDS: the cluster's signal table (open addressing over the touched signals; state = bit 31 deleted +
// the holder's header offset, else the occurrence count), per wave the merge's
// key lists and the recorded keys, the commit ring.  A cluster whose signals do not fit runs
// k_big_main's loop on wave 0.
#pragma once
#include "kernels.hpp"

namespace rs {

constexpr uint32_t kSpecTab = 16384;     // LDS hash slots (64 KB keys + 64 KB states)
constexpr uint32_t kSpecTabMax = 11800;  // signals per cluster at most (load factor 0.72)
constexpr uint32_t kSpecK = 192;         // per wave: keys its reduction's work lists held
constexpr uint32_t kSpecRing = 64;       // committed pivots (by row, modulo)

__device__ __forceinline__ uint32_t sp_slot(uint32_t s) { return (s * 0x9E3779B1u) >> 18; }  // 14 bits
__device__ __forceinline__ uint32_t sp_find(const uint32_t *tk, uint32_t s) {
  if (s == 0) return kTabEmpty;  // the constant: always forbidden
  uint32_t i = sp_slot(s);
  for (;;) {
    const uint32_t k = tk[i];
    if (k == s) return i;
    if (k == kTabEmpty) return kTabEmpty;
    i = (i + 1) & (kSpecTab - 1);
  }
}
__device__ __forceinline__ uint32_t lds_ld(const uint32_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(uint32_t *p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// Ordered LDS accesses between the waves of the workgroup.  The LDS performs one wave's accesses in
// issue order, so only the compiler must not reorder them -- a seq_cst atomic would also make the
// wave wait for its outstanding global stores (s_waitcnt vmcnt(0)), which the commit path avoids.
__device__ __forceinline__ uint32_t lds_ld_sc(const uint32_t *p) {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  const uint32_t v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  return v;
}
__device__ __forceinline__ void lds_st_sc(uint32_t *p, uint32_t v) {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}
// spin budget of any wait in the speculative loop (~1 s): past it the loop aborts with err bit 64
// instead of hanging the device
constexpr uint32_t kSpecSpin = 1u << 25;
__device__ __forceinline__ uint32_t rdlane(uint32_t x, uint32_t l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)x, (int)l);
}
__device__ __forceinline__ Fe fe_rdlane(const Fe &x, uint32_t l) {
  Fe r;
#pragma unroll
  for (int w = 0; w < 4; ++w)
    r.l[w] = (uint64_t)rdlane((uint32_t)x.l[w], l) | ((uint64_t)rdlane((uint32_t)(x.l[w] >> 32), l) << 32);
  return r;
}
__device__ __forceinline__ Fe fe_shfl(const Fe &x, uint32_t src) {
  Fe r;
#pragma unroll
  for (int w = 0; w < 4; ++w) r.l[w] = __shfl(x.l[w], (int)src);
  return r;
}
__device__ __forceinline__ uint32_t below64(uint64_t m, uint32_t k) {
  return (uint32_t)__popcll(k >= 64 ? m : (m & ((1ull << k) - 1ull)));
}

// masks over up to 64*E positions (E words)
template <int E>
struct Mask {
  uint64_t w[E];
};
template <int E>
__device__ __forceinline__ uint32_t mask_below(const Mask<E> &m, uint32_t k) {  // set bits below k
  uint32_t n = 0;
#pragma unroll
  for (int e = 0; e < E; ++e) n += below64(m.w[e], k >= 64u * e ? k - 64u * e : 0u);
  return n;
}
template <int E>
__device__ __forceinline__ uint32_t mask_count(const Mask<E> &m) {
  uint32_t n = 0;
#pragma unroll
  for (int e = 0; e < E; ++e) n += (uint32_t)__popcll(m.w[e]);
  return n;
}
template <int E>
__device__ __forceinline__ Mask<E> mask_low(const Mask<E> &m, uint32_t k) {  // bits below k only
  Mask<E> r;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const uint32_t b = 64u * e;
    r.w[e] = k >= b + 64 ? m.w[e] : (k <= b ? 0ull : m.w[e] & ((1ull << (k - b)) - 1ull));
  }
  return r;
}
template <int E>
__device__ __forceinline__ Mask<E> mask_shr(const Mask<E> &m, uint32_t k) {  // m >> k
  Mask<E> r;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const uint32_t s = 64u * e + k;  // source bit of r's bit 64e
    const uint32_t q = s >> 6, o = s & 63;
    uint64_t lo = 0, hi = 0;
#pragma unroll
    for (int f = 0; f < E; ++f) {
      if ((uint32_t)f == q) lo = m.w[f];
      if ((uint32_t)f == q + 1) hi = m.w[f];
    }
    r.w[e] = s >= 64u * E ? 0ull : (o ? (lo >> o) | (hi << (64 - o)) : lo);
  }
  return r;
}
// lower_bound over a sorted LDS list of n <= 64*E keys (branch-free; a[] readable up to 64E - 1)
template <int E>
__device__ __forceinline__ uint32_t lds_lb_e(const uint32_t *a, uint32_t n, uint32_t key, bool &hit) {
  uint32_t pos = 0;
#pragma unroll
  for (uint32_t step = 32 * E; step >= 1; step >>= 1) {
    const uint32_t q = pos + step;
    const uint32_t v = a[q - 1];
    pos = ((q <= n) & (v < key)) ? q : pos;
  }
  const uint32_t v = a[pos < 64 * E - 1 ? pos : 64 * E - 1];
  const bool lt = (pos < n) & (v < key);  // only when all 64E keys are below key
  hit = (pos < n) & (v == key);
  return pos + (lt ? 1u : 0u);
}

template <int NW>
struct SpecSmem {
  uint32_t tk[kSpecTab], tv[kSpecTab];
  uint32_t wk[NW][128], rk[NW][128], ix[NW][128];  // a merge's two key lists, its output permutation
  uint32_t kl[NW][kSpecK];                         // keys the wave's reduction saw
  uint32_t ring[kSpecRing];                        // pivot of committed row j at j % kSpecRing (or RS_NONE)
  uint32_t hoff[kSpecRing];                        // header offset of row j's new holder (or RS_NONE)
  uint32_t hrow[kSpecRing];                        // the row whose turn wrote hoff's slot
  uint32_t vis[kSpecRing];                         // j + 1 once row j's global stores are complete
  uint32_t s_next, s_turn, s_vis, s_m, s_nl, s_ok, s_nent, s_abort;
  uint64_t s_acur, s_aend;                         // the committer's pool chunk
  unsigned long long s_tend;                       // RS_PROF: when the last commit passed the turn on
  unsigned long long s_prof[8];
};
template <int NW>
union SpecLds {
  SpecSmem<NW> s;
  BigSmem<512> b;  // a cluster too large for the table runs k_big_main's loop (wave 0) on the same LDS
};

// one wave's row: the work list, entry p = 64 e + lane in register e (keys ascending), plus what
// validation needs.  E = 1 while speculating; the turn's exact pass of an overflowed row uses E = 2.
template <int E>
struct SpecRow {
  uint32_t key[E], slot[E];  // slot: the key's table slot, kTabEmpty = forbidden
  Fe val[E];
  uint32_t len;              // uniform
  uint32_t nk;               // recorded keys (uniform)
  bool serial;               // over 64 E entries: lane 0 finishes the row at the turn
  bool over;                 // more keys than the record holds: any pivot committed meanwhile is a conflict
  unsigned long long by, merges;
};

template <int E, class T>
__device__ __forceinline__ T sel_e(const T (&x)[E], uint32_t e) {  // x[e] for a uniform e
  T r = x[0];
#pragma unroll
  for (int f = 1; f < E; ++f)
    if ((uint32_t)f == e) r = x[f];
  return r;
}

// Commits pass the turn on without waiting for their global stores (the new holder's entries); a
// reader of a holder first checks that no row whose stores may still be in flight -- rows [s_vis,
// s_turn] -- wrote it.  Each committer marks its row visible after its stores completed, off the
// critical path, and the watermark s_vis follows in row order.
template <int NW>
__device__ __forceinline__ bool sp_visible(const SpecSmem<NW> &S, uint32_t lane, uint32_t ho) {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);  // after the state load that named the holder
  const uint32_t v = lds_ld_sc(&S.s_vis), t = lds_ld_sc(&S.s_turn);
  const uint32_t x = v + lane;  // rows [v, t]: a slot counts only once row x's turn has claimed it
  const bool pend = lane <= t - v && lane < kSpecRing && lds_ld_sc(&S.hrow[x % kSpecRing]) == x &&
                    lds_ld_sc(&S.hoff[x % kSpecRing]) == ho;
  return __ballot(pend) == 0;
}
template <int NW>
__device__ __forceinline__ void sp_wait_visible(SpecSmem<NW> &S, uint32_t lane, uint32_t ho) {
  for (uint32_t it = 0; !sp_visible<NW>(S, lane, ho); ++it) {
    if (it > kSpecSpin || lds_ld(&S.s_abort)) { lds_st(&S.s_abort, 1); break; }
    __builtin_amdgcn_s_sleep(1);
  }
  __atomic_signal_fence(__ATOMIC_SEQ_CST);  // the holder's loads after the check (same CU: its L1)
}
// a holder's header and right-hand side staged in registers: entry i (0 = the header) in lane
// i % 64 of register i / 64
template <int E>
__device__ __forceinline__ void sp_stage(const ElimArgs &A, uint32_t lane, uint32_t ho, uint32_t (&sk)[E], Fe (&sv)[E]) {
#pragma unroll
  for (int f = 0; f < E; ++f) {
    const uint64_t hi = (uint64_t)ho + 64u * f + lane;
    const bool inp = hi < A.pool_cap;
    sk[f] = inp ? A.pk[hi] : 0u;
    sv[f] = inp ? A.pv[hi] : fe_zero();
  }
}

// Reduce the row (keys `okey` / slots `osl` of its first 64 entries in the lanes, the rest and the
// values from the row) against the table's current state.  p4: until no deleted key is left; p3:
// until the largest takeable key is not deleted.  The holder the next merge will most likely need
// (the next pivot from the merged keys, assuming nothing cancels) is loaded under the current
// merge's products.
template <int E, int NW>
__device__ __forceinline__ void sp_reduce(const ElimArgs &A, SpecSmem<NW> &S, uint32_t wv, uint32_t lane, bool p4,
                                          uint64_t r_off, uint32_t olen, uint32_t okey, uint32_t osl, SpecRow<E> &R,
                                          uint32_t j) {
  const FieldP &F = A.F;
  constexpr uint32_t CAPL = 64 * E;
  R.len = olen;
  R.nk = 0;
  R.over = false;
  R.serial = olen > CAPL;
  R.by = 36ull * olen;
  R.merges = 0;
  if (R.serial) return;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const uint32_t p = 64 * e + lane;
    const uint32_t k = e == 0 ? okey : (p < olen ? A.rows.key[r_off + p] : 0u);
    R.key[e] = p < olen ? k : 0u;
    R.slot[e] = p < olen ? (e == 0 ? osl : sp_find(S.tk, k)) : kTabEmpty;
    R.val[e] = p < olen ? A.rows.val[r_off + p] : fe_zero();
    if (olen <= kSpecK && p < olen) S.kl[wv][p] = R.key[e];
  }
  if (olen <= kSpecK) R.nk = olen;
  else R.over = true;
  uint32_t pf_ho = RS_NONE;  // the staged holder
  uint32_t sk[E];
  Fe sv[E];
  for (;;) {
    if (lds_ld(&S.s_abort)) return;
    // a row still reducing when its turn comes is the critical path: its wave wins the SIMD's issue
    // arbitration from then on (the turn lowers it again)
    if (rdlane(lds_ld(&S.s_turn), 0) == j) __builtin_amdgcn_s_setprio(2);
    const uint32_t len = R.len;
    uint32_t st[E];
    uint64_t tm[E], dm[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const uint32_t p = 64 * e + lane;
      st[e] = (p < len && R.slot[e] != kTabEmpty) ? lds_ld(&S.tv[R.slot[e]]) : kStForb;
      const bool tkb = st[e] != kStForb;
      tm[e] = __ballot(tkb);
      dm[e] = __ballot(tkb && (st[e] & kStDel));
    }
    uint32_t oi = RS_NONE;
    if (p4) {  // take_signal_4: the first deleted key, ascending
#pragma unroll
      for (int e = E - 1; e >= 0; --e)
        if (dm[e]) oi = 64 * e + __ffsll((long long)dm[e]) - 1;
      if (oi == RS_NONE) return;
    } else {   // take_signal_3: the largest takeable key; a merge only if it is deleted
#pragma unroll
      for (int e = 0; e < E; ++e)
        if (tm[e]) oi = 64 * e + 63 - __clzll(tm[e]);
      if (oi == RS_NONE) return;
      if (!((sel_e<E>(dm, oi >> 6) >> (oi & 63)) & 1ull)) return;
    }
    const uint32_t oe = oi >> 6, ol = oi & 63;
    const uint32_t ho = rdlane(sel_e<E>(st, oe), ol) & ~kStDel;  // the holder's header in the pool
    const Fe coef = fneg(F, fe_rdlane(sel_e<E>(R.val, oe), ol));
    if (ho != pf_ho) {
      sp_wait_visible<NW>(S, lane, ho);
      sp_stage<E>(A, lane, ho, sk, sv);
    }
    pf_ho = RS_NONE;
    const uint32_t rl = rdlane(sk[0], 0);
    const Fe c2 = fe_rdlane(sv[0], 0);
    const uint32_t tot = len + rl;
    if (tot > CAPL) {  // beyond the lanes' capacity: lane 0 finishes the row at its turn
      R.serial = true;
      return;
    }
    uint32_t key[E], lb[E], rsl[E];
    bool isw[E], isr[E], hit[E], keep[E];
    Fe ev[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {  // RHS entry j (staged entry j + 1) to position len + j
      const uint32_t p = 64 * e + lane;
      isw[e] = p < len;
      isr[e] = !isw[e] && p < tot;
      const uint32_t si = p - len + 1;
      uint32_t k_ = (uint32_t)__shfl((int)sk[0], (int)(si & 63));
      ev[e] = fe_shfl(sv[0], si & 63);
#pragma unroll
      for (int f = 1; f < E; ++f) {
        const uint32_t k2 = (uint32_t)__shfl((int)sk[f], (int)(si & 63));
        const Fe v2 = fe_shfl(sv[f], si & 63);
        if ((si >> 6) == (uint32_t)f) { k_ = k2; ev[e] = v2; }
      }
      key[e] = isw[e] ? R.key[e] : (isr[e] ? k_ : 0xffffffffu);
      if (isw[e]) S.wk[wv][p] = key[e];
      if (isr[e]) S.rk[wv][p - len] = key[e];
    }
    wave_sync();
    uint32_t str[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      lb[e] = lds_lb_e<E>(isw[e] ? S.rk[wv] : S.wk[wv], isw[e] ? rl : (isr[e] ? len : 0u), key[e], hit[e]);
      rsl[e] = isr[e] ? sp_find(S.tk, key[e]) : kTabEmpty;
      str[e] = isr[e] && !hit[e] && rsl[e] != kTabEmpty ? lds_ld(&S.tv[rsl[e]]) : kStForb;
    }
    {  // the next pivot from the merged keys (none cancelled): stage its holder now
      uint32_t cand = RS_NONE, cst = 0;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const uint32_t p = 64 * e + lane;
        const uint32_t s2 = isw[e] ? (p != oi ? st[e] : kStForb) : str[e];
        const bool tkb = s2 != kStForb;
        // p4: the smallest deleted key; p3: the largest takeable key, if deleted
        const bool c = p4 ? (tkb && (s2 & kStDel)) : tkb;
        // p4: the wave minimum; p3: the maximum as the minimum of the complements (DPP, every lane active)
        const uint32_t kk = p4 ? wave_min_u32(c ? key[e] : 0xffffffffu) : ~wave_min_u32(c ? ~key[e] : 0xffffffffu);
        const uint64_t own = __ballot(c && key[e] == kk);
        if (own && (p4 ? kk < cand || cand == RS_NONE : kk > cand || cand == RS_NONE)) {
          cand = kk;
          cst = rdlane(s2, (uint32_t)__ffsll((long long)own) - 1);
        }
      }
      if (cand != RS_NONE && (cst & kStDel)) {
        const uint32_t nho = cst & ~kStDel;
        if (sp_visible<NW>(S, lane, nho)) {
          __atomic_signal_fence(__ATOMIC_SEQ_CST);
          sp_stage<E>(A, lane, nho, sk, sv);
          pf_ho = nho;
        }
      }
    }
    Fe val[E];
#pragma unroll
    for (int e = 0; e < E; ++e)
      if (64u * e < tot) val[e] = fmul256(F, isw[e] ? c2 : coef, isw[e] ? R.val[e] : ev[e]);
      else val[e] = fe_zero();
    Mask<E> M;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const uint32_t p = 64 * e + lane;
      // the RHS product of a shared key: position len + lb
      const uint32_t sp = (isw[e] && hit[e]) ? len + lb[e] : p;
      Fe rv = fe_shfl(val[0], sp & 63);
#pragma unroll
      for (int f = 1; f < E; ++f) {
        const Fe t = fe_shfl(val[f], sp & 63);
        if ((sp >> 6) == (uint32_t)f) rv = t;
      }
      keep[e] = false;
      if (isw[e]) {
        if (p != oi) {
          val[e] = hit[e] ? fsub(F, rv, val[e]) : fneg(F, val[e]);
          keep[e] = !fe_is_zero(val[e]);
        }
      } else if (isr[e]) {
        keep[e] = !hit[e] && !fe_is_zero(val[e]);
      }
      M.w[e] = __ballot(keep[e]);
    }
    const Mask<E> Wm = mask_low<E>(M, len), Rm = mask_shr<E>(M, len);
    const uint32_t nr = mask_count<E>(Rm), nlen = mask_count<E>(M);
    if (!R.over && R.nk + nr > kSpecK) R.over = true;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const uint32_t p = 64 * e + lane;
      if (!keep[e]) continue;
      const uint32_t dst = isw[e] ? mask_below<E>(Wm, p) + mask_below<E>(Rm, lb[e])
                                  : mask_below<E>(Rm, p - len) + mask_below<E>(Wm, lb[e]);
      S.ix[wv][dst] = p;
      if (!R.over && isr[e]) S.kl[wv][R.nk + mask_below<E>(Rm, p - len)] = key[e];
    }
    wave_sync();
    uint32_t slot[E];
#pragma unroll
    for (int e = 0; e < E; ++e) slot[e] = isw[e] ? R.slot[e] : rsl[e];
#pragma unroll
    for (int e = 0; e < E; ++e) {  // gather the output position q = 64 e + lane from its source position
      const uint32_t q = 64 * e + lane;
      const uint32_t s = q < nlen ? S.ix[wv][q] : q;
      const uint32_t sl = s & 63, se = s >> 6;
      uint32_t nk_ = (uint32_t)__shfl((int)key[0], (int)sl), ns_ = (uint32_t)__shfl((int)slot[0], (int)sl);
      Fe nv = fe_shfl(val[0], sl);
#pragma unroll
      for (int f = 1; f < E; ++f) {
        const uint32_t k2 = (uint32_t)__shfl((int)key[f], (int)sl), s2 = (uint32_t)__shfl((int)slot[f], (int)sl);
        const Fe v2 = fe_shfl(val[f], sl);
        if (se == (uint32_t)f) { nk_ = k2; ns_ = s2; nv = v2; }
      }
      R.key[e] = nk_;
      R.slot[e] = q < nlen ? ns_ : kTabEmpty;
      R.val[e] = nv;
    }
    if (!R.over) R.nk += nr;
    R.by += 36ull * (len + rl + nlen);
    R.merges++;
    R.len = nlen;
    wave_sync();
  }
}

// Did a pivot committed by rows [from, to) appear in the wave's recorded keys?
template <int NW, int E>
__device__ __forceinline__ bool sp_conflict(const SpecSmem<NW> &S, uint32_t wv, uint32_t lane, const SpecRow<E> &R,
                                            uint32_t from, uint32_t to) {
  for (uint32_t x = from; x < to; ++x) {
    const uint32_t p = lds_ld(&S.ring[x % kSpecRing]);
    if (p == RS_NONE) continue;
    if (R.over) return true;
    bool h = false;
    for (uint32_t t = lane; t < R.nk; t += 64) h |= S.kl[wv][t] == p;
    if (__ballot(h)) return true;
  }
  return false;
}

// the committer's pool allocation (one wave at a time, lane 0)
template <int NW>
__device__ __forceinline__ uint64_t sp_alloc(const ElimArgs &A, SpecSmem<NW> &S, uint64_t n) {
  Alloc al;
  al.cur = S.s_acur;
  al.end = S.s_aend;
  al.chunk = 4096;
  const uint64_t o = pool_alloc(A, al, n);
  S.s_acur = al.cur;
  S.s_aend = al.end;
  return o;
}
__device__ __forceinline__ uint64_t rdlane64(uint64_t x, uint32_t l) {
  return ((uint64_t)rdlane((uint32_t)(x >> 32), l) << 32) | rdlane((uint32_t)x, l);
}

// The turn's second half for a reduced row j: the pivot on the fresh counts -- take_signal_4 (no
// deleted key is left: min occurrences, ties -> the largest id) or take_signal_3 (the largest
// takeable key, not deleted) -- then the new holder (header, RHS with {0: 0} ensured) or the
// leftover.  The holder's offset is recorded for row j before its state is published.  Returns
// the new pivot, or RS_NONE.
template <int E, int NW>
__device__ __forceinline__ uint32_t sp_commit(const ElimArgs &A, SpecSmem<NW> &S, uint64_t b, uint32_t j, uint32_t lane,
                                              bool p4, const SpecRow<E> &R, unsigned long long &by) {
  const FieldP &F = A.F;
  const uint32_t len = R.len;
  if (len == 0) return RS_NONE;
  uint32_t st[E];
  uint64_t tm[E], dmf[E];
  unsigned long long best = ~0ull;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const uint32_t p = 64 * e + lane;
    st[e] = (p < len && R.slot[e] != kTabEmpty) ? lds_ld(&S.tv[R.slot[e]]) : kStForb;
    const bool tkb = st[e] != kStForb;
    tm[e] = __ballot(tkb);
    dmf[e] = __ballot(tkb && (st[e] & kStDel));
    if (tkb) {
      const unsigned long long vv = ((unsigned long long)st[e] << 32) | (0xffffffffu - p);
      best = vv < best ? vv : best;
    }
  }
  uint32_t oi = RS_NONE;
  if (p4) {  // the minimum of (occurrences << 32 | ~index): the high words' minimum, then the low words' among it
    const uint32_t mh = wave_min_u32((uint32_t)(best >> 32));
    const uint32_t ml = wave_min_u32((uint32_t)(best >> 32) == mh ? (uint32_t)best : 0xffffffffu);
    if (((unsigned long long)mh << 32 | ml) != ~0ull) oi = 0xffffffffu - ml;
  } else {
#pragma unroll
    for (int e = 0; e < E; ++e)
      if (tm[e]) oi = 64 * e + 63 - __clzll(tm[e]);
  }
  {  // a validated reduction leaves no deleted key (p4) / a takeable largest key (p3)
    bool bad = false;
#pragma unroll
    for (int e = 0; e < E; ++e) bad |= p4 && dmf[e] != 0;
    if (!p4 && oi != RS_NONE) bad = (sel_e<E>(dmf, oi >> 6) >> (oi & 63)) & 1ull;
    if (bad && lane == 0) atomicOr(A.err, 16);
  }
  if (oi == RS_NONE) {  // nothing takeable: leftover (lconst), unnormalised
    uint64_t o = 0;
    if (lane == 0) o = sp_alloc<NW>(A, S, len);
    o = rdlane64(o, 0);
    by += 36ull * len;
    if (o == RS_NONE) {
      if (lane == 0) S.s_ok = 0;
      return RS_NONE;
    }
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const uint32_t p = 64 * e + lane;
      if (p < len) { A.pk[o + p] = R.key[e]; A.pv[o + p] = R.val[e]; }
    }
    if (lane == 0) { A.l_off[b + S.s_nl] = o; A.l_len[b + S.s_nl] = len; S.s_nl = S.s_nl + 1; }
    return RS_NONE;
  }
  // new substitution p = -(work - v_p p) / v_p (clear_signal_not_normalized), header first
  const uint32_t oe = oi >> 6, ol = oi & 63;
  const uint32_t piv = rdlane(sel_e<E>(R.key, oe), ol);
  const uint32_t psl = rdlane(sel_e<E>(R.slot, oe), ol);
  const uint32_t sh = rdlane(R.key[0], 0) == 0 ? 0u : 1u;  // {0: 0} is inserted when absent
  const uint32_t mm = len - 1 + sh;
  const Fe cf = fneg(F, fe_rdlane(sel_e<E>(R.val, oe), ol));
  by += 36ull * mm;
  uint64_t o = 0;
  if (lane == 0) o = sp_alloc<NW>(A, S, (uint64_t)mm + 1);
  o = rdlane64(o, 0);
  if (o == RS_NONE) {
    if (lane == 0) S.s_ok = 0;
    return RS_NONE;
  }
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const uint32_t p = 64 * e + lane;
    if (p < len && p != oi) {
      const uint64_t q = o + 1 + (p < oi ? p : p - 1) + sh;
      A.pk[q] = R.key[e];
      A.pv[q] = R.val[e];
    }
  }
  if (lane == 0) {
    if (sh) { A.pk[o + 1] = 0; A.pv[o + 1] = fe_zero(); }
    A.pk[o] = mm;
    A.pv[o] = cf;
    d_set_holder(A, piv, b + S.s_m, cf, o + 1, mm);
    S.s_m = S.s_m + 1;
    A.occ[piv] = -1;
    A.del[piv] = 1;
    lds_st_sc(&S.hoff[j % kSpecRing], (uint32_t)o);  // row j may still be writing the holder at o
    if (psl != kTabEmpty) lds_st_sc(&S.tv[psl], kStDel | (uint32_t)o);
  }
  return piv;
}

template <int NW>
__global__ __launch_bounds__(64 * NW) void k_big_spec(ElimArgs A, const uint32_t *ids, uint64_t n_ids) {
  __shared__ SpecLds<NW> U;
  SpecSmem<NW> &S = U.s;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nt = 64 * NW;
  const bool prof = A.prof != nullptr;
  for (uint64_t ci = blockIdx.x; ci < n_ids; ci += gridDim.x) {
    if (A.skip && A.skip[ci]) continue;  // a giant cluster: giant_loop.hpp's component loops take it
    const uint64_t c = ids[ci];
    const uint64_t b = A.cl_off[c], e = A.cl_off[c + 1];
    const bool p4 = d_is_p4(A, (uint32_t)(e - b));
    const uint32_t n_loop = A.big_alive[ci];
    const uint32_t n_touch = A.big_touch_n[ci];
    const uint64_t touch_off = A.big_touch_off[ci];
    if (n_loop == 0) {  // nothing for the ordered loop (every row went to the uniques phase)
      if (tid == 0) A.n_left[c] = 0;
      continue;
    }
    // process_3 clusters have no touched list: the table is built from the rows, bounded by their entries
    if (tid == 0) S.s_nent = 0;
    __syncthreads();
    if (!p4) {
      unsigned long long n_ent = 0;
      for (uint32_t pos = tid; pos < n_loop; pos += nt) n_ent += A.row_len[b + pos];
      if (n_ent) atomicAdd(&S.s_nent, (uint32_t)min(n_ent, 0xffffffull));
    }
    __syncthreads();
    const uint32_t n_sig = p4 ? n_touch : S.s_nent;
    if (n_sig > kSpecTabMax || A.pool_cap >= (uint64_t)kStDel) {
      __syncthreads();
      if (wv == 0) {
        Alloc al0;
        al0.chunk = 4096;
        d_big_main_cluster<512>(A, ids, ci, U.b, al0);
      }
      __syncthreads();
      continue;
    }
    const unsigned long long t_1 = prof ? wall_clock64() : 0ull;
    // ---- the cluster's signal table
    for (uint32_t i = tid; i < kSpecTab; i += nt) S.tk[i] = kTabEmpty;
    for (uint32_t i = tid; i < kSpecRing; i += nt) {
      S.ring[i] = RS_NONE;
      S.hoff[i] = RS_NONE;
      S.hrow[i] = RS_NONE;
      S.vis[i] = 0;
    }
    __syncthreads();
    if (!p4) {  // every non-forbidden key of the rows, takeable (nothing is deleted yet)
      for (uint32_t pos = wv; pos < n_loop; pos += NW) {
        const uint64_t ro = A.row_off[b + pos];
        const uint32_t rl_ = A.row_len[b + pos];
        for (uint32_t i = lane; i < rl_; i += 64) {
          const uint32_t s = A.rows.key[ro + i];
          if (A.forb[s]) continue;
          uint32_t q = sp_slot(s);
          for (;;) {
            const uint32_t old = atomicCAS(&S.tk[q], kTabEmpty, s);
            if (old == kTabEmpty) { S.tv[q] = 0; break; }
            if (old == s) break;
            q = (q + 1) & (kSpecTab - 1);
          }
        }
      }
    }
    for (uint32_t t = tid; p4 && t < n_touch; t += nt) {
      const uint32_t sg = A.pk[touch_off + t];
      if (!sg) continue;
      uint32_t st;
      if (A.del[sg]) {
        st = kStDel | (uint32_t)(A.h_off[A.holder_idx[sg]] - 1);
      } else {
        const int32_t o = A.occ[sg];
        st = o < 0 ? 0u : (uint32_t)o;
      }
      uint32_t q = sp_slot(sg);
      for (;;) {
        const uint32_t old = atomicCAS(&S.tk[q], kTabEmpty, sg);
        if (old == kTabEmpty || old == sg) break;
        q = (q + 1) & (kSpecTab - 1);
      }
      S.tv[q] = st;
    }
    if (tid == 0) {
      S.s_next = 0;
      S.s_turn = 0;
      S.s_vis = 0;
      S.s_m = A.n_sub[c];
      S.s_nl = 0;
      S.s_ok = 1;
      S.s_abort = 0;
      S.s_acur = S.s_aend = 0;
      S.s_tend = t_1;
      for (int q = 0; q < 8; ++q) S.s_prof[q] = 0;
    }
    __syncthreads();
    // RS_PROF counters: [0] conflicts found at the turn, [1] rows finished on lane 0, [2] committed
    // merges, [3] merges thrown away by conflicts, [4] turn time (the critical path's own work), [5]
    // of it the exact passes of conflicted / overflowed rows, [6] turns that found their row still
    // speculating and [7] the time the turn waited for them
    unsigned long long by = 0, pc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    SpecRow<1> R;
    for (;;) {
      // ---- dispatch: the next row in pop order
      uint32_t j = 0;
      if (lane == 0) j = atomicAdd(&S.s_next, 1u);
      j = rdlane(j, 0);
      if (j >= n_loop) break;
      const uint32_t qi = n_loop - 1 - j;
      const uint64_t r_off = A.row_off[b + qi];
      const uint32_t olen = A.row_len[b + qi];
      const uint32_t okey = lane < olen ? A.rows.key[r_off + lane] : 0u;
      const uint32_t osl = lane < olen ? sp_find(S.tk, okey) : kTabEmpty;
      // ---- speculate
      uint32_t c0 = rdlane(lds_ld_sc(&S.s_turn), 0);
      sp_reduce<1, NW>(A, S, wv, lane, p4, r_off, olen, okey, osl, R, j);
      // ---- wait for the turn, validating the commits that land meanwhile; a conflict found
      // before the turn is reduced again right away (against the newer state)
      bool conflict = false, first = true, late = false;
      for (uint32_t it = 0;; ++it) {
        if (it > kSpecSpin || lds_ld(&S.s_abort)) { lds_st(&S.s_abort, 1); break; }
        const uint32_t sc = rdlane(lds_ld_sc(&S.s_turn), 0);
        if (!R.serial && !conflict && c0 < sc) conflict = sp_conflict<NW, 1>(S, wv, lane, R, c0, sc);
        c0 = sc;
        if (sc == j) { late = first; break; }
        first = false;
        if (conflict) {
          pc[3] += R.merges;
          sp_reduce<1, NW>(A, S, wv, lane, p4, r_off, olen, okey, osl, R, j);
          conflict = false;
          continue;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      // ---- the turn: the state is final for this row.  The committing wave is the critical path of
      // the whole loop: it takes the SIMD's issue arbitration from the speculating wave beside it
      // (MI355X_MICROARCH.md: VALU issue goes by priority, then age) until it passes the turn on.
      __builtin_amdgcn_s_setprio(3);
      const unsigned long long t_a = prof ? wall_clock64() : 0ull;
      if (prof && late) { pc[6]++; pc[7] += t_a - __hip_atomic_load(&S.s_tend, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
      if (conflict) {
        pc[0]++;
        pc[3] += R.merges;
        sp_reduce<1, NW>(A, S, wv, lane, p4, r_off, olen, okey, osl, R, j);
      }
      if (lds_ld(&S.s_abort)) break;  // a wait ran out of budget: every wave leaves, err bit 64
      const bool ok = lds_ld(&S.s_ok) != 0;
      uint32_t piv = RS_NONE;
      // row j's ring slots were row j - 64's: its stores must be known complete before they are reused
      {
        uint32_t it = 0;
        for (; lds_ld_sc(&S.s_vis) + kSpecRing <= j && it <= kSpecSpin; ++it) __builtin_amdgcn_s_sleep(1);
        if (it > kSpecSpin) {  // out of budget: the slot is not safe to reuse -- abort (err bit 64)
          lds_st(&S.s_abort, 1);
          break;
        }
      }
      if (lane == 0) {
        lds_st_sc(&S.hoff[j % kSpecRing], RS_NONE);
        lds_st_sc(&S.hrow[j % kSpecRing], j);
      }
      // remove_constraint (:94-106): occurrences of the original row's takeable, undeleted keys
      for (uint32_t i = lane; ok && i < olen; i += 64) {
        const uint32_t k = i < 64 ? okey : A.rows.key[r_off + i];
        const uint32_t ti = i < 64 ? osl : sp_find(S.tk, k);
        if (ti == kTabEmpty) continue;
        uint32_t st = lds_ld(&S.tv[ti]);
        if (!(st & kStDel) && st > 0) {
          st -= 1;
          lds_st(&S.tv[ti], st);
          A.occ[k] = (int32_t)st;
        }
      }
      bool done = !ok;
      if (!done && R.serial && olen <= 128) {  // two entries per lane, now that nothing else commits
        SpecRow<2> R2;
        sp_reduce<2, NW>(A, S, wv, lane, p4, r_off, olen, okey, osl, R2, j);
        if (!R2.serial) {
          pc[2] += R2.merges;
          by += R2.by;
          piv = sp_commit<2, NW>(A, S, b, j, lane, p4, R2, by);
          done = true;
        }
      }
      if (!done && R.serial) {  // lane 0 finishes the row on the global state (d_treat_scalar)
        pc[1]++;
        // every earlier row's global stores, and this row's occurrence writes, complete
        {
          uint32_t it = 0;
          for (; lds_ld_sc(&S.s_vis) < j && it <= kSpecSpin; ++it) __builtin_amdgcn_s_sleep(1);
          if (it > kSpecSpin) {  // out of budget: the global state may be incomplete -- abort (err bit 64)
            lds_st(&S.s_abort, 1);
            break;
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
        if (lane == 0) {
          uint32_t m = S.s_m, nl = S.s_nl;
          Alloc al;
          al.cur = S.s_acur;
          al.end = S.s_aend;
          al.chunk = 4096;
          if (!d_treat_scalar(A, al, b, A.rows.key + r_off, A.rows.val + r_off, olen, m, nl, p4)) S.s_ok = 0;
          S.s_acur = al.cur;
          S.s_aend = al.end;
          if (m > S.s_m) {  // its new substitution's pivot is deleted now
            piv = A.h_sig[b + m - 1];
            const uint32_t ti = sp_find(S.tk, piv);
            lds_st_sc(&S.hoff[j % kSpecRing], (uint32_t)(A.h_off[b + m - 1] - 1));
            if (ti != kTabEmpty) lds_st_sc(&S.tv[ti], kStDel | (uint32_t)(A.h_off[b + m - 1] - 1));
          }
          S.s_m = m;
          S.s_nl = nl;
        }
        piv = rdlane(piv, 0);
        by += 36ull * olen;
        done = true;
      }
      if (!done) {
        pc[2] += R.merges;
        by += R.by;
        piv = sp_commit<1, NW>(A, S, b, j, lane, p4, R, by);
      }
      if (prof) {
        const unsigned long long t_b = wall_clock64();
        pc[4] += t_b - t_a;
        if (conflict || R.serial) pc[5] += t_b - t_a;
        if (lane == 0) __hip_atomic_store(&S.s_tend, t_b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      // pass the turn on: LDS state in order (the LDS completes a wave's accesses in order), the
      // global stores not waited for -- readers check them (sp_visible)
      if (lane == 0) {
        lds_st_sc(&S.ring[j % kSpecRing], piv);
        lds_st_sc(&S.s_turn, j + 1);
      }
      __builtin_amdgcn_s_setprio(0);
      // then this row's global stores complete, and the watermark moves on (in row order: whoever
      // finds the next row's mark set advances it)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if (lane == 0) {
        lds_st_sc(&S.vis[j % kSpecRing], j + 1);
        for (;;) {
          const uint32_t v = lds_ld_sc(&S.s_vis);
          if (lds_ld_sc(&S.vis[v % kSpecRing]) != v + 1) break;
          atomicCAS(&S.s_vis, v, v + 1);
        }
      }
    }
    __builtin_amdgcn_s_setprio(0);  // an aborted turn may leave the loop at priority 3
    if (lane == 0) {
      atomicAdd(A.bytes_main, by);
      if (prof)
        for (int q = 0; q < 8; ++q) atomicAdd(&S.s_prof[q], pc[q]);
    }
    __syncthreads();
    if (tid == 0) {
      A.n_sub[c] = S.s_m;
      A.n_left[c] = S.s_nl;
      if (!S.s_ok) atomicOr(A.err, 8);
      if (S.s_abort) atomicOr(A.err, 64);
      if (prof) {
        unsigned long long *P = A.prof + kProfWords * ci;
        // [2] rows, [5] wall, [22] start; [8..15] the counters above (times in 100 MHz ticks)
        P[2] = n_loop;
        P[5] = wall_clock64() - t_1;
        P[22] = t_1;
        for (int q = 0; q < 8; ++q) P[8 + q] = S.s_prof[q];
      }
    }
    __syncthreads();
  }
}

}  // namespace rs
