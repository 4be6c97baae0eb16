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
// the holder's header offset, else the occurrence count -- as k_big_main_lds), per wave the merge's
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

template <int NW>
struct SpecSmem {
  uint32_t tk[kSpecTab], tv[kSpecTab];
  uint32_t wk[NW][64], rk[NW][64], ix[NW][64];  // a merge's two key lists, its output permutation
  uint32_t kl[NW][kSpecK];                      // keys the wave's reduction saw
  uint32_t ring[kSpecRing];                     // pivot of committed row j at j % kSpecRing (or RS_NONE)
  uint32_t s_next, s_turn, s_m, s_nl, s_ok, s_nent;
  uint64_t s_acur, s_aend;                      // the committer's pool chunk
  unsigned long long s_prof[4];                 // conflicts, serial rows, merges, recomputed merges
};
template <int NW>
union SpecLds {
  SpecSmem<NW> s;
  BigSmem<512> b;  // a cluster too large for the table runs k_big_main's loop (wave 0) on the same LDS
};

// one wave's row: the work list, one entry per lane (keys ascending), plus what validation needs
struct SpecRow {
  uint32_t key, slot;  // slot: the key's table slot, kTabEmpty = forbidden
  Fe val;
  uint32_t len;        // uniform
  uint32_t nk;         // recorded keys (uniform)
  bool serial;         // finish on lane 0 at the turn (over a lane's capacity)
  bool over;           // more keys than the record holds: any pivot committed meanwhile is a conflict
  unsigned long long by, merges;
};

// Reduce the row (keys `okey` / slots `osl` in lanes < olen, values from the row) against the table's
// current state.  p4: until no deleted key is left; p3: until the largest takeable key is not deleted.
template <int NW>
__device__ __forceinline__ void sp_reduce(const ElimArgs &A, SpecSmem<NW> &S, uint32_t wv, uint32_t lane, bool p4,
                                          uint64_t r_off, uint32_t olen, uint32_t okey, uint32_t osl, SpecRow &R) {
  const FieldP &F = A.F;
  R.len = olen;
  R.nk = 0;
  R.over = false;
  R.serial = olen > 64;
  R.by = 36ull * olen;
  R.merges = 0;
  if (R.serial) return;
  R.key = lane < olen ? okey : 0u;
  R.slot = lane < olen ? osl : kTabEmpty;
  R.val = lane < olen ? A.rows.val[r_off + lane] : fe_zero();
  if (olen <= kSpecK) {
    if (lane < olen) S.kl[wv][lane] = okey;
    R.nk = olen;
  } else {
    R.over = true;
  }
  for (;;) {
    const uint32_t len = R.len;
    const uint32_t st = (lane < len && R.slot != kTabEmpty) ? lds_ld(&S.tv[R.slot]) : kStForb;
    const bool tkb = st != kStForb, dl = tkb && (st & kStDel);
    const uint64_t tm = __ballot(tkb), dm = __ballot(dl);
    uint32_t oi;
    if (p4) {
      if (!dm) return;
      oi = __ffsll((long long)dm) - 1;
    } else {
      if (!tm) return;
      oi = 63 - __clzll(tm);
      if (!((dm >> oi) & 1ull)) return;
    }
    const uint32_t ho = rdlane(st, oi) & ~kStDel;  // the holder's header in the pool
    const Fe coef = fneg(F, fe_rdlane(R.val, oi));
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");  // the holder's entries were published before its state
    // one round trip: work lanes read the header (same address), lane len + j the RHS entry j
    const uint64_t hi = (uint64_t)ho + (lane < len ? 0u : 1u + lane - len);
    const bool inp = hi < A.pool_cap;
    const uint32_t ek = inp ? A.pk[hi] : 0u;
    const Fe ev = inp ? A.pv[hi] : fe_zero();
    const uint32_t rl = rdlane(ek, 0);
    const Fe c2 = fe_rdlane(ev, 0);
    if (len + rl > 64) {  // beyond a lane per entry: lane 0 finishes the row at its turn
      R.serial = true;
      return;
    }
    const bool isw = lane < len, isr = !isw && lane < len + rl;
    const uint32_t jr = lane - len;
    const uint32_t key = isw ? R.key : (isr ? ek : 0xffffffffu);
    if (isw) S.wk[wv][lane] = key;
    if (isr) S.rk[wv][jr] = key;
    wave_sync();
    bool hit;
    const uint32_t lb = lds_lb64(isw ? S.rk[wv] : S.wk[wv], isw ? rl : (isr ? len : 0u), key, hit);
    const uint32_t rsl = isr ? sp_find(S.tk, key) : kTabEmpty;
    Fe val = fmul256(F, isw ? c2 : coef, isw ? R.val : ev);
    const Fe rv = fe_shfl(val, (isw && hit) ? len + lb : lane);  // the RHS product of a shared key
    bool keep = false;
    if (isw) {
      if (lane != oi) {
        val = hit ? fsub(F, rv, val) : fneg(F, val);
        keep = !fe_is_zero(val);
      }
    } else if (isr) {
      keep = !hit && !fe_is_zero(val);
    }
    const uint64_t km = __ballot(keep);
    const uint64_t wmk = len >= 64 ? km : (km & ((1ull << len) - 1ull)), rmk = km >> len;
    const uint32_t dst = isw ? below64(wmk, lane) + below64(rmk, lb) : below64(rmk, jr) + below64(wmk, lb);
    if (keep) S.ix[wv][dst] = lane;
    const uint32_t nr = (uint32_t)__popcll(rmk);
    if (!R.over && R.nk + nr > kSpecK) R.over = true;
    if (!R.over && isr && keep) S.kl[wv][R.nk + below64(rmk, jr)] = key;
    wave_sync();
    const uint32_t nlen = (uint32_t)__popcll(km);
    const uint32_t src = lane < nlen ? S.ix[wv][lane] : lane;
    const uint32_t slot = isw ? R.slot : rsl;
    R.key = (uint32_t)__shfl((int)key, (int)src);
    R.slot = (uint32_t)__shfl((int)slot, (int)src);
    R.val = fe_shfl(val, src);
    if (!R.over) R.nk += nr;
    R.by += 36ull * (len + rl + nlen);
    R.merges++;
    R.len = nlen;
    wave_sync();
  }
}

// Did a pivot committed by rows [from, to) appear in the wave's recorded keys?
template <int NW>
__device__ __forceinline__ bool sp_conflict(const SpecSmem<NW> &S, uint32_t wv, uint32_t lane, const SpecRow &R,
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

template <int NW>
__global__ __launch_bounds__(64 * NW) void k_big_spec(ElimArgs A, const uint32_t *ids, uint64_t n_ids) {
  __shared__ SpecLds<NW> U;
  SpecSmem<NW> &S = U.s;
  const FieldP &F = A.F;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nt = 64 * NW;
  for (uint64_t ci = blockIdx.x; ci < n_ids; ci += gridDim.x) {
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
    const unsigned long long t_1 = A.prof ? wall_clock64() : 0ull;
    // ---- the cluster's signal table
    for (uint32_t i = tid; i < kSpecTab; i += nt) S.tk[i] = kTabEmpty;
    for (uint32_t i = tid; i < kSpecRing; i += nt) S.ring[i] = RS_NONE;
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
      S.s_m = A.n_sub[c];
      S.s_nl = 0;
      S.s_ok = 1;
      S.s_acur = S.s_aend = 0;
      S.s_prof[0] = S.s_prof[1] = S.s_prof[2] = S.s_prof[3] = 0;
    }
    __syncthreads();
    unsigned long long by = 0, n_conf = 0, n_serial = 0, n_merges = 0, n_remerges = 0;
    SpecRow R;
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
      uint32_t c0 = rdlane(__hip_atomic_load(&S.s_turn, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP), 0);
      sp_reduce<NW>(A, S, wv, lane, p4, r_off, olen, okey, osl, R);
      // ---- wait for the turn, validating the commits that land meanwhile
      bool conflict = false;
      for (;;) {
        const uint32_t sc = rdlane(__hip_atomic_load(&S.s_turn, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP), 0);
        if (!R.serial && !conflict && c0 < sc) conflict = sp_conflict<NW>(S, wv, lane, R, c0, sc);
        c0 = sc;
        if (sc == j) break;
        __builtin_amdgcn_s_sleep(1);
      }
      // ---- the turn: the state is final for this row
      if (conflict) {
        ++n_conf;
        n_remerges += R.merges;
        sp_reduce<NW>(A, S, wv, lane, p4, r_off, olen, okey, osl, R);
      }
      const bool ok = lds_ld(&S.s_ok) != 0;
      uint32_t piv = RS_NONE;
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
      if (!ok) {
      } else if (R.serial) {  // lane 0 finishes the row on the global state (d_treat_scalar)
        ++n_serial;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // the occurrence writes above
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
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (ti != kTabEmpty) lds_st(&S.tv[ti], kStDel | (uint32_t)(A.h_off[b + m - 1] - 1));
          }
          S.s_m = m;
          S.s_nl = nl;
        }
        piv = rdlane(piv, 0);
        by += 36ull * olen;
      } else {
        n_merges += R.merges;
        by += R.by;
        const uint32_t len = R.len;
        // the pivot on the fresh counts: take_signal_4 (no deleted key is left: min occurrences, ties
        // -> the largest id) or take_signal_3 (the largest takeable key, not deleted)
        const uint32_t st = (lane < len && R.slot != kTabEmpty) ? lds_ld(&S.tv[R.slot]) : kStForb;
        const bool tkb = st != kStForb;
        const uint64_t tm = __ballot(tkb), dmf = __ballot(tkb && (st & kStDel));
        if (dmf && (p4 || ((dmf >> (63 - __clzll(tm))) & 1ull)) && lane == 0)
          atomicOr(A.err, 16);  // a validated reduction left a deleted pivot candidate
        uint32_t oi = RS_NONE;
        if (tm) {
          if (!p4) {
            oi = 63 - __clzll(tm);
          } else {
            unsigned long long vv = tkb ? ((unsigned long long)st << 32) | (0xffffffffu - lane) : ~0ull;
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) {
              const unsigned long long w = __shfl_xor(vv, d);
              vv = w < vv ? w : vv;
            }
            oi = 0xffffffffu - (uint32_t)(vv & 0xffffffffu);
          }
        }
        if (len == 0) {
        } else if (oi == RS_NONE) {  // nothing takeable: leftover (lconst), unnormalised
          uint64_t o = 0;
          if (lane == 0) o = sp_alloc<NW>(A, S, len);
          o = ((uint64_t)rdlane((uint32_t)(o >> 32), 0) << 32) | rdlane((uint32_t)o, 0);
          by += 36ull * len;
          if (o == RS_NONE) {
            if (lane == 0) S.s_ok = 0;
          } else {
            if (lane < len) { A.pk[o + lane] = R.key; A.pv[o + lane] = R.val; }
            if (lane == 0) { A.l_off[b + S.s_nl] = o; A.l_len[b + S.s_nl] = len; S.s_nl = S.s_nl + 1; }
          }
        } else {  // new substitution p = -(work - v_p p) / v_p (clear_signal_not_normalized), header first
          piv = rdlane(R.key, oi);
          const uint32_t psl = rdlane(R.slot, oi);
          const uint32_t sh = rdlane(R.key, 0) == 0 ? 0u : 1u;  // {0: 0} is inserted when absent
          const uint32_t mm = len - 1 + sh;
          const Fe cf = fneg(F, fe_rdlane(R.val, oi));
          by += 36ull * mm;
          uint64_t o = 0;
          if (lane == 0) o = sp_alloc<NW>(A, S, (uint64_t)mm + 1);
          o = ((uint64_t)rdlane((uint32_t)(o >> 32), 0) << 32) | rdlane((uint32_t)o, 0);
          if (o == RS_NONE) {
            if (lane == 0) S.s_ok = 0;
            piv = RS_NONE;
          } else {
            if (lane < len && lane != oi) {
              const uint64_t q = o + 1 + (lane < oi ? lane : lane - 1) + sh;
              A.pk[q] = R.key;
              A.pv[q] = R.val;
            }
            if (lane == 0) {
              if (sh) { A.pk[o + 1] = 0; A.pv[o + 1] = fe_zero(); }
              A.pk[o] = mm;
              A.pv[o] = cf;
              d_set_holder(A, piv, b + S.s_m, cf, o + 1, mm);
              S.s_m = S.s_m + 1;
              A.occ[piv] = -1;
              A.del[piv] = 1;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // the holder before its state
            if (lane == 0 && psl != kTabEmpty) lds_st(&S.tv[psl], kStDel | (uint32_t)o);
          }
        }
      }
      if (lane == 0) {
        lds_st(&S.ring[j % kSpecRing], piv);
        __hip_atomic_store(&S.s_turn, j + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    if (lane == 0) {
      atomicAdd(A.bytes_main, by);
      if (A.prof) {
        atomicAdd(&S.s_prof[0], n_conf);
        atomicAdd(&S.s_prof[1], n_serial);
        atomicAdd(&S.s_prof[2], n_merges);
        atomicAdd(&S.s_prof[3], n_remerges);
      }
    }
    __syncthreads();
    if (tid == 0) {
      A.n_sub[c] = S.s_m;
      A.n_left[c] = S.s_nl;
      if (!S.s_ok) atomicOr(A.err, 8);
      if (A.prof) {
        unsigned long long *P = A.prof + kProfWords * ci;
        // [2] rows, [5] wall, [22] start; [8] conflicts (rows reduced again at their turn), [9] rows
        // finished on lane 0, [10] merges committed, [12] merges thrown away by the conflicts
        P[2] = n_loop;
        P[5] = wall_clock64() - t_1;
        P[22] = t_1;
        P[8] = S.s_prof[0];
        P[9] = S.s_prof[1];
        P[10] = S.s_prof[2];
        P[12] = S.s_prof[3];
      }
    }
    __syncthreads();
  }
}

}  // namespace rs
