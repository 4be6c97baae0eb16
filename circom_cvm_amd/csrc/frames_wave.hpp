// frames_wave.hpp -- the substitution frames on whole waves: the non-linear rows of round 1
// (obtain_and_simplify_non_linear, constraint_simplification.rs:281-325: frames 1-3 =
// Signal / constant / linear substitutions, then fix_constraint, algebra.rs:1279-1324) and the
// storage rows of rounds >= 2 (apply_substitution_to_map, :345-396: frame 3 + fix).
//
// A wave takes 64 consecutive rows (one per lane) and cuts them into batches whose terms fit its LDS
// slice.  A batch's groups are (row, linear combination) pairs -- A, B and C of every row side by
// side -- and the batch runs four stages, each with independent loads unrolled for memory-level
// parallelism:
//   entries  lane-per-entry: each entry classified after frames 1-2 (plain signal, constant -> key 0,
//            substituted -> its right-hand side of h_len terms); scans give every entry its first term
//   terms    lane-per-term: key of every term (substituted entries read their right-hand side's keys
//            with consecutive lanes on consecutive pool entries: coalesced)
//   rank     lane-per-term: a term's position in its group's sorted order = its index in its own run
//            plus, per other run of the group (each run is sorted: a right-hand side or one entry), a
//            binary search; ties between runs broken by run order, so the ranks are a permutation
//            (groups of many runs: pairwise merge rounds, fw_rank_rounds)
//   emit     lane-per-position over the sorted order: every term's value (coefficient x right-hand-
//            side coefficient, Montgomery products), runs of equal keys summed by a segmented scan;
//            output slots from a scan of the run ends, so consecutive lanes write consecutive
//            (key, value) slots of a group: coalesced stores, each output written once
// Sorting the union of the terms and summing equal keys equals the reference's sequence of frames
// (each frame a sort + combine + drop zeros): the per-key sums are the same field elements.
// fix_constraint clears A and B of a row whose A or B is empty; the rows with A or B one constant
// term (C - s * B) or a sum that cancelled to zero -- both rare -- re-run on the lane-per-row kernel.
//
// Rows whose terms or entries exceed a batch go to the lane-per-row kernels (k_nl_fill /
// k_round_fill) through a list; in rounds, the rows whose final A or B is constant or empty -- the
// ones that turn linear -- are listed for k_round_turn, which finds the substitution they turn at.
#pragma once

namespace rs {

#ifndef FW_T
#define FW_T 640
#endif
#ifndef FW_E
#define FW_E 320
#endif
#ifndef FW_OCC
#define FW_OCC 2                           // waves per SIMD the launch bounds ask for
#endif
constexpr uint32_t kFwT = FW_T;           // terms per batch (A, B and C of its rows)
constexpr uint32_t kFwE = FW_E;           // entries per batch
constexpr uint32_t kFwG = 192;            // groups: 64 rows x 3 linear combinations
constexpr uint32_t kFwPT = kFwT / 64;     // terms per lane
constexpr uint32_t kFwPE = kFwE / 64;     // entries per lane
constexpr uint32_t kFwWaves = 4;          // waves per workgroup (each with its own LDS slice)
constexpr uint32_t kFwRunsRank = 8;       // groups of more runs than this rank by merge rounds
#ifndef FW_KB
#define FW_KB 2                            // emit: sorted positions per lane whose loads go together
#endif

struct FrameWaveArgs {
  FrameArgs fr;             // frames 1-2 absent in rounds (eq_rep / ce_has null)
  DRows in[3], out[3];      // A, B, C
  const uint64_t *cap[3];   // k_nl_count / k_round_count capacities (their term counts + staging)
  int cap_by_row;           // caps indexed by row (rounds) or by list position (non-linear pass)
  const uint32_t *ids;      // list position -> row (nullptr: identity)
  uint64_t n;
  uint64_t x0;              // the list positions [x0, n) (the first pass in two halves: a snapshot after each)
  const uint64_t *late;     // non-linear phase 1: rows left for phase 2 (by row), else null
  uint32_t *big;            // out: rows too large for a batch -- positions (non-linear) or rows (rounds)
  unsigned *n_big;
  int round;                // rounds: set touched, list the rows that turn linear
  uint8_t *touched;
  uint32_t *turn_list;
  unsigned *n_turn;
  int *err;                 // a batch over its LDS bounds (cannot happen with consistent caps)
  unsigned long long *bytes;
  unsigned long long *clk;  // RS_FWCLK builds: shader clocks per stage (diagnostic)
};

#ifdef RS_FWCLK
#define FW_CLK(i)                                                                      \
  do {                                                                                 \
    const unsigned long long now_ = clock64();                                         \
    clk_acc[i] += now_ - clk_last;                                                     \
    clk_last = now_;                                                                   \
  } while (0)
#else
#define FW_CLK(i) do { } while (0)
#endif
#ifdef RS_FWCLK
#define FW_WAIT() asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory")
#else
#define FW_WAIT() do { } while (0)
#endif

struct FwLds {
  uint32_t tkey[kFwT];
  uint32_t tsrc[kFwT];      // entry << 10 | position in the entry's run
  uint16_t perm[kFwT];      // sorted position -> term
  uint64_t nzm[kFwPT + 1];  // emit: per 64 sorted positions, the non-zero key heads (ballot)
  uint32_t nzp[kFwPT + 1];  // and the count of non-zero heads before the block
  uint16_t e_t0[kFwE + 1];  // entry -> first term (e_t0[n_entries] = n_terms)
  uint32_t e_key[kFwE];     // plain: the signal after frame 1; constant: that signal; substituted: slot
  uint8_t e_kind[kFwE];     // bits 0-3: kind (fw_operands); 4-5: the part a fix-pass entry reads
  uint8_t e_grp[kFwE];
  uint16_t e_pos[kFwE];     // the entry's position in its group's input row
  uint64_t e_aux[kFwE];     // substituted: pool offset of the right-hand side
  uint16_t g_e0[kFwG + 1];  // group -> first entry / term
  uint16_t g_t0[kFwG + 1];
  uint64_t g_in[kFwG];      // the group's input / output offsets
  uint64_t g_out[kFwG];
  uint32_t g_k0[kFwG];      // the group's first emitted key
  // rows waiting for the fix pass (A or B one constant term), gathered over the wave's batches
  uint64_t fx_off[3][64];   // output offsets of A, B, C
  uint32_t fx_row[64];
  uint32_t fx_cc[64];       // the C region's expansion size: C' goes after it
  uint32_t fx_len[3][64];   // written lengths of A, B, C
  uint8_t fx_other[64];     // 1: C - s * B (A constant), 0: C - s * A
};

__device__ __forceinline__ uint32_t fw_scan(uint32_t x, uint32_t lane) {  // inclusive, over the wave
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d);
    if (lane >= (uint32_t)d) x += y;
  }
  return x;
}
__device__ __forceinline__ uint64_t fw_below(uint32_t lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }
__device__ __forceinline__ uint32_t fw_part(uint32_t g) { return g % 3u; }
__device__ __forceinline__ const uint32_t *fw_ikey(const FrameWaveArgs &A, uint32_t p) {
  return p == 0 ? A.in[0].key : (p == 1 ? A.in[1].key : A.in[2].key);
}
__device__ __forceinline__ const Fe *fw_ival(const FrameWaveArgs &A, uint32_t p) {
  return p == 0 ? A.in[0].val : (p == 1 ? A.in[1].val : A.in[2].val);
}
__device__ __forceinline__ uint32_t *fw_okey(const FrameWaveArgs &A, uint32_t p) {
  return p == 0 ? A.out[0].key : (p == 1 ? A.out[1].key : A.out[2].key);
}
__device__ __forceinline__ Fe *fw_oval(const FrameWaveArgs &A, uint32_t p) {
  return p == 0 ? A.out[0].val : (p == 1 ? A.out[1].val : A.out[2].val);
}
// last index i in [0, n) with a[i] <= x, given a[0] <= x < a[n]
__device__ __forceinline__ uint32_t fw_find(const uint16_t *a, uint32_t n, uint32_t x) {
  uint32_t lo = 0, hi = n;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a[mid] <= x) lo = mid;
    else hi = mid;
  }
  return lo;
}

// Entry kinds (e_kind bits 0-3; bits 4-5: the part the entry reads, for kinds 3 and 4):
//   0 plain      value = coefficient                               (input row of the group's part;
//                in rounds a block of consecutive plain entries: term j = input entry e_pos + j)
//   1 constant   value = coefficient * constant value, key 0       (frame 2)
//   2 substitute value = coefficient * right-hand side entry j     (frame 3, pool at e_aux)
//   3 copy       value = written output entry j                    (fix pass: the final C)
//   4 scaled     value = -(written output entry j) * s             (fix pass: the other of A / B;
//                s = the constant one's single value, at g_in[group] of part 1 - part)
__device__ __forceinline__ uint32_t fw_epart(const FwLds &L, uint32_t e) { return (L.e_kind[e] >> 4) & 3; }

__device__ __forceinline__ uint32_t fw_term_key(const FrameWaveArgs &A, const FwLds &L, uint32_t e, uint32_t j) {
  const uint32_t kd = L.e_kind[e] & 15;
  if (kd == 0) {
    if (j == 0) return L.e_key[e];
    const uint32_t g = L.e_grp[e];
    return fw_ikey(A, fw_part(g))[L.g_in[g] + L.e_pos[e] + j];
  }
  if (kd == 1) return 0u;
  if (kd == 2) return A.fr.pk[L.e_aux[e] + j];
  return fw_okey(A, fw_epart(L, e))[L.e_aux[e] + j];
}
// the operands of term (e, j): its value is c (kinds 0, 3), c * m (1, 2) or -(c * m) (4)
__device__ __forceinline__ void fw_operands(const FrameWaveArgs &A, const FwLds &L, uint32_t e, uint32_t j, Fe &c, Fe &m) {
  const uint32_t kd = L.e_kind[e] & 15, g = L.e_grp[e];
  if (kd <= 2) {
    c = fw_ival(A, fw_part(g))[L.g_in[g] + L.e_pos[e] + (kd == 0 ? j : 0u)];
    if (kd == 1) m = A.fr.ce_val[L.e_key[e]];
    else if (kd == 2) m = A.fr.pv[L.e_aux[e] + j];
  } else {
    const uint32_t pe = fw_epart(L, e);
    c = fw_oval(A, pe)[L.e_aux[e] + j];
    if (kd == 4) m = fw_oval(A, 1 - pe)[L.g_in[g]];
  }
}
__device__ __forceinline__ Fe fw_combine(const FieldP &F, uint32_t kd, const Fe &c, const Fe &m) {
  if (kd == 0 || kd == 3) return c;
  const Fe p = fmul(F, c, m);
  return kd == 4 ? fneg(F, p) : p;
}
// ---- the stages after the entries (shared by the main pass and the fix pass)

// keys of the terms (lane = every 64th term: consecutive lanes on consecutive right-hand-side entries,
// all of a lane's loads in flight together)
__device__ inline void fw_terms(const FrameWaveArgs &A, FwLds &L, uint32_t lane, uint32_t n_e, uint32_t n_t) {
  uint32_t ent[kFwPT], jj[kFwPT], tk[kFwPT];
#pragma unroll
  for (uint32_t k = 0; k < kFwPT; ++k) {
    const uint32_t t = lane + 64 * k;
    ent[k] = 0;
    jj[k] = 0;
    if (t < n_t) {
      ent[k] = L.perm[t];  // term -> entry, scattered by the entries' lanes (perm is free until fw_rank)
      jj[k] = t - L.e_t0[ent[k]];
    }
  }
#pragma unroll
  for (uint32_t k = 0; k < kFwPT; ++k) tk[k] = lane + 64 * k < n_t ? fw_term_key(A, L, ent[k], jj[k]) : 0u;
#pragma unroll
  for (uint32_t k = 0; k < kFwPT; ++k) {
    const uint32_t t = lane + 64 * k;
    if (t < n_t) {
      L.tkey[t] = tk[k];
      L.tsrc[t] = (ent[k] << 10) | jj[k];
    }
  }
}

// position of every term in its group's sorted order (lane = term): its index in its own run plus,
// per other run of the group (each run sorted), a binary search; ties broken by run order
__device__ inline void fw_rank(FwLds &L, uint32_t lane, uint32_t n_t) {
  for (uint32_t t = lane; t < n_t; t += 64) {
    const uint32_t key = L.tkey[t], src = L.tsrc[t], e = src >> 10, g = L.e_grp[e];
    uint32_t rank = src & 1023;
    const uint32_t eb = L.g_e0[g], ee = L.g_e0[g + 1];
    for (uint32_t e2 = eb; e2 < ee; ++e2) {
      if (e2 == e) continue;
      uint32_t a = L.e_t0[e2], b = L.e_t0[e2 + 1];
      const uint32_t lo = a;
      if (b - a == 1) {  // a single-term run (a plain or constant entry)
        const uint32_t k2 = L.tkey[a];
        rank += (e2 < e) ? (k2 <= key) : (k2 < key);
        continue;
      }
      if (e2 < e) {  // earlier runs precede on equal keys
        while (a < b) {
          const uint32_t m = (a + b) >> 1;
          if (L.tkey[m] <= key) a = m + 1;
          else b = m;
        }
      } else {
        while (a < b) {
          const uint32_t m = (a + b) >> 1;
          if (L.tkey[m] < key) a = m + 1;
          else b = m;
        }
      }
      rank += a - lo;
    }
    L.perm[L.g_t0[g] + rank] = (uint16_t)t;
  }
}

// The same ranks by pairwise merge rounds, for groups of many runs (fw_rank costs a binary search per
// other run and term): in round r every segment of 2^r consecutive runs of a group is sorted, and each
// pair of neighbouring segments merges -- a term's place in the merged segment is its offset in its own
// plus, in the partner segment, the count of keys below it (the left segment first on equal keys).
// Segments keep the position ranges of their runs, so only the keys move (registers -> LDS each round);
// ceil(log2 runs) rounds of one search each.
__device__ inline void fw_rank_rounds(FwLds &L, uint32_t lane, uint32_t n_t, uint32_t rounds) {
  uint32_t key[kFwPT], q[kFwPT];
#pragma unroll
  for (uint32_t k = 0; k < kFwPT; ++k) {
    const uint32_t t = lane + 64 * k;
    key[k] = t < n_t ? L.tkey[t] : 0u;
    q[k] = t;
  }
  for (uint32_t r = 0; r < rounds; ++r) {
    uint32_t nq[kFwPT];
#pragma unroll
    for (uint32_t k = 0; k < kFwPT; ++k) {
      const uint32_t t = lane + 64 * k;
      nq[k] = q[k];
      if (t >= n_t) continue;
      const uint32_t e = L.tsrc[t] >> 10, g = L.e_grp[e], e0 = L.g_e0[g], R = L.g_e0[g + 1] - e0, i = e - e0;
      const uint32_t S = i >> r, P = S ^ 1u;
      if ((P << r) >= R) continue;  // no partner segment this round
      uint32_t a = L.e_t0[e0 + (P << r)], b = L.e_t0[e0 + min((P + 1) << r, R)];
      const uint32_t os = L.e_t0[e0 + (S << r)], ms = L.e_t0[e0 + ((S & ~1u) << r)], lo = a;
      if (S < P) {  // left: partner keys below
        while (a < b) {
          const uint32_t mid = (a + b) >> 1;
          if (L.tkey[mid] < key[k]) a = mid + 1; else b = mid;
        }
      } else {      // right: partner keys up to and including
        while (a < b) {
          const uint32_t mid = (a + b) >> 1;
          if (L.tkey[mid] <= key[k]) a = mid + 1; else b = mid;
        }
      }
      nq[k] = ms + (q[k] - os) + (a - lo);
    }
    wave_sync();
#pragma unroll
    for (uint32_t k = 0; k < kFwPT; ++k) {
      if (lane + 64 * k < n_t) L.tkey[nq[k]] = key[k];
      q[k] = nq[k];
    }
    wave_sync();
  }
#pragma unroll
  for (uint32_t k = 0; k < kFwPT; ++k) {
    const uint32_t t = lane + 64 * k;
    if (t < n_t) {
      L.tkey[t] = key[k];  // back to term order (emit reads keys by term)
      L.perm[q[k]] = (uint16_t)t;
    }
  }
}

// non-zero key heads before sorted position q (from the emit ballots)
__device__ __forceinline__ uint32_t fw_nz_before(const FwLds &L, uint32_t q) {
  return L.nzp[q >> 6] + (uint32_t)__popcll(L.nzm[q >> 6] & fw_below(q & 63));
}
__device__ __forceinline__ uint32_t fw_glen(const FwLds &L, uint32_t g) {
  return fw_nz_before(L, L.g_t0[g + 1]) - fw_nz_before(L, L.g_t0[g]);
}

// Emit (lane = every 64th sorted position: consecutive lanes write consecutive slots).  Every position
// computes its term's value (all of a block's loads in flight together); a run of equal keys is summed
// by a segmented scan over the block's 64 lanes (a carry moves a run on into the next block), so a key
// that many right-hand sides share costs log 64 steps, not a serial walk of its run.  The last position
// of a run emits the sum unless it is zero -- the pool keeps the zero-valued entries of the reference's
// maps ({0: 0} from initialize_hashmap_for_expression, algebra.rs:1279-1294, and cancellations), so
// zero sums are common.  Output slots: ballots of the emitting positions per 64 positions (nzm) and
// their running count (nzp).
__device__ inline void fw_emit(const FrameWaveArgs &A, FwLds &L, uint32_t lane, uint32_t n_t
#ifdef RS_FWCLK
                               , unsigned long long *clk_acc, unsigned long long &clk_last
#endif
) {
  const FieldP &F = A.fr.F;
  constexpr uint32_t kB = FW_KB;
  static_assert(kFwPT % kB == 0, "emit blocks");
  uint32_t before = 0;  // emitted positions in the blocks done
  Fe carry = fe_zero();  // the running sum of a run that goes on past the block before
#pragma unroll
  for (uint32_t kb = 0; kb < kFwPT; kb += kB) {
    Fe c[kB], m[kB];
    uint32_t key[kB], kd[kB], gg[kB], fl[kB];  // fl: bit 0 valid, 1 run start, 2 run end
#pragma unroll
    for (uint32_t k = 0; k < kB; ++k) {
      const uint32_t p = lane + 64 * (kb + k);
      fl[k] = 0;
      kd[k] = 0;
      key[k] = 0;
      gg[k] = 0;
      if (p < n_t) {
        const uint32_t t = L.perm[p], src = L.tsrc[t], e = src >> 10, g = L.e_grp[e];
        key[k] = L.tkey[t];
        gg[k] = g;
        const bool st = p == L.g_t0[g] || L.tkey[L.perm[p - 1]] != key[k];
        const bool en = p + 1 == L.g_t0[g + 1] || L.tkey[L.perm[p + 1]] != key[k];
        fl[k] = 1u | (st ? 2u : 0u) | (en ? 4u : 0u);
        kd[k] = L.e_kind[e] & 15;
        fw_operands(A, L, e, src & 1023, c[k], m[k]);
      }
    }
    FW_WAIT();
    FW_CLK(16);
    uint64_t nz[kB];
    // one block's sums; written out per slot (not a loop) so the arrays stay in registers
    auto sums = [&](Fe &v, const Fe &mv, uint32_t kdv, uint32_t f) -> uint64_t {
      v = (f & 1) ? fw_combine(F, kdv, v, mv) : fe_zero();
      if (lane == 0 && (f & 3) == 1) v = fadd(F, v, carry);
      if (__ballot(lane > 0 && (f & 3) == 1)) {  // a run crosses lanes: segmented inclusive scan
        bool hd = (f & 3) != 1;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          Fe y;
#pragma unroll
          for (int w = 0; w < 4; ++w) y.l[w] = __shfl_up(v.l[w], d);
          const bool yh = __shfl_up(hd ? 1 : 0, d) != 0;
          if ((int)lane >= d) {
            if (!hd) v = fadd(F, v, y);
            hd = hd || yh;
          }
        }
      }
#pragma unroll
      for (int w = 0; w < 4; ++w) carry.l[w] = __shfl(v.l[w], 63);
      return __ballot((f & 5) == 5 && !fe_is_zero(v));
    };
    static_assert(kB <= 5, "sums() is applied to at most five slots");
#define FW_SUMS(i) \
  if constexpr (kB > i) nz[i] = sums(c[i], m[i], kd[i], fl[i]);
    FW_SUMS(0) FW_SUMS(1) FW_SUMS(2) FW_SUMS(3) FW_SUMS(4)
#undef FW_SUMS
#pragma unroll
    for (uint32_t k = 0; k < kB; ++k) {
      if (lane == 0) {
        L.nzm[kb + k] = nz[k];
        L.nzp[kb + k] = before;
      }
      before += (uint32_t)__popcll(nz[k]);
    }
    FW_CLK(17);
    wave_sync();
    FW_CLK(18);
#pragma unroll
    for (uint32_t k = 0; k < kB; ++k) {
      if (!((nz[k] >> lane) & 1)) continue;
      const uint32_t g = gg[k];
      const uint32_t at = L.nzp[kb + k] + (uint32_t)__popcll(nz[k] & fw_below(lane)), g0 = fw_nz_before(L, L.g_t0[g]);
      const uint64_t o = L.g_out[g] + (at - g0);
      const uint32_t part = fw_part(g);
      fw_okey(A, part)[o] = key[k];
      fw_oval(A, part)[o] = c[k];
      if (at == g0) L.g_k0[g] = key[k];
    }
    FW_WAIT();
    FW_CLK(19);
  }
  if (lane == 0) {
    L.nzp[kFwPT] = before;
    L.nzm[kFwPT] = 0;
  }
}

#ifdef RS_FWCLK
#define FW_EMIT(n_t) fw_emit(A, L, lane, n_t, clk_acc, clk_last)
#else
#define FW_EMIT(n_t) fw_emit(A, L, lane, n_t)
#endif

// sets e_t0 (n_e entries, the lane's weights w[] for entries lane * per + k) and g_t0; returns n_terms
template <uint32_t kPer>
__device__ inline uint32_t fw_starts(FwLds &L, uint32_t lane, uint32_t n_e, const uint32_t (&w)[kPer]) {
  uint32_t sum = 0;
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k) sum += w[k];
  const uint32_t incl = fw_scan(sum, lane);
  uint32_t run = incl - sum;
  const uint32_t n_t = __shfl(incl, 63);
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k) {
    const uint32_t e = lane * kPer + k;
    if (e < n_e) {
      L.e_t0[e] = (uint16_t)run;
      if (n_t <= kFwT)
        for (uint32_t t = run; t < run + w[k]; ++t) L.perm[t] = (uint16_t)e;
    }
    run += w[k];
  }
  if (lane == 63 && n_t <= kFwT) L.e_t0[n_e] = (uint16_t)n_t;
  wave_sync();
  for (uint32_t g = lane; g <= kFwG; g += 64) L.g_t0[g] = L.e_t0[L.g_e0[g]];
  return n_t;
}

// ---- fix pass: C' = C - s * other (fix_constraint with constant_linear_linear_reduction,
// algebra.rs:1309-1344) for the n queued rows (lane = queued row), through the same stages: per row
// one group of two sorted runs, the written C and the written other scaled by -s.  C' goes after the C
// region's expansion part; A and B are cleared.
__device__ inline void fw_fix(const FrameWaveArgs &A, FwLds &L, uint32_t lane, uint32_t n, unsigned long long &bytes
#ifdef RS_FWCLK
                              , unsigned long long *clk_acc, unsigned long long &clk_last
#endif
) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the queued rows were written by this wave
  wave_sync();
  const bool on = lane < n;
  const uint32_t other = on ? L.fx_other[lane] : 0u;
  const uint32_t lc = on ? L.fx_len[2][lane] : 0u, lo = on ? L.fx_len[other][lane] : 0u;
  const uint32_t fe = on ? 2u : 0u, fincl = fw_scan(fe, lane), f0 = fincl - fe, nf = __shfl(fincl, 63);
  const uint32_t tw = lc + lo, tincl = fw_scan(tw, lane), t0 = tincl - tw, nft = __shfl(tincl, 63);
  {
    const uint32_t g = 3 * lane;
    L.g_e0[g] = L.g_e0[g + 1] = L.g_e0[g + 2] = (uint16_t)f0;
    if (lane == 63) {
      L.g_e0[kFwG] = (uint16_t)nf;
      L.e_t0[nf] = (uint16_t)nft;
    }
    L.g_k0[g + 2] = RS_NONE;
    if (on) {
      L.g_out[g + 2] = L.fx_off[2][lane] + L.fx_cc[lane];
      L.g_in[g + 2] = L.fx_off[1 - other][lane];  // s: the constant part's single entry
      L.e_grp[f0] = L.e_grp[f0 + 1] = (uint8_t)(g + 2);
      L.e_kind[f0] = (uint8_t)(3 | (2 << 4));
      L.e_aux[f0] = L.fx_off[2][lane];
      L.e_kind[f0 + 1] = (uint8_t)(4 | (other << 4));
      L.e_aux[f0 + 1] = L.fx_off[other][lane];
      L.e_t0[f0] = (uint16_t)t0;
      L.e_t0[f0 + 1] = (uint16_t)(t0 + lc);
      for (uint32_t t = t0; t < t0 + lc; ++t) L.perm[t] = (uint16_t)f0;
      for (uint32_t t = t0 + lc; t < t0 + lc + lo; ++t) L.perm[t] = (uint16_t)(f0 + 1);
    }
  }
  wave_sync();
  for (uint32_t g = lane; g <= kFwG; g += 64) L.g_t0[g] = L.e_t0[L.g_e0[g]];
  fw_terms(A, L, lane, nf, nft);
  wave_sync();
  fw_rank(L, lane, nft);
  wave_sync();
  FW_EMIT(nft);
  wave_sync();
  if (on) {
    const uint32_t r = L.fx_row[lane], len = fw_glen(L, 3 * lane + 2);
    A.out[0].len[r] = 0;
    A.out[1].len[r] = 0;
    A.out[2].off[r] = L.fx_off[2][lane] + L.fx_cc[lane];
    A.out[2].len[r] = len;
    bytes += 36ull * (L.fx_len[0][lane] + L.fx_len[1][lane] + lc + lo + len);
    if (A.round) {  // fix_constraint cleared A and B: the row turns linear this round
      const unsigned pos = atomicAdd(A.n_turn, 1u);
      A.turn_list[pos] = r;
    }
  }
  wave_sync();
}

#ifdef RS_FWCLK
#define FW_CLK_ARGS , clk_acc, clk_last
#else
#define FW_CLK_ARGS
#endif

// One batch: rows [s, e) of the wave's 64 (lane = row in the row stages); ioff / ooff: the row's
// input / output offsets of A, B, C; cc: the size of its C region's expansion part (fix pass output
// goes after it).
__device__ inline void fw_batch(const FrameWaveArgs &A, FwLds &L, uint32_t lane, bool inb, uint64_t r, const uint32_t ln[3],
                                const uint64_t ioff[3], const uint64_t ooff[3], uint32_t cc, uint64_t x_of_row,
                                uint32_t &fx_n, uint32_t &fx_terms, unsigned long long &bytes
#ifdef RS_FWCLK
                                , unsigned long long *clk_acc
#endif
) {
#ifdef RS_FWCLK
  unsigned long long clk_last = clock64();
#endif
  // ---- groups (lane = row)
  const uint32_t n0 = inb ? ln[0] : 0, n1 = inb ? ln[1] : 0, n2 = inb ? ln[2] : 0;
  const uint32_t tot = n0 + n1 + n2, incl = fw_scan(tot, lane), ex = incl - tot;
  uint32_t n_e = __shfl(incl, 63);  // entries (rounds: after the plain blocks are merged)
  if (n_e > kFwE) {
    if (lane == 0) atomicOr(A.err, 8);
    return;
  }
  {
    const uint32_t g = 3 * lane;
    L.g_e0[g] = (uint16_t)ex;
    L.g_e0[g + 1] = (uint16_t)(ex + n0);
    L.g_e0[g + 2] = (uint16_t)(ex + n0 + n1);
    if (lane == 63) L.g_e0[kFwG] = (uint16_t)n_e;
    L.g_k0[g] = L.g_k0[g + 1] = L.g_k0[g + 2] = RS_NONE;
    for (uint32_t q = 0; q < tot; ++q) L.e_grp[ex + q] = (uint8_t)(g + (q >= n0) + (q >= n0 + n1));
    if (inb) {
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        L.g_in[g + p] = ioff[p];
        L.g_out[g + p] = ooff[p];
      }
    }
  }
  wave_sync();
  FW_CLK(0);
  // ---- entries (lane = its kFwPE consecutive entries; the loads of the lane's entries in flight together)
  uint32_t rhs_terms = 0, w[kFwPE];
  {
    uint32_t key[kFwPE], k1[kFwPE], kind[kFwPE], ek[kFwPE];
    uint64_t aux[kFwPE];
#pragma unroll
    for (uint32_t k = 0; k < kFwPE; ++k) {
      const uint32_t e = lane * kFwPE + k;
      key[k] = 0;
      if (e < n_e) {
        const uint32_t g = L.e_grp[e];
        key[k] = fw_ikey(A, fw_part(g))[L.g_in[g] + (e - L.g_e0[g])];
      }
    }
#pragma unroll
    for (uint32_t k = 0; k < kFwPE; ++k) {
      const int32_t t1 = (A.fr.eq_rep && lane * kFwPE + k < n_e) ? A.fr.eq_rep[key[k]] : -1;
      k1[k] = t1 >= 0 ? (uint32_t)t1 : key[k];
    }
#pragma unroll
    for (uint32_t k = 0; k < kFwPE; ++k) {
      const bool v = lane * kFwPE + k < n_e;
      // both loads issued together (a constant signal is never substituted: sub_of is read anyway)
      const bool ce = v && A.fr.ce_has && A.fr.ce_has[k1[k]];
      const int32_t sl0 = v ? A.fr.sub_of[k1[k]] : -1;
      const int32_t sl = ce ? -1 : sl0;
      kind[k] = ce ? 1u : (sl >= 0 ? 2u : 0u);
      ek[k] = sl >= 0 ? (uint32_t)sl : k1[k];
      w[k] = v ? 1u : 0u;
    }
#pragma unroll
    for (uint32_t k = 0; k < kFwPE; ++k) {
      aux[k] = 0;
      if (kind[k] == 2) {
        aux[k] = A.fr.h_off[ek[k]];
        w[k] = A.fr.h_len[ek[k]];
        rhs_terms += w[k];
      }
    }
    uint32_t pos[kFwPE], grp[kFwPE];
#pragma unroll
    for (uint32_t k = 0; k < kFwPE; ++k) {
      const uint32_t e = lane * kFwPE + k;
      grp[k] = e < n_e ? L.e_grp[e] : 0u;
      pos[k] = e < n_e ? e - L.g_e0[grp[k]] : 0u;
    }
    if (A.round) {
      // Rounds: the entries the round does not substitute are most of a storage row, and the row's keys
      // are sorted and distinct -- so each maximal block of consecutive plain entries of a group is ONE
      // sorted run (term j = input entry e_pos + j).  The rank stage then searches one run per block
      // and per substituted entry instead of one per entry.  A plain entry right after a plain entry of
      // its group (pos != 0) joins that block; the kept entries are renumbered densely.
      const uint32_t prev_kind = __shfl_up(kind[kFwPE - 1], 1);
      uint32_t keep[kFwPE], cnt = 0;
#pragma unroll
      for (uint32_t k = 0; k < kFwPE; ++k) {
        const uint32_t e = lane * kFwPE + k;
        const uint32_t pk = k ? kind[k - 1] : prev_kind;
        keep[k] = (e < n_e && !(kind[k] == 0 && pos[k] != 0 && pk == 0)) ? 1u : 0u;
        cnt += keep[k];
      }
      const uint32_t incl = fw_scan(cnt, lane);
      uint32_t ni[kFwPE], run = incl - cnt;
      const uint32_t n_e2 = __shfl(incl, 63);
#pragma unroll
      for (uint32_t k = 0; k < kFwPE; ++k) {
        ni[k] = run;
        run += keep[k];
      }
      // scratch until fw_starts: perm = kept entry -> original index, e_t0 = original -> kept index
      wave_sync();
#pragma unroll
      for (uint32_t k = 0; k < kFwPE; ++k) {
        const uint32_t e = lane * kFwPE + k;
        if (keep[k]) {
          L.perm[ni[k]] = (uint16_t)e;
          L.e_t0[e] = (uint16_t)ni[k];
        }
      }
      if (lane == 63) {
        L.perm[n_e2] = (uint16_t)n_e;
        L.e_t0[n_e] = (uint16_t)n_e2;
      }
      wave_sync();
#pragma unroll
      for (uint32_t k = 0; k < kFwPE; ++k)  // a block's length: up to the next kept entry (a group's first is kept)
        if (keep[k] && kind[k] == 0) w[k] = (uint32_t)L.perm[ni[k] + 1] - (lane * kFwPE + k);
      uint32_t ge[(kFwG + 64) / 64];
#pragma unroll
      for (uint32_t q = 0; q < (kFwG + 64) / 64; ++q) {
        const uint32_t g = lane + 64 * q;
        ge[q] = g <= kFwG ? L.e_t0[L.g_e0[g]] : 0u;
      }
      wave_sync();
#pragma unroll
      for (uint32_t q = 0; q < (kFwG + 64) / 64; ++q) {
        const uint32_t g = lane + 64 * q;
        if (g <= kFwG) L.g_e0[g] = (uint16_t)ge[q];
      }
#pragma unroll
      for (uint32_t k = 0; k < kFwPE; ++k) {
        if (!keep[k]) continue;
        const uint32_t d = ni[k];
        L.e_key[d] = ek[k];
        L.e_kind[d] = (uint8_t)kind[k];
        L.e_aux[d] = aux[k];
        L.e_grp[d] = (uint8_t)grp[k];
        L.e_pos[d] = (uint16_t)pos[k];
        L.perm[d] = (uint16_t)w[k];
      }
      wave_sync();
#pragma unroll
      for (uint32_t k = 0; k < kFwPE; ++k) {
        const uint32_t d = lane * kFwPE + k;
        w[k] = d < n_e2 ? (uint32_t)L.perm[d] : 0u;
      }
      wave_sync();
      n_e = n_e2;
    } else {
#pragma unroll
      for (uint32_t k = 0; k < kFwPE; ++k) {
        const uint32_t e = lane * kFwPE + k;
        if (e < n_e) {
          L.e_key[e] = ek[k];
          L.e_kind[e] = (uint8_t)kind[k];
          L.e_aux[e] = aux[k];
          L.e_pos[e] = (uint16_t)pos[k];
        }
      }
    }
  }
  const uint32_t n_t = fw_starts<kFwPE>(L, lane, n_e, w);
  if (n_t > kFwT) {
    if (lane == 0) atomicOr(A.err, 8);
    return;
  }
  bytes += 36ull * rhs_terms + (inb ? 36ull * tot + 72 : 0);  // right-hand sides read by this lane's entries
  FW_CLK(1);
  fw_terms(A, L, lane, n_e, n_t);
  wave_sync();
  FW_CLK(2);
  uint32_t rmax = 0;  // the most runs in one group of the batch
  if (inb) {
    const uint32_t g = 3 * lane;
    rmax = max((uint32_t)(L.g_e0[g + 1] - L.g_e0[g]), max((uint32_t)(L.g_e0[g + 2] - L.g_e0[g + 1]), (uint32_t)(L.g_e0[g + 3] - L.g_e0[g + 2])));
  }
  rmax = ~wave_min_u32(~rmax);  // the wave's maximum (DPP)
  if (rmax > kFwRunsRank) {
    uint32_t rounds = 0;
    while ((1u << rounds) < rmax) ++rounds;
    fw_rank_rounds(L, lane, n_t, rounds);
  } else {
    fw_rank(L, lane, n_t);
  }
  wave_sync();
  FW_CLK(3);
  FW_EMIT(n_t);
  wave_sync();
  FW_CLK(5);
  // ---- per row (lane = row): lengths and fix_constraint (algebra.rs:1309-1324)
  uint32_t len[3] = {0, 0, 0};
  int other = -1;  // fix: A (other = 1: C - s * B) or B (other = 0: C - s * A) is one constant term s
  if (inb) {
    const uint32_t g = 3 * lane;
#pragma unroll
    for (uint32_t p = 0; p < 3; ++p) len[p] = fw_glen(L, g + p);
    const bool ca = len[0] == 1 && L.g_k0[g] == 0;
    const bool cb = len[1] == 1 && L.g_k0[g + 1] == 0;
    const bool clear = len[0] == 0 || len[1] == 0;
    if (!clear && (ca || cb)) {
      other = ca ? 1 : 0;
    } else {
      if (clear) len[0] = len[1] = 0;
#pragma unroll
      for (int p = 0; p < 3; ++p) A.out[p].len[r] = len[p];
      bytes += 36ull * (len[0] + len[1] + len[2]);
      // the final A or B was empty (fix_constraint cleared both): the row turns linear this round
      if (A.round && clear) {
        const unsigned pos = atomicAdd(A.n_turn, 1u);
        A.turn_list[pos] = (uint32_t)r;
      }
    }
  }
  // ---- rows with a constant A or B wait for the fix pass (fw_fix), which runs once enough gathered
  const uint64_t fm = __ballot(other >= 0);
  if (fm) {
    const uint32_t nfix = (uint32_t)__popcll(fm);
    const uint32_t tw = other >= 0 ? len[2] + len[other] : 0u, tsum = __shfl(fw_scan(tw, lane), 63);
    if (fx_n + nfix > 64 || fx_terms + tsum > kFwT) {
      fw_fix(A, L, lane, fx_n, bytes FW_CLK_ARGS);
      fx_n = 0;
      fx_terms = 0;
    }
    if (other >= 0) {
      const uint32_t q = fx_n + (uint32_t)__popcll(fm & fw_below(lane));
      L.fx_row[q] = (uint32_t)r;
      L.fx_cc[q] = cc;
      L.fx_other[q] = (uint8_t)other;
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        L.fx_off[p][q] = ooff[p];
        L.fx_len[p][q] = len[p];
      }
    }
    fx_n += nfix;
    fx_terms += tsum;
  }
  (void)x_of_row;
  wave_sync();
  FW_CLK(6);
}

// kRound: 0 = the non-linear rows of round 1, 1 = the storage rows of rounds >= 2 (separate symbols so
// profiles tell the two apart)
template <int kRound>
__global__ __launch_bounds__(256, FW_OCC) void k_frames_wave(FrameWaveArgs A) {
  __shared__ FwLds lds[kFwWaves];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  FwLds &L = lds[wv];
  unsigned long long bytes = 0;
#ifdef RS_FWCLK
  unsigned long long clk_last = clock64(), clk_k0 = clk_last, clk_acc[20] = {};
#endif
  const uint64_t nw = (uint64_t)gridDim.x * kFwWaves;
  uint32_t fx_n = 0, fx_terms = 0;  // the fix-pass queue (uniform)
  for (uint64_t base = A.x0 + ((uint64_t)blockIdx.x * kFwWaves + wv) * 64; base < A.n; base += nw * 64) {
    const uint64_t x = base + lane;
    bool act = x < A.n;
    uint64_t r = 0, ioff[3] = {0, 0, 0}, ooff[3] = {0, 0, 0};
    uint32_t ln[3] = {0, 0, 0}, wt = 0, cc = 0;
    if (act) {
      r = A.ids ? A.ids[x] : x;
      // every per-row load in flight together (the skip flag, the capacities, lengths, offsets)
      const bool late = A.late && A.late[r];
      const uint64_t ci = A.cap_by_row ? r : x;
      const uint64_t ca = A.cap[0][ci], cb = A.cap[1][ci], cc2 = A.cap[2][ci];
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        ln[p] = A.in[p].len[r];
        ioff[p] = A.in[p].off[r];
        ooff[p] = A.out[p].off[r];
      }
      if (late) {
        act = false;
      } else {
        if (A.round) A.touched[r] = 1;
        const uint64_t mx = ca > cb ? ca : cb, c3 = (cc2 - mx) / 2;
        cc = (uint32_t)c3;
        // terms of A, B, C: the capacities less the staging slots
        const uint64_t t = (ca - 1 - ln[0]) + (cb - 1 - ln[1]) + (c3 - 1 - ln[2]);
        if (t > kFwT || (uint64_t)ln[0] + ln[1] + ln[2] > kFwE) {
          const unsigned pos = atomicAdd(A.n_big, 1u);
          A.big[pos] = (uint32_t)(A.cap_by_row ? r : x);
          act = false;
        } else {
          wt = (uint32_t)t;
        }
      }
    }
    if (!act) ln[0] = ln[1] = ln[2] = 0;
    FW_CLK(7);
    // batches: the longest runs of rows whose terms and entries fit
    const uint32_t P = fw_scan(wt, lane), Q = fw_scan(ln[0] + ln[1] + ln[2], lane);
    uint32_t s = 0;
    while (s < 64) {
      const uint32_t bp = s ? __shfl(P, s - 1) : 0, bq = s ? __shfl(Q, s - 1) : 0;
      const uint64_t bad = __ballot(lane >= s && (P - bp > kFwT || Q - bq > kFwE));
      const uint32_t e = bad ? (uint32_t)__builtin_ctzll(bad) : 64u;
      const bool inb = act && lane >= s && lane < e;
#ifdef RS_FWCLK
      if (__ballot(inb)) fw_batch(A, L, lane, inb, r, ln, ioff, ooff, cc, x, fx_n, fx_terms, bytes, clk_acc);
      clk_last = clock64();
      clk_acc[8] += 1;
#else
      if (__ballot(inb)) fw_batch(A, L, lane, inb, r, ln, ioff, ooff, cc, x, fx_n, fx_terms, bytes);
#endif
      s = e;
    }
  }
  if (fx_n) {
#ifdef RS_FWCLK
    unsigned long long clk_last2 = clock64();
    fw_fix(A, L, lane, fx_n, bytes, clk_acc, clk_last2);
#else
    fw_fix(A, L, lane, fx_n, bytes);
#endif
  }
#ifdef RS_FWCLK
  clk_acc[9] = clock64() - clk_k0;
  clk_acc[10] = 1;
  if (lane == 0 && A.clk)
    for (int i = 0; i < 20; ++i) atomicAdd(A.clk + i, clk_acc[i]);
#endif
  wave_atomic_add(A.bytes, bytes);
}

}  // namespace rs
