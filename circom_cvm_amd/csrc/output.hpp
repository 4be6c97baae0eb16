// output.hpp -- row extents of the result and the streamed D2H of rs_engine_simplify (ABI 8 layout).
//
// The result is the storage rows in storage order, then the linear rows the rounds left, then the
// host-side lconst rows (constraint_simplification.rs:648-729).  A storage row is final once round
// 1's substitution has run on it (non_linear_utils.rs:6-31) unless a later round's substitution
// touches it (:613-646; in the metric circuit 8 % of the rows).  So as soon as the first frames pass
// is done, its storage rows ("early") are gathered to an early region and copied to the host on the
// copy stream while the head's rows, the later rounds and the final assembly run; at the end only
// the rows that are not early, or that a round touched after all ("dirty"), are gathered after the
// early region, and every output row is given as [beg, end) into [early | late].  Included by
// engine.hip inside namespace rs, after U3.
#pragma once

__device__ __forceinline__ uint64_t u3_sel(const U3 &x, int q) { return q == 0 ? x.a : (q == 1 ? x.b : x.c); }

// The gathers of a snapshot run on the copy stream while the main stream goes on and may re-point
// rows (the second pass, the rounds): they read a copy of the selected rows' views, which the kernel
// that selects them writes (the other rows' entries are left as they were).
struct ViewCopy {
  uint64_t *off[3];
  uint32_t *len[3];
};
__device__ __forceinline__ void view_copy(const ViewCopy &v, const DRows &a, const DRows &b, const DRows &c, uint64_t i,
                                          uint32_t la, uint32_t lb, uint32_t lc) {
  v.off[0][i] = a.off[i];
  v.off[1][i] = b.off[i];
  v.off[2][i] = c.off[i];
  v.len[0][i] = la;
  v.len[1][i] = lb;
  v.len[2][i] = lc;
}

// early[i]: non-linear row i is done (not left to a second pass) and stayed non-linear -- a
// storage row (non_linear_utils.rs:6-31: A or B non-empty); elen[i]: its part lengths (0
// when not early).  Sharded: only the rows [lo, hi) this rank copies to the host count.
__global__ void k_snap_flags(DRows a, DRows b, DRows c, const uint64_t *late, uint64_t n, uint64_t lo, uint64_t hi, uint8_t *early,
                             U3 *elen, ViewCopy vc) {
  for (uint64_t i = gtid(); i < n; i += gstride()) {
    const bool done = (!late || !late[i]) && i >= lo && i < hi;
    const uint32_t la = done ? a.len[i] : 0, lb = done ? b.len[i] : 0, lc = done ? c.len[i] : 0;
    const bool ok = (la | lb) != 0;  // k_flag_linear: linear iff A and B are both empty
    early[i] = ok ? 1 : 0;
    elen[i] = ok ? U3{la, lb, lc} : U3{0, 0, 0};
    if (ok) view_copy(vc, a, b, c, i, la, lb, lc);
  }
}

// The second snapshot: the rows the second frames pass did (late[i]) that stayed storage rows --
// elen[i] their part lengths (else 0); once they fit behind the first snapshot, k_snap_mark2 makes
// them early at base + their offsets.
__global__ void k_snap_lens2(DRows a, DRows b, DRows c, const uint64_t *late, uint64_t n, U3 *elen, ViewCopy vc) {
  for (uint64_t i = gtid(); i < n; i += gstride()) {
    const bool ok = late[i] && (a.len[i] | b.len[i]) != 0;
    elen[i] = ok ? U3{a.len[i], b.len[i], c.len[i]} : U3{0, 0, 0};
    if (ok) view_copy(vc, a, b, c, i, a.len[i], b.len[i], c.len[i]);
  }
}
__global__ void k_snap_mark2(const uint64_t *late, const U3 *elen, const U3 *eoff2, U3 base, uint64_t n, uint8_t *early,
                             U3 *eoff) {
  for (uint64_t i = gtid(); i < n; i += gstride()) {
    if (!late[i] || (elen[i].a | elen[i].b) == 0) continue;
    early[i] = 1;
    eoff[i] = U3{base.a + eoff2[i].a, base.b + eoff2[i].b, base.c + eoff2[i].c};
  }
}

// The first pass in two halves (single engine): the second half's rows [lo, hi) that are done and
// stayed storage rows -- elen[i] their part lengths (else 0); k_snap_mark_sel makes every row with
// lengths early at base + its offset.
__global__ void k_snap_lens_rng(DRows a, DRows b, DRows c, const uint64_t *late, uint64_t lo, uint64_t hi, uint64_t n, U3 *elen,
                                ViewCopy vc) {
  for (uint64_t i = gtid(); i < n; i += gstride()) {
    const bool ok = i >= lo && i < hi && !(late && late[i]) && (a.len[i] | b.len[i]) != 0;
    elen[i] = ok ? U3{a.len[i], b.len[i], c.len[i]} : U3{0, 0, 0};
    if (ok) view_copy(vc, a, b, c, i, a.len[i], b.len[i], c.len[i]);
  }
}
__global__ void k_snap_mark_sel(const U3 *elen, const U3 *eoff2, U3 base, uint64_t n, uint8_t *early, U3 *eoff) {
  for (uint64_t i = gtid(); i < n; i += gstride()) {
    if ((elen[i].a | elen[i].b) == 0) continue;
    early[i] = 1;
    eoff[i] = U3{base.a + eoff2[i].a, base.b + eoff2[i].b, base.c + eoff2[i].c};
  }
}

// the early rows of one part, canonical, at their early-region offsets (R: a copy of the row views
// taken at the snapshot, so later rounds may move the rows meanwhile; only: the second snapshot's
// rows, else every early row; rows below lo are skipped -- the first pass's second half)
__global__ void k_snap_gather(FieldP F, DRows R, const uint8_t *early, const U3 *eoff, int q, uint64_t n, uint32_t *col,
                              uint64_t *val, const uint64_t *only, uint64_t lo) {
  for (uint64_t r = lo + gtid(); r < n; r += gstride()) {
    if (!early[r] || (only && !only[r])) continue;
    const uint64_t o = u3_sel(eoff[r], q), s = R.off[r];
    const uint32_t len = R.len[r];
    for (uint32_t t = 0; t < len; ++t) {
      col[o + t] = R.key[s + t];
      const Fe c = ffrom_mont(F, R.val[s + t]);
      val[4 * (o + t) + 0] = c.l[0];
      val[4 * (o + t) + 1] = c.l[1];
      val[4 * (o + t) + 2] = c.l[2];
      val[4 * (o + t) + 3] = c.l[3];
    }
  }
}

// A round's snapshot: the storage rows the round rewrote (touched), and the ones not sent yet, that stay
// storage rows (turn < 0) -- elen[r] their part lengths by storage id (else 0); k_snap_mark_round
// makes them early at base + their offsets (by non-linear row nl_of[r]) and clean again;
// k_snap_gather_st copies them.  (A later round may still rewrite one: dirty again, late at the end.)
__global__ void k_snap_lens_round(DRows a, DRows b, DRows c, const uint8_t *touched, const int32_t *turn, const uint32_t *nl_of,
                                  const uint8_t *early, uint64_t n, U3 *elen, ViewCopy vc) {
  for (uint64_t r = gtid(); r < n; r += gstride()) {
    const bool ok = (touched[r] || !early[nl_of[r]]) && turn[r] < 0 && (a.len[r] | b.len[r]) != 0;
    elen[r] = ok ? U3{a.len[r], b.len[r], c.len[r]} : U3{0, 0, 0};
    if (ok) view_copy(vc, a, b, c, r, a.len[r], b.len[r], c.len[r]);
  }
}
__global__ void k_snap_mark_round(const uint32_t *nl_of, const U3 *elen, const U3 *eoff3, U3 base, uint64_t n, uint8_t *early,
                                  U3 *eoff, uint8_t *dirty) {
  for (uint64_t r = gtid(); r < n; r += gstride()) {
    if ((elen[r].a | elen[r].b) == 0) continue;
    const uint32_t i = nl_of[r];
    early[i] = 1;
    eoff[i] = U3{base.a + eoff3[r].a, base.b + eoff3[r].b, base.c + eoff3[r].c};
    dirty[r] = 0;
  }
}
__global__ void k_snap_gather_st(FieldP F, DRows R, const U3 *elen, const U3 *eoff3, uint64_t base, int q, uint64_t n,
                                 uint32_t *col, uint64_t *val) {
  for (uint64_t r = gtid(); r < n; r += gstride()) {
    if ((elen[r].a | elen[r].b) == 0) continue;
    const uint64_t o = base + u3_sel(eoff3[r], q), s = R.off[r];
    const uint32_t len = R.len[r];
    for (uint32_t t = 0; t < len; ++t) {
      col[o + t] = R.key[s + t];
      const Fe c = ffrom_mont(F, R.val[s + t]);
      val[4 * (o + t) + 0] = c.l[0];
      val[4 * (o + t) + 1] = c.l[1];
      val[4 * (o + t) + 2] = c.l[2];
      val[4 * (o + t) + 3] = c.l[3];
    }
  }
}

__global__ void k_or_u8(const uint8_t *x, uint64_t n, uint8_t *acc) {
  for (uint64_t i = gtid(); i < n; i += gstride())
    if (x[i]) acc[i] = 1;
}

// storage row r (non-linear row nl_of[r]) keeps its early copy: early, and no later round touched it
__device__ __forceinline__ bool d_reused(const uint8_t *early, const uint8_t *dirty, const uint32_t *nl_of, uint32_t r) {
  return early && early[nl_of[r]] && !dirty[r];
}

// output rows ids[0..n) of one part: the length each needs in the late region (0: reused)
__global__ void k_out_late_lens(DRows R, const uint32_t *ids, uint64_t n, const uint32_t *nl_of, const uint8_t *early,
                                const uint8_t *dirty, uint64_t *late) {
  for (uint64_t i = gtid(); i < n; i += gstride()) {
    const uint32_t r = ids[i];
    late[i] = d_reused(early, dirty, nl_of, r) ? 0 : R.len[r];
  }
}

// their extents: a reused row keeps its early offset, the others go to base + lptr[i]
__global__ void k_out_extent(DRows R, const uint32_t *ids, uint64_t n, const uint32_t *nl_of, const uint8_t *early,
                             const uint8_t *dirty, const U3 *eoff, int q, uint64_t base, const uint64_t *lptr, uint64_t *beg,
                             uint64_t *end) {
  for (uint64_t i = gtid(); i < n; i += gstride()) {
    const uint32_t r = ids[i];
    const uint64_t b = d_reused(early, dirty, nl_of, r) ? u3_sel(eoff[nl_of[r]], q) : base + lptr[i];
    beg[i] = b;
    end[i] = b + R.len[r];
  }
}

// lconst rows [0, n_snap) went with the first early region (their C entries at c_base + their heap
// offset, in heap order: fix_constraint is applied as they enter the heap, so they are final there);
// the rest -- a later round's leftovers -- are late rows like any other
__global__ void k_lc_late_lens(DRows R, const uint32_t *ids, uint64_t n, uint64_t n_snap, uint64_t *late) {
  for (uint64_t i = gtid(); i < n; i += gstride()) {
    const uint32_t r = ids[i];
    late[i] = r < n_snap ? 0 : R.len[r];
  }
}
__global__ void k_lc_extent(DRows R, const uint32_t *ids, uint64_t n, uint64_t n_snap, uint64_t c_base, int q, uint64_t base,
                            const uint64_t *lptr, uint64_t *beg, uint64_t *end) {
  for (uint64_t i = gtid(); i < n; i += gstride()) {
    const uint32_t r = ids[i];
    const uint64_t b = r < n_snap && q == 2 ? c_base + R.off[r] : base + lptr[i];
    beg[i] = b;
    end[i] = b + R.len[r];
  }
}
__global__ void k_lc_gather_late(FieldP F, DRows R, const uint32_t *ids, uint64_t n, uint64_t n_snap, const uint64_t *lptr,
                                 uint32_t *col, uint64_t *val) {
  for (uint64_t i = gtid(); i < n; i += gstride()) {
    const uint32_t r = ids[i];
    if (r < n_snap) continue;
    const uint64_t o = lptr[i], s = R.off[r];
    for (uint32_t t = 0; t < R.len[r]; ++t) {
      col[o + t] = R.key[s + t];
      const Fe c = ffrom_mont(F, R.val[s + t]);
      val[4 * (o + t) + 0] = c.l[0];
      val[4 * (o + t) + 1] = c.l[1];
      val[4 * (o + t) + 2] = c.l[2];
      val[4 * (o + t) + 3] = c.l[3];
    }
  }
}
// the lconst heap's entries [0, n), canonical, behind the storage rows' C part of the early region
__global__ void k_lc_snap(FieldP F, const uint32_t *key, const Fe *v, uint64_t n, uint32_t *col, uint64_t *val) {
  for (uint64_t t = gtid(); t < n; t += gstride()) {
    col[t] = key[t];
    const Fe c = ffrom_mont(F, v[t]);
    val[4 * t + 0] = c.l[0];
    val[4 * t + 1] = c.l[1];
    val[4 * t + 2] = c.l[2];
    val[4 * t + 3] = c.l[3];
  }
}

// the late rows, canonical, at lptr[i] of the late region
__global__ void k_gather_late(FieldP F, DRows R, const uint32_t *ids, uint64_t n, const uint32_t *nl_of, const uint8_t *early,
                              const uint8_t *dirty, const uint64_t *lptr, uint32_t *col, uint64_t *val) {
  for (uint64_t i = gtid(); i < n; i += gstride()) {
    const uint32_t r = ids[i];
    if (d_reused(early, dirty, nl_of, r)) continue;
    const uint64_t o = lptr[i], s = R.off[r];
    const uint32_t len = R.len[r];
    for (uint32_t t = 0; t < len; ++t) {
      col[o + t] = R.key[s + t];
      const Fe c = ffrom_mont(F, R.val[s + t]);
      val[4 * (o + t) + 0] = c.l[0];
      val[4 * (o + t) + 1] = c.l[1];
      val[4 * (o + t) + 2] = c.l[2];
      val[4 * (o + t) + 3] = c.l[3];
    }
  }
}

// device -> (pinned, mapped) host memory, 16 bytes per lane per step, fully coalesced
__global__ void k_to_host(const uint4 *src, uint4 *dst, uint64_t n16) {
  for (uint64_t i = gtid(); i < n16; i += gstride()) dst[i] = src[i];
}

__global__ void k_set_u64(uint64_t *p, uint64_t v) {
  if (gtid() == 0) *p = v;
}

// sharded result: this rank's output rows are the kept storage rows whose non-linear row lies in
// [lo, hi) -- a contiguous run of the (ascending) keep list: out[0] = its first index, out[1] = its end
__global__ void k_keep_range(const uint32_t *keep, uint64_t n_keep, const uint32_t *nl_of, uint64_t lo, uint64_t hi, uint64_t *out) {
  const uint64_t t = gtid();
  if (t >= 2) return;
  const uint64_t bound = t ? hi : lo;
  uint64_t a = 0, b = n_keep;
  while (a < b) {
    const uint64_t m = (a + b) / 2;
    if (nl_of[keep[m]] < bound) a = m + 1; else b = m;
  }
  out[t] = a;
}
__global__ void k_add_u64(const uint64_t *in, uint64_t n, uint64_t add, uint64_t *out) {
  for (uint64_t i = gtid(); i < n; i += gstride()) out[i] = in[i] + add;
}

// ABI 8's row layout from the extents [beg, end) of rows [0, m): len[i] = the row's entries, bit 31
// (RS_ROW_JUMP) when it does not start where row i - 1 ended (row 0: unless it starts at 0; always
// when first_jump -- a rank's first row in the shared layout); jf[i] = that bit, for the jump table
// (a row's keys are distinct signals below max_signal < 2^31, so its length never reaches bit 31)
__global__ void k_out_jumps(const uint64_t *beg, const uint64_t *end, uint64_t m, int first_jump, uint32_t *len, uint64_t *jf) {
  for (uint64_t i = gtid(); i < m; i += gstride()) {
    const uint64_t b = beg[i], l = end[i] - b;
    const bool j = i == 0 ? (first_jump || b != 0) : b != end[i - 1];
    len[i] = (uint32_t)l | (j ? RS_ROW_JUMP : 0u);
    jf[i] = j ? 1 : 0;
  }
}
// the jump table: the starts of the rows that jump, in row order (+ add: a rank's base in the shared layout)
__global__ void k_out_jtab(const uint64_t *beg, const uint64_t *jf, const uint64_t *jpos, uint64_t m, uint64_t add, uint64_t *jtab) {
  for (uint64_t i = gtid(); i < m; i += gstride())
    if (jf[i]) jtab[jpos[i]] = beg[i] + add;
}

