// refcpu.cpp -- canonical C++ CPU restatement of circom's R1CS simplification.
//
// TEST INFRASTRUCTURE / ORACLE.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
// leg may load this library; the product (circom_cvm_amd/, librs_simplify.so) never does.
//
// Parity pinning: tests/test_oracle.py checks this file against (1) the reference's own unit
// tests over F_257 (circom_algebra/src/algebra.rs:1401-1493, modular_arithmetic.rs:221-268),
// (2) the docs worked example basic.circom at O1/O2 (mkdocs/docs/circom-language/formats/
// constraints-json.md:57-59, 95-96; sym.md:46-51, 81-86), and (3) oracle/pyref.py, an
// independent literal Python restatement, on hundreds of seeded random systems.
//
// Follows, function by function (file:line in /root/reference):
//   build_clusters                 constraint_list/src/constraint_simplification.rs:45-99
//   rebuild_witness                 :101-124
//   eq_cluster_simplification       :126-196      eq_simplification            :198-251
//   constant_eq_simplification      :253-273      linear_simplification        :275-325
//   build_non_linear_signal_map     :327-343      apply_substitution_to_map    :345-396
//   build_relevant_set              :398-429      remove_not_relevant          :431-438
//   simplification                  :442-730
//   obtain_and_simplify_non_linear  constraint_list/src/non_linear_utils.rs:6-31
//   full_simplification + helpers   circom_algebra/src/simplification_utils.rs:24-581
//   raw_substitution, fix_raw_constraint, clear_signal*, ...   circom_algebra/src/algebra.rs
//
// Determinism: every HashMap/HashSet iteration that influences the result is
// done in ascending signal id; thread-pool results are collected in cluster-index order; the
// substitutions of one cluster are emitted in ascending `from`.
//
// Parallel structure mirrors the reference: a pool of n_threads over eq clusters of size > 1
// and over linear clusters (constraint_simplification.rs:212, :293); everything else serial.
//
// Algorithmic bytes (the roofline numerator; refcpu_last_alg): counted over the LOGICAL
// operations of this canonical execution, so they do not depend on how an implementation moves the
// data.  With w = 4 + field bytes per (signal, coefficient) entry:
//   B_alg = w * (Z_in + Z_out + subs + app + rowupd + merges) + 8 * (R_in + R_out) + 8 * max_signal
//   Z_in / Z_out   entries of the input blocks / of the result;  R_in / R_out their rows
//   subs           entries of every substitution written: eq and constant substitutions, the holders
//                  (clear_signal_not_normalized), their normalised copies (normalize_substitutions)
//   app            for every application of a substitution to a row or to another substitution
//                  (fast_encoded_constraint_substitution, apply_substitution_to_map, the lconst
//                  passes, create_nonoverlapping_substitutions): the entries of its right-hand side
//   rowupd         per row rewritten by one substitution pass (the eq + constant frames of a linear
//                  row; the three frames + fix of a non-linear row; one round's substitutions of a
//                  storage row or an lconst row; one composition step of a substitution; the ordered
//                  loop's reduction of a popped row into its holder or leftover): entries before +
//                  entries after
//   merges         per conflict merge of treat_constraint_3/4: |work| + |conflicting RHS| + |new work|

#include "refcpu_field.h"
#include "../include/rs_simplify.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

// Optional instrumentation of the ordered loop (tools/elim_trace.cpp defines these; no-ops here).
#ifndef RC_TRACE_CLUSTER
#define RC_TRACE_CLUSTER(n_rows, n_uniq) do { } while (0)
#define RC_TRACE_CLUSTER3(n_rows) do { } while (0)
#define RC_TRACE_ROW(len) do { } while (0)
#define RC_TRACE_MERGE(key, wlen, hidx, hlen) do { } while (0)
#define RC_TRACE_INSERT(key, hidx, len) do { } while (0)
#define RC_TRACE_LEFT(len) do { } while (0)
#define RC_TRACE_END() do { } while (0)
#endif

namespace refcpu {

struct Term {
  uint32_t k;
  Fe v;
};
typedef std::vector<Term> Map;  // sorted by k, unique keys, zero values allowed
struct Con {
  Map a, b, c;
};
struct Sub {
  uint32_t from;
  Map to;
};

static const uint64_t kPrimes[8][4] = {
    {0x43e1f593f0000001ULL, 0x2833e84879b97091ULL, 0xb85045b68181585dULL, 0x30644e72e131a029ULL},
    {0xffffffff00000001ULL, 0x53bda402fffe5bfeULL, 0x3339d80809a1d805ULL, 0x73eda753299d7d48ULL},
    {0xffffffff00000001ULL, 0, 0, 0},
    {0x3c208c16d87cfd47ULL, 0x97816a916871ca8dULL, 0xb85045b68181585dULL, 0x30644e72e131a029ULL},
    {0x992d30ed00000001ULL, 0x224698fc094cf91bULL, 0x0000000000000000ULL, 0x4000000000000000ULL},
    {0x8c46eb2100000001ULL, 0x224698fc0994a8ddULL, 0x0000000000000000ULL, 0x4000000000000000ULL},
    {0xffffffffffffffffULL, 0x00000000ffffffffULL, 0x0000000000000000ULL, 0xffffffff00000001ULL},
    {0x0a11800000000001ULL, 0x59aa76fed0000001ULL, 0x60b44d1e5c37b001ULL, 0x12ab655e9a2ca556ULL}};

// the B_alg terms (entries, except the row counts); summed per cluster, so parallel workers never share one
struct Alg {
  uint64_t z_in = 0, z_out = 0, subs = 0, app = 0, rowupd = 0, merges = 0, r_in = 0, r_out = 0;
  void add(const Alg &o) {
    z_in += o.z_in; z_out += o.z_out; subs += o.subs; app += o.app;
    rowupd += o.rowupd; merges += o.merges; r_in += o.r_in; r_out += o.r_out;
  }
};
struct Ctx {
  Alg alg;
  Field F;
  uint64_t max_signal = 0;
  std::vector<uint8_t> forbidden;
  int n_threads = 1;
  // dense per-signal scratch shared by the cluster workers (clusters are signal-disjoint)
  std::vector<int32_t> holder_idx, occ, noov_idx;
  std::vector<uint8_t> del;
  std::vector<int32_t> sig2cl;
};

// ------------------------------------------------------------------ map helpers (algebra.rs)
static inline int find(const Map &m, uint32_t k) {
  int lo = 0, hi = (int)m.size() - 1;
  while (lo <= hi) {
    int mid = (lo + hi) >> 1;
    if (m[mid].k == k) return mid;
    if (m[mid].k < k) lo = mid + 1; else hi = mid - 1;
  }
  return -1;
}
// initialize_hashmap_for_expression (algebra.rs:158-163): key 0 is the smallest key.
static inline void init_map(Map &m) {
  if (m.empty() || m[0].k != 0) m.insert(m.begin(), Term{0, fe_zero()});
}
static inline void remove_zero(Map &m) {
  size_t w = 0;
  for (size_t i = 0; i < m.size(); ++i)
    if (!m[i].v.is_zero()) m[w++] = m[i];
  m.resize(w);
}
// raw_substitution (algebra.rs:1279-1294): change[from] is replaced by change[from]*to, every key
// of `to` (and the constant key) is inserted even when the sum is zero.
static void raw_substitution(const Field &F, Map &change, uint32_t from, const Map &to) {
  init_map(change);
  int idx = find(change, from);
  if (idx < 0) return;
  Fe val = change[idx].v;
  change.erase(change.begin() + idx);
  Map out;
  out.reserve(change.size() + to.size() + 1);
  size_t i = 0, j = 0;
  bool virt0 = to.empty() || to[0].k != 0;  // coefficients.initialize adds {0: 0}
  while (i < change.size() || j < to.size() || virt0) {
    uint32_t kj;
    Fe vj;
    bool hj;
    if (virt0) { kj = 0; vj = fe_zero(); hj = true; }
    else if (j < to.size()) { kj = to[j].k; vj = to[j].v; hj = true; }
    else { kj = 0; vj = fe_zero(); hj = false; }
    if (i < change.size() && (!hj || change[i].k < kj)) {
      out.push_back(change[i++]);
    } else if (i < change.size() && change[i].k == kj) {
      out.push_back(Term{kj, F.add(change[i].v, F.mul(val, vj))});
      ++i;
      if (virt0) virt0 = false; else ++j;
    } else {
      out.push_back(Term{kj, F.mul(val, vj)});
      if (virt0) virt0 = false; else ++j;
    }
  }
  change.swap(out);
}
static inline bool is_linear(const Con &c) { return c.a.empty() && c.b.empty(); }
static inline bool is_empty(const Con &c) { return c.a.empty() && c.b.empty() && c.c.empty(); }
static inline bool is_constant_expression(const Map &m) { return m.size() == 1 && m[0].k == 0; }

// take_cloned_signals (algebra.rs:1078-1091), ascending.
static void take_signals(const Con &c, std::vector<uint32_t> &out) {
  out.clear();
  for (const Map *m : {&c.a, &c.b, &c.c})
    for (const Term &t : *m)
      if (t.k != 0) out.push_back(t.k);
  std::sort(out.begin(), out.end());
  out.erase(std::unique(out.begin(), out.end()), out.end());
}
static void apply_substitution(const Field &F, Con &c, uint32_t from, const Map &to) {
  raw_substitution(F, c.a, from, to);
  raw_substitution(F, c.b, from, to);
  raw_substitution(F, c.c, from, to);
}
// constant_linear_linear_reduction (algebra.rs:1326-1344): c := c - a0 * b.
static void const_lin_reduction(const Field &F, Map &a, Map &b, Map &c) {
  init_map(c);
  init_map(b);
  Fe a0 = a[0].v;
  Fe m1 = F.neg(F.one);
  Map scaled = b;
  for (Term &t : scaled) t.v = F.mul(F.mul(t.v, a0), m1);
  Map out;
  size_t i = 0, j = 0;
  while (i < c.size() || j < scaled.size()) {
    if (j >= scaled.size() || (i < c.size() && c[i].k < scaled[j].k)) out.push_back(c[i++]);
    else if (i >= c.size() || scaled[j].k < c[i].k) out.push_back(scaled[j++]);
    else { out.push_back(Term{c[i].k, F.add(c[i].v, scaled[j].v)}); ++i; ++j; }
  }
  remove_zero(out);
  c.swap(out);
  a.clear();
  b.clear();
}
// fix_raw_constraint (algebra.rs:1309-1324)
static void fix_constraint(const Field &F, Con &c) {
  remove_zero(c.a);
  remove_zero(c.b);
  remove_zero(c.c);
  if (c.a.empty() || c.b.empty()) {
    c.a.clear();
    c.b.clear();
  } else if (is_constant_expression(c.a)) {
    const_lin_reduction(F, c.a, c.b, c.c);
  } else if (is_constant_expression(c.b)) {
    const_lin_reduction(F, c.b, c.a, c.c);
  }
}

// ------------------------------------------------------------------ thread pool
template <class Fn>
static void parallel_for(int n_threads, size_t n, Fn fn) {
  if (n_threads <= 1 || n < 2) {
    for (size_t i = 0; i < n; ++i) fn(i);
    return;
  }
  std::atomic<size_t> next(0);
  std::vector<std::thread> th;
  int nt = (int)std::min<size_t>(n_threads, n);
  for (int t = 0; t < nt; ++t)
    th.emplace_back([&]() {
      for (;;) {
        size_t i = next.fetch_add(1);
        if (i >= n) break;
        fn(i);
      }
    });
  for (auto &x : th) x.join();
}

// ------------------------------------------------------------------ build_clusters (:45-99)
// rows: constraints (only keys are used).  Returns clusters as lists of row indices in the
// reference's list order (dest ++ src on every merge).
static std::vector<std::vector<uint32_t>> build_clusters(Ctx &X, const std::vector<Con> &rows) {
  std::vector<int32_t> head, tail, c2c, slot_row;
  std::vector<int32_t> next(rows.size(), -1);
  std::vector<uint32_t> sigs, touched;
  auto findr = [&](int32_t org) {
    int32_t cur = org;
    while (cur != c2c[cur]) cur = c2c[cur];
    while (org != cur) {
      int32_t nx = c2c[org];
      c2c[org] = cur;
      org = nx;
    }
    return cur;
  };
  for (size_t r = 0; r < rows.size(); ++r) {
    if (is_empty(rows[r])) continue;
    take_signals(rows[r], sigs);
    int32_t dest = (int32_t)head.size();
    head.push_back((int32_t)r);
    tail.push_back((int32_t)r);
    c2c.push_back(dest);
    for (uint32_t s : sigs) {
      int32_t prev = X.sig2cl[s];
      if (prev < 0) touched.push_back(s);
      X.sig2cl[s] = dest;
      if (prev >= 0) {
        int32_t cd = findr(dest), cs = findr(prev);
        if (cs != cd) {
          next[tail[cd]] = head[cs];
          tail[cd] = tail[cs];
          head[cs] = -1;
          c2c[cs] = cd;
        }
      }
    }
  }
  for (uint32_t s : touched) X.sig2cl[s] = -1;
  std::vector<std::vector<uint32_t>> clusters;
  for (size_t slot = 0; slot < head.size(); ++slot) {
    if (head[slot] < 0) continue;
    std::vector<uint32_t> cl;
    for (int32_t r = head[slot]; r >= 0; r = next[r]) cl.push_back((uint32_t)r);
    clusters.push_back(std::move(cl));
  }
  return clusters;
}

// ------------------------------------------------------------------ eq (:126-251)
static Map signal_map1(const Field &F, uint32_t s) {
  Map m;
  m.push_back(Term{s, F.one});
  return m;
}
static void eq_cluster(Ctx &X, const std::vector<Con> &rows, const std::vector<uint32_t> &cl,
                       std::vector<Sub> &subs, std::vector<Con> &cons) {
  const Field &F = X.F;
  std::vector<uint32_t> sig;
  if (cl.size() == 1) {
    const Con &c = rows[cl[0]];
    take_signals(c, sig);
    uint32_t s0 = sig[0], s1 = sig[1];
    bool f0 = X.forbidden[s0], f1 = X.forbidden[s1];
    if (f0 && f1) cons.push_back(c);
    else if (f0) subs.push_back(Sub{s1, signal_map1(F, s0)});
    else if (f1) subs.push_back(Sub{s0, signal_map1(F, s1)});
    else subs.push_back(Sub{std::max(s0, s1), signal_map1(F, std::min(s0, s1))});
    return;
  }
  std::vector<uint32_t> remains, remove;
  for (uint32_t r : cl) {
    take_signals(rows[r], sig);
    for (uint32_t s : sig) (X.forbidden[s] ? remains : remove).push_back(s);
  }
  std::sort(remains.begin(), remains.end());
  remains.erase(std::unique(remains.begin(), remains.end()), remains.end());
  std::sort(remove.begin(), remove.end());
  remove.erase(std::unique(remove.begin(), remove.end()), remove.end());
  uint32_t rh;
  if (!remains.empty()) { rh = remains[0]; remains.erase(remains.begin()); }
  else { rh = remove[0]; remove.erase(remove.begin()); }
  for (uint32_t s : remains) {
    // transform(sub(Signal s, Signal rh)): c = {0: 0, rh: 1, s: -1}, a = b = {0: 0}
    // (algebra.rs:113-145, 441-450).  a and b only ever reach fix_constraint, which clears them,
    // before anything observes them, so they are kept empty here.
    Con c;
    c.c.push_back(Term{0, fe_zero()});
    Term t1{rh, F.one}, t2{s, F.neg(F.one)};
    if (rh < s) { c.c.push_back(t1); c.c.push_back(t2); }
    else { c.c.push_back(t2); c.c.push_back(t1); }
    cons.push_back(std::move(c));
  }
  for (uint32_t s : remove) subs.push_back(Sub{s, signal_map1(F, rh)});
}

// ------------------------------------------------------------------ full_simplification
struct Holder {
  std::vector<uint32_t> sig;
  std::vector<Fe> coef;
  std::vector<Map> to;
};

// clear_signal_not_normalized (algebra.rs:1126-1136)
static void clear_nn(const Field &F, const Map &c, uint32_t key, Fe &coef, Map &to) {
  to.clear();
  to.reserve(c.size());
  coef = fe_zero();
  for (const Term &t : c) {
    if (t.k == key) coef = F.neg(t.v);
    else to.push_back(t);
  }
  if (coef.is_zero()) throw std::runtime_error("clear_signal on a zero coefficient (algebra.rs:1132)");
  init_map(to);
}
// conflict merge of treat_constraint_3/4: work.c = coef*R - c2*L, zeros removed
static void merge_conflict(const Field &F, const Fe &coef, const Map &L, const Fe &c2, const Map &R,
                           Map &out) {
  out.clear();
  size_t i = 0, j = 0;
  while (i < L.size() || j < R.size()) {
    Fe v;
    uint32_t k;
    if (j >= R.size() || (i < L.size() && L[i].k < R[j].k)) {
      k = L[i].k; v = F.neg(F.mul(c2, L[i].v)); ++i;
    } else if (i >= L.size() || R[j].k < L[i].k) {
      k = R[j].k; v = F.mul(coef, R[j].v); ++j;
    } else {
      k = L[i].k; v = F.sub(F.mul(coef, R[j].v), F.mul(c2, L[i].v)); ++i; ++j;
    }
    if (!v.is_zero()) out.push_back(Term{k, v});
  }
}

struct Simplified {
  std::vector<Map> lconst;  // leftover linear constraints (C part)
  std::vector<Sub> subs;    // ascending from
  Alg alg;                  // this cluster's B_alg terms
};

static void normalize_and_compose(Ctx &X, Holder &H, const std::vector<uint32_t> *order,
                                  Simplified &res) {
  const Field &F = X.F;
  size_t m = H.sig.size();
  // BTreeMap order (ascending signal): multi_inv over coefficients (modular_arithmetic.rs:71-91)
  std::vector<uint32_t> perm(m);
  for (size_t i = 0; i < m; ++i) perm[i] = (uint32_t)i;
  std::sort(perm.begin(), perm.end(), [&](uint32_t x, uint32_t y) { return H.sig[x] < H.sig[y]; });
  std::vector<Fe> pre(m + 1);
  pre[0] = F.one;
  for (size_t i = 0; i < m; ++i) pre[i + 1] = F.mul(pre[i], H.coef[perm[i]]);
  Fe inv = F.inv(pre[m]);
  std::vector<Fe> invs(m);
  for (size_t i = m; i > 0; --i) {
    invs[i - 1] = F.mul(pre[i - 1], inv);
    inv = F.mul(inv, H.coef[perm[i - 1]]);
  }
  for (size_t i = 0; i < m; ++i) {
    for (Term &t : H.to[perm[i]]) t.v = F.mul(t.v, invs[i]);
    res.alg.subs += H.to[perm[i]].size();  // the normalised copy
  }
  // create_nonoverlapping_substitutions(_4) (simplification_utils.rs:451-479)
  std::vector<uint32_t> seq;
  if (order) seq.assign(order->rbegin(), order->rend());  // newest first
  else for (size_t i = 0; i < m; ++i) seq.push_back(H.sig[perm[i]]);
  std::vector<uint32_t> apply;
  for (uint32_t s : seq) {
    int32_t hi = X.holder_idx[s];
    Map &to = H.to[hi];
    apply.clear();
    for (const Term &t : to)
      if (X.noov_idx[t.k] >= 0) apply.push_back(t.k);
    for (uint32_t k : apply) {
      const Map &rk = H.to[X.noov_idx[k]];
      const uint64_t before = to.size();
      raw_substitution(F, to, k, rk);
      res.alg.app += rk.size();
      res.alg.rowupd += before + to.size();
    }
    X.noov_idx[s] = hi;
  }
  for (size_t i = 0; i < m; ++i) {
    uint32_t s = H.sig[perm[i]];
    X.noov_idx[s] = -1;
    X.holder_idx[s] = -1;
    res.subs.push_back(Sub{s, std::move(H.to[perm[i]])});
  }
}

static void process_3(Ctx &X, std::vector<Map> &cons, Simplified &res) {
  const Field &F = X.F;
  Holder H;
  Map to, work;
  Fe coef;
  RC_TRACE_CLUSTER3(cons.size());
  while (!cons.empty()) {
    work.swap(cons.back());
    cons.pop_back();
    RC_TRACE_ROW(work.size());
    const uint64_t popped = work.size();
    uint64_t written = 0;
    for (;;) {
      if (work.empty()) break;
      int64_t out = -1;
      for (size_t i = work.size(); i-- > 0;)
        if (!X.forbidden[work[i].k]) { out = work[i].k; break; }
      if (out < 0) { RC_TRACE_LEFT(work.size()); written = work.size(); res.lconst.push_back(work); break; }
      clear_nn(F, work, (uint32_t)out, coef, to);
      int32_t hi = X.holder_idx[out];
      if (hi >= 0) RC_TRACE_MERGE((uint32_t)out, work.size(), hi, H.to[hi].size());
      if (hi < 0) {
        RC_TRACE_INSERT((uint32_t)out, H.sig.size(), to.size());
        X.holder_idx[out] = (int32_t)H.sig.size();
        H.sig.push_back((uint32_t)out);
        H.coef.push_back(coef);
        H.to.push_back(to);
        written = to.size();
        res.alg.subs += to.size();
        break;
      }
      const uint64_t w0 = work.size();
      merge_conflict(F, coef, to, H.coef[hi], H.to[hi], work);
      res.alg.merges += w0 + H.to[hi].size() + work.size();
    }
    res.alg.rowupd += popped + written;
  }
  RC_TRACE_END();
  normalize_and_compose(X, H, nullptr, res);
}

static void process_4(Ctx &X, std::vector<Map> &vec, Simplified &res) {
  const Field &F = X.F;
  Holder H;
  std::vector<uint32_t> order;  // deletion order (oldest first); iterated reversed
  std::vector<uint32_t> touched;
  std::vector<std::pair<uint32_t, uint32_t>> uniques;
  std::vector<int32_t> repv;
  // SignalsInformation::new (simplification_utils.rs:66-92)
  for (size_t pos = 0; pos < vec.size(); ++pos)
    for (const Term &t : vec[pos])
      if (!X.forbidden[t.k]) {
        if (X.occ[t.k] < 0) { X.occ[t.k] = 1; touched.push_back(t.k); repv.push_back((int32_t)pos); }
        else X.occ[t.k]++;
      }
  for (size_t i = 0; i < touched.size(); ++i)
    if (X.occ[touched[i]] == 1) uniques.push_back({touched[i], (uint32_t)repv[i]});
  std::sort(uniques.begin(), uniques.end());
  RC_TRACE_CLUSTER(vec.size(), uniques.size());
  auto remove_constraint = [&](const Map &c) {
    for (const Term &t : c)
      if (!X.forbidden[t.k] && X.occ[t.k] >= 0) X.occ[t.k]--;
  };
  auto insert = [&](uint32_t s, const Fe &coef, Map &to) {
    X.holder_idx[s] = (int32_t)H.sig.size();
    H.sig.push_back(s);
    H.coef.push_back(coef);
    H.to.push_back(to);
    X.occ[s] = -1;  // remove_signal
    X.del[s] = 1;
    order.push_back(s);
  };
  Map to, work;
  Fe coef;
  for (auto &u : uniques) {
    if (vec[u.second].empty()) continue;
    Map actual;
    actual.swap(vec[u.second]);
    remove_constraint(actual);
    clear_nn(F, actual, u.first, coef, to);
    RC_TRACE_INSERT(u.first, H.sig.size(), to.size());
    res.alg.rowupd += actual.size() + to.size();
    res.alg.subs += to.size();
    insert(u.first, coef, to);
  }
  while (!vec.empty()) {
    work.swap(vec.back());
    vec.pop_back();
    remove_constraint(work);
    RC_TRACE_ROW(work.size());
    const uint64_t popped = work.size();
    uint64_t written = 0;
    for (;;) {
      if (work.empty()) break;
      // take_signal_4 (simplification_utils.rs:379-411), HashMap order := ascending
      int64_t ret = -1;
      int32_t occ_ret = -1;
      for (const Term &t : work) {
        if (X.forbidden[t.k]) continue;
        if (X.del[t.k]) { ret = t.k; break; }
        int32_t n = X.occ[t.k];
        if (n < 0) throw std::runtime_error("take_signal_4: missing occurrence count");
        if (occ_ret < 0 || n < occ_ret) { ret = t.k; occ_ret = n; }
        else if (n == occ_ret && ret < (int64_t)t.k) ret = t.k;
      }
      if (ret < 0) { RC_TRACE_LEFT(work.size()); written = work.size(); res.lconst.push_back(work); break; }
      clear_nn(F, work, (uint32_t)ret, coef, to);
      int32_t hi = X.holder_idx[ret];
      if (hi < 0) {
        RC_TRACE_INSERT((uint32_t)ret, H.sig.size(), to.size());
        written = to.size();
        res.alg.subs += to.size();
        insert((uint32_t)ret, coef, to);
        break;
      }
      RC_TRACE_MERGE((uint32_t)ret, work.size(), hi, H.to[hi].size());
      const uint64_t w0 = work.size();
      merge_conflict(F, coef, to, H.coef[hi], H.to[hi], work);
      res.alg.merges += w0 + H.to[hi].size() + work.size();
    }
    res.alg.rowupd += popped + written;
  }
  RC_TRACE_END();
  for (uint32_t s : touched) X.occ[s] = -1;
  for (uint32_t s : order) X.del[s] = 0;
  normalize_and_compose(X, H, &order, res);
}

static Simplified full_simplification(Ctx &X, std::vector<Map> &&cons, bool old_heur) {
  Simplified res;
  size_t n = cons.size();
  if (n >= 350 && n < 1000000 && !old_heur) process_4(X, cons, res);
  else process_3(X, cons, res);
  return res;
}

// linear_simplification (:275-325)
static void linear_simplification(Ctx &X, const std::vector<Con> &linear, bool old_heur,
                                  std::vector<Sub> &subs, std::vector<Con> &cons,
                                  uint64_t *n_clusters) {
  auto clusters = build_clusters(X, linear);
  if (n_clusters) *n_clusters += clusters.size();
  std::vector<Simplified> results(clusters.size());
  parallel_for(X.n_threads, clusters.size(), [&](size_t i) {
    std::vector<Map> rows;
    rows.reserve(clusters[i].size());
    for (uint32_t r : clusters[i]) rows.push_back(linear[r].c);
    results[i] = full_simplification(X, std::move(rows), old_heur);
  });
  for (auto &r : results) {
    X.alg.add(r.alg);
    for (auto &m : r.lconst) { Con c; c.c = std::move(m); cons.push_back(std::move(c)); }
    for (auto &s : r.subs) subs.push_back(std::move(s));
  }
}

// fast_encoded_constraint_substitution (simplification_utils.rs:496-507)
static bool fast_encoded(const Field &F, Con &c, const std::vector<int32_t> &idx,
                         const std::vector<Sub> &subs, std::vector<uint32_t> &sig, uint64_t *app = nullptr) {
  take_signals(c, sig);
  bool applied = false;
  for (uint32_t s : sig) {
    int32_t i = idx[s];
    if (i >= 0) {
      apply_substitution(F, c, s, subs[i].to);
      applied = true;
      if (app) *app += subs[i].to.size();
    }
  }
  return applied;
}
static inline uint64_t con_size(const Con &c) { return c.a.size() + c.b.size() + c.c.size(); }

// ------------------------------------------------------------------ simplification (:442-730)
struct Input {
  std::vector<Con> cons_eq, eq, linear, nonlin;
  uint64_t n_pub_out, n_pub_in, n_priv_in;
};
struct Output {
  std::vector<Con> constraints;
  std::vector<int32_t> label_to_wire;
  uint64_t n_wires = 0, no_private_inputs_witness = 0;
  uint64_t rounds = 0, n_clusters = 0;
};

static void simplification(Ctx &X, Input &in, uint32_t flag_s, uint64_t no_rounds, bool old_heur,
                           Output &out) {
  const Field &F = X.F;
  const uint64_t S = X.max_signal;
  bool apply_linear = !flag_s;
  std::vector<uint8_t> deleted(S, 0);
  std::vector<Con> lconst;
  std::vector<uint32_t> sig;

  auto relevant_set = [&](const std::vector<int32_t> *ren, const std::vector<Sub> *rsubs,
                          const std::vector<int32_t> *del) {
    std::vector<uint8_t> rel(S, 0);
    for (const Con &c : in.nonlin) {
      take_signals(c, sig);
      for (uint32_t s : sig) {
        uint32_t s2 = s;
        if (ren && (*ren)[s] >= 0) {
          const Map &to = (*rsubs)[(*ren)[s]].to;  // eq subs: {rep: 1} -> Signal rep
          s2 = to[0].k;
        }
        if (!(del && (*del)[s2] >= 0)) rel[s2] = 1;
      }
    }
    return rel;
  };
  std::vector<uint8_t> relevant = relevant_set(nullptr, nullptr, nullptr);

  // ---- eq_simplification
  std::vector<Sub> eq_subs;
  {
    auto clusters = build_clusters(X, in.eq);
    std::vector<std::vector<Con>> aux(clusters.size());
    std::vector<std::vector<Sub>> subs_of(clusters.size());
    std::vector<size_t> multi;
    for (size_t i = 0; i < clusters.size(); ++i) {
      if (clusters[i].size() == 1) {
        eq_cluster(X, in.eq, clusters[i], subs_of[i], aux[i]);
        for (auto &s : subs_of[i]) eq_subs.push_back(std::move(s));
      } else {
        multi.push_back(i);
      }
    }
    parallel_for(X.n_threads, multi.size(),
                 [&](size_t j) { eq_cluster(X, in.eq, clusters[multi[j]], subs_of[multi[j]], aux[multi[j]]); });
    for (size_t j : multi)
      for (auto &s : subs_of[j]) eq_subs.push_back(std::move(s));
    for (auto &v : aux)
      for (auto &c : v) lconst.push_back(std::move(c));
  }
  std::vector<int32_t> eq_idx(S, -1);
  for (size_t i = 0; i < eq_subs.size(); ++i) eq_idx[eq_subs[i].from] = (int32_t)i;
  for (const Sub &sb : eq_subs) X.alg.subs += sb.to.size();
  // B_alg: a linear row's eq + constant frames are one update (its size before them, after both)
  std::vector<uint32_t> lin0(in.linear.size());
  std::vector<uint8_t> lin_touched(in.linear.size(), 0);
  for (size_t i = 0; i < in.linear.size(); ++i) lin0[i] = (uint32_t)con_size(in.linear[i]);
  for (size_t i = 0; i < in.linear.size(); ++i) {
    Con &c = in.linear[i];
    if (fast_encoded(F, c, eq_idx, eq_subs, sig, &X.alg.app)) { fix_constraint(F, c); lin_touched[i] = 1; }
  }
  for (Con &c : in.cons_eq) {
    const uint64_t before = con_size(c);
    if (fast_encoded(F, c, eq_idx, eq_subs, sig, &X.alg.app)) { fix_constraint(F, c); X.alg.rowupd += before + con_size(c); }
  }
  for (const Sub &s : eq_subs) deleted[s.from] = 1;
  std::vector<int32_t> single_idx(S, -1);  // remove_not_relevant
  for (size_t i = 0; i < eq_subs.size(); ++i)
    if (relevant[eq_subs[i].from]) single_idx[eq_subs[i].from] = (int32_t)i;

  // ---- constant_eq_simplification
  std::vector<Sub> c_subs;
  for (Con &c : in.cons_eq) {
    take_signals(c, sig);
    if (sig.empty()) throw std::runtime_error("constant equality without a signal");
    uint32_t s = sig.back();
    if (X.forbidden[s]) { lconst.push_back(c); continue; }
    // clear_signal (algebra.rs:1108-1124): to = rest / (-k), zeros removed
    Fe k = fe_zero();
    Map rest;
    for (const Term &t : c.c) {
      if (t.k == s) k = t.v; else rest.push_back(t);
    }
    if (k.is_zero()) throw std::runtime_error("clear_signal on a zero coefficient");
    init_map(rest);
    Fe inv = F.inv(F.neg(k));
    for (Term &t : rest) t.v = F.mul(t.v, inv);
    remove_zero(rest);
    X.alg.subs += rest.size();
    c_subs.push_back(Sub{s, std::move(rest)});
  }
  std::vector<int32_t> c_idx(S, -1);
  for (size_t i = 0; i < c_subs.size(); ++i) c_idx[c_subs[i].from] = (int32_t)i;  // last wins
  for (size_t i = 0; i < in.linear.size(); ++i) {
    Con &c = in.linear[i];
    if (fast_encoded(F, c, c_idx, c_subs, sig, &X.alg.app)) { fix_constraint(F, c); lin_touched[i] = 1; }
    if (lin_touched[i]) X.alg.rowupd += lin0[i] + con_size(c);
  }
  for (const Sub &s : c_subs) deleted[s.from] = 1;

  relevant = relevant_set(&single_idx, &eq_subs, &c_idx);

  // ---- linear round 1
  std::vector<Sub> l_subs;
  std::vector<int32_t> l_idx(S, -1);
  if (apply_linear) {
    std::vector<Sub> subs;
    std::vector<Con> cons;
    linear_simplification(X, in.linear, old_heur, subs, cons, &out.n_clusters);
    out.rounds++;
    for (Sub &s : subs) {
      deleted[s.from] = 1;
      if (relevant[s.from]) l_subs.push_back(std::move(s));
    }
    for (size_t i = 0; i < l_subs.size(); ++i) l_idx[l_subs[i].from] = (int32_t)i;
    for (auto &c : cons) lconst.push_back(std::move(c));
    for (Con &c : lconst) {
      const uint64_t before = con_size(c);
      if (fast_encoded(F, c, l_idx, l_subs, sig, &X.alg.app)) { fix_constraint(F, c); X.alg.rowupd += before + con_size(c); }
    }
  } else {
    for (auto &c : in.linear) lconst.push_back(std::move(c));
  }

  // ---- obtain_and_simplify_non_linear (non_linear_utils.rs:6-31)
  std::vector<Con> storage, linear;
  for (Con &c : in.nonlin) {  // B_alg: the three frames and the fix are one update of the row
    const uint64_t before = con_size(c);
    fast_encoded(F, c, single_idx, eq_subs, sig, &X.alg.app);
    fast_encoded(F, c, c_idx, c_subs, sig, &X.alg.app);
    fast_encoded(F, c, l_idx, l_subs, sig, &X.alg.app);
    fix_constraint(F, c);
    X.alg.rowupd += before + con_size(c);
    if (is_linear(c)) linear.push_back(std::move(c));
    else storage.push_back(std::move(c));
  }
  if (no_rounds > 0) no_rounds--;

  bool apply_round = apply_linear && no_rounds > 0 && !linear.empty();
  std::vector<std::vector<uint32_t>> nl_map(S);  // build_non_linear_signal_map (:327-343)
  for (size_t id = 0; id < storage.size(); ++id) {
    take_signals(storage[id], sig);
    for (uint32_t s : sig) nl_map[s].push_back((uint32_t)id);
  }
  std::vector<int32_t> r_idx(S, -1);
  std::vector<uint8_t> round_seen(storage.size(), 0);
  while (apply_round) {
    std::vector<Sub> subs;
    std::vector<Con> constants;
    linear_simplification(X, linear, old_heur, subs, constants, &out.n_clusters);
    out.rounds++;
    for (const Sub &s : subs) deleted[s.from] = 1;
    for (auto &c : constants) lconst.push_back(std::move(c));
    // for constraint in lconst { for sub in subs { apply } fix }  (:629-634)
    for (size_t i = 0; i < subs.size(); ++i) r_idx[subs[i].from] = (int32_t)i;
    for (Con &c : lconst) {
      const uint64_t before = con_size(c);
      bool touched = false;
      if (!subs.empty()) {
        init_map(c.a);
        init_map(c.b);
        init_map(c.c);
        take_signals(c, sig);
        std::vector<int32_t> which;
        for (uint32_t s : sig)
          if (r_idx[s] >= 0) which.push_back(r_idx[s]);
        std::sort(which.begin(), which.end());
        for (int32_t w : which) { apply_substitution(F, c, subs[w].from, subs[w].to); X.alg.app += subs[w].to.size(); }
        touched = !which.empty();
      }
      fix_constraint(F, c);
      if (touched) X.alg.rowupd += before + con_size(c);
    }
    for (const Sub &s : subs) r_idx[s.from] = -1;
    // apply_substitution_to_map (:345-396)
    std::vector<uint32_t> linear_id;
    std::vector<std::pair<uint32_t, uint64_t>> first_touch;  // B_alg: a storage row's round is one update
    for (const Sub &sub : subs) {
      if (nl_map[sub.from].empty()) continue;
      std::vector<uint32_t> c_ids = nl_map[sub.from];
      for (uint32_t cid : c_ids) {
        Con &c = storage[cid];
        if (!round_seen[cid]) { round_seen[cid] = 1; first_touch.push_back({cid, con_size(c)}); }
        X.alg.app += sub.to.size();
        apply_substitution(F, c, sub.from, sub.to);
        fix_constraint(F, c);
        if (is_linear(c)) linear_id.push_back(cid);
        for (const Term &t : sub.to) nl_map[t.k].push_back(cid);
      }
    }
    for (const auto &ft : first_touch) {
      X.alg.rowupd += ft.second + con_size(storage[ft.first]);
      round_seen[ft.first] = 0;
    }
    linear.clear();
    for (uint32_t cid : linear_id) {
      linear.push_back(storage[cid]);
      storage[cid] = Con();
    }
    if (no_rounds > 0) no_rounds--;
    apply_round = !linear.empty() && no_rounds > 0;
  }
  for (Con &c : linear) {
    take_signals(c, sig);
    uint32_t id = (uint32_t)storage.size();
    storage.push_back(std::move(c));
    for (uint32_t s : sig) nl_map[s].push_back(id);
  }
  for (Con &c : lconst) {
    fix_constraint(F, c);
    take_signals(c, sig);
    uint32_t id = (uint32_t)storage.size();
    storage.push_back(std::move(c));
    for (uint32_t s : sig) nl_map[s].push_back(id);
  }
  for (Con &c : storage)
    if (!is_empty(c)) out.constraints.push_back(std::move(c));
  for (const Con &c : out.constraints) X.alg.z_out += con_size(c);
  X.alg.r_out = out.constraints.size();
  // rebuild_witness (:101-124): the kept signals, ranked
  out.label_to_wire.assign(S, -1);
  int64_t w = 0;
  for (uint64_t s = 0; s < S; ++s) {
    if (deleted[s]) continue;
    if (!X.forbidden[s] && nl_map[s].empty()) { deleted[s] = 1; continue; }
    out.label_to_wire[s] = w++;
  }
  out.n_wires = (uint64_t)w;
  uint64_t maxin = in.n_pub_out + in.n_pub_in + in.n_priv_in, del_in = 0;
  for (uint64_t s = in.n_pub_out + 1; s <= maxin && s < S; ++s) del_in += deleted[s];
  out.no_private_inputs_witness = in.n_priv_in - del_in;
}

}  // namespace refcpu

// ==================================================================== C API (ctypes)
using namespace refcpu;

static thread_local std::string g_err;
static thread_local uint64_t g_alg[11];  // the last refcpu_simplify's B_alg and its terms (refcpu_last_alg)

static bool load_block(const Ctx &X, const rs_lc &b, std::vector<Con> &rows, int part,
                       bool need_rows) {
  if (need_rows) rows.resize(b.n_rows);
  if (rows.size() != b.n_rows) return false;
  for (uint64_t r = 0; r < b.n_rows; ++r) {
    Map &m = part == 0 ? rows[r].a : part == 1 ? rows[r].b : rows[r].c;
    for (uint64_t e = b.ptr[r]; e < b.ptr[r + 1]; ++e) {
      Fe v;
      memcpy(v.l, b.val + 4 * e, 32);
      if (b.col[e] >= X.max_signal || !X.F.canonical(v.l) || v.is_zero()) return false;
      m.push_back(Term{b.col[e], X.F.to_mont(v)});
    }
    std::sort(m.begin(), m.end(), [](const Term &x, const Term &y) { return x.k < y.k; });
    for (size_t i = 1; i < m.size(); ++i)
      if (m[i].k == m[i - 1].k) return false;
  }
  return true;
}

static void store_block(const Field &F, const std::vector<Con> &rows, int part, rs_lc &b) {
  b.n_rows = rows.size();
  b.ptr = (uint64_t *)malloc(sizeof(uint64_t) * (rows.size() + 1));
  uint64_t nnz = 0;
  for (size_t r = 0; r < rows.size(); ++r) {
    b.ptr[r] = nnz;
    nnz += (part == 0 ? rows[r].a : part == 1 ? rows[r].b : rows[r].c).size();
  }
  b.ptr[rows.size()] = nnz;
  b.nnz = nnz;
  b.col = (uint32_t *)malloc(sizeof(uint32_t) * (nnz ? nnz : 1));
  b.val = (uint64_t *)malloc(32 * (nnz ? nnz : 1));
  uint64_t e = 0;
  for (const Con &c : rows) {
    const Map &m = part == 0 ? c.a : part == 1 ? c.b : c.c;
    for (const Term &t : m) {
      b.col[e] = t.k;
      Fe v = F.from_mont(t.v);
      memcpy(b.val + 4 * e, v.l, 32);
      ++e;
    }
  }
}

extern "C" {

const char *refcpu_last_error(void) { return g_err.c_str(); }

// The last refcpu_simplify's algorithmic bytes (this thread): out[0] = B_alg, out[1..10] = Z_in, Z_out,
// subs, app, rowupd, merges (entries), R_in, R_out, max_signal, w (bytes per entry).
void refcpu_last_alg(uint64_t out[11]) { memcpy(out, g_alg, sizeof g_alg); }

// Runs the canonical restatement on a host rs_input.  *ms = wall time of simplification()
// alone (input already converted to the oracle's in-memory form), n_threads = pool size.
int refcpu_simplify(const rs_input *in, const rs_flags *fl, int n_threads, rs_output **out,
                    double *ms, uint64_t *rounds_out) {
  try {
    Ctx X;
    uint64_t p[4];
    if (in->prime_id == RS_PRIME_CUSTOM) memcpy(p, in->prime, 32);
    else if (in->prime_id < 8) memcpy(p, kPrimes[in->prime_id], 32);
    else { g_err = "unknown prime"; return RS_E_INVALID; }
    X.F.init(p);
    X.max_signal = in->max_signal;
    X.n_threads = n_threads < 1 ? 1 : n_threads;
    X.forbidden.assign(X.max_signal, 0);
    for (uint64_t i = 0; i < in->n_forbidden; ++i)
      if (in->forbidden[i] < X.max_signal) X.forbidden[in->forbidden[i]] = 1;
    if (X.max_signal == 0 || !X.forbidden[0]) { g_err = "signal 0 must be forbidden"; return RS_E_INVALID; }
    X.holder_idx.assign(X.max_signal, -1);
    X.occ.assign(X.max_signal, -1);
    X.noov_idx.assign(X.max_signal, -1);
    X.del.assign(X.max_signal, 0);
    X.sig2cl.assign(X.max_signal, -1);
    Input I;
    I.n_pub_out = in->n_pub_out;
    I.n_pub_in = in->n_pub_in;
    I.n_priv_in = in->n_priv_in;
    bool ok = load_block(X, in->cons_eq, I.cons_eq, 2, true) && load_block(X, in->eq, I.eq, 2, true) &&
              load_block(X, in->linear, I.linear, 2, true) &&
              load_block(X, in->nl_a, I.nonlin, 0, true) && load_block(X, in->nl_b, I.nonlin, 1, false) &&
              load_block(X, in->nl_c, I.nonlin, 2, false);
    if (!ok) { g_err = "invalid input block"; return RS_E_INVALID; }
    Output O;
    for (const rs_lc *b : {&in->cons_eq, &in->eq, &in->linear, &in->nl_a, &in->nl_b, &in->nl_c}) X.alg.z_in += b->nnz;
    X.alg.r_in = in->cons_eq.n_rows + in->eq.n_rows + in->linear.n_rows + in->nl_a.n_rows;
    auto t0 = std::chrono::steady_clock::now();
    simplification(X, I, fl->flag_s, fl->no_rounds, fl->use_old_heuristics != 0, O);
    auto t1 = std::chrono::steady_clock::now();
    {  // refcpu_last_alg: w = 4 + the field's r1cs element size (r1cs_porting.rs:6-10)
      int bits = 256;
      while (bits > 1 && !((p[(bits - 1) / 64] >> ((bits - 1) % 64)) & 1)) --bits;
      const uint64_t fb = bits % 64 == 0 ? bits / 8 : (bits / 64 + 1) * 8, w = 4 + fb;
      const Alg &a = X.alg;
      g_alg[0] = w * (a.z_in + a.z_out + a.subs + a.app + a.rowupd + a.merges) + 8 * (a.r_in + a.r_out) + 8 * X.max_signal;
      g_alg[1] = a.z_in; g_alg[2] = a.z_out; g_alg[3] = a.subs; g_alg[4] = a.app; g_alg[5] = a.rowupd;
      g_alg[6] = a.merges; g_alg[7] = a.r_in; g_alg[8] = a.r_out; g_alg[9] = X.max_signal; g_alg[10] = w;
    }
    if (ms) *ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
    if (rounds_out) *rounds_out = O.rounds;
    rs_output *o = (rs_output *)calloc(1, sizeof(rs_output));
    o->n_constraints = O.constraints.size();
    store_block(X.F, O.constraints, 0, o->a);
    store_block(X.F, O.constraints, 1, o->b);
    store_block(X.F, O.constraints, 2, o->c);
    o->n_labels = X.max_signal;
    o->label_to_wire = (int32_t *)malloc(sizeof(int32_t) * (X.max_signal ? X.max_signal : 1));
    memcpy(o->label_to_wire, O.label_to_wire.data(), sizeof(int32_t) * X.max_signal);
    o->n_wires = O.n_wires;
    o->no_private_inputs_witness = O.no_private_inputs_witness;
    *out = o;
    return RS_OK;
  } catch (const std::exception &e) {
    g_err = e.what();
    return RS_E_INTERNAL;
  }
}

void refcpu_output_free(rs_output *o) {
  if (!o) return;
  for (rs_lc *b : {&o->a, &o->b, &o->c}) { free(b->ptr); free(b->col); free(b->val); }
  free(o->label_to_wire);
  free(o);
}

// Field self-test hook for the F_257 unit tests: op 0 add, 1 sub, 2 mul, 3 div, 4 neg.
int refcpu_field_op(const uint64_t p[4], int op, const uint64_t a[4], const uint64_t b[4], uint64_t r[4]) {
  Field F;
  F.init(p);
  Fe x, y;
  memcpy(x.l, a, 32);
  memcpy(y.l, b, 32);
  x = F.to_mont(x);
  y = F.to_mont(y);
  Fe z;
  switch (op) {
    case 0: z = F.add(x, y); break;
    case 1: z = F.sub(x, y); break;
    case 2: z = F.mul(x, y); break;
    case 3: if (y.is_zero()) return -1; z = F.mul(x, F.inv(y)); break;
    case 4: z = F.neg(x); break;
    default: return -1;
  }
  z = F.from_mont(z);
  memcpy(r, z.l, 32);
  return 0;
}

}  // extern "C"
