// flatten.hpp -- SURVEY 8(f) rank 1: the DAG -> constraint-list flattening that feeds the hot path
// (rs_flatten_dag, include/rs_simplify.h).
//
// The reference walks the component tree twice in the same DFS order: map_tree
// (dag/src/map_to_constraint_list.rs:12-44) appends every instance's local signals to the witness
// list and sorts its offset constraints into the constant-equality / equality / linear lists, and
// the EncodingIterator (constraint_list/src/lib.rs:65-108, state_utils.rs:14-35) yields the
// non-linear ones.  Both are a pre-order of the instance tree, so an instance's position in the
// output is a prefix sum over the instances before it:
//   host   per template: classify its constraints once (offsets do not change the class), their rank
//          and entry prefix within their class; per template the number of instances in its subtree
//          and, per edge, the instances of the earlier siblings' subtrees
//   device the instance tree level by level: a child's DFS index = parent + 1 + the earlier siblings'
//          subtree sizes, its offset = parent's + the edge's in_number (k_fl_expand)
//   device per-instance row / entry / signal counts, one exclusive scan of them (k_fl_counts)
//   device one thread per (instance, template constraint): the row's position, its entries with
//          the instance offset (key 0 stays the constant) (k_fl_emit); custom-gate instances' signals
//          into the forbidden list (k_fl_forbidden)
#pragma once
// (included by engine.hip inside namespace rs, after its scan helpers)

// per-instance counts, scanned together
constexpr int kFlN = 13;  // rows ce, eq, lin, nl | entries ce, eq, lin, nl_a, nl_b, nl_c | pairs | forbidden | locals
struct FlCnt {
  uint64_t v[kFlN];
};
struct FlCntPlus {
  __host__ __device__ FlCnt operator()(const FlCnt &x, const FlCnt &y) const {
    FlCnt r;
    for (int i = 0; i < kFlN; ++i) r.v[i] = x.v[i] + y.v[i];
    return r;
  }
};

struct FlArgs {
  // templates (device copies)
  const uint64_t *cons_off, *local_off, *edge_off, *edge_in, *edge_pre, *lc_ptr[3];
  const uint32_t *locals, *edge_to, *lc_key[3];
  const uint64_t *lc_val[3];
  const uint8_t *custom_gate;
  const uint8_t *cls;      // per template constraint: 0 ce, 1 eq, 2 lin, 3 nl, 4 empty (lin in main only)
  const uint32_t *rank;    // its row rank in its class within the template (lin: empties counted)
  const uint32_t *rank_ne; // lin: the rank among non-empty linear rows
  const uint64_t *zpre;    // its entry prefix within its class in the template: [3 * t + part]
  const uint64_t *tcount;  // per template: kFlN counts for a non-main instance
  uint32_t main_node;
  // instances (DFS order)
  uint32_t *inst_node;
  uint64_t *inst_off;
  uint64_t n_inst;
  FlCnt *cnt, *pre;
  // output blocks: 0 ce, 1 eq, 2 lin, 3 nl_a, 4 nl_b, 5 nl_c
  uint64_t *optr[6];
  uint32_t *okey[6];
  uint64_t *oval[6];
  uint32_t *oforb;
  int *err;
};

// One level of the instance tree: frontier instance i (DFS index fr[i]) gets its children.
__global__ void k_fl_expand(FlArgs A, const uint64_t *fr, uint64_t n_fr, const uint64_t *epos, uint64_t *nfr) {
  for (uint64_t i = gtid(); i < n_fr; i += gstride()) {
    const uint64_t d = fr[i];
    const uint32_t nd = A.inst_node[d];
    const uint64_t off = A.inst_off[d];
    uint64_t w = epos[i];
    for (uint64_t e = A.edge_off[nd]; e < A.edge_off[nd + 1]; ++e, ++w) {
      const uint64_t c = d + 1 + A.edge_pre[e];
      if (c >= A.n_inst) { atomicOr(A.err, 1); continue; }
      A.inst_node[c] = A.edge_to[e];
      A.inst_off[c] = off + A.edge_in[e];
      nfr[w] = c;
    }
  }
}
__global__ void k_fl_edges(FlArgs A, const uint64_t *fr, uint64_t n_fr, uint64_t *ne) {
  for (uint64_t i = gtid(); i < n_fr; i += gstride()) {
    const uint32_t nd = A.inst_node[fr[i]];
    ne[i] = A.edge_off[nd + 1] - A.edge_off[nd];
  }
}

// per instance: its template's counts (main: the linear rows include the empty constraints)
__global__ void k_fl_counts(FlArgs A, const uint64_t *main_count) {
  for (uint64_t i = gtid(); i < A.n_inst; i += gstride()) {
    const uint32_t nd = A.inst_node[i];
    FlCnt c;
    const uint64_t *src = i == 0 ? main_count : A.tcount + (uint64_t)kFlN * nd;
    for (int k = 0; k < kFlN; ++k) c.v[k] = src[k];
    A.cnt[i] = c;
  }
}

__device__ __forceinline__ void fl_copy(const FlArgs &A, int part, uint64_t t, uint64_t off, int ob, uint64_t row, uint64_t z) {
  const uint64_t b = A.lc_ptr[part][t], e = A.lc_ptr[part][t + 1];
  A.optr[ob][row] = z;
  for (uint64_t q = b; q < e; ++q, ++z) {
    const uint32_t k = A.lc_key[part][q];
    A.okey[ob][z] = k == 0 ? 0u : (uint32_t)(k + off);
    const uint64_t *v = A.lc_val[part] + 4 * q;
    uint64_t *o = A.oval[ob] + 4 * z;
    o[0] = v[0];
    o[1] = v[1];
    o[2] = v[2];
    o[3] = v[3];
  }
}

// one thread per (instance, template constraint) pair; pairs of instance i start at pre[i].v[10]
__global__ void k_fl_emit(FlArgs A, uint64_t n_pairs) {
  for (uint64_t x = gtid(); x < n_pairs; x += gstride()) {
    uint64_t lo = 0, hi = A.n_inst;  // last instance whose first pair <= x
    while (hi - lo > 1) {
      const uint64_t mid = (lo + hi) >> 1;
      if (A.pre[mid].v[10] <= x) lo = mid;
      else hi = mid;
    }
    const uint64_t i = lo;
    const uint32_t nd = A.inst_node[i];
    const uint64_t t = A.cons_off[nd] + (x - A.pre[i].v[10]);
    const uint8_t cl = A.cls[t];
    const uint64_t off = A.inst_off[i];
    const FlCnt &P = A.pre[i];
    if (cl == 4 && i != 0) continue;  // Tree::go_to_subtree drops empty constraints
    if (cl == 3) {
      const uint64_t row = P.v[3] + A.rank[t];
      fl_copy(A, 0, t, off, 3, row, P.v[7] + A.zpre[3 * t]);
      fl_copy(A, 1, t, off, 4, row, P.v[8] + A.zpre[3 * t + 1]);
      fl_copy(A, 2, t, off, 5, row, P.v[9] + A.zpre[3 * t + 2]);
    } else {
      const int c = cl == 4 ? 2 : cl;
      const uint64_t row = P.v[c] + (c == 2 && i != 0 ? A.rank_ne[t] : A.rank[t]);
      fl_copy(A, 2, t, off, c, row, P.v[4 + c] + A.zpre[3 * t + 2]);
    }
  }
}

// custom-gate instances: their local signals (with the offset) into the forbidden list
__global__ void k_fl_forbidden(FlArgs A) {
  for (uint64_t i = gtid(); i < A.n_inst; i += gstride()) {
    const uint32_t nd = A.inst_node[i];
    if (!A.custom_gate[nd]) continue;
    uint64_t w = A.pre[i].v[11];
    for (uint64_t q = A.local_off[nd]; q < A.local_off[nd + 1]; ++q) A.oforb[w++] = (uint32_t)(A.locals[q] + A.inst_off[i]);
  }
}
__global__ void k_fl_ptr_end(uint64_t *const *ptrs, const uint64_t *rows, const uint64_t *nnz) {
  if (threadIdx.x < 6) ptrs[threadIdx.x][rows[threadIdx.x]] = nnz[threadIdx.x];
}

// signal_equals_signal's coefficient test: c0 == -c1 (mod p) for canonical non-zero c0, c1
static bool fl_neg_equal(const uint64_t p[4], const uint64_t *c0, const uint64_t *c1) {
  unsigned __int128 carry = 0;
  for (int i = 0; i < 4; ++i) {
    carry += (unsigned __int128)c0[i] + c1[i];
    if ((uint64_t)carry != p[i]) return false;
    carry >>= 64;
  }
  return carry == 0;
}

template <class T>
static T *fl_up(rs_engine *E, const std::string &name, const T *h, uint64_t n) {
  T *d = E->A.get<T>("fl." + name, n);
  if (n) HC(hipMemcpyAsync(d, h, sizeof(T) * n, hipMemcpyHostToDevice, E->st));
  return d;
}

// buf(slot, bytes): the destination of each output array -- slots 3q, 3q + 1, 3q + 2 for block q's ptr,
// col, val (cons_eq, eq, linear, nl_a, nl_b, nl_c), 18 for forbidden (malloc for rs_flatten_dag, the
// engine's page-locked buffers for rs_engine_flatten_dag, whose D2H then runs at link speed)
static void flatten_dag(rs_engine *E, const rs_dag *D, rs_input *in, const std::function<void *(int, size_t)> &buf) {
  hipStream_t st = E->st;
  uint64_t p[4];
  if (D->prime_id == RS_PRIME_CUSTOM) memcpy(p, D->prime, 32);
  else if (D->prime_id < 8) memcpy(p, kPrimes[D->prime_id], 32);
  else throw RsError(RS_E_INVALID, "rs_flatten_dag: unknown prime");
  const uint32_t N = D->n_nodes;
  if (N == 0 || D->main_node >= N) throw RsError(RS_E_INVALID, "rs_flatten_dag: bad main node");
  const uint64_t T = D->cons_off[N];
  for (const rs_lc *b : {&D->a, &D->b, &D->c})
    if (b->n_rows != T) throw RsError(RS_E_INVALID, "rs_flatten_dag: a/b/c row count differs from cons_off");
  const uint64_t n_edges = D->edge_off[N];
  for (uint32_t v = 0; v < N; ++v)
    if (D->cons_off[v] > D->cons_off[v + 1] || D->local_off[v] > D->local_off[v + 1] || D->edge_off[v] > D->edge_off[v + 1])
      throw RsError(RS_E_INVALID, "rs_flatten_dag: offsets decrease");
  for (uint64_t e = 0; e < n_edges; ++e)
    if (D->edge_to[e] >= N) throw RsError(RS_E_INVALID, "rs_flatten_dag: edge to a missing node");
  // the CSR blocks: every row's entries inside [0, nnz) (the host classification and the device
  // copy read col / val up to ptr[T])
  for (const rs_lc *b : {&D->a, &D->b, &D->c}) {
    if (b->ptr[0] != 0 || b->ptr[T] != b->nnz) throw RsError(RS_E_INVALID, "rs_flatten_dag: ptr[0] != 0 or ptr[T] != nnz");
    for (uint64_t t = 0; t < T; ++t)
      if (b->ptr[t] > b->ptr[t + 1]) throw RsError(RS_E_INVALID, "rs_flatten_dag: row pointers decrease");
  }
  // the largest node-local id of every node (its constraints' keys, its own signals)
  std::vector<uint64_t> maxkey(N, 0);
  for (uint32_t v = 0; v < N; ++v) {
    for (uint64_t i = D->local_off[v]; i < D->local_off[v + 1]; ++i) maxkey[v] = std::max<uint64_t>(maxkey[v], D->locals[i]);
    for (const rs_lc *b : {&D->a, &D->b, &D->c})
      for (uint64_t e = b->ptr[D->cons_off[v]]; e < b->ptr[D->cons_off[v + 1]]; ++e) maxkey[v] = std::max<uint64_t>(maxkey[v], b->col[e]);
  }
  // ---- templates (host): classes, ranks and entry prefixes within the class, counts
  std::vector<uint8_t> cls(T);
  std::vector<uint32_t> rank(T), rank_ne(T);
  std::vector<uint64_t> zpre(3 * T), tcount((uint64_t)kFlN * N, 0), mcount(kFlN, 0);
  auto len = [](const rs_lc &b, uint64_t t) { return b.ptr[t + 1] - b.ptr[t]; };
  for (uint32_t v = 0; v < N; ++v) {
    uint64_t *tc = tcount.data() + (uint64_t)kFlN * v;
    uint32_t rows[5] = {0, 0, 0, 0, 0};  // ce, eq, lin (with empties), nl, lin without empties
    uint64_t z[6] = {0, 0, 0, 0, 0, 0};  // ce, eq, lin, nl_a, nl_b, nl_c
    for (uint64_t t = D->cons_off[v]; t < D->cons_off[v + 1]; ++t) {
      const uint64_t na = len(D->a, t), nb = len(D->b, t), nc = len(D->c, t);
      uint8_t c;
      if (na || nb) {
        c = 3;
      } else if (nc == 0) {
        c = 4;  // empty: linear (is_linear), but only main keeps it
      } else {
        const uint32_t *k = D->c.col + D->c.ptr[t];
        bool has0 = false;
        for (uint64_t q = 0; q < nc; ++q) has0 |= k[q] == 0;
        if ((has0 && nc == 2) || (!has0 && nc == 1)) c = 0;  // signal_equals_constant (algebra.rs:1362-1372)
        else if (!has0 && nc == 2 && fl_neg_equal(p, D->c.val + 4 * D->c.ptr[t], D->c.val + 4 * (D->c.ptr[t] + 1)))
          c = 1;  // signal_equals_signal (:1346-1360)
        else c = 2;
      }
      cls[t] = c;
      const int rc = c == 4 ? 2 : c;
      rank[t] = rows[rc]++;
      rank_ne[t] = rows[4];
      if (c == 2) rows[4]++;
      if (c == 3) {
        zpre[3 * t] = z[3];
        zpre[3 * t + 1] = z[4];
        zpre[3 * t + 2] = z[5];
        z[3] += na;
        z[4] += nb;
        z[5] += nc;
      } else {
        zpre[3 * t] = zpre[3 * t + 1] = 0;
        zpre[3 * t + 2] = z[rc];
        z[rc] += nc;
      }
    }
    tc[0] = rows[0];
    tc[1] = rows[1];
    tc[2] = rows[4];
    tc[3] = rows[3];
    for (int k = 0; k < 6; ++k) tc[4 + k] = z[k];
    tc[10] = D->cons_off[v + 1] - D->cons_off[v];
    tc[11] = D->custom_gate[v] ? D->local_off[v + 1] - D->local_off[v] : 0;
    tc[12] = D->local_off[v + 1] - D->local_off[v];
    if (v == D->main_node) {
      for (int k = 0; k < kFlN; ++k) mcount[k] = tc[k];
      mcount[2] = rows[2];  // main keeps its empty constraints in the linear list
    }
  }
  // subtree sizes (instances) in reverse topological order; per edge, the earlier siblings' subtrees
  std::vector<uint64_t> sz(N, 0), epre(n_edges);
  std::vector<uint32_t> post;  // DFS post-order of the nodes reachable from main
  {
    std::vector<uint8_t> state(N, 0);  // 0 new, 1 on the stack, 2 done
    std::vector<std::pair<uint32_t, uint64_t>> stk;
    stk.push_back({D->main_node, D->edge_off[D->main_node]});
    state[D->main_node] = 1;
    while (!stk.empty()) {
      auto &top = stk.back();
      const uint32_t v = top.first;
      if (top.second < D->edge_off[v + 1]) {
        const uint32_t w = D->edge_to[top.second++];
        if (state[w] == 1) throw RsError(RS_E_INVALID, "rs_flatten_dag: the graph has a cycle");
        if (state[w] == 0) {
          state[w] = 1;
          stk.push_back({w, D->edge_off[w]});
        }
        continue;
      }
      uint64_t s = 1;
      for (uint64_t e = D->edge_off[v]; e < D->edge_off[v + 1]; ++e) {
        epre[e] = s - 1;
        s += sz[D->edge_to[e]];
        if (s > (1ull << 40)) throw RsError(RS_E_INVALID, "rs_flatten_dag: too many instances");
      }
      sz[v] = s;
      state[v] = 2;
      post.push_back(v);
      stk.pop_back();
    }
  }
  const uint64_t n_inst = sz[D->main_node];
  {  // the largest instance offset of every reachable node (reverse post-order is topological):
     // every offset id (offset + local id) must stay below the engine's 2^31 signal bound
    std::vector<uint64_t> maxoff(N, 0);
    for (size_t i = post.size(); i-- > 0;) {
      const uint32_t v = post[i];
      if (maxoff[v] + maxkey[v] >= (1ull << 31)) throw RsError(RS_E_INVALID, "rs_flatten_dag: signal ids overflow 2^31");
      for (uint64_t e = D->edge_off[v]; e < D->edge_off[v + 1]; ++e) {
        if (D->edge_in[e] >= (1ull << 31)) throw RsError(RS_E_INVALID, "rs_flatten_dag: signal ids overflow 2^31");
        maxoff[D->edge_to[e]] = std::max(maxoff[D->edge_to[e]], maxoff[v] + D->edge_in[e]);
      }
    }
  }
  // ---- device: upload the templates, expand the instance tree level by level
  FlArgs A{};
  A.cons_off = fl_up(E, "cons_off", D->cons_off, N + 1);
  A.local_off = fl_up(E, "local_off", D->local_off, N + 1);
  A.edge_off = fl_up(E, "edge_off", D->edge_off, N + 1);
  A.edge_in = fl_up(E, "edge_in", D->edge_in, n_edges);
  A.edge_pre = fl_up(E, "edge_pre", epre.data(), n_edges);
  A.edge_to = fl_up(E, "edge_to", D->edge_to, n_edges);
  A.locals = fl_up(E, "locals", D->locals, D->local_off[N]);
  A.custom_gate = fl_up(E, "cgate", D->custom_gate, N);
  const rs_lc *lcs[3] = {&D->a, &D->b, &D->c};
  for (int q = 0; q < 3; ++q) {
    const std::string nm = std::string("lc") + (char)('a' + q);
    A.lc_ptr[q] = fl_up(E, nm + ".ptr", lcs[q]->ptr, T + 1);
    A.lc_key[q] = fl_up(E, nm + ".key", lcs[q]->col, lcs[q]->nnz);
    A.lc_val[q] = fl_up(E, nm + ".val", lcs[q]->val, 4 * lcs[q]->nnz);
  }
  A.cls = fl_up(E, "cls", cls.data(), T);
  A.rank = fl_up(E, "rank", rank.data(), T);
  A.rank_ne = fl_up(E, "rank_ne", rank_ne.data(), T);
  A.zpre = fl_up(E, "zpre", zpre.data(), 3 * T);
  A.tcount = fl_up(E, "tcount", tcount.data(), (uint64_t)kFlN * N);
  const uint64_t *d_mcount = fl_up(E, "mcount", mcount.data(), kFlN);
  A.main_node = D->main_node;
  A.n_inst = n_inst;
  A.inst_node = E->A.get<uint32_t>("fl.inst_node", n_inst);
  A.inst_off = E->A.get<uint64_t>("fl.inst_off", n_inst);
  A.err = E->A.get<int>("fl.err", 1);
  HC(hipMemsetAsync(A.err, 0, 4, st));
  {
    const uint64_t zero = 0;
    HC(hipMemcpyAsync(A.inst_node, &D->main_node, 4, hipMemcpyHostToDevice, st));
    HC(hipMemcpyAsync(A.inst_off, &zero, 8, hipMemcpyHostToDevice, st));
    uint64_t *fr = E->A.get<uint64_t>("fl.fr0", n_inst), *nfr = E->A.get<uint64_t>("fl.fr1", n_inst);
    uint64_t *ne = E->A.get<uint64_t>("fl.ne", n_inst), *epos = E->A.get<uint64_t>("fl.epos", n_inst);
    HC(hipMemcpyAsync(fr, &zero, 8, hipMemcpyHostToDevice, st));
    uint64_t n_fr = 1, done = 1;
    while (n_fr) {
      launch(st, k_fl_edges, n_fr, A, (const uint64_t *)fr, n_fr, ne);
      const uint64_t n_next = excl_scan_u64(E, ne, epos, n_fr, "fl");
      if (n_next) launch(st, k_fl_expand, n_fr, A, (const uint64_t *)fr, n_fr, (const uint64_t *)epos, nfr);
      std::swap(fr, nfr);
      n_fr = n_next;
      done += n_next;
      if (done > n_inst) throw RsError(RS_E_INTERNAL, "rs_flatten_dag: instance count mismatch");
    }
  }
  // ---- per-instance counts and their prefix sums
  A.cnt = E->A.get<FlCnt>("fl.cnt", n_inst);
  A.pre = E->A.get<FlCnt>("fl.pre", n_inst);
  launch(st, k_fl_counts, n_inst, A, d_mcount);
  size_t tb = 0;
  FlCnt zero{};
  HC(rocprim::exclusive_scan(nullptr, tb, A.cnt, A.pre, zero, (size_t)n_inst, FlCntPlus(), st));
  void *tmp = E->A.get<uint8_t>("fl.scan", tb);
  HC(rocprim::exclusive_scan(tmp, tb, A.cnt, A.pre, zero, (size_t)n_inst, FlCntPlus(), st));
  FlCnt last_c, last_p, tot;
  HC(hipMemcpyAsync(&last_c, A.cnt + n_inst - 1, sizeof(FlCnt), hipMemcpyDeviceToHost, st));
  HC(hipMemcpyAsync(&last_p, A.pre + n_inst - 1, sizeof(FlCnt), hipMemcpyDeviceToHost, st));
  HC(hipStreamSynchronize(st));
  for (int k = 0; k < kFlN; ++k) tot.v[k] = last_c.v[k] + last_p.v[k];
  if (tot.v[12] + 1 >= (1ull << 31)) throw RsError(RS_E_INVALID, "rs_flatten_dag: 2^31 signals or more");
  // ---- emit the blocks
  const uint64_t rows[6] = {tot.v[0], tot.v[1], tot.v[2], tot.v[3], tot.v[3], tot.v[3]};
  const uint64_t nnz[6] = {tot.v[4], tot.v[5], tot.v[6], tot.v[7], tot.v[8], tot.v[9]};
  for (int q = 0; q < 6; ++q) {
    const std::string nm = "fl.o" + std::to_string(q);
    A.optr[q] = E->A.get<uint64_t>(nm + ".ptr", rows[q] + 1);
    A.okey[q] = E->A.get<uint32_t>(nm + ".key", nnz[q]);
    A.oval[q] = E->A.get<uint64_t>(nm + ".val", 4 * nnz[q]);
  }
  A.oforb = E->A.get<uint32_t>("fl.forb", tot.v[11]);
  if (tot.v[10]) launch(st, k_fl_emit, tot.v[10], A, tot.v[10]);
  if (tot.v[11]) launch(st, k_fl_forbidden, n_inst, A);
  uint64_t *const hp[6] = {A.optr[0], A.optr[1], A.optr[2], A.optr[3], A.optr[4], A.optr[5]};  // alive until the sync
  {
    uint64_t *const *dp = fl_up(E, "ptrs", hp, 6);
    const uint64_t *drows = fl_up(E, "rows", rows, 6), *dnnz = fl_up(E, "nnz", nnz, 6);
    hipLaunchKernelGGL(k_fl_ptr_end, dim3(1), dim3(64), 0, st, dp, drows, dnnz);
    HC(hipGetLastError());
  }
  int err = 0;
  HC(hipMemcpyAsync(&err, A.err, 4, hipMemcpyDeviceToHost, st));
  HC(hipStreamSynchronize(st));
  if (err) throw RsError(RS_E_INTERNAL, "rs_flatten_dag: instance expansion out of range");
  // ---- the rs_input
  in->prime_id = D->prime_id;
  memcpy(in->prime, p, 32);
  in->max_signal = tot.v[12] + 1;  // the witness list: signal 0 and every instance's locals
  in->n_pub_out = D->n_pub_out;
  in->n_pub_in = D->n_pub_in;
  in->n_priv_in = D->n_priv_in;
  rs_lc *outs[6] = {&in->cons_eq, &in->eq, &in->linear, &in->nl_a, &in->nl_b, &in->nl_c};
  for (int q = 0; q < 6; ++q) {
    rs_lc &o = *outs[q];
    o.n_rows = rows[q];
    o.nnz = nnz[q];
    o.ptr = (uint64_t *)buf(3 * q, 8 * (rows[q] + 1));
    o.col = (uint32_t *)buf(3 * q + 1, 4 * std::max<uint64_t>(nnz[q], 1));
    o.val = (uint64_t *)buf(3 * q + 2, 32 * std::max<uint64_t>(nnz[q], 1));
    HC(hipMemcpyAsync(o.ptr, A.optr[q], 8 * (rows[q] + 1), hipMemcpyDeviceToHost, st));
    if (nnz[q]) {
      HC(hipMemcpyAsync(o.col, A.okey[q], 4 * nnz[q], hipMemcpyDeviceToHost, st));
      HC(hipMemcpyAsync(o.val, A.oval[q], 32 * nnz[q], hipMemcpyDeviceToHost, st));
    }
  }
  std::vector<uint32_t> forb(D->forbidden, D->forbidden + D->n_forbidden);
  forb.resize(D->n_forbidden + tot.v[11]);
  if (tot.v[11]) HC(hipMemcpyAsync(forb.data() + D->n_forbidden, A.oforb, 4 * tot.v[11], hipMemcpyDeviceToHost, st));
  HC(hipStreamSynchronize(st));
  std::sort(forb.begin(), forb.end());
  forb.erase(std::unique(forb.begin(), forb.end()), forb.end());
  in->n_forbidden = forb.size();
  in->forbidden = (uint32_t *)buf(18, 4 * std::max<size_t>(forb.size(), 1));
  if (!forb.empty()) memcpy(in->forbidden, forb.data(), 4 * forb.size());
}
