// elim_trace.cpp -- statistics of process_4's ordered loop on the largest clusters of a synthetic
// circuit (analysis tool; links the CPU oracle with its trace hooks switched on).
//   g++ -O2 -std=c++17 -o /tmp/elim_trace tools/elim_trace.cpp circom_cvm_amd/csrc/synth.cpp \
//       circom_cvm_amd/csrc/host_common.cpp circom_cvm_amd/csrc/r1cs_io.cpp -lpthread
//   /tmp/elim_trace <kind> <rows> [seed] [min_cluster]
#include <cstdint>
#include <cstdio>
#include <map>
#include <mutex>
#include <set>
#include <vector>

namespace tr {
inline size_t tr_bucket(size_t x) { size_t b = 0; while ((1ull << b) < x + 1) ++b; return b; }
struct Cl {
  bool on = false;
  size_t rows = 0, uniq = 0, row_i = 0, merges = 0, inserts = 0, lefts = 0;
  std::vector<long> hrow;                // holder index -> loop row it was created at (-1: uniques)
  std::vector<size_t> hlen;
  std::set<uint32_t> row_keys;           // keys of the popped row (before any merge)
  size_t cur_merges = 0;
  std::map<size_t, size_t> merges_per_row, age_hist, hlen_hist, wlen_hist, sum_hist;
  size_t over64 = 0, max_sum = 0, max_row = 0, nonempty_rows = 0, over128 = 0, len_over64 = 0;
  bool p3 = false, agg = false;
  size_t from_row = 0, introduced = 0, uniq_holder = 0, sum_h = 0, sum_w = 0, max_chain = 0;
  // speculation distance: non-empty loop rows back to the latest row whose pivot this row's work saw
  std::map<uint32_t, long> del_at;       // signal -> non-empty loop row index that deleted it
  long ne_i = -1;                        // current non-empty row index
  long dep = -1;                         // latest creator row seen by the current row
  std::map<size_t, size_t> dist_hist;
  // discovery depth: merges grouped into levels (a key the row starts with: level 0; a key a merge at
  // level L brings in: L + 1) -- the dependent holder fetches of a loop that fetches every deleted
  // key's holder as soon as the key is known
  std::map<uint32_t, int> lvl;
  int last_lvl = -1, row_depth = 0;
  size_t depth_sum = 0;
  std::map<size_t, size_t> depth_hist;
  void depth_end() {
    if (row_depth) { depth_hist[row_depth]++; depth_sum += row_depth; }
    row_depth = 0;
    last_lvl = -1;
    lvl.clear();
  }
  template <class W> void see(const W &w) {
    for (const auto &t : w) {
      auto it = del_at.find(t.k);
      if (it != del_at.end() && it->second > dep) dep = it->second;
    }
  }
  void row_end() {
    if (ne_i < 0) return;
    dist_hist[dep < 0 ? 99 : tr_bucket((size_t)(ne_i - dep))]++;
  }
};
thread_local Cl C;
size_t g_min = 2000;
size_t g_tail_min = 32;  // clusters in [g_tail_min, g_min): one aggregate line (the "tail")
struct Agg { size_t clusters = 0, rows = 0, merges = 0, over64 = 0, over128 = 0, len_over64 = 0; std::map<size_t, size_t> sum_hist; };
Agg g_agg[2];  // [0] process_4, [1] process_3
std::mutex g_mu;
inline size_t bucket(size_t x) { size_t b = 0; while ((1ull << b) < x + 1) ++b; return b; }
}  // namespace tr

#define RC_TRACE_CLUSTER3(n_rows)                                                   \
  do {                                                                              \
    tr::C = tr::Cl();                                                               \
    tr::C.p3 = true;                                                                \
    tr::C.agg = (n_rows) >= tr::g_tail_min;                                         \
    tr::C.on = tr::C.agg;                                                           \
    tr::C.rows = (n_rows);                                                          \
  } while (0)
#define RC_TRACE_CLUSTER(n_rows, n_uniq)                                            \
  do {                                                                              \
    tr::C = tr::Cl();                                                               \
    tr::C.agg = (n_rows) >= tr::g_tail_min && (n_rows) < tr::g_min;                 \
    tr::C.on = (n_rows) >= tr::g_tail_min;                                          \
    tr::C.rows = (n_rows);                                                          \
    tr::C.uniq = (n_uniq);                                                          \
  } while (0)
#define RC_TRACE_ROW(len)                                                           \
  do {                                                                              \
    if (!tr::C.on) break;                                                           \
    if (tr::C.row_i) { tr::C.merges_per_row[tr::C.cur_merges]++; }                  \
    if (!work.empty()) { tr::C.row_end(); tr::C.ne_i++; tr::C.dep = -1; tr::C.nonempty_rows++; \
      tr::C.max_row = std::max<size_t>(tr::C.max_row, work.size());                 \
      if (work.size() > 64) tr::C.len_over64++; }                                   \
    tr::C.max_chain = std::max(tr::C.max_chain, tr::C.cur_merges);                  \
    tr::C.cur_merges = 0;                                                           \
    tr::C.row_i++;                                                                  \
    tr::C.row_keys.clear();                                                         \
    for (const Term &t_ : work) tr::C.row_keys.insert(t_.k);                        \
    tr::C.depth_end();                                                              \
    for (const Term &t_ : work) tr::C.lvl[t_.k] = 0;                                \
  } while (0)
#define RC_TRACE_MERGE(key, wlen, hidx, hl)                                          \
  do {                                                                              \
    if (!tr::C.on) break;                                                           \
    tr::C.merges++;                                                                 \
    tr::C.see(work);                                                                \
    tr::C.cur_merges++;                                                             \
    long hr_ = tr::C.hrow[hidx];                                                    \
    if (hr_ < 0) tr::C.uniq_holder++;                                               \
    else tr::C.age_hist[tr::bucket(tr::C.row_i - (size_t)hr_)]++;                   \
    tr::C.hlen_hist[tr::bucket(hl)]++;                                              \
    tr::C.wlen_hist[tr::bucket(wlen)]++;                                            \
    tr::C.sum_hist[tr::bucket((wlen) + (hl))]++;                                    \
    if ((wlen) + (hl) > 65) tr::C.over64++;                                         \
    if ((wlen) + (hl) > 129) tr::C.over128++;                                       \
    tr::C.max_sum = std::max<size_t>(tr::C.max_sum, (wlen) + (hl));                 \
    tr::C.sum_h += (hl);                                                            \
    tr::C.sum_w += (wlen);                                                          \
    if (tr::C.row_keys.count(key)) tr::C.from_row++; else tr::C.introduced++;       \
    for (const Term &t_ : work) tr::C.lvl.emplace(t_.k, tr::C.last_lvl + 1);        \
    tr::C.last_lvl = tr::C.lvl[key];                                                \
    tr::C.row_depth = std::max(tr::C.row_depth, tr::C.last_lvl + 1);                \
  } while (0)
#define RC_TRACE_INSERT(key, hidx, len)                                             \
  do {                                                                              \
    if (!tr::C.on) break;                                                           \
    tr::C.inserts++;                                                                \
    if (tr::C.row_i) { tr::C.see(work); tr::C.del_at[key] = tr::C.ne_i; }           \
    tr::C.hrow.push_back(tr::C.row_i ? (long)tr::C.row_i : -1L);                    \
    tr::C.hlen.push_back(len);                                                      \
  } while (0)
#define RC_TRACE_LEFT(len)                                                          \
  do {                                                                              \
    if (tr::C.on) { tr::C.lefts++; tr::C.see(work); }                               \
  } while (0)
#define RC_TRACE_END()                                                              \
  do {                                                                              \
    if (!tr::C.on) break;                                                           \
    if (tr::C.agg) {                                                                \
      std::lock_guard<std::mutex> lk_(tr::g_mu);                                    \
      tr::Agg &a_ = tr::g_agg[tr::C.p3 ? 1 : 0];                                    \
      a_.clusters++; a_.rows += tr::C.nonempty_rows; a_.merges += tr::C.merges;     \
      a_.over64 += tr::C.over64; a_.over128 += tr::C.over128;                       \
      a_.len_over64 += tr::C.len_over64;                                            \
      for (auto &kv : tr::C.sum_hist) a_.sum_hist[kv.first] += kv.second;           \
      break;                                                                        \
    }                                                                               \
    tr::C.merges_per_row[tr::C.cur_merges]++;                                       \
    tr::C.row_end();                                                                \
    tr::C.depth_end();                                                              \
    std::lock_guard<std::mutex> lk_(tr::g_mu);                                      \
    auto &c_ = tr::C;                                                               \
    printf("cluster rows=%zu uniq=%zu loop_rows=%zu inserts=%zu lefts=%zu merges=%zu " \
           "max_merges_per_row=%zu mean_hlen=%.1f mean_wlen=%.1f from_row=%zu introduced=%zu " \
           "uniq_holder=%zu\n",                                                     \
           c_.rows, c_.uniq, c_.row_i, c_.inserts, c_.lefts, c_.merges, c_.max_chain, \
           c_.merges ? (double)c_.sum_h / c_.merges : 0.0,                          \
           c_.merges ? (double)c_.sum_w / c_.merges : 0.0, c_.from_row, c_.introduced, \
           c_.uniq_holder);                                                         \
    printf("  merges/row:");                                                        \
    for (auto &kv : c_.merges_per_row) printf(" %zu:%zu", kv.first, kv.second);     \
    printf("\n  holder age (log2 rows):");                                          \
    for (auto &kv : c_.age_hist) printf(" %zu:%zu", kv.first, kv.second);           \
    printf("\n  holder len (log2):");                                               \
    for (auto &kv : c_.hlen_hist) printf(" %zu:%zu", kv.first, kv.second);          \
    printf("\n  spec distance (log2 non-empty rows; 99 = none):");                  \
    for (auto &kv : c_.dist_hist) printf(" %zu:%zu", kv.first, kv.second);          \
    printf("\n  len+rl (log2):");                                                   \
    for (auto &kv : c_.sum_hist) printf(" %zu:%zu", kv.first, kv.second);           \
    printf("\n  nonempty=%zu over64=%zu max_sum=%zu max_row=%zu", c_.nonempty_rows, c_.over64, c_.max_sum, c_.max_row); \
    printf("\n  work len (log2):");                                                 \
    for (auto &kv : c_.wlen_hist) printf(" %zu:%zu", kv.first, kv.second);          \
    printf("\n  discovery depth (levels per row; sum %zu):", c_.depth_sum);          \
    for (auto &kv : c_.depth_hist) printf(" %zu:%zu", kv.first, kv.second);         \
    printf("\n");                                                                   \
  } while (0)

#include "../oracle/refcpu.cpp"

int main(int argc, char **argv) {
  unsigned kind = argc > 1 ? (unsigned)atoi(argv[1]) : 0;
  uint64_t rows = argc > 2 ? strtoull(argv[2], nullptr, 10) : 10000000ull;
  uint64_t seed = argc > 3 ? strtoull(argv[3], nullptr, 10) : 42ull;
  if (argc > 4) tr::g_min = strtoull(argv[4], nullptr, 10);
  rs_input *in = nullptr;
  if (rs_synth(kind, rows, seed, 0, &in) != 0) { fprintf(stderr, "synth failed\n"); return 1; }
  rs_flags fl{};
  fl.no_rounds = ~0ull;
  rs_output *out = nullptr;
  int rc = refcpu_simplify(in, &fl, 8, &out, nullptr, nullptr);
  printf("rc=%d\n", rc);
  for (int q = 0; q < 2; ++q) {
    const tr::Agg &a = tr::g_agg[q];
    printf("tail %s: clusters=%zu rows=%zu merges=%zu len+rl>64: %zu  >128: %zu  rows>64: %zu  len+rl(log2):", q ? "p3" : "p4",
           a.clusters, a.rows, a.merges, a.over64, a.over128, a.len_over64);
    for (auto &kv : a.sum_hist) printf(" %zu:%zu", kv.first, kv.second);
    printf("\n");
  }
  return rc;
}
