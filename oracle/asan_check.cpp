// asan_check.cpp -- TEST INFRASTRUCTURE (SURVEY §5 "ASan/UBSan CPU-oracle build").
//
// Built by `make -C oracle asan` with -fsanitize=address,undefined together with the oracle
// (refcpu.cpp) and the host-side pieces of the product library that need no GPU: the --O0 reader,
// the .r1cs/.sym/.json writers and the synthetic generator (circom_cvm_amd/csrc/{r1cs_io,synth,
// host_common}.cpp).  It drives them over every generator kind, several primes and flag levels,
// checks that the oracle's output does not depend on its thread count, round-trips the writer
// through the reader, and feeds the reader every truncation of a file plus corrupted headers.  Any
// sanitizer report aborts with a non-zero status; tests/test_oracle.py::test_asan_ubsan_check runs it.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../include/rs_simplify.h"

extern "C" {
int refcpu_simplify(const rs_input *in, const rs_flags *fl, int n_threads, rs_output **out, double *ms,
                    uint64_t *rounds_out);
void refcpu_output_free(rs_output *o);
const char *refcpu_last_error(void);
}

static int g_fail = 0;
#define CHECK(c, ...)                               \
  do {                                              \
    if (!(c)) {                                     \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);                 \
      fprintf(stderr, "\n");                        \
      ++g_fail;                                     \
    }                                               \
  } while (0)

static bool same_lc(const rs_lc &x, const rs_lc &y) {
  if (x.n_rows != y.n_rows || x.nnz != y.nnz) return false;
  if (memcmp(x.ptr, y.ptr, 8 * (x.n_rows + 1))) return false;
  return x.nnz == 0 || (!memcmp(x.col, y.col, 4 * x.nnz) && !memcmp(x.val, y.val, 32 * x.nnz));
}
static bool same_out(const rs_output *x, const rs_output *y) {
  return x->n_constraints == y->n_constraints && same_lc(x->a, y->a) && same_lc(x->b, y->b) && same_lc(x->c, y->c) &&
         x->n_wires == y->n_wires && x->no_private_inputs_witness == y->no_private_inputs_witness &&
         !memcmp(x->label_to_wire, y->label_to_wire, 4 * x->n_labels);
}
static std::vector<uint8_t> slurp(const std::string &p) {
  std::vector<uint8_t> b;
  FILE *f = fopen(p.c_str(), "rb");
  if (!f) return b;
  int c;
  while ((c = fgetc(f)) != EOF) b.push_back((uint8_t)c);
  fclose(f);
  return b;
}
static void dump(const std::string &p, const uint8_t *d, size_t n) {
  FILE *f = fopen(p.c_str(), "wb");
  if (n) fwrite(d, 1, n, f);
  fclose(f);
}

int main(int argc, char **argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  struct Case {
    uint32_t kind;
    uint64_t rows;
    uint32_t prime;
  };
  const Case cases[] = {{0, 3000, 0}, {1, 2000, 1}, {2, 2500, 0}, {3, 4000, 3}, {4, 3000, 2}, {0, 1500, 7}};
  for (const Case &cs : cases) {
    rs_input *in = nullptr;
    CHECK(rs_synth(cs.kind, cs.rows, 11 + cs.kind, cs.prime, &in) == 0, "rs_synth: %s", rs_last_error());
    if (!in) continue;
    for (int level = 0; level < 3; ++level) {
      rs_flags fl;
      memset(&fl, 0, sizeof(fl));
      fl.flag_s = level == 0;
      fl.no_rounds = level == 0 ? 0 : (level == 1 ? 2 : UINT64_MAX);
      fl.emit_substitution_log = level == 2;
      rs_output *o1 = nullptr, *o3 = nullptr;
      double ms = 0;
      uint64_t rounds = 0;
      CHECK(refcpu_simplify(in, &fl, 1, &o1, &ms, &rounds) == 0, "refcpu: %s", refcpu_last_error());
      CHECK(refcpu_simplify(in, &fl, 3, &o3, &ms, &rounds) == 0, "refcpu: %s", refcpu_last_error());
      if (!o1 || !o3) continue;
      CHECK(same_out(o1, o3), "kind %u level %d: thread count changes the output", cs.kind, level);
      const std::string r1 = dir + "/asan.r1cs", js = dir + "/asan.json", sj = dir + "/asan_sub.json";
      CHECK(rs_write_r1cs(r1.c_str(), in, o1) == 0, "write r1cs: %s", rs_last_error());
      CHECK(rs_write_constraints_json(js.c_str(), o1) == 0, "write json: %s", rs_last_error());
      if (fl.emit_substitution_log) CHECK(rs_write_substitution_json(sj.c_str(), o1) == 0, "write sub json");
      rs_input *back = nullptr;
      CHECK(rs_read_r1cs_o0(r1.c_str(), &back) == 0, "re-read: %s", rs_last_error());
      if (back) {
        CHECK(back->nl_a.n_rows + back->cons_eq.n_rows + back->eq.n_rows + back->linear.n_rows == o1->n_constraints,
              "re-read row count");
        rs_input_free(back);
      }
      refcpu_output_free(o1);
      refcpu_output_free(o3);
    }
    rs_input_free(in);
  }
  // the reader on every prefix of a small file and on corrupted section sizes / counts
  {
    rs_input *in = nullptr;
    CHECK(rs_synth(0, 200, 5, 0, &in) == 0, "rs_synth small");
    rs_flags fl;
    memset(&fl, 0, sizeof(fl));
    fl.no_rounds = UINT64_MAX;
    rs_output *o = nullptr;
    double ms;
    uint64_t rounds;
    CHECK(refcpu_simplify(in, &fl, 1, &o, &ms, &rounds) == 0, "refcpu small");
    const std::string r1 = dir + "/asan_small.r1cs", t = dir + "/asan_trunc.r1cs";
    CHECK(rs_write_r1cs(r1.c_str(), in, o) == 0, "write small");
    const std::vector<uint8_t> full = slurp(r1);
    for (size_t n = 0; n < full.size(); n += (n < 64 ? 1 : 37)) {
      dump(t, full.data(), n);
      rs_input *x = nullptr;
      const int rc = rs_read_r1cs_o0(t.c_str(), &x);
      CHECK(rc == RS_E_INVALID, "prefix %zu: rc %d", n, rc);
      if (x) rs_input_free(x);
    }
    for (size_t pos = 8; pos + 8 <= full.size() && pos < 400; pos += 4) {
      std::vector<uint8_t> bad = full;
      const uint32_t big = 0xfffffff7u;
      memcpy(&bad[pos], &big, 4);
      dump(t, bad.data(), bad.size());
      rs_input *x = nullptr;
      (void)rs_read_r1cs_o0(t.c_str(), &x);  // any status; the sanitizers judge the accesses
      if (x) rs_input_free(x);
    }
    refcpu_output_free(o);
    rs_input_free(in);
  }
  if (g_fail) {
    fprintf(stderr, "asan_check: %d failure(s)\n", g_fail);
    return 1;
  }
  printf("asan_check: OK\n");
  return 0;
}
