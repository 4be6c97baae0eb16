// cli.cpp -- circom-simplify: the drop-in seam exercised from files.
//
//   circom-simplify <in_O0.r1cs> [<in_O0.sym>] --O1|--O2|--O2round N
//                   [--use_old_simplification_heuristics] [--json] [--simplification_substitution]
//                   [--device D] -o <out_prefix>
//
// Reads an --O0 export (which losslessly holds what simplification() consumes, SURVEY CS-4),
// runs the GPU back end and writes <out_prefix>.r1cs (+ .sym), like `circom --r1cs --sym` at the
// given level (circom/src/input_user.rs:286-306 for the flag semantics); --json adds
// <out_prefix>_constraints.json and --simplification_substitution <out_prefix>_substitutions.json
// (the file names circom derives from its output base, input_user.rs).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/rs_simplify.h"

int main(int argc, char **argv) {
  const char *in_r1cs = nullptr, *in_sym = nullptr;
  std::string out;
  bool json = false;
  rs_flags fl;
  memset(&fl, 0, sizeof(fl));
  fl.flag_s = 1;  // --O1 is circom's default since 2.2.0 (input_user.rs:304)
  fl.no_rounds = 0;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--O1") { fl.flag_s = 1; fl.no_rounds = 0; }
    else if (a == "--O2") { fl.flag_s = 0; fl.no_rounds = UINT64_MAX; }
    else if (a == "--O2round" && i + 1 < argc) {
      uint64_t n = strtoull(argv[++i], nullptr, 10);
      if (n == 0) { fl.flag_s = 1; fl.no_rounds = 0; }
      else { fl.flag_s = 0; fl.no_rounds = n; }
    } else if (a == "--use_old_simplification_heuristics") fl.use_old_heuristics = 1;
    else if (a == "--json") json = true;
    else if (a == "--simplification_substitution") fl.emit_substitution_log = 1;
    else if (a == "--device" && i + 1 < argc) fl.device = atoi(argv[++i]);
    else if (a == "-o" && i + 1 < argc) out = argv[++i];
    else if (!in_r1cs) in_r1cs = argv[i];
    else if (!in_sym) in_sym = argv[i];
    else { fprintf(stderr, "unexpected argument %s\n", argv[i]); return 2; }
  }
  if (!in_r1cs || out.empty()) {
    fprintf(stderr, "usage: circom-simplify in_O0.r1cs [in_O0.sym] --O1|--O2|--O2round N [--json] "
                    "[--simplification_substitution] -o out_prefix\n");
    return 2;
  }
  rs_input *in = nullptr;
  if (rs_read_r1cs_o0(in_r1cs, &in)) { fprintf(stderr, "error: %s\n", rs_last_error()); return 1; }
  rs_output *o = nullptr;
  auto t0 = std::chrono::steady_clock::now();
  int rc = rs_simplify(in, &fl, &o);
  auto t1 = std::chrono::steady_clock::now();
  if (rc) { fprintf(stderr, "error %d: %s\n", rc, rs_last_error()); rs_input_free(in); return 1; }
  if (rs_write_r1cs_gates((out + ".r1cs").c_str(), in, o, in_r1cs)) { fprintf(stderr, "error: %s\n", rs_last_error()); return 1; }
  if (in_sym && rs_write_sym(in_sym, (out + ".sym").c_str(), o)) { fprintf(stderr, "error: %s\n", rs_last_error()); return 1; }
  if (json && rs_write_constraints_json((out + "_constraints.json").c_str(), o)) { fprintf(stderr, "error: %s\n", rs_last_error()); return 1; }
  if (fl.emit_substitution_log && rs_write_substitution_json((out + "_substitutions.json").c_str(), o)) {
    fprintf(stderr, "error: %s\n", rs_last_error());
    return 1;
  }
  // constraint_writers/src/log_writer.rs:24-47
  uint64_t nl = 0, l = 0;
  rs_rows ia, ib;
  rs_rows_begin(o, 0, &ia);
  rs_rows_begin(o, 1, &ib);
  for (uint64_t r = 0; r < o->n_constraints; ++r) {
    uint64_t ba, la, bb, lb;
    rs_rows_next(&ia, r, &ba, &la);
    rs_rows_next(&ib, r, &bb, &lb);
    ((la | lb) == 0 ? l : nl)++;
  }
  printf("non-linear constraints: %llu\n", (unsigned long long)nl);
  printf("linear constraints: %llu\n", (unsigned long long)l);
  printf("public inputs: %llu\n", (unsigned long long)in->n_pub_in);
  if (in->n_priv_in == o->no_private_inputs_witness)
    printf("private inputs: %llu\n", (unsigned long long)in->n_priv_in);
  else if (o->no_private_inputs_witness == 0)
    printf("private inputs: %llu (none belong to witness)\n", (unsigned long long)in->n_priv_in);
  else
    printf("private inputs: %llu (%llu belong to witness)\n", (unsigned long long)in->n_priv_in,
           (unsigned long long)o->no_private_inputs_witness);
  printf("public outputs: %llu\n", (unsigned long long)in->n_pub_out);
  printf("wires: %llu\n", (unsigned long long)o->n_wires);
  printf("labels: %llu\n", (unsigned long long)o->n_labels);
  fprintf(stderr, "simplification: %.3f ms\n", std::chrono::duration<double, std::milli>(t1 - t0).count());
  rs_output_free(o);
  rs_input_free(in);
  return 0;
}
