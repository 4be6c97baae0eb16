/*
 * rs_simplify.h -- C ABI of librs_simplify, the MI355X-native R1CS constraint-simplification
 * back end for circom (--O1 / --O2 / --O2round N).
 *
 * This is the drop-in seam.  In the reference (circom 2.2.2, /root/reference) the path is the
 * body of
 *     constraint_list::constraint_simplification::simplification(&mut Simplifier)
 *         -> (ConstraintStorage, SignalMap, usize)
 *     constraint_list/src/constraint_simplification.rs:442-730
 * called only from Simplifier::simplify_constraints (constraint_list/src/lib.rs:131-144).
 * The reference has no FFI and no plugin registry; these entry points are what a Rust shim in
 * constraint_list would bind with `extern "C"` (see INTEGRATION.md for the binding).
 *
 * Conventions
 *   - Field elements are 4 little-endian u64 limbs, canonical (< p).  The field is one of the
 *     eight circom primes (program_structure/src/utils/constants.rs:3-13) or a custom odd prime
 *     < 2^256 (used by tests, e.g. the reference unit tests' F_257).
 *   - Linear combinations are CSR blocks.  Column 0 is the constant-one signal (the reference's
 *     ArithmeticExpression::constant_coefficient(), algebra.rs:155-157).  Within a row the columns
 *     must be distinct; order is free.  Rows must be clean (no zero coefficient), as
 *     DAG::clean_constraints guarantees for every row the reference hands to simplification()
 *     (dag/src/constraint_correctness_analysis.rs:146-157); RS_E_INVALID otherwise.
 *   - All entry points are synchronous and blocking; one call at a time per engine.
 *   - Errors: 0 on success, a negative RS_E_* code otherwise; rs_last_error() explains.  The
 *     reference panics on the same internal invariants (e.g. algebra.rs:1114).
 */
#ifndef RS_SIMPLIFY_H
#define RS_SIMPLIFY_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RS_ABI_VERSION 9

enum rs_status {
  RS_OK = 0,
  RS_E_INVALID = -1,    /* malformed input (shape, unclean row, unknown prime, ...)          */
  RS_E_OOM_DEVICE = -2, /* device allocation failed                                           */
  RS_E_HIP = -3,        /* a HIP runtime call failed                                          */
  RS_E_RCCL = -4,       /* reserved: collective failure (multi-GPU)                           */
  RS_E_INTERNAL = -5,   /* an invariant the reference asserts was violated                    */
  RS_E_NODEVICE = -6    /* no usable gfx950 device: the library never falls back to the CPU   */
};

/* program_structure/src/utils/constants.rs:3-13, the --prime names of circom/src/input_user.rs */
enum rs_prime {
  RS_PRIME_BN128 = 0,
  RS_PRIME_BLS12381 = 1,
  RS_PRIME_GOLDILOCKS = 2,
  RS_PRIME_GRUMPKIN = 3,
  RS_PRIME_PALLAS = 4,
  RS_PRIME_VESTA = 5,
  RS_PRIME_SECQ256R1 = 6,
  RS_PRIME_BLS12377 = 7,
  RS_PRIME_CUSTOM = 255
};

/* One CSR matrix of linear combinations (HashMap<usize, BigInt> per row in the reference). */
typedef struct rs_lc {
  uint64_t n_rows;
  uint64_t nnz;
  uint64_t *ptr; /* n_rows + 1 offsets                                         */
  uint32_t *col; /* nnz signal ids                                             */
  uint64_t *val; /* nnz * 4 limbs (little endian, canonical)                   */
} rs_lc;

/*
 * The Simplifier bundle (constraint_list/src/lib.rs:110-129) as plain arrays.
 *   cons_eq / eq / linear : Simplifier.{cons_equalities, equalities, linear} -- linear rows,
 *                           only their C part (A = B = empty), in the reference's list order
 *                           (DFS order of dag/src/map_to_constraint_list.rs:12-44).
 *   nl_a / nl_b / nl_c    : the non-linear rows of the DAG encoding in EncodingIterator DFS
 *                           order (constraint_list/src/lib.rs:65-108); same n_rows each.
 *   forbidden             : Simplifier.forbidden = {0} u outputs u public inputs u custom-gate
 *                           signals (dag/src/lib.rs:174, 179-204; map_to_constraint_list.rs:22-24).
 */
typedef struct rs_input {
  uint32_t prime_id;     /* enum rs_prime                                                  */
  uint64_t prime[4];     /* only read when prime_id == RS_PRIME_CUSTOM                      */
  uint64_t max_signal;   /* Simplifier.max_signal (= number of labels)                      */
  uint64_t n_pub_out;
  uint64_t n_pub_in;
  uint64_t n_priv_in;
  uint64_t n_forbidden;
  uint32_t *forbidden;
  rs_lc cons_eq;
  rs_lc eq;
  rs_lc linear;
  rs_lc nl_a;
  rs_lc nl_b;
  rs_lc nl_c;
} rs_input;

/* SimplificationFlags (dag/src/lib.rs:546-554) + execution knobs. */
typedef struct rs_flags {
  uint32_t flag_s;             /* --O1: no linear elimination (apply_linear = !flag_s)      */
  uint32_t use_old_heuristics; /* --use_old_simplification_heuristics                        */
  uint64_t no_rounds;          /* UINT64_MAX for --O2, N for --O2round N, 0 for --O1         */
  uint32_t emit_substitution_log; /* --simplification_substitution: fill rs_output.log_*     */
  int32_t device;              /* HIP device ordinal                                        */
} rs_flags;

/*
 * Result: (ConstraintStorage, SignalMap, no_private_inputs_witness) of simplification().
 * Constraints are in storage order with ORIGINAL signal ids (the caller applies label_to_wire,
 * exactly like ConstraintList::r1cs does with apply_correspondence, r1cs_porting.rs:23-33).
 */
typedef struct rs_output {
  uint64_t n_constraints;
  rs_lc a, b, c;                  /* owned by the library; free with rs_output_free         */
  uint64_t n_labels;              /* = max_signal                                           */
  int32_t *label_to_wire;         /* n_labels entries, -1 = not a wire (int32)  */
  uint64_t n_wires;               /* = SignalMap.len()                                      */
  uint64_t no_private_inputs_witness;
  /* The substitution log (--simplification_substitution, constraint_simplification.rs:9-17),
   * only when rs_flags.emit_substitution_log: every Substitution the reference hands to
   * log_substitutions, in its order -- eq_simplification (:249; size-1 clusters, then the others,
   * by cluster index), constant_eq_simplification (:271; row order), then each round's
   * linear_simplification (:320; cluster index order, ascending `from`).  Entry i is
   * log_from[i] := row i of log_to, with ORIGINAL signal ids, keys ascending and the values the
   * reference's `to` map holds (zero values included, e.g. the constant key's {0: 0}). */
  uint64_t n_log;
  uint32_t *log_from;
  rs_lc log_to;
  /* ABI 8: the row layout of a / b / c.  NULL: the block is CSR (row i = [ptr[i], ptr[i+1])), as
   * rs_simplify / rs_engine_fetch return it.  Non-NULL (rs_engine_simplify's streamed result): ptr is
   * NULL and rows are walked in storage order: row i holds {a,b,c}_len[i] & ~RS_ROW_JUMP entries of
   * col / val, starting where row i - 1's ended -- or, when bit 31 (RS_ROW_JUMP) is set, at the next
   * offset of {a,b,c}_jump (row 0 starts at 0 unless it jumps).  The storage rows that were final
   * after the first round went to the host while the later rounds ran and the rest follow them, so
   * col / val may hold entries no row refers to; nnz is the extent of col / val.  rs_rows_begin /
   * rs_rows_next below walk either layout.  (ABI 7 sent a u64 start and a u64 end per row and part:
   * 48 bytes a row on the PCIe link against 12 + a few jumps.) */
  uint32_t *a_len, *b_len, *c_len;
  uint64_t *a_jump, *b_jump, *c_jump;
  uint64_t a_njump, b_njump, c_njump;
} rs_output;

#define RS_ROW_JUMP 0x80000000u
/* The rows of result block q (0 a, 1 b, 2 c) in order, for either layout: rs_rows_begin, then
 * rs_rows_next(&it, r, &beg, &len) for r = 0, 1, 2, ... (a CSR block also allows any order). */
typedef struct rs_rows {
  const rs_lc *L;
  const uint32_t *len;
  const uint64_t *jump;
  uint64_t pos, j;
} rs_rows;
static inline void rs_rows_begin(const rs_output *o, int q, rs_rows *it) {
  it->L = q == 0 ? &o->a : (q == 1 ? &o->b : &o->c);
  it->len = q == 0 ? o->a_len : (q == 1 ? o->b_len : o->c_len);
  it->jump = q == 0 ? o->a_jump : (q == 1 ? o->b_jump : o->c_jump);
  it->pos = 0;
  it->j = 0;
}
static inline void rs_rows_next(rs_rows *it, uint64_t r, uint64_t *beg, uint64_t *len) {
  if (!it->len) {
    *beg = it->L->ptr[r];
    *len = it->L->ptr[r + 1] - it->L->ptr[r];
    return;
  }
  const uint32_t x = it->len[r];
  if (x & RS_ROW_JUMP) it->pos = it->jump[it->j++];
  *beg = it->pos;
  *len = x & ~RS_ROW_JUMP;
  it->pos += *len;
}

/* Phase timings of the last rs_engine_run (milliseconds, HIP events + host clock). */
typedef struct rs_stats {
  double total_ms;             /* device-resident input -> device-resident output             */
  double eq_ms;                /* eq + const-eq renaming                                     */
  double cluster_ms;           /* union-find clustering (all rounds)                         */
  double elim_ms;              /* per-cluster elimination + normalisation + composition      */
  double subst_ms;             /* substitution application (non-linear rows, rounds >= 2)    */
  double final_ms;             /* compaction, rebuild_witness, output assembly               */
  double apply_kernel_ms;      /* device time of the non-linear frames passes (k_frames_wave<0>) */
  uint64_t apply_kernel_launches;
  uint64_t apply_bytes;        /* its algorithmic bytes (sum over launches)                  */
  double elim_kernel_ms;       /* device time of the per-cluster elimination (every kernel)  */
  uint64_t elim_kernel_launches;
  uint64_t elim_bytes;         /* its algorithmic bytes (sum over launches)                  */
  double elim_big_ms;          /* device time of the workgroup kernels (head + tail streams)  */
  double elim_small_ms;        /* device time of the small-cluster kernel (k_eliminate)      */
  double nl_ms;                /* non-linear frames (count, scan, fill, split)               */
  double map_ms;               /* host copy of the non-linear signal map (rounds >= 2)       */
  double rounds_ms;            /* storage updates + bookkeeping of rounds >= 2               */
  double big_prep_ms;          /* k_wide_* + k_big_prep (occurrences + uniques)              */
  double big_main_ms;          /* the ordered elimination loops (k_big_spec<12> + k_big_main<256>) */
  double big_finish_ms;        /* normalisation + composition (k_batch_inv_*, k_big_finish, levels) */
  uint64_t big_main_bytes;     /* algorithmic bytes of the ordered loops (sum over launches)  */
  uint64_t big_finish_bytes;   /* algorithmic bytes of normalisation + composition           */
  uint64_t big_launches;       /* launches of each of the three workgroup kernels            */
  uint64_t rounds;             /* linear-elimination rounds executed                         */
  uint64_t n_clusters;
  uint64_t n_substitutions;
  uint64_t max_cluster;
  double exchange_ms;          /* sharded runs: the eliminated-signal-map exchange (all rounds) */
  uint64_t exchange_bytes;     /* bytes each rank received + contributed in those collectives  */
  uint64_t world;              /* ranks the elimination was sharded over (1 = single GPU)       */
  /* ABI 4: the ordered elimination loop split into the head (the largest clusters, one launch
   * on the second stream, the critical path) and the tail (every other workgroup cluster), each
   * with its own HIP-event time and in-kernel algorithmic bytes; the storage-row kernel of
   * rounds >= 2; the host -> host legs of rs_engine_simplify. */
  double head_main_ms;         /* k_big_spec<12> (head: the 96 largest clusters)             */
  uint64_t head_main_bytes;
  uint64_t head_launches;
  double tail_main_ms;         /* k_big_main<256> (tail)                                     */
  uint64_t tail_main_bytes;
  uint64_t tail_launches;
  double round_fill_ms;        /* k_frames_wave<1> + k_round_fill (apply_substitution_to_map) */
  uint64_t round_fill_bytes;
  uint64_t round_fill_launches;
  uint64_t alg_bytes;          /* B_alg of the run: every in-kernel counter +
                                  36 (Z_in + Z_out) + 8 (R_in + R_out) + 8 max_signal       */
  double h2d_wait_ms;          /* host time the run spent waiting for input groups to land  */
  double d2h_ms;               /* D2H of the result into the engine's pinned buffers        */
  double host_total_ms;        /* rs_engine_simplify: host input -> host output             */
  double write_ms;             /* ABI 5: the last rs_engine_write_r1cs (device image + file)  */
  /* ABI 8: the rest of the elimination's kernels, each with its HIP-event time (on the stream it runs
   * on) and in-kernel algorithmic bytes, so the per-kernel rooflines cover the GPU time */
  double tail_fin_ms;          /* k_batch_inv_flat + k_big_finish<4>: the tail's normalisation + composition (both groups) */
  uint64_t tail_fin_bytes;
  uint64_t tail_fin_launches;
  double head_fin_ms;          /* the head's k_batch_inv_tree, k_normalize, k_big_finish<8>, Kahn levels, k_big_emit */
  uint64_t head_fin_bytes;
  uint64_t head_fin_launches;
  double small_ms;             /* k_eliminate (clusters under 32 rows, one lane each)               */
  uint64_t small_bytes;
  uint64_t small_launches;
  double prep_ms;              /* the tail's k_big_prep + k_p3_fast (both groups)                    */
  uint64_t prep_launches;
  double cluster_dev_ms;       /* build_clusters on the device (pair sort, union-find, arena replays) */
  uint64_t cluster_bytes;      /* its keys read, (signal, row) pairs written, sorted and linked, per-row arrays */
  uint64_t cluster_launches;
  double giant_ms;             /* the giant path (giant_loop.hpp): component loops of the largest clusters */
  uint64_t giant_bytes;
  uint64_t giant_launches;
  uint64_t giant_merges;        /* merges work = c2*work - c*R the giant path's table loop performed (configs[1]: 21.6 M) */
  double check_ms;             /* the input's device checks (k_check_ptr, k_check_keys, k_sort_validate; copy stream) */
  uint64_t check_bytes;        /* row pointers, keys (+ values: k_sort_validate) read */
  uint64_t check_launches;
  double ragged_ms;            /* CSR -> ragged rows (k_make_ragged) and the linear rows' eq / constant frames */
  uint64_t ragged_bytes;       /* 72 B an entry converted, 77 B an entry framed, + per-row extents */
  uint64_t ragged_launches;
  double gather_ms;            /* the result's gathers: snapshots, late rows, the compact CSR */
  uint64_t gather_bytes;       /* 72 B an entry gathered (read + canonical write) + per-row selection */
  uint64_t gather_launches;
  /* ABI 9: the host's share of the clustering (build_clusters): time the calling thread spent blocked
   * in its read-backs and synchronisations and replaying the largest clusters' arena order, inside the
   * span cluster_dev_ms brackets on the main stream */
  double cluster_host_ms;
} rs_stats;

typedef struct rs_engine rs_engine;

const char *rs_last_error(void);
int rs_abi_version(void);

/* One-shot: host input -> host output (H2D, simplification on the GPU, D2H). */
int rs_simplify(const rs_input *in, const rs_flags *fl, rs_output **out);
void rs_output_free(rs_output *out);

/* Engine API used by the benchmark: stage the input in HBM once, run many times. */
int rs_engine_create(int device, rs_engine **eng);
int rs_engine_load(rs_engine *eng, const rs_input *in);   /* H2D copy of the host input        */
int rs_engine_run(rs_engine *eng, const rs_flags *fl);    /* the timed region                   */
int rs_engine_fetch(rs_engine *eng, rs_output **out);     /* D2H of the last result             */
int rs_engine_stats(rs_engine *eng, rs_stats *st);
void rs_engine_destroy(rs_engine *eng);

/*
 * Host -> host on a persistent engine: the whole of simplification() (constraint_simplification.rs
 * :442-730) from the host CSR blocks to the host result, the SURVEY 8(d) T_simplify region.
 * The H2D copy of `in` runs on a copy stream in three groups (cons_eq + eq, linear, non-linear),
 * each validated on the device as it lands, and the simplification consumes a group as soon as it
 * is there, so the upload of the later groups overlaps the eq / clustering / elimination phases.
 * The result is copied into pinned buffers the engine owns; *out points at them and stays valid
 * until the next call on `eng` or rs_engine_destroy (do not rs_output_free it).  `in` is read
 * only during the call.  Host buffers from rs_host_alloc move at full PCIe speed; pageable ones
 * work too (HIP stages them), slower.
 */
int rs_engine_simplify(rs_engine *eng, const rs_input *in, const rs_flags *fl, const rs_output **out);

/* The engine's last result written as a .r1cs (constraint_list/src/r1cs_porting.rs:4-124; SURVEY
 * 8(f) rank 2): byte-identical to rs_write_r1cs on the fetched output, with the constraint section
 * (wire correspondence + LE-byte key order per row) built on the device and streamed to the file.
 * o0_r1cs (may be NULL): copy its custom-gate sections like rs_write_r1cs_gates.  Time in
 * rs_stats.write_ms. */
int rs_engine_write_r1cs(rs_engine *eng, const char *path, const char *o0_r1cs);

/* Page-locked host memory (hipHostMalloc) for the CSR blocks a caller marshals the Simplifier into,
 * so rs_engine_simplify's H2D runs at PCIe speed.  NULL without a device. */
void *rs_host_alloc(uint64_t bytes);
void rs_host_free(void *p);

/*
 * Multi-GPU: ONE circuit sharded over W ranks.  Every rank loads the same input;
 * the global phases (eq / const-eq renaming, build_clusters) run on every rank, the clusters are
 * dealt to the ranks by size (snake order), each rank eliminates its own, and the eliminated-signal
 * map (substitutions, leftovers, their pool entries) is exchanged after every round -- RCCL over
 * xGMI in production.  Every rank ends with the complete, identical output (byte-identical to a
 * single-GPU run).  Join before rs_engine_run; all ranks must run with the same flags.
 *
 * RCCL, one process per GPU (what bench.py does under torch.distributed.run):
 *   rank 0: rs_comm_unique_id(id); broadcast the RS_COMM_ID_BYTES bytes to the other ranks;
 *   every rank: rs_engine_join_rccl(eng, world, rank, id)   (collective: blocks until all joined)
 * In one process (threads; a device may be listed twice, e.g. to test on one GPU):
 *   g = rs_group_create(world); rank r's thread: rs_engine_join_group(eng_r, g, r); ...
 *   rs_group_destroy(g) after every engine of the group is destroyed.
 * rs_simplify_multi: the one-shot entry point over n_devices GPUs of this process (threads; RCCL
 * when the devices are distinct, the in-process transport otherwise).
 */
#define RS_COMM_ID_BYTES 128
typedef struct rs_group rs_group;
int rs_comm_unique_id(uint8_t id[RS_COMM_ID_BYTES]);
int rs_engine_join_rccl(rs_engine *eng, int world, int rank, const uint8_t id[RS_COMM_ID_BYTES]);
rs_group *rs_group_create(int world);
int rs_engine_join_group(rs_engine *eng, rs_group *g, int rank);
void rs_group_destroy(rs_group *g);
int rs_simplify_multi(const rs_input *in, const rs_flags *fl, int n_devices, const int *devices, rs_output **out);
/* ABI 9, a test transport: the ranks are processes of one host (e.g. two processes on ONE GPU, where RCCL
 * refuses a second rank), their collectives staged through POSIX shared memory; every rank passes the
 * same `tag` (a name for the group's control block).  The shared result region is made exactly as for
 * RCCL ranks, so the one-GPU box runs the multi-process result path (shared host memory mapped and
 * registered by every process, each rank's share streamed into it). */
int rs_engine_join_host(rs_engine *eng, int world, int rank, const char *tag);

/* Fault injection (tests; SURVEY 5 "failure detection / fault injection"): the engine's next
 * rs_engine_run / rs_engine_simplify fails with RS_E_INTERNAL at `where` (1: the start of the first
 * linear elimination round, after the run's first collectives; 0: cancel).  A failure belongs to the
 * call it happens in: the other ranks of an in-process group leave that call with RS_E_RCCL, and the
 * group runs the ranks' next calls normally.  RCCL ranks are not released (a failed rank there ends
 * the job). */
int rs_engine_inject_fault(rs_engine *eng, int where);

/* --O0 .r1cs -> rs_input (host arrays owned by the library; free with rs_input_free).
 * Classifies rows exactly like dag/src/map_to_constraint_list.rs:12-44.  The signals of the
 * custom-gate applications (section 5, dag/src/r1cs_porting.rs:74-107) join `forbidden`, as
 * map_tree inserts them (map_to_constraint_list.rs:22-24).  Every read is bounds-checked against
 * its section and the file: a truncated or malformed file is RS_E_INVALID. */
int rs_read_r1cs_o0(const char *path, rs_input **in);
void rs_input_free(rs_input *in);
/* Writes the simplified .r1cs (constraint_list/src/r1cs_porting.rs:4-124). */
int rs_write_r1cs(const char *path, const rs_input *in, const rs_output *out);
/* The same, plus the --O0 file's custom-gate sections as the O2 writer re-emits them
 * (r1cs_porting.rs:54-121): section 4 unchanged, section 5 with its signals mapped label -> wire
 * (5 sections in all).  Without sections 4/5 in `o0_r1cs` the output equals rs_write_r1cs's. */
int rs_write_r1cs_gates(const char *path, const rs_input *in, const rs_output *out, const char *o0_r1cs);
/* Rewrites an --O0 .sym with the witness column of `out` (constraint_list/src/sym_porting.rs). */
int rs_write_sym(const char *o0_sym, const char *path, const rs_output *out);
/* --json: <prefix>_constraints.json (constraint_list/src/json_porting.rs:36-48 port_constraints,
 * constraint_writers/src/json_writer.rs:4-45 ConstraintJSON): the rows in storage order with the
 * witness correspondence applied, keys ascending, decimal values. */
int rs_write_constraints_json(const char *path, const rs_output *out);
/* --simplification_substitution: <prefix>_substitutions.json (json_porting.rs:28-33
 * port_substitution, json_writer.rs:94-131 SubstitutionJSON) from out->log_*, original ids. */
int rs_write_substitution_json(const char *path, const rs_output *out);

/* Seeded synthetic --O0 systems for benchmarks/tests (see DESIGN.md "Workloads").
 * kind: 0 = mixed (metric circuit, BASELINE configs[4]), 1 = purely linear (configs[1]), 2 = chain
 * (configs[3] ECDSA stand-in: deep composition, 8 rounds), 3 = Poseidon(16) Merkle (configs[2]),
 * 4 = sha256-like bit gadgets (configs[0]), 5 = templated (64-row template instances replicated with
 * signal offsets, wired into chains; SURVEY 8(d) config 5's replication), 6 = templated whose first
 * chain has 9,000 instances (one ~2e5-row linear cluster: config 5's replication and its tail). */
int rs_synth(uint32_t kind, uint64_t rows, uint64_t seed, uint32_t prime_id, rs_input **in);

/* ---- the DAG -> constraint-list flattening that produces rs_input.
 * Replaces dag::map_to_constraint_list::map's walk (dag/src/map_to_constraint_list.rs:12-44 map_tree,
 * :111-150 map) and the non-linear rows of the EncodingIterator DFS (constraint_list/src/lib.rs:65-108,
 * state_utils.rs:14-35): every component instance in DFS order from main (offset 0), its local
 * signals appended to the witness list, its constraints with the instance offset applied (key 0 stays
 * the constant) and classified like map_tree -- constant equality, equality, linear (empty
 * constraints only in main; Tree::go_to_subtree drops them), else non-linear.  Custom-gate
 * instances' signals join main's forbidden_if_main.  Instance expansion and the constraint copy run
 * on the device (prefix sums over the instance tree); the per-template classification is a host
 * pass over the templates.  The result is an ordinary rs_input (freed with rs_input_free). */
typedef struct rs_dag {
  uint32_t prime_id;           /* enum rs_prime                                                 */
  uint64_t prime[4];           /* only read when prime_id == RS_PRIME_CUSTOM                     */
  uint64_t n_pub_out, n_pub_in, n_priv_in;
  uint64_t n_forbidden;        /* main's forbidden_if_main (main's offset is 0: global ids)      */
  const uint32_t *forbidden;
  uint32_t n_nodes;            /* DAG nodes (templates with their parameters)                   */
  uint32_t main_node;
  const uint64_t *cons_off;    /* [n_nodes + 1]: node -> its constraints, rows of a / b / c       */
  rs_lc a, b, c;               /* every node's constraints, node-local ids (0 = the constant)     */
  const uint64_t *local_off;   /* [n_nodes + 1]: node -> its local signals                        */
  const uint32_t *locals;      /* node-local ids of the node's own signals, ascending             */
  const uint8_t *custom_gate;  /* [n_nodes]                                                       */
  const uint64_t *edge_off;    /* [n_nodes + 1]: node -> its edges, in adjacency order            */
  const uint32_t *edge_to;     /* child node                                                      */
  const uint64_t *edge_in;     /* the edge's in_number: the child's signal offset in the parent   */
} rs_dag;
/* device: the GPU to run on.  Rejects (RS_E_INVALID) a cyclic graph, an edge to a missing node,
 * malformed CSR blocks (ptr[0] != 0, decreasing pointers, ptr[T] != nnz) and a graph whose offset
 * signal ids (instance offset + node-local id) or signal count reach 2^31. */
int rs_flatten_dag(int device, const rs_dag *dag, rs_input **in);
/* The same on a persistent engine (its device buffers stay allocated across calls), into page-locked
 * buffers the engine owns, so the blocks' D2H runs at PCIe speed and the result feeds
 * rs_engine_simplify's H2D at full speed too.  *in views those buffers: valid until the next
 * rs_engine_flatten_dag on `eng` or rs_engine_destroy (do not rs_input_free it). */
int rs_engine_flatten_dag(rs_engine *eng, const rs_dag *dag, const rs_input **in);

#ifdef __cplusplus
}
#endif
#endif /* RS_SIMPLIFY_H */
