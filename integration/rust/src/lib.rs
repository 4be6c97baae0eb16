//! Raw bindings of `include/rs_simplify.h` (ABI 9), one item per C declaration, same order and
//! layout.  The safe wrapper a caller uses is `constraint_list_glue.rs` (the body that replaces
//! `constraint_list::constraint_simplification::simplification`, constraint_simplification.rs:442).
#![allow(non_camel_case_types)]
use std::os::raw::{c_char, c_int, c_void};

pub const RS_ABI_VERSION: c_int = 9;
pub const RS_COMM_ID_BYTES: usize = 128;

pub const RS_OK: c_int = 0;
pub const RS_E_INVALID: c_int = -1;
pub const RS_E_OOM_DEVICE: c_int = -2;
pub const RS_E_HIP: c_int = -3;
pub const RS_E_RCCL: c_int = -4;
pub const RS_E_INTERNAL: c_int = -5;
pub const RS_E_NODEVICE: c_int = -6;

#[repr(C)]
#[derive(Clone, Copy)]
pub struct rs_lc {
    pub n_rows: u64,
    pub nnz: u64,
    pub ptr: *mut u64,
    pub col: *mut u32,
    pub val: *mut u64,
}

#[repr(C)]
pub struct rs_input {
    pub prime_id: u32,
    pub prime: [u64; 4],
    pub max_signal: u64,
    pub n_pub_out: u64,
    pub n_pub_in: u64,
    pub n_priv_in: u64,
    pub n_forbidden: u64,
    pub forbidden: *mut u32,
    pub cons_eq: rs_lc,
    pub eq: rs_lc,
    pub linear: rs_lc,
    pub nl_a: rs_lc,
    pub nl_b: rs_lc,
    pub nl_c: rs_lc,
}

#[repr(C)]
pub struct rs_flags {
    pub flag_s: u32,
    pub use_old_heuristics: u32,
    pub no_rounds: u64,
    pub emit_substitution_log: u32,
    pub device: i32,
}

#[repr(C)]
pub struct rs_output {
    pub n_constraints: u64,
    pub a: rs_lc,
    pub b: rs_lc,
    pub c: rs_lc,
    pub n_labels: u64,
    pub label_to_wire: *mut i32,
    pub n_wires: u64,
    pub no_private_inputs_witness: u64,
    pub n_log: u64,
    pub log_from: *mut u32,
    pub log_to: rs_lc,
    /// ABI 8 row layout (null: CSR through `ptr`): row lengths, bit 31 = RS_ROW_JUMP
    pub a_len: *mut u32,
    pub b_len: *mut u32,
    pub c_len: *mut u32,
    pub a_jump: *mut u64,
    pub b_jump: *mut u64,
    pub c_jump: *mut u64,
    pub a_njump: u64,
    pub b_njump: u64,
    pub c_njump: u64,
}

pub const RS_ROW_JUMP: u32 = 0x8000_0000;

/// rs_rows_begin / rs_rows_next (include/rs_simplify.h): the rows of block q (0 a, 1 b, 2 c) in
/// order, for either layout; `next(r)` must be called for r = 0, 1, 2, ... and returns (start, len).
pub struct RowCursor<'a> {
    lc: &'a rs_lc,
    len: *const u32,
    jump: *const u64,
    pos: u64,
    j: usize,
}

impl<'a> RowCursor<'a> {
    pub fn new(o: &'a rs_output, q: usize) -> Self {
        let (lc, len, jump) = match q {
            0 => (&o.a, o.a_len, o.a_jump),
            1 => (&o.b, o.b_len, o.b_jump),
            _ => (&o.c, o.c_len, o.c_jump),
        };
        RowCursor { lc, len, jump, pos: 0, j: 0 }
    }
    pub fn lc(&self) -> &'a rs_lc {
        self.lc
    }
    pub fn next(&mut self, r: usize) -> (usize, usize) {
        unsafe {
            if self.len.is_null() {
                let lo = *self.lc.ptr.add(r);
                return (lo as usize, (*self.lc.ptr.add(r + 1) - lo) as usize);
            }
            let x = *self.len.add(r);
            if x & RS_ROW_JUMP != 0 {
                self.pos = *self.jump.add(self.j);
                self.j += 1;
            }
            let l = (x & !RS_ROW_JUMP) as u64;
            let b = self.pos;
            self.pos += l;
            (b as usize, l as usize)
        }
    }
}

/// the component DAG rs_flatten_dag expands (dag/src/lib.rs Node / Edge).
#[repr(C)]
pub struct rs_dag {
    pub prime_id: u32,
    pub prime: [u64; 4],
    pub n_pub_out: u64,
    pub n_pub_in: u64,
    pub n_priv_in: u64,
    pub n_forbidden: u64,
    pub forbidden: *const u32,
    pub n_nodes: u32,
    pub main_node: u32,
    pub cons_off: *const u64,
    pub a: rs_lc,
    pub b: rs_lc,
    pub c: rs_lc,
    pub local_off: *const u64,
    pub locals: *const u32,
    pub custom_gate: *const u8,
    pub edge_off: *const u64,
    pub edge_to: *const u32,
    pub edge_in: *const u64,
}

#[repr(C)]
pub struct rs_stats {
    pub total_ms: f64,
    pub eq_ms: f64,
    pub cluster_ms: f64,
    pub elim_ms: f64,
    pub subst_ms: f64,
    pub final_ms: f64,
    pub apply_kernel_ms: f64,
    pub apply_kernel_launches: u64,
    pub apply_bytes: u64,
    pub elim_kernel_ms: f64,
    pub elim_kernel_launches: u64,
    pub elim_bytes: u64,
    pub elim_big_ms: f64,
    pub elim_small_ms: f64,
    pub nl_ms: f64,
    pub map_ms: f64,
    pub rounds_ms: f64,
    pub big_prep_ms: f64,
    pub big_main_ms: f64,
    pub big_finish_ms: f64,
    pub big_main_bytes: u64,
    pub big_finish_bytes: u64,
    pub big_launches: u64,
    pub rounds: u64,
    pub n_clusters: u64,
    pub n_substitutions: u64,
    pub max_cluster: u64,
    pub exchange_ms: f64,
    pub exchange_bytes: u64,
    pub world: u64,
    pub head_main_ms: f64,
    pub head_main_bytes: u64,
    pub head_launches: u64,
    pub tail_main_ms: f64,
    pub tail_main_bytes: u64,
    pub tail_launches: u64,
    pub round_fill_ms: f64,
    pub round_fill_bytes: u64,
    pub round_fill_launches: u64,
    pub alg_bytes: u64,
    pub h2d_wait_ms: f64,
    pub d2h_ms: f64,
    pub host_total_ms: f64,
    pub write_ms: f64,
    pub tail_fin_ms: f64,
    pub tail_fin_bytes: u64,
    pub tail_fin_launches: u64,
    pub head_fin_ms: f64,
    pub head_fin_bytes: u64,
    pub head_fin_launches: u64,
    pub small_ms: f64,
    pub small_bytes: u64,
    pub small_launches: u64,
    pub prep_ms: f64,
    pub prep_launches: u64,
    pub cluster_dev_ms: f64,
    pub cluster_bytes: u64,
    pub cluster_launches: u64,
    pub giant_ms: f64,
    pub giant_bytes: u64,
    pub giant_launches: u64,
    pub giant_merges: u64,
    pub check_ms: f64,
    pub check_bytes: u64,
    pub check_launches: u64,
    pub ragged_ms: f64,
    pub ragged_bytes: u64,
    pub ragged_launches: u64,
    pub gather_ms: f64,
    pub gather_bytes: u64,
    pub gather_launches: u64,
    pub cluster_host_ms: f64,
}

#[repr(C)]
pub struct rs_engine {
    _private: [u8; 0],
}
#[repr(C)]
pub struct rs_group {
    _private: [u8; 0],
}

extern "C" {
    pub fn rs_last_error() -> *const c_char;
    pub fn rs_abi_version() -> c_int;
    pub fn rs_simplify(inp: *const rs_input, fl: *const rs_flags, out: *mut *mut rs_output) -> c_int;
    pub fn rs_output_free(out: *mut rs_output);
    pub fn rs_engine_create(device: c_int, eng: *mut *mut rs_engine) -> c_int;
    pub fn rs_engine_load(eng: *mut rs_engine, inp: *const rs_input) -> c_int;
    pub fn rs_engine_run(eng: *mut rs_engine, fl: *const rs_flags) -> c_int;
    pub fn rs_engine_fetch(eng: *mut rs_engine, out: *mut *mut rs_output) -> c_int;
    pub fn rs_engine_stats(eng: *mut rs_engine, st: *mut rs_stats) -> c_int;
    pub fn rs_engine_destroy(eng: *mut rs_engine);
    pub fn rs_engine_simplify(eng: *mut rs_engine, inp: *const rs_input, fl: *const rs_flags, out: *mut *const rs_output) -> c_int;
    pub fn rs_engine_write_r1cs(eng: *mut rs_engine, path: *const c_char, o0_r1cs: *const c_char) -> c_int;
    pub fn rs_host_alloc(bytes: u64) -> *mut c_void;
    pub fn rs_host_free(p: *mut c_void);
    pub fn rs_comm_unique_id(id: *mut u8) -> c_int;
    pub fn rs_engine_join_rccl(eng: *mut rs_engine, world: c_int, rank: c_int, id: *const u8) -> c_int;
    pub fn rs_group_create(world: c_int) -> *mut rs_group;
    pub fn rs_engine_join_group(eng: *mut rs_engine, g: *mut rs_group, rank: c_int) -> c_int;
    pub fn rs_group_destroy(g: *mut rs_group);
    pub fn rs_simplify_multi(inp: *const rs_input, fl: *const rs_flags, n_devices: c_int, devices: *const c_int, out: *mut *mut rs_output) -> c_int;
    /// Test transport: the ranks are processes of one host, collectives through POSIX shared memory.
    pub fn rs_engine_join_host(eng: *mut rs_engine, world: c_int, rank: c_int, tag: *const c_char) -> c_int;
    /// Fault injection (tests): the engine's next run fails with RS_E_INTERNAL at `where_`.
    pub fn rs_engine_inject_fault(eng: *mut rs_engine, where_: c_int) -> c_int;
    pub fn rs_read_r1cs_o0(path: *const c_char, inp: *mut *mut rs_input) -> c_int;
    pub fn rs_input_free(inp: *mut rs_input);
    pub fn rs_write_r1cs(path: *const c_char, inp: *const rs_input, out: *const rs_output) -> c_int;
    pub fn rs_write_r1cs_gates(path: *const c_char, inp: *const rs_input, out: *const rs_output, o0_r1cs: *const c_char) -> c_int;
    pub fn rs_write_sym(o0_sym: *const c_char, path: *const c_char, out: *const rs_output) -> c_int;
    pub fn rs_write_constraints_json(path: *const c_char, out: *const rs_output) -> c_int;
    pub fn rs_write_substitution_json(path: *const c_char, out: *const rs_output) -> c_int;
    pub fn rs_synth(kind: u32, rows: u64, seed: u64, prime_id: u32, inp: *mut *mut rs_input) -> c_int;
    pub fn rs_flatten_dag(device: c_int, dag: *const rs_dag, inp: *mut *mut rs_input) -> c_int;
    /// The same into the engine's page-locked buffers (the view lives until the next call on `eng`).
    pub fn rs_engine_flatten_dag(eng: *mut rs_engine, dag: *const rs_dag, inp: *mut *const rs_input) -> c_int;
}
