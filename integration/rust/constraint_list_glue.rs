// constraint_list_glue.rs -- goes into the reference's constraint_list crate as
// `src/gpu_glue.rs` (with `rs-simplify-sys` as a dependency behind a `mi355x` feature).  It is the
// body that replaces `constraint_simplification::simplification(&mut Simplifier)`
// (constraint_list/src/constraint_simplification.rs:442) when the feature is on:
//
//     pub fn simplification(smp: &mut Simplifier) -> (ConstraintStorage, SignalMap, usize) {
//         #[cfg(feature = "mi355x")]
//         { return crate::gpu_glue::simplification_mi355x(smp); }
//         // ... the reference body, unchanged ...
//     }
//
// Marshalling: the three LinkedLists are already in the DFS order map_tree built them
// (dag/src/map_to_constraint_list.rs:12-44); the non-linear rows come from the DAG encoding in the
// EncodingIterator DFS (constraint_list/src/lib.rs:65-108), offsets applied.  The library takes
// canonical 4 x u64 little-endian coefficients and returns the storage order with ORIGINAL signal
// ids plus an int32 label -> wire map; the glue rebuilds ConstraintStorage and SignalMap from them.
// A non-zero status panics with rs_last_error(), as the reference panics on its own invariants.
//
// BigInt <-> limbs goes through the byte conversions the reference itself uses: `to_bytes_le`
// (constraint_writers/src/r1cs_writer.rs:25-28) and `BigInt::from_bytes_le(Sign::Plus, ..)`
// (constraint_writers/src/r1cs_reader.rs:41); `is_zero` comes from num_traits::Zero as in
// circom_algebra/src/algebra.rs:4.  tests/test_integration.py rejects any other BigInt method.
// Not compiled in this repository (no cargo in the build image); the bindings it uses are checked
// against include/rs_simplify.h by tests/test_integration.py.
use crate::{EncodingIterator, SignalMap, Simplifier};
use circom_algebra::algebra::Constraint;
use circom_algebra::constraint_storage::ConstraintStorage;
use circom_algebra::num_bigint::{BigInt, Sign};
use circom_algebra::num_traits::Zero;
use rs_simplify_sys as ffi;
use std::collections::HashMap;
use std::ffi::{CStr, CString};

type C = Constraint<usize>;

/// A canonical (non-negative, < 2^256) field element as 4 little-endian u64 limbs.
fn to_limbs(v: &BigInt) -> [u64; 4] {
    let (_, bytes) = v.to_bytes_le();
    let mut limbs = [0u64; 4];
    for (i, b) in bytes.iter().enumerate().take(32) {
        limbs[i / 8] |= (*b as u64) << (8 * (i % 8));
    }
    limbs
}

/// The inverse of `to_limbs` (the library returns canonical values).
fn from_limbs(limbs: &[u64]) -> BigInt {
    let mut bytes = Vec::with_capacity(32);
    for l in limbs {
        bytes.extend_from_slice(&l.to_le_bytes());
    }
    BigInt::from_bytes_le(Sign::Plus, &bytes)
}

/// One owned CSR block (the arrays an rs_lc points at).
struct Csr {
    ptr: Vec<u64>,
    col: Vec<u32>,
    val: Vec<u64>,
}
impl Csr {
    fn new() -> Csr {
        Csr { ptr: vec![0], col: Vec::new(), val: Vec::new() }
    }
    /// Appends one linear combination; keys ascending (the library sorts too, but sorted rows let
    /// rs_engine_simplify start build_clusters before the values arrive).
    fn push(&mut self, m: &HashMap<usize, BigInt>) {
        let mut keys: Vec<_> = m.iter().filter(|(_, v)| !v.is_zero()).collect();
        keys.sort_by_key(|(k, _)| **k);
        for (k, v) in keys {
            self.col.push(*k as u32);
            self.val.extend_from_slice(&to_limbs(v)); // canonical (< p)
        }
        self.ptr.push(self.col.len() as u64);
    }
    fn lc(&mut self) -> ffi::rs_lc {
        ffi::rs_lc {
            n_rows: (self.ptr.len() - 1) as u64,
            nnz: self.col.len() as u64,
            ptr: self.ptr.as_mut_ptr(),
            col: self.col.as_mut_ptr(),
            val: self.val.as_mut_ptr(),
        }
    }
}

fn prime_id(field: &BigInt) -> (u32, [u64; 4]) {
    // every --prime of program_structure/src/utils/constants.rs:3-13 is passed as its value
    (255, to_limbs(field)) // RS_PRIME_CUSTOM: the library derives its field constants from the value
}

fn non_linear_rows(iter: EncodingIterator, a: &mut Csr, b: &mut Csr, c: &mut Csr) {
    let mut iter = iter;
    let (_, non_linear) = EncodingIterator::take(&mut iter);
    for row in non_linear {
        a.push(row.a());
        b.push(row.b());
        c.push(row.c());
    }
    for edge in EncodingIterator::edges(&iter) {
        let next = EncodingIterator::next(&iter, edge);
        non_linear_rows(next, a, b, c);
    }
}

pub fn simplification_mi355x(smp: &mut Simplifier) -> (ConstraintStorage, SignalMap, usize) {
    let (mut ce, mut eq, mut lin) = (Csr::new(), Csr::new(), Csr::new());
    for r in &smp.cons_equalities {
        ce.push(r.c());
    }
    for r in &smp.equalities {
        eq.push(r.c());
    }
    for r in &smp.linear {
        lin.push(r.c());
    }
    let (mut na, mut nb, mut nc) = (Csr::new(), Csr::new(), Csr::new());
    non_linear_rows(EncodingIterator::new(&smp.dag_encoding), &mut na, &mut nb, &mut nc);
    let mut forbidden: Vec<u32> = smp.forbidden.iter().map(|s| *s as u32).collect();
    forbidden.sort_unstable();
    let (pid, prime) = prime_id(&smp.field);
    let input = ffi::rs_input {
        prime_id: pid,
        prime,
        max_signal: smp.max_signal as u64,
        n_pub_out: smp.no_public_outputs as u64,
        n_pub_in: smp.no_public_inputs as u64,
        n_priv_in: smp.no_private_inputs as u64,
        n_forbidden: forbidden.len() as u64,
        forbidden: forbidden.as_mut_ptr(),
        cons_eq: ce.lc(),
        eq: eq.lc(),
        linear: lin.lc(),
        nl_a: na.lc(),
        nl_b: nb.lc(),
        nl_c: nc.lc(),
    };
    let flags = ffi::rs_flags {
        flag_s: smp.flag_s as u32,
        use_old_heuristics: smp.flag_old_heuristics as u32,
        no_rounds: smp.no_rounds as u64,
        emit_substitution_log: smp.port_substitution as u32,
        device: 0,
    };
    let mut out: *mut ffi::rs_output = std::ptr::null_mut();
    let rc = unsafe { ffi::rs_simplify(&input, &flags, &mut out) };
    if rc != ffi::RS_OK {
        let msg = unsafe { CStr::from_ptr(ffi::rs_last_error()) }.to_string_lossy().into_owned();
        panic!("rs_simplify failed ({}): {}", rc, msg);
    }
    let o = unsafe { &*out };
    // rows in order through ffi::RowCursor (CSR here; ABI 8's streamed layout walks the same way)
    let map_of = |cur: &mut ffi::RowCursor, r: usize| -> HashMap<usize, BigInt> {
        let mut m = HashMap::new();
        let lc = cur.lc();
        let (lo, n) = cur.next(r);
        for e in lo..lo + n {
            let k = unsafe { *lc.col.add(e) } as usize;
            let limbs: Vec<u64> = (0..4).map(|i| unsafe { *lc.val.add(4 * e + i) }).collect();
            m.insert(k, from_limbs(&limbs)); // canonical, non-negative
        }
        m
    };
    let mut storage = ConstraintStorage::new();
    let (mut ca, mut cb, mut cc) = (ffi::RowCursor::new(o, 0), ffi::RowCursor::new(o, 1), ffi::RowCursor::new(o, 2));
    for r in 0..o.n_constraints as usize {
        // Constraint::new is private (algebra.rs:1012): the shim adds `pub fn new_unchecked(a, b, c)`
        storage.add_constraint(C::new_unchecked(map_of(&mut ca, r), map_of(&mut cb, r), map_of(&mut cc, r)));
    }
    let mut signal_map = SignalMap::with_capacity(o.n_wires as usize);
    for s in 0..o.n_labels as usize {
        let w = unsafe { *o.label_to_wire.add(s) };
        if w >= 0 {
            signal_map.insert(s, w as usize);
        }
    }
    let npiw = o.no_private_inputs_witness as usize;
    if smp.port_substitution {
        // --simplification_substitution: the reference opens SubstitutionJSON at json_substitutions
        // and logs every substitution (constraint_simplification.rs:448-453, 9-17); the library
        // returned the same log in out->log_* and writes the same file.
        let path = CString::new(smp.json_substitutions.clone()).expect("path without NUL");
        let rc = unsafe { ffi::rs_write_substitution_json(path.as_ptr(), out) };
        if rc != ffi::RS_OK {
            let msg = unsafe { CStr::from_ptr(ffi::rs_last_error()) }.to_string_lossy().into_owned();
            panic!("rs_write_substitution_json failed ({}): {}", rc, msg);
        }
    }
    unsafe { ffi::rs_output_free(out) };
    (storage, signal_map, npiw)
}
