"""ctypes mirror of include/rs_simplify.h plus converters between oracle/pyref.py systems and the
C ABI.  Shared by the oracle tests, the GPU parity tests and bench.py."""
from __future__ import annotations

import ctypes as C
import os
import random
import sys
from typing import List

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyref as R  # noqa: E402

sys.path.insert(0, ROOT)
from circom_cvm_amd.abi import (PRIME_IDS, U64_MAX, RsFlags, RsInput, RsLc, RsOutput,  # noqa: E402
                                RsStats, block_csr, make_flags)


def flags(level="O2", rounds=None, old=False, device=0, log=False) -> RsFlags:
    return make_flags(level, rounds, old, device, log)


def py_flags(fl: RsFlags) -> "R.Flags":
    """The pyref Flags of an RsFlags."""
    return R.Flags(flag_s=bool(fl.flag_s), no_rounds=int(fl.no_rounds), use_old_heuristics=bool(fl.use_old_heuristics))


# --------------------------------------------------------------------------- pyref <-> C ABI
def _limbs(v: int):
    return [(v >> (64 * i)) & U64_MAX for i in range(4)]


class _Block:
    def __init__(self, maps: List[dict]):
        ptr = [0]
        cols, vals = [], []
        for m in maps:
            for k in sorted(m):
                cols.append(k)
                vals.extend(_limbs(m[k]))
            ptr.append(len(cols))
        self.ptr = np.array(ptr, dtype=np.uint64)
        self.col = np.array(cols if cols else [0], dtype=np.uint32)
        self.val = np.array(vals if vals else [0, 0, 0, 0], dtype=np.uint64)
        self.lc = RsLc(len(maps), len(cols), self.ptr.ctypes.data_as(C.POINTER(C.c_uint64)),
                       self.col.ctypes.data_as(C.POINTER(C.c_uint32)),
                       self.val.ctypes.data_as(C.POINTER(C.c_uint64)))


class InputHolder:
    """Keeps the numpy arrays behind an RsInput alive."""

    def __init__(self, sys_: "R.System", prime_name: str | None = None):
        cons_eq, eq, lin, nonlin = R.classify(sys_)
        self.blocks = [_Block([c.c for c in cons_eq]), _Block([c.c for c in eq]),
                       _Block([c.c for c in lin]), _Block([c.a for c in nonlin]),
                       _Block([c.b for c in nonlin]), _Block([c.c for c in nonlin])]
        self.forb = np.array(sorted(sys_.forbidden), dtype=np.uint32)
        inp = RsInput()
        if prime_name is not None:
            inp.prime_id = PRIME_IDS[prime_name]
        else:
            inp.prime_id = 255
        for i, l in enumerate(_limbs(sys_.p)):
            inp.prime[i] = l
        inp.max_signal = sys_.max_signal
        inp.n_pub_out, inp.n_pub_in, inp.n_priv_in = sys_.n_pub_out, sys_.n_pub_in, sys_.n_priv_in
        inp.n_forbidden = len(self.forb)
        inp.forbidden = self.forb.ctypes.data_as(C.POINTER(C.c_uint32))
        inp.cons_eq, inp.eq, inp.linear, inp.nl_a, inp.nl_b, inp.nl_c = [b.lc for b in self.blocks]
        self.inp = inp


def _read_block(b: RsLc, end=None) -> List[dict]:
    n = b.n_rows
    if n == 0:
        return []
    ptr, col, val = _lc_arrays(b, end)
    out = []
    for r in range(n):
        m = {}
        for e in range(int(ptr[r]), int(ptr[r + 1])):
            v = 0
            for i in range(4):
                v |= int(val[4 * e + i]) << (64 * i)
            m[int(col[e])] = v
        out.append(m)
    return out


def output_to_py(o: RsOutput):
    """-> (list of pyref.Con, signal_map dict label->wire, n_wires, no_private_inputs_witness)."""
    a, b, c = (_read_block(*o.block(q)) for q in range(3))
    cons = [R.Con(a[i], b[i], c[i]) for i in range(o.n_constraints)]
    l2w = np.ctypeslib.as_array(o.label_to_wire, shape=(max(o.n_labels, 1),))[: o.n_labels]
    sm = {i: int(w) for i, w in enumerate(l2w) if w >= 0}
    return cons, sm, int(o.n_wires), int(o.no_private_inputs_witness)


def same_result(res: "R.Result", got) -> str | None:
    """None if equal, else a description of the first difference."""
    cons, sm, nw, npiw = got
    if sm != res.signal_map:
        return f"signal_map differs: {len(sm)} vs {len(res.signal_map)} wires"
    if nw != len(res.signal_map):
        return "n_wires differs"
    if npiw != res.no_private_inputs_witness:
        return f"no_private_inputs_witness {npiw} vs {res.no_private_inputs_witness}"
    if len(cons) != len(res.constraints):
        return f"#constraints {len(cons)} vs {len(res.constraints)}"
    for i, (x, y) in enumerate(zip(cons, res.constraints)):
        if (x.a, x.b, x.c) != (y.a, y.b, y.c):
            return f"constraint {i} differs: {x} vs {y}"
    return None


def output_log(o: RsOutput):
    """The substitution log of an rs_output as [(from, {signal: value})] (reference order)."""
    n = int(o.n_log)
    if n == 0:
        return []
    frm = np.ctypeslib.as_array(o.log_from, shape=(n,))
    rows = _read_block(o.log_to)
    return [(int(frm[i]), rows[i]) for i in range(n)]


def pyref_log(log):
    """pyref's log (list of Sub) as [(from, {signal: value})]."""
    return [(s.frm, dict(s.to)) for s in log]


# --------------------------------------------------------------------------- JSON text formats
# Restatements of the reference writers, for the tests: json_porting.rs:16-26 (hashmap_as_json, keys
# sorted as numbers, decimal values) with JsonValue::to_string (compact), ConstraintJSON
# (json_writer.rs:4-45) and SubstitutionJSON (json_writer.rs:94-131).
def json_map(m: dict) -> str:
    return "{" + ",".join(f'"{k}":"{m[k]}"' for k in sorted(m)) + "}"


def constraints_json_text(cons, signal_map) -> str:
    """port_constraints (json_porting.rs:36-48): rows with apply_correspondence."""
    out = '{\n"constraints": ['
    for i, c in enumerate(cons):
        row = ",".join(json_map({signal_map[k]: v for k, v in m.items()}) for m in (c.a, c.b, c.c))
        out += ("\n[" if i == 0 else ",\n[") + row + "]"
    return out + "\n]\n}"


def substitutions_json_text(log) -> str:
    """log_substitutions -> SubstitutionJSON::write_substitution for each (from, to)."""
    out = "{"
    for i, (frm, to) in enumerate(log):
        out += ("\n" if i == 0 else ",\n") + f'"{frm}" : ' + json_map(to)
    return out + "\n}"


class OutputHolder:
    """An RsOutput over numpy arrays, built from a pyref Result (+ log): feeds the product's file
    writers on the CPU."""

    def __init__(self, res: "R.Result", n_labels: int, log=()):
        self.blocks = [_Block([c.a for c in res.constraints]), _Block([c.b for c in res.constraints]),
                       _Block([c.c for c in res.constraints])]
        self.l2w = np.array([res.signal_map.get(i, -1) for i in range(n_labels)] or [0], dtype=np.int32)
        self.log_blk = _Block([to for _, to in log])
        self.log_from = np.array([f for f, _ in log] or [0], dtype=np.uint32)
        o = RsOutput()
        o.n_constraints = len(res.constraints)
        o.a, o.b, o.c = [b.lc for b in self.blocks]
        o.n_labels = n_labels
        o.label_to_wire = self.l2w.ctypes.data_as(C.POINTER(C.c_int32))
        o.n_wires = len(res.signal_map)
        o.no_private_inputs_witness = res.no_private_inputs_witness
        o.n_log = len(log)
        o.log_from = self.log_from.ctypes.data_as(C.POINTER(C.c_uint32))
        o.log_to = self.log_blk.lc
        self.out = o


# --------------------------------------------------------------------------- oracle library
_ORACLE = None


def oracle_lib():
    global _ORACLE
    if _ORACLE is None:
        path = os.path.join(ROOT, "oracle", "_ref", "librefcpu.so")
        if not os.path.exists(path):
            import subprocess
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        lib = C.CDLL(path)
        lib.refcpu_simplify.argtypes = [C.POINTER(RsInput), C.POINTER(RsFlags), C.c_int,
                                        C.POINTER(C.POINTER(RsOutput)), C.POINTER(C.c_double),
                                        C.POINTER(C.c_uint64)]
        lib.refcpu_simplify.restype = C.c_int
        lib.refcpu_output_free.argtypes = [C.POINTER(RsOutput)]
        lib.refcpu_last_alg.argtypes = [C.c_uint64 * 11]
        lib.refcpu_last_alg.restype = None
        lib.refcpu_last_error.restype = C.c_char_p
        lib.refcpu_field_op.argtypes = [C.c_uint64 * 4, C.c_int, C.c_uint64 * 4, C.c_uint64 * 4,
                                        C.c_uint64 * 4]
        _ORACLE = lib
    return _ORACLE


def oracle_run(inp: RsInput, fl: RsFlags, threads=1):
    lib = oracle_lib()
    out = C.POINTER(RsOutput)()
    ms = C.c_double()
    rounds = C.c_uint64()
    rc = lib.refcpu_simplify(C.byref(inp), C.byref(fl), threads, C.byref(out), C.byref(ms),
                             C.byref(rounds))
    if rc != 0:
        raise RuntimeError(f"refcpu rc={rc}: {lib.refcpu_last_error().decode()}")
    try:
        return output_to_py(out.contents), ms.value, rounds.value
    finally:
        lib.refcpu_output_free(out)


# --------------------------------------------------------------------------- random systems
def gen_system(seed: int, p: int, n_sig: int = 60, n_rows: int = 80, n_out: int = 2,
               n_pub: int = 2, big_cluster: int = 0, density: float = 1.0, extra_forb: float = 0.0) -> "R.System":
    """Seeded random --O0 system that exercises every branch of the path: eq clusters of size 1
    and > 1 with forbidden ends, duplicate/forbidden constant equalities, linear clusters for
    process_3 and (big_cluster >= 350) process_4, non-linear rows that turn linear in round 1 and
    in later rounds, constant-A reductions and coefficient cancellations (small p).  extra_forb: the
    share of the other signals that are forbidden too (custom-gate signals, forbidden intermediates)."""
    rng = random.Random(seed)
    S = n_sig + 1
    n_priv = max(1, min(4, n_sig - n_out - n_pub))

    def coef():
        r = rng.random()
        if r < 0.35:
            return 1
        if r < 0.55:
            return p - 1
        if r < 0.7:
            return pow(2, rng.randrange(1, 8), p)
        return rng.randrange(1, p)

    def sig():
        return rng.randrange(1, S)

    def lc(nmin, nmax, const_prob=0.3):
        m = {}
        for _ in range(rng.randint(nmin, nmax)):
            m[sig()] = coef()
        if rng.random() < const_prob:
            m[0] = coef()
        return {k: v for k, v in m.items() if v % p}

    rows = []
    for _ in range(n_rows):
        r = rng.random()
        if r < 0.22:        # equality x - y (scaled)
            x, y = sig(), sig()
            if x == y:
                continue
            k = coef()
            rows.append(R.Con({}, {}, {x: k, y: (p - k) % p}))
        elif r < 0.30:      # constant equality
            m = {sig(): coef()}
            if rng.random() < 0.6:
                m[0] = coef()
            rows.append(R.Con({}, {}, m))
        elif r < 0.62:      # linear
            m = lc(2, int(2 + 4 * density))
            if len([k for k in m if k]) >= 2:
                rows.append(R.Con({}, {}, m))
        else:               # quadratic
            a = lc(1, 2, 0.15)
            b = lc(1, 3, 0.2)
            if rng.random() < 0.08:
                a = {0: coef()}
            c = lc(0, 3, 0.2)
            if a or b:
                rows.append(R.Con(a, b, c))
    if big_cluster:
        base = rng.randrange(1, max(2, S - 8))
        for i in range(big_cluster):
            m = {}
            for _ in range(rng.randint(2, 4)):
                m[1 + (base + rng.randrange(0, 24) + i // 2) % (S - 1)] = coef()
            if rng.random() < 0.3:
                m[0] = coef()
            m = {k: v for k, v in m.items() if v}
            if len([k for k in m if k]) >= 3:
                rows.append(R.Con({}, {}, m))
    forb = {0} | set(range(1, n_out + n_pub + 1))
    if extra_forb:
        frng = random.Random(seed ^ 0x5eed)
        forb |= {s for s in range(n_out + n_pub + 1, S) if frng.random() < extra_forb}
    return R.System(p, S, n_out, n_pub, n_priv, forb, rows)


# --------------------------------------------------------------------------- array comparison
def _lc_arrays(b: RsLc, end=None):
    return block_csr(b, end)


def output_arrays(o: RsOutput):
    """All arrays of an rs_output, copied (numpy): for size-independent comparisons at full size."""
    d = {"n_constraints": int(o.n_constraints), "n_wires": int(o.n_wires),
         "npiw": int(o.no_private_inputs_witness), "n_labels": int(o.n_labels)}
    for q, nm in enumerate(("a", "b", "c")):
        d[nm] = _lc_arrays(*o.block(q))
    d["l2w"] = np.ctypeslib.as_array(o.label_to_wire, shape=(max(int(o.n_labels), 1),))[: int(o.n_labels)].copy()
    return d


def diff_output_arrays(x, y) -> str | None:
    for k in ("n_constraints", "n_wires", "npiw", "n_labels"):
        if x[k] != y[k]:
            return f"{k}: {x[k]} vs {y[k]}"
    if not np.array_equal(x["l2w"], y["l2w"]):
        return f"label_to_wire differs at {int(np.argmax(x['l2w'] != y['l2w']))}"
    for nm in ("a", "b", "c"):
        for i, part in enumerate(("ptr", "col", "val")):
            if not np.array_equal(x[nm][i], y[nm][i]):
                return f"{nm}.{part} differs"
    return None


ALG_TERMS = ("B_alg", "z_in", "z_out", "subs", "app", "rowupd", "merges", "r_in", "r_out", "max_signal", "w")


def oracle_last_alg() -> dict:
    """The algorithmic bytes of this thread's last oracle run (refcpu_last_alg: SURVEY 8(d)'s B_alg over
    the canonical execution's logical operations) and its terms."""
    a = (C.c_uint64 * 11)()
    oracle_lib().refcpu_last_alg(a)
    return dict(zip(ALG_TERMS, (int(x) for x in a)))


def oracle_arrays(inp: RsInput, fl: RsFlags, threads=1):
    lib = oracle_lib()
    out = C.POINTER(RsOutput)()
    ms = C.c_double()
    rounds = C.c_uint64()
    rc = lib.refcpu_simplify(C.byref(inp), C.byref(fl), threads, C.byref(out), C.byref(ms), C.byref(rounds))
    if rc != 0:
        raise RuntimeError(f"refcpu rc={rc}: {lib.refcpu_last_error().decode()}")
    try:
        return output_arrays(out.contents), ms.value
    finally:
        lib.refcpu_output_free(out)
