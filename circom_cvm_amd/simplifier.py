"""Host-side mirror of the reference interface for this path.

    Simplifier { field, forbidden, cons_equalities, equalities, linear, dag_encoding, max_signal,
                 no_rounds, flag_s, flag_old_heuristics, ... }.simplify_constraints()
        -> ConstraintList { constraints, signal_map, no_private_inputs_witness, ... }
    (constraint_list/src/lib.rs:110-202) with the ConstraintExporter methods r1cs / sym /
    json_constraints (constraint_writers/src/lib.rs:8-12).

The inputs are an rs_input (the Simplifier bundle as arrays); the work is done by librs_simplify on
the GPU.  Same names, argument meaning and error behaviour (errors surface as RsError where the
reference panics or returns Err(()))."""
from __future__ import annotations

import ctypes as C
from typing import Dict, List

import numpy as np

from . import abi
from .abi import Engine, Input, Output, RsInput, check, lib, make_flags


class ConstraintList:
    """Result of Simplifier.simplify_constraints (constraint_list/src/lib.rs:155-202)."""

    def __init__(self, inp: Input | RsInput, out: Output):
        self._inp = inp
        self._out = out

    @property
    def _rs_input(self) -> RsInput:
        return self._inp.c if isinstance(self._inp, Input) else self._inp

    @property
    def no_private_inputs_witness(self) -> int:
        return int(self._out.c.no_private_inputs_witness)

    def no_labels(self) -> int:
        return int(self._out.c.n_labels)

    def no_wires(self) -> int:
        return int(self._out.c.n_wires)

    def label_to_wire(self) -> np.ndarray:
        o = self._out.c
        return np.ctypeslib.as_array(o.label_to_wire, shape=(max(int(o.n_labels), 1),))[: o.n_labels].copy()

    def get_witness(self) -> Dict[int, int]:
        l2w = self.label_to_wire()
        return {int(s): int(w) for s, w in enumerate(l2w) if w >= 0}

    def get_witness_as_vec(self) -> List[int]:
        """constraint_list/src/lib.rs:187-193."""
        l2w = self.label_to_wire()
        wit = [0] * self.no_wires()
        for s, w in enumerate(l2w):
            if w >= 0:
                wit[int(w)] = s
        return wit

    def r1cs(self, out: str, custom_gates: bool = False) -> None:
        if custom_gates:
            raise NotImplementedError("custom gates are out of scope for this back end")
        check(lib().rs_write_r1cs(out.encode(), C.byref(self._rs_input), self._out.ptr))

    def sym(self, o0_sym: str, out: str) -> None:
        check(lib().rs_write_sym(o0_sym.encode(), out.encode(), self._out.ptr))

    def json_constraints_file(self, out: str) -> None:
        """ConstraintExporter::json_constraints (constraint_list/src/lib.rs:195-201): --json."""
        check(lib().rs_write_constraints_json(out.encode(), self._out.ptr))

    def substitutions(self) -> list:
        """The --simplification_substitution log as [(from, {signal: value})] (original ids, reference
        order); empty unless the Simplifier was built with port_substitution=True."""
        o = self._out.c
        n = int(o.n_log)
        if n == 0:
            return []
        frm = np.ctypeslib.as_array(o.log_from, shape=(n,))
        ptr = np.ctypeslib.as_array(o.log_to.ptr, shape=(n + 1,))
        nnz = int(ptr[n])
        col = np.ctypeslib.as_array(o.log_to.col, shape=(max(nnz, 1),))
        val = np.ctypeslib.as_array(o.log_to.val, shape=(max(nnz, 1) * 4,))
        res = []
        for i in range(n):
            m = {}
            for e in range(int(ptr[i]), int(ptr[i + 1])):
                m[int(col[e])] = sum(int(val[4 * e + t]) << (64 * t) for t in range(4))
            res.append((int(frm[i]), m))
        return res

    def substitution_json_file(self, out: str) -> None:
        """SubstitutionJSON (constraint_writers/src/json_writer.rs:94-131) of the log."""
        check(lib().rs_write_substitution_json(out.encode(), self._out.ptr))

    def json_constraints(self) -> list:
        """constraint_list/src/json_porting.rs:8-48 as Python objects (wire ids, decimal strings)."""
        o = self._out.c
        l2w = self.label_to_wire()
        out = []
        blocks = []
        for q in range(3):
            blocks.append(abi.block_csr(*o.block(q)))
        for r in range(int(o.n_constraints)):
            row = []
            for ptr, col, val in blocks:
                m = {}
                for e in range(int(ptr[r]), int(ptr[r + 1])):
                    k = int(col[e])
                    w = 0 if k == 0 else int(l2w[k])
                    v = sum(int(val[4 * e + i]) << (64 * i) for i in range(4))
                    m[w] = str(v)
                row.append({str(k): m[k] for k in sorted(m)})
            out.append(row)
        return out


class Simplifier:
    """constraint_list::Simplifier (lib.rs:110-153) over an rs_input bundle."""

    def __init__(self, inp: Input | RsInput, no_rounds: int | None = None, flag_s: bool = False,
                 flag_old_heuristics: bool = False, device: int = 0, port_substitution: bool = False):
        self.inp = inp
        if flag_s:
            self.flags = make_flags("O1", old=flag_old_heuristics, device=device, log=port_substitution)
        else:
            self.flags = make_flags("O2", rounds=no_rounds, old=flag_old_heuristics, device=device,
                                    log=port_substitution)
        self.device = device

    def no_labels(self) -> int:
        c = self.inp.c if isinstance(self.inp, Input) else self.inp
        return int(c.max_signal)

    def simplify_constraints(self) -> ConstraintList:
        rs_in = self.inp.c if isinstance(self.inp, Input) else self.inp
        eng = Engine(self.device)
        try:
            eng.load(rs_in)
            eng.run(self.flags)
            out = eng.fetch()
        finally:
            eng.close()
        return ConstraintList(self.inp, out)
