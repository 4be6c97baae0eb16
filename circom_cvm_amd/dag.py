"""Host-side builder of an rs_dag: the reference's component DAG (dag/src/lib.rs:141-176 Node, :87-100
Edge) in the flat arrays rs_flatten_dag expands on the device.

`nodes` are objects with `.constraints` (each with `.a`, `.b`, `.c`: {node-local signal: coefficient},
0 = the constant), `.locals` (the node's own signal ids), `.custom_gate` and `.edges` ([(child, in_number)]
in adjacency order) -- oracle/pyref.py's DagNode has that shape, as does anything a Rust shim would
marshal from `DAG::nodes` / `DAG::adjacency`."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi


def _limbs(v: int):
    return [(v >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(4)]


class _Csr:
    def __init__(self, maps, p):
        ptr, col, val = [0], [], []
        for m in maps:
            for k in sorted(m):
                col.append(k)
                val.extend(_limbs(m[k] % p))
            ptr.append(len(col))
        self.ptr = np.array(ptr, dtype=np.uint64)
        self.col = np.array(col if col else [0], dtype=np.uint32)
        self.val = np.array(val if val else [0, 0, 0, 0], dtype=np.uint64)
        self.lc = abi.RsLc(len(ptr) - 1, len(col), self.ptr.ctypes.data_as(C.POINTER(C.c_uint64)),
                           self.col.ctypes.data_as(C.POINTER(C.c_uint32)),
                           self.val.ctypes.data_as(C.POINTER(C.c_uint64)))


class Dag:
    """Owns the arrays behind an RsDag (`.c`)."""

    def __init__(self, p: int, nodes, main: int, n_pub_out: int, n_pub_in: int, n_priv_in: int, forbidden,
                 prime_name: str | None = None):
        cons = [c for nd in nodes for c in nd.constraints]
        self.parts = [_Csr([c.a for c in cons], p), _Csr([c.b for c in cons], p), _Csr([c.c for c in cons], p)]
        self.cons_off = np.cumsum([0] + [len(nd.constraints) for nd in nodes]).astype(np.uint64)
        self.local_off = np.cumsum([0] + [len(nd.locals) for nd in nodes]).astype(np.uint64)
        self.locals = np.array([s for nd in nodes for s in sorted(nd.locals)] or [0], dtype=np.uint32)
        self.cgate = np.array([1 if nd.custom_gate else 0 for nd in nodes], dtype=np.uint8)
        self.edge_off = np.cumsum([0] + [len(nd.edges) for nd in nodes]).astype(np.uint64)
        self.edge_to = np.array([e[0] for nd in nodes for e in nd.edges] or [0], dtype=np.uint32)
        self.edge_in = np.array([e[1] for nd in nodes for e in nd.edges] or [0], dtype=np.uint64)
        self.forb = np.array(sorted(forbidden) or [0], dtype=np.uint32)
        d = abi.RsDag()
        d.prime_id = abi.PRIME_IDS[prime_name] if prime_name else abi.RS_PRIME_CUSTOM
        for i, l in enumerate(_limbs(p)):
            d.prime[i] = l
        d.n_pub_out, d.n_pub_in, d.n_priv_in = n_pub_out, n_pub_in, n_priv_in
        d.n_forbidden = len(forbidden)
        d.forbidden = self.forb.ctypes.data_as(C.POINTER(C.c_uint32))
        d.n_nodes = len(nodes)
        d.main_node = main
        d.cons_off = self.cons_off.ctypes.data_as(C.POINTER(C.c_uint64))
        d.a, d.b, d.c = (x.lc for x in self.parts)
        d.local_off = self.local_off.ctypes.data_as(C.POINTER(C.c_uint64))
        d.locals = self.locals.ctypes.data_as(C.POINTER(C.c_uint32))
        d.custom_gate = self.cgate.ctypes.data_as(C.POINTER(C.c_uint8))
        d.edge_off = self.edge_off.ctypes.data_as(C.POINTER(C.c_uint64))
        d.edge_to = self.edge_to.ctypes.data_as(C.POINTER(C.c_uint32))
        d.edge_in = self.edge_in.ctypes.data_as(C.POINTER(C.c_uint64))
        self.c = d

    def flatten(self, device: int = 0) -> abi.Input:
        """rs_flatten_dag: the classified, offset constraint lists of every instance (an rs_input)."""
        p = C.POINTER(abi.RsInput)()
        abi.check(abi.lib().rs_flatten_dag(device, C.byref(self.c), C.byref(p)))
        return abi.Input(p)
