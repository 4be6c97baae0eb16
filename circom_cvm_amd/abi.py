"""ctypes binding of include/rs_simplify.h (librs_simplify.so, built in-tree for gfx950).

The library is the product: there is no Python or CPU fallback.  Loading fails loudly when the
shared object is missing, and every compute entry point returns RS_E_NODEVICE without a gfx950
GPU."""
from __future__ import annotations

import ctypes as C

import numpy as np
import os

PKG = os.path.dirname(os.path.abspath(__file__))
# RS_LIB: an alternative build of the same library (e.g. the RS_KCLOCKS diagnostic variant)
LIB_PATH = os.environ.get("RS_LIB") or os.path.join(PKG, "librs_simplify.so")

U64_MAX = (1 << 64) - 1
PRIME_IDS = {"bn128": 0, "bls12381": 1, "goldilocks": 2, "grumpkin": 3, "pallas": 4,
             "vesta": 5, "secq256r1": 6, "bls12377": 7}
RS_PRIME_CUSTOM = 255
ERRORS = {0: "RS_OK", -1: "RS_E_INVALID", -2: "RS_E_OOM_DEVICE", -3: "RS_E_HIP",
          -4: "RS_E_RCCL", -5: "RS_E_INTERNAL", -6: "RS_E_NODEVICE"}


class RsLc(C.Structure):
    _fields_ = [("n_rows", C.c_uint64), ("nnz", C.c_uint64), ("ptr", C.POINTER(C.c_uint64)),
                ("col", C.POINTER(C.c_uint32)), ("val", C.POINTER(C.c_uint64))]


class RsInput(C.Structure):
    _fields_ = [("prime_id", C.c_uint32), ("prime", C.c_uint64 * 4), ("max_signal", C.c_uint64),
                ("n_pub_out", C.c_uint64), ("n_pub_in", C.c_uint64), ("n_priv_in", C.c_uint64),
                ("n_forbidden", C.c_uint64), ("forbidden", C.POINTER(C.c_uint32)),
                ("cons_eq", RsLc), ("eq", RsLc), ("linear", RsLc),
                ("nl_a", RsLc), ("nl_b", RsLc), ("nl_c", RsLc)]


class RsFlags(C.Structure):
    _fields_ = [("flag_s", C.c_uint32), ("use_old_heuristics", C.c_uint32),
                ("no_rounds", C.c_uint64), ("emit_substitution_log", C.c_uint32),
                ("device", C.c_int32)]


class RsOutput(C.Structure):
    _fields_ = [("n_constraints", C.c_uint64), ("a", RsLc), ("b", RsLc), ("c", RsLc),
                ("n_labels", C.c_uint64), ("label_to_wire", C.POINTER(C.c_int32)),
                ("n_wires", C.c_uint64), ("no_private_inputs_witness", C.c_uint64),
                ("n_log", C.c_uint64), ("log_from", C.POINTER(C.c_uint32)), ("log_to", RsLc),
                ("a_len", C.POINTER(C.c_uint32)), ("b_len", C.POINTER(C.c_uint32)), ("c_len", C.POINTER(C.c_uint32)),
                ("a_jump", C.POINTER(C.c_uint64)), ("b_jump", C.POINTER(C.c_uint64)), ("c_jump", C.POINTER(C.c_uint64)),
                ("a_njump", C.c_uint64), ("b_njump", C.c_uint64), ("c_njump", C.c_uint64)]

    def block(self, q: int):
        """(rs_lc, its ABI 8 row layout (len, jump, n_jump) or None for CSR) of part q = 0/1/2 (a/b/c)."""
        lc = (self.a, self.b, self.c)[q]
        ln = (self.a_len, self.b_len, self.c_len)[q]
        if not ln:
            return lc, None
        return lc, (ln, (self.a_jump, self.b_jump, self.c_jump)[q], int((self.a_njump, self.b_njump, self.c_njump)[q]))


ROW_JUMP = 0x80000000


def row_starts(lens: np.ndarray, jumps: np.ndarray) -> np.ndarray:
    """The storage start of every row of ABI 8's streamed layout (rs_rows_next, include/rs_simplify.h):
    a row starts where the previous one ended unless RS_ROW_JUMP is set, then at the next jump."""
    n = lens.shape[0]
    j = (lens & ROW_JUMP) != 0
    ln = (lens & ~np.uint32(ROW_JUMP)).astype(np.int64)
    if int(j.sum()) != jumps.shape[0]:
        raise ValueError("row layout: %d jumping rows, %d jump offsets" % (int(j.sum()), jumps.shape[0]))
    seg = np.cumsum(j) - 1  # the jump each row's run starts from (-1: the run from offset 0)
    last = np.maximum.accumulate(np.where(j, np.arange(n), -1)) if n else np.zeros(0, np.int64)
    ex = np.zeros(n + 1, np.int64)
    np.cumsum(ln, out=ex[1:])
    base = np.where(seg >= 0, jumps.astype(np.int64)[np.maximum(seg, 0)] if jumps.size else 0, 0)
    return base + ex[:-1] - np.where(last >= 0, ex[np.maximum(last, 0)], 0)


def block_csr(lc: "RsLc", layout=None):
    """Copies of one result block as compact CSR numpy arrays (ptr u64[n+1], col u32, val u64[4 nnz]):
    a block in ABI 8's streamed layout (row lengths + jumps) is compacted row by row."""
    n = int(lc.n_rows)
    if n == 0:
        return np.zeros(1, np.uint64), np.zeros(0, np.uint32), np.zeros(0, np.uint64)
    ext = int(lc.nnz)
    col = np.ctypeslib.as_array(lc.col, shape=(max(ext, 1),))
    val = np.ctypeslib.as_array(lc.val, shape=(max(ext, 1) * 4,))
    if layout is None:
        beg = np.ctypeslib.as_array(lc.ptr, shape=(n + 1,)).copy()
        nnz = int(beg[n])
        return beg, col[:nnz].copy(), val[:4 * nnz].copy()
    lp, jp, nj = layout
    lens = np.ctypeslib.as_array(lp, shape=(n,))
    jumps = np.ctypeslib.as_array(jp, shape=(nj,)) if nj else np.zeros(0, np.uint64)
    b = row_starts(lens, jumps)
    ln = (lens & ~np.uint32(ROW_JUMP)).astype(np.int64)
    if n and int((b + ln).max()) > ext:
        raise ValueError("row layout reaches past the block's entries")
    ptr = np.zeros(n + 1, np.uint64)
    np.cumsum(ln, out=ptr[1:])
    idx = np.repeat(b - ptr[:-1].astype(np.int64), ln) + np.arange(int(ptr[n]), dtype=np.int64)
    v4 = val[: 4 * ext].reshape(-1, 4)
    return ptr, col[idx].copy(), v4[idx].reshape(-1).copy()


class RsStats(C.Structure):
    _fields_ = [("total_ms", C.c_double), ("eq_ms", C.c_double), ("cluster_ms", C.c_double),
                ("elim_ms", C.c_double), ("subst_ms", C.c_double), ("final_ms", C.c_double),
                ("apply_kernel_ms", C.c_double), ("apply_kernel_launches", C.c_uint64),
                ("apply_bytes", C.c_uint64), ("elim_kernel_ms", C.c_double),
                ("elim_kernel_launches", C.c_uint64), ("elim_bytes", C.c_uint64),
                ("elim_big_ms", C.c_double), ("elim_small_ms", C.c_double), ("nl_ms", C.c_double),
                ("map_ms", C.c_double), ("rounds_ms", C.c_double),
                ("big_prep_ms", C.c_double), ("big_main_ms", C.c_double), ("big_finish_ms", C.c_double),
                ("big_main_bytes", C.c_uint64), ("big_finish_bytes", C.c_uint64), ("big_launches", C.c_uint64),
                ("rounds", C.c_uint64), ("n_clusters", C.c_uint64),
                ("n_substitutions", C.c_uint64), ("max_cluster", C.c_uint64),
                ("exchange_ms", C.c_double), ("exchange_bytes", C.c_uint64), ("world", C.c_uint64),
                ("head_main_ms", C.c_double), ("head_main_bytes", C.c_uint64), ("head_launches", C.c_uint64),
                ("tail_main_ms", C.c_double), ("tail_main_bytes", C.c_uint64), ("tail_launches", C.c_uint64),
                ("round_fill_ms", C.c_double), ("round_fill_bytes", C.c_uint64),
                ("round_fill_launches", C.c_uint64), ("alg_bytes", C.c_uint64), ("h2d_wait_ms", C.c_double),
                ("d2h_ms", C.c_double), ("host_total_ms", C.c_double), ("write_ms", C.c_double),
                ("tail_fin_ms", C.c_double), ("tail_fin_bytes", C.c_uint64), ("tail_fin_launches", C.c_uint64), ("head_fin_ms", C.c_double), ("head_fin_bytes", C.c_uint64), ("head_fin_launches", C.c_uint64), ("small_ms", C.c_double), ("small_bytes", C.c_uint64), ("small_launches", C.c_uint64), ("prep_ms", C.c_double), ("prep_launches", C.c_uint64), ("cluster_dev_ms", C.c_double), ("cluster_bytes", C.c_uint64), ("cluster_launches", C.c_uint64), ("giant_ms", C.c_double), ("giant_bytes", C.c_uint64), ("giant_launches", C.c_uint64), ("giant_merges", C.c_uint64),
                ("check_ms", C.c_double), ("check_bytes", C.c_uint64), ("check_launches", C.c_uint64),
                ("ragged_ms", C.c_double), ("ragged_bytes", C.c_uint64), ("ragged_launches", C.c_uint64),
                ("gather_ms", C.c_double), ("gather_bytes", C.c_uint64), ("gather_launches", C.c_uint64),
                ("cluster_host_ms", C.c_double)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class RsDag(C.Structure):
    """rs_dag: the component DAG rs_flatten_dag expands."""
    _fields_ = [("prime_id", C.c_uint32), ("prime", C.c_uint64 * 4),
                ("n_pub_out", C.c_uint64), ("n_pub_in", C.c_uint64), ("n_priv_in", C.c_uint64),
                ("n_forbidden", C.c_uint64), ("forbidden", C.POINTER(C.c_uint32)),
                ("n_nodes", C.c_uint32), ("main_node", C.c_uint32),
                ("cons_off", C.POINTER(C.c_uint64)), ("a", RsLc), ("b", RsLc), ("c", RsLc),
                ("local_off", C.POINTER(C.c_uint64)), ("locals", C.POINTER(C.c_uint32)),
                ("custom_gate", C.POINTER(C.c_uint8)),
                ("edge_off", C.POINTER(C.c_uint64)), ("edge_to", C.POINTER(C.c_uint32)),
                ("edge_in", C.POINTER(C.c_uint64))]


# (name, restype, argtypes) of every symbol include/rs_simplify.h declares
SYMBOLS = [
    ("rs_last_error", C.c_char_p, []),
    ("rs_abi_version", C.c_int, []),
    ("rs_simplify", C.c_int, [C.POINTER(RsInput), C.POINTER(RsFlags), C.POINTER(C.POINTER(RsOutput))]),
    ("rs_output_free", None, [C.POINTER(RsOutput)]),
    ("rs_engine_create", C.c_int, [C.c_int, C.POINTER(C.c_void_p)]),
    ("rs_engine_load", C.c_int, [C.c_void_p, C.POINTER(RsInput)]),
    ("rs_engine_run", C.c_int, [C.c_void_p, C.POINTER(RsFlags)]),
    ("rs_engine_fetch", C.c_int, [C.c_void_p, C.POINTER(C.POINTER(RsOutput))]),
    ("rs_engine_stats", C.c_int, [C.c_void_p, C.POINTER(RsStats)]),
    ("rs_engine_destroy", None, [C.c_void_p]),
    ("rs_engine_write_r1cs", C.c_int, [C.c_void_p, C.c_char_p, C.c_char_p]),
    ("rs_engine_simplify", C.c_int, [C.c_void_p, C.POINTER(RsInput), C.POINTER(RsFlags),
                                     C.POINTER(C.POINTER(RsOutput))]),
    ("rs_host_alloc", C.c_void_p, [C.c_uint64]),
    ("rs_host_free", None, [C.c_void_p]),
    ("rs_comm_unique_id", C.c_int, [C.POINTER(C.c_uint8)]),
    ("rs_engine_join_rccl", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_uint8)]),
    ("rs_group_create", C.c_void_p, [C.c_int]),
    ("rs_engine_join_group", C.c_int, [C.c_void_p, C.c_void_p, C.c_int]),
    ("rs_engine_join_host", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_char_p]),
    ("rs_group_destroy", None, [C.c_void_p]),
    ("rs_simplify_multi", C.c_int, [C.POINTER(RsInput), C.POINTER(RsFlags), C.c_int, C.POINTER(C.c_int),
                                    C.POINTER(C.POINTER(RsOutput))]),
    ("rs_engine_inject_fault", C.c_int, [C.c_void_p, C.c_int]),
    ("rs_read_r1cs_o0", C.c_int, [C.c_char_p, C.POINTER(C.POINTER(RsInput))]),
    ("rs_input_free", None, [C.POINTER(RsInput)]),
    ("rs_write_r1cs", C.c_int, [C.c_char_p, C.POINTER(RsInput), C.POINTER(RsOutput)]),
    ("rs_write_r1cs_gates", C.c_int, [C.c_char_p, C.POINTER(RsInput), C.POINTER(RsOutput), C.c_char_p]),
    ("rs_write_sym", C.c_int, [C.c_char_p, C.c_char_p, C.POINTER(RsOutput)]),
    ("rs_write_constraints_json", C.c_int, [C.c_char_p, C.POINTER(RsOutput)]),
    ("rs_write_substitution_json", C.c_int, [C.c_char_p, C.POINTER(RsOutput)]),
    ("rs_synth", C.c_int, [C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint32, C.POINTER(C.POINTER(RsInput))]),
    ("rs_flatten_dag", C.c_int, [C.c_int, C.POINTER(RsDag), C.POINTER(C.POINTER(RsInput))]),
    ("rs_engine_flatten_dag", C.c_int, [C.c_void_p, C.POINTER(RsDag), C.POINTER(C.POINTER(RsInput))]),
]

_LIB = None


class RsError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


def lib():
    """The loaded librs_simplify.so (raises if it was not built)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: run `python -c 'import __graft_entry__ as g; g.build()'`")
        L = C.CDLL(LIB_PATH)
        for name, res, args in SYMBOLS:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _LIB = L
    return _LIB


def check(rc: int):
    if rc != 0:
        raise RsError(rc, lib().rs_last_error().decode(errors="replace"))


def make_flags(level: str = "O2", rounds: int | None = None, old: bool = False, device: int = 0,
               log: bool = False) -> RsFlags:
    """--O1 / --O2 / --O2round N (circom/src/input_user.rs:286-306); log = --simplification_substitution."""
    f = RsFlags()
    f.emit_substitution_log = 1 if log else 0
    if level == "O1" or rounds == 0:
        f.flag_s, f.no_rounds = 1, 0
    elif level == "O2":
        f.flag_s, f.no_rounds = 0, U64_MAX if rounds is None else rounds
    else:
        raise ValueError(level)
    f.use_old_heuristics = 1 if old else 0
    f.device = device
    return f


COMM_ID_BYTES = 128


def comm_unique_id() -> bytes:
    """rs_comm_unique_id: the RCCL id rank 0 creates and broadcasts before rs_engine_join_rccl."""
    buf = (C.c_uint8 * COMM_ID_BYTES)()
    check(lib().rs_comm_unique_id(buf))
    return bytes(buf)


class Group:
    """An in-process rank group (rs_group_*): several engines in one process, one per thread, with
    host-staged collectives -- the sharded path on a single GPU."""

    def __init__(self, world: int):
        self.world = world
        self._h = lib().rs_group_create(world)
        if not self._h:
            raise ValueError(f"bad world size {world}")

    def close(self):
        if self._h:
            lib().rs_group_destroy(self._h)
            self._h = None


def simplify_multi(inp: RsInput, flags: RsFlags, devices) -> "Output":
    """rs_simplify_multi: one-shot sharded simplification over `devices` (threads in this process)."""
    arr = (C.c_int * len(devices))(*devices)
    out = C.POINTER(RsOutput)()
    check(lib().rs_simplify_multi(C.byref(inp), C.byref(flags), len(devices), arr, C.byref(out)))
    return Output(out)


class Engine:
    """HBM-resident simplification engine (rs_engine_*)."""

    def __init__(self, device: int = 0):
        self._h = C.c_void_p()
        check(lib().rs_engine_create(device, C.byref(self._h)))

    def join_rccl(self, world: int, rank: int, uid: bytes):
        """Rank `rank` of a sharded run over RCCL (collective: every rank must call it)."""
        buf = (C.c_uint8 * COMM_ID_BYTES).from_buffer_copy(uid)
        check(lib().rs_engine_join_rccl(self._h, world, rank, buf))

    def join_group(self, group: Group, rank: int):
        check(lib().rs_engine_join_group(self._h, group._h, rank))

    def join_host(self, world: int, rank: int, tag: str):
        """Rank `rank` of a group of processes on one host (rs_engine_join_host: the test transport
        whose collectives go through POSIX shared memory; collective, every rank passes `tag`)."""
        check(lib().rs_engine_join_host(self._h, world, rank, tag.encode()))

    def load(self, inp: RsInput):
        check(lib().rs_engine_load(self._h, C.byref(inp)))

    def run(self, flags: RsFlags):
        check(lib().rs_engine_run(self._h, C.byref(flags)))

    def stats(self) -> RsStats:
        s = RsStats()
        check(lib().rs_engine_stats(self._h, C.byref(s)))
        return s

    def fetch(self):
        out = C.POINTER(RsOutput)()
        check(lib().rs_engine_fetch(self._h, C.byref(out)))
        return Output(out)

    def simplify(self, inp: RsInput, flags: RsFlags) -> RsOutput:
        """rs_engine_simplify: host input -> host output (the SURVEY 8(d) T_simplify region).  The
        returned struct views the engine's pinned buffers: valid until the next call on this engine."""
        out = C.POINTER(RsOutput)()
        check(lib().rs_engine_simplify(self._h, C.byref(inp), C.byref(flags), C.byref(out)))
        return out.contents

    def flatten_dag(self, dag) -> RsInput:
        """rs_engine_flatten_dag: `dag` (circom_cvm_amd.Dag) flattened into this engine's page-locked
        buffers; the returned struct views them until the next flatten_dag on this engine."""
        p = C.POINTER(RsInput)()
        check(lib().rs_engine_flatten_dag(self._h, C.byref(dag.c), C.byref(p)))
        return p.contents

    def inject_fault(self, where: int = 1):
        """rs_engine_inject_fault: the next run / simplify on this engine fails at `where` (tests)."""
        check(lib().rs_engine_inject_fault(self._h, where))

    def write_r1cs(self, path: str, o0_r1cs: str | None = None) -> float:
        """rs_engine_write_r1cs: the last result as a .r1cs file (device-built constraint section).
        Returns the write time (ms)."""
        check(lib().rs_engine_write_r1cs(self._h, path.encode(), o0_r1cs.encode() if o0_r1cs else None))
        return self.stats().write_ms

    def close(self):
        if self._h:
            lib().rs_engine_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Output:
    """Owns an rs_output*."""

    def __init__(self, ptr):
        self.ptr = ptr

    @property
    def c(self) -> RsOutput:
        s = self.ptr.contents
        s._owner = self  # the struct keeps its owner (and so the library's buffers) alive
        return s

    def free(self):
        if self.ptr:
            lib().rs_output_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Input:
    """Owns an rs_input* made by the library (r1cs reader or synthetic generator)."""

    def __init__(self, ptr):
        self.ptr = ptr

    @property
    def c(self) -> RsInput:
        s = self.ptr.contents
        s._owner = self
        return s

    @staticmethod
    def read_r1cs(path: str) -> "Input":
        p = C.POINTER(RsInput)()
        check(lib().rs_read_r1cs_o0(path.encode(), C.byref(p)))
        return Input(p)

    @staticmethod
    def synth(kind: int, rows: int, seed: int, prime: str = "bn128") -> "Input":
        p = C.POINTER(RsInput)()
        check(lib().rs_synth(kind, rows, seed, PRIME_IDS[prime], C.byref(p)))
        return Input(p)

    def rows(self) -> int:
        c = self.c
        return int(c.cons_eq.n_rows + c.eq.n_rows + c.linear.n_rows + c.nl_a.n_rows)

    def free(self):
        if self.ptr:
            lib().rs_input_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class PinnedInput:
    """A copy of an rs_input in page-locked host memory (rs_host_alloc), as a Rust shim marshalling
    the Simplifier into library-provided buffers would hold it: rs_engine_simplify's H2D then runs at
    PCIe speed."""

    _BLOCKS = ("cons_eq", "eq", "linear", "nl_a", "nl_b", "nl_c")

    def __init__(self, src: RsInput):
        L = lib()
        self._bufs = []
        dst = RsInput()
        C.memmove(C.byref(dst), C.byref(src), C.sizeof(RsInput))  # header + forbidden (borrowed from src)
        for nm in self._BLOCKS:
            b = getattr(src, nm)
            n, nnz = int(b.n_rows), int(b.nnz)
            ptr = self._copy(b.ptr, 8 * (n + 1) if n else 0, C.c_uint64)
            col = self._copy(b.col, 4 * nnz, C.c_uint32)
            val = self._copy(b.val, 32 * nnz, C.c_uint64)
            setattr(dst, nm, RsLc(n, nnz, ptr, col, val))
        self._src = src
        self.c = dst

    def _copy(self, src_ptr, nbytes, ctype):
        p = lib().rs_host_alloc(max(nbytes, 8))
        if not p:
            raise RuntimeError("rs_host_alloc failed (no device?)")
        self._bufs.append(p)
        if nbytes:
            C.memmove(p, src_ptr, nbytes)
        return C.cast(p, C.POINTER(ctype))

    def free(self):
        for p in self._bufs:
            lib().rs_host_free(p)
        self._bufs = []

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
