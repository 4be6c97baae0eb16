"""CPU tests of the drop-in boundary (include/rs_simplify.h, librs_simplify.so): the library loads,
exports exactly what the header declares, refuses to compute without a gfx950 GPU (no CPU fallback),
and its host-side pieces -- .r1cs reader/classifier, .r1cs/.sym writers, synthetic generator -- agree
with the oracle byte for byte.  No GPU compute is called here."""
import ctypes as C
import dataclasses
import os
import struct
import re
import subprocess
import tempfile

import numpy as np
import pytest

import rsio
import circom_cvm_amd as M
from circom_cvm_amd import abi

R = rsio.R
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "rs_simplify.h")
GOLD = os.path.join(ROOT, "tests", "golden")


def _header_functions():
    txt = open(HDR).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    txt = re.sub(r"^static inline .*$", "", txt, flags=re.M)  # header-only helpers (rs_rows_begin, rs_rows_next)
    return sorted(set(re.findall(r"^[A-Za-z_][\w \*]*?\b(rs_\w+)\s*\(", txt, flags=re.M)))


def _gpu_present():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def test_library_exports_every_header_symbol():
    L = abi.lib()
    declared = _header_functions()
    assert declared, "no declarations parsed"
    for name in declared:
        assert hasattr(L, name), f"{name} declared in rs_simplify.h but not exported"
    assert sorted(n for n, _, _ in abi.SYMBOLS) == declared


def test_abi_version_matches_header():
    v = int(re.search(r"#define RS_ABI_VERSION (\d+)", open(HDR).read()).group(1))
    assert abi.lib().rs_abi_version() == v


def test_status_codes_match_header():
    txt = open(HDR).read()
    for code, name in abi.ERRORS.items():
        if code:
            assert re.search(rf"{name}\s*=\s*{code}\b", txt), name


@pytest.mark.skipif(_gpu_present(), reason="checks the no-device path")
def test_no_cpu_fallback():
    """Without a gfx950 device every compute entry point fails loudly (RS_E_NODEVICE)."""
    L = abi.lib()
    h = C.c_void_p()
    rc = L.rs_engine_create(0, C.byref(h))
    assert rc == -6, rc
    assert b"gfx950" in L.rs_last_error() or b"device" in L.rs_last_error().lower()
    sys_ = R.System(257, 3, 1, 0, 1, {0, 1}, [R.Con({}, {}, {1: 1, 2: 256})])
    inp = rsio.InputHolder(sys_)
    out = C.POINTER(abi.RsOutput)()
    rc = L.rs_simplify(C.byref(inp.inp), C.byref(rsio.flags("O2")), C.byref(out))
    assert rc == -6 and not out


def test_synth_is_seeded_and_host_side():
    a = M.Input.synth(0, 20000, 7)
    b = M.Input.synth(0, 20000, 7)
    c = M.Input.synth(0, 20000, 8)

    def digest(inp):
        x = inp.c
        parts = []
        for blk in (x.cons_eq, x.eq, x.linear, x.nl_a, x.nl_b, x.nl_c):
            n = int(blk.n_rows)
            ptr = np.ctypeslib.as_array(blk.ptr, shape=(n + 1,)).copy()
            nnz = int(ptr[-1])
            parts += [ptr.tobytes(), np.ctypeslib.as_array(blk.col, shape=(max(nnz, 1),))[:nnz].tobytes(),
                      np.ctypeslib.as_array(blk.val, shape=(max(nnz, 1) * 4,))[:4 * nnz].tobytes()]
        return hash(b"".join(parts))

    assert a.rows() >= 20000
    assert digest(a) == digest(b) != digest(c)


def test_synth_rows_are_clean_and_classified():
    """Generator rows obey the input contract (sorted distinct columns, no zero, canonical) and land
    in the block map_tree would put them in (dag/src/map_to_constraint_list.rs:12-44)."""
    inp = M.Input.synth(0, 5000, 3, "bn128")
    x = inp.c
    p = R.PRIMES["bn128"]

    def rows(blk):
        return rsio._read_block(blk)

    for blk in (x.cons_eq, x.eq, x.linear, x.nl_a, x.nl_b, x.nl_c):
        for m in rows(blk):
            assert all(0 < v < p for v in m.values())
    for m in rows(x.cons_eq):
        assert R.is_constant_equality(R.Con({}, {}, m))
    for m in rows(x.eq):
        assert R.is_equality(R.Con({}, {}, m), p)
    for m in rows(x.linear):
        c = R.Con({}, {}, m)
        assert not R.is_constant_equality(c) and not R.is_equality(c, p)
    na, nb = rows(x.nl_a), rows(x.nl_b)
    assert len(na) == len(nb) == x.nl_c.n_rows
    assert all(a and b for a, b in zip(na, nb))


def _write(tmp, name, data):
    path = os.path.join(tmp, name)
    with open(path, "wb" if isinstance(data, bytes) else "w") as f:
        f.write(data)
    return path


def test_r1cs_reader_classifies_like_map_tree():
    sys_ = rsio.gen_system(31, R.PRIMES["bn128"], n_sig=60, n_rows=120)
    ident = R.Result(sys_.rows, {i: i for i in range(sys_.max_signal)}, sys_.n_priv_in)
    with tempfile.TemporaryDirectory() as tmp:
        path = _write(tmp, "in.r1cs", R.result_to_r1cs(sys_, ident))
        inp = M.Input.read_r1cs(path)
        x = inp.c
        ce, eq, lin, nl = R.classify(sys_)
        assert rsio._read_block(x.cons_eq) == [c.c for c in ce]
        assert rsio._read_block(x.eq) == [c.c for c in eq]
        assert rsio._read_block(x.linear) == [c.c for c in lin]
        assert rsio._read_block(x.nl_a) == [c.a for c in nl]
        assert rsio._read_block(x.nl_b) == [c.b for c in nl]
        assert rsio._read_block(x.nl_c) == [c.c for c in nl]
        forb = np.ctypeslib.as_array(x.forbidden, shape=(x.n_forbidden,)).tolist()
        assert forb == sorted(sys_.forbidden)
        assert (x.max_signal, x.n_pub_out, x.n_pub_in, x.n_priv_in) == (
            sys_.max_signal, sys_.n_pub_out, sys_.n_pub_in, sys_.n_priv_in)


@pytest.mark.parametrize("level", ["O1", "O2"])
def test_writers_match_oracle_bytes(level):
    """rs_write_r1cs / rs_write_sym (product) on the oracle's simplification result == the oracle's
    own byte writer (r1cs_porting.rs:4-124, sym_porting.rs:5-37), for the docs circuit."""
    with tempfile.TemporaryDirectory() as tmp:
        inp = M.Input.read_r1cs(os.path.join(GOLD, "docs_basic_O0.r1cs"))
        lib = rsio.oracle_lib()
        out = C.POINTER(abi.RsOutput)()
        ms, rounds = C.c_double(), C.c_uint64()
        assert lib.refcpu_simplify(C.byref(inp.c), C.byref(rsio.flags(level)), 1, C.byref(out),
                                   C.byref(ms), C.byref(rounds)) == 0
        try:
            r1 = os.path.join(tmp, "o.r1cs")
            sy = os.path.join(tmp, "o.sym")
            abi.check(abi.lib().rs_write_r1cs(r1.encode(), C.byref(inp.c), out))
            abi.check(abi.lib().rs_write_sym(os.path.join(GOLD, "docs_basic_O0.sym").encode(), sy.encode(), out))
        finally:
            lib.refcpu_output_free(out)
        assert open(r1, "rb").read() == open(os.path.join(GOLD, f"docs_basic_{level}.r1cs"), "rb").read()
        assert open(sy).read() == open(os.path.join(GOLD, f"docs_basic_{level}.sym")).read()


def test_writer_key_order_random():
    """LE-byte key order of the r1cs writer (r1cs_writer.rs:49-72) on rows with many signals > 255."""
    sys_ = rsio.gen_system(41, R.PRIMES["bls12381"], n_sig=700, n_rows=300, density=3.0)
    h = rsio.InputHolder(sys_, "bls12381")
    (cons, sm, nw, npiw), _, _ = rsio.oracle_run(h.inp, rsio.flags("O2"), 2)
    res = R.Result(cons, sm, npiw)
    lib = rsio.oracle_lib()
    out = C.POINTER(abi.RsOutput)()
    ms, rounds = C.c_double(), C.c_uint64()
    assert lib.refcpu_simplify(C.byref(h.inp), C.byref(rsio.flags("O2")), 1, C.byref(out), C.byref(ms),
                               C.byref(rounds)) == 0
    with tempfile.TemporaryDirectory() as tmp:
        r1 = os.path.join(tmp, "o.r1cs")
        try:
            abi.check(abi.lib().rs_write_r1cs(r1.encode(), C.byref(h.inp), out))
        finally:
            lib.refcpu_output_free(out)
        assert open(r1, "rb").read() == R.result_to_r1cs(sys_, res)


def _gate_system(seed=57):
    """A random system with one custom gate (section 4) applied twice (section 5) over signals that
    occur in its rows: map_tree makes them forbidden (dag/src/map_to_constraint_list.rs:22-24)."""
    sys_ = rsio.gen_system(seed, R.PRIMES["bn128"], n_sig=80, n_rows=150)
    used = struct.pack("<I", 1) + b"CMul\x00" + struct.pack("<I", 1) + (7).to_bytes(32, "little")
    apps = [(0, [10, 11, 12]), (0, [40, 41, 12])]
    gsig = {x for _, sig in apps for x in sig}
    return dataclasses.replace(sys_, forbidden=sys_.forbidden | gsig, gates=(used, apps))


def test_custom_gate_sections_forbidden_and_rewritten():
    """Sections 4/5 of an --O0 file: the reader adds the applied signals to `forbidden`; the writer
    re-emits section 4 and section 5 mapped label -> wire (r1cs_porting.rs:54-121), byte for byte
    what pyref's restatement writes for its own simplification of the same system."""
    sys_ = _gate_system()
    ident = R.Result(sys_.rows, {i: i for i in range(sys_.max_signal)}, sys_.n_priv_in)
    with tempfile.TemporaryDirectory() as tmp:
        o0 = _write(tmp, "in.r1cs", R.result_to_r1cs(sys_, ident))
        back, _ = R.read_r1cs_bytes(open(o0, "rb").read())
        assert back.forbidden == sys_.forbidden and back.gates == sys_.gates
        inp = M.Input.read_r1cs(o0)
        forb = np.ctypeslib.as_array(inp.c.forbidden, shape=(inp.c.n_forbidden,)).tolist()
        assert forb == sorted(sys_.forbidden)
        for level in ("O1", "O2"):
            fl = rsio.flags(level)
            want = R.simplification(sys_, rsio.py_flags(fl))
            lib = rsio.oracle_lib()
            out = C.POINTER(abi.RsOutput)()
            ms, rounds = C.c_double(), C.c_uint64()
            assert lib.refcpu_simplify(C.byref(inp.c), C.byref(fl), 1, C.byref(out), C.byref(ms), C.byref(rounds)) == 0
            r1 = os.path.join(tmp, f"{level}.r1cs")
            try:
                abi.check(abi.lib().rs_write_r1cs_gates(r1.encode(), C.byref(inp.c), out, o0.encode()))
            finally:
                lib.refcpu_output_free(out)
            got = open(r1, "rb").read()
            assert got == R.result_to_r1cs(sys_, want)
            assert got[8] == 5


def test_reader_rejects_truncated_and_malformed_files():
    """A truncated or malformed .r1cs is RS_E_INVALID, never an over-read (every read is checked
    against its section and the file)."""
    sys_ = _gate_system(58)
    ident = R.Result(sys_.rows, {i: i for i in range(sys_.max_signal)}, sys_.n_priv_in)
    data = R.result_to_r1cs(sys_, ident)
    with tempfile.TemporaryDirectory() as tmp:
        cuts = sorted(set([0, 4, 11, 12, 20, 23, 40, 100, len(data) // 3, len(data) // 2, len(data) - 9,
                           len(data) - 1]))
        for n in cuts:
            path = _write(tmp, "t.r1cs", data[:n])
            with pytest.raises(abi.RsError) as e:
                M.Input.read_r1cs(path)
            assert e.value.code == -1, n
        # a section size beyond the file
        bad = bytearray(data)
        struct.pack_into("<Q", bad, 16, len(data) * 2)
        with pytest.raises(abi.RsError):
            M.Input.read_r1cs(_write(tmp, "s.r1cs", bytes(bad)))
        # a constraint entry count beyond its section
        bad = bytearray(data)
        struct.pack_into("<I", bad, 24, 0x7fffffff)
        with pytest.raises(abi.RsError):
            M.Input.read_r1cs(_write(tmp, "c.r1cs", bytes(bad)))
        # a signal id >= n_labels
        bad = bytearray(data)
        struct.pack_into("<I", bad, 28, 0xfffffff0)
        with pytest.raises(abi.RsError):
            M.Input.read_r1cs(_write(tmp, "k.r1cs", bytes(bad)))
        assert M.Input.read_r1cs(_write(tmp, "ok.r1cs", data)).c.max_signal == sys_.max_signal


def test_cli_usage():
    exe = os.path.join(ROOT, "circom_cvm_amd", "circom-simplify")
    assert os.path.exists(exe)
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 2 and "usage" in r.stderr


# ---- --json / --simplification_substitution writers against the reference docs' exact texts
_M1 = str(R.PRIMES["bn128"] - 1)
DOCS_JSON_TEXT = {  # constraints-json.md:55-60 (--O1) and :93-97 (--O2), typed in as data
    "O1": '{\n"constraints": [\n[{"2":"%s"},{"4":"1"},{"1":"%s"}],\n[{},{},{"0":"1","2":"2","3":"1","4":"%s"}]\n]\n}'
          % (_M1, _M1, _M1),
    "O2": '{\n"constraints": [\n[{"2":"%s"},{"0":"1","2":"2","3":"1"},{"1":"%s"}]\n]\n}' % (_M1, _M1),
}
DOCS_SUBS_TEXT = {  # simplification-json.md:48-51 (--O1) and :77-81 (--O2)
    "O1": '{\n"5" : {"2":"1"},\n"4" : {"1":"1"}\n}',
    "O2": '{\n"5" : {"2":"1"},\n"4" : {"1":"1"},\n"6" : {"0":"1","2":"2","3":"1"}\n}',
}


def _docs_result(level):
    import make_golden as G
    sys_ = G.docs_system()
    return sys_, R.simplification(sys_, G.flags_of(level), want_log=True)


@pytest.mark.parametrize("level", ["O1", "O2"])
def test_json_writers_docs_text(level):
    """rs_write_constraints_json / rs_write_substitution_json (product) on the oracle's result for the
    docs circuit reproduce the reference docs' file texts byte for byte; so does the Python restatement
    the GPU tests compare with."""
    import sys
    sys.path.insert(0, GOLD)
    sys_, res = _docs_result(level)
    log = rsio.pyref_log(res.log)
    assert rsio.constraints_json_text(res.constraints, res.signal_map) == DOCS_JSON_TEXT[level]
    assert rsio.substitutions_json_text(log) == DOCS_SUBS_TEXT[level]
    h = rsio.OutputHolder(res, sys_.max_signal, log)
    with tempfile.TemporaryDirectory() as tmp:
        cj, sj = os.path.join(tmp, "c.json"), os.path.join(tmp, "s.json")
        abi.check(abi.lib().rs_write_constraints_json(cj.encode(), C.byref(h.out)))
        abi.check(abi.lib().rs_write_substitution_json(sj.encode(), C.byref(h.out)))
        assert open(cj).read() == DOCS_JSON_TEXT[level]
        assert open(sj).read() == DOCS_SUBS_TEXT[level]


@pytest.mark.parametrize("seed,prime,level", [(61, "bls12381", "O2"), (62, "goldilocks", "O1"), (63, 257, "O2")])
def test_json_writers_random(seed, prime, level):
    """Decimal conversion (limb carries, zero values, multi-digit keys sorted as numbers) on random
    systems: product writers == the Python restatement of json_writer.rs."""
    p = prime if isinstance(prime, int) else R.PRIMES[prime]
    sys_ = rsio.gen_system(seed, p, n_sig=400, n_rows=300, big_cluster=380 if seed % 2 else 0)
    import sys
    sys.path.insert(0, GOLD)
    import make_golden as G
    res = R.simplification(sys_, G.flags_of(level), want_log=True)
    log = rsio.pyref_log(res.log)
    h = rsio.OutputHolder(res, sys_.max_signal, log)
    with tempfile.TemporaryDirectory() as tmp:
        cj, sj = os.path.join(tmp, "c.json"), os.path.join(tmp, "s.json")
        abi.check(abi.lib().rs_write_constraints_json(cj.encode(), C.byref(h.out)))
        abi.check(abi.lib().rs_write_substitution_json(sj.encode(), C.byref(h.out)))
        assert open(cj).read() == rsio.constraints_json_text(res.constraints, res.signal_map)
        assert open(sj).read() == rsio.substitutions_json_text(log)


def test_json_decimal_edges():
    """Values across limb boundaries (2^64 - 1, 2^64, 10^19 multiples, p - 1 of a 256-bit prime)."""
    p = R.PRIMES["secq256r1"]
    vals = [1, 9, 10, (1 << 64) - 1, 1 << 64, 10 ** 19, 10 ** 19 - 1, 10 ** 38, (1 << 192) + 7, p - 1]
    log = [(i + 1, {0: v, 3 * i + 1000: 0}) for i, v in enumerate(vals)]
    res = R.Result([], {0: 0}, 0)
    h = rsio.OutputHolder(res, 1, log)
    with tempfile.TemporaryDirectory() as tmp:
        sj = os.path.join(tmp, "s.json")
        abi.check(abi.lib().rs_write_substitution_json(sj.encode(), C.byref(h.out)))
        assert open(sj).read() == rsio.substitutions_json_text(log)
        cj = os.path.join(tmp, "c.json")
        abi.check(abi.lib().rs_write_constraints_json(cj.encode(), C.byref(h.out)))
        assert open(cj).read() == '{\n"constraints": [\n]\n}'


def _streamed_copy(o, rng):
    """ABI 8's streamed layout of CSR result `o` (rs_engine_simplify's form): each block's rows in a
    shuffled storage order with unused entries between runs, u32 lengths with RS_ROW_JUMP, jump tables.
    Returns (RsOutput, keepalive arrays)."""
    keep = []
    s = abi.RsOutput()
    s.n_constraints = o.n_constraints
    s.n_labels, s.label_to_wire, s.n_wires = o.n_labels, o.label_to_wire, o.n_wires
    s.no_private_inputs_witness = o.no_private_inputs_witness
    n = int(o.n_constraints)
    for q, nm in enumerate("abc"):
        lc = getattr(o, nm)
        ptr, col, val = abi.block_csr(lc)
        lens = np.diff(ptr.astype(np.int64))
        # storage: rows cut into runs (a random split), runs placed in a shuffled order with gaps
        cuts = sorted(set([0, n] + [int(x) for x in rng.choice(np.arange(1, max(n, 2)), size=min(n // 2, 6), replace=False)]))
        runs = [(cuts[i], cuts[i + 1]) for i in range(len(cuts) - 1) if cuts[i] < cuts[i + 1]]
        order = list(range(len(runs)))
        rng.shuffle(order)
        start = np.zeros(n, np.int64)
        pos = 0
        ncol, nval = [], []
        for ri in order:
            lo, hi = runs[ri]
            pos += int(rng.integers(0, 3))  # unused entries before the run
            ncol.append(np.full(pos - sum(len(x) for x in ncol), 0xdeadbeef, np.uint32))
            nval.append(np.full(4 * (pos - sum(len(x) for x in nval) // 4), 7, np.uint64))
            for r in range(lo, hi):
                start[r] = pos
                a, b = int(ptr[r]), int(ptr[r + 1])
                ncol.append(col[a:b])
                nval.append(val[4 * a:4 * b])
                pos += b - a
        c2 = np.concatenate(ncol) if ncol else np.zeros(0, np.uint32)
        v2 = np.concatenate(nval) if nval else np.zeros(0, np.uint64)
        c2 = np.ascontiguousarray(np.concatenate([c2, np.zeros(1, np.uint32)]))
        v2 = np.ascontiguousarray(np.concatenate([v2, np.zeros(4, np.uint64)]))
        ln = lens.astype(np.uint32)
        jumps = []
        for r in range(n):
            prev_end = start[r - 1] + lens[r - 1] if r else 0
            if start[r] != prev_end:
                ln[r] |= np.uint32(abi.ROW_JUMP)
                jumps.append(start[r])
        jt = np.ascontiguousarray(np.array(jumps + [0], np.uint64))
        keep += [c2, v2, ln, jt]
        L = abi.RsLc()
        L.n_rows, L.nnz = n, pos
        L.ptr = C.POINTER(C.c_uint64)()
        L.col = c2.ctypes.data_as(C.POINTER(C.c_uint32))
        L.val = v2.ctypes.data_as(C.POINTER(C.c_uint64))
        setattr(s, nm, L)
        setattr(s, nm + "_len", ln.ctypes.data_as(C.POINTER(C.c_uint32)))
        setattr(s, nm + "_jump", jt.ctypes.data_as(C.POINTER(C.c_uint64)))
        setattr(s, nm + "_njump", len(jumps))
    return s, keep


@pytest.mark.parametrize("seed", [3, 4])
def test_streamed_row_layout_readers_and_writers(seed):
    """ABI 8's streamed result layout (lengths + RS_ROW_JUMP + jump tables, include/rs_simplify.h
    rs_rows_next): the host .r1cs / constraints-json writers and abi.block_csr read it exactly as the
    CSR form of the same result."""
    rng = np.random.default_rng(seed)
    sys_ = rsio.gen_system(90 + seed, R.PRIMES["bn128"], n_sig=80, n_rows=120)
    h = rsio.InputHolder(sys_)
    lib = rsio.oracle_lib()
    out = C.POINTER(abi.RsOutput)()
    ms, rounds = C.c_double(), C.c_uint64()
    assert lib.refcpu_simplify(C.byref(h.inp), C.byref(rsio.flags("O2")), 1, C.byref(out), C.byref(ms), C.byref(rounds)) == 0
    try:
        o = out.contents
        st, keep = _streamed_copy(o, rng)
        assert any(getattr(st, nm + "_njump") for nm in "abc")
        for q in range(3):
            a = abi.block_csr(*o.block(q))
            b = abi.block_csr(*st.block(q))
            assert all(np.array_equal(x, y) for x, y in zip(a, b))
        with tempfile.TemporaryDirectory() as tmp:
            for name, fn in (("r1cs", lambda p, x: abi.lib().rs_write_r1cs(p, C.byref(h.inp), C.byref(x))),
                             ("json", lambda p, x: abi.lib().rs_write_constraints_json(p, C.byref(x)))):
                p1, p2 = os.path.join(tmp, "csr." + name), os.path.join(tmp, "st." + name)
                abi.check(fn(p1.encode(), o))
                abi.check(fn(p2.encode(), st))
                assert open(p1, "rb").read() == open(p2, "rb").read(), name
    finally:
        lib.refcpu_output_free(out)
