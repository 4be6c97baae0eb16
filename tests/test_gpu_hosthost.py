"""rs_engine_simplify: the host -> host entry point the benchmark times (SURVEY 8(d) T_simplify).
Pipelined H2D + device validation + simplification + D2H into pinned buffers, compared array for
array with the oracle; malformed inputs are rejected with RS_E_INVALID and leave the engine usable."""
import numpy as np
import pytest

import rsio
import circom_cvm_amd as M

pytestmark = pytest.mark.gpu
R = rsio.R
_ENG = None


def engine():
    global _ENG
    if _ENG is None:
        _ENG = M.Engine(0)
    return _ENG


@pytest.fixture(scope="module", autouse=True)
def _release_engine():
    """The module's engine goes when its tests are done (later modules -- the 20 M sharded child --
    need the device memory)."""
    yield
    global _ENG
    if _ENG is not None:
        _ENG.close()
        _ENG = None


@pytest.mark.parametrize("seed,prime", [(1, "bn128"), (2, "bls12381"), (3, "goldilocks"), (4, "secq256r1")])
def test_hosthost_random_systems(seed, prime):
    p = R.PRIMES[prime]
    for k in range(6):
        sys_ = rsio.gen_system(100 * seed + k, p, n_sig=120, n_rows=200, big_cluster=400 if k % 2 else 0)
        h = rsio.InputHolder(sys_, prime)
        for fl in (rsio.flags("O2"), rsio.flags("O1"), rsio.flags("O2", rounds=1)):
            got = rsio.output_arrays(engine().simplify(h.inp, fl))  # pageable input: HIP stages it
            ref, _ = rsio.oracle_arrays(h.inp, fl)
            assert rsio.diff_output_arrays(got, ref) is None


@pytest.mark.parametrize("kind,rows,prime", [(0, 1_000_000, "bn128"), (1, 300_000, "bn128"), (2, 200_000, "bls12381")])
def test_hosthost_pinned_synth(kind, rows, prime):
    inp = M.Input.synth(kind, rows, 11, prime)
    pin = M.PinnedInput(inp.c)
    fl = rsio.flags("O2")
    got = rsio.output_arrays(engine().simplify(pin.c, fl))
    st = engine().stats()
    assert st.host_total_ms >= st.total_ms > 0
    assert st.alg_bytes > 0
    ref, _ = rsio.oracle_arrays(inp.c, fl, threads=16)
    assert rsio.diff_output_arrays(got, ref) is None
    # the HBM-resident path on the same engine agrees
    e = engine()
    e.load(pin.c)
    e.run(fl)
    out = e.fetch()
    assert rsio.diff_output_arrays(rsio.output_arrays(out.c), ref) is None
    pin.free()


def _small():
    p = R.PRIMES["bn128"]
    return rsio.gen_system(7, p, n_sig=80, n_rows=150)


def _expect_invalid(h):
    with pytest.raises(M.RsError) as ei:
        engine().simplify(h.inp, rsio.flags("O2"))
    assert ei.value.code == -1
    # the engine recovers: a good input right after
    g = rsio.InputHolder(_small(), "bn128")
    got = rsio.output_arrays(engine().simplify(g.inp, rsio.flags("O2")))
    ref, _ = rsio.oracle_arrays(g.inp, rsio.flags("O2"))
    assert rsio.diff_output_arrays(got, ref) is None


@pytest.mark.parametrize("blk", [0, 2, 3])
def test_hosthost_rejects_bad_row_pointers(blk):
    h = rsio.InputHolder(_small(), "bn128")
    b = h.blocks[blk]
    assert len(b.ptr) > 3
    b.ptr[1], b.ptr[2] = b.ptr[2] + 5, b.ptr[1]  # decreasing: a wrapped row length without the check
    _expect_invalid(h)


def test_hosthost_rejects_ptr_nnz_mismatch():
    h = rsio.InputHolder(_small(), "bn128")
    h.blocks[2].ptr[-1] += 1  # ptr[n] != nnz
    _expect_invalid(h)


def test_hosthost_rejects_signal_out_of_range():
    h = rsio.InputHolder(_small(), "bn128")
    h.blocks[3].col[0] = h.inp.max_signal + 7
    _expect_invalid(h)


def test_hosthost_rejects_duplicate_key():
    h = rsio.InputHolder(_small(), "bn128")
    b = h.blocks[2]
    r = int(np.argmax(np.diff(b.ptr.astype(np.int64)) >= 2))
    b.col[b.ptr[r] + 1] = b.col[b.ptr[r]]
    _expect_invalid(h)


def test_hosthost_unsorted_long_rows():
    """Rows arrive in any key order (the shim marshals HashMaps): long rows take the heap-sort path."""
    p = R.PRIMES["bn128"]
    rows = []
    for i in range(40):
        rows.append(R.Con({}, {}, {1 + ((7 * j + i) % 300): 1 + j for j in range(60)}))
    sys_ = R.System(p, 301, 1, 2, 2, {0, 1, 2, 3}, rows)
    h = rsio.InputHolder(sys_, "bn128")
    ref, _ = rsio.oracle_arrays(h.inp, rsio.flags("O2"))
    b = h.blocks[2]
    rng = np.random.default_rng(3)
    for r in range(len(b.ptr) - 1):
        s, e = int(b.ptr[r]), int(b.ptr[r + 1])
        perm = rng.permutation(e - s)
        b.col[s:e] = b.col[s:e][perm]
        v = b.val.reshape(-1, 4)
        v[s:e] = v[s:e][perm]
    got = rsio.output_arrays(engine().simplify(h.inp, rsio.flags("O2")))
    assert rsio.diff_output_arrays(got, ref) is None


@pytest.mark.parametrize("kind,rows,prime", [(0, 400_000, "bn128"), (2, 200_000, "bls12381"), (5, 300_000, "bn128")])
def test_hosthost_streamed_layout(kind, rows, prime):
    """rs_engine_simplify streams the storage rows final after round 1 while later rounds run (ABI 7
    row ends): every row lies inside col / val, the compacted rows equal the oracle's, the rows a
    round >= 3 reaches after all (chain: 8 rounds) are taken from the late region, and
    rs_engine_fetch of the same result is the compact CSR."""
    inp = M.Input.synth(kind, rows, 5, prime)
    pin = M.PinnedInput(inp.c)
    fl = rsio.flags("O2")
    ref, _ = rsio.oracle_arrays(inp.c, fl, threads=16)
    # three calls: the first sizes the early regions, the later ones take every snapshot (the head rows'
    # pass, each round's rewritten rows, the lconst rows) into them
    for _ in range(3):
        o = engine().simplify(pin.c, fl)
        got = rsio.output_arrays(o)
        n = int(o.n_constraints)
        for q in range(3):
            lc, lay = o.block(q)
            assert lay is not None and not lc.ptr, "a run with storage rows streams (ABI 8 layout)"
            lens = np.ctypeslib.as_array(lay[0], shape=(n,))
            jumps = np.ctypeslib.as_array(lay[1], shape=(lay[2],)) if lay[2] else np.zeros(0, np.uint64)
            b = M.abi.row_starts(lens, jumps)
            e = b + (lens & ~np.uint32(M.abi.ROW_JUMP)).astype(np.int64)
            assert (e <= int(lc.nnz)).all() and lay[2] <= n
        assert rsio.diff_output_arrays(got, ref) is None
    out = engine().fetch()
    assert not out.c.a_len and not out.c.b_len and not out.c.c_len and out.c.a.ptr
    assert rsio.diff_output_arrays(rsio.output_arrays(out.c), ref) is None
    pin.free()


@pytest.mark.parametrize("kind,rows,frac", [(0, 400_000, "0.5"), (5, 300_000, "0.2"), (2, 200_000, "0.9")])
def test_hosthost_first_pass_halves(kind, rows, frac, monkeypatch):
    """The first frames pass in two parts with a snapshot after each (engine.hip nl_phase / snap_take_h2;
    by default only from 1 M non-linear rows on): forced here on smaller circuits and at other split
    points, the streamed result equals the oracle's on every call, and the off switch gives the same."""
    inp = M.Input.synth(kind, rows, 11, "bn128")
    pin = M.PinnedInput(inp.c)
    fl = rsio.flags("O2")
    ref, _ = rsio.oracle_arrays(inp.c, fl, threads=16)
    monkeypatch.setenv("RS_HALVES_MIN", "2")
    monkeypatch.setenv("RS_HALF_FRAC", frac)
    for _ in range(3):  # the first call sizes the regions from its first part; later ones reuse them
        assert rsio.diff_output_arrays(rsio.output_arrays(engine().simplify(pin.c, fl)), ref) is None
    monkeypatch.setenv("RS_NO_HALVES", "1")
    assert rsio.diff_output_arrays(rsio.output_arrays(engine().simplify(pin.c, fl)), ref) is None
    pin.free()


@pytest.mark.parametrize("level,rounds", [("O1", None), ("O2", 1), ("O2", 2)])
def test_hosthost_streamed_levels(level, rounds):
    """The streamed result at --O1 (every linear row joins lconst and goes with the first early region)
    and at --O2round 1 / 2 (truncated rounds leave the linear tail late), repeated on one engine."""
    inp = M.Input.synth(0, 500_000, 8, "bn128")
    pin = M.PinnedInput(inp.c)
    fl = rsio.flags(level, rounds)
    ref, _ = rsio.oracle_arrays(inp.c, fl, threads=16)
    for _ in range(3):
        got = rsio.output_arrays(engine().simplify(pin.c, fl))
        assert rsio.diff_output_arrays(got, ref) is None
    pin.free()


def test_engine_calls_keep_caller_affinity():
    """engine creation and calls run the calling thread on the GPU's NUMA-local CPUs only for
    the duration of a call (threads the call starts inherit that); the caller's own mask is unchanged
    after rs_engine_create and after every call, so a second engine (or a host thread pool created
    later) is not narrowed by the first."""
    import os
    before = os.sched_getaffinity(0)  # pid 0: the calling thread's mask
    e1, e2 = M.Engine(0), M.Engine(0)
    try:
        assert os.sched_getaffinity(0) == before
        inp = M.Input.synth(0, 50_000, 5, "bn128")
        fl = rsio.flags("O2")
        got = rsio.output_arrays(e1.simplify(inp.c, fl))
        assert os.sched_getaffinity(0) == before
        e2.load(inp.c)
        e2.run(fl)
        assert rsio.diff_output_arrays(got, rsio.output_arrays(e2.fetch().c)) is None
        assert os.sched_getaffinity(0) == before
        inp.free()
    finally:
        e1.close()
        e2.close()
    assert os.sched_getaffinity(0) == before
