"""GPU parity on the fallback paths the synthetic workloads rarely reach:
  * a process_4 cluster longer than the LDS arena replay (cluster.hpp kClLds = 32768 rows), whose
    rows are not consumed by the uniques phase (lane replay in global memory);
  * dense rows whose work lists outgrow k_big_main's LDS buffers (kBigCap = 512: lane-serial spill)
    and whose substitutions outgrow the wave composition (kComposeCap: serial composition);
  * process_3 clusters between the lane kernel and process_4 (32..349 rows) with long rows;
  * leftovers (rows with only forbidden signals) inside workgroup clusters."""
import random

import pytest

import rsio

R = rsio.R
pytestmark = pytest.mark.gpu
_ENG = None


def engine():
    global _ENG
    if _ENG is None:
        import circom_cvm_amd as M
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


def check(sys_, level="O2", rounds=None, old=False, threads=8):
    h = rsio.InputHolder(sys_)
    fl = rsio.flags(level, rounds, old)
    e = engine()
    e.load(h.inp)
    e.run(fl)
    out = e.fetch()  # keep the owner alive while the arrays are copied
    got = rsio.output_arrays(out.c)
    ref, _ = rsio.oracle_arrays(h.inp, fl, threads)
    assert rsio.diff_output_arrays(got, ref) is None


def _coef(rng, p):
    return rng.randrange(1, p)


def long_chain(seed, p, n, n_w=50, n_forb=3):
    """x_i - c_i x_{i+1} - d_i w_{i mod n_w} = 0: every x but the ends sits in two rows."""
    rng = random.Random(seed)
    forb = set(range(0, n_forb + 1))
    base = n_forb + 1
    x = lambda i: base + i
    w = lambda j: base + n + 1 + j
    rows = []
    for i in range(n):
        m = {x(i): 1, x(i + 1): _coef(rng, p), w(i % n_w): _coef(rng, p)}
        if rng.random() < 0.2:
            m[0] = _coef(rng, p)
        rows.append(R.Con({}, {}, m))
    # a few quadratic rows on the chain so substitutions reach the non-linear part
    for _ in range(200):
        a, b = rng.randrange(n + 1), rng.randrange(n + 1)
        rows.append(R.Con({x(a): 1}, {x(b): 1}, {w(rng.randrange(n_w)): 1}))
    S = base + n + 1 + n_w
    return R.System(p, S, 1, 2, 5, forb, rows)


def dense_cluster(seed, p, n_rows, n_sig, row_len, n_forb=4, forb_rows=3):
    rng = random.Random(seed)
    forb = set(range(0, n_forb + 1))
    pool = list(range(n_forb + 1, n_forb + 1 + n_sig))
    rows = []
    for _ in range(n_rows):
        keys = rng.sample(pool, row_len)
        m = {k: _coef(rng, p) for k in keys}
        if rng.random() < 0.3:
            m[0] = _coef(rng, p)
        rows.append(R.Con({}, {}, m))
    for _ in range(forb_rows):  # rows of forbidden signals only: leftovers of the cluster
        rows.append(R.Con({}, {}, {1: 1, 2: _coef(rng, p), pool[0]: 1}))
        rows.append(R.Con({}, {}, {1: _coef(rng, p), 3: 1}))
    for _ in range(40):
        a, b, c = rng.sample(pool, 3)
        rows.append(R.Con({a: 1}, {b: _coef(rng, p)}, {c: 1}))
    return R.System(p, n_forb + 1 + n_sig, 1, 3, 5, forb, rows)


def wide_chain(seed, p, n=600, wide=3, width=530):
    """A process_4 chain plus a few rows holding `width` chain signals each: those rows exceed the
    LDS work buffers (row-level lane fallback), and their substitutions exceed the wave
    composition (serial composition)."""
    s = long_chain(seed, p, n)
    rng = random.Random(seed + 1)
    base = 4
    for _ in range(wide):
        m = {base + i: _coef(rng, p) for i in rng.sample(range(n + 1), width)}
        m[0] = _coef(rng, p)
        s.rows.append(R.Con({}, {}, m))
    return s


def test_cluster_beyond_lds_replay():
    check(long_chain(1, R.PRIMES["bn128"], 40000))


def test_cluster_beyond_lds_replay_old_heuristics():
    check(long_chain(2, R.PRIMES["goldilocks"], 36000), old=True)


@pytest.mark.parametrize("n_rows,n_sig,row_len", [(100, 300, 70), (60, 200, 150)])
def test_dense_process3_long_lists(n_rows, n_sig, row_len):
    check(dense_cluster(n_rows + row_len, R.PRIMES["bn128"], n_rows, n_sig, row_len))


@pytest.mark.parametrize("seed", [1, 2])
def test_wide_rows_process4(seed):
    check(wide_chain(seed, R.PRIMES["bn128"]))
    check(wide_chain(seed, R.PRIMES["bn128"]), old=True)


def test_dense_rows_rounds():
    for lvl, rd in (("O1", None), ("O2", 1), ("O2", 2)):
        check(dense_cluster(7, R.PRIMES["bls12381"], 90, 250, 60), lvl, rd)
