"""GPU parity: librs_simplify (HIP, gfx950) vs the canonical CPU oracle, bit for bit.

Small seeded systems exercise every branch (eq clusters, constant equalities, process_3 and
process_4 clusters, rounds >= 2, --O2round truncation, old heuristics, 5 primes); synthetic
workloads check the same at scale, and size-independent properties at the full sizes."""
import pytest

import rsio
import circom_cvm_amd as M

R = rsio.R
pytestmark = pytest.mark.gpu

_ENG = None


def engine():
    global _ENG
    if _ENG is None:
        _ENG = M.Engine(0)
    return _ENG


def gpu_run(inp, fl):
    e = engine()
    e.load(inp)
    e.run(fl)
    out = e.fetch()
    return rsio.output_to_py(out.c), e.stats()


def check(inp, fl, threads=1):
    got, st = gpu_run(inp, fl)
    ref, _, _ = rsio.oracle_run(inp, fl, threads)
    if got != ref:
        diff = rsio.same_result(R.Result(ref[0], ref[1], ref[3]), got)
        raise AssertionError(f"GPU != oracle: {diff}")
    return st


def test_docs_example():
    p = R.PRIMES["bn128"]
    m = p - 1
    rows = [R.Con({}, {}, {2: 1, 5: m}), R.Con({}, {}, {0: 1, 2: 2, 3: 1, 6: m}),
            R.Con({}, {}, {1: m, 4: 1}), R.Con({5: m}, {6: 1}, {4: m})]
    sys_ = R.System(p, 7, 1, 0, 2, {0, 1}, rows)
    h = rsio.InputHolder(sys_, "bn128")
    for lvl in ("O1", "O2"):
        got, _ = gpu_run(h.inp, rsio.flags(lvl))
        ref = R.simplification(sys_, R.Flags(flag_s=lvl == "O1", no_rounds=0 if lvl == "O1" else (1 << 64) - 1))
        assert rsio.same_result(ref, got) is None


@pytest.mark.parametrize("p", [257, 97, R.PRIMES["bn128"], R.PRIMES["secq256r1"], R.PRIMES["goldilocks"]])
def test_random_small(p):
    for seed in range(40):
        sys_ = rsio.gen_system(seed, p, n_sig=40 + seed % 50, n_rows=60 + seed % 80)
        h = rsio.InputHolder(sys_)
        for lvl, rd in (("O1", None), ("O2", None), ("O2", 1), ("O2", 2)):
            check(h.inp, rsio.flags(lvl, rd))


@pytest.mark.parametrize("p", [257, R.PRIMES["bn128"]])
def test_random_forbidden_intermediates(p):
    """Forbidden signals beyond the public ones (circom's custom-gate signals): equality clusters whose
    forbidden members sit several union-find links below the root (eq_cluster_simplification
    :158-187 keeps one `f - rh` row per forbidden member), forbidden-only linear rows and constant
    equalities on forbidden signals."""
    m = p - 1
    # the chain (5, 6), (2, 5) links 6 under 5 under 2: 6 is met only as a second key
    rows = [R.Con({}, {}, {5: 3, 6: p - 3}), R.Con({}, {}, {2: 1, 5: m}), R.Con({}, {}, {3: 1, 4: m, 6: 2}),
            R.Con({3: 1}, {4: 1}, {1: 1})]
    sys_ = R.System(p, 7, 1, 1, 1, {0, 1, 2, 5, 6}, rows)
    h = rsio.InputHolder(sys_)
    for lvl in ("O1", "O2"):
        check(h.inp, rsio.flags(lvl))
    for seed in range(30):
        sys_ = rsio.gen_system(5000 + seed, p, n_sig=30 + seed % 40, n_rows=50 + seed % 60, extra_forb=0.1 + 0.02 * (seed % 10))
        h = rsio.InputHolder(sys_)
        for lvl, rd in (("O1", None), ("O2", None), ("O2", 1)):
            check(h.inp, rsio.flags(lvl, rd))


@pytest.mark.parametrize("p", [257, R.PRIMES["bn128"], R.PRIMES["bls12381"]])
def test_random_process4(p):
    for seed in range(6):
        sys_ = rsio.gen_system(2000 + seed, p, n_sig=300, n_rows=250, big_cluster=600 + 40 * seed)
        h = rsio.InputHolder(sys_)
        for lvl, rd, old in (("O2", None, False), ("O2", None, True), ("O2", 2, False)):
            check(h.inp, rsio.flags(lvl, rd, old), threads=4)


@pytest.mark.parametrize("kind,rows", [(0, 20000), (0, 200000), (1, 20000), (2, 50000)])
def test_synth_vs_oracle(kind, rows):
    inp = M.Input.synth(kind, rows, 42)
    st = check(inp.c, rsio.flags("O2"), threads=8)
    assert st.total_ms > 0
