"""GPU parity of the giant path (circom_cvm_amd/csrc/giant_loop.hpp): head clusters of kGiantRows
(11,800) rows or more run as independent takeable components, one workgroup each, with 256-lane
merges.  The split is exact because forbidden signals -- which glue the components into one
cluster in build_clusters (constraint_simplification.rs:45-99) -- are never taken, counted or
deleted by the loop (simplification_utils.rs:60-113, 312-411); every case here is compared with the
CPU oracle (whole-cluster loop) array for array or map for map.

Covered: several chains glued by public inputs (process_4 and, with the old heuristics,
process_3), rows that reduce to forbidden keys only (leftovers: unnormalised, so their scale is the
reference's merge sequence's) and to nothing, rows too long for the LDS lists (the lane-serial
continuation), non-linear rows over the chains (the substitutions reach the output), rounds >= 2,
and BASELINE configs[1]'s generator at reduced size."""
import random

import pytest

import rsio
import circom_cvm_amd as M

R = rsio.R
pytestmark = pytest.mark.gpu

_ENG = {}


def engine():
    if "e" not in _ENG:
        _ENG["e"] = M.Engine(0)
    return _ENG["e"]


@pytest.fixture(scope="module", autouse=True)
def _release():
    yield
    for e in _ENG.values():
        e.close()
    _ENG.clear()


def giant_system(seed, p, n_chains=6, chain_len=2400, n_pub=3, window=24, long_rows=0, n_quad=400):
    """n_chains chains over disjoint signal ranges, glued into ONE linear cluster by public inputs
    (forbidden): one takeable component per chain.  Some rows are copies of an earlier row of the
    chain plus a public-input term (the later-popped copy reduces to forbidden keys only: a
    leftover), some exact multiples of one (reduce to nothing), some long (past the LDS lists)."""
    rng = random.Random(seed)
    n_out = 1
    forb = {0} | set(range(1, n_out + n_pub + 1))
    nxt = n_out + n_pub + 1

    def coef():
        r = rng.random()
        if r < 0.3:
            return 1
        if r < 0.5:
            return p - 1
        if r < 0.65:
            return pow(2, rng.randrange(1, 200), p)
        return rng.randrange(1, p)

    rows, chains = [], []
    for _ in range(n_chains):
        base = nxt
        nxt += chain_len + window + 2
        chains.append(base)
        made = []
        for i in range(chain_len):
            m = {}
            for _ in range(rng.randint(2, 4)):
                m[base + i + rng.randrange(0, window)] = coef()
            if rng.random() < 0.08:
                m[rng.randrange(1, n_out + n_pub + 1)] = coef()
            if rng.random() < 0.3:
                m[0] = coef()
            m = {k: v % p for k, v in m.items() if v % p}
            if len([k for k in m if k]) < 2:
                continue
            rows.append(m)
            made.append(m)
            r = rng.random()
            if r < 0.03 and made:  # an earlier row + a public input: one of the pair becomes a leftover
                src = rng.choice(made)
                cp = dict(src)
                pub = rng.randrange(1, n_out + n_pub + 1)
                cp[pub] = (cp.get(pub, 0) + coef()) % p
                cp = {k: v for k, v in cp.items() if v}
                rows.append(cp)
            elif r < 0.045 and made:  # a multiple of an earlier row: reduces to nothing
                src = rng.choice(made)
                k = coef()
                rows.append({kk: v * k % p for kk, v in src.items()})
        for _ in range(long_rows):  # past the 256-entry LDS lists
            m = {base + j: coef() for j in rng.sample(range(chain_len + window), 300)}
            rows.append(m)
    for _ in range(n_pub * 4):  # public inputs only: immediate leftovers
        rows.append({rng.randrange(1, n_out + n_pub + 1): coef(), 0: coef()})
    cons = [R.Con({}, {}, m) for m in rows]
    for _ in range(n_quad):  # non-linear rows over the chains
        base = rng.choice(chains)
        a = {base + rng.randrange(0, chain_len): coef()}
        b = {base + rng.randrange(0, chain_len): coef(), 0: coef()}
        c = {nxt: 1}
        nxt += 1
        cons.append(R.Con(a, b, c))
    return R.System(p, nxt + 1, n_out, n_pub, 2, forb, cons)


def check(sys_, fl):
    h = rsio.InputHolder(sys_)
    ref, _, _ = rsio.oracle_run(h.inp, fl, 8)
    e = engine()
    e.load(h.inp)
    e.run(fl)
    out = e.fetch()  # keep the owner alive while its struct is read
    got = rsio.output_to_py(out.c)
    if got != ref:
        raise AssertionError(str(rsio.same_result(R.Result(ref[0], ref[1], ref[3]), got)))
    return e.stats()


@pytest.mark.parametrize("p", [R.PRIMES["bn128"], 257, R.PRIMES["goldilocks"]])
def test_giant_chains_process4(p):
    for seed in range(3):
        st = check(giant_system(100 + seed, p), rsio.flags("O2"))
        assert st.max_cluster >= 11800


def test_giant_chains_process3_old_heuristics():
    p = R.PRIMES["bn128"]
    for seed in range(2):
        check(giant_system(200 + seed, p), rsio.flags("O2", old=True))


def test_giant_long_rows_and_rounds():
    """Rows past the LDS lists finish on one lane; --O2round 1 and full rounds."""
    p = R.PRIMES["bn128"]
    sys_ = giant_system(300, p, n_chains=5, chain_len=2600, long_rows=3)
    for fl in (rsio.flags("O2"), rsio.flags("O2", 1), rsio.flags("O1")):
        check(sys_, fl)


@pytest.mark.parametrize("rows,seed", [(150_000, 1), (300_000, 7)])
def test_giant_synth_linear(rows, seed):
    """BASELINE configs[1]'s generator (synth_linear) at reduced size: one cluster of ~0.55 of the
    rows, glued by public inputs, array for array."""
    inp = M.Input.synth(1, rows, seed)
    fl = rsio.flags("O2")
    ref, _ = rsio.oracle_arrays(inp.c, fl, threads=16)
    e = engine()
    e.load(inp.c)
    e.run(fl)
    out = e.fetch()
    got = rsio.output_arrays(out.c)
    assert rsio.diff_output_arrays(got, ref) is None
    assert e.stats().max_cluster >= 11800
