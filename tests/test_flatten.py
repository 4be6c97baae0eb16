"""the DAG -> constraint-list flattening (rs_flatten_dag) against its oracle,
oracle/pyref.py flatten_dag (a restatement of dag/src/map_to_constraint_list.rs:12-44 / :111-150
and the EncodingIterator DFS, constraint_list/src/lib.rs:65-108): the rs_input blocks, the forbidden
set and max_signal array for array, then the flattened input through the simplifier against pyref.
Parity unpinned beyond the oracle: the reference holds no DAG fixtures (its DAGs come from the
compiler front end)."""
import ctypes as C

import numpy as np
import pytest

import dagio
import rsio
import circom_cvm_amd as M

R = rsio.R


def blocks_of(inp):
    """rs_input -> (cons_eq, eq, linear, nl as Con lists, forbidden set, max_signal)."""
    rb = rsio._read_block
    ce, eq, lin = rb(inp.cons_eq), rb(inp.eq), rb(inp.linear)
    na, nb, nc = rb(inp.nl_a), rb(inp.nl_b), rb(inp.nl_c)
    forb = set(np.ctypeslib.as_array(inp.forbidden, shape=(max(inp.n_forbidden, 1),))[: inp.n_forbidden].tolist())
    nl = [R.Con(na[i], nb[i], nc[i]) for i in range(len(na))]
    return ([R.Con({}, {}, m) for m in ce], [R.Con({}, {}, m) for m in eq], [R.Con({}, {}, m) for m in lin], nl,
            forb, int(inp.max_signal))


def _eq_blocks(got, ref_blocks, sys_):
    ce, eq, lin, nl, forb, ms = got
    for name, g, r in (("cons_eq", ce, ref_blocks["cons_eq"]), ("eq", eq, ref_blocks["eq"]),
                       ("linear", lin, ref_blocks["linear"]), ("non_linear", nl, ref_blocks["non_linear"])):
        assert len(g) == len(r), (name, len(g), len(r))
        for i, (x, y) in enumerate(zip(g, r)):
            assert (x.a, x.b, x.c) == (y.a, y.b, y.c), (name, i, x, y)
    assert forb == sys_.forbidden
    assert ms == sys_.max_signal


# ---------------------------------------------------------------- CPU: the oracle
def test_oracle_known_answer():
    p = R.PRIMES["bn128"]
    leaf = R.DagNode([R.Con({}, {}, {1: 1, 0: 5}), R.Con({}, {}, {})], [1, 2])
    mid = R.DagNode([R.Con({1: 1}, {2: 1}, {3: 1})], [3], edges=[(0, 0)])
    main = R.DagNode([R.Con({}, {}, {1: 1, 2: p - 1}), R.Con({}, {}, {})], [1, 2], edges=[(1, 2), (0, 5)])
    sys_, b = R.flatten_dag(p, [leaf, mid, main], 2, 1, 0, 1, {0, 1})
    # DFS: main (offset 0), mid (offset 2) with its leaf (offset 2), leaf (offset 5); signals 1..7
    assert b["witness"] == [0, 1, 2, 5, 3, 4, 6, 7]
    assert sys_.max_signal == 8
    assert [c.c for c in b["eq"]] == [{1: 1, 2: p - 1}]
    assert [c.c for c in b["linear"]] == [{}]                      # main keeps its empty constraint
    assert [c.c for c in b["cons_eq"]] == [{3: 1, 0: 5}, {6: 1, 0: 5}]  # the leaves' ones are dropped
    assert [(c.a, c.b, c.c) for c in b["non_linear"]] == [({3: 1}, {4: 1}, {5: 1})]


@pytest.mark.parametrize("seed", range(6))
def test_oracle_blocks_are_map_tree_classes(seed):
    p = R.PRIMES["bn128"]
    nodes, main, no, npb, npr, forb = dagio.gen_dag(seed, p)
    sys_, b = R.flatten_dag(p, nodes, main, no, npb, npr, forb)
    ce, eq, lin, nl = R.classify(sys_)
    assert (ce, eq, lin, nl) == (b["cons_eq"], b["eq"], b["linear"], b["non_linear"])
    assert sorted(b["witness"]) == list(range(sys_.max_signal))  # the numbering is a permutation


def test_dag_builder_arrays():
    p = R.PRIMES["bn128"]
    nodes, main, no, npb, npr, forb = dagio.gen_dag(3, p)
    d = M.Dag(p, nodes, main, no, npb, npr, forb, "bn128")
    assert d.c.n_nodes == len(nodes) and d.c.main_node == main
    assert int(d.cons_off[-1]) == sum(len(n.constraints) for n in nodes) == d.c.c.n_rows
    assert int(d.edge_off[-1]) == sum(len(n.edges) for n in nodes)


# ---------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("prime", ["bn128", "bls12381", "goldilocks"])
def test_flatten_parity_random(prime):
    p = R.PRIMES[prime]
    for seed in range(12):
        nodes, main, no, npb, npr, forb = dagio.gen_dag(seed, p, n_templates=4 + seed % 5, empties=seed % 2 == 1,
                                                        custom_gates=seed % 3 == 0)
        sys_, b = R.flatten_dag(p, nodes, main, no, npb, npr, forb)
        inp = M.Dag(p, nodes, main, no, npb, npr, forb, prime).flatten(0)
        _eq_blocks(blocks_of(inp.c), b, sys_)


@pytest.mark.gpu
def test_flatten_then_simplify():
    p = R.PRIMES["bn128"]
    eng = M.Engine(0)
    for seed in range(8):
        nodes, main, no, npb, npr, forb = dagio.gen_dag(100 + seed, p, n_templates=6)
        sys_, _ = R.flatten_dag(p, nodes, main, no, npb, npr, forb)
        inp = M.Dag(p, nodes, main, no, npb, npr, forb, "bn128").flatten(0)
        for lvl in ("O1", "O2"):
            eng.load(inp.c)
            eng.run(rsio.flags(lvl))
            out = eng.fetch()  # keep the Output alive while its arrays are read
            got = rsio.output_to_py(out.c)
            ref = R.simplification(sys_, rsio.py_flags(rsio.flags(lvl)))
            assert rsio.same_result(ref, got) is None, (seed, lvl)
    eng.close()


@pytest.mark.gpu
def test_flatten_wide_and_deep():
    """A DAG whose instances number in the tens of thousands (shared subtrees expanded many times)."""
    p = R.PRIMES["bn128"]
    nodes, main, no, npb, npr, forb = dagio.gen_dag(7, p, n_templates=16, max_children=6, cons_per_template=(6, 20))
    sys_, b = R.flatten_dag(p, nodes, main, no, npb, npr, forb)
    assert len(sys_.rows) > 30000
    inp = M.Dag(p, nodes, main, no, npb, npr, forb, "bn128").flatten(0)
    _eq_blocks(blocks_of(inp.c), b, sys_)


@pytest.mark.gpu
def test_flatten_rejects_cycle_and_bad_edge():
    p = R.PRIMES["bn128"]
    a = R.DagNode([R.Con({}, {}, {1: 1})], [1], edges=[(1, 1)])
    b = R.DagNode([R.Con({}, {}, {1: 1})], [1], edges=[(0, 1)])
    with pytest.raises(M.RsError):
        M.Dag(p, [a, b], 0, 0, 0, 0, {0}, "bn128").flatten(0)
    c = R.DagNode([R.Con({}, {}, {1: 1})], [1], edges=[(7, 1)])
    with pytest.raises(M.RsError):
        M.Dag(p, [c], 0, 0, 0, 0, {0}, "bn128").flatten(0)
