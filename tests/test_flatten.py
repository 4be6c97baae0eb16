"""the DAG -> constraint-list flattening (rs_flatten_dag) against its oracle,
oracle/pyref.py flatten_dag (a restatement of dag/src/map_to_constraint_list.rs:12-44 / :111-150
and the EncodingIterator DFS, constraint_list/src/lib.rs:65-108): the rs_input blocks, the forbidden
set and max_signal array for array, then the flattened input through the simplifier against pyref.
Pinned to reference data by the docs' basic.circom (Main + one Internal multiplier): flattening its
two-node DAG must give the --O0 constraint list of mkdocs/docs/circom-language/formats/
constraints-json.md:77-81 and the --O0 witness / component columns of formats/sym.md:65-70, and the
flattened input simplified must give the O1 / O2 texts (constraints-json.md:57-59, 95-96; sym.md:46-51,
81-86).  Random DAGs beyond that are checked against pyref alone."""
import ctypes as C
import os
import sys

import numpy as np
import pytest

import dagio
import rsio
import circom_cvm_amd as M

R = rsio.R
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import make_golden as G  # noqa: E402


def docs_basic_dag():
    """basic.circom / symbols.circom of the docs as the DAG constraint_generation builds: node 0 =
    Internal (locals out=1, in[0]=2, in[1]=3; `out <== in[0]*in[1]` with C negated,
    algebra.rs:113-145), node 1 = Main (locals out=1, in[0]=2, in[1]=3; its component c at
    in_number 3, so c's signals are 4..6; the three `<==` of Main).  Node ids are the sym.md #c
    column: main.* -> 1, main.c.* -> 0."""
    p = R.PRIMES["bn128"]
    m = p - 1
    internal = R.DagNode([R.Con({2: m}, {3: 1}, {1: m})], [1, 2, 3])
    main = R.DagNode([R.Con({}, {}, {2: 1, 5: m}), R.Con({}, {}, {0: 1, 2: 2, 3: 1, 6: m}),
                      R.Con({}, {}, {1: m, 4: 1})], [1, 2, 3], edges=[(0, 3)])
    d = G.DOCS
    return p, [internal, main], 1, d["n_pub_out"], d["n_pub_in"], d["n_priv_in"], {0, 1}


def _docs_o0_classes():
    """constraints-json.md:77-81 split the way map_tree classifies (map_to_constraint_list.rs:12-44),
    each class keeping the docs' (DFS) order."""
    sys_ = G.docs_system()
    ce, eq, lin, nl = R.classify(sys_)
    return sys_, {"cons_eq": ce, "eq": eq, "linear": lin, "non_linear": nl}


def _sym_o0():
    return [tuple(int(x) if i < 3 else x for i, x in enumerate(l.split(",", 3))) for l in G.DOCS["sym_o0"]]


def test_docs_basic_flatten_oracle():
    """pyref.flatten_dag on the docs DAG = the reference's published --O0 export."""
    p, nodes, main, no, npb, npr, forb = docs_basic_dag()
    sys_, b = R.flatten_dag(p, nodes, main, no, npb, npr, forb)
    # the --O0 constraint list, in DFS order (constraints-json.md:77-81)
    assert G.rows_to_json(sys_.rows) == G.DOCS["constraints"]["O0"]
    ref_sys, classes = _docs_o0_classes()
    for k in classes:
        assert [(c.a, c.b, c.c) for c in b[k]] == [(c.a, c.b, c.c) for c in classes[k]], k
    assert (sys_.max_signal, sys_.forbidden) == (ref_sys.max_signal, ref_sys.forbidden)
    # sym.md:65-70: --O0 witness = signal order; the #c column names the instance's node
    assert b["witness"] == [0] + [ln[1] for ln in _sym_o0()]
    owner = {s: (1 if s <= 3 else 0) for s in range(1, 7)}
    assert all(ln[2] == owner[ln[0]] for ln in _sym_o0())
    # and simplified: the O1 / O2 texts of the docs
    for lvl in ("O1", "O2"):
        res = R.simplification(sys_, G.flags_of(lvl))
        assert R.to_json_constraints(res.constraints, res.signal_map) == G.DOCS["constraints"][lvl]
        assert R.result_to_sym(_sym_o0(), res).splitlines() == G.DOCS["sym"][lvl]


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
def test_docs_basic_flatten_device():
    """rs_flatten_dag on the docs DAG = the --O0 export of constraints-json.md:77-81 (class by class,
    DFS order), then the device simplifier on that input = the docs' O1 / O2 constraints and
    witness columns (constraints-json.md:57-59, 95-96; sym.md:46-51, 81-86)."""
    p, nodes, main, no, npb, npr, forb = docs_basic_dag()
    inp = M.Dag(p, nodes, main, no, npb, npr, forb, "bn128").flatten(0)
    ce, eq, lin, nl, fb, ms = blocks_of(inp.c)
    ref_sys, classes = _docs_o0_classes()
    for name, got in (("cons_eq", ce), ("eq", eq), ("linear", lin), ("non_linear", nl)):
        assert [(c.a, c.b, c.c) for c in got] == [(c.a, c.b, c.c) for c in classes[name]], name
    assert (ms, fb) == (ref_sys.max_signal, ref_sys.forbidden)
    eng = M.Engine(0)
    for lvl in ("O1", "O2"):
        eng.load(inp.c)
        eng.run(rsio.flags(lvl))
        out = eng.fetch()
        cons, sm, _, npiw = rsio.output_to_py(out.c)
        res = R.Result(cons, sm, npiw)
        assert R.to_json_constraints(res.constraints, res.signal_map) == G.DOCS["constraints"][lvl], lvl
        assert R.result_to_sym(_sym_o0(), res).splitlines() == G.DOCS["sym"][lvl], lvl
    eng.close()


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
def test_engine_flatten_dag_pinned():
    """rs_engine_flatten_dag (page-locked, engine-owned result): the same blocks as rs_flatten_dag and
    the pyref flattening for DAGs of growing size on ONE engine (its buffers grow and are reused), and
    the view fed straight to rs_engine_simplify on that engine equals the oracle."""
    p = R.PRIMES["bn128"]
    eng = M.Engine(0)
    for seed, nt in ((3, 4), (4, 9), (5, 6)):
        nodes, main, no, npb, npr, forb = dagio.gen_dag(300 + seed, p, n_templates=nt, custom_gates=seed % 2 == 1)
        sys_, b = R.flatten_dag(p, nodes, main, no, npb, npr, forb)
        d = M.Dag(p, nodes, main, no, npb, npr, forb, "bn128")
        view = eng.flatten_dag(d)
        _eq_blocks(blocks_of(view), b, sys_)
        one = d.flatten(0)
        assert blocks_of(one.c) == blocks_of(view)
        fl = rsio.flags("O2")
        ref, _, _ = rsio.oracle_run(view, fl)
        got = rsio.output_to_py(eng.simplify(view, fl))
        assert got == ref, seed
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


@pytest.mark.gpu
def test_flatten_rejects_malformed_blocks():
    """Row pointers that leave [0, nnz) and offsets past the 2^31 signal bound are RS_E_INVALID,
    before anything is read out of bounds (host classification or device copy)."""
    p = R.PRIMES["bn128"]
    leaf = R.DagNode([R.Con({}, {}, {1: 1, 2: 3})], [1, 2])
    main = R.DagNode([R.Con({1: 1}, {2: 1}, {3: 1})], [1, 2], edges=[(0, 2)])
    d = M.Dag(p, [leaf, main], 1, 1, 0, 1, {0, 1}, "bn128")
    d.flatten(0).free()  # well-formed: accepted
    d.parts[2].ptr[-1] += 1  # C's ptr[T] past nnz
    with pytest.raises(M.RsError):
        d.flatten(0)
    d.parts[2].ptr[-1] -= 1
    d.edge_in[0] = 1 << 31  # the leaf's ids past 2^31
    with pytest.raises(M.RsError):
        d.flatten(0)
    d.edge_in[0] = (1 << 31) - 2  # leaf id 2 + offset reaches 2^31
    with pytest.raises(M.RsError):
        d.flatten(0)
