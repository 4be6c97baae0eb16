"""Diagnosis of test_engine_flatten_dag_pinned: the engine-flattened view simplified four ways."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import dagio  # noqa: E402
import rsio  # noqa: E402
import circom_cvm_amd as M  # noqa: E402

R = rsio.R
p = R.PRIMES["bn128"]
eng = M.Engine(0)
for seed, nt in ((3, 4), (4, 9), (5, 6)):
    nodes, main, no, npb, npr, forb = dagio.gen_dag(300 + seed, p, n_templates=nt, custom_gates=seed % 2 == 1)
    d = M.Dag(p, nodes, main, no, npb, npr, forb, "bn128")
    one = d.flatten(0)
    fl = rsio.flags("O2")
    ref, _, _ = rsio.oracle_run(one.c, fl)
    view = eng.flatten_dag(d)
    ref_v, _, _ = rsio.oracle_run(view, fl)
    e2 = M.Engine(0)
    a = rsio.output_to_py(e2.simplify(one.c, fl))
    e2.load(one.c)
    e2.run(fl)
    o = e2.fetch()
    b = rsio.output_to_py(o.c)
    c = rsio.output_to_py(eng.simplify(view, fl))
    eng.load(view)
    eng.run(fl)
    o2 = eng.fetch()
    dd = rsio.output_to_py(o2.c)
    print(seed, "oracle(one)==oracle(view)", ref == ref_v, "simplify(one)", a == ref,
          "load/run(one)", b == ref, "simplify(view) on flatten engine", c == ref, "load/run(view)", dd == ref, flush=True)
    if a != ref:
        print("  first diff simplify(one):", rsio.same_result(R.Result(ref[0], ref[1], ref[3]), a))
    e2.close()
eng.close()
