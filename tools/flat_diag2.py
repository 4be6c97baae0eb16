"""The seed-303 custom-gate DAG system (forbidden intermediates): engine vs oracle, printed in full."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import dagio  # noqa: E402
import rsio  # noqa: E402
import circom_cvm_amd as M  # noqa: E402

R = rsio.R
p = R.PRIMES["bn128"]


def sh(m):
    return {k: (v if v < 1000 else ("-%d" % (p - v) if p - v < 1000 else "b%d" % (v % 997))) for k, v in sorted(m.items())}


nodes, main, no, npb, npr, forb = dagio.gen_dag(303, p, n_templates=4, custom_gates=True)
sys_, b = R.flatten_dag(p, nodes, main, no, npb, npr, forb)
h = rsio.InputHolder(sys_)
eng = M.Engine(0)
for lvl in ("O1", "O2"):
    fl = rsio.flags(lvl)
    ref, _, _ = rsio.oracle_run(h.inp, fl)
    eng.load(h.inp)
    eng.run(fl)
    o = eng.fetch()
    got = rsio.output_to_py(o.c)
    print(lvl, "oracle", len(ref[0]), "engine", len(got[0]), ref[1:] == got[1:])
    for name, cs in (("oracle", ref[0]), ("engine", got[0])):
        print(" ", name)
        for c in cs:
            print("   ", sh(c.a), sh(c.b), sh(c.c))
eng.close()
