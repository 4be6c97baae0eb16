"""Debug helper (GPU box): find seeded systems where GPU != oracle and dump the differing rows."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import rsio
import circom_cvm_amd as M
R = rsio.R

def fmt(c):
    return [{k: v for k, v in sorted(m.items())} for m in (c.a, c.b, c.c)]

eng = M.Engine(0)
p = int(sys.argv[1]) if len(sys.argv) > 1 else 257
levels = [("O1", None), ("O2", 1), ("O2", 2), ("O2", None)]
nfail = 0
for seed in range(40):
    sys_ = rsio.gen_system(seed, p, n_sig=40 + seed % 50, n_rows=60 + seed % 80)
    h = rsio.InputHolder(sys_)
    res = []
    for lvl, rd in levels:
        fl = rsio.flags(lvl, rd)
        eng.load(h.inp); eng.run(fl)
        st = eng.stats()
        out = eng.fetch(); got = rsio.output_to_py(out.c)
        ref, _, rounds = rsio.oracle_run(h.inp, fl)
        ok = got == ref
        res.append((lvl, rd, ok, st.rounds, rounds))
        if not ok and nfail < 3:
            nfail += 1
            print("FAIL seed", seed, lvl, rd, "gpu rounds", st.rounds, "ref rounds", rounds,
                  "n", len(got[0]), len(ref[0]), "wires", got[2], ref[2])
            for i in range(max(len(got[0]), len(ref[0]))):
                a = fmt(got[0][i]) if i < len(got[0]) else None
                b = fmt(ref[0][i]) if i < len(ref[0]) else None
                if a != b:
                    print("  row", i, "\n    GPU", a, "\n    REF", b)
            if got[1] != ref[1]:
                print("  sm GPU", sorted(got[1].items()), "\n  sm REF", sorted(ref[1].items()))
    print(seed, res)
