import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import rsio
import circom_cvm_amd as M
p, seed, rd = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
sys_ = rsio.gen_system(seed, p, n_sig=40 + seed % 50, n_rows=60 + seed % 80)
h = rsio.InputHolder(sys_)
fl = rsio.flags("O2", rd)
ref, _, _ = rsio.oracle_run(h.inp, fl)
for trial in range(2):
    eng = M.Engine(0); eng.load(h.inp)
    seq = [rsio.flags("O1"), fl] if trial else [fl]
    for f in seq:
        eng.run(f)
    out = eng.fetch(); got = rsio.output_to_py(out.c)
    print("trial", trial, "equal", got == ref, flush=True)
    if got != ref:
        for i in range(len(ref[0])):
            if i < len(got[0]) and (got[0][i].c != ref[0][i].c):
                print("  row", i, "C gpu", got[0][i].c, "ref", ref[0][i].c)
