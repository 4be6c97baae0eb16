import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import rsio
import circom_cvm_amd as M
sys_ = rsio.gen_system(0, 257, n_sig=40, n_rows=60)
h = rsio.InputHolder(sys_)
eng = M.Engine(0); eng.load(h.inp)
for f in [rsio.flags("O1"), rsio.flags("O2", 2)]:
    print("=== run", f.flag_s, f.no_rounds, file=sys.stderr, flush=True)
    eng.run(f)
