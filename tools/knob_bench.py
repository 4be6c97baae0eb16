import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import circom_cvm_amd as M
inp = M.Input.synth(0, int(os.environ.get("ROWS", "10000000")), 42)
eng = M.Engine(0); eng.load(inp.c)
fl = M.make_flags("O2")
eng.run(fl)
best = 1e9
for it in range(3):
    t = time.time(); eng.run(fl); dt = time.time() - t
    st = eng.stats()
    best = min(best, dt)
print(os.environ.get("TAG", ""), "best %.1f ms" % (best * 1e3), "prep %.1f main %.1f finish %.1f small %.1f" % (
    st.big_prep_ms, st.big_main_ms, st.big_finish_ms, st.elim_small_ms), flush=True)
