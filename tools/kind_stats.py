"""Per-phase engine statistics of one synthetic workload (host -> host), e.g. to find where a
generator's circuit spends its time: python tools/kind_stats.py KIND ROWS [SEED]."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import circom_cvm_amd as M  # noqa: E402

kind, rows = int(sys.argv[1]), int(sys.argv[2])
seed = int(sys.argv[3]) if len(sys.argv) > 3 else 42
inp = M.Input.synth(kind, rows, seed, "bn128")
pin = M.PinnedInput(inp.c)
eng = M.Engine(0)
fl = M.make_flags("O2")
for it in range(3):
    t = time.time()
    eng.simplify(pin.c, fl)
    dt = time.time() - t
    st = eng.stats().as_dict()
    print(kind, inp.rows(), "step %.1f ms" % (dt * 1e3),
          {k: (round(v, 2) if isinstance(v, float) else v) for k, v in st.items()}, flush=True)
eng.close()
