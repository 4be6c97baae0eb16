import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import circom_cvm_amd as M
for rows in [int(x) for x in sys.argv[1:]] or [1000000]:
    t = time.time(); inp = M.Input.synth(0, rows, 42); tg = time.time() - t
    eng = M.Engine(0); eng.load(inp.c)
    for it in range(3):
        t = time.time(); eng.run(M.make_flags("O2")); dt = time.time() - t
        st = eng.stats().as_dict()
        print(rows, "run %.3fs" % dt, "rate %.0f c/s" % (inp.rows() / dt), {k: (round(v, 2) if isinstance(v, float) else v) for k, v in st.items()}, flush=True)
    eng.close()
