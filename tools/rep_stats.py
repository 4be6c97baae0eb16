import sys, time, json, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import circom_cvm_amd as M
eng = M.Engine(0); fl = M.make_flags("O2")
inp = M.Input.synth(0, 10_000_000, 42, "bn128"); pin = M.PinnedInput(inp.c)
for i in range(int(sys.argv[1])):
    t0 = time.perf_counter(); out = eng.simplify(pin.c, fl); dt = (time.perf_counter() - t0) * 1000
    s = eng.stats().as_dict()
    print(json.dumps({"i": i, "ms": round(dt, 2), **{k: round(s[k], 2) for k in ("total_ms", "h2d_wait_ms", "d2h_ms", "host_total_ms", "eq_ms", "elim_ms", "cluster_ms", "subst_ms", "nl_ms", "tail_fin_ms", "tail_main_ms", "head_main_ms", "head_fin_ms", "apply_kernel_ms", "rounds_ms", "final_ms", "gather_ms")}}), flush=True)
