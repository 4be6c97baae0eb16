"""Runs one synthetic workload through the engine under the current environment and compares it
with the CPU oracle (diagnostic: bisect kernel variants by env knobs).
usage: python tools/bisect_env.py kind rows [seed]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import rsio  # noqa: E402
import circom_cvm_amd as M  # noqa: E402

kind, rows = int(sys.argv[1]), int(sys.argv[2])
seed = int(sys.argv[3]) if len(sys.argv) > 3 else 42
inp = M.Input.synth(kind, rows, seed)
eng = M.Engine(0)
eng.load(inp.c)
fl = rsio.flags("O2")
eng.run(fl)
out = eng.fetch()
got = rsio.output_to_py(out.c)
ref, _, _ = rsio.oracle_run(inp.c, fl, 8)
env = {k: v for k, v in os.environ.items() if k.startswith("RS_")}
if got != ref:
    print(env, "DIFF", rsio.same_result(rsio.R.Result(ref[0], ref[1], ref[3]), got), flush=True)
else:
    print(env, "OK", flush=True)
