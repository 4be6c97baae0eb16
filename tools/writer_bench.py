"""rs_engine_write_r1cs on the metric circuit's result: best of --reps writes into a temporary
directory (RS_PROF=1 prints the device build / D2H + writers split)."""
import argparse
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import circom_cvm_amd as M  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=10_000_000)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--dir", default=None)
args = ap.parse_args()
inp = M.Input.synth(0, args.rows, 42)
pin = M.PinnedInput(inp.c)
eng = M.Engine(0)
fl = M.make_flags("O2")
eng.simplify(pin.c, fl)
best = None
with tempfile.TemporaryDirectory(dir=args.dir) as tmp:
    path = os.path.join(tmp, "w.r1cs")
    for _ in range(args.reps):
        t0 = time.perf_counter()
        eng.write_r1cs(path)
        dt = (time.perf_counter() - t0) * 1000
        best = dt if best is None else min(best, dt)
    size = os.path.getsize(path)
print(f"write_r1cs best {best:.1f} ms, {size / 1e6:.0f} MB, {size / best / 1e6:.2f} GB/s", flush=True)
eng.close()
