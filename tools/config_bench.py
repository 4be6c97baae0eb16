"""Per-config GPU timing (host -> host rs_engine_simplify, best of N) of every BASELINE.json config's
synthetic stand-in, with the run's stats; optional oracle check.  Usage:
  python tools/config_bench.py [--check] [--reps 3] [name ...]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import circom_cvm_amd as M  # noqa: E402

CONFIGS = {  # name: (kind, rows, seed, prime)
    "sha": (4, 30_000, 1, "bn128"),
    "linear1M": (1, 1_000_000, 1, "bn128"),
    "poseidon4M": (3, 4_000_000, 2, "bn128"),
    "chain1.5M": (2, 1_500_000, 3, "bn128"),
    "mixed10M": (0, 10_000_000, 42, "bn128"),
    "bls20M": (0, 20_000_000, 42, "bls12381"),
    "templated10M": (5, 10_000_000, 42, "bn128"),
    "templated_tail10M": (6, 10_000_000, 42, "bn128"),
}

ap = argparse.ArgumentParser()
ap.add_argument("names", nargs="*")
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--check", action="store_true")
args = ap.parse_args()
eng = M.Engine(0)
fl = M.make_flags("O2")
for name in args.names or list(CONFIGS):
    kind, rows, seed, prime = CONFIGS[name]
    inp = M.Input.synth(kind, rows, seed, prime)
    pin = M.PinnedInput(inp.c)
    best = None
    all_ms = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        out = eng.simplify(pin.c, fl)
        dt = time.perf_counter() - t0
        st = eng.stats()
        all_ms.append(round(dt * 1000, 1))
        if best is None or dt < best[0]:
            best = (dt, st.as_dict())
    dt, st = best
    line = {"config": name, "rows": inp.rows(), "ms": round(dt * 1000, 2), "Mrows_per_s": round(inp.rows() / dt / 1e6, 2), "all_ms": all_ms,
            "stats": {k: (round(v, 3) if isinstance(v, float) else v) for k, v in st.items()}}
    if args.check:
        import rsio
        got = rsio.output_arrays(out)
        ref, ms = rsio.oracle_arrays(inp.c, fl, threads=16)
        line["bit_exact"] = rsio.diff_output_arrays(got, ref) is None
        line["oracle_ms"] = round(ms, 1)
    print(json.dumps(line), flush=True)
    pin.free()
    inp.free()
