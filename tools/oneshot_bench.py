"""PCIe-inclusive rate: rs_simplify (host input -> H2D -> GPU simplification -> D2H host output)."""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import circom_cvm_amd as M
from circom_cvm_amd import abi

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
inp = M.Input.synth(0, rows, 42)
fl = M.make_flags("O2")
for it in range(3):
    out = C.POINTER(abi.RsOutput)()
    t = time.perf_counter()
    abi.check(abi.lib().rs_simplify(C.byref(inp.c), C.byref(fl), C.byref(out)))
    dt = time.perf_counter() - t
    print(f"rs_simplify {inp.rows()} rows: {dt * 1000:.1f} ms -> {inp.rows() / dt / 1e6:.2f} M constraints/s "
          f"(out {out.contents.n_constraints} constraints)", flush=True)
    abi.lib().rs_output_free(out)
