"""PCIe probe (GPU box): pinned host <-> HBM copy rates with hipMemcpyAsync (torch copies), one
direction at a time and both at once, for chunk sizes the engine uses.  Run it under different
copy-engine settings (e.g. HSA_ENABLE_SDMA=0) to compare.  usage: python tools/pcie_probe.py"""
import time

import torch

MB = 1 << 20


def rate(fn, nbytes, reps=5):
    torch.cuda.synchronize()
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return nbytes * reps / (time.perf_counter() - t) / 1e9


n = 512 * MB
h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
h2 = torch.empty(n, dtype=torch.uint8, pin_memory=True)
d = torch.empty(n, dtype=torch.uint8, device="cuda")
d2 = torch.empty(n, dtype=torch.uint8, device="cuda")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
for chunk in (4 * MB, 16 * MB, 64 * MB, 512 * MB):
    def h2d():
        with torch.cuda.stream(s1):
            for o in range(0, n, chunk):
                d[o:o + chunk].copy_(h[o:o + chunk], non_blocking=True)

    def d2h():
        with torch.cuda.stream(s2):
            for o in range(0, n, chunk):
                h2[o:o + chunk].copy_(d2[o:o + chunk], non_blocking=True)

    def both():
        h2d()
        d2h()
    print(f"chunk {chunk // MB:4d} MB: H2D {rate(h2d, n):6.1f} GB/s  D2H {rate(d2h, n):6.1f} GB/s  "
          f"both {rate(both, 2 * n):6.1f} GB/s (sum)", flush=True)
