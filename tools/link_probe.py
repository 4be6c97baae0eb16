"""D2H / H2D bandwidth of 32 MiB chunks between HBM and page-locked host memory (torch), the
result stream's pattern: python3 tools/link_probe.py [total MiB]"""
import sys
import time
import torch

tot = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
chunk = 32 << 20
dev = torch.empty(tot << 20, dtype=torch.uint8, device="cuda")
host = torch.empty(tot << 20, dtype=torch.uint8, pin_memory=True)
for name, src, dst in (("D2H", dev, host), ("H2D", host, dev)):
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for o in range(0, tot << 20, chunk):
            dst[o:o + chunk].copy_(src[o:o + chunk], non_blocking=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"{name} {tot} MiB in 32 MiB chunks: {dt * 1e3:.2f} ms, {(tot << 20) / dt / 1e9:.1f} GB/s", flush=True)
