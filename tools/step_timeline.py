"""One host -> host step of a rocprofv3 --kernel-trace --memory-copy-trace of bench.py: steps begin at the
first host-to-device copy after a pause of the uploads (> --pause ms); prints the step's kernels over
--min-ms and its copies merged into runs per stream and direction, with the per-stream busy time.
usage: python3 tools/step_timeline.py <prefix> [--step N] [--min-ms T]"""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("prefix")
ap.add_argument("--step", type=int, default=1)
ap.add_argument("--min-ms", type=float, default=0.25)
ap.add_argument("--pause", type=float, default=8.0)
a = ap.parse_args()
ev = []
for r in csv.DictReader(open(a.prefix + "_kernel_trace.csv")):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "s" + r["Stream_Id"],
               r["Kernel_Name"].split("(")[0].replace("void ", "")[:44], "k"))
for r in csv.DictReader(open(a.prefix + "_memory_copy_trace.csv")):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "s" + r["Stream_Id"], r["Direction"].replace("MEMORY_COPY_", ""), "c"))
ev.sort()
h2d = [e for e in ev if e[4] == "c" and e[3] == "HOST_TO_DEVICE" and e[1] - e[0] > 50000]
starts, last = [], None
for e in h2d:
    if last is None or e[0] - last > a.pause * 1e6:
        starts.append(e[0])
    last = e[1]
print(f"{len(starts)} steps")
t0 = starts[a.step]
t1 = starts[a.step + 1] if a.step + 1 < len(starts) else max(e[1] for e in ev)
step = [e for e in ev if t0 - 2e6 <= e[0] < t1]
runs = {}
for s, e, q, n, k in step:
    if k == "c":
        key = (q, n)
        if key in runs and s - runs[key][-1][1] < 0.3e6:
            runs[key][-1][1] = e
            runs[key][-1][2] += 1
        else:
            runs.setdefault(key, []).append([s, e, 1])
out = []
for (q, n), rs in runs.items():
    for s, e, c in rs:
        if (e - s) / 1e6 >= 0.1:
            out.append((s, e, q, f"copy {n} x{c}"))
for s, e, q, n, k in step:
    if k == "k" and (e - s) / 1e6 >= a.min_ms:
        out.append((s, e, q, n))
out.sort()
for s, e, q, n in out:
    print(f"{(s - t0) / 1e6:8.2f} {(e - s) / 1e6:7.2f} {q:>4} {n}")
busy = {}
for s, e, q, n, k in step:
    busy[q] = busy.get(q, 0) + e - s
print(f"step {(t1 - t0) / 1e6:.2f} ms; busy: " + ", ".join(f"{q} {v / 1e6:.1f}" for q, v in sorted(busy.items())))
