"""The result stream of one host -> host step from a rocprofv3 --kernel-trace --memory-copy-trace:
every device-to-host copy of 0.1 ms or more (the trace has no sizes), with the idle time before it,
and the stream's busy time; plus when the step's kernels end.
usage: python3 tools/d2h_gaps.py <prefix> [--step N]"""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("prefix")
ap.add_argument("--step", type=int, default=1)
ap.add_argument("--pause", type=float, default=8.0)
a = ap.parse_args()
cp = [r for r in csv.DictReader(open(a.prefix + "_memory_copy_trace.csv"))]
kt = [r for r in csv.DictReader(open(a.prefix + "_kernel_trace.csv"))]
h2d = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in cp
             if r["Direction"].endswith("HOST_TO_DEVICE") and int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) > 50000)
starts, last = [], None
for s, e in h2d:
    if last is None or s - last > a.pause * 1e6:
        starts.append(s)
    last = e
t0 = starts[a.step]
t1 = starts[a.step + 1] if a.step + 1 < len(starts) else None
d2h = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"]) for r in cp
             if r["Direction"].endswith("DEVICE_TO_HOST") and int(r["Start_Timestamp"]) >= t0 and (t1 is None or int(r["Start_Timestamp"]) < t1))
up_end = max(e for s, e in h2d if t0 <= s and (t1 is None or s < t1))
print(f"step {a.step}: upload ends at {(up_end - t0) / 1e6:.2f} ms")
prev, busy, idle = None, 0, 0
for s, e, q in d2h:
    if e - s < 100000:
        continue
    gap = (s - prev) / 1e6 if prev is not None else 0.0
    print(f"{(s - t0) / 1e6:8.2f} {(e - s) / 1e6:6.2f} ms  s{q}  gap {gap:.2f}")
    if prev is not None and s > prev:
        idle += s - prev
    prev = max(prev or 0, e)
    busy += e - s
ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in kt if int(r["Start_Timestamp"]) >= t0 and (t1 is None or int(r["Start_Timestamp"]) < t1)]
print(f"copies >= 0.1 ms: busy {busy / 1e6:.2f} ms, idle between them {idle / 1e6:.2f} ms; last kernel ends at "
      f"{(max(e for s, e in ks) - t0) / 1e6:.2f} ms; last copy ends at {(max(e for s, e, q in d2h) - t0) / 1e6:.2f} ms")
