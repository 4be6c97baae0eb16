"""Kernel + copy timeline of rs_engine calls from a rocprofv3 --kernel-trace [--memory-copy-trace]
csv pair: the trace is cut into calls at idle gaps, and one call is printed as start offset,
duration, stream and name of every kernel / copy above a threshold, plus per-stream busy time.
usage: python3 tools/timeline.py <prefix_or_kernel_trace.csv> [--call N] [--min-ms T] [--gap-ms G]"""
import argparse
import csv
import os

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--call", type=int, default=-1, help="which call (default: the last)")
ap.add_argument("--min-ms", type=float, default=0.15)
ap.add_argument("--gap-ms", type=float, default=4.0)
args = ap.parse_args()

kt = args.trace if args.trace.endswith(".csv") else args.trace + "_kernel_trace.csv"
ct = kt.replace("_kernel_trace.csv", "_memory_copy_trace.csv")
ev = []  # (start, end, stream, name)
for r in csv.DictReader(open(kt)):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "s" + r["Stream_Id"],
               r["Kernel_Name"].split("(")[0].replace("void ", "")[:48] + f" g={r['Grid_Size_X']}"))
if os.path.exists(ct):
    for r in csv.DictReader(open(ct)):
        d = r["Direction"].replace("MEMORY_COPY_", "")
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "s" + r["Stream_Id"], "copy " + d))
ev.sort()
calls, cur, last_end = [], [], None
for e in ev:
    if last_end is not None and e[0] - last_end > args.gap_ms * 1e6 and cur:
        calls.append(cur)
        cur = []
    cur.append(e)
    last_end = e[1] if last_end is None else max(last_end, e[1])
if cur:
    calls.append(cur)
print(f"{len(calls)} calls: " + " ".join(f"{(c[-1][1] - c[0][0]) / 1e6:.1f}ms/{len(c)}" for c in calls))
call = calls[args.call]
T0 = call[0][0]
busy = {}
for s, e, q, n in call:
    busy.setdefault(q, 0)
    busy[q] += e - s
    if (e - s) / 1e6 >= args.min_ms:
        print(f"{(s - T0) / 1e6:8.2f} {(e - s) / 1e6:7.2f} {q:>4} {n}")
end = max(e for _, e, _, _ in call)
print(f"end {(end - T0) / 1e6:.2f} ms; busy per stream: " + ", ".join(f"{q} {v / 1e6:.1f}" for q, v in sorted(busy.items())))
# the link after the input: D2H-idle gaps (no device -> host copy in flight) between the end of the
# last host -> device copy and the end of the call
h2d = [e for s, e, q, n in call if n == "copy HOST_TO_DEVICE"]
d2h = sorted((s, e) for s, e, q, n in call if n == "copy DEVICE_TO_HOST")
if h2d and d2h:
    t_in = max(h2d)
    gaps, cov = [], t_in
    for s, e in d2h:
        if e <= t_in:
            continue
        if s > cov:
            gaps.append(((cov - T0) / 1e6, (s - cov) / 1e6))
        cov = max(cov, e)
    if end > cov:
        gaps.append(((cov - T0) / 1e6, (end - cov) / 1e6))
    big = [g for g in gaps if g[1] > 0.5]
    print(f"H2D ends {(t_in - T0) / 1e6:.2f} ms; D2H-idle gaps after it over 0.5 ms (start, length): "
          + (", ".join(f"{a:.2f}+{b:.2f}" for a, b in big) if big else "none")
          + f"; longest {max((g[1] for g in gaps), default=0.0):.2f} ms")
