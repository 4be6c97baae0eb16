"""Prints the kernel timeline of the last rs_engine_run in a rocprofv3 --kernel-trace csv (one step of
bench.py): start offset, duration and queue of every kernel above a threshold.
usage: python3 tools/timeline.py <kernel_trace.csv> [min_ms]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
thr = float(sys.argv[2]) if len(sys.argv) > 2 else 0.15
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"].split("(")[0].replace("void ", "")[:44] for r in rows]
starts = [i for i, n in enumerate(names) if n == "rs::k_mark_list"]
firsts = [starts[0]] + [b for a, b in zip(starts, starts[1:]) if b - a > 20]
a = firsts[-1]
T0 = int(rows[a]["Start_Timestamp"])
end = 0
for r, n in zip(rows[a:], names[a:]):
    s = (int(r["Start_Timestamp"]) - T0) / 1e6
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    end = max(end, (int(r["End_Timestamp"]) - T0) / 1e6)
    if d >= thr:
        print(f"{s:8.2f} {d:7.2f} q{r['Queue_Id']} {n} grid={r['Grid_Size_X']}")
print(f"end {end:.2f} ms")
