"""Side-by-side kernel times of tools/ab_kernels.sh runs: total ms per kernel name divided by the
number of host->host steps (reps + the config_bench warm-up rep is included, so compare columns, not
absolute values), plus each run's best host->host ms from its log.
usage: python tools/kstats.py <dir> TAG:... TAG:..."""
import csv
import glob
import json
import os
import sys

d, tags = sys.argv[1], [a.split(":", 1)[0] for a in sys.argv[2:]]
tab, best = {}, {}
for t in tags:
    f = glob.glob(os.path.join(d, t, "**", "*kernel_stats.csv"), recursive=True)
    if not f:
        continue
    for r in csv.DictReader(open(f[0])):
        name = r["Name"].split("(")[0].replace("void ", "").replace("rs::", "")[:40]
        tab.setdefault(name, {})[t] = float(r["TotalDurationNs"]) / 1e6
    try:
        best[t] = [json.loads(l)["ms"] for l in open(os.path.join(d, t + ".log")) if l.startswith("{")]
    except OSError:
        pass
top = sorted(tab, key=lambda n: -max(tab[n].values()))[:22]
print("%-40s" % "kernel (total ms)" + "".join("%12s" % t for t in tags))
for n in top:
    print("%-40s" % n + "".join("%12.2f" % tab[n].get(t, 0.0) for t in tags))
print("%-40s" % "host->host ms per config" + "".join("%12s" % ("/".join("%.1f" % x for x in best.get(t, []))) for t in tags))
