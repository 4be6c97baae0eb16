"""FETCH_SIZE / WRITE_SIZE calibration for this library's access patterns (MI355X_MICROARCH.md 'HBM':
only 16 B/lane streaming reads and writes are calibrated there).  Reads the two rocprofv3 --pmc passes
of tools/micro/pmc_calib (one FETCH_SIZE, one WRITE_SIZE) and the byte counts the program printed, and
writes per pattern the counter's bytes over the bytes the kernel moved.

usage: python tools/pmc_calib.py <fetch_dir> <write_dir> <calib.txt> -o profiles/roundN_pmc_calib.json
The factors divide a kernel's counters into bytes moved (tools/pmc_traffic.py --calib): a factor
above 1 means the memory system moved more than the program asked for (e.g. 64-byte requests for
32-byte random reads), below 1 that the counter under-reports (FETCH_SIZE's 1/2 for wide streams)."""
import argparse
import csv
import glob
import json
import os


def dispatches(d, counter):
    """[(kernel name, value KiB)] in dispatch order of one pass."""
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r.get("Counter_Name") == counter:
                    rows.append((int(r.get("Dispatch_Id", 0)), r.get("Kernel_Name", ""), float(r["Counter_Value"])))
    rows.sort()
    return [(n, v) for _, n, v in rows]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("calib_txt")
    ap.add_argument("-o", "--out", required=True)
    args = ap.parse_args()
    known = []
    for line in open(args.calib_txt):
        p = line.split()
        if len(p) == 3 and p[0].startswith("k_"):
            known.append((p[0], int(p[1]), int(p[2])))
    fe, wr = dispatches(args.fetch_dir, "FETCH_SIZE"), dispatches(args.write_dir, "WRITE_SIZE")
    res = {"source": "tools/micro/pmc_calib under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes); "
                     "factor = counter bytes / bytes the kernel moved (the last launch of each kernel)",
           "fetch_factor": {}, "write_factor": {}}
    for i, (name, rd, wb) in enumerate(known):
        for tab, b, key in ((fe, rd, "fetch_factor"), (wr, wb, "write_factor")):
            if i < len(tab) and name in tab[i][0] and b:
                res[key][name] = round(tab[i][1] * 1024.0 / b, 4)
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
