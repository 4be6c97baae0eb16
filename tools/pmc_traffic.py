"""Per-launch HBM traffic of the bench's kernels from separate rocprofv3 --pmc passes (FETCH_SIZE,
WRITE_SIZE), corrected as MI355X_MICROARCH.md 'HBM' prescribes for gfx950: FETCH_SIZE reports half
the bytes of wide streaming reads, so it is doubled; WRITE_SIZE is taken as is.  rocprofv3 reports
both counters in KiB.

usage: python tools/pmc_traffic.py <fetch_dir> <write_dir> -o profiles/roundN_pmc_traffic.json
           [--wrreq <dir of a TCC_EA0_WRREQ / TCC_EA0_WRREQ_64B pass>] [--steps K] [--commit SHA]
The JSON's `bytes_per_launch` / `bytes_per_step` / `launches_per_step` keys are bench.py's KERNELS
names (the passes run `bench.py --steps K --warmup 0`, so dispatches / K = launches per step of the
profiled code); bench.py reads the newest profiles/round*_pmc_traffic.json into roofline.traffic and
reports the profile's launch count beside its own, so a version skew between the two shows."""
import argparse
import csv
import glob
import json
import os
import sys

# bench.py KERNELS name -> substring of the rocprofv3 kernel name
# (the tail's in-kernel byte counter also counts k_p3_fast, which runs just before k_big_main on the
# same clusters' list: its traffic is added to the tail's, per launch of k_big_main)
GROUPS = {
    "k_big_spec<12> (head)": ("k_big_spec<",),
    "k_big_main<256> (tail)": ("k_big_main<256u>", "k_p3_fast"),
    "k_frames_wave<0> (non-linear)": ("k_frames_wave<0>",),
    "k_frames_wave<1> (rounds)": ("k_frames_wave<1>",),
    "k_batch_inv_flat + k_big_finish<4> (tail normalisation + composition)": ("k_big_finish<4>", "k_batch_inv_flat"),
    "k_batch_inv_tree .. k_big_emit (head normalisation + composition)": (
        "k_big_finish<8>", "k_batch_inv_tree", "k_normalize(", "k_compose_level<", "k_compose_rest<", "k_compose_big(",
        "k_big_emit<"),
    "k_eliminate (clusters under 32 rows)": ("k_eliminate(",),
    "build_clusters (k_cl_*, pair sort, arena replays)": ("k_cl_link(", "k_cl_root(", "k_cl_count(", "k_cl_replay_wave<",
                                                          "k_cl_replay_lane("),
    "k_gi_* (giant clusters' component loops)": ("k_gi_loop(", "k_gi_state(", "k_gi_union(", "k_gi_rowkey(",
                                                "k_gi_segment(", "k_gi_gather(", "k_gi_scatter("),
    "input checks (k_check_ptr, k_check_keys, k_sort_validate)": ("k_sort_validate(", "k_check_ptr(", "k_check_keys("),
    "ragged conversion + linear frames (k_make_ragged, k_lin_*frames*)": ("k_make_ragged(", "k_lin_valframes(",
                                                                          "k_lin_keyframes(", "k_linear_frames12("),
    "result gathers (k_snap_gather*, k_lc_*, k_gather_late, k_gather_rows)": ("k_snap_gather(", "k_snap_gather_st(",
                                                                              "k_lc_snap(", "k_gather_late(",
                                                                              "k_lc_gather_late(", "k_gather_rows("),
}


def coverage(stats_csv):
    """Share of the trace's kernel time the groups cover (rocprofv3 --stats kernel_stats.csv; the
    runtime's own copy / fill kernels are left out of the total)."""
    tot, cov, per = 0.0, 0.0, {}
    for r in csv.DictReader(open(stats_csv)):
        name, ns = r["Name"], float(r["TotalDurationNs"])
        if name.startswith("__amd_rocclr_"):
            continue
        tot += ns
        for g, pats in GROUPS.items():
            if any(p in name for p in pats):
                cov += ns
                per[g] = per.get(g, 0.0) + ns
                break
    return {"covered": round(cov / tot, 4) if tot else None, "kernel_ms_total": round(tot / 1e6, 2),
            "group_ms": {g: round(v / 1e6, 2) for g, v in per.items()}, "source": stats_csv}


def per_dispatch(d, counter):
    """{kernel name: [value per dispatch]} for one counter of one pass."""
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                out.setdefault(row.get("Kernel_Name", ""), []).append(float(row["Counter_Value"]))
    return out


def group_avg(tab, pat):
    vals = [v for name, vs in tab.items() if pat in name for v in vs]
    return (sum(vals) / len(vals), len(vals)) if vals else (None, 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("-o", "--out", required=True)
    ap.add_argument("--wrreq", default=None)
    ap.add_argument("--steps", type=int, default=1, help="bench steps of each pass (warmup 0)")
    ap.add_argument("--commit", default=None, help="git commit the profiled tree was at")
    ap.add_argument("--calib", default=None, help="profiles/roundN_pmc_calib.json (tools/pmc_calib.py): bytes moved "
                    "from the counters with the factors of the gather / emit patterns instead of FETCH_SIZE x2")
    ap.add_argument("--bench", default="bench.py --steps K --warmup 0 --no-cpu", help="what the passes ran (for the record)")
    ap.add_argument("--stats", default=None, help="rocprofv3 --stats kernel_stats.csv of the bench: the groups' coverage")
    args = ap.parse_args()
    fe = per_dispatch(args.fetch_dir, "FETCH_SIZE")
    wr = per_dispatch(args.write_dir, "WRITE_SIZE")
    req = per_dispatch(args.wrreq, "TCC_EA0_WRREQ_sum") if args.wrreq else {}
    req64 = per_dispatch(args.wrreq, "TCC_EA0_WRREQ_64B_sum") if args.wrreq else {}
    cal = json.load(open(args.calib)) if args.calib else None
    res = {"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes of `{args.bench}`; "
                     "FETCH_SIZE x2 (gfx950), KiB -> bytes" + ("; calibrated: FETCH_SIZE / fetch_factor[k_runs36] + "
                                                             "WRITE_SIZE / write_factor[k_emit36] from " + args.calib if cal else ""),
           "commit": args.commit, "steps": args.steps,
           "bytes_per_launch": {}, "bytes_per_step": {}, "launches_per_step": {}, "detail": {}}
    for name, pats in GROUPS.items():
        pat = pats[0]
        f, nf = group_avg(fe, pat)
        w, nw = group_avg(wr, pat)
        if f is None or w is None:
            continue
        for extra in pats[1:]:  # added per launch of the main kernel
            fx, nfx = group_avg(fe, extra)
            wx, nwx = group_avg(wr, extra)
            if fx is not None and nf:
                f += fx * nfx / nf
            if wx is not None and nw:
                w += wx * nwx / nw
        fetch = 2.0 * f * 1024.0
        write = w * 1024.0
        if cal:  # the gather pattern's read factor, the consecutive-slot write pattern's write factor
            fetch = f * 1024.0 / cal["fetch_factor"]["k_runs36"]
            write = w * 1024.0 / cal["write_factor"]["k_emit36"]
        res["bytes_per_launch"][name] = int(fetch + write)
        res["bytes_per_step"][name] = int((fetch + write) * nf / args.steps)
        res["launches_per_step"][name] = nf / args.steps
        det = {"fetch_bytes_x2": int(2.0 * f * 1024.0), "write_bytes_raw": int(w * 1024.0), "fetch_bytes": int(fetch),
               "write_bytes": int(write), "dispatches": [nf, nw]}
        r, _ = group_avg(req, pat)
        r64, _ = group_avg(req64, pat)
        if r is not None and r64 is not None:
            det["wrreq"] = int(r)
            det["wrreq_64B"] = int(r64)
            det["wrreq_32B"] = int(r - r64)
        res["detail"][name] = det
        sys.stderr.write(f"{name}: FETCH_SIZE(x2) {fetch / 1e6:.1f} MB + WRITE_SIZE {write / 1e6:.1f} MB per launch"
                         + (f"; write requests {det.get('wrreq')} ({det.get('wrreq_64B')} of 64 B)" if "wrreq" in det else "")
                         + "\n")
    if args.stats:
        res["coverage"] = coverage(args.stats)
        sys.stderr.write(f"coverage of the kernel time: {res['coverage']['covered']}\n")
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
