"""bench.py -- constraints simplified/sec (--O2) on the 10M-constraint synthetic circuit.

One step = one full --O2 simplification measured as SURVEY 8(d) defines T_simplify: the Simplifier
bundle as CSR blocks in HOST memory -> the simplified constraints + label->wire map in HOST memory
(rs_engine_simplify on a persistent engine: H2D of the input overlapped with the simplification,
device validation, the whole of constraint_simplification.rs:442-730 on the GPU, D2H of the result
into pinned buffers).  The input blocks live in page-locked memory from rs_host_alloc, the buffers a
Rust shim marshals the Simplifier into.

N = 1: the metric circuit on one GPU.  N > 1 (one process per GPU, torch.distributed over RCCL):
`value` is the SAME circuit sharded over the N ranks (its clusters dealt to the ranks, the
eliminated-signal map exchanged over RCCL; strong scaling); the independent-shard number (each rank
its own circuit, no collective; weak scaling) is the extra object `weak_shards`.

Rank 0 prints ONE JSON line with: the roofline of the dominant kernel (HIP events on the library's
streams, in-kernel algorithmic bytes; head and tail of the ordered elimination split), the
whole-path roofline B_alg / T_simplify, the HBM-resident rate as an extra key, the CPU baseline (the
canonical CPU oracle oracle/refcpu.cpp on this box's cores, plus a 1-thread leg on a bounded sample)
and `bit_exact`: the last timed step's output compared array for array with the oracle's."""
from __future__ import annotations

import argparse
import glob
import json
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "constraints simplified/sec (--O2) on 10M-constraint circuit; bit-exact .r1cs"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def cpu_threads() -> int:
    """Host threads for the CPU baseline: this process's CPU share (the box exports
    OMP_NUM_THREADS = its share; os.sched_getaffinity lists the whole machine there)."""
    aff = len(os.sched_getaffinity(0))
    env = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(aff, int(env))) if env and env.isdigit() else aff


def cpu_baseline(M, inp, threads: int, j1_rows: int, seed: int, prime: str):
    """The canonical CPU oracle (oracle/refcpu.cpp) on the rank-0 workload on `threads` threads (its
    output is the bit-exactness reference), and on 1 thread over a bounded sample (the same generator,
    j1_rows rows)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import rsio
    arrays, ms = rsio.oracle_arrays(inp.c, rsio.flags("O2"), threads=threads)
    alg = rsio.oracle_last_alg()  # B_alg of the same run (the roofline path's numerator)
    res = {"value": round(inp.rows() / (ms / 1000.0), 1), "unit": "constraints/s", "cores": threads,
           "kind": "port", "affinity_cpus": len(os.sched_getaffinity(0)),
           "sample": f"the full rank-0 workload ({inp.rows()} rows), oracle/refcpu.cpp simplification() "
                     f"on {threads} threads: {ms / 1000.0:.2f} s"}
    if j1_rows > 0:
        smp = M.Input.synth(0, j1_rows, seed, prime)
        _, ms1 = rsio.oracle_arrays(smp.c, rsio.flags("O2"), threads=1)
        res["j1"] = {"value": round(smp.rows() / (ms1 / 1000.0), 1), "unit": "constraints/s", "cores": 1,
                     "sample": f"synth_mixed rows={smp.rows()} seed={seed} {prime} --O2 on 1 thread: "
                               f"{ms1 / 1000.0:.2f} s"}
        smp.free()
    return res, arrays, alg


def reduce_over_ranks(dist, dt: float, n_rows: int, device):
    """(max over ranks of the timed region, total constraints over ranks); identity without dist."""
    if dist is None:
        return dt, n_rows
    import torch
    t = torch.tensor([dt, float(n_rows)], device=device, dtype=torch.float64)
    mx = t.clone()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    sm = t.clone()
    dist.all_reduce(sm, op=dist.ReduceOp.SUM)
    return float(mx[0]), int(sm[1])


def share_comm_id(dist, rank: int, make):
    """Rank 0 makes the RCCL unique id (`make()`), every rank returns it (broadcast over the
    torch.distributed group): the rendezvous of rs_engine_join_rccl."""
    obj = [make() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    return obj[0]


def shard_seed(seed: int, rank: int) -> int:
    """Weak-scaling mode: rank r simplifies its own circuit, the generator seeded with seed + r."""
    return seed + rank


KERNELS = (  # (name, stats fields: ms, bytes, launches)
    # the first three are ONE kernel each between their HIP events (SINGLE below); the rest are groups
    ("k_big_spec<12> (head)", "head_main_ms", "head_main_bytes", "head_launches"),
    # the tail's byte counter includes k_p3_fast's clusters (its PMC traffic is added likewise);
    # the time is k_big_main's
    ("k_big_main<256> (tail)", "tail_main_ms", "tail_main_bytes", "tail_launches"),
    ("k_frames_wave<0> (non-linear)", "apply_kernel_ms", "apply_bytes", "apply_kernel_launches"),
    ("k_frames_wave<1> (rounds)", "round_fill_ms", "round_fill_bytes", "round_fill_launches"),
    # ABI 8: the rest of the elimination and the clustering (HIP events on their own streams)
    ("k_batch_inv_flat + k_big_finish<4> (tail normalisation + composition)", "tail_fin_ms", "tail_fin_bytes",
     "tail_fin_launches"),
    ("k_batch_inv_tree .. k_big_emit (head normalisation + composition)", "head_fin_ms", "head_fin_bytes",
     "head_fin_launches"),
    ("k_eliminate (clusters under 32 rows)", "small_ms", "small_bytes", "small_launches"),
    ("build_clusters (k_cl_*, pair sort, arena replays)", "cluster_dev_ms", "cluster_bytes", "cluster_launches"),
    ("k_gi_* (giant clusters' component loops)", "giant_ms", "giant_bytes", "giant_launches"),
    ("input checks (k_check_ptr, k_check_keys, k_sort_validate)", "check_ms", "check_bytes", "check_launches"),
    ("ragged conversion + linear frames (k_make_ragged, k_lin_*frames*)", "ragged_ms", "ragged_bytes", "ragged_launches"),
    ("result gathers (k_snap_gather*, k_lc_*, k_gather_late, k_gather_rows)", "gather_ms", "gather_bytes", "gather_launches"),
)


# entries whose HIP-event pair brackets exactly one kernel launch, with that kernel's rocprof name: the
# headline roofline's "dominant kernel" is chosen among these by device time (a group's span can hold
# several kernels, host waits and syncs -- the clustering's did -- so it is reported, not ranked)
SINGLE = {
    "k_big_spec<12> (head)": "rs::k_big_spec<12>(",
    "k_big_main<256> (tail)": "rs::k_big_main<256u>(",
    "k_frames_wave<0> (non-linear)": "rs::k_frames_wave<0>(",
}


def kernel_profile():
    """Per-kernel rows (calls, average ns) of the newest committed rocprofv3 --kernel-trace --stats summary
    of the metric circuit (profiles/round*_kernel_stats.csv; the templated circuit's file is not it)."""
    import csv
    files = sorted(f for f in glob.glob(os.path.join(ROOT, "profiles", "round*_kernel_stats.csv"))
                   if re.fullmatch(r"round\d+_kernel_stats\.csv", os.path.basename(f)))
    if not files:
        return [], None
    with open(files[-1]) as f:
        rows = [(r["Name"], int(r["Calls"]), float(r["AverageNs"]), float(r["TotalDurationNs"])) for r in csv.DictReader(f)]
    rows.sort(key=lambda r: -r[3])
    return rows, os.path.relpath(files[-1], ROOT)


def link_probe(device: int, mib: int = 512):
    """The box's PCIe link between HBM and page-locked host memory: H2D and D2H of `mib` MiB in 32 MiB
    chunks on one stream (the input's and the result stream's pattern), best of 3 each -- so a host ->
    host number can be read against the link it ran on.  Through the HIP runtime the library already
    loaded (ctypes; no torch, whose bundled runtime would be a second one in the process)."""
    import ctypes as C
    hip = C.CDLL("libamdhip64.so.7")

    def chk(rc, what):
        if rc:
            raise RuntimeError(f"{what}: hip error {rc}")
    n, chunk = mib << 20, 32 << 20
    dev, host, st = C.c_void_p(), C.c_void_p(), C.c_void_p()
    chk(hip.hipSetDevice(device), "hipSetDevice")
    chk(hip.hipMalloc(C.byref(dev), C.c_size_t(n)), "hipMalloc")
    chk(hip.hipHostMalloc(C.byref(host), C.c_size_t(n), 0), "hipHostMalloc")
    chk(hip.hipStreamCreateWithFlags(C.byref(st), 1), "hipStreamCreate")
    res = {}
    try:
        for name, kind in (("h2d_GBps", 1), ("d2h_GBps", 2)):
            best = 0.0
            for _ in range(3):
                chk(hip.hipStreamSynchronize(st), "sync")
                t0 = time.perf_counter()
                for o in range(0, n, chunk):
                    d, h = C.c_void_p(dev.value + o), C.c_void_p(host.value + o)
                    src, dst = (h, d) if kind == 1 else (d, h)
                    chk(hip.hipMemcpyAsync(dst, src, C.c_size_t(min(chunk, n - o)), kind, st), "hipMemcpyAsync")
                chk(hip.hipStreamSynchronize(st), "sync")
                best = max(best, n / (time.perf_counter() - t0) / 1e9)
            res[name] = round(best, 1)
    finally:
        hip.hipStreamDestroy(st)
        hip.hipFree(dev)
        hip.hipHostFree(host)
    res["what"] = f"{mib} MiB in 32 MiB chunks between HBM and pinned host memory, best of 3, before the timed region"
    return res


def fs_write_bound(dirname: str, size: int, reps: int = 2) -> float:
    """GB/s of the file system under `dirname` for a fresh file of `size` bytes written from host memory
    (32 MB pwrites after fallocate, one writer, best of reps): the bound the .r1cs writer is held to."""
    chunk = 32 << 20
    mv = memoryview(bytearray(os.urandom(1 << 20)) * 32)
    best = 0.0
    for k in range(reps):
        path = os.path.join(dirname, f"fs_probe{k}.bin")
        t0 = time.perf_counter()
        fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
        try:
            os.posix_fallocate(fd, 0, size)
        except OSError:
            os.ftruncate(fd, size)
        for o in range(0, size, chunk):
            os.pwrite(fd, mv[:min(chunk, size - o)], o)
        os.close(fd)
        best = max(best, size / (time.perf_counter() - t0) / 1e9)
        os.unlink(path)
    return best


def hip_runtime():
    """The HIP runtime and RCCL this process mapped (torch ships its own libamdhip64.so.7 with the same
    SONAME: whichever loads first serves both; at N = 1 torch is not loaded)."""
    libs = set()
    try:
        with open("/proc/self/maps") as f:
            for ln in f:
                p = ln.split()[-1] if ln.strip() else ""
                if any(x in p for x in ("libamdhip64", "librccl", "libhsa-runtime64")):
                    libs.add(p)
    except OSError:
        pass
    return sorted(libs)


def pmc_traffic():
    """HBM bytes per launch per kernel from the newest committed PMC summary (profiles/
    round*_pmc_traffic.json, written by tools/pmc_traffic.py from separate FETCH_SIZE / WRITE_SIZE
    rocprofv3 passes of this bench)."""
    # the metric circuit's file only (round4_templated_pmc_traffic.json is the templated circuit's)
    files = sorted(f for f in glob.glob(os.path.join(ROOT, "profiles", "round*_pmc_traffic.json"))
                   if re.fullmatch(r"round\d+_pmc_traffic\.json", os.path.basename(f)))
    if not files:
        return {}, None
    with open(files[-1]) as f:
        d = json.load(f)
    tab = {k: {"per_launch": v, "per_step": d.get("bytes_per_step", {}).get(k),
               "launches_per_step": d.get("launches_per_step", {}).get(k)}
           for k, v in d.get("bytes_per_launch", {}).items()}
    src = os.path.relpath(files[-1], ROOT) + (f" @ {d['commit']}" if d.get("commit") else "")
    return tab, src


class _Con:  # the .a / .b / .c shape circom_cvm_amd.Dag reads
    __slots__ = ("a", "b", "c")

    def __init__(self, a, b, c):
        self.a, self.b, self.c = a, b, c


class _Node:  # DagNode's shape: constraints, locals, custom_gate, edges
    __slots__ = ("constraints", "locals", "custom_gate", "edges")

    def __init__(self, constraints, locals_, edges=()):
        self.constraints, self.locals, self.custom_gate, self.edges = constraints, locals_, False, list(edges)


def flatten_bench(seed: int, prime: str, mids: int = 12000, leaves: int = 20, reps: int = 3):
    """SURVEY 8(f) rank 1 measured: rs_flatten_dag on a 3-level synthetic component DAG (main -> `mids`
    mid templates -> `leaves` leaf templates each; ~9.8 M instance constraints, 252 k instances) --
    the DAG a circuit of the metric's size hands to map().  Checked by a size-independent property:
    every block's row count equals the templates' class counts times their instance counts."""
    import random

    import circom_cvm_amd as M
    p = _prime_value(prime)
    rng = random.Random(seed)

    def coef():
        return rng.randrange(1, p)
    L_LEAF, L_MID = 30, 10
    lc = []
    for _ in range(4):  # constant equalities
        lc.append(_Con({}, {}, {rng.randint(1, L_LEAF): 1, 0: coef()}))
    for _ in range(10):  # equalities
        x, y = rng.sample(range(1, L_LEAF + 1), 2)
        c = coef()
        lc.append(_Con({}, {}, {x: c, y: p - c}))
    for _ in range(14):  # linear
        lc.append(_Con({}, {}, {k: coef() for k in rng.sample(range(1, L_LEAF + 1), 4)}))
    for _ in range(12):  # quadratic
        x, y, z = rng.sample(range(1, L_LEAF + 1), 3)
        lc.append(_Con({x: coef()}, {y: coef()}, {z: 1}))
    leaf = _Node(lc, list(range(1, L_LEAF + 1)))
    s_mid = L_MID + leaves * L_LEAF
    mc = []
    for k in range(leaves):
        c = coef()
        mc.append(_Con({}, {}, {1 + k % L_MID: c, L_MID + L_LEAF * k + 1: p - c}))
    mid = _Node(mc, list(range(1, L_MID + 1)), [(0, L_MID + L_LEAF * k) for k in range(leaves)])
    main = _Node([_Con({}, {}, {1: 1, 2: 1, 3: 1, 4: 1}), _Con({}, {}, {1: 2, 2: 3, 3: 1, 5: 1})], [1, 2, 3],
                 [(1, 3 + s_mid * j) for j in range(mids)])
    dag = M.Dag(p, [leaf, mid, main], 2, 1, 1, 1, {0, 1, 2}, prime)
    n_leaf = mids * leaves
    want = {"cons_eq": 4 * n_leaf, "eq": 10 * n_leaf + leaves * mids, "linear": 14 * n_leaf + 2,
            "nl": 12 * n_leaf}
    times, ok = [], True
    eng = M.Engine(0)
    for _ in range(reps):
        t0 = time.perf_counter()
        c = eng.flatten_dag(dag)
        times.append(time.perf_counter() - t0)
        got = {"cons_eq": c.cons_eq.n_rows, "eq": c.eq.n_rows, "linear": c.linear.n_rows, "nl": c.nl_a.n_rows}
        ok &= got == want and c.max_signal == 1 + 3 + mids * (L_MID + leaves * L_LEAF)
    eng.close()
    n = sum(want.values())
    best = min(times)
    return {"ms": round(best * 1e3, 2), "constraints": n, "instances": 1 + mids * (1 + leaves),
            "value": round(n / best, 1), "unit": "constraints/s", "counts_ok": bool(ok),
            "what": "rs_engine_flatten_dag host DAG -> host rs_input in the engine's page-locked buffers "
                    "(templates up, every instance's rows classified and offset on the device, blocks back "
                    "over PCIe at link speed), best of %d" % reps}


def _prime_value(name: str) -> int:
    """The field's modulus as the library knows it (a 1-row synthetic input carries it)."""
    import circom_cvm_amd as M
    inp = M.Input.synth(1, 1, 0, name)
    v = sum(int(inp.c.prime[i]) << (64 * i) for i in range(4))
    inp.free()
    return v


def timed_steps(eng, inp_c, fl, steps, barrier):
    """K host -> host steps between barriers; per-kernel device time/bytes summed over them."""
    acc = {k: [0.0, 0, 0] for k, *_ in KERNELS}
    tot = {"alg_bytes": 0, "total_ms": 0.0, "h2d_wait_ms": 0.0, "d2h_ms": 0.0, "host_total_ms": 0.0,
           "cluster_ms": 0.0, "cluster_host_ms": 0.0}
    barrier()
    t0 = time.perf_counter()
    out = None
    per = {"step_ms": [], "cluster_ms": []}  # per-step spread (the line's value is total / K)
    for _ in range(steps):
        ts = time.perf_counter()
        out = eng.simplify(inp_c, fl)
        per["step_ms"].append((time.perf_counter() - ts) * 1000.0)
        st = eng.stats()
        per["cluster_ms"].append(st.cluster_ms)
        for k, fm, fb, fn in KERNELS:
            acc[k][0] += getattr(st, fm)
            acc[k][1] += getattr(st, fb)
            acc[k][2] += getattr(st, fn)
        for k in tot:
            if k != "per_step":
                tot[k] += getattr(st, k)
    barrier()
    tot["per_step"] = per
    return time.perf_counter() - t0, acc, tot, out, eng.stats()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=80)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--prime", default="bn128")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: this process's CPU share")
    ap.add_argument("--cpu-j1-rows", type=int, default=2_000_000)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-weak", action="store_true", help="N>1: skip the independent-shard extra run")
    ap.add_argument("--no-flatten", action="store_true", help="skip the rs_flatten_dag extra measurement")
    ap.add_argument("--no-templated", action="store_true", help="skip the template-replicated extra circuit")
    ap.add_argument("--no-o1", action="store_true", help="skip the --O1 extra (the metric circuit at circom's default level)")
    ap.add_argument("--no-linear1m", action="store_true", help="skip BASELINE configs[1] (1 M purely linear rows, one run)")
    ap.add_argument("--no-link", action="store_true", help="skip the PCIe link probe")
    ap.add_argument("--no-hbm", action="store_true", help="skip the HBM-resident extra (profiling passes: host -> host steps only)")
    ap.add_argument("--no-write", action="store_true", help="skip the .r1cs writer extra")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # N > 1: torch first.  torch bundles its own HIP runtime and RCCL; loaded first, the library binds to
    # them (same SONAME), loaded after the library torch maps a second runtime beside /opt/rocm's and the
    # two do not mix.  N = 1 needs no torch: the library runs on /opt/rocm's runtime, as under a Rust host.
    # RS_BENCH_HOSTCOMM=1: a one-GPU rehearsal of the N > 1 path -- every rank on device 0, joined over
    # the host transport (rs_engine_join_host; RCCL refuses two ranks on one device), torch's own
    # collectives over gloo.  The driver's N > 1 runs never set it.
    rehearse = world > 1 and os.environ.get("RS_BENCH_HOSTCOMM") == "1"
    red_dev = "cpu" if rehearse else "cuda"
    if world > 1:
        import torch
        import torch.distributed as dist_
        if rehearse:
            local = 0
            dist_.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist_.init_process_group("nccl", device_id=torch.device("cuda", local))
        dist = dist_
    import circom_cvm_amd as M
    M.abi.lib()
    sys.path.insert(0, os.path.join(ROOT, "tests"))

    def barrier():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    fl = M.make_flags("O2", device=local)
    link = None
    if not args.no_link:
        try:
            link = link_probe(local)
        except Exception as e:  # noqa: BLE001 -- a missing torch / device leaves the field out, not the bench
            link = {"error": str(e)[:200]}
    # ---- the headline: the metric circuit (ONE circuit over all ranks when N > 1), host -> host
    inp = M.Input.synth(0, args.rows, args.seed, args.prime)
    n_rows = inp.rows()
    pin = M.PinnedInput(inp.c)
    eng = M.Engine(local)
    if rehearse:
        eng.join_host(world, rank, "bench" + os.environ.get("MASTER_PORT", "0"))
    elif world > 1:
        eng.join_rccl(world, rank, share_comm_id(dist, rank, M.comm_unique_id))
    for _ in range(args.warmup):
        eng.simplify(pin.c, fl)
    dt, acc, tot, out, last = timed_steps(eng, pin.c, fl, args.steps, barrier)
    dt, _ = reduce_over_ranks(dist, dt, n_rows, red_dev)
    got = None
    if rank == 0 and not args.no_cpu:
        import rsio
        got = rsio.output_arrays(out)  # copy of the last timed step's result (the view is reused)
    # the last result written as .r1cs by the device writer (8(d): write timed apart)
    write = None
    if rank == 0 and not args.no_write:
        import tempfile
        try:
            with tempfile.TemporaryDirectory() as tmp:
                path = os.path.join(tmp, "bench_O2.r1cs")
                ms_w = eng.write_r1cs(path)
                nb = os.path.getsize(path)
                os.unlink(path)
                fsb = fs_write_bound(tmp, nb)
                write = {"ms": round(ms_w, 2), "bytes": nb, "GBps": round(nb / ms_w / 1e6, 2),
                         "fs_bound_GBps": round(fsb, 2), "of_fs_bound": round(nb / ms_w / 1e6 / max(fsb, 1e-9), 3),
                         "what": "rs_engine_write_r1cs: the last step's result as a .r1cs file (constraint section "
                                 "built on the device, streamed to a fresh file in a temporary directory); fs_bound: the "
                                 "same number of bytes written from host memory into a fresh file there (no GPU)"}
        except Exception as e:  # noqa: BLE001 -- N > 1: an extra's failure is reported in the line, not fatal
            if world == 1:
                raise
            write = {"error": str(e)[:300]}
    # the DAG flattening that produces such an input, timed on its own
    flat = flatten_bench(args.seed, args.prime) if rank == 0 and not args.no_flatten else None
    # SURVEY 8(d) config 5's template replication (64-row instances sharing coefficients, wired
    # into chains): the same metric on that circuit, host -> host (parity: tests/test_gpu_configs.py)
    tmpl = None
    if rank == 0 and world == 1 and not args.no_templated:
        tinp = M.Input.synth(5, args.rows, args.seed, args.prime)
        tpin = M.PinnedInput(tinp.c)
        for _ in range(2):
            eng.simplify(tpin.c, fl)
        k_t = min(args.steps, 20)
        tdt, _, _, _, tst = timed_steps(eng, tpin.c, fl, k_t, lambda: None)
        tmpl = {"value": round(tinp.rows() * k_t / tdt, 1), "unit": "constraints/s",
                "ms_per_step": round(tdt * 1000.0 / k_t, 3), "steps": k_t, "constraints": tinp.rows(),
                "max_cluster": int(tst.max_cluster), "rounds": int(tst.rounds),
                "elim_ms": round(tst.elim_ms, 2),
                "workload": f"synth_templated rows={args.rows} seed={args.seed} {args.prime} --O2: 16 templates "
                            f"of 64 rows replicated with signal offsets, instances wired into log-normal chains "
                            f"(SURVEY 8(d) config 5's replication), host -> host"}
        tpin.free()
        tinp.free()
    # ---- extra: BASELINE configs[1], 1 M purely linear rows (synth_linear seed 1: one 559 k-row cluster
    # whose largest takeable component -- 100 k rows, 9.9 M merges -- runs the giant path's table loop;
    # latency-bound).  One host -> host run (the pool is sized for it up front); parity at
    # reduced size in tests/test_gpu_giant.py
    lin = None
    if rank == 0 and world == 1 and not args.no_linear1m:
        linp = M.Input.synth(1, 1_000_000, 1, args.prime)
        lpin = M.PinnedInput(linp.c)
        t0 = time.perf_counter()
        eng.simplify(lpin.c, fl)
        ldt = time.perf_counter() - t0
        lst = eng.stats()
        lin = {"value": round(linp.rows() / ldt, 1), "unit": "constraints/s", "ms_per_step": round(ldt * 1000.0, 1),
               "steps": 1, "constraints": linp.rows(), "max_cluster": int(lst.max_cluster),
               "giant_ms": round(lst.giant_ms, 1), "giant_merges": int(lst.giant_merges),
               "merges_per_us": round(lst.giant_merges / max(lst.giant_ms * 1000.0, 1e-9), 3),
               "workload": f"synth_linear rows=1000000 seed=1 {args.prime} --O2 (BASELINE configs[1]), host -> host"}
        lpin.free()
        linp.free()
    # ---- extra: --O1, circom's default since 2.2.0 (circom/src/input_user.rs:304): the same circuit,
    # host -> host; no linear elimination, the linear rows join lconst (constraint_simplification.rs:575-577)
    o1 = None
    if rank == 0 and world == 1 and not args.no_o1:
        fl1 = M.make_flags("O1", device=local)
        for _ in range(2):
            eng.simplify(pin.c, fl1)
        k1 = min(args.steps, 20)
        o1dt, _, _, o1out, _ = timed_steps(eng, pin.c, fl1, k1, lambda: None)
        o1 = {"value": round(n_rows * k1 / o1dt, 1), "unit": "constraints/s", "ms_per_step": round(o1dt * 1000.0 / k1, 3),
              "steps": k1, "constraints": n_rows, "n_constraints_out": int(o1out.n_constraints),
              "workload": f"synth_mixed rows={args.rows} seed={args.seed} {args.prime} --O1, host -> host"}
        if not args.no_cpu:
            import rsio
            o1["_arrays"] = rsio.output_arrays(o1out)  # checked against the oracle below, then dropped
    # ---- extra: the same engine with the input resident in HBM (rs_engine_run only)
    dt_hbm = None
    if not args.no_hbm:
        eng.load(pin.c)
        barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            eng.run(fl)
        barrier()
        dt_hbm, _ = reduce_over_ranks(dist, time.perf_counter() - t0, n_rows, red_dev)
    eng.close()
    pin.free()
    # ---- extra at N > 1: independent circuits per rank (weak scaling, no data-path collective)
    weak = None
    if world > 1 and not args.no_weak:
        winp = M.Input.synth(0, args.rows, shard_seed(args.seed, rank), args.prime)
        wpin = M.PinnedInput(winp.c)
        weng = M.Engine(local)
        for _ in range(args.warmup):
            weng.simplify(wpin.c, fl)
        wdt, _, _, _, _ = timed_steps(weng, wpin.c, fl, args.steps, barrier)
        wdt, wrows = reduce_over_ranks(dist, wdt, winp.rows(), red_dev)
        weng.close()
        wpin.free()
        winp.free()
        weak = {"scaling": "weak", "value": round(wrows * args.steps / wdt, 1), "unit": "constraints/s",
                "ms_per_step": round(wdt * 1000.0 / args.steps, 3),
                "workload": f"each rank its own synth_mixed rows={args.rows} seed={args.seed}+rank circuit "
                            f"(no data-path collective), host -> host"}

    if rank == 0:
        K = args.steps
        ms_step = dt * 1000.0 / K
        value = n_rows * K / dt
        # the dominant kernel: the largest device time over the timed region among the entries that time
        # one kernel (SINGLE); rocprof's own summary of the same bench names the same kernel first
        k_name = max((k for k in acc if k in SINGLE), key=lambda k: acc[k][0])
        traffic_tab, traffic_src = pmc_traffic()
        prof_rows, prof_src = kernel_profile()

        def kline(k):
            ms, by, n = acc[k]
            per_s = (ms / 1000.0) / max(n, 1)
            per_b = by / max(n, 1)
            ach = per_b / per_s / 1e9 if per_s > 0 else 0.0
            tr = traffic_tab.get(k) or {}
            r = {"achieved": round(ach, 3), "frac": round(ach / HBM_PEAK_GBS, 6),
                 "avg_launch_ms": round(per_s * 1000.0, 4), "alg_bytes_per_launch": int(per_b),
                 "launches_per_step": n / K, "ms_per_step": round(ms / K, 3),
                 "traffic": tr.get("per_launch")}
            if tr.get("per_step") is not None:
                # per step, so a launch-count difference cannot skew the ratio; the profile's own
                # launch count is reported beside this run's
                r["traffic_per_step"] = tr["per_step"]
                r["traffic_launches_per_step"] = tr.get("launches_per_step")
                r["traffic_over_alg"] = round(tr["per_step"] / max(by / K, 1.0), 3)
            return r
        dom = kline(k_name)
        path_ach = tot["alg_bytes"] / K / (ms_step / 1000.0) / 1e9
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "constraints/s", "n_gpus": world,
            "steps": K, "warmup": args.warmup, "ms_per_step": round(ms_step, 3),
            "higher_is_better": True, "scaling": "strong" if world > 1 else "weak", "vs_baseline": None,
            "dtype": "u64x4 (F_p, 256-bit Montgomery)", "data": "synthetic",
            "config": {"workload": f"synth_mixed rows={args.rows} prime={args.prime} seed={args.seed} --O2 "
                                   f"(metric circuit, SURVEY 8(d) config 5), host CSR -> host CSR + "
                                   f"label_to_wire (T_simplify)" + (f", ONE circuit sharded over {world} ranks "
                                                                    f"(RCCL exchange of the eliminated-signal map)"
                                                                    if world > 1 else ""),
                       "constraints": n_rows, "parallelism": f"clusters{world}" if world > 1 else "single"},
            "roofline": {"bound": "hbm", "kernel": k_name, "achieved": dom["achieved"], "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": dom["frac"], "traffic": dom["traffic"],
                         "traffic_per_step": dom.get("traffic_per_step"),
                         "traffic_launches_per_step": dom.get("traffic_launches_per_step"),
                         "traffic_over_alg": dom.get("traffic_over_alg"),
                         "traffic_source": traffic_src, "avg_launch_ms": dom["avg_launch_ms"],
                         "alg_bytes_per_launch": dom["alg_bytes_per_launch"],
                         "launches_per_step": dom["launches_per_step"],
                         "timing": "HIP events around each launch of this one kernel on the stream it runs on",
                         "path": {"alg_bytes_per_step": int(tot["alg_bytes"] / K), "T_simplify_ms": round(ms_step, 3),
                                  "achieved": round(path_ach, 2), "frac": round(path_ach / HBM_PEAK_GBS, 5)},
                         "kernels": {k: kline(k) for k in acc if acc[k][2]}},
            "phases_ms": {"device_run": round(tot["total_ms"] / K, 3), "h2d_wait": round(tot["h2d_wait_ms"] / K, 3),
                          "d2h": round(tot["d2h_ms"] / K, 3), "host_total": round(tot["host_total_ms"] / K, 3)},
            "last_step": {k: round(getattr(last, k), 2) for k in
                          ("eq_ms", "cluster_ms", "elim_ms", "subst_ms", "final_ms", "rounds")},
            "hbm_resident": None if dt_hbm is None else
            {"value": round(n_rows * K / dt_hbm, 1), "unit": "constraints/s", "ms_per_step": round(dt_hbm * 1000.0 / K, 3),
             "what": "rs_engine_run: input already in HBM -> result in HBM (no PCIe)"},
        }
        if prof_rows:
            # the same kernel in the committed rocprofv3 summary: its average launch and the roofline
            # fraction recomputed from it (the line's frac must follow from the profile)
            pat = SINGLE[k_name]
            hit = next((r for r in prof_rows if pat in r[0]), None)
            top = prof_rows[0]
            rf = line["roofline"]
            rf["profile"] = {"source": prof_src, "top_kernel": top[0], "top_kernel_share": round(top[3] / sum(r[3] for r in prof_rows), 4)}
            if hit is not None:
                pavg = hit[2] / 1e6
                pach = dom["alg_bytes_per_launch"] / (pavg / 1000.0) / 1e9
                rf["profile"].update({"kernel": hit[0], "calls": hit[1], "avg_launch_ms": round(pavg, 4),
                                      "avg_over_bench": round(pavg / max(dom["avg_launch_ms"], 1e-9), 3),
                                      "achieved_from_profile": round(pach, 3), "frac_from_profile": round(pach / HBM_PEAK_GBS, 6)})
        # the clustering group's span (HIP events on the main stream) split into the device-busy part and
        # the host's round trips inside it (synchronisations, the host replay)
        line["clustering"] = {"span_ms": round(acc["build_clusters (k_cl_*, pair sort, arena replays)"][0] / K, 3),
                              "host_wait_ms": round(tot["cluster_host_ms"] / K, 3),
                              "host_ms": round(tot["cluster_ms"] / K, 3)}
        def spread(xs):
            xs = sorted(xs)
            return {"min": round(xs[0], 3), "median": round(xs[len(xs) // 2], 3), "max": round(xs[-1], 3)} if xs else None
        line["per_step"] = {k: spread(v) for k, v in tot["per_step"].items()}
        if link is not None:
            line["link"] = link
        line["hip_runtime"] = hip_runtime()
        if write is not None:
            line["write_r1cs"] = write
        if flat is not None:
            line["flatten_dag"] = flat
        if tmpl is not None:
            line["templated"] = tmpl
        if lin is not None:
            line["linear1M"] = lin
        if o1 is not None:
            got1 = o1.pop("_arrays", None)
            if got1 is not None:
                import rsio
                ref1, ms1 = rsio.oracle_arrays(inp.c, rsio.flags("O1"), threads=args.cpu_threads or cpu_threads())
                o1["bit_exact"] = rsio.diff_output_arrays(got1, ref1) is None
                o1["cpu_oracle_ms"] = round(ms1, 1)
            line["o1"] = o1
        if weak is not None:
            line["weak_shards"] = weak
        if not args.no_cpu and world > 1:
            # N > 1: the oracle only as the checker of rank 0's view of the whole result (the CPU
            # baseline is an N = 1 field)
            import rsio
            ref, _ = rsio.oracle_arrays(inp.c, rsio.flags("O2"), threads=args.cpu_threads or cpu_threads())
            diff = rsio.diff_output_arrays(got, ref)
            line["cpu_baseline"] = None
            line["bit_exact"] = diff is None
            if diff is not None:
                line["bit_exact_diff"] = diff
        elif not args.no_cpu:
            threads = args.cpu_threads or cpu_threads()
            cb, ref, alg = cpu_baseline(M, inp, threads, args.cpu_j1_rows, args.seed, args.prime)
            line["cpu_baseline"] = cb
            # the whole-path roofline from the oracle's B_alg (implementation-independent: counted over
            # the canonical execution's logical operations, oracle/refcpu.cpp header); the device's own
            # in-kernel total stays beside it
            p = line["roofline"]["path"]
            p["alg_bytes_device_per_step"] = p.pop("alg_bytes_per_step")
            p["achieved_device"] = p.pop("achieved")
            p.pop("frac", None)
            p["alg_bytes_refcpu"] = alg["B_alg"]
            p["alg_terms_refcpu"] = {k: v for k, v in alg.items() if k != "B_alg"}
            ach = alg["B_alg"] / (ms_step / 1000.0) / 1e9
            p["achieved"] = round(ach, 2)
            p["frac"] = round(ach / HBM_PEAK_GBS, 5)
            p["device_over_refcpu"] = round(p["alg_bytes_device_per_step"] / max(alg["B_alg"], 1), 3)
            import rsio
            diff = rsio.diff_output_arrays(got, ref)
            line["bit_exact"] = diff is None
            if diff is not None:
                line["bit_exact_diff"] = diff
        else:
            line["cpu_baseline"] = None
            line["bit_exact"] = None
        print(json.dumps(line), flush=True)
    inp.free()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
