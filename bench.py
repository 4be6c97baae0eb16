"""bench.py -- constraints simplified/sec (--O2) on the 10M-constraint synthetic circuit.

One step = one full --O2 simplification (rs_engine_run): the Simplifier bundle already resident in
HBM -> simplified constraints + label->wire map resident in HBM.  N ranks (one process per GPU,
torch.distributed over RCCL) each own an independent shard of template instances (weak scaling;
the shards share no signal, so no exchange step is needed -- see DESIGN.md "Multi-GPU").

Prints ONE JSON line (rank 0) with the roofline of the dominant kernel (HIP events around it on
the library's own stream) and the CPU baseline (the canonical CPU oracle, oracle/refcpu.cpp, on a
bounded sample of the same workload, rank 0 only)."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "constraints simplified/sec (--O2) on 10M-constraint circuit; bit-exact .r1cs"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def cpu_baseline(rows: int, seed: int, threads: int, prime: str):
    """The canonical CPU oracle (oracle/refcpu.cpp) on the same synthetic circuit as rank 0 (or a
    smaller bounded sample when --cpu-rows is lower), on `threads` host threads."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import rsio
    import circom_cvm_amd as M
    inp = M.Input.synth(0, rows, seed, prime)
    t0 = time.time()
    _, ms = rsio.oracle_arrays(inp.c, rsio.flags("O2"), threads=threads)
    wall = time.time() - t0
    return {"value": round(inp.rows() / (ms / 1000.0), 1), "unit": "constraints/s", "cores": threads,
            "kind": "port",
            "sample": f"synth_mixed rows={inp.rows()} seed={seed} {prime} --O2 (the rank-0 workload), "
                      f"oracle/refcpu.cpp simplification() on {threads} threads: {ms / 1000.0:.1f} s "
                      f"({wall:.1f} s incl. output copy)"}


def shard_seed(seed: int, rank: int) -> int:
    """Rank r simplifies its own circuit shard: the synthetic generator seeded with seed + r."""
    return seed + rank


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


def sharded_one_circuit(M, dist, args, world, rank, local, fl, barrier):
    """The SAME 10M metric circuit on every rank, its clusters dealt to the ranks and the
    eliminated-signal map exchanged over RCCL (SURVEY 8(e), strong scaling).  Returns the max over
    ranks of ms/step and the exchange time, measured like the headline."""
    uid = share_comm_id(dist, rank, M.comm_unique_id)
    inp = M.Input.synth(0, args.rows, args.seed, args.prime)
    eng = M.Engine(local)
    eng.join_rccl(world, rank, uid)
    eng.load(inp.c)
    for _ in range(args.warmup):
        eng.run(fl)
    barrier()
    t0 = time.perf_counter()
    xms = 0.0
    for _ in range(args.steps):
        eng.run(fl)
        xms += eng.stats().exchange_ms
    barrier()
    dt = time.perf_counter() - t0
    dt, _ = reduce_over_ranks(dist, dt, 0, "cuda")
    xmax, _ = reduce_over_ranks(dist, xms, 0, "cuda")
    n = inp.rows()
    st = eng.stats()
    eng.close()
    return {"workload": f"synth_mixed rows={args.rows} prime={args.prime} seed={args.seed} --O2, ONE circuit "
                        f"on {world} ranks (clusters dealt by size, RCCL exchange of the eliminated-signal map)",
            "scaling": "strong", "constraints": n, "ms_per_step": round(dt * 1000.0 / args.steps, 3),
            "value": round(n * args.steps / dt, 1), "unit": "constraints/s",
            "exchange_ms_per_step": round(xmax / args.steps, 3), "exchange_bytes_per_rank": int(st.exchange_bytes)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--prime", default="bn128")
    ap.add_argument("--cpu-rows", type=int, default=10_000_000)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--mode", choices=("shards", "both"), default="both",
                    help="N>1: shards = the headline only (each rank its own circuit shard, weak "
                         "scaling); both = the headline + ONE circuit sharded over all ranks with the "
                         "RCCL exchange (strong scaling), as the extra object sharded_one_circuit")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist_
        torch.cuda.set_device(local)
        dist_.init_process_group("nccl", device_id=torch.device("cuda", local))
        dist = dist_

    import circom_cvm_amd as M

    # each rank: its own shard of instances (seed + rank), staged in HBM once
    inp = M.Input.synth(0, args.rows, shard_seed(args.seed, rank), args.prime)
    n_rows = inp.rows()
    eng = M.Engine(local)
    eng.load(inp.c)
    fl = M.make_flags("O2", device=local)
    for _ in range(args.warmup):
        eng.run(fl)

    def barrier():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    barrier()
    # device time + algorithmic bytes per kernel over the timed region (HIP events recorded by the
    # library on its own stream around each launch; bytes counted in-kernel, SURVEY 8(d) B_alg terms)
    K = {"k_big_main": [0.0, 0, 0], "k_big_finish": [0.0, 0, 0], "k_nl_fill": [0.0, 0, 0]}
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.run(fl)  # synchronous: returns after its stream has drained
        st = eng.stats()
        for k, ms, by, n in (("k_big_main", st.big_main_ms, st.big_main_bytes, st.big_launches),
                             ("k_big_finish", st.big_finish_ms, st.big_finish_bytes, st.big_launches),
                             ("k_nl_fill", st.apply_kernel_ms, st.apply_bytes, st.apply_kernel_launches)):
            K[k][0] += ms
            K[k][1] += by
            K[k][2] += n
    barrier()
    dt = time.perf_counter() - t0
    dt, total_rows = reduce_over_ranks(dist, dt, n_rows, "cuda")
    last = eng.stats()
    sharded = None
    if dist is not None and args.mode == "both":
        eng.close()  # free the headline engine's HBM before the second one
        sharded = sharded_one_circuit(M, dist, args, world, rank, local, fl, barrier)
    if rank == 0:
        ms_step = dt * 1000.0 / args.steps
        value = total_rows * args.steps / dt
        # dominant kernel: the largest device time over the timed region
        k_name = max(K, key=lambda k: K[k][0])
        k_ms, k_bytes, k_launch = K[k_name]
        per_launch_s = (k_ms / 1000.0) / max(k_launch, 1)
        per_launch_bytes = k_bytes / max(k_launch, 1)
        achieved = per_launch_bytes / per_launch_s / 1e9 if per_launch_s > 0 else 0.0
        traffic = None
        tf = os.environ.get("RS_PMC_TRAFFIC_BYTES")  # from profiles/ PMC pass, per launch
        if tf:
            traffic = float(tf)
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "constraints/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "u64x4 (F_p, 256-bit Montgomery)", "data": "synthetic",
            "config": {"workload": f"synth_mixed rows={args.rows}/rank prime={args.prime} "
                                   f"seed={args.seed}+rank --O2 (metric circuit, SURVEY 8(d))",
                       "constraints_per_rank": n_rows, "parallelism": f"shards{world}"},
            "roofline": {"bound": "hbm", "kernel": k_name, "achieved": round(achieved, 2),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": traffic, "launches_per_step": k_launch / args.steps,
                         "avg_launch_ms": round(per_launch_s * 1000.0, 4),
                         "alg_bytes_per_launch": int(per_launch_bytes)},
            "kernels_ms_per_step": {k: round(v[0] / args.steps, 3) for k, v in K.items()},
            "phases_ms": {k: round(getattr(last, k), 2) for k in
                          ("total_ms", "eq_ms", "cluster_ms", "elim_ms", "subst_ms", "final_ms")},
        }
        if sharded is not None:
            line["sharded_one_circuit"] = sharded
        if not args.no_cpu:
            line["cpu_baseline"] = cpu_baseline(args.cpu_rows, shard_seed(args.seed, 0), args.cpu_threads,
                                                args.prime)
        else:
            line["cpu_baseline"] = None
        print(json.dumps(line), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
