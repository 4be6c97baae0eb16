"""Multi-process path of bench.py on CPU (gloo, world size 2): shard assignment, the max/sum
reduction the N-GPU line is computed from, and the unique-id rendezvous of the sharded
(one-circuit, RCCL exchange) line.  The exchange itself needs GPUs: tests/test_gpu_sharded.py runs
it with W engines on one device."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        import circom_cvm_amd as M
        inp = M.Input.synth(0, 3000, bench.shard_seed(42, rank))
        rows = inp.rows()
        dt, total = bench.reduce_over_ranks(dist, 1.0 + rank, rows, "cpu")
        g = [None] * world
        dist.all_gather_object(g, (rows, int(inp.c.max_signal)))
        # the RCCL rendezvous of the sharded line: rank 0's id reaches every rank unchanged
        uid = bench.share_comm_id(dist, rank, lambda: bytes(range(128)))
        q.put((rank, dt, total, g, uid))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_reduction_and_shards():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    rows = [g[0] for g in res[0][3]]
    for rank, dt, total, g, uid in res:
        assert dt == 2.0                      # max over ranks of the timed region
        assert total == sum(rows)             # whole-job constraints
        assert uid == bytes(range(128))       # rs_engine_join_rccl rendezvous id
    assert res[0][3] == res[1][3]
    # distinct shards (different seeds) of the same workload size
    assert all(r >= 3000 for r in rows)


def test_single_process_identity():
    import sys
    sys.path.insert(0, ROOT)
    import bench
    assert bench.reduce_over_ranks(None, 3.5, 10, "cpu") == (3.5, 10)
    assert bench.shard_seed(42, 3) == 45
