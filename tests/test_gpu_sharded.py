"""GPU parity of the SHARDED path: one circuit, W ranks, clusters dealt by size, the
eliminated-signal map exchanged after every round.  On the one-GPU box the ranks are W engines on
device 0 in W threads of this process, joined to an in-process group (host-staged collectives); the
RCCL transport is the same code path behind another Comm (covered at world 1 here, at world N by the
driver's multi-GPU bench).  Every rank's output must equal the single-GPU oracle's, bit for bit."""
import threading

import pytest

import rsio
import circom_cvm_amd as M

R = rsio.R
pytestmark = pytest.mark.gpu

_GROUPS = {}


def release_groups():
    """Closes the cached in-process groups' engines (their device memory)."""
    for _, engs in _GROUPS.values():
        for e in engs:
            e.close()
    _GROUPS.clear()


@pytest.fixture(scope="module", autouse=True)
def _release_groups():
    yield
    release_groups()


def group(world):
    """W engines on device 0 joined to one in-process group (reused across tests)."""
    if world not in _GROUPS:
        g = M.Group(world)
        engs = [M.Engine(0) for _ in range(world)]
        for r, e in enumerate(engs):
            e.join_group(g, r)
        _GROUPS[world] = (g, engs)
    return _GROUPS[world][1]


def sharded_run(inp, fl, world, arrays=False):
    engs = group(world)
    outs, errs = [None] * world, [None] * world

    def work(r):
        try:
            engs[r].load(inp)
            engs[r].run(fl)
            out = engs[r].fetch()
            outs[r] = (rsio.output_arrays(out.c) if arrays else rsio.output_to_py(out.c), engs[r].stats())
        except Exception as ex:  # noqa: BLE001 -- reported below
            errs[r] = ex

    th = [threading.Thread(target=work, args=(r,), daemon=True) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=240)
        assert not t.is_alive(), "sharded run hung"
    for e in errs:
        if e is not None:
            raise e
    return outs


def check(inp, fl, world, threads=1):
    ref, _, _ = rsio.oracle_run(inp, fl, threads)
    outs = sharded_run(inp, fl, world)
    for r, (got, st) in enumerate(outs):
        if got != ref:
            diff = rsio.same_result(R.Result(ref[0], ref[1], ref[3]), got)
            raise AssertionError(f"rank {r}/{world} != oracle: {diff}")
        assert st.world == world
    return outs


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("p", [257, R.PRIMES["bn128"], R.PRIMES["goldilocks"]])
def test_sharded_random_small(world, p):
    for seed in range(12):
        sys_ = rsio.gen_system(seed, p, n_sig=40 + seed % 50, n_rows=60 + seed % 80)
        h = rsio.InputHolder(sys_)
        for lvl, rd in (("O1", None), ("O2", None), ("O2", 1), ("O2", 2)):
            check(h.inp, rsio.flags(lvl, rd), world)


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_process4(world):
    p = R.PRIMES["bn128"]
    for seed in range(4):
        sys_ = rsio.gen_system(2000 + seed, p, n_sig=300, n_rows=250, big_cluster=600 + 40 * seed)
        h = rsio.InputHolder(sys_)
        for lvl, rd, old in (("O2", None, False), ("O2", None, True), ("O2", 2, False)):
            check(h.inp, rsio.flags(lvl, rd, old), world, threads=4)


@pytest.mark.parametrize("kind,rows,world", [(0, 200_000, 4), (0, 300_000, 3), (1, 100_000, 2), (2, 50_000, 3)])
def test_sharded_synth_arrays(kind, rows, world):
    """Synthetic workloads (mixed / purely linear / deep chains) array for array on every rank."""
    inp = M.Input.synth(kind, rows, 42)
    fl = rsio.flags("O2")
    ref, _ = rsio.oracle_arrays(inp.c, fl, threads=8)
    outs = sharded_run(inp.c, fl, world, arrays=True)
    for r, (got, st) in enumerate(outs):
        assert rsio.diff_output_arrays(got, ref) is None, f"rank {r}"
        assert st.world == world and st.exchange_bytes > 0
    assert len({st.n_substitutions for _, st in outs}) == 1  # every rank holds the whole map


@pytest.mark.parametrize("kind,rows,prime,world", [(2, 1_500_000, "bn128", 4), (0, 2_000_000, "bls12381", 8)])
def test_sharded_baseline_configs(kind, rows, prime, world):
    """The sharded forms BASELINE.json names: configs[3] (the ECDSA stand-in, deep chains, 1.5 M rows)
    dealt over 4 ranks and configs[4]'s --prime bls12381 over 8 ranks (2 M rows of the mixed
    circuit), every rank array for array equal to the single-GPU oracle."""
    inp = M.Input.synth(kind, rows, 3, prime)
    fl = rsio.flags("O2")
    ref, _ = rsio.oracle_arrays(inp.c, fl, threads=16)
    outs = sharded_run(inp.c, fl, world, arrays=True)
    for r, (got, st) in enumerate(outs):
        assert rsio.diff_output_arrays(got, ref) is None, f"rank {r}/{world}"
        assert st.world == world and st.exchange_bytes > 0
    assert len({st.n_substitutions for _, st in outs}) == 1


def test_simplify_multi_one_device_listed_twice():
    """rs_simplify_multi (the one-shot entry point) with device 0 listed twice: in-process transport."""
    sys_ = rsio.gen_system(77, R.PRIMES["bn128"], n_sig=300, n_rows=250, big_cluster=700)
    h = rsio.InputHolder(sys_)
    fl = rsio.flags("O2")
    out = M.simplify_multi(h.inp, fl, [0, 0])
    ref, _, _ = rsio.oracle_run(h.inp, fl)
    assert rsio.output_to_py(out.c) == ref


def test_rccl_world1_join():
    """The RCCL transport's plumbing on one GPU: unique id, communicator init, a run at world 1."""
    e = M.Engine(0)
    e.join_rccl(1, 0, M.comm_unique_id())
    inp = M.Input.synth(0, 20_000, 9)
    fl = rsio.flags("O2")
    e.load(inp.c)
    e.run(fl)
    out = e.fetch()  # keep the owner alive while its arrays are read
    got = rsio.output_arrays(out.c)
    ref, _ = rsio.oracle_arrays(inp.c, fl, threads=4)
    assert rsio.diff_output_arrays(got, ref) is None
    assert e.stats().world == 1
    e.close()


# ---------------------------------------------------------------- host -> host, split PCIe legs
def sharded_simplify(inp, fl, world, engs=None, arrays=True, reps=1):
    """rs_engine_simplify on every rank at once: each rank uploads its share of the input (the ranks
    complete the blocks over the group's allgathervs) and copies its share of the result into the
    group's shared host region; every rank's returned view must be the whole result."""
    engs = engs or group(world)
    outs, errs = [None] * world, [None] * world

    def work(r):
        try:
            for _ in range(reps):
                out = engs[r].simplify(inp, fl)
            outs[r] = (rsio.output_arrays(out) if arrays else rsio.output_to_py(out), engs[r].stats())
        except Exception as ex:  # noqa: BLE001 -- reported below
            errs[r] = ex

    th = [threading.Thread(target=work, args=(r,), daemon=True) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=280)
        assert not t.is_alive(), "sharded simplify hung"
    for e in errs:
        if e is not None:
            raise e
    return outs


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_hosthost_random_small(world):
    """Split input / output legs on small random systems (every flag level, two primes): each rank's
    view equals the single-GPU oracle's result."""
    for p in (257, R.PRIMES["bn128"]):
        for seed in range(8):
            sys_ = rsio.gen_system(300 + seed, p, n_sig=60 + seed % 40, n_rows=90 + seed % 60)
            h = rsio.InputHolder(sys_)
            for lvl, rd in (("O1", None), ("O2", None), ("O2", 1)):
                fl = rsio.flags(lvl, rd)
                ref, _, _ = rsio.oracle_run(h.inp, fl)
                for r, (got, st) in enumerate(sharded_simplify(h.inp, fl, world, arrays=False)):
                    if got != ref:
                        raise AssertionError(f"rank {r}/{world} {lvl}/{rd}: {rsio.same_result(R.Result(ref[0], ref[1], ref[3]), got)}")


@pytest.mark.parametrize("kind,rows,world", [(0, 300_000, 2), (0, 400_000, 4), (2, 60_000, 3), (1, 100_000, 4), (5, 200_000, 2),
                                             (0, 2_000_000, 8)])
def test_sharded_hosthost_synth_arrays(kind, rows, world):
    """Synthetic workloads host -> host over 2-4 ranks, array for array on every rank, three calls on
    the same engines (the shared region is reused and grows as needed)."""
    inp = M.Input.synth(kind, rows, 42)
    fl = rsio.flags("O2")
    ref, _ = rsio.oracle_arrays(inp.c, fl, threads=8)
    for r, (got, st) in enumerate(sharded_simplify(inp.c, fl, world, reps=3)):
        assert rsio.diff_output_arrays(got, ref) is None, f"rank {r}/{world}"
        assert st.world == world


def _run_expect_fail(engs, inp, fl, mode):
    """Every rank runs `mode` ('simplify' or 'load+run') on its own input; returns the per-rank
    exception (None on success).  A hang fails the test."""
    world = len(engs)
    errs = [None] * world

    def work(r):
        try:
            if mode == "simplify":
                engs[r].simplify(inp[r], fl[r])
            else:
                engs[r].load(inp[r])
                engs[r].run(fl[r])
        except Exception as ex:  # noqa: BLE001 -- returned
            errs[r] = ex

    th = [threading.Thread(target=work, args=(r,), daemon=True) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
        assert not t.is_alive(), "a rank hung after another rank's failure"
    return errs


def _fresh_group(world):
    g = M.Group(world)
    engs = [M.Engine(0) for _ in range(world)]
    for r, e in enumerate(engs):
        e.join_group(g, r)
    return g, engs


def test_group_survives_rejected_input():
    """a failure is scoped to the call it happened in.  An input every rank rejects (a key
    past max_signal, caught by the device checks) fails the call on every rank; the same persistent
    in-process group then runs a valid input host -> host and load + run, equal to the oracle."""
    world = 2
    g, engs = _fresh_group(world)
    try:
        p = R.PRIMES["bn128"]
        good = rsio.InputHolder(rsio.gen_system(91, p, n_sig=80, n_rows=120))
        bad = rsio.InputHolder(rsio.gen_system(91, p, n_sig=80, n_rows=120))
        bad.blocks[2].col[0] = bad.inp.max_signal + 7  # the first linear row's first key: out of range
        fl = rsio.flags("O2")
        for mode in ("simplify", "load+run"):
            errs = _run_expect_fail(engs, [bad.inp] * world, [fl] * world, mode)
            assert all(isinstance(e, M.RsError) for e in errs), errs
        ref, _, _ = rsio.oracle_run(good.inp, fl)
        for _ in range(2):
            for r, (got, _st) in enumerate(sharded_simplify(good.inp, fl, world, engs=engs, arrays=False)):
                assert got == ref, f"rank {r} after the rejected input"
        outs = [None] * world

        def work(r):
            engs[r].load(good.inp)
            engs[r].run(fl)
            o = engs[r].fetch()
            outs[r] = rsio.output_to_py(o.c)
        th = [threading.Thread(target=work, args=(r,), daemon=True) for r in range(world)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=120)
            assert not t.is_alive()
        assert all(o == ref for o in outs)
    finally:
        for e in engs:
            e.close()


def test_one_rank_fails_others_released():
    """when ONE rank's run fails mid-way (an injected fault at the start of its first
    elimination round, after the run's first collectives), the other ranks of the in-process group
    leave their collectives with RS_E_RCCL instead of waiting forever -- for load + run and for host ->
    host -- and the same group then runs valid calls equal to the oracle."""
    world = 3
    g, engs = _fresh_group(world)
    try:
        p = R.PRIMES["bn128"]
        good = rsio.InputHolder(rsio.gen_system(92, p, n_sig=300, n_rows=250, big_cluster=700))
        fl = rsio.flags("O2")
        ref, _, _ = rsio.oracle_run(good.inp, fl)
        for mode in ("load+run", "simplify"):
            engs[2].inject_fault(1)
            errs = _run_expect_fail(engs, [good.inp] * world, [fl] * world, mode)
            assert isinstance(errs[2], M.RsError) and errs[2].code == -5, errs  # RS_E_INTERNAL: the fault
            for r in range(2):
                assert isinstance(errs[r], M.RsError) and errs[r].code == -4, errs  # RS_E_RCCL: released
            for r, (got, _st) in enumerate(sharded_simplify(good.inp, fl, world, engs=engs, arrays=False)):
                assert got == ref, f"rank {r} after the fault ({mode})"
    finally:
        for e in engs:
            e.close()


def _run_20m(world):
    """The body of test_sharded_hosthost_bls12381_20m_world{4,8}, run in a child process (python
    tests/test_gpu_sharded.py 20m WORLD): its engines each hold the whole 20 M-row problem (~36 GB of
    device memory at world 1), which leaves no room for the engines the earlier tests of this process
    keep; eight of them fit the card's 309 GB."""
    import sys
    import time
    t0 = time.time()

    def say(what):  # progress (a quiet minute reads as a hang on the GPU box)
        print(f"[20M world {world}] {what} at {time.time() - t0:.0f} s", file=sys.stderr, flush=True)

    def tick():
        while True:
            time.sleep(30)
            say("still running")
    threading.Thread(target=tick, daemon=True).start()
    inp = M.Input.synth(0, 20_000_000, 42, "bls12381")
    say("input generated")
    pin = M.PinnedInput(inp.c)
    fl = rsio.flags("O2")
    g = M.Group(world)
    engs = [M.Engine(0) for _ in range(world)]
    try:
        for r, e in enumerate(engs):
            e.join_group(g, r)
        outs = sharded_simplify(pin.c, fl, world, engs=engs)
        say("sharded run done")
        ref, _ = rsio.oracle_arrays(inp.c, fl, threads=16)
        say("oracle done")
        for r, (got, st) in enumerate(outs):
            assert rsio.diff_output_arrays(got, ref) is None, f"rank {r}/{world}"
            assert st.world == world and st.exchange_bytes > 0
    finally:
        for e in engs:
            e.close()
        pin.free()
    say("arrays equal on every rank")


@pytest.mark.parametrize("world", [4, 8])
def test_sharded_hosthost_bls12381_20m(world):
    """BASELINE configs[4] at its stated size: --prime bls12381, the 20 M-row mixed circuit, ONE circuit
    over 4 and 8 ranks host -> host (split upload, sharded elimination with the exchange, split result
    copy), every rank array for array equal to the single-GPU oracle.  In one child process on one GPU
    (the engines and an in-process group made for it)."""
    import os
    import subprocess
    import sys
    release_groups()
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "20m", str(world)], stdout=sys.__stderr__,
                       stderr=sys.__stderr__, timeout=290, cwd=os.path.dirname(os.path.abspath(__file__)))
    assert r.returncode == 0, f"child exited with {r.returncode}"


if __name__ == "__main__":
    import sys
    if sys.argv[1:2] == ["20m"]:
        _run_20m(int(sys.argv[2]) if len(sys.argv) > 2 else 4)


@pytest.mark.parametrize("kind,rows,world", [(0, 300_000, 2), (5, 200_000, 2), (2, 60_000, 3)])
def test_two_process_host_transport(kind, rows, world):
    """the multi-process path -- one process per rank, the shared result region created by
    rank 0 as a POSIX shm object, mapped and hipHostRegister'ed by every process, each rank's share of
    the result streamed into it -- run for real on one GPU: `world` processes on device 0 joined by the
    host transport (rs_engine_join_host; RCCL refuses two ranks on one device, so its collectives go
    through shared memory), host -> host three times and load/run/fetch once, every rank's view equal to
    the oracle's."""
    import os
    import subprocess
    import sys
    child = os.path.join(os.path.dirname(os.path.abspath(__file__)), "hostcomm_child.py")
    tag = f"t{os.getpid()}_{kind}_{rows}_{world}"
    procs = [subprocess.Popen([sys.executable, "-u", child, str(world), str(r), tag, str(kind), str(rows), "3"],
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in range(world)]
    outs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=240)
            outs.append(out)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for r, (p, out) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, f"rank {r} exited {p.returncode}:\n{out[-3000:]}"
        assert f"rank {r} ok" in out


def test_sharded_engine_writes_r1cs():
    """bench.py's N > 1 line has rank 0 write its result with the device writer
    (rs_engine_write_r1cs) after a sharded host -> host call: on every rank of a sharded group the
    file is byte-identical to the host writer's over the same engine's (whole, shared) result."""
    import ctypes as C
    import os
    import tempfile

    from circom_cvm_amd import abi

    world = 2
    inp = M.Input.synth(0, 300_000, 42)
    fl = rsio.flags("O2")
    engs = group(world)
    outs, errs = [None] * world, [None] * world

    def work(r):
        try:
            outs[r] = engs[r].simplify(inp.c, fl)
        except Exception as ex:  # noqa: BLE001 -- reported below
            errs[r] = ex

    th = [threading.Thread(target=work, args=(r,), daemon=True) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=280)
        assert not t.is_alive(), "sharded simplify hung"
    for e in errs:
        if e is not None:
            raise e
    with tempfile.TemporaryDirectory() as tmp:
        ph, pd = os.path.join(tmp, "h.r1cs"), os.path.join(tmp, "d.r1cs")
        for r in range(world):
            abi.check(abi.lib().rs_write_r1cs(ph.encode(), C.byref(inp.c), C.byref(outs[r])))
            assert engs[r].write_r1cs(pd) > 0
            with open(ph, "rb") as f:
                a = f.read()
            with open(pd, "rb") as f:
                b = f.read()
            assert len(a) == len(b), f"rank {r}"
            assert a == b, f"rank {r}"
