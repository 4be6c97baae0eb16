"""rs_engine_write_r1cs on the metric circuit's result: best of --reps writes into a temporary
directory (RS_PROF=1 prints the device build / D2H + writers split), and the file system's own bound
for a file of the same size written from host memory (no GPU): 1 and 4 pwrite threads in 32 MB chunks,
with and without fallocate, in the same directory and in /dev/shm (tmpfs)."""
import argparse
import os
import sys
import tempfile
import threading
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import circom_cvm_amd as M  # noqa: E402


def pinned_buffer(nbytes: int):
    """A page-locked buffer from the HIP runtime the library loaded (hipHostMalloc), as a memoryview."""
    import ctypes as C
    hip = C.CDLL("libamdhip64.so.7")
    p = C.c_void_p()
    if hip.hipHostMalloc(C.byref(p), C.c_size_t(nbytes), 0):
        raise OSError("hipHostMalloc failed")
    buf = (C.c_uint8 * nbytes).from_address(p.value)
    C.memset(p, 7, nbytes)
    return memoryview(buf).cast("B")


def fs_probe(dirname: str, size: int, threads: int, falloc: bool, reps: int = 3, pinned: bool = False) -> float:
    """GB/s of writing `size` bytes into a fresh file of `dirname` from a host buffer (best of reps);
    pinned: the source is page-locked memory from hipHostMalloc (the writer's staging buffers)."""
    chunk = 32 << 20
    mv = pinned_buffer(chunk) if pinned else memoryview(bytearray(os.urandom(1 << 20)) * 32)
    best = 0.0
    for _ in range(reps):
        path = os.path.join(dirname, "probe.bin")
        t0 = time.perf_counter()
        fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
        if falloc:
            os.posix_fallocate(fd, 0, size)
        else:
            os.ftruncate(fd, size)
        offs = list(range(0, size, chunk))

        def work(k):
            for o in offs[k::threads]:
                n = min(chunk, size - o)
                os.pwrite(fd, mv[:n], o)
        th = [threading.Thread(target=work, args=(k,)) for k in range(threads)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        os.close(fd)
        dt = time.perf_counter() - t0
        os.unlink(path)
        best = max(best, size / dt / 1e9)
    return best


ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=10_000_000)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--dir", default=None)
args = ap.parse_args()
inp = M.Input.synth(0, args.rows, 42)
pin = M.PinnedInput(inp.c)
eng = M.Engine(0)
fl = M.make_flags("O2")
eng.simplify(pin.c, fl)
best = None
with tempfile.TemporaryDirectory(dir=args.dir) as tmp:
    path = os.path.join(tmp, "w.r1cs")
    for _ in range(args.reps):
        t0 = time.perf_counter()
        eng.write_r1cs(path)
        dt = (time.perf_counter() - t0) * 1000
        best = dt if best is None else min(best, dt)
    size = os.path.getsize(path)
    os.unlink(path)
    print(f"write_r1cs best {best:.1f} ms, {size / 1e6:.0f} MB, {size / best / 1e6:.2f} GB/s", flush=True)
    for d in (tmp, "/dev/shm"):
        for th, fa, pn in ((1, False, False), (4, False, False), (4, True, False), (1, False, True), (4, True, True)):
            try:
                r = fs_probe(d, size, th, fa, pinned=pn)
                print(f"fs bound {d}: {th} writer(s){' + fallocate' if fa else ''}{' from pinned memory' if pn else ''}: "
                      f"{r:.2f} GB/s", flush=True)
            except OSError as e:
                print(f"fs bound {d}: {e}", flush=True)
eng.close()
