"""the device-built .r1cs (rs_engine_write_r1cs) is byte-identical to the host
writer rs_write_r1cs on the same result -- which test_abi.py pins to pyref's restatement of
r1cs_porting.rs:4-124 / r1cs_writer.rs:49-72 -- on random systems over several primes, the metric
circuit at full size, and a system with custom-gate sections."""
import ctypes as C
import dataclasses
import os
import struct
import tempfile

import pytest

import rsio
import circom_cvm_amd as M
from circom_cvm_amd import abi

pytestmark = pytest.mark.gpu
R = rsio.R


def host_bytes(path, inp, out, o0=None):
    if o0:
        abi.check(abi.lib().rs_write_r1cs_gates(path.encode(), C.byref(inp), C.byref(out), o0.encode()))
    else:
        abi.check(abi.lib().rs_write_r1cs(path.encode(), C.byref(inp), C.byref(out)))
    with open(path, "rb") as f:
        return f.read()


def device_bytes(eng, path, o0=None):
    ms = eng.write_r1cs(path, o0)
    assert ms > 0
    with open(path, "rb") as f:
        return f.read()


@pytest.mark.parametrize("prime", ["bn128", "bls12381", "goldilocks", "secq256r1"])
def test_device_writer_random(prime):
    p = R.PRIMES[prime]
    eng = M.Engine(0)
    with tempfile.TemporaryDirectory() as tmp:
        for seed in range(4):
            sys_ = rsio.gen_system(900 + seed, p, n_sig=900, n_rows=700, density=2.5)
            h = rsio.InputHolder(sys_, prime)
            for lvl in ("O1", "O2"):
                out = eng.simplify(h.inp, rsio.flags(lvl))
                a = host_bytes(os.path.join(tmp, "h.r1cs"), h.inp, out)
                b = device_bytes(eng, os.path.join(tmp, "d.r1cs"))
                assert a == b, (prime, seed, lvl)
    eng.close()


@pytest.mark.parametrize("kind,rows", [(0, 10_000_000), (2, 300_000), (3, 400_000)])
def test_device_writer_synth(kind, rows):
    inp = M.Input.synth(kind, rows, 7, "bn128")
    pin = M.PinnedInput(inp.c)
    eng = M.Engine(0)
    with tempfile.TemporaryDirectory() as tmp:
        out = eng.simplify(pin.c, rsio.flags("O2"))
        a = host_bytes(os.path.join(tmp, "h.r1cs"), pin.c, out)
        b = device_bytes(eng, os.path.join(tmp, "d.r1cs"))
        assert len(a) == len(b)
        assert a == b
    eng.close()
    pin.free()


def test_device_writer_custom_gates():
    sys_ = rsio.gen_system(57, R.PRIMES["bn128"], n_sig=80, n_rows=150)
    used = struct.pack("<I", 1) + b"CMul\x00" + struct.pack("<I", 1) + (7).to_bytes(32, "little")
    apps = [(0, [10, 11, 12]), (0, [40, 41, 12])]
    gsig = {x for _, sig in apps for x in sig}
    sys_ = dataclasses.replace(sys_, forbidden=sys_.forbidden | gsig, gates=(used, apps))
    ident = R.Result(sys_.rows, {i: i for i in range(sys_.max_signal)}, sys_.n_priv_in)
    eng = M.Engine(0)
    with tempfile.TemporaryDirectory() as tmp:
        o0 = os.path.join(tmp, "in.r1cs")
        with open(o0, "wb") as f:
            f.write(R.result_to_r1cs(sys_, ident))
        inp = M.Input.read_r1cs(o0)
        for lvl in ("O1", "O2"):
            out = eng.simplify(inp.c, rsio.flags(lvl))
            a = host_bytes(os.path.join(tmp, "h.r1cs"), inp.c, out, o0)
            b = device_bytes(eng, os.path.join(tmp, "d.r1cs"), o0)
            assert a == b
            assert b == R.result_to_r1cs(sys_, R.simplification(sys_, rsio.py_flags(rsio.flags(lvl))))
    eng.close()


def test_writer_host_fallback_same_bytes(monkeypatch):
    """Outputs past the device sort key's range (2^28 rows or 2^32 entries of a part) are written by
    the host writer over the fetched result; forced here (RS_WRITER_HOST), the bytes are the device
    writer's."""
    p = R.PRIMES["bn128"]
    eng = M.Engine(0)
    with tempfile.TemporaryDirectory() as tmp:
        sys_ = rsio.gen_system(977, p, n_sig=900, n_rows=700, density=2.5)
        h = rsio.InputHolder(sys_, "bn128")
        eng.simplify(h.inp, rsio.flags("O2"))
        a = device_bytes(eng, os.path.join(tmp, "d.r1cs"))
        monkeypatch.setenv("RS_WRITER_HOST", "1")
        b = device_bytes(eng, os.path.join(tmp, "h.r1cs"))
        assert a == b
    eng.close()
