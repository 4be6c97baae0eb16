"""GPU parity at the benchmark sizes (BASELINE.json configs), array for array against the C++ oracle
(16 host threads), plus size-independent properties of the result."""
import numpy as np
import pytest

import rsio
import circom_cvm_amd as M

pytestmark = pytest.mark.gpu
_ENG = None


def engine():
    global _ENG
    if _ENG is None:
        _ENG = M.Engine(0)
    return _ENG


@pytest.fixture(scope="module", autouse=True)
def _release_engine():
    """The module's engine goes when its tests are done (later modules -- the 20 M sharded child --
    need the device memory)."""
    yield
    global _ENG
    if _ENG is not None:
        _ENG.close()
        _ENG = None


def gpu_arrays(inp, fl):
    e = engine()
    e.load(inp)
    e.run(fl)
    out = e.fetch()
    return rsio.output_arrays(out.c), e.stats()


def properties(x):
    """Invariants of any simplification result: no empty row, every signal in a row is a wire,
    wires are the order-preserving compaction 0..n_wires-1 of the kept labels."""
    l2w = x["l2w"]
    kept = l2w[l2w >= 0]
    assert len(kept) == x["n_wires"]
    assert np.array_equal(kept, np.arange(x["n_wires"]))
    nz = np.zeros(x["n_constraints"], bool)
    for nm in ("a", "b", "c"):
        ptr, col, _ = x[nm]
        if x["n_constraints"]:
            nz |= np.diff(ptr.astype(np.int64)) > 0
        assert np.all(l2w[col] >= 0), f"{nm}: removed signal in the output"
    assert nz.all(), "empty constraint in the output"


@pytest.mark.parametrize("kind,rows,prime,label", [
    (0, 10_000_000, "bn128", "metric circuit: synth_mixed 10M bn128 (BASELINE configs[4] shape, 1 GPU)"),
    (1, 1_000_000, "bn128", "configs[1]: synthetic 1M purely linear, BN254"),
    (0, 2_000_000, "bls12381", "configs[4] field: bls12381 mixed (2M shard)"),
    (2, 300_000, "bn128", "configs[3] shape: deep substitution chains"),
])
def test_full_size_parity(kind, rows, prime, label):
    inp = M.Input.synth(kind, rows, 42, prime)
    fl = rsio.flags("O2")
    got, st = gpu_arrays(inp.c, fl)
    properties(got)
    ref, _ = rsio.oracle_arrays(inp.c, fl, threads=16)
    assert rsio.diff_output_arrays(got, ref) is None, label


def test_repeat_runs_identical():
    """Engine reuse: the same input run twice gives identical arrays (no stale device state)."""
    inp = M.Input.synth(0, 1_000_000, 5)
    fl = rsio.flags("O2")
    a, _ = gpu_arrays(inp.c, fl)
    other = M.Input.synth(1, 200_000, 6)
    gpu_arrays(other.c, fl)
    b, _ = gpu_arrays(inp.c, fl)
    assert rsio.diff_output_arrays(a, b) is None
