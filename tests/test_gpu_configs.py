"""Every BASELINE.json config at full size on the HIP path, array for array against the C++ oracle
(16 host threads): the synthetic stand-ins of csrc/synth.cpp (circomlib / circom-ecdsa sources are not
available offline), through the host -> host entry point the benchmark times, plus every prime of
program_structure/src/utils/constants.rs:3-13 on the metric generator."""
import numpy as np
import pytest

import rsio
import circom_cvm_amd as M
from test_gpu_full import properties

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


def run_and_check(kind, rows, seed, prime, label):
    inp = M.Input.synth(kind, rows, seed, prime)
    pin = M.PinnedInput(inp.c)
    fl = rsio.flags("O2")
    got = rsio.output_arrays(engine().simplify(pin.c, fl))
    st = engine().stats()
    pin.free()
    properties(got)
    ref, _ = rsio.oracle_arrays(inp.c, fl, threads=16)
    assert rsio.diff_output_arrays(got, ref) is None, label
    return got, st


def test_config0_sha256_like():
    """configs[0]: circomlib sha256_2 stand-in (one compression, ~30k rows) -- and 10 of them."""
    run_and_check(4, 30_000, 1, "bn128", "sha-like 30k")
    run_and_check(4, 300_000, 5, "bn128", "sha-like 300k")


def test_config2_poseidon_merkle_4M():
    """configs[2]: Poseidon(16) 16-ary Merkle paths of depth 20, ~4M rows."""
    got, st = run_and_check(3, 4_000_000, 2, "bn128", "poseidon 4M")
    assert st.max_cluster >= 2000  # the partial rounds' process_4 clusters


def test_config3_deep_chains_1_5M():
    """configs[3]: ECDSA stand-in, 1.5M rows: composed right-hand sides of ~2,000 terms (they surface
    as the expanded A/B of the quadratic rows over chain signals) and 9 rounds."""
    got, st = run_and_check(2, 1_500_000, 3, "bn128", "chain 1.5M")
    ptr = got["a"][0].astype(np.int64)
    assert np.diff(ptr).max() >= 1000
    assert st.rounds >= 4


def test_config4_bls12381_20M():
    """configs[4] field and size: 20M-row metric generator over bls12381 on ONE GPU."""
    run_and_check(0, 20_000_000, 42, "bls12381", "bls12381 20M")


def test_config4_templated_10M():
    """configs[4] with SURVEY 8(d) config 5's replication: 64-row template instances (16 templates,
    coefficients shared by every instance) wired into log-normal chains; 2M and the full 10M."""
    got, st = run_and_check(5, 2_000_000, 7, "bn128", "templated 2M")
    assert st.max_cluster >= 350 and st.rounds >= 2
    got, st = run_and_check(5, 10_000_000, 42, "bn128", "templated 10M")
    assert st.max_cluster >= 5_000


@pytest.mark.parametrize("prime", ["grumpkin", "pallas", "vesta", "bls12377", "goldilocks", "secq256r1"])
def test_every_prime_1M(prime):
    run_and_check(0, 1_000_000, 9, prime, f"mixed 1M {prime}")
