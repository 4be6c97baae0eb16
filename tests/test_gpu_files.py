"""The drop-in seam from files: circom-simplify (GPU) on --O0 exports writes .r1cs/.sym byte-identical
to the oracle's writer; the one-shot C entry point and the golden fixtures through the GPU."""
import ctypes as C
import json
import os
import subprocess
import sys
import tempfile

import pytest

import rsio
import circom_cvm_amd as M
from circom_cvm_amd import abi

R = rsio.R
pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
EXE = os.path.join(ROOT, "circom_cvm_amd", "circom-simplify")
sys.path.insert(0, GOLD)
import make_golden as G  # noqa: E402


def run_cli(r1cs, sym, level, out_prefix, extra=()):
    args = [EXE, r1cs, sym, *level.split(), "-o", out_prefix, *extra]
    r = subprocess.run(args, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return r


@pytest.mark.parametrize("level", ["O1", "O2"])
def test_cli_docs_basic_bit_exact(level):
    with tempfile.TemporaryDirectory() as tmp:
        pre = os.path.join(tmp, "basic")
        run_cli(os.path.join(GOLD, "docs_basic_O0.r1cs"), os.path.join(GOLD, "docs_basic_O0.sym"),
                f"--{level}", pre)
        assert open(pre + ".r1cs", "rb").read() == open(os.path.join(GOLD, f"docs_basic_{level}.r1cs"), "rb").read()
        assert open(pre + ".sym").read() == open(os.path.join(GOLD, f"docs_basic_{level}.sym")).read()


@pytest.mark.parametrize("seed,prime,level", [(1, "bn128", "--O2"), (2, "bls12381", "--O2"),
                                              (3, "goldilocks", "--O1"), (4, "bn128", "--O2round 1"),
                                              (5, "secq256r1", "--O2")])
def test_cli_random_bit_exact(seed, prime, level):
    p = R.PRIMES[prime]
    sys_ = rsio.gen_system(100 + seed, p, n_sig=300, n_rows=260, big_cluster=400 if seed % 2 else 0)
    ident = R.Result(sys_.rows, {i: i for i in range(sys_.max_signal)}, sys_.n_priv_in)
    sym_lines = [(i, i, i % 3, f"main.s[{i}]") for i in range(1, sys_.max_signal)]
    lv = level.split()
    flags = G.flags_of("O1") if lv[0] == "--O1" else G.flags_of("O2", int(lv[1]) if len(lv) > 1 else None)
    res = R.simplification(sys_, flags)
    with tempfile.TemporaryDirectory() as tmp:
        r1 = os.path.join(tmp, "in.r1cs")
        sy = os.path.join(tmp, "in.sym")
        open(r1, "wb").write(R.result_to_r1cs(sys_, ident))
        open(sy, "w").write("".join(f"{a},{b},{c},{d}\n" for a, b, c, d in sym_lines))
        pre = os.path.join(tmp, "out")
        run_cli(r1, sy, level, pre)
        assert open(pre + ".r1cs", "rb").read() == R.result_to_r1cs(sys_, res)
        assert open(pre + ".sym").read() == R.result_to_sym(sym_lines, res)


def test_one_shot_entry_point():
    """rs_simplify: host input -> host output in one call (the entry point a Rust shim binds)."""
    sys_ = rsio.gen_system(55, R.PRIMES["bn128"], n_sig=200, n_rows=300, big_cluster=380)
    h = rsio.InputHolder(sys_)
    for lvl in ("O1", "O2"):
        out = C.POINTER(abi.RsOutput)()
        abi.check(abi.lib().rs_simplify(C.byref(h.inp), C.byref(rsio.flags(lvl)), C.byref(out)))
        try:
            got = rsio.output_to_py(out.contents)
        finally:
            abi.lib().rs_output_free(out)
        ref, _, _ = rsio.oracle_run(h.inp, rsio.flags(lvl))
        assert got == ref


@pytest.mark.parametrize("fname", sorted(f for f in os.listdir(GOLD) if f.startswith("oracle_")))
def test_golden_on_gpu(fname):
    with open(os.path.join(GOLD, fname)) as f:
        fx = json.load(f)
    sys_ = R.System(int(fx["p"]), fx["max_signal"], fx["n_pub_out"], fx["n_pub_in"], fx["n_priv_in"],
                    set(fx["forbidden"]), G.rows_from_json(fx["rows"]))
    h = rsio.InputHolder(sys_)
    eng = M.Engine(0)
    try:
        for ex in fx["expected"]:
            eng.load(h.inp)
            eng.run(rsio.flags(ex["level"], ex["rounds"], ex["old"]))
            out = eng.fetch()
            cons, sm, nw, npiw = rsio.output_to_py(out.c)
            assert G.result_to_json(R.Result(cons, sm, npiw)) == {
                k: ex[k] for k in ("constraints", "signal_map", "no_private_inputs_witness")}
    finally:
        eng.close()


@pytest.mark.parametrize("level", ["O1", "O2"])
def test_simplifier_mirror_docs(level):
    """Simplifier(...).simplify_constraints() -> ConstraintList, like constraint_list/src/lib.rs:131-202:
    json_constraints, r1cs and sym reproduce the reference docs' basic.circom outputs."""
    inp = M.Input.read_r1cs(os.path.join(GOLD, "docs_basic_O0.r1cs"))
    smp = M.Simplifier(inp, flag_s=(level == "O1"))
    cl = smp.simplify_constraints()
    assert cl.json_constraints() == G.DOCS["constraints"][level]
    with tempfile.TemporaryDirectory() as tmp:
        cl.r1cs(os.path.join(tmp, "o.r1cs"))
        cl.sym(os.path.join(GOLD, "docs_basic_O0.sym"), os.path.join(tmp, "o.sym"))
        assert open(os.path.join(tmp, "o.r1cs"), "rb").read() == open(os.path.join(GOLD, f"docs_basic_{level}.r1cs"), "rb").read()
        assert open(os.path.join(tmp, "o.sym")).read().splitlines() == G.DOCS["sym"][level]
    assert cl.no_wires() == len(cl.get_witness_as_vec())
