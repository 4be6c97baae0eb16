"""GPU parity of the flag surface around the path: the --simplification_substitution log
(constraint_simplification.rs:9-17, logged at :249, :271 and :320 of every round) and the --json
constraints file (json_porting.rs:36-48) of the device path, against the literal Python oracle
(oracle/pyref.py keeps the reference's `to` maps exactly, zero-valued keys included) and the
reference docs' exact file texts (tests/test_abi.py DOCS_*_TEXT)."""
import os
import subprocess
import tempfile

import pytest

import rsio
import circom_cvm_amd as M
from test_abi import DOCS_JSON_TEXT, DOCS_SUBS_TEXT
import test_gpu_sharded as SH

R = rsio.R
pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
EXE = os.path.join(ROOT, "circom_cvm_amd", "circom-simplify")

_ENG = None


def engine():
    global _ENG
    if _ENG is None:
        _ENG = M.Engine(0)
    return _ENG


def gpu_log(inp, fl):
    e = engine()
    e.load(inp)
    e.run(fl)
    out = e.fetch()
    return rsio.output_log(out.c), rsio.output_to_py(out.c)


def first_diff(got, ref):
    if len(got) != len(ref):
        return f"{len(got)} entries vs {len(ref)}"
    for i, (x, y) in enumerate(zip(got, ref)):
        if x != y:
            return f"entry {i}: {x} vs {y}"
    return None


def check_log(sys_, fl):
    h = rsio.InputHolder(sys_)
    got, out = gpu_log(h.inp, fl)
    res = R.simplification(sys_, rsio.py_flags(fl), want_log=True)
    ref = rsio.pyref_log(res.log)
    d = first_diff(got, ref)
    assert d is None, f"log differs: {d}"
    assert rsio.same_result(res, out) is None  # the log flag does not perturb the result
    return len(got)


@pytest.mark.parametrize("p", [257, 97, R.PRIMES["bn128"], R.PRIMES["goldilocks"]])
def test_log_random_small(p):
    n = 0
    for seed in range(12):
        sys_ = rsio.gen_system(300 + seed, p, n_sig=40 + seed % 50, n_rows=60 + seed % 80)
        for lvl, rd in (("O1", None), ("O2", None), ("O2", 1), ("O2", 2)):
            n += check_log(sys_, rsio.flags(lvl, rd, log=True))
    assert n > 0


@pytest.mark.parametrize("p", [257, R.PRIMES["bls12381"]])
def test_log_process4(p):
    for seed in range(2):
        sys_ = rsio.gen_system(3000 + seed, p, n_sig=300, n_rows=250, big_cluster=600 + 40 * seed)
        for lvl, rd, old in (("O2", None, False), ("O2", None, True), ("O2", 2, False)):
            check_log(sys_, rsio.flags(lvl, rd, old, log=True))


def test_log_off_is_empty():
    sys_ = rsio.gen_system(5, 257, n_sig=60, n_rows=90)
    h = rsio.InputHolder(sys_)  # keeps the arrays behind the RsInput alive
    got, _ = gpu_log(h.inp, rsio.flags("O2"))
    assert got == []


def test_log_sharded_world2():
    """The sharded path logs the same stream on every rank (cluster order, not rank order)."""
    sys_ = rsio.gen_system(3100, R.PRIMES["bn128"], n_sig=300, n_rows=250, big_cluster=620)
    h = rsio.InputHolder(sys_)
    fl = rsio.flags("O2", log=True)
    ref = rsio.pyref_log(R.simplification(sys_, rsio.py_flags(fl), want_log=True).log)
    engs = SH.group(2)
    import threading
    logs = [None, None]

    def work(r):
        engs[r].load(h.inp)
        engs[r].run(fl)
        out = engs[r].fetch()  # owns the rs_output while it is read
        logs[r] = rsio.output_log(out.c)

    th = [threading.Thread(target=work, args=(r,), daemon=True) for r in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=240)
        assert not t.is_alive()
    for r in range(2):
        assert first_diff(logs[r], ref) is None


@pytest.mark.parametrize("level", ["O1", "O2"])
def test_cli_json_outputs_docs(level):
    """circom-simplify --json --simplification_substitution on the docs circuit writes the docs' texts."""
    with tempfile.TemporaryDirectory() as tmp:
        pre = os.path.join(tmp, "basic")
        r = subprocess.run([EXE, os.path.join(GOLD, "docs_basic_O0.r1cs"), os.path.join(GOLD, "docs_basic_O0.sym"),
                            f"--{level}", "--json", "--simplification_substitution", "-o", pre],
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        assert open(pre + "_constraints.json").read() == DOCS_JSON_TEXT[level]
        assert open(pre + "_substitutions.json").read() == DOCS_SUBS_TEXT[level]


def test_cli_json_random():
    """--json / --simplification_substitution through the CLI on a random bls12381 system with a
    process_4 cluster and two rounds."""
    sys_ = rsio.gen_system(3200, R.PRIMES["bls12381"], n_sig=300, n_rows=260, big_cluster=420)
    ident = R.Result(sys_.rows, {i: i for i in range(sys_.max_signal)}, sys_.n_priv_in)
    res = R.simplification(sys_, R.Flags(flag_s=False), want_log=True)
    with tempfile.TemporaryDirectory() as tmp:
        r1 = os.path.join(tmp, "in.r1cs")
        open(r1, "wb").write(R.result_to_r1cs(sys_, ident))
        pre = os.path.join(tmp, "out")
        r = subprocess.run([EXE, r1, "--O2", "--json", "--simplification_substitution", "-o", pre],
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        assert open(pre + "_constraints.json").read() == rsio.constraints_json_text(res.constraints, res.signal_map)
        assert open(pre + "_substitutions.json").read() == rsio.substitutions_json_text(rsio.pyref_log(res.log))


def test_simplifier_mirror_log():
    """Simplifier(port_substitution=True).simplify_constraints().substitutions() (the mirror API)."""
    inp = M.Input.read_r1cs(os.path.join(GOLD, "docs_basic_O0.r1cs"))
    cl = M.Simplifier(inp, port_substitution=True).simplify_constraints()
    assert [(f, {k: str(v) for k, v in to.items()}) for f, to in cl.substitutions()] == [
        (5, {2: "1"}), (4, {1: "1"}), (6, {0: "1", 2: "2", 3: "1"})]
