"""CPU tests of the oracle: the literal Python restatement (oracle/pyref.py) pinned against the
reference's own known answers, and the canonical C++ restatement (oracle/refcpu.cpp, the checker the
GPU parity tests use) cross-checked against it.  No GPU needed."""
import json
import os
import random
import sys

import pytest

import rsio

R = rsio.R
HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
sys.path.insert(0, GOLD)
import make_golden as G  # noqa: E402

LEVELS = {"O1": ("O1", None), "O2": ("O2", None), "O2r1": ("O2", 1), "O2r2": ("O2", 2)}


# ------------------------------------------------------------------ reference unit tests (F_257)
def test_modulus_of_negative():
    """modular_arithmetic.rs:224-229 (mod_check): (-8) mod 5 == 2."""
    assert R.modulus(-8, 5) == 2


def test_clear_signal_f257():
    """algebra.rs:1423-1454: x + y + 3 = 0, clear x  =>  x = 256*y + 254 over F_257."""
    p = 257
    sub = R.clear_signal({1: 1, 2: 1, 0: 3}, 1, p)
    assert sub[2] == R.m_sub(p, 1, p) == 256
    assert sub[0] == 254


def test_apply_substitution_f257():
    """algebra.rs:1456-1492: (x + y + 4 = 0)[x := 2y + 3]  =>  3y + 7 = 0 over F_257.

    The reference test asserts `constraint.a.is_empty()`, but raw_substitution (algebra.rs:1279-1294)
    first calls initialize_hashmap_for_expression, which inserts {0: 0} into the empty A and B.  The
    restatement follows the code; on the simplification path every apply_substitution is followed by
    fix_constraint, whose remove_zero_value_coefficients drops that entry, so the observable rows are
    the same either way (checked below)."""
    p = 257
    con = R.Con({}, {}, {1: 1, 2: 1, 0: 4})
    sub = R.sub_new(1, R.AE.linear({2: 2, 0: 3}))
    R.apply_substitution(con, sub, p)
    assert con.a == {0: 0} and con.b == {0: 0}
    assert con.c[2] == 3 and con.c[0] == 7 and 1 not in con.c
    R.fix_constraint(con, p)
    assert con.a == {} and con.b == {} and con.c == {2: 3, 0: 7}


def test_constraint_offset_semantics():
    """algebra.rs:1401-1421: apply_offset shifts every signal but the constant -- the DAG numbering
    the --O0 input already carries (rows of basic.circom use global ids)."""
    sys_ = G.docs_system()
    assert all(k < sys_.max_signal for c in sys_.rows for m in (c.a, c.b, c.c) for k in m)


# ------------------------------------------------------------------ field arithmetic of refcpu
def _limbs(v):
    return [(v >> (64 * i)) & ((1 << 64) - 1) for i in range(4)]


def _field_op(p, op, a, b):
    lib = rsio.oracle_lib()
    T = rsio.C.c_uint64 * 4
    r = T()
    lib.refcpu_field_op(T(*_limbs(p)), op, T(*_limbs(a)), T(*_limbs(b)), r)
    return sum(int(r[i]) << (64 * i) for i in range(4))


@pytest.mark.parametrize("name", sorted(R.PRIMES) + ["f257", "f97"])
def test_refcpu_field_ops(name):
    """Montgomery 4x64 arithmetic of the C++ oracle == Python big ints (add, sub, mul, inverse)."""
    p = {"f257": 257, "f97": 97}.get(name) or R.PRIMES[name]
    rng = random.Random(p & 0xffff)
    vals = [0, 1, 2, p - 1, p - 2] + [rng.randrange(p) for _ in range(40)]
    for a in vals:
        b = rng.randrange(p)
        assert _field_op(p, 0, a, b) == (a + b) % p
        assert _field_op(p, 1, a, b) == (a - b) % p
        assert _field_op(p, 2, a, b) == (a * b) % p
        if a:
            assert _field_op(p, 3, 1, a) == pow(a, -1, p)
            assert _field_op(p, 3, b, a) == b * pow(a, -1, p) % p
        assert _field_op(p, 4, a, 0) == (-a) % p


def test_device_field_host_build(tmp_path):
    """The device field arithmetic (csrc/field.hpp, the functions every kernel inlines) built for the
    host and checked against Python big ints on all 8 primes and F_257 / F_97: add, sub, Montgomery
    product, square and Fermat inverse.  Covers the 256-bit radix-2^29 path and the one-word path
    that primes below 2^64 (goldilocks, F_257, F_97) take (SURVEY §7 layer 1), which shares the
    256-bit path's Montgomery form (checked: fmul256 on the same residues gives the same product)."""
    import shutil
    import subprocess
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("no hipcc")
    root = os.path.dirname(HERE)
    exe = str(tmp_path / "field_host_check")
    subprocess.check_call([hipcc, "-O2", "-std=c++17", "-I", os.path.join(root, "circom_cvm_amd", "csrc"),
                           os.path.join(HERE, "field_host_check.cpp"), "-o", exe])
    cases = []
    for p in sorted(R.PRIMES.values()) + [257, 97]:
        rng = random.Random(p & 0xffffff)
        vals = [0, 1, 2, p - 1, p - 2] + [rng.randrange(p) for _ in range(60)]
        cases += [(p, a, rng.choice([rng.randrange(p), p - 1, 0, 1])) for a in vals]
    stdin = "".join(f"{p:x} {a:x} {b:x}\n" for p, a, b in cases)
    out = subprocess.run([exe], input=stdin, capture_output=True, text=True, check=True).stdout.split("\n")
    for (p, a, b), line in zip(cases, out):
        s, d, m, inv, sq, m256 = (int(x, 16) for x in line.split())
        assert (s, d, m, sq, m256) == ((a + b) % p, (a - b) % p, a * b % p, a * a % p, a * b % p), (p, a, b)
        assert inv == (pow(a, -1, p) if a else 0), (p, a)


# ------------------------------------------------------------------ docs known answers
def test_docs_constraints_json():
    """constraints-json.md: basic.circom at --O1 and --O2 (witness numbering)."""
    sys_ = G.docs_system()
    for lvl in ("O1", "O2"):
        res = R.simplification(sys_, G.flags_of(lvl))
        assert R.to_json_constraints(res.constraints, res.signal_map) == G.DOCS["constraints"][lvl]


def test_docs_sym():
    """sym.md: the witness column at --O1 and --O2."""
    sys_ = G.docs_system()
    lines = [tuple(int(x) if i < 3 else x for i, x in enumerate(l.split(",", 3))) for l in G.DOCS["sym_o0"]]
    for lvl in ("O1", "O2"):
        res = R.simplification(sys_, G.flags_of(lvl))
        assert R.result_to_sym(lines, res).splitlines() == G.DOCS["sym"][lvl]


def test_docs_substitution_log():
    """simplification-json.md: the substitutions at --O1 and --O2."""
    sys_ = G.docs_system()
    for lvl in ("O1", "O2"):
        res = R.simplification(sys_, G.flags_of(lvl), want_log=True)
        got = {str(s.frm): {str(k): str(v) for k, v in sorted(s.to.items()) if v} for s in res.log}
        assert got == G.DOCS["substitutions"][lvl]


def test_docs_files_match_fixtures():
    """The committed --O1/--O2 .r1cs/.sym of basic.circom are what the oracle writes today."""
    sys_ = G.docs_system()
    lines = [tuple(int(x) if i < 3 else x for i, x in enumerate(l.split(",", 3))) for l in G.DOCS["sym_o0"]]
    for lvl in ("O1", "O2"):
        res = R.simplification(sys_, G.flags_of(lvl))
        with open(os.path.join(GOLD, f"docs_basic_{lvl}.r1cs"), "rb") as f:
            assert f.read() == R.result_to_r1cs(sys_, res)
        with open(os.path.join(GOLD, f"docs_basic_{lvl}.sym")) as f:
            assert f.read() == R.result_to_sym(lines, res)


def test_r1cs_reader_roundtrip():
    with open(os.path.join(GOLD, "docs_basic_O0.r1cs"), "rb") as f:
        sys_, hdr = R.read_r1cs_bytes(f.read())
    ref = G.docs_system()
    assert [(c.a, c.b, c.c) for c in sys_.rows] == [(c.a, c.b, c.c) for c in ref.rows]
    assert (sys_.n_pub_out, sys_.n_pub_in, sys_.n_priv_in, sys_.max_signal) == (1, 0, 2, 7)
    assert hdr["fs"] == 32


# ------------------------------------------------------------------ golden fixtures
def _fixture_system(fx):
    return R.System(int(fx["p"]), fx["max_signal"], fx["n_pub_out"], fx["n_pub_in"], fx["n_priv_in"],
                    set(fx["forbidden"]), G.rows_from_json(fx["rows"]))


def _fixtures():
    return sorted(f for f in os.listdir(GOLD) if f.startswith("oracle_") and f.endswith(".json"))


@pytest.mark.parametrize("fname", _fixtures())
def test_golden_pyref(fname):
    with open(os.path.join(GOLD, fname)) as f:
        fx = json.load(f)
    sys_ = _fixture_system(fx)
    for ex in fx["expected"]:
        res = R.simplification(sys_, G.flags_of(ex["level"], ex["rounds"], ex["old"]))
        assert G.result_to_json(res) == {k: ex[k] for k in ("constraints", "signal_map",
                                                              "no_private_inputs_witness")}


@pytest.mark.parametrize("fname", _fixtures())
def test_golden_refcpu(fname):
    """The C++ oracle (the GPU tests' checker) reproduces every golden vector."""
    with open(os.path.join(GOLD, fname)) as f:
        fx = json.load(f)
    sys_ = _fixture_system(fx)
    h = rsio.InputHolder(sys_)
    for ex in fx["expected"]:
        (cons, sm, nw, npiw), _, _ = rsio.oracle_run(h.inp, rsio.flags(ex["level"], ex["rounds"], ex["old"]), 2)
        res = R.Result(cons, sm, npiw)
        assert G.result_to_json(res) == {k: ex[k] for k in ("constraints", "signal_map",
                                                              "no_private_inputs_witness")}
        assert nw == len(sm)


# ------------------------------------------------------------------ refcpu vs pyref, random systems
@pytest.mark.parametrize("p", [257, 97, R.PRIMES["bn128"], R.PRIMES["goldilocks"], R.PRIMES["bls12377"]])
def test_refcpu_vs_pyref_random(p):
    for seed in range(12):
        sys_ = rsio.gen_system(500 + seed, p, n_sig=30 + 3 * seed, n_rows=50 + 5 * seed)
        h = rsio.InputHolder(sys_)
        for key in ("O1", "O2", "O2r1", "O2r2"):
            lvl, rd = LEVELS[key]
            ref = R.simplification(sys_, G.flags_of(lvl, rd))
            got, _, _ = rsio.oracle_run(h.inp, rsio.flags(lvl, rd), 1 + seed % 3)
            assert rsio.same_result(ref, got) is None, (seed, key)


@pytest.mark.parametrize("p", [257, R.PRIMES["bn128"]])
def test_refcpu_vs_pyref_forbidden_intermediates(p):
    """Forbidden signals beyond the public ones (custom-gate signals): eq clusters with several
    forbidden members, forbidden-only linear rows, constant equalities on forbidden signals."""
    for seed in range(10):
        sys_ = rsio.gen_system(5000 + seed, p, n_sig=30 + seed % 40, n_rows=50 + seed % 60, extra_forb=0.1 + 0.02 * seed)
        h = rsio.InputHolder(sys_)
        for key in ("O1", "O2", "O2r1"):
            lvl, rd = LEVELS[key]
            ref = R.simplification(sys_, G.flags_of(lvl, rd))
            got, _, _ = rsio.oracle_run(h.inp, rsio.flags(lvl, rd), 1 + seed % 3)
            assert rsio.same_result(ref, got) is None, (seed, key)


@pytest.mark.parametrize("old", [False, True])
def test_refcpu_vs_pyref_process4(old):
    for seed in range(3):
        sys_ = rsio.gen_system(900 + seed, R.PRIMES["bn128"], n_sig=300, n_rows=200, big_cluster=380 + 50 * seed)
        h = rsio.InputHolder(sys_)
        ref = R.simplification(sys_, G.flags_of("O2", None, old))
        got, _, _ = rsio.oracle_run(h.inp, rsio.flags("O2", None, old), 4)
        assert rsio.same_result(ref, got) is None


def test_refcpu_threads_deterministic():
    """Cluster results are collected in cluster-index order: the thread count
    never changes the output."""
    sys_ = rsio.gen_system(77, R.PRIMES["bn128"], n_sig=300, n_rows=300, big_cluster=500)
    h = rsio.InputHolder(sys_)
    outs = [rsio.oracle_run(h.inp, rsio.flags("O2"), t)[0] for t in (1, 2, 8)]
    assert outs[0] == outs[1] == outs[2]


def test_asan_ubsan_check(tmp_path):
    """the oracle and the product's host-side pieces (--O0 reader, writers, generator)
    built with -fsanitize=address,undefined and driven over every generator kind, three flag levels,
    1/3 oracle threads, and every truncation of an .r1cs (oracle/asan_check.cpp)."""
    import shutil
    import subprocess
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.check_call(["make", "-s", "-C", os.path.join(root, "oracle"), "asan"])
    r = subprocess.run([os.path.join(root, "oracle", "_ref", "asan_check"), str(tmp_path)],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "asan_check: OK" in r.stdout


def test_map_lists_across_rounds(tmp_path):
    """The lazily built row lists of the non-linear signal map (csrc/maplists.hpp; the appends of
    apply_substitution_to_map, constraint_simplification.rs:369-377) equal the plain recursion over
    the rounds' substitution batches, with ONE memo living through 8 rounds as in the engine: a list
    memoised in an earlier round must never answer for another (signal, bound) pair after more
    batches arrive (round-3 advisor finding: the memo key depended on the batch count)."""
    import subprocess
    root = os.path.dirname(HERE)
    exe = str(tmp_path / "maplists_check")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-I", os.path.join(root, "circom_cvm_amd", "csrc"),
                           os.path.join(HERE, "maplists_check.cpp"), "-o", exe])
    for seed in range(1, 13):
        for rounds, signals in ((8, 40), (5, 200), (12, 25)):
            out = subprocess.run([exe, str(seed), str(rounds), str(signals)], capture_output=True, text=True)
            assert out.returncode == 0 and out.stdout.startswith("ok"), out.stdout


def test_refcpu_alg_bytes():
    """SURVEY 8(d)'s B_alg as the oracle counts it (refcpu_last_alg; the roofline path's numerator in
    bench.py): deterministic across thread counts, the formula over its terms, Z_in = the input's
    entries, Z_out / R_out = the result's, and on the docs circuit (basic.circom at --O2) the value
    counted by hand from the reference's steps."""
    R = rsio.R
    for seed, p in ((3, 257), (11, R.PRIMES["bn128"]), (12, R.PRIMES["goldilocks"])):
        sys_ = rsio.gen_system(seed, p, n_sig=300, n_rows=250, big_cluster=700)
        h = rsio.InputHolder(sys_)
        fl = rsio.flags("O2")
        res = []
        for threads in (1, 4):
            arrays, _ = rsio.oracle_arrays(h.inp, fl, threads)
            res.append(rsio.oracle_last_alg())
        a = res[0]
        assert res[0] == res[1]
        assert a["B_alg"] == a["w"] * (a["z_in"] + a["z_out"] + a["subs"] + a["app"] + a["rowupd"] + a["merges"]) + \
            8 * (a["r_in"] + a["r_out"] + a["max_signal"])
        assert a["z_in"] == sum(b.lc.nnz for b in h.blocks)
        assert a["r_out"] == arrays["n_constraints"]
        assert a["z_out"] == sum(len(arrays[x][1]) for x in ("a", "b", "c"))
        assert a["w"] == (12 if p < 2 ** 64 else 36) and a["merges"] > 0  # 4 + r1cs_porting.rs:6-10 field size
    # basic.circom (constraints-json.md:57-96), counted by hand.  Input: eq rows {2: 1, 5: -1},
    # {1: -1, 4: 1}; the linear row {0: 1, 2: 2, 3: 1, 6: -1}; the non-linear row [5: -1] * [6: 1] =
    # [4: -1] -- 11 entries, 4 rows.  eq_simplification: 5 := 2 and 4 := 1 (1 forbidden), 1 entry each;
    # the eq frame renames nothing in the linear row.  Its cluster (1 row, process_3) pops it: pivot 6
    # (the largest takeable key), a holder of {0, 2, 3} (row update 4 + 3 entries) and its normalised
    # copy.  The non-linear row reads the two eq substitutions (both relevant) and the one of 6 (3
    # entries) and grows from 3 to 5 entries (A {2}, B {0, 2, 3}, C {1}) -- the result (:95-96).
    p = R.PRIMES["bn128"]
    m = p - 1
    rows = [R.Con({}, {}, {2: 1, 5: m}), R.Con({}, {}, {0: 1, 2: 2, 3: 1, 6: m}),
            R.Con({}, {}, {1: m, 4: 1}), R.Con({5: m}, {6: 1}, {4: m})]
    h = rsio.InputHolder(R.System(p, 7, 1, 0, 2, {0, 1}, rows))
    arrays, _ = rsio.oracle_arrays(h.inp, rsio.flags("O2"), 1)
    a = rsio.oracle_last_alg()
    assert (a["z_in"], a["r_in"], a["r_out"], a["z_out"]) == (11, 4, 1, 5)
    assert (a["subs"], a["app"], a["rowupd"], a["merges"]) == (2 + 3 + 3, 1 + 1 + 3, (4 + 3) + (3 + 5), 0), a
    assert a["B_alg"] == 36 * (11 + 5 + 8 + 5 + 15) + 8 * (4 + 1 + 7)
