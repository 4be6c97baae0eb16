"""SURVEY 8(f) rank 4 without cargo: the Rust side of the seam (integration/rust) is checked against
the C header it binds -- every declared function is bound with the same arity, and every #[repr(C)]
struct lists the header's fields in order with the matching Rust type -- so a layout change on
either side fails here.  Plus the r1cs parity tool (tools/r1cs_diff.py, a restatement of
constraint_writers/src/r1cs_reader.rs:453-564) on identical, reordered and different files."""
import os
import re
import subprocess
import sys
import tempfile

import rsio

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "rs_simplify.h")
RS = os.path.join(ROOT, "integration", "rust", "src", "lib.rs")
R = rsio.R

C2RUST = {"uint32_t": "u32", "uint64_t": "u64", "int32_t": "i32", "uint8_t": "u8", "double": "f64", "rs_lc": "rs_lc"}


def _strip_c_comments(s):
    return re.sub(r"/\*.*?\*/", "", s, flags=re.S)


def c_structs():
    src = _strip_c_comments(open(HDR).read())
    out = {}
    for name, body in re.findall(r"typedef struct (\w+) \{(.*?)\} \1;", src, flags=re.S):
        fields = []
        for decl in body.split(";"):
            decl = " ".join(decl.split())
            if not decl:
                continue
            const = decl.startswith("const ")
            if const:
                decl = decl[len("const "):]
            m = re.match(r"(\w+)\s*(\*?)\s*(.+)", decl)
            ty, star, names = m.group(1), m.group(2), m.group(3)
            for nm in names.split(","):
                nm = nm.strip()
                ptr = star or nm.startswith("*")
                nm = nm.lstrip("*").strip()
                arr = re.match(r"(\w+)\[(\d+)\]", nm)
                rt = C2RUST[ty]
                if arr:
                    nm, rt = arr.group(1), f"[{rt}; {arr.group(2)}]"
                elif ptr:
                    rt = f"*const {rt}" if const else f"*mut {rt}"
                fields.append((nm, rt))
        out[name] = fields
    return out


def rust_structs():
    src = open(RS).read()
    out = {}
    for name, body in re.findall(r"pub struct (\w+) \{(.*?)\n\}", src, flags=re.S):
        out[name] = [(n, " ".join(t.split())) for n, t in re.findall(r"pub (\w+): ([^,\n]+),", body)]
    return out


def c_functions():
    src = _strip_c_comments(open(HDR).read())
    return {m.group(1): len([p for p in m.group(2).split(",") if p.strip() and p.strip() != "void"])
            for m in re.finditer(r"^[\w\s\*]*?\b(rs_\w+)\s*\(([^)]*)\)\s*;", src, flags=re.M)}


def rust_functions():
    src = open(RS).read()
    return {m.group(1): len([p for p in m.group(2).split(",") if p.strip()])
            for m in re.finditer(r"pub fn (rs_\w+)\(([^)]*)\)", src)}


def test_rust_bindings_cover_every_function():
    cf, rf = c_functions(), rust_functions()
    assert len(cf) >= 25
    assert set(cf) == set(rf), (set(cf) ^ set(rf))
    for name in cf:
        assert cf[name] == rf[name], name


def test_rust_structs_match_header_layout():
    cs, rs = c_structs(), rust_structs()
    for name in ("rs_lc", "rs_input", "rs_flags", "rs_output", "rs_stats", "rs_dag"):
        assert cs[name] == rs[name], (name, [x for x in zip(cs[name], rs[name]) if x[0] != x[1]][:3])


def test_rust_abi_version_matches_header():
    ver = re.search(r"#define RS_ABI_VERSION (\d+)", open(HDR).read()).group(1)
    assert f"pub const RS_ABI_VERSION: c_int = {ver};" in open(RS).read()


def _tool(*args):
    return subprocess.run([sys.executable, os.path.join(ROOT, "tools", "r1cs_diff.py"), *args],
                          capture_output=True, text=True, timeout=120)


def test_r1cs_diff_tool():
    sys_ = rsio.gen_system(61, R.PRIMES["bn128"], n_sig=90, n_rows=120)
    res = R.simplification(sys_, R.Flags())
    data = R.result_to_r1cs(sys_, res)
    with tempfile.TemporaryDirectory() as tmp:
        a, b, c = (os.path.join(tmp, x) for x in ("a.r1cs", "b.r1cs", "c.r1cs"))
        open(a, "wb").write(data)
        open(b, "wb").write(data)
        r = _tool(a, b)
        assert r.returncode == 0, r.stdout + r.stderr
        # the same constraints in another order: equal as sets (the reference's own order is not
        # canonical), not byte-identical
        rev = R.Result(list(reversed(res.constraints)), res.signal_map, res.no_private_inputs_witness)
        open(c, "wb").write(R.result_to_r1cs(sys_, rev))
        r = _tool(a, c)
        assert r.returncode == 2, r.stdout + r.stderr
        # one coefficient changed
        cons = list(res.constraints)
        k = next(iter(cons[0].c))
        cons[0] = R.Con(cons[0].a, cons[0].b, {**cons[0].c, k: (cons[0].c[k] + 1) % sys_.p or 1})
        open(c, "wb").write(R.result_to_r1cs(sys_, R.Result(cons, res.signal_map, res.no_private_inputs_witness)))
        r = _tool(a, c)
        assert r.returncode == 1 and "constraint" in r.stdout, r.stdout + r.stderr


GLUE = os.path.join(ROOT, "integration", "rust", "constraint_list_glue.rs")
# num-bigint(-dig) BigInt API the reference itself calls on the path's data (file:line in
# /root/reference): to_bytes_le (constraint_writers/src/r1cs_writer.rs:26), from_bytes_le
# (r1cs_reader.rs:41), to/from_signed_bytes_le (circom_algebra/src/constraint_storage/logic.rs:7,25),
# is_zero via num_traits::Zero (circom_algebra/src/algebra.rs:4), BigInt::from (algebra.rs passim).
BIGINT_ALLOWED = {"to_bytes_le", "from_bytes_le", "to_signed_bytes_le", "from_signed_bytes_le", "is_zero", "from"}
# other BigInt / BigUint methods of num-bigint: none may appear in the glue (the pinned
# num-bigint-dig 0.8.4 is not vendored, so only calls the reference makes are known to exist)
BIGINT_API = {"to_u64_digits", "to_u32_digits", "from_slice", "from_slice_native", "from_biguint", "to_biguint",
              "from_radix_be", "from_radix_le", "to_radix_be", "to_radix_le", "to_str_radix", "parse_bytes",
              "magnitude", "into_parts", "bits", "from_bytes_be", "to_bytes_be", "from_signed_bytes_be",
              "to_signed_bytes_be", "modpow", "sqrt", "cbrt", "nth_root", "trailing_zeros", "set_bit", "bit",
              "mod_inverse", "to_u64", "to_i64", "from_u64", "new", "assign_from_slice", "iter_u64_digits",
              "iter_u32_digits", "to_usize"}


def test_rust_glue_uses_only_reference_bigint_calls():
    src = re.sub(r"//[^\n]*", "", open(GLUE).read())
    calls = set(re.findall(r"\.(\w+)\(", src)) | set(re.findall(r"BigInt::(\w+)\(", src))
    bad = (calls & BIGINT_API) - BIGINT_ALLOWED
    assert not bad, f"BigInt methods the reference never calls: {sorted(bad)}"
    for m in re.findall(r"BigInt::(\w+)\(", src):
        assert m in BIGINT_ALLOWED, m
    if ".is_zero(" in src:
        assert re.search(r"use circom_algebra::num_traits::Zero;", src), "is_zero needs num_traits::Zero in scope"
    if "Sign::" in src:
        assert re.search(r"use circom_algebra::num_bigint::\{[^}]*\bSign\b", src)
    # every ffi call in the glue is a function the header declares
    for f in re.findall(r"ffi::(rs_\w+)\(", src):
        assert f in c_functions(), f
    # --simplification_substitution writes the log file (constraint_simplification.rs:448-453)
    assert "rs_write_substitution_json" in src and "json_substitutions" in src


def test_rust_lib_doc_abi_matches_header():
    ver = re.search(r"#define RS_ABI_VERSION (\d+)", open(HDR).read()).group(1)
    assert f"(ABI {ver})" in open(RS).read().splitlines()[0]


PATCH = os.path.join(ROOT, "integration", "rust", "circom_algebra_new_unchecked.patch")
REF_ALGEBRA = "/root/reference/circom_algebra/src/algebra.rs"


def test_rust_glue_constraint_calls_come_from_reference_or_patch(tmp_path):
    """The drop-in is complete as committed: every Constraint associated function the glue calls is
    public in the reference's circom_algebra (algebra.rs) or added by the committed patch
    (integration/rust/circom_algebra_new_unchecked.patch: `pub fn new_unchecked`, next to the private
    Constraint::new of algebra.rs:1012), and the patch applies to the reference's file."""
    src = re.sub(r"//[^\n]*", "", open(GLUE).read())
    calls = set(re.findall(r"\bC::(\w+)\(", src)) | set(re.findall(r"\bConstraint::(\w+)\(", src))
    patch = open(PATCH).read()
    added = set(re.findall(r"^\+[ \t]*pub fn (\w+)\(", patch, flags=re.M))
    assert added == {"new_unchecked"}
    assert re.search(r"^\+\s*pub fn new_unchecked\(a: HashMap<C, BigInt>, b: HashMap<C, BigInt>, c: HashMap<C, BigInt>\)"
                     r" -> Constraint<C> \{\n\+\s*Constraint::new\(a, b, c\)", patch, flags=re.M)
    assert "new_unchecked" in calls
    if not os.path.exists(REF_ALGEBRA):  # the GPU box has no reference tree
        assert calls <= added
        return
    public = set(re.findall(r"^\s*pub fn (\w+)\(", open(REF_ALGEBRA).read(), flags=re.M))
    assert "new_unchecked" not in public
    assert calls <= public | added, calls - public - added
    dst = tmp_path / "circom_algebra" / "src"
    dst.mkdir(parents=True)
    (dst / "algebra.rs").write_bytes(open(REF_ALGEBRA, "rb").read())
    r = subprocess.run(["patch", "-p1", "--dry-run", "-d", str(tmp_path), "-i", PATCH], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
