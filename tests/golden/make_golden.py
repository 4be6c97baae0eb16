"""Writes the golden fixtures under tests/golden/ (run: python tests/golden/make_golden.py).

Two kinds of vectors:
  * docs_basic.json -- the reference's own known-answer data for the `basic.circom` circuit, typed in
    from /root/reference/mkdocs/docs/circom-language/formats/constraints-json.md:57-59, 77-81, 95-96
    (constraint JSON at --O1/--O0/--O2), sym.md:46-51, 65-70, 81-86 (.sym at --O1/--O0/--O2) and
    simplification-json.md:49-50, 78-80 (substitution log at --O1/--O2).  Plus the --O0 .r1cs/.sym of
    that circuit and the expected --O1/--O2 files, written with the oracle's byte writer.
  * oracle_*.json -- seeded small systems (several primes, every simplification branch) with the
    outputs of the literal Python restatement oracle/pyref.py, which the tests pin against the docs
    data above and the reference unit tests (algebra.rs:1401-1493, modular_arithmetic.rs:221-268).

The reference itself is Rust and cannot be built or imported here, so these are the
vectors parity rests on.  Nothing under /root/reference is read by this script."""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import pyref as R  # noqa: E402

P = R.PRIMES["bn128"]
M1 = str(P - 1)

# ---- docs KAT (basic.circom): inputs
DOCS_O0_ROWS = [  # constraints-json.md:77-81 (--O0 = the system simplification() consumes)
    [{}, {}, {"2": "1", "5": M1}],
    [{}, {}, {"0": "1", "2": "2", "3": "1", "6": M1}],
    [{}, {}, {"1": M1, "4": "1"}],
    [{"5": M1}, {"6": "1"}, {"4": M1}],
]
DOCS = {
    "prime": "bn128", "max_signal": 7, "n_pub_out": 1, "n_pub_in": 0, "n_priv_in": 2,
    "o0_rows": DOCS_O0_ROWS,
    "constraints": {  # constraints-json.md (witness numbering)
        "O1": [[{"2": M1}, {"4": "1"}, {"1": M1}],
               [{}, {}, {"0": "1", "2": "2", "3": "1", "4": M1}]],
        "O0": DOCS_O0_ROWS,
        "O2": [[{"2": M1}, {"0": "1", "2": "2", "3": "1"}, {"1": M1}]],
    },
    "sym_o0": ["1,1,1,main.out", "2,2,1,main.in[0]", "3,3,1,main.in[1]",
               "4,4,0,main.c.out", "5,5,0,main.c.in[0]", "6,6,0,main.c.in[1]"],
    "sym": {  # sym.md
        "O1": ["1,1,1,main.out", "2,2,1,main.in[0]", "3,3,1,main.in[1]",
               "4,-1,0,main.c.out", "5,-1,0,main.c.in[0]", "6,4,0,main.c.in[1]"],
        "O2": ["1,1,1,main.out", "2,2,1,main.in[0]", "3,3,1,main.in[1]",
               "4,-1,0,main.c.out", "5,-1,0,main.c.in[0]", "6,-1,0,main.c.in[1]"],
    },
    "substitutions": {  # simplification-json.md
        "O1": {"5": {"2": "1"}, "4": {"1": "1"}},
        "O2": {"5": {"2": "1"}, "4": {"1": "1"}, "6": {"0": "1", "2": "2", "3": "1"}},
    },
}


def rows_from_json(rows):
    return [R.Con(*[{int(k): int(v) for k, v in m.items()} for m in r]) for r in rows]


def rows_to_json(rows):
    return [[{str(k): str(m[k]) for k in sorted(m)} for m in (c.a, c.b, c.c)] for c in rows]


def docs_system():
    d = DOCS
    forb = {0} | set(range(1, d["n_pub_out"] + d["n_pub_in"] + 1))
    return R.System(R.PRIMES[d["prime"]], d["max_signal"], d["n_pub_out"], d["n_pub_in"],
                    d["n_priv_in"], forb, rows_from_json(d["o0_rows"]))


def flags_of(level: str, rounds=None, old=False) -> "R.Flags":
    if level == "O1":
        return R.Flags(flag_s=True, no_rounds=0, use_old_heuristics=old)
    return R.Flags(flag_s=False, no_rounds=(1 << 64) - 1 if rounds is None else rounds,
                   use_old_heuristics=old)


def result_to_json(res: "R.Result"):
    return {"constraints": rows_to_json(res.constraints),
            "signal_map": {str(k): v for k, v in sorted(res.signal_map.items())},
            "no_private_inputs_witness": res.no_private_inputs_witness}


# fixture cases: (name, seed, prime, gen kwargs, [(level, rounds, old)])
CASES = [
    ("f257_a", 11, 257, dict(n_sig=40, n_rows=60), [("O1", None, False), ("O2", None, False), ("O2", 1, False)]),
    ("f257_b", 12, 257, dict(n_sig=70, n_rows=110), [("O1", None, False), ("O2", None, False), ("O2", 2, False)]),
    ("f97", 13, 97, dict(n_sig=50, n_rows=90), [("O2", None, False)]),
    ("bn128", 14, R.PRIMES["bn128"], dict(n_sig=60, n_rows=100), [("O1", None, False), ("O2", None, False)]),
    ("bls12381", 15, R.PRIMES["bls12381"], dict(n_sig=60, n_rows=100), [("O2", None, False)]),
    ("goldilocks", 16, R.PRIMES["goldilocks"], dict(n_sig=60, n_rows=100), [("O2", None, False)]),
    ("secq256r1", 17, R.PRIMES["secq256r1"], dict(n_sig=60, n_rows=100), [("O2", None, False)]),
    ("process4_bn128", 18, R.PRIMES["bn128"], dict(n_sig=300, n_rows=200, big_cluster=420),
     [("O2", None, False), ("O2", None, True)]),
]


def main():
    import rsio
    sys_ = docs_system()
    with open(os.path.join(HERE, "docs_basic.json"), "w") as f:
        json.dump(DOCS, f, indent=1, sort_keys=True)
    # --O0 export of basic.circom and the expected --O1 / --O2 files (identity wire map at O0)
    ident = R.Result(sys_.rows, {i: i for i in range(sys_.max_signal)}, sys_.n_priv_in)
    with open(os.path.join(HERE, "docs_basic_O0.r1cs"), "wb") as f:
        f.write(R.result_to_r1cs(sys_, ident))
    with open(os.path.join(HERE, "docs_basic_O0.sym"), "w") as f:
        f.write("".join(line + "\n" for line in DOCS["sym_o0"]))
    sym_lines = [tuple(int(x) if i < 3 else x for i, x in enumerate(line.split(",", 3)))
                 for line in DOCS["sym_o0"]]
    for lvl in ("O1", "O2"):
        res = R.simplification(sys_, flags_of(lvl))
        with open(os.path.join(HERE, f"docs_basic_{lvl}.r1cs"), "wb") as f:
            f.write(R.result_to_r1cs(sys_, res))
        with open(os.path.join(HERE, f"docs_basic_{lvl}.sym"), "w") as f:
            f.write(R.result_to_sym(sym_lines, res))
    # seeded systems with oracle outputs
    for name, seed, p, kw, runs in CASES:
        s = rsio.gen_system(seed, p, **kw)
        fx = {"p": str(p), "max_signal": s.max_signal, "n_pub_out": s.n_pub_out,
              "n_pub_in": s.n_pub_in, "n_priv_in": s.n_priv_in, "forbidden": sorted(s.forbidden),
              "rows": rows_to_json(s.rows), "expected": []}
        for lvl, rd, old in runs:
            res = R.simplification(s, flags_of(lvl, rd, old))
            fx["expected"].append({"level": lvl, "rounds": rd, "old": old, **result_to_json(res)})
        with open(os.path.join(HERE, f"oracle_{name}.json"), "w") as f:
            json.dump(fx, f, separators=(",", ":"), sort_keys=True)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
