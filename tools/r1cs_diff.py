"""Compare two .r1cs files the way the reference's reader sees them.

A restatement of constraint_writers/src/r1cs_reader.rs:453-564 (read_r1cs: magic + version,
section table, header section 1, constraint section 2, wire->label section 3, custom-gate
sections 4/5, each located by type wherever it lies in the file), then a comparison:

  exit 0  byte-identical
  exit 2  same content, different bytes: equal headers, wire->label maps and custom-gate sections,
          and the same constraints as a multiset (the reference's storage order is not canonical
          across implementations); the first differing byte offset is printed
  exit 1  different content; the first difference is printed

usage: python tools/r1cs_diff.py A.r1cs B.r1cs"""
import struct
import sys
from collections import Counter


class Bad(Exception):
    pass


def read_r1cs(data: bytes) -> dict:
    """r1cs_reader.rs:453-481 read_r1cs + :498-564 read_sections."""
    if len(data) < 12 or data[:4] != b"r1cs":
        raise Bad("not an r1cs file")
    (version,) = struct.unpack_from("<I", data, 4)
    (nsec,) = struct.unpack_from("<I", data, 8)
    off, secs = 12, {}
    for _ in range(nsec):
        if off + 12 > len(data):
            raise Bad("truncated section table")
        t, sz = struct.unpack_from("<IQ", data, off)
        off += 12
        if off + sz > len(data):
            raise Bad(f"section {t} runs past the end")
        secs.setdefault(t, (off, sz))
        off += sz
    if 1 not in secs or 2 not in secs:
        raise Bad("header or constraint section missing")
    ho, _ = secs[1]
    (fs,) = struct.unpack_from("<I", data, ho)
    prime = int.from_bytes(data[ho + 4: ho + 4 + fs], "little")
    n_wires, n_out, n_pub, n_prv, n_labels, n_cons = struct.unpack_from("<IIIIQI", data, ho + 4 + fs)
    r = dict(version=version, field_size=fs, prime=prime, n_wires=n_wires, n_pub_out=n_out,
             n_pub_in=n_pub, n_priv_in=n_prv, n_labels=n_labels, n_constraints=n_cons)
    o, end = secs[2][0], secs[2][0] + secs[2][1]
    cons = []
    for _ in range(n_cons):
        lcs = []
        for _ in range(3):
            (n,) = struct.unpack_from("<I", data, o)
            o += 4
            terms = []
            for _ in range(n):
                (k,) = struct.unpack_from("<I", data, o)
                terms.append((k, int.from_bytes(data[o + 4: o + 4 + fs], "little")))
                o += 4 + fs
            lcs.append(tuple(sorted(terms)))
        if o > end:
            raise Bad("constraint section overrun")
        cons.append(tuple(lcs))
    r["constraints"] = cons
    if 3 in secs:
        so, ssz = secs[3]
        r["wire_to_label"] = list(struct.unpack_from(f"<{ssz // 8}Q", data, so))
    r["gates_used"] = data[secs[4][0]: secs[4][0] + secs[4][1]] if 4 in secs else None
    r["gates_applied"] = data[secs[5][0]: secs[5][0] + secs[5][1]] if 5 in secs else None
    return r


def first_diff(a: bytes, b: bytes) -> int:
    n = min(len(a), len(b))
    for i in range(0, n, 1 << 16):
        if a[i: i + (1 << 16)] != b[i: i + (1 << 16)]:
            for j in range(i, min(n, i + (1 << 16))):
                if a[j] != b[j]:
                    return j
    return n


def compare(a: bytes, b: bytes):
    """(exit code, message)."""
    if a == b:
        return 0, f"identical ({len(a)} bytes)"
    ra, rb = read_r1cs(a), read_r1cs(b)
    for k in ("version", "field_size", "prime", "n_wires", "n_pub_out", "n_pub_in", "n_priv_in",
              "n_labels", "n_constraints"):
        if ra[k] != rb[k]:
            return 1, f"header {k}: {ra[k]} != {rb[k]}"
    if ra.get("wire_to_label") != rb.get("wire_to_label"):
        wa, wb = ra.get("wire_to_label") or [], rb.get("wire_to_label") or []
        i = next((i for i, (x, y) in enumerate(zip(wa, wb)) if x != y), min(len(wa), len(wb)))
        return 1, f"wire->label map differs at wire {i}"
    for k in ("gates_used", "gates_applied"):
        if ra[k] != rb[k]:
            return 1, f"custom-gate section {k} differs"
    ca, cb = Counter(ra["constraints"]), Counter(rb["constraints"])
    if ca != cb:
        only_a = ca - cb
        i = next(i for i, c in enumerate(ra["constraints"]) if c in only_a)
        return 1, f"constraint {i} of the first file is not in the second ({len(only_a)} differ)"
    return 2, f"same content, different order (first differing byte {first_diff(a, b)})"


def main(argv):
    if len(argv) != 3:
        sys.stderr.write(__doc__)
        return 64
    with open(argv[1], "rb") as f:
        a = f.read()
    with open(argv[2], "rb") as f:
        b = f.read()
    try:
        code, msg = compare(a, b)
    except (Bad, struct.error) as e:
        print(f"unreadable: {e}")
        return 1
    print(msg)
    return code


if __name__ == "__main__":
    sys.exit(main(sys.argv))
