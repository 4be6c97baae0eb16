"""Diagnostic: the substitution log of one synthetic workload under two environments (run as two
processes), compared entry by entry.  usage: python tools/logdiff.py kind rows ENV=VAL"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1 and sys.argv[1] == "--dump":
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import rsio
    import circom_cvm_amd as M
    kind, rows, path = int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    inp = M.Input.synth(kind, rows, 42)
    eng = M.Engine(0)
    eng.load(inp.c)
    eng.run(rsio.flags("O2", log=True))
    out = eng.fetch()
    o = out.c
    n = int(o.n_log)
    frm = np.ctypeslib.as_array(o.log_from, shape=(max(n, 1),))[:n].astype(np.int64)
    ptr = np.ctypeslib.as_array(o.log_to.ptr, shape=(n + 1,)).astype(np.int64)
    nnz = int(ptr[-1])
    keys = np.ctypeslib.as_array(o.log_to.col, shape=(max(nnz, 1),))[:nnz].astype(np.int64)
    vals = np.ctypeslib.as_array(o.log_to.val, shape=(max(4 * nnz, 1),))[:4 * nnz].copy()
    np.savez(path, frm=frm, ptr=ptr, keys=keys, vals=vals)
    print("dumped", n, flush=True)
    sys.exit(0)
kind, rows = sys.argv[1], sys.argv[2]
env2 = dict(os.environ)
for kv in sys.argv[3:]:
    k, v = kv.split("=", 1)
    env2[k] = v
a, b = "/tmp/logA.npz", "/tmp/logB.npz"
subprocess.check_call([sys.executable, __file__, "--dump", kind, rows, a])
subprocess.check_call([sys.executable, __file__, "--dump", kind, rows, b], env=env2)
A, B = np.load(a), np.load(b)
print("log lengths", len(A["frm"]), len(B["frm"]))
def index(X):
    return {int(f): i for i, f in enumerate(X["frm"])}
ia, ib = index(A), index(B)
def entry(X, i):
    p0, p1 = int(X["ptr"][i]), int(X["ptr"][i + 1])
    return (X["keys"][p0:p1].tolist(), X["vals"][4 * p0:4 * p1].tolist())
class Lazy(dict):
    def __init__(self, X, ix):
        super().__init__()
        self.X, self.ix = X, ix
    def keys_(self):
        return self.ix.keys()
da, db = ia, ib
only_a = sorted(set(da) - set(db))
only_b = sorted(set(db) - set(da))
print("only in A:", len(only_a), only_a[:10], flush=True)
print("only in B:", len(only_b), only_b[:10], flush=True)
nd = 0
for f in sorted(set(da) & set(db)):
    ea, eb = entry(A, da[f]), entry(B, db[f])
    if ea != eb:
        nd += 1
        if nd <= 5:
            print("differs", f, "A:", ea[0][:12], "B:", eb[0][:12], flush=True)
print("different RHS:", nd, flush=True)
first = next((i for i in range(min(len(A["frm"]), len(B["frm"]))) if A["frm"][i] != B["frm"][i]), None)
print("first order difference at", first)
