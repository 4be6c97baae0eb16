import sys, os
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "tests"))
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import rsio
import circom_cvm_amd as M
R = rsio.R
p = 257
for seed in range(6):
    sys_ = rsio.gen_system(2000 + seed, p, n_sig=300, n_rows=250, big_cluster=600 + 40 * seed)
    h = rsio.InputHolder(sys_)
    for lvl, rd, old in (("O2", None, False), ("O2", None, True), ("O2", 2, False)):
        fl = rsio.flags(lvl, rd, old)
        eng = M.Engine(0); eng.load(h.inp); eng.run(fl)
        out = eng.fetch(); got = rsio.output_to_py(out.c)
        ref, _, _ = rsio.oracle_run(h.inp, fl, 4)
        ok = got == ref
        print(seed, lvl, rd, old, "OK" if ok else "DIFF " + str(rsio.same_result(R.Result(ref[0], ref[1], ref[3]), got))[:300], flush=True)
        eng.close()
