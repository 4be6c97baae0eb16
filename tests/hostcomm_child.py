"""One rank of the two-process host-transport test (tests/test_gpu_sharded.py::test_two_process_host_transport):
an engine on device 0 joins the group `tag` as `rank` (rs_engine_join_host), simplifies the synthetic
circuit host -> host `reps` times (the result streamed into the group's shared host region, made by the
same code as RCCL ranks'), and checks its view against the oracle, array for array.
usage: hostcomm_child.py <world> <rank> <tag> <kind> <rows> <reps>"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import rsio  # noqa: E402
import circom_cvm_amd as M  # noqa: E402

world, rank, tag, kind, rows, reps = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], int(sys.argv[4]), int(sys.argv[5]), int(sys.argv[6])
e = M.Engine(0)
e.join_host(world, rank, tag)
inp = M.Input.synth(kind, rows, 42)
fl = rsio.flags("O2")
ref, _ = rsio.oracle_arrays(inp.c, fl, threads=4)
for i in range(reps):
    got = rsio.output_arrays(e.simplify(inp.c, fl))
    diff = rsio.diff_output_arrays(got, ref)
    if diff is not None:
        print(f"rank {rank} call {i}: differs from the oracle: {diff}", flush=True)
        sys.exit(3)
st = e.stats()
assert st.world == world, st.world
# the run-resident path too (rs_engine_load + rs_engine_run + rs_engine_fetch over the same group)
e.load(inp.c)
e.run(fl)
out = e.fetch()
if rsio.diff_output_arrays(rsio.output_arrays(out.c), ref) is not None:
    print(f"rank {rank}: load/run/fetch differs from the oracle", flush=True)
    sys.exit(4)
e.close()
print(f"rank {rank} ok", flush=True)
