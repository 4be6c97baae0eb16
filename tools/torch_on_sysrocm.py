"""torch.distributed (nccl = RCCL) after librs_simplify has loaded /opt/rocm's HIP runtime and RCCL (the
order bench.py uses): a world-1 process group, one all_reduce and a barrier, and the libraries mapped."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import circom_cvm_amd as M  # noqa: E402

M.abi.lib()
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
t = torch.ones(4, device="cuda")
dist.all_reduce(t)
dist.barrier()
torch.cuda.synchronize()
print("all_reduce ok:", t.tolist())
libs = sorted({ln.split()[-1] for ln in open("/proc/self/maps") if any(x in ln for x in ("libamdhip64", "librccl"))})
print("mapped:", libs)
dist.destroy_process_group()
