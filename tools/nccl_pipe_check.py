"""GatherPipeline on the nccl (RCCL) backend with a single rank on one GPU:
exercises the async all_gather_into_tensor + stream-ordered waits of the
bench's overlapped gather (the driver runs the multi-rank case)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "diffopt.jl_amd")]
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
import torch
import torch.distributed as dist
from diffopt_amd import parallel
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
pipe = parallel.GatherPipeline(4, 6, torch.float64, "cuda")
for k in range(6):
    pipe.next_buffer().copy_(torch.full((4, 6), float(k), device="cuda"))
    pipe.submit()
    if k >= 1:
        assert torch.equal(pipe.result(k - 1), torch.full((4, 6), float(k - 1), device="cuda"))
pipe.drain()
torch.cuda.synchronize()
assert torch.equal(pipe.result(5), torch.full((4, 6), 5.0, device="cuda"))
dist.destroy_process_group()
print("nccl gather pipeline ok")
