"""Diagnostic: in-kernel phase cycle breakdown of the fused QP kernel (config 2)."""
import os, sys, time
os.environ["DOPT_STAMPS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "diffopt.jl_amd")]
import numpy as np
import torch
from diffopt_amd.qp import QPBatch
from diffopt_amd.synthetic import qp_torch
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
d = qp_torch(B, 200, 300, 0, 0.3, 20250309)
e = QPBatch(B, 200, 300, 0)
e.set(d["Q"], d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
e.forward_reverse(d["dl_dz"], dq=d["dq"], dh=d["dh"])
buf = np.zeros(8, dtype=np.int64)
e.lib.dopt_debug_stamps(e.h, buf.ctypes.data, 8)
torch.cuda.synchronize()
t0 = time.perf_counter()
e.forward_reverse(d["dl_dz"], dq=d["dq"], dh=d["dh"])
torch.cuda.synchronize()
dt = time.perf_counter() - t0
e.lib.dopt_debug_stamps(e.h, buf.ctypes.data, 8)
names = ["prepare", "assemble", "lu_panel", "lu_linv", "lu_update", "reverse", "forward"]
tot = buf[:7].sum()
print(f"step {dt*1e3:.3f} ms; cycles per problem (avg over {B}):")
for n, v in zip(names, buf):
    print(f"  {n:10s} {v / B:12.0f} cyc  {100.0 * v / tot:5.1f}%")
