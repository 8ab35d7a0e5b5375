"""Diagnostic: in-kernel phase cycle breakdown of the blocked panel kernel
(DOPT_STAMPS=1, forced blocked path).  python tools/stamps_blocked.py CFG B"""
import os, sys, time
os.environ["DOPT_STAMPS"] = "1"
os.environ.setdefault("DOPT_FAST_MAX", "0")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "diffopt.jl_amd")]
import numpy as np
import torch
from diffopt_amd.qp import QPBatch
from diffopt_amd.synthetic import qp_torch
cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
n, m = (200, 300) if cfg == 2 else (1000, 1500)
d = qp_torch(B, n, m, 0, 0.3, 20250309)
e = QPBatch(B, n, m, 0)
e.set(d["Q"], d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
e.forward_reverse(d["dl_dz"], dq=d["dq"], dh=d["dh"])
buf = np.zeros(8, dtype=np.int64)
e.lib.dopt_debug_stamps(e.h, buf.ctypes.data, 8)
torch.cuda.synchronize()
e.forward_reverse(d["dl_dz"], dq=d["dq"], dh=d["dh"])
torch.cuda.synchronize()
e.lib.dopt_debug_stamps(e.h, buf.ctypes.data, 8)
names = ["load", "columns", "writeback", "inverses", "dinv", "u12"]
tot = buf[:6].sum()
npan = (n + int(0.3 * m) + 31) // 32
print(f"cfg{cfg} B={B}: cycles per problem-panel (avg over {B}×{npan}):")
for k, v in zip(names, buf):
    print(f"  {k:10s} {v / B / npan:12.0f} cyc  {100.0 * v / tot:5.1f}%")
