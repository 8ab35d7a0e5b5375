"""Fused (one WG per problem) vs blocked (batched step launches) route sweep
over reduced KKT sizes and batch sizes, to pick the default fast_max."""
import os, sys, time, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "diffopt.jl_amd")]
import torch
from diffopt_amd.qp import QPBatch
from diffopt_amd.synthetic import qp_torch

res = []
for n in [44, 66, 88, 110, 132, 176, 200, 300]:
    m = int(1.5 * n)
    for B in [1024, 128]:
        d = qp_torch(B, n, m, 0, 0.3, 7)
        for fm in [512, 0]:
            e = QPBatch(B, n, m, 0)
            e.set_fast_max(fm)
            e.set(d["Q"], d["G"], d["h"], None, d["z"], d["lam"], None)
            for _ in range(2):
                e.forward_reverse(d["dl_dz"], dq=d["dq"], dh=d["dh"])
            torch.cuda.synchronize()
            k = 5
            t0 = time.perf_counter()
            for _ in range(k):
                e.forward_reverse(d["dl_dz"], dq=d["dq"], dh=d["dh"])
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / k
            Np = int(e.system_size().mean())
            e.close()
            r = dict(n=n, m=m, Nred=Np, batch=B, fast_max=fm, ms=round(dt * 1e3, 4),
                     solves_per_s=round(B / dt, 1))
            print(json.dumps(r), flush=True)
            res.append(r)
