#!/usr/bin/env python3
"""Multi-RHS timing on config 2 or 3 (device-resident inputs, one factorisation):
k single-seed dopt_qp_reverse / _forward calls against one dopt_qp_reverse_k /
_forward_k call (qp_multi.hip).  Prints one JSON line per k.

  python tools/bench_multi_rhs.py [--batch 1024] [--k 1 7 32]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diffopt.jl_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2, choices=[2, 3])
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--k", type=int, nargs="+", default=[1, 7, 32])
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch
    from diffopt_amd.qp import QPBatch
    from diffopt_amd.synthetic import QP_CONFIGS, SEED0, qp_torch
    c = QP_CONFIGS[a.config]
    B, n, m, p = a.batch, c["n"], c["m"], c["p"]
    d = qp_torch(B, n, m, p, c["phi"], SEED0 + a.config)
    e = QPBatch(B, n, m, p)
    e.set(d["Q"], d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
    e.factor()
    g = torch.Generator(device="cuda")
    g.manual_seed(7)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        best = 1e30
        for _ in range(a.reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        return best

    for k in a.k:
        dl = torch.randn(k, B, n, generator=g, device="cuda", dtype=torch.float64)
        dq = torch.randn(k, B, n, generator=g, device="cuda", dtype=torch.float64)
        t_loop_r = timed(lambda: [e.reverse(dl[j]) for j in range(k)])
        t_multi_r = timed(lambda: e.reverse_k(dl))
        t_loop_f = timed(lambda: [e.forward(dq=dq[j]) for j in range(k)])
        t_multi_f = timed(lambda: e.forward_k(dq=dq))
        print(json.dumps({"config": f"config {a.config} (n={n}, m={m}), factor kept", "batch": B, "k": k,
                          "reverse_loop_ms": round(1e3 * t_loop_r, 3), "reverse_k_ms": round(1e3 * t_multi_r, 3),
                          "forward_loop_ms": round(1e3 * t_loop_f, 3), "forward_k_ms": round(1e3 * t_multi_f, 3),
                          "seed_solves_per_s_k": round(2 * k * B / (t_multi_r + t_multi_f), 1),
                          "speedup": round((t_loop_r + t_loop_f) / (t_multi_r + t_multi_f), 2)}), flush=True)


if __name__ == "__main__":
    main()
