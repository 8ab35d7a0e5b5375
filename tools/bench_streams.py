#!/usr/bin/env python3
"""Experiment: config 2 split into S sub-batches, each on its own handle,
stream and host thread (ctypes releases the GIL), so one sub-batch's
memory-bound assembly can overlap another's MFMA-bound LU.  Prints ms per
step for S = 1 and S = 2, 4.

  python tools/bench_streams.py [--steps 20] [--warmup 3]
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "diffopt.jl_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1024)
    args = ap.parse_args()
    import torch
    from diffopt_amd.qp import QPBatch
    from diffopt_amd.synthetic import SEED0, qp_torch
    n, m, p, phi = 200, 300, 0, 0.3
    B = args.batch
    d = qp_torch(B, n, m, p, phi, SEED0 + 2)
    res = {}
    for S in (1, 2, 4, 8, 1, 4):
        b = B // S
        streams = [torch.cuda.Stream() for _ in range(S)]
        engs, outs, parts = [], [], []
        for s in range(S):
            sl = slice(s * b, (s + 1) * b)
            part = {k: v[sl] for k, v in d.items()}
            with torch.cuda.stream(streams[s]):
                e = QPBatch(b, n, m, p)
                e.set(part["Q"], part["G"], part["h"], part["A"], part["z"], part["lam"], part["nu"])
            engs.append(e)
            parts.append(part)
            outs.append((torch.empty(b, n + m, dtype=torch.float64, device="cuda"),
                         torch.empty(b, n + m, dtype=torch.float64, device="cuda")))
        torch.cuda.synchronize()

        def work(s, k):
            with torch.cuda.stream(streams[s]):
                for _ in range(k):
                    pt = parts[s]
                    engs[s].forward_reverse(pt["dl_dz"], dq=pt["dq"], dh=pt["dh"], out_rev=outs[s][0],
                                            out_fwd=outs[s][1])

        def run(k):
            th = [threading.Thread(target=work, args=(s, k)) for s in range(S)]
            for t in th:
                t.start()
            for t in th:
                t.join()
            torch.cuda.synchronize()

        run(args.warmup)
        t0 = time.perf_counter()
        run(args.steps)
        ms = 1e3 * (time.perf_counter() - t0) / args.steps
        res[S] = round(ms, 4)
        print(json.dumps({"slices": S, "ms_per_step": res[S], "solves_per_s": round(B / ms * 1e3, 1)}), flush=True)
        for e in engs:
            e.close()


if __name__ == "__main__":
    main()
