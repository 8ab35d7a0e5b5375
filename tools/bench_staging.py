#!/usr/bin/env python3
"""Host→device staging cost on config 2: what a caller
that holds the problems on the host — the reference's `copy_to` into the
MOI matrix form (`_gradient_cache`, QuadraticProgram.jl:182-213;
`sparse_array_representation`, utils.jl:46-69) — pays per step.

Per step, one of:
  device   inputs resident in HBM (the bench.py line: no staging)
  dense    host column-major Q/G (+ vectors) through dopt_qp_set (PCIe copy)
  csc      host Julia-style CSC arrays (Int64, 1-based) through dopt_qp_set_csc,
           densified on the device
followed by one dopt_qp_forward_reverse of every problem.  The CSC arrays are
built once outside the timed region (the Julia side holds them already).
Prints one JSON line per mode.

  python tools/bench_staging.py [--batch 1024] [--steps 10]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diffopt.jl_amd"))


def _csc_arrays(mats):
    import scipy.sparse as sp
    cps, rvs, nzs, off = [], [], [], 0
    for M in mats:
        M = sp.csc_matrix(M)
        cps.append(M.indptr.astype(np.int64) + off + 1)
        rvs.append(M.indices.astype(np.int64) + 1)
        nzs.append(M.data.astype(np.float64))
        off += M.nnz
    return (np.ascontiguousarray(np.concatenate(cps)), np.ascontiguousarray(np.concatenate(rvs)),
            np.ascontiguousarray(np.concatenate(nzs)), off)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    import torch
    from diffopt_amd import _lib
    from diffopt_amd.qp import QPBatch
    from diffopt_amd.synthetic import QP_CONFIGS, SEED0, qp_config_numpy

    c = QP_CONFIGS[2]
    B, n, m, p = a.batch, c["n"], c["m"], c["p"]
    d = qp_config_numpy(2, batch=B)
    L = n + m + p
    # column-major, batch-major host buffers (the ABI's dense layout)
    Qc = np.ascontiguousarray(np.transpose(d["Q"], (0, 2, 1)))
    Gc = np.ascontiguousarray(np.transpose(d["G"], (0, 2, 1)))
    vec = {k: np.ascontiguousarray(d[k]) for k in ("h", "z", "lam", "dl_dz", "dq", "dh")}
    Qs = _csc_arrays([d["Q"][b] for b in range(B)])
    Gs = _csc_arrays([d["G"][b] for b in range(B)])
    e = QPBatch(B, n, m, p)
    lib, h = e.lib, e.h
    P = lambda x: None if x is None else x.ctypes.data

    def fwd_rev_host():
        o1 = np.empty((B, L)); o2 = np.empty((B, L))
        _lib.check(lib.dopt_qp_forward_reverse(h, P(vec["dl_dz"]), None, P(vec["dq"]), None, P(vec["dh"]),
                                               None, None, P(o1), P(o2)), h)

    def step_dense():
        _lib.check(lib.dopt_set_memory(h, _lib.DOPT_MEM_HOST), h)
        _lib.check(lib.dopt_qp_set(h, P(Qc), P(Gc), P(vec["h"]), None, P(vec["z"]), P(vec["lam"]), None), h)
        fwd_rev_host()

    def step_csc():
        _lib.check(lib.dopt_set_memory(h, _lib.DOPT_MEM_HOST), h)
        _lib.check(lib.dopt_qp_set_csc(h, P(Qs[0]), P(Qs[1]), P(Qs[2]), Qs[3], P(Gs[0]), P(Gs[1]), P(Gs[2]), Gs[3],
                                       None, None, None, 0, P(vec["h"]), P(vec["z"]), P(vec["lam"]), None), h)
        fwd_rev_host()

    td = {k: torch.from_numpy(v).cuda() for k, v in vec.items()}
    Qd, Gd = torch.from_numpy(d["Q"]).cuda(), torch.from_numpy(d["G"]).cuda()
    od1 = torch.empty(B, L, dtype=torch.float64, device="cuda")
    od2 = torch.empty(B, L, dtype=torch.float64, device="cuda")
    e.set(Qd, Gd, td["h"], None, td["z"], td["lam"], None)

    def step_device():
        e.forward_reverse(td["dl_dz"], dq=td["dq"], dh=td["dh"], out_rev=od1, out_fwd=od2)

    def timed(fn, label):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.steps

    res = {}
    for label, fn in (("device", step_device), ("dense", step_dense), ("csc", step_csc)):
        res[label] = timed(fn, label)
    # the three modes give the same sensitivities (same data): checked bit for bit
    e._mem = None                      # the host-mode calls above switched the handle's memory mode
    e.set(Qd, Gd, td["h"], None, td["z"], td["lam"], None)
    step_device()
    r_dev = od1.cpu().numpy()
    o1 = np.empty((B, L)); o2 = np.empty((B, L))
    _lib.check(lib.dopt_set_memory(h, _lib.DOPT_MEM_HOST), h)
    _lib.check(lib.dopt_qp_set_csc(h, P(Qs[0]), P(Qs[1]), P(Qs[2]), Qs[3], P(Gs[0]), P(Gs[1]), P(Gs[2]), Gs[3],
                                   None, None, None, 0, P(vec["h"]), P(vec["z"]), P(vec["lam"]), None), h)
    _lib.check(lib.dopt_qp_forward_reverse(h, P(vec["dl_dz"]), None, P(vec["dq"]), None, P(vec["dh"]),
                                           None, None, P(o1), P(o2)), h)
    same = bool(np.array_equal(o1, r_dev))

    in_bytes = {"dense": 8 * B * (n * n + m * n + 2 * m + n),
                "csc": int(Qs[0].nbytes + Qs[1].nbytes + Qs[2].nbytes + Gs[0].nbytes + Gs[1].nbytes
                           + Gs[2].nbytes + 8 * B * (2 * m + n)),
                "device": 0}
    for label in ("device", "dense", "csc"):
        t = res[label]
        print(json.dumps({"workload": "config 2 (n=200, m=300), set + forward_reverse per step", "batch": B,
                          "mode": label, "ms_per_step": round(1e3 * t, 3),
                          "staging_ms": round(1e3 * (t - res["device"]), 3),
                          "host_bytes_per_step": in_bytes[label],
                          "solves_per_s": round(B / t, 1),
                          "bit_identical_csc_vs_device": same}), flush=True)


if __name__ == "__main__":
    main()
