#!/usr/bin/env python3
"""Latency of the drop-in path, one model at a time: the
call sequence the Julia back-ends issue per model — QPModel (`_ensure!`:
dopt_qp_set_csc of the MOI matrix form, then dopt_qp_reverse; forward on the
same factorisation) and the narrow `LinearAlgebraSolver` plug point
(MI355XSolver: dopt_lhs_solve with LHS, then LHS') — at config-1 and config-2
shapes, batch 1, host buffers, beside the oracle's single solve on one core
(the reference algorithm: assemble the full KKT, SuperLU, refactorised per
direction, QuadraticProgram.jl:316-446).  Prints one JSON line per case.
The `qpmodel_*_ms` fields time the Python wrapper calls; `qpmodel_*_abi_ms`
time the ABI calls alone with their arrays and pointers ready, as the Julia
ccalls issue them (`qpmodel_set_csc_ms` is that already).

  python tools/bench_dropin.py [--reps 30]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "diffopt.jl_amd"))


def _med(ts):
    return float(np.median(ts)) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    import scipy.sparse as sp
    from diffopt_amd.qp import MI355XSolver, QPBatch
    from diffopt_amd.synthetic import QP_CONFIGS, SEED0, qp_numpy
    from oracle import qp as oqp   # the CPU baseline only (test infrastructure)

    for cfg in (1, 2):
        c = QP_CONFIGS[cfg]
        n, m, p = c["n"], c["m"], c["p"]
        d = qp_numpy(a.reps + 1, n, m, p, c["phi"], SEED0 + cfg)
        prob = lambda r: [d[k][r] for k in ("Q", "G", "h", "A", "z", "lam", "nu")]
        # oracle: one reverse + one forward solve per model (CPU, 1 core)
        t_or = []
        for r in range(a.reps):
            Q, G, h, A, z, lam, nu = prob(r)
            t0 = time.perf_counter()
            oqp.reverse_differentiate(Q, G, h, A, z, lam, nu, d["dl_dz"][r])
            oqp.forward_differentiate(Q, G, h, A, z, lam, nu, dq=d["dq"][r], dh=d["dh"][r],
                                      db=d["db"][r] if p else None)
            t_or.append(time.perf_counter() - t0)
        # QPModel: handle once, then per model set_csc + reverse + forward
        e = QPBatch(1, n, m, p)
        t_first = time.perf_counter()
        Q, G, h, A, z, lam, nu = prob(a.reps)
        e.set_csc([sp.csc_matrix(Q)], [sp.csc_matrix(G)], h[None],
                  [sp.csc_matrix(A)] if p else None, z[None], lam[None], nu[None] if p else None)
        e.reverse(d["dl_dz"][a.reps][None])
        t_first = time.perf_counter() - t_first
        t_set, t_rev, t_fwd, t_py = [], [], [], []
        t_rev_abi, t_fwd_abi = [], []
        lib = e.lib
        out_r = np.empty((1, n + m + p)); out_f = np.empty((1, n + m + p))
        for r in range(a.reps):
            Q, G, h, A, z, lam, nu = prob(r)
            # the MOI matrix form as Julia holds it (CSC arrays built outside
            # the timed ABI call; the Python conversion timed on its own)
            tp = time.perf_counter()
            args = e.set_csc([sp.csc_matrix(Q)], [sp.csc_matrix(G)], h[None], [sp.csc_matrix(A)] if p else None,
                             z[None], lam[None], nu[None] if p else None)
            t_py.append(time.perf_counter() - tp)
            t0 = time.perf_counter()
            e.set_csc_args(args)
            t1 = time.perf_counter()
            e.reverse(d["dl_dz"][r][None])
            t2 = time.perf_counter()
            e.forward(dq=d["dq"][r][None], dh=d["dh"][r][None], db=d["db"][r][None] if p else None)
            t3 = time.perf_counter()
            t_set.append(t1 - t0); t_rev.append(t2 - t1); t_fwd.append(t3 - t2)
            # the same two calls as the Julia ccalls issue them: arrays and
            # pointers ready, the ABI call alone timed (set_csc above likewise)
            e.set_csc_args(args)
            dl = np.ascontiguousarray(d["dl_dz"][r][None])
            vq, vh = np.ascontiguousarray(d["dq"][r][None]), np.ascontiguousarray(d["dh"][r][None])
            vb = np.ascontiguousarray(d["db"][r][None]) if p else None
            pv = [vq.ctypes.data, vh.ctypes.data, vb.ctypes.data if p else None]
            t4 = time.perf_counter()
            rc = lib.dopt_qp_reverse(e.h, dl.ctypes.data, out_r.ctypes.data)
            t5 = time.perf_counter()
            rc |= lib.dopt_qp_forward(e.h, None, pv[0], None, pv[1], None, pv[2], out_f.ctypes.data)
            t6 = time.perf_counter()
            assert rc == 0
            t_rev_abi.append(t5 - t4); t_fwd_abi.append(t6 - t5)
        e.close()
        # the LinearAlgebraSolver plug point: LHS (reverse) and LHS' (forward)
        def plug(solver):
            ts = []
            for r in range(a.reps):
                Q, G, h, A, z, lam, nu = prob(r)
                L = oqp.create_LHS_matrix(z, lam, Q, G, h, A)
                L = np.asarray(L.todense() if hasattr(L, "todense") else L)
                rhs = np.concatenate([d["dl_dz"][r], np.zeros(L.shape[0] - n)])
                t0 = time.perf_counter()
                if solver is None:
                    s = MI355XSolver()
                    s.solve_system(L, rhs); s.solve_system(L.T, rhs)
                    s.close()
                else:
                    solver.solve_system(L, rhs); solver.solve_system(L.T, rhs)
                ts.append(time.perf_counter() - t0)
            return ts
        s = MI355XSolver()
        plug(s)                      # warm
        t_cached = plug(s)
        s.close()
        t_fresh = plug(None)
        print(json.dumps(dict(
            case=f"config {cfg} shape, batch 1 (n={n}, m={m}, p={p})",
            oracle_rev_fwd_ms=round(_med(t_or), 3),
            qpmodel_first_call_ms=round(t_first * 1e3, 3),
            qpmodel_set_csc_ms=round(_med(t_set), 3), python_csc_build_and_set_ms=round(_med(t_py), 3),
            qpmodel_reverse_ms=round(_med(t_rev), 3),
            qpmodel_forward_ms=round(_med(t_fwd), 3),
            qpmodel_model_ms=round(_med(np.add(np.add(t_set, t_rev), t_fwd)), 3),
            qpmodel_reverse_abi_ms=round(_med(t_rev_abi), 3),
            qpmodel_forward_abi_ms=round(_med(t_fwd_abi), 3),
            qpmodel_model_abi_ms=round(_med(np.add(np.add(t_set, t_rev_abi), t_fwd_abi)), 3),
            plug_point_cached_handle_ms=round(_med(t_cached), 3),
            plug_point_handle_per_call_ms=round(_med(t_fresh), 3),
            reps=a.reps)), flush=True)


if __name__ == "__main__":
    main()
