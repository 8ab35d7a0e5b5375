"""Oracle-only measurement behind tests/test_conic_gpu.py::test_config4_bench_shape:
how far LSQR's terminal state moves, at config 4's bench shape (istop 7,
maxiter 1001), when the right-hand side is perturbed by one ulp (relative
2^-52, seeded).  Writes profiles/r03/conic_cfg4_maxiter_spread.txt."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "diffopt.jl_amd")]
from diffopt_amd.synthetic import SEED0, conic_numpy  # noqa: E402
from oracle import conic as ocn  # noqa: E402
from oracle.lsqr import lsqr  # noqa: E402

keys = ("rnorm", "arnorm", "xnorm", "anorm")
cones = [(3, 25)] * 20
d = conic_numpy(2, 500, cones, SEED0 + 4)
lines = ["# config-4 bench shape, oracle LSQR on 1-ulp-perturbed right-hand sides (run 0 unperturbed)",
         "# columns: rnorm arnorm xnorm anorm (LSQR estimates) |Mx-b| |M^T(Mx-b)|/(|M||Mx-b|) iterations istop"]
for b in range(2):
    cache = ocn.Cache(d["A"][b], d["b"][b], d["c"][b], d["x"][b], d["s"][b], d["y"][b], cones)
    M = cache.M()
    M2 = np.linalg.norm(M, 2)
    frhs = ocn.forward_rhs(cache, d["dA"][b], d["db"][b], d["dc"][b])
    rrhs = np.concatenate([d["dx"][b], np.zeros(cache.m), [-(cache.x @ d["dx"][b])]])
    for name, rhs in (("fwd", frhs), ("rev", rrhs)):
        rng = np.random.default_rng(7)
        rows = []
        for t in range(5):
            rr = rhs if t == 0 else rhs * (1.0 + 2.0 ** -52 * rng.standard_normal(rhs.shape))
            st = {}
            x, it, istop = lsqr(cache.matvec, cache.rmatvec, rr, len(rr), return_info=True, stats=st)
            r = M @ x - rhs
            rows.append([st[k] for k in keys] + [np.linalg.norm(r), np.linalg.norm(M.T @ r) / (M2 * np.linalg.norm(r)),
                                                 it, istop])
        rows = np.array(rows)
        for t, row in enumerate(rows):
            lines.append(f"problem {b} {name} run {t}: " + " ".join(f"{v:.6e}" for v in row[:6])
                         + f" {int(row[6])} {int(row[7])}")
        rel = (rows.max(0) - rows.min(0))[:6] / np.abs(rows[:, :6]).max(0)
        lines.append(f"problem {b} {name} relative spread: " + " ".join(f"{v:.2e}" for v in rel))
out = os.path.join(ROOT, "profiles", "r03", "conic_cfg4_maxiter_spread.txt")
os.makedirs(os.path.dirname(out), exist_ok=True)
open(out, "w").write("\n".join(lines) + "\n")
print("\n".join(lines))
