"""Oracle-only calibration behind tests/test_conic_gpu.py::test_capped_lsqr_istop7:
on the shapes whose LSQR runs to maxiter (istop 7, an ill-conditioned M), how
far the oracle's LSQR iterate after k iterations moves when its right-hand-side
data is perturbed by one ulp (relative 2^-52, 5 seeded trials) — the k where
that spread first passes 1e-6 bounds the iteration counts at which the engine
can be held to the 1e-6 bar.  Writes profiles/r05/conic_capped_spread.txt."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "diffopt.jl_amd")]
from diffopt_amd.synthetic import SEED0, conic_numpy  # noqa: E402
from oracle import conic as ocn  # noqa: E402

SHAPES = [("config-4 bench shape", 2, 500, [(3, 25)] * 20, SEED0 + 4, False),
          ("mixed cones", 3, 30, [(0, 3), (1, 10), (3, 6), (2, 4), (4, 6)], 11, False),
          ("SOC only", 2, 40, [(3, 5)] * 8, 12, False),
          ("PSD blocks", 3, 25, [(4, 10), (4, 15), (1, 5)], 13, False),
          ("CSC shape", 3, 20, [(0, 3), (1, 10), (3, 6), (4, 6)], 31, True)]
KS = list(range(1, 41)) + [50, 100, 200, 1001]


def relfro(a, b):
    nb = np.linalg.norm(b)
    return np.linalg.norm(a - b) / nb if nb > 0 else np.linalg.norm(a)


def main():
    lines = ["# oracle LSQR capped at k iterations: max relative change of the solution (fwd: [du|dv|dw], "
             "rev: g) over 5 one-ulp perturbations of the right-hand-side data; '*' marks > 1e-6"]
    for name, B, n, cones, seed, csc in SHAPES:
        d = conic_numpy(B, n, cones, seed)
        A = d["A"].copy()
        if csc:
            A[:, :, 2] = 0.0
        N = n + A.shape[1] + 1
        first = None
        for k in [k for k in KS if k <= N] + ([N] if N not in KS else []):
            worst = 0.0
            for b in range(B):
                cache = ocn.Cache(A[b], d["b"][b], d["c"][b], d["x"][b], d["s"][b], d["y"][b], cones)
                f0 = ocn.forward_differentiate(cache, d["dA"][b], d["db"][b], d["dc"][b], maxiter=k)
                f0 = np.concatenate([f0[1], f0[2], [f0[3]]])
                g0 = ocn.reverse_differentiate(cache, d["dx"][b], maxiter=k)[0]
                rng = np.random.default_rng(7)
                for _ in range(5):
                    p = lambda a: np.asarray(a, float) * (1.0 + 2.0 ** -52 * rng.standard_normal(np.shape(a)))
                    f1 = ocn.forward_differentiate(cache, d["dA"][b], p(d["db"][b]), p(d["dc"][b]), maxiter=k)
                    f1 = np.concatenate([f1[1], f1[2], [f1[3]]])
                    g1 = ocn.reverse_differentiate(cache, p(d["dx"][b]), maxiter=k)[0]
                    worst = max(worst, relfro(f1, f0), relfro(g1, g0))
            if worst > 1e-6 and first is None:
                first = k
            if first is not None and k > first + 3 and k not in (50, 100, 200, 1001):
                continue
            lines.append(f"{name:22s} N={N:5d} k={k:5d}  spread {worst:.2e}{' *' if worst > 1e-6 else ''}")
            print(lines[-1], flush=True)
        lines.append(f"{name:22s} first k with spread > 1e-6: {first}")
    out = os.path.join(ROOT, "profiles", "r05", "conic_capped_spread.txt")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    open(out, "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
