"""Transcribe the reference's known-answer tests into JSON golden fixtures.

Run once in the build container (reads /root/reference, which does not exist
on the GPU box):  python tests/golden/make_golden.py

Every fixture holds (a) the problem data exactly as written in the reference
test, (b) the primal–dual point — given by the test, or derived here in closed
form / by exact active-set enumeration where the test delegates it to a
solver (HiGHS/Ipopt/SCS are not available; a QP's KKT point is unique under
strict complementarity, so the derivation is solver-free), and (c) the
expected sensitivities with the test's own tolerance.  Nothing in here is the
oracle: tests/test_oracle_golden.py checks the oracle against these values.
"""

import itertools
import json
import math
import os

import numpy as np

REF = "/root/reference/test"
OUT = os.path.dirname(os.path.abspath(__file__))
R2 = math.sqrt(2.0)


def _lists(d):
    out = {}
    for k, v in d.items():
        if isinstance(v, np.ndarray):
            out[k] = v.tolist()
        elif isinstance(v, dict):
            out[k] = _lists(v)
        elif isinstance(v, list):
            out[k] = [_lists(e) if isinstance(e, dict) else e for e in v]
        else:
            out[k] = v
    return out


def kkt_point(Q, q, G, h, A, b, tol=1e-12):
    """Exact KKT point of a small strictly convex QP by active-set enumeration
    (OptNet sign: Qz + q + Gᵀλ + Aᵀν = 0, λ ≥ 0, Gz ≤ h, Az = b)."""
    n = Q.shape[0]
    m = G.shape[0]
    p = A.shape[0]
    for k in range(0, min(m, n) + 1):
        for act in itertools.combinations(range(m), k):
            act = list(act)
            Ga = G[act]
            K = np.zeros((n + k + p, n + k + p))
            K[:n, :n] = Q
            K[:n, n:n + k] = Ga.T
            K[:n, n + k:] = A.T
            K[n:n + k, :n] = Ga
            K[n + k:, :n] = A
            rhs = np.concatenate([-q, h[act], b])
            try:
                sol = np.linalg.solve(K, rhs)
            except np.linalg.LinAlgError:
                continue
            z = sol[:n]
            lam = np.zeros(m)
            lam[act] = sol[n:n + k]
            nu = sol[n + k:]
            if np.all(lam >= -tol) and np.all(G @ z - h <= tol):
                lam[np.abs(lam) < tol] = 0.0
                return z, lam, nu
    raise RuntimeError("no KKT point")


def qp_fixtures():
    fx = []
    # --- test/quadratic_program.jl:232-293 (test_differentiating_moi_examples_2)
    Q = np.array([[4, 1.0], [1, 2]])
    q = np.array([1, 1.0])
    G = np.array([[-1, 0.0], [0, -1]])
    h = np.array([0, 0.0])
    A = np.array([[1, 1.0]])
    b = np.array([1.0])
    dQ = np.array([[-0.05, -0.05], [-0.05, 0.15]])
    dq = np.array([-0.2, 0.2])
    dG = np.zeros((2, 2))
    dh = np.zeros(2)
    dA = np.array([[0.375, -1.075]])
    db = np.array([0.7])
    fx.append(dict(
        name="qp_moi_example_2", source="test/quadratic_program.jl:232-293",
        Q=Q, q=q, G=G, h=h, A=A, b=b,
        z=np.array([0.25, 0.75]), lam=np.zeros(2), nu=np.array([-2.75]),
        dzb=np.array([1.3, 0.5]),
        fwd=dict(dQ=dQ, dq=dq, dG=dG, dh=dh, dA=dA, db=db),
        expect=dict(dQb=dQ, dqb=dq, dGb=dG, dhb=dh, dAb=dA, dbb=db,
                    dzf=np.array([1.4875, -0.075]),
                    grad_zf=np.array([-1.28125, 3.25625]),
                    grad_zb=np.array([-0.2, 0.2]),
                    grad_lamb=np.array([0.8, -0.8 / 3]),
                    grad_nub=np.array([-0.7])),
        atol=2e-4, rtol=2e-4, point="given by the test"))
    # --- test/quadratic_program.jl:131-176 (quadprog example)
    Q = np.array([[1.0, -1.0, 1.0], [-1.0, 2.0, -2.0], [1.0, -2.0, 4.0]])
    q = np.array([2.0, -3.0, 1.0])
    G = np.array([[0, 0, 1.0], [0, 1, 0], [1, 0, 0], [0, 0, -1], [0, -1, 0],
                  [-1, 0, 0]])
    h = np.array([1.0, 1.0, 1.0, 0.0, 0.0, 0.0])
    A = np.array([[1.0, 1.0, 1.0]])
    b = np.array([0.5])
    z, lam, nu = kkt_point(Q, q, G, h, A, b)
    fx.append(dict(
        name="qp_quadprog", source="test/quadratic_program.jl:131-176",
        Q=Q, q=q, G=G, h=h, A=A, b=b, z=z, lam=lam, nu=nu, dzb=np.ones(3),
        fwd=dict(dQ=np.ones((3, 3)), dq=np.ones(3), dG=np.ones((6, 3)),
                 dh=np.ones(6), dA=np.ones((1, 3)), db=np.ones(1)),
        expect=dict(z=np.array([0.0, 0.5, 0.0]), dQb=np.zeros((3, 3)),
                    dqb=np.zeros(3), dGb=np.zeros((6, 3)), dhb=np.zeros(6),
                    dAb=np.array([[0.0, -0.5, 0.0]]), dbb=np.array([1.0])),
        atol=2e-4, rtol=2e-4, point="exact active-set KKT point"))
    # --- test/quadratic_program.jl:181-227 (MOI contquadratic example 1)
    Q = np.array([[2.0, 1.0, 0.0], [1.0, 2.0, 1.0], [0.0, 1.0, 2.0]])
    q = np.zeros(3)
    G = np.array([[-1.0, -2.0, -3.0], [-1.0, -1.0, 0.0]])
    h = np.array([-4.0, -1.0])
    A = np.zeros((0, 3))
    b = np.zeros(0)
    z, lam, nu = kkt_point(Q, q, G, h, A, b)
    dQ = np.array([[-0.12244895, 0.01530609, -0.11224488],
                   [0.01530609, 0.09183674, 0.07653058],
                   [-0.11224488, 0.07653058, -0.06122449]])
    dq = np.array([-0.2142857, 0.21428567, -0.07142857])
    dG = np.array([[0.05102692, 0.30612244, 0.25510856],
                   [0.06120519, 0.36734693, 0.30610315]])
    dh = np.array([-0.35714284, -0.4285714])
    fx.append(dict(
        name="qp_moi_example_1", source="test/quadratic_program.jl:181-227",
        Q=Q, q=q, G=G, h=h, A=A, b=b, z=z, lam=lam, nu=nu, dzb=np.ones(3),
        fwd=dict(dQ=dQ, dq=dq, dG=dG, dh=dh),
        expect=dict(dQb=dQ, dqb=dq, dGb=dG, dhb=dh),
        atol=2e-4, rtol=2e-4, point="exact active-set KKT point"))
    # --- test/quadratic_program.jl:62-91 (trivial QP 1) and the cache test
    #     test/conic_program.jl:649-735 (grad_wrt_h ≈ -1 = constant)
    Q = np.array([[4.0, 1.0], [1.0, 2.0]])
    q = np.array([1.0, 1.0])
    G = np.array([[1.0, 1.0]])
    h = np.array([-1.0])
    z, lam, nu = kkt_point(Q, q, G, h, np.zeros((0, 2)), np.zeros(0))
    fx.append(dict(
        name="qp_trivial_1", source="test/quadratic_program.jl:62-91",
        Q=Q, q=q, G=G, h=h, A=np.zeros((0, 2)), b=np.zeros(0), z=z, lam=lam,
        nu=nu, dzb=np.ones(2),
        fwd=dict(dQ=-np.ones((2, 2)), dq=np.ones(2), dG=np.ones((1, 2)),
                 dh=-np.ones(1)),
        expect=dict(z=np.array([-0.25, -0.75]), dhb=np.ones(1)),
        atol=2e-4, rtol=2e-4, point="exact active-set KKT point"))
    # --- test/quadratic_program.jl:295-350 + test/data/*.txt
    rd = lambda nm: np.loadtxt(os.path.join(REF, "data", nm + ".txt"), ndmin=2)
    Q, q, G, h, A, b = (rd(k) for k in ["P", "q", "G", "h", "A", "b"])
    q, h, b = q.ravel(), h.ravel(), b.ravel()
    z = np.linalg.solve(A, b)               # A is 10×10 nonsingular
    s = G @ z - h
    assert np.all(s < 0), "all inequalities must be inactive"
    lam = np.zeros(G.shape[0])
    nu = -np.linalg.solve(A.T, Q @ z + q)
    nz = Q.shape[0]
    fx.append(dict(
        name="qp_data_txt", source="test/quadratic_program.jl:295-350; test/data/*.txt",
        Q=Q, q=q, G=G, h=h, A=A, b=b, z=z, lam=lam, nu=nu, dzb=np.ones(nz),
        fwd=dict(dQ=np.ones((nz, nz)), dq=np.ones(nz), dG=np.ones(G.shape),
                 dh=np.ones(len(h)), dA=np.ones(A.shape), db=np.ones(len(b))),
        expect=dict(dqb=rd("dq").ravel(), dhb=rd("dh").ravel(),
                    dbb=rd("db").ravel()),
        atol=1e-3, rtol=1e-3,
        point="z = A⁻¹b (A square), λ = 0 (all rows inactive), ν = −A⁻ᵀ(Qz+q)"))
    return fx


def lp_fixtures():
    fx = []
    # test/linear_program.jl:223-246 (nonactive constraints)
    G = -np.ones((2, 1))
    h = np.array([0.0, -3.0])
    fx.append(dict(
        name="lp_nonactive", source="test/linear_program.jl:223-246",
        Q=np.zeros((1, 1)), q=np.array([1.0]), G=G, h=h, A=np.zeros((0, 1)),
        b=np.zeros(0), z=np.array([3.0]), lam=np.array([0.0, 1.0]),
        nu=np.zeros(0), dzb=-np.ones(1),
        fwd=dict(dq=np.zeros(1), dh=np.array([0.0, 1.0])),
        expect=dict(dhb=np.array([0.0, 1.0]), dzf=-np.ones(1),
                    grad_zb=np.zeros(1), grad_lamb=np.array([0.0, -1.0])),
        atol=2e-4, rtol=2e-4, point="given by the test"))
    # test/linear_program.jl:31-49 (same LP, other seeds)
    fx.append(dict(
        name="lp_nonactive_2", source="test/linear_program.jl:31-49",
        Q=np.zeros((1, 1)), q=np.array([1.0]), G=G, h=h, A=np.zeros((0, 1)),
        b=np.zeros(0), z=np.array([3.0]), lam=np.array([0.0, 1.0]),
        nu=np.zeros(0), dzb=np.ones(1), fwd=dict(dq=np.ones(1)),
        expect=dict(dGb=np.array([[0.0], [3.0]]), dhb=np.array([0.0, -1.0])),
        atol=2e-4, rtol=2e-4, point="z = 3, λ = (0, 1) by inspection"))
    # test/linear_program.jl:70-102 (simplex example, max 2x+3y+4z)
    G = np.array([[3.0, 2.0, 1.0], [2.0, 5.0, 3.0], [-1.0, 0, 0], [0, -1.0, 0],
                  [0, 0, -1.0]])
    h = np.array([10.0, 15.0, 0.0, 0.0, 0.0])
    fx.append(dict(
        name="lp_simplex", source="test/linear_program.jl:70-102",
        Q=np.zeros((3, 3)), q=np.array([-2.0, -3.0, -4.0]), G=G, h=h,
        A=np.zeros((0, 3)), b=np.zeros(0), z=np.array([0.0, 0.0, 5.0]),
        lam=np.array([0.0, 4 / 3, 2 / 3, 11 / 3, 0.0]), nu=np.zeros(0),
        dzb=np.ones(3), fwd=dict(dq=np.ones(3)),
        expect=dict(dqb=np.zeros(3),
                    dGb=np.array([[0, 0, 0], [0, 0, -5 / 3], [0, 0, 5 / 3],
                                  [0, 0, -10 / 3], [0, 0, 0.0]]),
                    dhb=np.array([0.0, 1 / 3, -1 / 3, 2 / 3, 0.0])),
        atol=2e-4, rtol=2e-4,
        point="vertex (0,0,5); λ from stationarity on the active rows"))
    # test/linear_program.jl:147-176 (fixed x1 = 0 as an equality)
    G = np.array([[3.0, 2.0, 1.0], [2.0, 5.0, 3.0], [0, -1.0, 0], [0, 0, -1.0]])
    h = np.array([10.0, 15.0, 0.0, 0.0])
    fx.append(dict(
        name="lp_fixed", source="test/linear_program.jl:147-176",
        Q=np.zeros((3, 3)), q=np.array([-2.0, -3.0, -4.0]), G=G, h=h,
        A=np.array([[1.0, 0, 0]]), b=np.array([0.0]),
        z=np.array([0.0, 0.0, 5.0]), lam=np.array([0.0, 4 / 3, 11 / 3, 0.0]),
        nu=np.array([-2 / 3]), dzb=np.ones(3), fwd=dict(dq=np.ones(3)),
        expect=dict(dqb=np.zeros(3),
                    dGb=np.array([[0, 0, 0], [0, 0, -5 / 3], [0, 0, -10 / 3],
                                  [0, 0, 0.0]]),
                    dhb=np.array([0.0, 1 / 3, 2 / 3, 0.0]),
                    dAb=np.array([[0.0, 0.0, -5 / 3]]), dbb=np.array([1 / 3])),
        atol=2e-4, rtol=2e-4,
        point="vertex (0,0,5); λ, ν from stationarity on the active rows"))
    return fx


def conic_fixtures():
    fx = []
    # test/conic_program.jl:29-120 (SOC2, eq_vec = true); vars (x, y, t);
    # rows Zeros(1), Nonnegatives(1), SecondOrderCone(3) as in the test's s/y
    A_moi = np.array([[0, 0, -1.0], [0, 1.0, 0], [0, 0, 1.0], [1.0, 0, 0],
                      [0, 1.0, 0]])
    b_moi = np.array([1.0, -1 / R2, 0, 0, 0])
    dA = np.array([[1.0, 0, 0], [0, 1.0, 0], [0, 0, 1.0], [0, 0, 0], [0, 0, 0]])
    fx.append(dict(
        name="conic_soc", source="test/conic_program.jl:29-120",
        cones=[[0, 1], [1, 1], [3, 3]], A=A_moi, b=b_moi, c=np.array([1.0, 0, 0]),
        max_sense=False, x=np.array([-1 / R2, 1 / R2, 1.0]),
        s=np.array([0.0, 0.0, 1.0, -1 / R2, 1 / R2]),
        y=np.array([R2, 1.0, R2, 1.0, -1.0]),
        forward=[dict(dA=dA, db=np.zeros(5), dc=np.zeros(3),
                      dx=np.array([1.12132144, 1 / R2, 1 / R2]),
                      atol=2e-4, rtol=2e-4)],
        reverse=[]))
    # test/conic_program.jl:134-210 and :801-844 (2×2 PSD, X2 = 1);
    # rows PSD-triangle(3), Zeros(1); duals as matrix entries (set_dot)
    A_moi = np.array([[1.0, 0, 0], [0, 1.0, 0], [0, 0, 1.0], [0, 1.0, 0]])
    b_moi = np.array([0, 0, 0, -1.0])
    fx.append(dict(
        name="conic_psd2", source="test/conic_program.jl:134-210, 801-844",
        cones=[[4, 3], [0, 1]], A=A_moi, b=b_moi, c=np.array([1.0, 0, 1.0]),
        max_sense=False, x=np.ones(3), s=np.array([1.0, 1.0, 1.0, 0.0]),
        y=np.array([1.0, -1.0, 1.0, 2.0]),
        forward=[dict(dA=np.zeros((4, 3)), db=np.array([0, 0, 0, 1.0]),
                      dc=np.zeros(3), dx=-np.ones(3), atol=2e-4, rtol=2e-4),
                 dict(dA=np.zeros((4, 3)), db=np.zeros(4),
                      dc=np.array([-1.0, 0, 1.0]), dx=np.array([1.0, 0, -1.0]),
                      atol=2e-4, rtol=2e-4)],
        reverse=[dict(dx=np.array([1.0, 0, 0]), rows=[3],
                      db=np.array([-1.0]), atol=2e-4, rtol=2e-4)]))
    # test/conic_program.jl:581-647 and :737-790 (3×3 PSD, min x)
    fx.append(dict(
        name="conic_psd3", source="test/conic_program.jl:581-647, 737-790",
        cones=[[4, 6]], A=np.array([[1.0], [0], [1.0], [0], [0], [1.0]]),
        b=np.array([0, 1.0, 0, 1.0, 1.0, 0]), c=np.array([1.0]),
        max_sense=False, x=np.array([1.0]), s=np.ones(6),
        y=np.array([1 / 3, -1 / 6, 1 / 3, -1 / 6, -1 / 6, 1 / 3]),
        forward=[dict(dA=np.zeros((6, 1)), db=np.ones(6), dc=np.zeros(1),
                      dx=np.array([-0.5]), atol=1e-2, rtol=2e-4),
                 dict(dA=np.zeros((6, 1)), db=np.zeros(6), dc=np.ones(1),
                      dx=np.array([0.0]), atol=1e-2, rtol=2e-4)],
        reverse=[]))
    # test/conic_program.jl:378-579 (PSD + POS, MAX sense); rows Zeros(1),
    # Nonnegatives(1), Nonnegatives(6), PSD-triangle(3) as in the test's s/y
    x = np.array([20 / 3.0, 0.0, 10 / 3.0, 0.0, 0.0, 0.0, 1.90192379])
    al, de = 0.8, 0.9
    A_moi = np.zeros((11, 7))
    # c4: Zeros, all-zero coefficients
    A_moi[1, 0:6] = -1.0                      # c1: η − Σ x[1:6] ≥ 0
    for i in range(6):
        A_moi[2 + i, i] = 1.0                 # c2: x[1:6] ≥ 0
    rows = [1] * 7 + [2] * 5 + [3] * 6        # c3 terms (output index)
    coef = [de / 2, al, de, de / 4, de / 8, 0.0, -1.0,
            -de / (2 * R2), -de / 4, 0, -de / (8 * R2), 0.0,
            de / 2, de - al, 0, de / 8, de / 4, -1.0]
    var = [0, 1, 2, 3, 4, 5, 6, 0, 1, 2, 4, 5, 0, 1, 2, 4, 5, 6]
    for r, cf, j in zip(rows, coef, var):
        A_moi[7 + r, j] += cf
    b_moi = np.zeros(11)
    b_moi[1] = 10.0
    s = np.array([0.0, 0.0, 20 / 3.0, 0.0, 10 / 3.0, 0.0, 0.0, 0.0,
                  4.09807621, -2.12132, 1.09807621])
    y = np.array([0.0, 0.19019238, 0.0, 0.12597667, 0.0, 0.14264428,
                  0.14264428, 0.01274047, 0.21132487, 0.408248, 0.78867513])
    fx.append(dict(
        name="conic_psd_pos", source="test/conic_program.jl:378-579",
        cones=[[0, 1], [1, 1], [1, 6], [4, 3]], A=A_moi, b=b_moi,
        c=np.array([0, 0, 0, 0, 0, 0, 1.0]), max_sense=True, x=x, s=s, y=y,
        forward=[dict(dA=np.ones((11, 7)), db=np.ones(11), dc=np.ones(7),
                      dx=np.array([-39.6066, 10.8953, -14.9189, 10.9054,
                                   10.883, 10.9118, -21.7508]),
                      atol=0.3, rtol=0.01)],
        reverse=[]))
    return fx


def main():
    for name, fx in [("qp", qp_fixtures()), ("lp", lp_fixtures()),
                     ("conic", conic_fixtures())]:
        path = os.path.join(OUT, f"{name}_fixtures.json")
        with open(path, "w") as f:
            json.dump([_lists(d) for d in fx], f, indent=1)
        print("wrote", path, len(fx))


if __name__ == "__main__":
    main()
