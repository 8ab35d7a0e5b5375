"""Transcribe the reference's NonLinearProgram known-answer tests into JSON
golden fixtures (tests/golden/nlp_fixtures.json).

Run once in the build container (reads /root/reference/test/data for the
QP-data problem):  python tests/golden/make_nlp_golden.py

Each fixture holds (a) a problem from test/nlp_program.jl or
test/data/nlp_problems.jl, (b) its primal-dual point — Ipopt is not
available, so the point is derived here exactly (closed form / the active
set's square KKT system; the problems are small and strictly complementary)
in MOI's dual convention (``ConstraintDual``: ≥ rows and lower bounds ≥ 0,
≤ rows and upper bounds ≤ 0, stationarity ∇f − sense·Σ yᵢ∇cᵢ = 0), (c) the
derivatives the MOI Nonlinear evaluator would return at that point
(Hessian of ``f − sense·yᵀc``, constraint Jacobian; written out by hand),
and (d) the expected sensitivities: the test's own analytic values, or — for
the tests that compare against ``FiniteDiff.finite_difference_jacobian`` of
re-solved problems — central differences of the exact solution map here.
Nothing in here is the oracle: tests/test_nlp_oracle.py checks oracle/nlp.py
against these values.
"""

import json
import math
import os

import numpy as np

REF = "/root/reference/test"
OUT = os.path.dirname(os.path.abspath(__file__))


def _lists(v):
    if isinstance(v, np.ndarray):
        return v.tolist()
    if isinstance(v, dict):
        return {k: _lists(e) for k, e in v.items()}
    if isinstance(v, (list, tuple)):
        return [_lists(e) for e in v]
    return v


def fixture(name, source, con_kind, has_low, has_up, sense, point, **extra):
    n = len(has_low)
    c = len(con_kind)
    P = np.asarray(point["Hxp"]).shape[1]
    full = dict(xl=np.zeros(n), xu=np.zeros(n), yl=np.zeros(n), yu=np.zeros(n), cval=np.zeros(c),
                crhs=np.zeros(c), y=np.zeros(c))
    full.update(point)
    for k in ("Hxx", "Hxp", "Jx", "Jp"):
        full[k] = np.asarray(full[k], dtype=float).reshape({"Hxx": (n, n), "Hxp": (n, P), "Jx": (c, n),
                                                            "Jp": (c, P)}[k])
    d = dict(name=name, source=source, con_kind=list(con_kind), has_low=[int(b) for b in has_low],
             has_up=[int(b) for b in has_up], sense=sense, point=full)
    d.update(extra)
    return d


# ---------------------------------------------------------------------------
# test/nlp_program.jl:334-499 — DICT_PROBLEMS_Analytical_no_cc (one variable x,
# one parameter p; linear constraints, so the Hessian is ∇²f alone)
# ---------------------------------------------------------------------------
def analytical():
    out = []

    def one(name, gen, p, dp, dx, dy, dvl, x, cons, sense, hxx, bounds=None):
        # cons: list of (kind, Jx, Jp, cval, crhs, y)
        kind = [k for k, *_ in cons]
        low = [bounds is not None and "low" in bounds]
        up = [bounds is not None and "up" in bounds]
        pt = dict(Hxx=[[hxx]], Hxp=[[0.0]], Jx=[[j] for _, j, *_ in cons], Jp=[[jp] for _, _, jp, *_ in cons],
                  x=[x], cval=[cv for *_, cv, _, _ in cons], crhs=[cr for *_, cr, _ in cons],
                  y=[yy for *_, yy in cons])
        if bounds:
            for k, v in bounds.items():
                pt.update({("xl" if k == "low" else "xu"): [v[0]], ("yl" if k == "low" else "yu"): [v[1]]})
        exp = dict(dx=dx, dy=dy)
        if dvl is not None:
            exp["dvl"] = dvl
        out.append(fixture(name, f"test/nlp_program.jl:334-499 ({name}); test/data/nlp_problems.jl ({gen})",
                           kind, low, up, sense, pt, p=[p], fwd=dict(dp=[dp]), expect_fwd=exp, atol=1e-4))

    # create_jump_model_1: min x², con1: x − p ≥ 0, con2: x ≥ 2
    one("geq no impact", "create_jump_model_1", 1.5, 0.2, [0.0], [0.0, 0.0], None, 2.0,
        [(1, 1.0, -1.0, 2.0 - 1.5, 0.0, 0.0), (1, 1.0, 0.0, 2.0, 2.0, 4.0)], 1, 2.0)
    one("geq impact", "create_jump_model_1", 2.1, 0.2, [0.2], [0.4, 0.0], None, 2.1,
        [(1, 1.0, -1.0, 0.0, 0.0, 4.2), (1, 1.0, 0.0, 2.1, 2.0, 0.0)], 1, 2.0)
    # create_jump_model_2: x ≥ 2 (bound), con1: x − p ≥ 0, min x²
    one("geq bound impact", "create_jump_model_2", 2.1, 0.2, [0.2], [0.4], [0.0], 2.1,
        [(1, 1.0, -1.0, 0.0, 0.0, 4.2)], 1, 2.0, bounds={"low": (2.0, 0.0)})
    # create_jump_model_3: min −x, con1: x − p ≤ 0, con2: x ≤ −2
    one("leq no impact", "create_jump_model_3", -1.5, -0.2, [0.0], [0.0, 0.0], None, -2.0,
        [(2, 1.0, -1.0, -2.0 + 1.5, 0.0, 0.0), (2, 1.0, 0.0, -2.0, -2.0, -1.0)], 1, 0.0)
    one("leq impact", "create_jump_model_3", -2.1, -0.2, [-0.2], [0.0, 0.0], None, -2.1,
        [(2, 1.0, -1.0, 0.0, 0.0, -1.0), (2, 1.0, 0.0, -2.1, -2.0, 0.0)], 1, 0.0)
    # create_jump_model_4: max x, con1: x − p ≤ 0, con2: x ≤ 2
    one("leq no impact max", "create_jump_model_4", 2.1, 0.2, [0.0], [0.0, 0.0], None, 2.0,
        [(2, 1.0, -1.0, 2.0 - 2.1, 0.0, 0.0), (2, 1.0, 0.0, 2.0, 2.0, -1.0)], -1, 0.0)
    one("leq impact max", "create_jump_model_4", 1.5, 0.2, [0.2], [0.0, 0.0], None, 1.5,
        [(2, 1.0, -1.0, 0.0, 0.0, -1.0), (2, 1.0, 0.0, 1.5, 2.0, 0.0)], -1, 0.0)
    # create_jump_model_5: max −x, con1: x − p ≥ 0, con2: x ≥ 2
    one("geq no impact max", "create_jump_model_5", 1.5, 0.2, [0.0], [0.0, 0.0], None, 2.0,
        [(1, 1.0, -1.0, 2.0 - 1.5, 0.0, 0.0), (1, 1.0, 0.0, 2.0, 2.0, 1.0)], -1, 0.0)
    one("geq impact max", "create_jump_model_5", 2.1, 0.2, [0.2], [0.0, 0.0], None, 2.1,
        [(1, 1.0, -1.0, 0.0, 0.0, 1.0), (1, 1.0, 0.0, 2.1, 2.0, 0.0)], -1, 0.0)
    return out


# ---------------------------------------------------------------------------
# test/nlp_program.jl:121-328 — test_analytical_simple (P = 2): min Σx,
# x_i − p_i ≥ 0 at p = 0.5, bounds 0 ≤ x ≤ 1 as variable bounds or as rows;
# test_ReverseConstraintDual (:711-753); test_changing_factorization (:797-857)
# ---------------------------------------------------------------------------
def simple():
    out = []
    P = 2
    I2 = np.eye(P)
    base = dict(Hxx=np.zeros((P, P)), Hxp=np.zeros((P, P)), x=np.full(P, 0.5))
    # bounds as variable bounds (VariableIndex-in-GreaterThan / LessThan)
    pt = dict(base, Jx=I2, Jp=-I2, cval=np.zeros(P), crhs=np.zeros(P), y=np.ones(P),
              xl=np.zeros(P), xu=np.ones(P), yl=np.zeros(P), yu=np.zeros(P))
    out.append(fixture("simple bounds bounds", "test/nlp_program.jl:122-195", [1] * P, [1] * P, [1] * P, 1, pt,
                       fwd=dict(dp=np.full(P, 0.1)),
                       expect_fwd=dict(dx=np.full(P, 0.1), dy=np.zeros(P)), atol=1e-8))
    # bounds as constraint rows: x ≥ 0 (2 rows), x ≤ 1 (2 rows), x − p ≥ 0 (2 rows)
    Jx = np.vstack([I2, I2, I2])
    Jp = np.vstack([np.zeros((P, P)), np.zeros((P, P)), -I2])
    pt = dict(base, Jx=Jx, Jp=Jp, cval=np.concatenate([np.full(P, 0.5), np.full(P, 0.5), np.zeros(P)]),
              crhs=np.concatenate([np.zeros(P), np.ones(P), np.zeros(P)]),
              y=np.concatenate([np.zeros(P), np.zeros(P), np.ones(P)]))
    out.append(fixture("simple bounds as rows", "test/nlp_program.jl:196-239, 797-857",
                       [1] * P + [2] * P + [1] * P, [0] * P, [0] * P, 1, pt, fwd=dict(dp=np.full(P, 0.1)),
                       expect_fwd=dict(dx=np.full(P, 0.1)), atol=1e-8))
    # test_ReverseConstraintDual: x free, x − p ≥ 0; reverse with Δλ = 0.1 → Δp = 0
    pt = dict(base, Jx=I2, Jp=-I2, cval=np.zeros(P), crhs=np.zeros(P), y=np.ones(P))
    out.append(fixture("reverse constraint dual", "test/nlp_program.jl:711-753", [1] * P, [0] * P, [0] * P, 1,
                       pt, rev=dict(dx=np.zeros(P), ddual=np.full(P, 0.1)), expect_rev=dict(dp=np.zeros(P)),
                       atol=1e-8))
    return out


# ---------------------------------------------------------------------------
# test/nlp_program.jl:514-642 — finite-difference tests, QP_sIpopt and NLP_1
# (create_nonlinear_jump_model_sipopt / _1), ismin ∈ {true, false}
# ---------------------------------------------------------------------------
def jac_fd(fun, p, h=1e-6):
    p = np.asarray(p, dtype=float)
    cols = []
    for j in range(len(p)):
        e = np.zeros(len(p))
        e[j] = h * max(1.0, abs(p[j]))
        cols.append((fun(p + e) - fun(p - e)) / (2 * e[j]))
    return np.stack(cols, axis=1)


def sipopt_solution(p):
    """min Σx², 6x1+3x2+2x3 − p1 = 0, p2x1 + x2 − x3 − 1 = 0, x ≥ 0: the
    active set {both equalities, x3 ≥ 0} (strictly complementary at p_a)."""
    p1, p2 = p
    x1 = (p1 - 3.0) / (6.0 - 3.0 * p2)
    x = np.array([x1, 1.0 - p2 * x1, 0.0])
    # stationarity of min Σx² (MOI: ∇f = Σ yᵢ∇cᵢ + yl): rows 1, 2 → (y1, y2)
    y = np.linalg.solve(np.array([[6.0, p2], [3.0, 1.0]]), 2.0 * x[:2])
    yl3 = 2.0 * x[2] - 2.0 * y[0] + y[1]
    return x, y, np.array([0.0, 0.0, yl3])


def sipopt():
    out = []
    p_a, dp = np.array([4.5, 1.0]), np.array([0.001, 0.0])
    for sense in (1, -1):
        x, y, yl = sipopt_solution(p_a)
        assert yl[2] > 1e-3 and np.all(x[:2] > 1e-3)
        g = -sense   # μ = −sense·y; ∇²f = ±2I
        Hxx = 2.0 * sense * np.eye(3)
        Hxp = np.zeros((3, 2))
        Hxp[0, 1] = g * y[1]   # ∂²c2/∂x1∂p2 = 1
        Jx = np.array([[6.0, 3.0, 2.0], [p_a[1], 1.0, -1.0]])
        Jp = np.array([[-1.0, 0.0], [0.0, x[0]]])
        sol = lambda p: np.concatenate(sipopt_solution(p)[:2])
        ds = jac_fd(sol, p_a) @ dp
        pt = dict(Hxx=Hxx, Hxp=Hxp, Jx=Jx, Jp=Jp, x=x, cval=np.zeros(2), crhs=np.zeros(2), y=y, xl=np.zeros(3),
                  yl=yl)
        out.append(fixture(f"QP_sIpopt {'min' if sense == 1 else 'max'}",
                           "test/nlp_program.jl:514-642 (QP_sIpopt); test/data/nlp_problems.jl:34-48",
                           [0, 0], [1, 1, 1], [0, 0, 0], sense, pt, p=p_a, fwd=dict(dp=dp),
                           expect_fwd=dict(dx=ds[:3], dy=ds[3:]), atol=1e-4))
    return out


def nlp1_solution(p):
    """create_nonlinear_jump_model_1 at p = (p1, p2, p3): con1 (y − p1 sin x ≥
    0) and con2 (x + y − p1 = 0) active, con3 (p2 x ≥ 0.1) inactive — the
    vertex x: p1 − x − p1 sin x = 0, y = p1 − x; duals from stationarity."""
    p1, p2, p3 = p
    x = 0.8
    for _ in range(60):   # Newton on p1 − x − p1 sin x
        x -= (p1 - x - p1 * math.sin(x)) / (-1.0 - p1 * math.cos(x))
    y = p1 - x
    fx = -2.0 * (1.0 - x) - 4.0 * p3 * x * (y - x * x)
    fy = 2.0 * p3 * (y - x * x)
    # ∇f = y1∇c1 + y2∇c2 (y3 = 0): ∇c1 = (−p1 cos x, 1), ∇c2 = (1, 1)
    yd = np.linalg.solve(np.array([[-p1 * math.cos(x), 1.0], [1.0, 1.0]]), np.array([fx, fy]))
    return np.array([x, y]), np.array([yd[0], yd[1], 0.0])


def nlp1():
    out = []
    p_a = np.array([3.0, 2.0, 200.0])
    # the DICT_PROBLEMS_no_cc entries for create_nonlinear_jump_model_1
    dps = {"NLP_1": [0.001, 0.0, 0.0], "NLP_1_2": [0.0, 0.001, 0.0], "NLP_1_3": [0.0, 0.0, 0.001],
           "NLP_1_4": [0.5, -0.5, 0.1]}
    xy, yv = nlp1_solution(p_a)
    x, y = xy
    p1, p2, p3 = p_a
    assert yv[0] > 1e-3 and p2 * x - 0.1 > 1e-3
    sol = lambda p: np.concatenate(nlp1_solution(p))
    J = jac_fd(sol, p_a)
    for sense in (1, -1):
        f_xx = 2.0 - 4.0 * p3 * y + 12.0 * p3 * x * x
        f_xy = -4.0 * p3 * x
        f_yy = 2.0 * p3
        mu = -sense * yv   # Hessian of sense·f ... written as ∇²(f_s) + Σ μ_i ∇²c_i with f_s = sense·f
        Hxx = np.array([[sense * f_xx + mu[0] * p1 * math.sin(x), sense * f_xy], [sense * f_xy, sense * f_yy]])
        Hxp = np.array([[mu[0] * (-math.cos(x)), mu[2] * 1.0, sense * (-4.0 * x * (y - x * x))],
                        [0.0, 0.0, sense * 2.0 * (y - x * x)]])
        Jx = np.array([[-p1 * math.cos(x), 1.0], [1.0, 1.0], [p2, 0.0]])
        Jp = np.array([[-math.sin(x), 0.0, 0.0], [-1.0, 0.0, 0.0], [0.0, x, 0.0]])
        cval = np.array([y - p1 * math.sin(x), x + y - p1, p2 * x])
        crhs = np.array([0.0, 0.0, 0.1])
        pt = dict(Hxx=Hxx, Hxp=Hxp, Jx=Jx, Jp=Jp, x=xy, cval=cval, crhs=crhs, y=yv)
        for nm, dp in dps.items():
            ds = J @ np.array(dp)
            out.append(fixture(f"{nm} {'min' if sense == 1 else 'max'}",
                               f"test/nlp_program.jl:514-642 ({nm}); test/data/nlp_problems.jl:191-213",
                               [1, 0, 1], [0, 0], [0, 0], sense, pt, p=p_a, fwd=dict(dp=dp),
                               expect_fwd=dict(dx=ds[:2], dy=ds[2:]), atol=1e-4))
    return out


# ---------------------------------------------------------------------------
# test/nlp_program.jl:651-709 — test_differentiating_non_trivial_convex_qp_jump:
# min xᵀQx + qᵀx, Gx − p_le ≤ h, Ax − p_eq = b (test/data/*.txt); reverse with
# Δx = 1 → Δp_le ≈ dh, Δp_eq ≈ db (atol = rtol = 1e-2)
# ---------------------------------------------------------------------------
def qp_data():
    import itertools
    rd = lambda nm: np.loadtxt(os.path.join(REF, "data", nm + ".txt"), ndmin=2)
    Q, q, G, h, A, b = (rd(k) for k in ("P", "q", "G", "h", "A", "b"))
    q, h, b = q.ravel(), h.ravel(), b.ravel()
    n, m, p = Q.shape[0], G.shape[0], A.shape[0]
    H = Q + Q.T
    # exact KKT point: the smallest active set whose square system is primal-
    # and dual-feasible (OptNet signs: Hx + q + Gᵀλ + Aᵀν = 0, λ ≥ 0)
    found = None
    for k in range(0, 4):   # the point has few active rows; stop early otherwise
        for act in itertools.combinations(range(m), k):
            act = list(act)
            K = np.zeros((n + k + p, n + k + p))
            K[:n, :n] = H
            K[:n, n:n + k] = G[act].T
            K[:n, n + k:] = A.T
            K[n:n + k, :n] = G[act]
            K[n + k:, :n] = A
            try:
                s = np.linalg.solve(K, np.concatenate([-q, h[act], b]))
            except np.linalg.LinAlgError:
                continue
            x = s[:n]
            lam = np.zeros(m)
            lam[act] = s[n:n + k]
            if np.all(G @ x - h <= 1e-9) and np.all(lam >= -1e-12):
                found = (x, lam, s[n + k:])
                break
        if found:
            break
    x, lam, nu = found
    Jx = np.vstack([G, A])
    Jp = -np.eye(m + p)
    pt = dict(Hxx=H, Hxp=np.zeros((n, m + p)), Jx=Jx, Jp=Jp, x=x, cval=np.concatenate([G @ x, A @ x]),
              crhs=np.concatenate([h, b]), y=np.concatenate([-lam, -nu]))
    return [fixture("QP data reverse", "test/nlp_program.jl:651-709; test/data/{P,q,G,h,A,b,dh,db}.txt",
                    [2] * m + [0] * p, [0] * n, [0] * n, 1, pt, rev=dict(dx=np.ones(n), ddual=np.zeros(m + p)),
                    expect_rev=dict(dp=np.concatenate([rd("dh").ravel(), rd("db").ravel()])), atol=1e-2,
                    rtol=1e-2)]


# ---------------------------------------------------------------------------
# test/nlp_program.jl:761-795 — test_inertia_correction: a singular KKT
# Jacobian, _inertia_correction(M, 3, 2) must factorise
# ---------------------------------------------------------------------------
def inertia():
    x1, x2 = 0.33, 0.33
    l1, l2 = 0.333, 0.0
    mu = 0.0
    M = np.array([[0, 0, -1, -2, -1], [0, 0, -2, -1, 0], [-l1, -2 * l1, 1 - x1 - 2 * x2, 0, 0],
                  [-2 * l2, -l2, 0, 1 - 2 * x1 - x2, 0], [mu, 0, 0, 0, x1]], dtype=float)
    return dict(name="inertia correction", source="test/nlp_program.jl:761-795", M=M, num_cons=3, num_w=2,
                expect=dict(singular=True, corrected=True))


def main():
    fx = analytical() + simple() + sipopt() + nlp1() + qp_data()
    doc = dict(fixtures=fx, kkt=[inertia()])
    with open(os.path.join(OUT, "nlp_fixtures.json"), "w") as f:
        json.dump(_lists(doc), f, indent=1)
    print(f"wrote {len(fx)} NLP fixtures + 1 KKT fixture")


if __name__ == "__main__":
    main()
