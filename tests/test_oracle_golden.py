"""Pin the CPU oracle against the reference's own known-answer tests
(tests/golden/*.json, transcribed by tests/golden/make_golden.py from
test/quadratic_program.jl, test/linear_program.jl, test/conic_program.jl and
test/data/*.txt).  CPU only."""

import json
import os

import numpy as np
import pytest

from oracle import cones, conic, lsqr, qp

HERE = os.path.dirname(os.path.abspath(__file__))


def _load(name):
    with open(os.path.join(HERE, "golden", name)) as f:
        return json.load(f)


def qp_arrays(fx):
    a = {k: np.array(v, dtype=float) for k, v in fx.items() if isinstance(v, list)}
    n = a["Q"].shape[0]
    a["G"] = a["G"].reshape(-1, n)
    a["A"] = a["A"].reshape(-1, n)
    fw = {k: np.array(v, dtype=float) for k, v in fx["fwd"].items()}
    if "dG" in fw:
        fw["dG"] = fw["dG"].reshape(a["G"].shape)
    if "dA" in fw:
        fw["dA"] = fw["dA"].reshape(a["A"].shape)
    return a, fw


def qp_outputs(a, fw, solve_rev=None, solve_fwd=None):
    """All quantities the reference tests check (test/utils.jl:147-312)."""
    Q, G, h, A, z, lam, nu = (a[k] for k in ["Q", "G", "h", "A", "z", "lam", "nu"])
    if solve_rev is None:
        dz, dl, dn = qp.reverse_differentiate(Q, G, h, A, z, lam, nu, a["dzb"])
        dzf, _, _ = qp.forward_differentiate(Q, G, h, A, z, lam, nu, **fw)
    else:
        dz, dl, dn = solve_rev()
        dzf = solve_fwd()
    dqb, dQb = qp.reverse_objective(z, dz)
    dGb, cle = qp.reverse_constraint_le(z, lam, dz, dl)
    dAb, ceq = qp.reverse_constraint_eq(z, nu, dz, dn)
    rhs = qp.forward_rhs(Q, G, h, A, z, lam, nu, **fw)
    return dict(z=z, dQb=dQb, dqb=dqb, dGb=dGb, dhb=-cle, dAb=dAb, dbb=-ceq,
                dzf=dzf, grad_zb=dz, grad_lamb=dl, grad_nub=dn,
                grad_zf=rhs[:Q.shape[0]])


QP_FX = _load("qp_fixtures.json") + _load("lp_fixtures.json")


@pytest.mark.parametrize("fx", QP_FX, ids=[f["name"] for f in QP_FX])
def test_qp_oracle_matches_reference_fixture(fx):
    a, fw = qp_arrays(fx)
    got = qp_outputs(a, fw)
    for k, v in fx["expect"].items():
        exp = np.array(v, dtype=float).reshape(np.shape(got[k]))
        np.testing.assert_allclose(got[k], exp, atol=fx["atol"], rtol=fx["rtol"], err_msg=k)


@pytest.mark.parametrize("fx", QP_FX, ids=[f["name"] for f in QP_FX])
def test_qp_optnet_identities(fx):
    """OptNet eq. (7)/(8) identities the reference asserts (test/utils.jl:236-261)."""
    a, fw = qp_arrays(fx)
    Q, G, h, A, z, lam, nu = (a[k] for k in ["Q", "G", "h", "A", "z", "lam", "nu"])
    dz, dl, dn = qp.reverse_differentiate(Q, G, h, A, z, lam, nu, a["dzb"])
    # eq. (7): −(Q∇z + Gᵀ(λ∘∇λ) + Aᵀ∇ν) = dl/dz
    np.testing.assert_allclose(-(Q @ dz + G.T @ (lam * dl) + A.T @ dn), a["dzb"], atol=1e-8)
    # −(G∇z + (Gz − h)∘∇λ) = 0 ; −A∇z = 0
    np.testing.assert_allclose(-(G @ dz + (G @ z - h) * dl), 0 * dl, atol=1e-8)
    np.testing.assert_allclose(-(A @ dz), np.zeros(A.shape[0]), atol=1e-8)


def test_qp_iterative_branch_selection():
    """`iterative = norm(Q) ≈ 0` is an exact-zero test (QuadraticProgram.jl:333)."""
    assert qp.is_iterative(np.zeros((3, 3)))
    assert not qp.is_iterative(np.eye(3) * 1e-300)
    assert not qp.is_iterative(np.full((2, 2), np.nan))
    assert qp.is_iterative(-np.zeros((2, 2)))


CONIC_FX = _load("conic_fixtures.json")


def _cache(fx, conv="S2JSm2"):
    return conic.Cache(np.array(fx["A"], dtype=float), fx["b"], fx["c"], fx["x"], fx["s"],
                       fx["y"], [tuple(c) for c in fx["cones"]], fx["max_sense"], conv)


@pytest.mark.parametrize("fx", CONIC_FX, ids=[f["name"] for f in CONIC_FX])
def test_conic_oracle_matches_reference_fixture(fx):
    cache = _cache(fx)
    for t in fx["forward"]:
        dx, *_ = conic.forward_differentiate(cache, np.array(t["dA"], dtype=float), t["db"], t["dc"])
        np.testing.assert_allclose(dx, t["dx"], atol=t["atol"], rtol=t["rtol"])
    for t in fx["reverse"]:
        g, _ = conic.reverse_differentiate(cache, t["dx"])
        _, db, _ = conic.reverse_outputs(cache, g)
        np.testing.assert_allclose(db[t["rows"]], t["db"], atol=t["atol"], rtol=t["rtol"])


def test_psd_convention_is_pinned_by_fixtures():
    """Only Dπ_PSD = S²JS⁻² (= Jᵀ) reproduces every PSD fixture."""
    def fits(conv):
        ok = True
        for fx in CONIC_FX:
            if "psd" not in fx["name"]:
                continue
            cache = _cache(fx, conv)
            for t in fx["forward"]:
                dx, *_ = conic.forward_differentiate(cache, np.array(t["dA"], dtype=float), t["db"], t["dc"])
                ok &= np.allclose(dx, t["dx"], atol=t["atol"], rtol=t["rtol"])
        return ok
    assert fits("S2JSm2")
    assert not fits("S2J")
    assert not fits("J")
    assert not fits("SJSinv")


def test_psd_dpi_is_transpose_of_unscaled_jacobian():
    rng = np.random.default_rng(0)
    v = rng.standard_normal(10)  # 4×4 triangle
    J = cones.psd_jacobian_unscaled(v)
    D = cones.dproj(cones.PSD, v)
    np.testing.assert_allclose(D, J.T, atol=1e-12)
    # J is the derivative of the projection (finite differences)
    eps = 1e-6
    for k in range(10):
        e = np.zeros(10)
        e[k] = eps
        fd = (cones.proj(cones.PSD, v + e) - cones.proj(cones.PSD, v - e)) / (2 * eps)
        np.testing.assert_allclose(J[:, k], fd, atol=1e-6)


def test_soc_projection_cases():
    t = np.array([2.0, 1.0, 0.0])      # ‖x‖ ≤ t
    np.testing.assert_allclose(cones.proj(cones.SOC, t), t)
    np.testing.assert_allclose(cones.dproj(cones.SOC, t), np.eye(3))
    t = np.array([-2.0, 1.0, 0.0])     # ‖x‖ ≤ −t
    np.testing.assert_allclose(cones.proj(cones.SOC, t), 0 * t)
    t = np.array([0.5, 3.0, 4.0])      # else
    p = cones.proj(cones.SOC, t)
    assert abs(np.linalg.norm(p[1:]) - p[0]) < 1e-12
    eps = 1e-6
    D = cones.dproj(cones.SOC, t)
    for k in range(3):
        e = np.zeros(3)
        e[k] = eps
        fd = (cones.proj(cones.SOC, t + e) - cones.proj(cones.SOC, t - e)) / (2 * eps)
        np.testing.assert_allclose(D[:, k], fd, atol=1e-6)


def test_lsqr_matches_lstsq_min_norm():
    rng = np.random.default_rng(1)
    A = rng.standard_normal((30, 20))
    b = rng.standard_normal(30)
    x = lsqr.lsqr_dense(A, b)
    np.testing.assert_allclose(x, np.linalg.lstsq(A, b, rcond=None)[0], rtol=1e-6, atol=1e-8)
    # rank-deficient consistent system → minimum-norm solution
    B = rng.standard_normal((20, 5)) @ rng.standard_normal((5, 20))
    xb = B @ rng.standard_normal(20)
    x = lsqr.lsqr_dense(B, xb)
    np.testing.assert_allclose(x, np.linalg.pinv(B) @ xb, rtol=1e-5, atol=1e-7)


def test_conic_matrix_free_products_match_dense_M():
    rng = np.random.default_rng(2)
    fx = CONIC_FX[-1]
    cache = _cache(fx)
    M = cache.M()
    v = rng.standard_normal(M.shape[0])
    np.testing.assert_allclose(cache.matvec(v), M @ v, atol=1e-12)
    np.testing.assert_allclose(cache.rmatvec(v), M.T @ v, atol=1e-12)


def test_structured_psd_matches_dense():
    """oracle.cones.PSDStructured (large PSD sides: Dπ through the
    eigendecomposition, no dense k × k Jacobian) equals the dense S²JS⁻²
    block and its transpose to rounding, including a PSD (identity) point."""
    from oracle import cones as C
    rng = np.random.default_rng(3)
    for d in (3, 12, 30):
        k = d * (d + 1) // 2
        for v in (rng.standard_normal(k), C.tri(np.eye(d) * 2.0)):
            Dd = C.dproj(C.PSD, v)
            S = C.PSDStructured(v)
            w = rng.standard_normal(k)
            np.testing.assert_allclose(S @ w, Dd @ w, rtol=1e-12, atol=1e-13)
            np.testing.assert_allclose(S.T @ w, Dd.T @ w, rtol=1e-12, atol=1e-13)


LP_FX = [f for f in _load("lp_fixtures.json") if not np.any(np.array(f["Q"], dtype=float))]


@pytest.mark.parametrize("fx", LP_FX, ids=[f["name"] for f in LP_FX])
def test_sparse_lp_oracle_matches_reference_fixture(fx):
    """The sparse route's checker (oracle/qp.py lp_sparse_differentiate: the
    reference's LHS built as a scipy CSC, never dense, + the LSQR restatement)
    pinned by the reference's own LP fixtures (test/linear_program.jl), for
    the fixtures whose forward tangents are vectors (dq, dh, db): its reverse
    reproduces the reference's expected values at the fixture's tolerances and
    both directions equal the dense oracle's to 1e-6."""
    import scipy.sparse as sp
    a, fw = qp_arrays(fx)
    if any(k in fw and fw[k].size and np.any(fw[k]) for k in ("dQ", "dG", "dA")):
        pytest.skip("matrix tangents: the sparse checker takes vector tangents only")
    n, m, p = a["Q"].shape[0], a["G"].shape[0], a["A"].shape[0]
    rev, fwd, _, _ = qp.lp_sparse_differentiate(sp.csc_matrix(a["G"]) if m else None, a["h"],
                                                sp.csc_matrix(a["A"]) if p else None, a["z"], a["lam"], a["nu"],
                                                a["dzb"], fw.get("dq"), fw.get("dh") if m else None,
                                                fw.get("db") if p else None)
    got = qp_outputs(a, fw, solve_rev=lambda: (rev[:n], rev[n:n + m], rev[n + m:]), solve_fwd=lambda: fwd[:n])
    for k, v in fx["expect"].items():
        exp = np.array(v, dtype=float).reshape(np.shape(got[k]))
        np.testing.assert_allclose(got[k], exp, atol=fx["atol"], rtol=fx["rtol"], err_msg=k)
    dz, dl, dn = qp.reverse_differentiate(a["Q"], a["G"], a["h"], a["A"], a["z"], a["lam"], a["nu"], a["dzb"])
    fz, fl, fn = qp.forward_differentiate(a["Q"], a["G"], a["h"], a["A"], a["z"], a["lam"], a["nu"], **fw)
    for got_v, ref in ((rev, np.concatenate([dz, dl, dn])), (fwd, np.concatenate([fz, fl, fn]))):
        assert np.linalg.norm(got_v - ref) <= 1e-6 * max(np.linalg.norm(ref), 1e-300)
