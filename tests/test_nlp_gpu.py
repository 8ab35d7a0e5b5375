"""NLP back-end on the GPU (csrc/nlp.hip through the C-ABI) against the
oracle (oracle/nlp.py, pinned by tests/test_nlp_oracle.py) and the
reference's own expected values: the golden fixtures, seeded synthetic
batches (mixed row kinds, bounds, MIN and MAX, both LU routes), the inertia
correction (KKT mode with the reference's singular matrix, and a structured
problem with a dependent constraint), device-mode inputs and the adjoint
identity.  Bar: north_star's 1e-6 relative Frobenius against the oracle (the
fixtures additionally at their reference tolerance)."""

import json
import os

import numpy as np
import pytest

from oracle import nlp as onlp

pytestmark = pytest.mark.gpu
RTOL = 1e-6
GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "nlp_fixtures.json")))
KEYS = ["Hxx", "Hxp", "Jx", "Jp", "x", "cval", "crhs", "y", "xl", "xu", "yl", "yu"]


def relfro(a, b):
    a, b = np.asarray(a, dtype=float), np.asarray(b, dtype=float)
    nb = np.linalg.norm(b)
    return np.linalg.norm(a - b) / (nb if nb > 0 else 1.0)


@pytest.fixture(params=["nopiv", "pivot"])
def lu_mode(request, monkeypatch):
    if request.param == "pivot":
        monkeypatch.setenv("DOPT_LU", "0")
    else:
        monkeypatch.delenv("DOPT_LU", raising=False)
    return request.param


def engine(st, pt, B):
    from diffopt_amd.nlp import NLPBatch
    n = pt["x"].shape[1]
    c = pt["Jx"].shape[1]
    P = pt["Hxp"].shape[2]
    e = NLPBatch(B, n, c, P)
    e.set_structure(st["con_kind"], st["has_low"], st["has_up"], st["sense"])
    e.set(*[pt[k] for k in KEYS])
    e.factor()
    return e


def oracle_problem(st, pt, b):
    return onlp.compute_sensitivity(st["con_kind"], st["has_low"], st["has_up"], st["sense"],
                                    *[pt[k][b] for k in KEYS], return_info=True)


def check_against_oracle(e, st, pt, dp, dx, dd, problems):
    fx, fd = e.forward(dp)
    rp = e.reverse(dx, dd)
    J = e.jacobian()
    worst = 0.0
    for b in problems:
        ds, L, M, N, corr = oracle_problem(st, pt, b)
        ox, od = onlp.forward(ds, L, dp[b])
        op = onlp.reverse(ds, L, dx[b], dd[b])
        # the forward output as one vector (∂s·Δp restricted to primal and duals):
        # a block can be ~0 in exact arithmetic (NLP_1_3: x does not depend on p3)
        worst = max(worst, relfro(np.concatenate([fx[b], fd[b]]), np.concatenate([ox, od])), relfro(rp[b], op),
                    relfro(J[b], ds))
    assert worst <= RTOL, worst
    return fx, fd, rp, J


# ---- golden fixtures -------------------------------------------------------
def _fixture_batch(f, B=2):
    st = dict(con_kind=np.asarray(f["con_kind"], np.int32), has_low=np.asarray(f["has_low"], np.int8),
              has_up=np.asarray(f["has_up"], np.int8), sense=f["sense"])
    pt = {k: np.stack([np.asarray(f["point"][k], dtype=float)] * B) for k in KEYS}
    return st, pt


@pytest.mark.parametrize("f", GOLD["fixtures"], ids=lambda f: f["name"])
def test_fixture(f, lu_mode):
    st, pt = _fixture_batch(f)
    e = engine(st, pt, 2)
    assert (e.corrections() == 0).all()
    B, P = 2, pt["Hxp"].shape[2]
    nd = e.ndual
    rng = np.random.default_rng(11)
    dp = np.stack([np.asarray(f["fwd"]["dp"], float)] * B) if "fwd" in f else rng.standard_normal((B, P))
    if "rev" in f:
        dx = np.stack([np.asarray(f["rev"]["dx"], float)] * B)
        dd = np.stack([np.asarray(f["rev"]["ddual"], float)] * B)
    else:
        dx, dd = rng.standard_normal((B, pt["x"].shape[1])), rng.standard_normal((B, nd))
    fx, fd, rp, _ = check_against_oracle(e, st, pt, dp, dx, dd, range(B))
    tol = dict(atol=f["atol"], rtol=f.get("rtol", 0.0))
    c, nlowp = len(f["con_kind"]), e.layout()["nlow_primal"]
    for key, want in f.get("expect_fwd", {}).items():
        got = {"dx": fx[0], "dy": fd[0, :c], "dvl": fd[0, c:c + nlowp], "dvu": fd[0, c + nlowp:]}[key]
        np.testing.assert_allclose(got, want, err_msg=key, **tol)
    if "expect_rev" in f:
        np.testing.assert_allclose(rp[0], f["expect_rev"]["dp"], **tol)


# ---- synthetic batches -----------------------------------------------------
@pytest.mark.parametrize("sense", [1, -1])
def test_synthetic_batch(lu_mode, sense):
    from diffopt_amd.synthetic import nlp_numpy
    st, pt, dp, dx, dd = nlp_numpy(8, 60, 40, 7, 1234 + sense, sense=sense)
    e = engine(st, pt, 8)
    lay = e.layout()
    assert lay["rows"] == onlp.Layout(st["con_kind"], st["has_low"], st["has_up"]).rows
    check_against_oracle(e, st, pt, dp, dx, dd, range(8))


def test_synthetic_multiblock():
    """M larger than one 64-column LU block step pair (rows ≈ 420): the
    blocked LU's paired trailing updates and the multi-RHS Jacobian."""
    from diffopt_amd.synthetic import nlp_numpy
    st, pt, dp, dx, dd = nlp_numpy(4, 150, 110, 20, 99)
    e = engine(st, pt, 4)
    assert e.layout()["rows"] > 256
    check_against_oracle(e, st, pt, dp, dx, dd, [0, 3])


def test_adjoint_identity():
    """⟨Δw, ∂s·Δp⟩ = ⟨∂sᵀΔw, Δp⟩ through the engine's two solves."""
    from diffopt_amd.synthetic import nlp_numpy
    st, pt, dp, dx, dd = nlp_numpy(6, 50, 30, 9, 5)
    e = engine(st, pt, 6)
    fx, fd = e.forward(dp)
    rp = e.reverse(dx, dd)
    lhs = np.einsum("bi,bi->b", dx, fx) + np.einsum("bi,bi->b", dd, fd)
    rhs = np.einsum("bi,bi->b", rp, dp)
    np.testing.assert_allclose(lhs, rhs, rtol=1e-10, atol=1e-12)


# ---- inertia correction ------------------------------------------------------
def test_kkt_mode_inertia_correction():
    """test_inertia_correction (test/nlp_program.jl:767-795) in KKT mode — the
    NonLinearKKTJacobianFactorization plug point: the singular M is corrected
    (k = 1, as the oracle) and K \\ rhs matches the oracle's corrected factor;
    a regular M in the same batch is not touched."""
    from diffopt_amd.nlp import NLPBatch
    k = GOLD["kkt"][0]
    M = np.asarray(k["M"], dtype=float)
    rng = np.random.default_rng(8)
    R = rng.standard_normal((5, 5)) + 5 * np.eye(5)
    Ms = np.stack([M, R, M])
    e = NLPBatch(3, 5, 0, 0)
    e.set_kkt(Ms, k["num_w"], k["num_cons"])
    e.factor()
    Ko, corr = onlp.inertia_correction(M, k["num_cons"], k["num_w"])
    np.testing.assert_array_equal(e.corrections(), [corr, 0, corr])
    rhs = rng.standard_normal((4, 3, 5))
    x = e.kkt_solve(rhs)
    for j in range(4):
        for b, want in ((0, Ko.solve(rhs[j, 0])), (1, np.linalg.solve(R, rhs[j, 1])), (2, Ko.solve(rhs[j, 2]))):
            assert relfro(x[j, b], want) <= 1e-8, (j, b)


def test_structured_dependent_constraint():
    """Two identical equality rows (LICQ fails): M is exactly singular, the
    inertia correction regularises it; the engine's correction count and ∂s
    match the oracle's."""
    from diffopt_amd.synthetic import nlp_numpy
    st, pt, dp, dx, dd = nlp_numpy(3, 20, 12, 4, 77)
    kinds = st["con_kind"]
    eq = np.flatnonzero(kinds == 0)
    assert len(eq) >= 2
    i, j = eq[:2]
    b = 1   # only problem 1 becomes singular
    pt["Jx"][b, j] = pt["Jx"][b, i]
    pt["Jp"][b, j] = pt["Jp"][b, i]
    e = engine(st, pt, 3)
    _, _, _, _, corr = oracle_problem(st, pt, b)
    assert corr >= 1
    got = e.corrections()
    assert got[0] == 0 and got[2] == 0 and got[1] == corr, (got, corr)
    fx, fd = e.forward(dp)
    ds, L, *_ = oracle_problem(st, pt, b)
    ox, od = onlp.forward(ds, L, dp[b])
    # the corrected system is ill-conditioned (shift 1e-6·k): a looser bar
    assert relfro(np.concatenate([fx[b], fd[b]]), np.concatenate([ox, od])) <= 1e-4


@pytest.mark.parametrize("shape", [(20, 12, 4), (100, 60, 8)], ids=["rows32", "rows160"])
def test_saddle_only(lu_mode, shape):
    """Equality constraints only, no bounds: M = [W Jxᵀ; Jx 0] is the one NLP
    shape the no-pivot LU takes (nlp.hip: saddle_only).  Its factor keeps the
    32×32 diagonal blocks only as inverses (dinv), so the singularity verdict
    must read u_ii from there: no correction may be applied (the reference's
    lu(M) is non-singular), and ∂s matches the oracle.  Rows 32 (one diagonal
    block) and 160 (a trailing update and a 32-wide last block)."""
    from diffopt_amd import _lib
    from diffopt_amd.synthetic import nlp_numpy
    n, c, P = shape
    st, pt, dp, dx, dd = nlp_numpy(4, n, c, P, 314, frac_geq=0, frac_leq=0, frac_low=0, frac_up=0)
    assert (st["con_kind"] == 0).all()
    e = engine(st, pt, 4)
    assert e.layout()["rows"] == n + c
    want = _lib.LU_KIND_NOPIV if lu_mode == "nopiv" else _lib.LU_KIND_PIVOT
    assert (e.lu_kind() == want).all(), e.lu_kind()
    for b in range(4):
        assert oracle_problem(st, pt, b)[4] == 0
    np.testing.assert_array_equal(e.corrections(), 0)
    check_against_oracle(e, st, pt, dp, dx, dd, range(4))


@pytest.mark.parametrize("shape", [(20, 12, 4), (100, 60, 8)], ids=["rows32", "rows160"])
def test_saddle_only_dependent_equality(lu_mode, shape):
    """A saddle-only problem with two identical equality rows: M is singular in
    exact arithmetic, but here no elimination order cancels the dependent
    pivot to exactly zero — SuperLU leaves 4e-16 (rows 32) / 8e-33 (rows 160)
    and does not flag it, and the reference's `lu(M; check=false).status`
    (NonLinearProgram.jl:408-409) is then decided by UMFPACK's rounding, pinned
    by no fixture.  The engine's rank-revealing verdict flags it and applies
    the reference's correction loop: the count must equal the oracle's
    `inertia_correction` on the same M (k = 1), and the regular neighbours are
    untouched and at parity."""
    from diffopt_amd.synthetic import nlp_numpy
    n, c, P = shape
    st, pt, dp, dx, dd = nlp_numpy(3, n, c, P, 2718, frac_geq=0, frac_leq=0, frac_low=0, frac_up=0)
    b = 1
    pt["Jx"][b, c - 1] = pt["Jx"][b, 0]
    pt["Jp"][b, c - 1] = pt["Jp"][b, 0]
    _, lay, M, _, _ = oracle_problem(st, pt, b)
    Md = np.asarray(M.todense() if hasattr(M, "todense") else M)
    corr = onlp.inertia_correction(Md, c, lay.num_w)[1]
    assert corr >= 1
    e = engine(st, pt, 3)
    got = e.corrections()
    assert got[0] == 0 and got[2] == 0 and got[1] == corr, (got, corr)
    check_against_oracle(e, st, pt, dp, dx, dd, [0, 2])


@pytest.mark.parametrize("delta", [1e-13, 1e-11])
def test_near_singular_verdict(lu_mode, delta):
    """The singularity verdict on a *near*-singular M:
    the dependent-row problem of test_structured_dependent_constraint with
    the duplicated row's Jacobian moved by delta·N(0,1).  The reference's
    lu(M; check = false) flags only an exactly zero pivot, so UMFPACK (and the
    oracle's SuperLU) factorise it without correction.  The engine's
    rank-revealing test |u_ii| ≤ rows·ε·max|M| ≈ 2.4e-14 (nlp.hip) sits 7×
    below the smallest pivot delta = 1e-13 leaves (1.7e-13), so it agrees:
    0 corrections, as the oracle.  (Below roughly rows·ε·max|M| ≈ 1e-14 the
    two rules can disagree: there UMFPACK's verdict depends on its rounding
    and ordering, and no fixture of the reference pins it.)"""
    from diffopt_amd.synthetic import nlp_numpy
    st, pt, dp, dx, dd = nlp_numpy(3, 20, 12, 4, 77)
    eq = np.flatnonzero(st["con_kind"] == 0)
    i, j = eq[:2]
    b = 1
    rng = np.random.default_rng(5)
    pt["Jx"][b, j] = pt["Jx"][b, i] + delta * rng.standard_normal(pt["Jx"].shape[2])
    pt["Jp"][b, j] = pt["Jp"][b, i]
    corr = oracle_problem(st, pt, b)[4]
    assert corr == 0
    e = engine(st, pt, 3)
    np.testing.assert_array_equal(e.corrections(), [0, corr, 0])
    check_against_oracle(e, st, pt, dp, dx, dd, [0, 2])


@pytest.mark.parametrize("reduce", ["1", "0"], ids=["reduced", "full"])
def test_interior_point_bounds_singularity_scale(monkeypatch, reduce):
    """interior-point duals leave an active bound at
    d = x − x_L ≈ 1e-9 with V ≈ 1, so the reduced route's eliminated-bound
    term δ = V/d is ≈ 1e9.  The singularity test's scale must be max |M| of the
    full M (|H|, |J|, |V|, |d|, 1), not max |R| (which holds δ): with max |R|
    the tolerance rows·ε·max|R| ≈ 1e-5 flags the regular pivots of a problem
    with modest curvature (H scaled by 1e-6: pivots ~1e-7) as singular and
    applies inertia corrections the reference's lu(M) (an exactly zero pivot
    only, NonLinearProgram.jl:394-422) never would.  Corrections must match the
    oracle's (0) on both routes, and the sensitivities the oracle."""
    from diffopt_amd.synthetic import nlp_numpy
    monkeypatch.setenv("DOPT_NLP_REDUCE", reduce)
    B, n, c, P = 3, 40, 20, 5
    st, pt, dp, dx, dd = nlp_numpy(B, n, c, P, 4242, frac_low=0.6, frac_up=0.4, active=0.5)
    moved = 0
    for b in range(B):
        for j in range(n):
            if st["has_low"][j] and pt["xl"][b, j] == pt["x"][b, j]:
                pt["xl"][b, j] -= 1e-9
                moved += 1
            if st["has_up"][j] and pt["xu"][b, j] == pt["x"][b, j]:
                pt["xu"][b, j] += 1e-9
                moved += 1
    assert moved >= 10
    pt["Hxx"][1] *= 1e-6
    for b in range(B):
        assert oracle_problem(st, pt, b)[4] == 0
    e = engine(st, pt, B)
    np.testing.assert_array_equal(e.corrections(), 0)
    check_against_oracle(e, st, pt, dp, dx, dd, range(B))
    e.close()


def test_config6_shape():
    """bench.py --config 6's shape (n = 200, c = 100, P = 20, 607 rows, partial
    pivoting): two problems of the bench generator vs the oracle at 1e-6."""
    from diffopt_amd.synthetic import SEED0, nlp_numpy
    st, pt, dp, dx, dd = nlp_numpy(2, 200, 100, 20, SEED0 + 6)
    e = engine(st, pt, 2)
    assert e.layout()["rows"] > 560
    np.testing.assert_array_equal(e.corrections(), 0)
    check_against_oracle(e, st, pt, dp, dx, dd, range(2))


# ---- memory modes and errors -------------------------------------------------
def test_device_mode_matches_host():
    import torch
    from diffopt_amd.nlp import NLPBatch
    from diffopt_amd.synthetic import nlp_numpy
    st, pt, dp, dx, dd = nlp_numpy(4, 30, 20, 5, 21)
    eh = engine(st, pt, 4)
    hx, hd = eh.forward(dp)
    hp = eh.reverse(dx, dd)
    t = lambda a: torch.as_tensor(a, device="cuda")
    ed = NLPBatch(4, 30, 20, 5)
    ed.set_structure(st["con_kind"], st["has_low"], st["has_up"], st["sense"])
    ed.set(*[t(pt[k]) for k in KEYS])
    ed.factor()
    gx, gd = ed.forward(t(dp))
    gp = ed.reverse(t(dx), t(dd))
    torch.cuda.synchronize()
    np.testing.assert_allclose(gx.cpu().numpy(), hx, rtol=1e-13, atol=1e-14)
    np.testing.assert_allclose(gd.cpu().numpy(), hd, rtol=1e-13, atol=1e-14)
    np.testing.assert_allclose(gp.cpu().numpy(), hp, rtol=1e-13, atol=1e-14)


def test_argument_errors():
    from diffopt_amd import EngineError
    from diffopt_amd.nlp import NLPBatch
    e = NLPBatch(2, 3, 2, 1)
    with pytest.raises(EngineError, match="set_structure"):
        e.set(np.zeros((2, 3, 3)), np.zeros((2, 3, 1)), np.zeros((2, 2, 3)), np.zeros((2, 2, 1)), np.zeros((2, 3)),
              np.zeros((2, 2)), np.zeros((2, 2)), np.zeros((2, 2)))
    with pytest.raises(EngineError, match="con_kind"):
        e.set_structure([0, 5])
    with pytest.raises(EngineError, match="sense"):
        e.set_structure([0, 1], sense=0)


# ---- the reduced KKT route (bounds and slacks eliminated exactly) ----------
@pytest.mark.parametrize("sense", [1, -1])
def test_reduced_route_sizes_and_parity(sense, monkeypatch):
    """Every strictly complementary problem takes the reduced route (system
    size n + c, no-pivot LU) and matches the oracle's full-M sensitivities;
    DOPT_NLP_REDUCE=0 (the full M) gives the same outputs to 1e-9."""
    from diffopt_amd.synthetic import nlp_numpy
    B, n, c, P = 6, 40, 25, 5
    st, pt, dp, dx, dd = nlp_numpy(B, n, c, P, 7100 + sense, sense=sense)
    monkeypatch.delenv("DOPT_NLP_REDUCE", raising=False)
    e = engine(st, pt, B)
    assert (e.system_size() == n + c).all()
    fx, fd, rp, J = check_against_oracle(e, st, pt, dp, dx, dd, range(B))
    e.close()
    monkeypatch.setenv("DOPT_NLP_REDUCE", "0")
    f = engine(st, pt, B)
    assert (f.system_size() == f.layout()["rows"]).all()
    gx, gd = f.forward(dp)
    assert relfro(np.concatenate([gx, gd], axis=1), np.concatenate([fx, fd], axis=1)) <= 1e-9
    assert relfro(f.reverse(dx, dd), rp) <= 1e-9
    assert relfro(f.jacobian(), J) <= 1e-9
    f.close()


def test_reduced_route_mixed_with_full_route():
    """One batch mixing problems the elimination cannot take — an active bound
    with a zero dual (M singular: the inertia correction on the full M), and a
    primal variable pinned by both bounds — with reduced ones: the reduced
    problems keep n + c, the others the full M, all match the oracle."""
    from diffopt_amd.synthetic import nlp_numpy
    B, n, c, P = 4, 30, 18, 4
    st, pt, dp, dx, dd = nlp_numpy(B, n, c, P, 7300)
    low = np.flatnonzero(st["has_low"])
    both = np.flatnonzero(st["has_low"].astype(bool) & st["has_up"].astype(bool))
    j = int(low[0])
    pt["xl"][1, j], pt["yl"][1, j] = pt["x"][1, j], 0.0   # problem 1: active lower bound, zero dual
    if len(both):
        k = int(both[0])                                   # problem 2: both bounds active on k
        pt["xl"][2, k] = pt["xu"][2, k] = pt["x"][2, k]
        pt["yl"][2, k], pt["yu"][2, k] = 0.7, -0.4
    e = engine(st, pt, B)
    sizes = e.system_size()
    rows = e.layout()["rows"]
    assert sizes[0] == n + c and sizes[3] == n + c
    assert sizes[1] == rows
    if len(both):
        assert sizes[2] == rows
    corr = e.corrections()
    for b in range(B):
        assert corr[b] == oracle_problem(st, pt, b)[4]
    check_against_oracle(e, st, pt, dp, dx, dd, range(B))
    e.close()


# ---- forward + reverse in one call (dopt_nlp_forward_reverse) ---------------
@pytest.mark.parametrize("case", ["synthetic", "full_route", "mixed_routes", "config6", "device", "no_seeds"])
def test_forward_reverse_equals_separate_calls(case, lu_mode, monkeypatch):
    """One call for both directions (the P-symmetric problems' solves as one
    pair launch over the factors) gives exactly the separate forward and
    reverse calls' outputs — the pair kernel does each direction's arithmetic
    in the same order — on the reduced and the full route, a batch mixing the
    two, config 6's shape, device-mode tensors and absent reverse seeds; and
    the outputs match the oracle at north_star's 1e-6."""
    import torch
    from diffopt_amd.synthetic import SEED0, nlp_numpy
    if case == "full_route":
        monkeypatch.setenv("DOPT_NLP_REDUCE", "0")
    shape = {"config6": (2, 200, 100, 20)}.get(case, (5, 40, 25, 6))
    B = shape[0]
    st, pt, dp, dx, dd = nlp_numpy(*shape, SEED0 + 6 if case == "config6" else 8100)
    if case == "mixed_routes":
        j = int(np.flatnonzero(st["has_low"])[0])
        pt["xl"][1, j], pt["yl"][1, j] = pt["x"][1, j], 0.0   # problem 1 leaves the reduced route
    if case == "no_seeds":
        dx = dd = None
    e = engine(st, pt, B)
    if case == "mixed_routes":   # problem 1 on the full M (partial pivoting: the factor's slow path)
        assert e.system_size()[1] == e.layout()["rows"] and e.corrections()[1] == oracle_problem(st, pt, 1)[4]
    fx, fd = e.forward(dp)
    rp = e.reverse(dx, dd)
    if case == "device":
        from diffopt_amd.nlp import NLPBatch
        t = lambda a: torch.as_tensor(a, device="cuda")
        ed = NLPBatch(*shape)
        ed.set_structure(st["con_kind"], st["has_low"], st["has_up"], st["sense"])
        ed.set(*[t(pt[k]) for k in KEYS])
        ed.factor()
        gx, gd, gp = (a.cpu().numpy() for a in ed.forward_reverse(t(dp), t(dx), t(dd)))
    else:
        gx, gd, gp = e.forward_reverse(dp, dx, dd)
    np.testing.assert_array_equal(gx, fx)
    np.testing.assert_array_equal(gd, fd)
    np.testing.assert_array_equal(gp, rp)
    zx = np.zeros_like(fx) if dx is None else dx
    zd = np.zeros_like(fd) if dd is None else dd
    for b in range(min(B, 2)):
        ds, L, *_ = oracle_problem(st, pt, b)
        ox, od = onlp.forward(ds, L, dp[b])
        assert relfro(np.concatenate([gx[b], gd[b]]), np.concatenate([ox, od])) <= RTOL
        assert relfro(gp[b], onlp.reverse(ds, L, zx[b], zd[b])) <= RTOL


# ---- the speculative LU launch (no metadata read-back before the LU) --------
@pytest.mark.parametrize("deferred", [False, True], ids=["sync", "deferred"])
@pytest.mark.parametrize("call", ["forward_reverse", "forward", "reverse", "jacobian"])
def test_speculative_launch_miss(call, deferred):
    """dopt_nlp_factor launches the LU on the guess that every problem is
    reduced and symmetric; a batch breaking it (problem 1 leaves the reduced
    route) is re-factorised from the read-back by the next call, whose right-
    hand sides were already queued — on a handle whose previous factorisation
    guessed right, and again on the same handle (guessing now off).  Each call
    matches a fresh engine's and the oracle."""
    from diffopt_amd.synthetic import nlp_numpy
    B, n, c, P = 4, 30, 18, 4
    st, good, dp, dx, dd = nlp_numpy(B, n, c, P, 7400)
    bad = {k: v.copy() for k, v in good.items()}
    j = int(np.flatnonzero(st["has_low"])[0])
    bad["xl"][1, j], bad["yl"][1, j] = bad["x"][1, j], 0.0
    e = engine(st, good, B)
    if deferred:   # opt-in: factor() returns with the LU queued, the next call finishes it
        e.lib.dopt_nlp_set_deferred(e.h, 1)
    assert (e.system_size() == n + c).all()

    def run(eng):
        if call == "forward_reverse":
            return eng.forward_reverse(dp, dx, dd)
        if call == "forward":
            return eng.forward(dp)
        if call == "reverse":
            return (eng.reverse(dx, dd),)
        return (eng.jacobian(),)

    for _ in range(2):
        e.set(*[bad[k] for k in KEYS])
        e.factor()
        # read straight after factor (in the deferred form the
        # finish step must run first — a missed guess changes the kinds / sizes)
        kinds, sizes = e.lu_kind(), e.system_size()
        got = run(e)
        assert e.system_size()[1] == e.layout()["rows"] and e.system_size()[0] == n + c
        ref = engine(st, bad, B)
        np.testing.assert_array_equal(kinds, ref.lu_kind())
        np.testing.assert_array_equal(sizes, ref.system_size())
        want = run(ref)
        for g, w in zip(got, want):
            np.testing.assert_allclose(g, w, rtol=0, atol=1e-12 * max(1.0, np.abs(w).max()))
        ref.close()
    ds, L, *_ = oracle_problem(st, bad, 1)
    if call in ("forward", "forward_reverse"):
        ox, od = onlp.forward(ds, L, dp[1])
        assert relfro(np.concatenate([got[0][1], got[1][1]]), np.concatenate([ox, od])) <= RTOL
    e.set(*[good[k] for k in KEYS])
    e.factor()
    check_against_oracle(e, st, good, dp, dx, dd, range(B))
    e.close()


def test_factor_contract_sync_and_deferred():
    """dopt_nlp_factor is synchronous at return by
    default (every verdict final, nothing queued — including the
    re-factorisation of a missed speculative launch); the deferred return is
    opt-in (dopt_nlp_set_deferred), documented in the header and INTEGRATION.md
    as needing the device-mode inputs unchanged until the next call.  Problem 1
    misses the speculative launch (it leaves the reduced route).  Both forms,
    inputs left alone, give bit-identical outputs, corrections and kinds, and
    match a fresh engine; switching the deferred form off finishes a pending
    factorisation."""
    import torch
    from diffopt_amd.nlp import NLPBatch
    from diffopt_amd.synthetic import nlp_numpy
    B, n, c, P = 4, 30, 18, 4
    st, pt, dp, dx, dd = nlp_numpy(B, n, c, P, 7401)
    j = int(np.flatnonzero(st["has_low"])[0])
    pt["xl"][1, j], pt["yl"][1, j] = pt["x"][1, j], 0.0
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a), device="cuda")
    outs = {}
    for deferred in (False, True):
        e = NLPBatch(B, n, c, P, deferred=deferred)
        e.set_structure(st["con_kind"], st["has_low"], st["has_up"], st["sense"])
        dev = {k: t(pt[k]) for k in KEYS}
        e.set(*[dev[k] for k in KEYS])
        e.factor()
        if deferred:   # off again: the pending factorisation is finished by the switch itself
            assert e.lib.dopt_nlp_set_deferred(e.h, 0) == 0
            assert e.lib.dopt_nlp_set_deferred(e.h, 1) == 0
        got = e.forward_reverse(t(dp), t(dx), t(dd))
        torch.cuda.synchronize()
        outs[deferred] = [g.cpu().numpy() for g in got] + [e.corrections(), e.lu_kind(), e.system_size()]
        e.close()
    for a, b in zip(outs[False], outs[True]):
        np.testing.assert_array_equal(a, b)
    ref = engine(st, pt, B)
    want = ref.forward_reverse(dp, dx, dd)
    for a, w in zip(outs[False], want):
        np.testing.assert_allclose(a, w, rtol=0, atol=1e-12 * max(1.0, np.abs(w).max()))
    ref.close()
