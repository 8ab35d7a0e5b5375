"""ConicProgram sensitivity path on the GPU (via the C-ABI) against the CPU
oracle and the reference's own fixtures (test/conic_program.jl, see
tests/golden/make_golden.py).  Tolerance: north_star's 1e-6 relative
Frobenius against the oracle; the fixture tolerances for the reference's
expected values."""

import json
import os

import numpy as np
import pytest

from oracle import conic as ocn

pytestmark = pytest.mark.gpu
RTOL = 1e-6
HERE = os.path.dirname(os.path.abspath(__file__))


def relfro(a, b):
    a, b = np.asarray(a, dtype=float).ravel(), np.asarray(b, dtype=float).ravel()
    nb = np.linalg.norm(b)
    return np.linalg.norm(a - b) / nb if nb > 0 else np.linalg.norm(a)


def relcomb(a, b, scale):
    """Relative error of an output derived linearly from the LSQR solution
    (dx = −(du − x·dw), dc = g_x − g_end·x, …), normalised by the bound that
    a 1e-6-relative error of the solution itself propagates to (`scale` =
    ‖solution‖ × the derivation's gain), so a component that cancels to ~0 in
    exact arithmetic is not judged on its rounding noise."""
    a, b = np.asarray(a, dtype=float).ravel(), np.asarray(b, dtype=float).ravel()
    den = max(np.linalg.norm(b), scale)
    return np.linalg.norm(a - b) / den if den > 0 else np.linalg.norm(a)


def noise_envelope(solve, args, ref, trials=4):
    """Rounding-noise envelope of the oracle at one input: the largest relative
    change of its output when the right-hand side data is perturbed by one ulp
    (relative 2⁻⁵², seeded).  For a singular M whose LSQR stops at maxiter
    (istop 7 — e.g. the PSD+POS fixture, cond(M) ≈ 8e16) this is ≫ 1e-6: the
    reference itself then returns a different vector under another BLAS or
    summation order, so no implementation can meet 1e-6 there.  The bar for
    such inputs is "within 10× the oracle's own 1-ulp spread" (plus the
    reference fixture's tolerance, asserted separately)."""
    rng = np.random.default_rng(7)
    worst = 0.0
    for _ in range(trials):
        pert = [np.asarray(a, float) * (1.0 + 2.0 ** -52 * rng.standard_normal(np.shape(a)))
                for a in args]
        worst = max(worst, relfro(solve(*pert), ref))
    return worst


def parity_bar(solve, args, ref):
    env = noise_envelope(solve, args, ref)
    return RTOL if env <= RTOL / 10 else 10.0 * env


@pytest.fixture(scope="module")
def ConicBatch():
    from diffopt_amd.conic import ConicBatch
    return ConicBatch


FX = json.load(open(os.path.join(HERE, "golden", "conic_fixtures.json")))


@pytest.mark.parametrize("fx", FX, ids=[f["name"] for f in FX])
def test_fixture_forward_reverse(ConicBatch, fx):
    A = np.array(fx["A"], dtype=float)
    m, n = A.shape
    cones = [tuple(c) for c in fx["cones"]]
    c = -np.array(fx["c"]) if fx["max_sense"] else np.array(fx["c"], dtype=float)
    cache = ocn.Cache(A, fx["b"], fx["c"], fx["x"], fx["s"], fx["y"], cones, fx["max_sense"])
    e = ConicBatch(1, n, cones)
    e.set(A[None], np.array(fx["b"])[None], c[None], np.array(fx["x"])[None],
          np.array(fx["s"])[None], np.array(fx["y"])[None])
    for t in fx["forward"]:
        dA = np.array(t["dA"], dtype=float)
        out, dx = e.forward(dA[None], np.array(t["db"])[None], np.array(t["dc"])[None])
        np.testing.assert_allclose(dx[0], t["dx"], atol=t["atol"], rtol=t["rtol"])
        odx, du, dv, dw = ocn.forward_differentiate(cache, dA, t["db"], t["dc"])
        ref = np.concatenate([du, dv, [dw]])

        def fsolve(dA_, db_, dc_):
            _, a, b_, c_ = ocn.forward_differentiate(cache, dA_, db_, dc_)
            return np.concatenate([a, b_, [c_]])
        bar = parity_bar(fsolve, [dA, t["db"], t["dc"]], ref)
        assert relfro(out[0], ref) <= bar
        x = np.array(fx["x"], dtype=float)
        sol = np.linalg.norm(ref)
        assert relcomb(dx[0], odx, sol * (1 + np.linalg.norm(x))) <= bar
    for t in fx["reverse"]:
        g, dA, db, dc = e.reverse(np.array(t["dx"], dtype=float)[None])
        np.testing.assert_allclose(db[0][t["rows"]], t["db"], atol=t["atol"], rtol=t["rtol"])
        og, _ = ocn.reverse_differentiate(cache, t["dx"])
        bar = parity_bar(lambda dx_: ocn.reverse_differentiate(cache, dx_)[0], [t["dx"]], og)
        assert relfro(g[0], og) <= bar
    e.close()


def _oracle_outputs(cache, dA, db, dc, dx):
    odx, du, dv, dw = ocn.forward_differentiate(cache, dA, db, dc)
    og, _ = ocn.reverse_differentiate(cache, dx)
    odA, odb, odc = ocn.reverse_outputs(cache, og)
    return dict(fwd=np.concatenate([du, dv, [dw]]), dx=odx, g=og, dA=odA, db=odb, dc=odc)


def _errors(got, ref, cache):
    """Per-output error metrics (relfro for the LSQR solutions, relcomb for
    the outputs derived from them)."""
    nx, nvp = np.linalg.norm(cache.x), np.linalg.norm(cache.vp)
    sol, ng = np.linalg.norm(ref["fwd"]), np.linalg.norm(ref["g"])
    return dict(fwd=relfro(got["fwd"], ref["fwd"]),
                dx=relcomb(got["dx"], ref["dx"], sol * (1 + nx)),
                g=relfro(got["g"], ref["g"]),
                dA=relcomb(got["dA"], ref["dA"], ng * (nx + nvp)),
                db=relcomb(got["db"], ref["db"], ng * (1 + nvp)),
                dc=relcomb(got["dc"], ref["dc"], ng * (1 + nx)))


def _synthetic_check(ConicBatch, B, n, cones, seed):
    """GPU vs oracle per problem and output.  Bar: RTOL, or 10× the oracle's
    own 1-ulp rounding envelope where that exceeds RTOL/10 (LSQR on the
    singular M — see noise_envelope)."""
    from diffopt_amd.synthetic import conic_numpy
    d = conic_numpy(B, n, cones, seed)
    e = ConicBatch(B, n, cones)
    e.set(d["A"], d["b"], d["c"], d["x"], d["s"], d["y"])
    out, dx = e.forward(d["dA"], d["db"], d["dc"])
    g, dA, db, dc = e.reverse(d["dx"])
    e.close()
    rng = np.random.default_rng(7)
    worst = {}
    for b in range(B):
        cache = ocn.Cache(d["A"][b], d["b"][b], d["c"][b], d["x"][b], d["s"][b], d["y"][b], cones)
        args = [d["dA"][b], d["db"][b], d["dc"][b], d["dx"][b]]
        ref = _oracle_outputs(cache, *args)
        got = dict(fwd=out[b], dx=dx[b], g=g[b], dA=dA[b], db=db[b], dc=dc[b])
        err = _errors(got, ref, cache)
        env = dict.fromkeys(err, 0.0)
        for _ in range(3):
            pert = [a * (1.0 + 2.0 ** -52 * rng.standard_normal(a.shape)) for a in args]
            pe = _errors(_oracle_outputs(cache, *pert), ref, cache)
            env = {k: max(env[k], pe[k]) for k in env}
        for k in err:
            bar = RTOL if env[k] <= RTOL / 10 else 10.0 * env[k]
            assert err[k] <= bar, (b, k, err[k], env[k])
            worst[k] = max(worst.get(k, 0.0), err[k])
    return worst


def test_well_posed_batch(ConicBatch):
    # m > n (unique primal) and LSQR converging (istop 1): the oracle's own
    # envelope is ~1e-6 here (LSQR stops at a √eps-relative residual), so the
    # GPU must agree to within ~1e-5
    w = _synthetic_check(ConicBatch, 2, 100, [(3, 10)] * 20, 21)
    assert max(w.values()) <= 1e-5, w


def test_mixed_cones_batch(ConicBatch):
    _synthetic_check(ConicBatch, 6, 30, [(0, 3), (1, 10), (3, 6), (2, 4), (4, 6)], 11)


def test_soc_only_batch(ConicBatch):
    _synthetic_check(ConicBatch, 4, 40, [(3, 5)] * 8, 12)


def test_psd_blocks_batch(ConicBatch):
    _synthetic_check(ConicBatch, 3, 25, [(4, 10), (4, 15), (1, 5)], 13)


def test_config4_shape_small_batch(ConicBatch):
    # BASELINE config 4 shape (n=500, 20 SOCs; cone dim 50 so m = 1000 > n and
    # the instance is non-degenerate) at batch 2
    w = _synthetic_check(ConicBatch, 2, 500, [(3, 50)] * 20, 14)
    assert max(w.values()) <= 1e-5, w


def test_zero_rhs_gives_zero(ConicBatch):
    from diffopt_amd.synthetic import conic_numpy
    cones = [(1, 6), (3, 4)]
    d = conic_numpy(2, 8, cones, 15)
    e = ConicBatch(2, 8, cones)
    e.set(d["A"], d["b"], d["c"], d["x"], d["s"], d["y"])
    out, dx = e.forward(None, None, None)          # RHS exactly zero (:320)
    assert np.all(out == 0) and np.all(dx == 0)
    g, _, _, _ = e.reverse(np.full((2, 8), 1e-6))  # ‖dz‖ ≤ 1e-4 (:369-370)
    assert np.all(g == 0)
    e.close()


def test_csc_staging_matches_dense(ConicBatch):
    """dopt_conic_set_csc (A_moi as Julia CSC arrays, 1-based, densified on the
    device) is bit-identical to dopt_conic_set with the same dense A; a
    malformed colptr raises."""
    import scipy.sparse as sp
    from diffopt_amd import EngineError
    from diffopt_amd.synthetic import conic_numpy
    cones = [(0, 3), (1, 10), (3, 6), (4, 6)]
    d = conic_numpy(3, 20, cones, 31)
    A = d["A"].copy()
    A[:, :, 2] = 0.0                      # an empty column
    outs = []
    for mode in ("dense", "csc"):
        e = ConicBatch(3, 20, cones)
        if mode == "dense":
            e.set(A, d["b"], d["c"], d["x"], d["s"], d["y"])
        else:
            e.set_csc([sp.csc_matrix(a) for a in A], d["b"], d["c"], d["x"], d["s"], d["y"])
        out, dx = e.forward(None, d["db"], d["dc"])
        g = e.reverse(d["dx"])[0]
        outs.append((np.asarray(out), np.asarray(dx), np.asarray(g)))
        e.close()
    for a, b in zip(*outs):
        np.testing.assert_array_equal(a, b)
    e = ConicBatch(1, 20, cones)
    bad = sp.csc_matrix(A[0])
    bad.indptr[5] = bad.indptr[4] - 1     # non-monotone colptr
    with pytest.raises(EngineError):
        e.set_csc(bad, d["b"][:1], d["c"][:1], d["x"][:1], d["s"][:1], d["y"][:1])
    e.close()


# ---------------------------------------------------------------------------
# split path (row-block × problem grids, conic_split_* kernels): forced with
# DOPT_CONIC_SPLIT=1 on the shapes above, and taken automatically for
# m > 1024 (several row blocks per problem, partial Aᵀ products reduced)
# ---------------------------------------------------------------------------
@pytest.fixture
def SplitConicBatch(ConicBatch, monkeypatch):
    monkeypatch.setenv("DOPT_CONIC_SPLIT", "1")
    return ConicBatch


def test_split_mixed_cones_batch(SplitConicBatch):
    _synthetic_check(SplitConicBatch, 6, 30, [(0, 3), (1, 10), (3, 6), (2, 4), (4, 6)], 11)


def test_split_well_posed_batch(SplitConicBatch):
    w = _synthetic_check(SplitConicBatch, 2, 100, [(3, 10)] * 20, 21)
    assert max(w.values()) <= 1e-5, w


def test_split_psd_blocks_batch(SplitConicBatch):
    _synthetic_check(SplitConicBatch, 3, 25, [(4, 10), (4, 15), (1, 5)], 13)


def test_split_zero_rhs_gives_zero(SplitConicBatch):
    test_zero_rhs_gives_zero(SplitConicBatch)


def test_split_matches_persistent_kernel(ConicBatch, monkeypatch):
    # same problems through both LSQR drivers: identical algorithm, different
    # summation order of the A products → agreement to the oracle bar
    from diffopt_amd.synthetic import conic_numpy
    cones = [(3, 10)] * 20
    d = conic_numpy(3, 100, cones, 21)
    res = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("DOPT_CONIC_SPLIT", mode)
        e = ConicBatch(3, 100, cones)
        e.set(d["A"], d["b"], d["c"], d["x"], d["s"], d["y"])
        out, _ = e.forward(d["dA"], d["db"], d["dc"])
        g = e.reverse(d["dx"])[0]
        res[mode] = (np.asarray(out), np.asarray(g), e.iterations())
        e.close()
    assert relfro(res["1"][0], res["0"][0]) <= 1e-5
    assert relfro(res["1"][1], res["0"][1]) <= 1e-5


def test_config5_shape_multi_rowblock(ConicBatch):
    # BASELINE config 5 structure (PSD(50) cones, m ≫ n) scaled to oracle
    # speed: 3 PSD(50) → m = 3825 = 8 row blocks, auto split path
    _synthetic_check(ConicBatch, 2, 100, [(4, 1275)] * 3, 16)
