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
        assert relfro(out[0], np.concatenate([du, dv, [dw]])) <= RTOL
        x = np.array(fx["x"], dtype=float)
        sol = np.linalg.norm(np.concatenate([du, dv, [dw]]))
        assert relcomb(dx[0], odx, sol * (1 + np.linalg.norm(x))) <= RTOL
    for t in fx["reverse"]:
        g, dA, db, dc = e.reverse(np.array(t["dx"], dtype=float)[None])
        np.testing.assert_allclose(db[0][t["rows"]], t["db"], atol=t["atol"], rtol=t["rtol"])
        og, _ = ocn.reverse_differentiate(cache, t["dx"])
        assert relfro(g[0], og) <= RTOL
    e.close()


def _synthetic_check(ConicBatch, B, n, cones, seed):
    from diffopt_amd.synthetic import conic_numpy
    d = conic_numpy(B, n, cones, seed)
    e = ConicBatch(B, n, cones)
    e.set(d["A"], d["b"], d["c"], d["x"], d["s"], d["y"])
    out, dx = e.forward(d["dA"], d["db"], d["dc"])
    g, dA, db, dc = e.reverse(d["dx"])
    worst = 0.0
    for b in range(B):
        cache = ocn.Cache(d["A"][b], d["b"][b], d["c"][b], d["x"][b], d["s"][b], d["y"][b], cones)
        odx, du, dv, dw = ocn.forward_differentiate(cache, d["dA"][b], d["db"][b], d["dc"][b])
        og, _ = ocn.reverse_differentiate(cache, d["dx"][b])
        odA, odb, odc = ocn.reverse_outputs(cache, og)
        nx, nvp = np.linalg.norm(d["x"][b]), np.linalg.norm(cache.vp)
        sol = np.linalg.norm(np.concatenate([du, dv, [dw]]))
        ng = np.linalg.norm(og)
        worst = max(worst,
                    relfro(out[b], np.concatenate([du, dv, [dw]])),
                    relcomb(dx[b], odx, sol * (1 + nx)),
                    relfro(g[b], og),
                    relcomb(dA[b], odA, ng * (nx + nvp)),
                    relcomb(db[b], odb, ng * (1 + nvp)),
                    relcomb(dc[b], odc, ng * (1 + nx)))
    e.close()
    assert worst <= RTOL, worst


def test_mixed_cones_batch(ConicBatch):
    _synthetic_check(ConicBatch, 6, 30, [(0, 3), (1, 10), (3, 6), (2, 4), (4, 6)], 11)


def test_soc_only_batch(ConicBatch):
    _synthetic_check(ConicBatch, 4, 40, [(3, 5)] * 8, 12)


def test_psd_blocks_batch(ConicBatch):
    _synthetic_check(ConicBatch, 3, 25, [(4, 10), (4, 15), (1, 5)], 13)


def test_config4_shape_small_batch(ConicBatch):
    # BASELINE config 4 shape (n=500, 20 × SOC(25)) at batch 2
    _synthetic_check(ConicBatch, 2, 500, [(3, 25)] * 20, 14)


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
