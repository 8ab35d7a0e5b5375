"""The NLP oracle (oracle/nlp.py) against the reference's own known answers
(tests/golden/nlp_fixtures.json, transcribed by tests/golden/make_nlp_golden.py
from test/nlp_program.jl and test/data/nlp_problems.jl): the analytic
sensitivity tables, the finite-difference problems (QP_sIpopt, NLP_1, MIN and
MAX), the reverse-mode tests and the inertia correction — each at the
tolerance the reference test uses."""

import json
import os

import numpy as np
import pytest

from oracle import nlp

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "nlp_fixtures.json")))
FIX = GOLD["fixtures"]


def _point(f):
    return {k: np.asarray(v, dtype=float) for k, v in f["point"].items()}


def sensitivity(f):
    pt = _point(f)
    return nlp.compute_sensitivity(f["con_kind"], f["has_low"], f["has_up"], f["sense"], pt["Hxx"], pt["Hxp"],
                                   pt["Jx"], pt["Jp"], pt["x"], pt["cval"], pt["crhs"], pt["y"], pt["xl"],
                                   pt["xu"], pt["yl"], pt["yu"], return_info=True)


def split_duals(L, dd):
    c, nlo = L.c, len(L.low_p)
    return dict(dy=dd[:c], dvl=dd[c:c + nlo], dvu=dd[c + nlo:])


@pytest.mark.parametrize("f", [f for f in FIX if "fwd" in f], ids=lambda f: f["name"])
def test_forward_matches_reference_values(f):
    ds, L, M, N, corr = sensitivity(f)
    assert corr == 0
    dx, dd = nlp.forward(ds, L, np.asarray(f["fwd"]["dp"], dtype=float))
    got = dict(dx=dx, **split_duals(L, dd))
    for key, want in f["expect_fwd"].items():
        np.testing.assert_allclose(got[key], want, atol=f["atol"], rtol=f.get("rtol", 0.0), err_msg=key)


@pytest.mark.parametrize("f", [f for f in FIX if "rev" in f], ids=lambda f: f["name"])
def test_reverse_matches_reference_values(f):
    ds, L, M, N, corr = sensitivity(f)
    dp = nlp.reverse(ds, L, np.asarray(f["rev"]["dx"], dtype=float), np.asarray(f["rev"]["ddual"], dtype=float))
    np.testing.assert_allclose(dp, f["expect_rev"]["dp"], atol=f["atol"], rtol=f.get("rtol", 0.0))


def test_forward_reverse_adjoint():
    """⟨Δw, ∂s·Δp⟩ = ⟨∂sᵀΔw, Δp⟩ on the NLP_1 fixture (the two directions
    use one ∂s, NonLinearProgram.jl:519-520, 572)."""
    f = next(f for f in FIX if f["name"] == "NLP_1_4 min")
    ds, L, *_ = sensitivity(f)
    rng = np.random.default_rng(3)
    dp = rng.standard_normal(ds.shape[1])
    dx_seed = rng.standard_normal(L.n)
    dd_seed = rng.standard_normal(len(L.index_duals))
    fx, fd = nlp.forward(ds, L, dp)
    back = nlp.reverse(ds, L, dx_seed, dd_seed)
    assert abs((dx_seed @ fx + dd_seed @ fd) - back @ dp) <= 1e-12 * (1 + abs(back @ dp))


def test_inertia_correction_matrix():
    """test_inertia_correction (test/nlp_program.jl:767-795): the KKT Jacobian
    is exactly singular; _inertia_correction(M, 3, 2) factorises it."""
    k = GOLD["kkt"][0]
    M = np.asarray(k["M"], dtype=float)
    assert nlp._lu(M) is None
    K, corr = nlp.inertia_correction(M, k["num_cons"], k["num_w"])
    assert K is not None and corr >= 1


def test_layout_index_duals():
    """index_duals skips the slack-bound duals (NonLinearProgram.jl:480-484)."""
    L = nlp.Layout([1, 2, 0, 1], [1, 0, 1], [0, 1, 0])
    # w = 3 + 2 geq + 1 leq = 6; c = 4; lower: 2 primal + 2 geq slacks; upper: 1 + 1
    assert (L.num_w, L.nlo, L.nup, L.rows) == (6, 4, 2, 16)
    np.testing.assert_array_equal(L.index_duals, [6, 7, 8, 9, 10, 11, 14])
