"""ParametricOptInterface glue of the QP back-end on the GPU
(dopt_qp_params_reverse / _forward, csrc/params.hip) against the oracle
restatement of reference src/parameters.jl (oracle/poi.py), and the adjoint
identity ⟨dl/dz, dz(dp)⟩ = ⟨dL/dp, dp⟩ that ties the two directions to the
QP solves (which are pinned by the reference fixtures)."""

import numpy as np
import pytest

from oracle import poi
from oracle import qp as oqp

pytestmark = pytest.mark.gpu


def _problem(B, n, m, p, seed, nparam, nterms):
    from diffopt_amd.synthetic import qp_numpy
    d = qp_numpy(B, n, m, p, 0.4, seed)
    rng = np.random.default_rng(seed)
    lim = {0: m, 1: p, 2: 1, 3: n}
    kinds = [k for k in rng.integers(0, 4, nterms) if lim[int(k)] > 0]
    terms = [(int(rng.integers(nparam)), int(k), int(rng.integers(lim[int(k)])), float(rng.standard_normal()))
             for k in kinds]
    return d, terms


def _engine(d):
    from diffopt_amd.qp import QPBatch
    B, n = d["z"].shape
    m, p = d["lam"].shape[1], d["nu"].shape[1]
    e = QPBatch(B, n, m, p)
    e.set(d["Q"], d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
    return e


@pytest.mark.parametrize("shape", [(3, 20, 30, 4), (2, 200, 300, 0), (2, 12, 0, 5)])
def test_params_reverse_forward_vs_oracle(shape):
    B, n, m, p = shape
    nparam = 7
    d, terms = _problem(B, n, m, p, 11 + n, nparam, 60)
    e = _engine(d)
    e.factor()
    rev = e.reverse(d["dl_dz"])
    dLdp = e.params_reverse(rev, terms, nparam)
    rng = np.random.default_rng(3)
    dpt = rng.standard_normal((B, nparam))
    dq, dh, db = e.params_forward(dpt, terms)
    fwd = e.forward(dq=dq, dh=dh if m else None, db=db if p else None)
    for b in range(B):
        ref = poi.reverse(terms, nparam, d["lam"][b], rev[b], n, m, p)
        np.testing.assert_allclose(dLdp[b], ref, rtol=1e-13, atol=1e-14)
        oq, oh, ob = poi.forward(terms, dpt[b], n, m, p)
        np.testing.assert_allclose(dq[b], oq, rtol=1e-13, atol=1e-14)
        if m:
            np.testing.assert_allclose(dh[b], oh, rtol=1e-13, atol=1e-14)
        if p:
            np.testing.assert_allclose(db[b], ob, rtol=1e-13, atol=1e-14)
        # adjoint identity: the POI maps are transposes and so are the solves
        lhs = d["dl_dz"][b] @ fwd[b, :n]
        rhs = dLdp[b] @ dpt[b]
        assert abs(lhs - rhs) <= 1e-9 * max(1.0, abs(lhs)), (lhs, rhs)


def test_params_end_to_end_against_oracle_solves():
    """dp → (dq, dh, db) → forward on the GPU, against the oracle's forward
    with the oracle's POI tangents (north_star's 1e-6)."""
    d, terms = _problem(2, 30, 40, 3, 77, 5, 40)
    e = _engine(d)
    dpt = np.random.default_rng(4).standard_normal((2, 5))
    dq, dh, db = e.params_forward(dpt, terms)
    fwd = e.forward(dq=dq, dh=dh, db=db)
    for b in range(2):
        args = [d[k][b] for k in ["Q", "G", "h", "A", "z", "lam", "nu"]]
        oq, oh, ob = poi.forward(terms, dpt[b], 30, 40, 3)
        ref = np.concatenate(oqp.forward_differentiate(*args, dq=oq, dh=oh, db=ob))
        err = np.linalg.norm(fwd[b] - ref) / np.linalg.norm(ref)
        assert err <= 1e-6, err


def test_params_term_validation():
    from diffopt_amd import EngineError
    d, _ = _problem(1, 5, 6, 2, 3, 2, 0)
    e = _engine(d)
    rev = e.reverse(d["dl_dz"])
    with pytest.raises(EngineError, match="out of range"):
        e.params_reverse(rev, [(0, 0, 6, 1.0)], 2)         # LessThan row 6 of 6
    with pytest.raises(EngineError, match="out of range"):
        e.params_reverse(rev, [(2, 1, 0, 1.0)], 2)         # parameter 2 of 2
