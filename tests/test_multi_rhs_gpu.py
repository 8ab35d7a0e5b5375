"""Multi-RHS solves on one factorisation (dopt_qp_reverse_k / dopt_qp_forward_k,
csrc/qp_multi.hip): k seeds / tangents per problem, k ∈ {1, 7, 32}.

The reference re-solves per seed (reverse_differentiate! / forward_differentiate!
on the same model, QuadraticProgram.jl:316-446, 486-496; callers loop seeds,
e.g. docs/src/examples/sensitivity-analysis-ridge.jl:120-131).  Each seed's
result is held to north_star's 1e-6 relative Frobenius against the oracle, and
to rounding against the single-seed calls on the same handle (the multi-RHS
path sweeps with MFMA block products instead of per-row dot products, so the
summation order differs)."""

import numpy as np
import pytest

from oracle import qp as oqp

pytestmark = pytest.mark.gpu
RTOL = 1e-6


def relfro(a, b):
    a, b = np.asarray(a, dtype=float), np.asarray(b, dtype=float)
    nb = np.linalg.norm(b)
    return np.linalg.norm(a - b) / (nb if nb > 0 else 1.0)


@pytest.fixture(scope="module")
def QPBatch():
    from diffopt_amd.qp import QPBatch
    return QPBatch


@pytest.fixture(params=["nopiv", "pivot"])
def lu_mode(request, monkeypatch):
    if request.param == "pivot":
        monkeypatch.setenv("DOPT_LU", "0")
    else:
        monkeypatch.delenv("DOPT_LU", raising=False)
    return request.param


def _data(B, n, m, p, seed, k, lam_eps=0.0):
    from diffopt_amd.synthetic import qp_numpy
    d = qp_numpy(B, n, m, p, 0.4, seed, lam_eps=lam_eps)
    rng = np.random.default_rng(seed + 1)
    d["dl_k"] = rng.standard_normal((k, B, n))
    d["dq_k"] = rng.standard_normal((k, B, n))
    d["dh_k"] = rng.standard_normal((k, B, m))
    d["db_k"] = rng.standard_normal((k, B, p))
    return d


def _engine(QPBatch, d):
    B, n = d["z"].shape
    m, p = d["lam"].shape[1], d["nu"].shape[1]
    e = QPBatch(B, n, m, p)
    e.set(d["Q"], d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
    return e


def _check(QPBatch, d, k, oracle_problems=None):
    e = _engine(QPBatch, d)
    e.factor()
    rev = e.reverse_k(d["dl_k"])
    fwd = e.forward_k(dq=d["dq_k"], dh=d["dh_k"], db=d["db_k"])
    B = d["z"].shape[0]
    assert rev.shape == (k, B, e.L) and fwd.shape == (k, B, e.L)
    worst = 0.0
    for b in (range(B) if oracle_problems is None else oracle_problems):
        args = [d[key][b] for key in ["Q", "G", "h", "A", "z", "lam", "nu"]]
        for j in range(k):
            r = np.concatenate(oqp.reverse_differentiate(*args, d["dl_k"][j, b]))
            f = np.concatenate(oqp.forward_differentiate(*args, dq=d["dq_k"][j, b], dh=d["dh_k"][j, b],
                                                         db=d["db_k"][j, b]))
            worst = max(worst, relfro(rev[j, b], r), relfro(fwd[j, b], f))
    assert worst <= RTOL, worst
    # the single-seed calls on the same factors, to rounding
    for j in (0, k - 1):
        np.testing.assert_allclose(rev[j], e.reverse(d["dl_k"][j]), rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(fwd[j], e.forward(dq=d["dq_k"][j], dh=d["dh_k"][j], db=d["db_k"][j]),
                                   rtol=1e-10, atol=1e-12)
    return e


@pytest.mark.parametrize("k", [1, 7, 32])
def test_multi_rhs_cfg1_shape(QPBatch, lu_mode, k):
    _check(QPBatch, _data(4, 50, 70, 5, 101, k), k)


@pytest.mark.parametrize("k", [7, 32])
def test_multi_rhs_cfg2_shape(QPBatch, lu_mode, k):
    # the bench problem shape (n=200, m=300), 32-seed chunks straddling 16
    _check(QPBatch, _data(3, 200, 300, 0, 202, k), k, oracle_problems=[0, 2])


def test_multi_rhs_large_system_lds_opt_in(QPBatch):
    """No elimination (λ = 1e-9): N' = 500, Np = 512 — the chunk's LDS image is
    66 KB, above the 64 KB default (hipFuncAttributeMaxDynamicSharedMemorySize)."""
    d = _data(2, 200, 300, 0, 303, 7, lam_eps=1e-9)
    e = _check(QPBatch, d, 7, oracle_problems=[1])
    assert (e.system_size() == 500).all()


def test_multi_rhs_tall_system_global_chunk(QPBatch):
    """Config-3 shape (N' ≈ 1600, Np > 1190): the 16-seed chunk (≥ 150 KB)
    does not fit LDS and lives in a global workspace — one launch still."""
    d = _data(2, 1000, 1500, 0, 606, 7)
    _check(QPBatch, d, 7, oracle_problems=[0])


def test_multi_rhs_mixed_factor_kinds(QPBatch):
    """No-pivot and partial-pivoting problems in one batch (relabelled rows)."""
    d = _data(6, 60, 80, 5, 404, 7)
    rng = np.random.default_rng(5)
    for b in (1, 4):   # symmetric indefinite Q with a tiny diagonal: the threshold test rejects
        S = rng.standard_normal((60, 60))
        Q = (S + S.T) / 2
        Q[np.diag_indices(60)] = 1e-4
        d["Q"][b] = Q
    e = _check(QPBatch, d, 7)
    np.testing.assert_array_equal(e.lu_kind(), [1, 2, 1, 1, 2, 1])


def test_multi_rhs_argument_errors(QPBatch):
    """k ≤ 0 is rejected with a message (rc < 0), nothing is launched."""
    from diffopt_amd import EngineError, _lib
    d = _data(2, 10, 12, 2, 505, 1)
    e = _engine(QPBatch, d)
    out = np.empty(2 * e.L)
    rc = e.lib.dopt_qp_reverse_k(e.h, 0, d["dl_k"].ctypes.data, out.ctypes.data)
    assert rc < 0
    with pytest.raises(EngineError, match="k must be positive"):
        _lib.check(rc, e.h)
