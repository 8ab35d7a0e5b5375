"""The one-workgroup small-problem path (qp_small.hip):
dopt_qp_reverse of a batch of at most SM_BATCH problems not yet factorised
takes one launch (prepare, reduced KKT in LDS, no-pivot LU with the batched
route's acceptance tests, the solve, the outputs); dopt_qp_forward reuses its
factors.  Held to the oracle at the north_star bar (1e-6 relative Frobenius)
at the config-1 shape (QuadraticProgram.jl:316-446), and to the batched route;
problems it cannot take fall back to the batched route in the same call."""
import numpy as np
import pytest

from oracle import qp as oqp

pytestmark = pytest.mark.gpu
RTOL = 1e-6
SMALL = 3   # _lib.LU_KIND_SMALL


def relfro(a, b):
    nb = np.linalg.norm(b)
    return np.linalg.norm(np.asarray(a) - b) / nb if nb > 0 else np.linalg.norm(a)


@pytest.fixture(scope="module")
def QPBatch():
    from diffopt_amd.qp import QPBatch
    return QPBatch


def _data(B, n, m, p, phi, seed):
    from diffopt_amd.synthetic import qp_numpy
    return qp_numpy(B, n, m, p, phi, seed)


def _oracle(d, b, p):
    args = [d[k][b] for k in ("Q", "G", "h", "A", "z", "lam", "nu")]
    rev = np.concatenate(oqp.reverse_differentiate(*args, d["dl_dz"][b]))
    fwd = np.concatenate(oqp.forward_differentiate(*args, dq=d["dq"][b], dh=d["dh"][b],
                                                   db=d["db"][b] if p else None))
    return rev, fwd


@pytest.mark.parametrize("B", [1, 4, 8])
def test_small_path_config1_shape(QPBatch, B):
    n, m, p = 50, 80, 30
    d = _data(B, n, m, p, 0.2, 20250307 + 1)
    e = QPBatch(B, n, m, p)
    e.set(d["Q"], d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
    rev = e.reverse(d["dl_dz"])
    assert (e.lu_kind() == SMALL).all(), e.lu_kind()
    fwd = e.forward(dq=d["dq"], dh=d["dh"], db=d["db"])
    kept = e.kept()
    e.close()
    for b in range(B):
        ref_r, ref_f = _oracle(d, b, p)
        assert relfro(rev[b], ref_r) <= RTOL
        assert relfro(fwd[b], ref_f) <= RTOL
        # the kept set bit-exact (s in the prepare kernel's order)
        s = np.array([sum(d["G"][b][i, j] * d["z"][b][j] for j in range(n)) for i in range(m)]) - d["h"][b]
        want = ~((d["lam"][b] == 0.0) & (s != 0.0))
        np.testing.assert_array_equal(kept[b].astype(bool), want)


def test_small_path_matches_batched_route(QPBatch):
    """The same problems through the small path (batch 4) and the batched route
    (batch 16 > SM_BATCH: the first four are the same problems) agree to
    rounding; the fused forward_reverse call (batched route) on the small
    path's handle refactorises and agrees too."""
    n, m, p = 50, 80, 30
    d16 = _data(16, n, m, p, 0.2, 77)
    d4 = {k: v[:4] for k, v in d16.items()}
    es = QPBatch(4, n, m, p)
    es.set(d4["Q"], d4["G"], d4["h"], d4["A"], d4["z"], d4["lam"], d4["nu"])
    r_s = es.reverse(d4["dl_dz"])
    f_s = es.forward(dq=d4["dq"], dh=d4["dh"], db=d4["db"])
    r_f, f_f = es.forward_reverse(d4["dl_dz"], dq=d4["dq"], dh=d4["dh"], db=d4["db"])
    assert (es.lu_kind() != SMALL).all()
    es.close()
    eb = QPBatch(16, n, m, p)
    eb.set(d16["Q"], d16["G"], d16["h"], d16["A"], d16["z"], d16["lam"], d16["nu"])
    r_b = eb.reverse(d16["dl_dz"])
    f_b = eb.forward(dq=d16["dq"], dh=d16["dh"], db=d16["db"])
    eb.close()
    for b in range(4):
        assert relfro(r_s[b], r_b[b]) <= 1e-10 and relfro(f_s[b], f_b[b]) <= 1e-10
        assert relfro(r_f[b], r_b[b]) <= 1e-10 and relfro(f_f[b], f_b[b]) <= 1e-10


def test_small_path_fallbacks(QPBatch):
    """Problems the small path cannot take run the batched route in the same
    call: a Q == 0 problem (the LSQR branch), a reduced system over 128
    unknowns (interior-point duals: nothing eliminated), and with DOPT_LU=0 the
    path is off; all against the oracle."""
    n, m, p = 30, 60, 10
    d = _data(2, n, m, p, 0.2, 5)
    d["Q"][1] = 0.0                          # LSQR branch for problem 1
    e = QPBatch(2, n, m, p)
    e.set(d["Q"], d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
    rev = e.reverse(d["dl_dz"])
    assert (e.lu_kind() != SMALL).all()
    for b in range(2):
        args = [d[k][b] for k in ("Q", "G", "h", "A", "z", "lam", "nu")]
        ref = np.concatenate(oqp.reverse_differentiate(*args, d["dl_dz"][b]))
        assert relfro(rev[b], ref) <= RTOL
    e.close()
    # interior-point duals (λ = 1e-9 on the inactive rows): nothing is
    # eliminated, N' = n + m + p = 150 > 128
    from diffopt_amd.synthetic import qp_numpy
    n, m, p = 60, 80, 10
    d = qp_numpy(1, n, m, p, 0.2, 6, lam_eps=1e-9)
    e = QPBatch(1, n, m, p)
    e.set(d["Q"], d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
    rev = e.reverse(d["dl_dz"])
    assert e.lu_kind()[0] != SMALL
    args = [d[k][0] for k in ("Q", "G", "h", "A", "z", "lam", "nu")]
    assert relfro(rev[0], np.concatenate(oqp.reverse_differentiate(*args, d["dl_dz"][0]))) <= RTOL
    e.close()


def test_small_path_off_under_partial_pivoting(QPBatch, monkeypatch):
    monkeypatch.setenv("DOPT_LU", "0")
    n, m, p = 50, 80, 30
    d = _data(1, n, m, p, 0.2, 8)
    e = QPBatch(1, n, m, p)
    e.set(d["Q"], d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
    rev = e.reverse(d["dl_dz"])
    assert e.lu_kind()[0] == 2   # partial pivoting
    ref_r, _ = _oracle(d, 0, p)
    assert relfro(rev[0], ref_r) <= RTOL
    e.close()


def test_small_path_singular_reports_info(QPBatch):
    """A singular reduced KKT (two identical equality rows) falls back to the
    batched route, which reports the reference's SingularException column."""
    from diffopt_amd import SingularException
    n, m, p = 20, 30, 4
    d = _data(1, n, m, p, 0.2, 9)
    d["A"][0][1] = d["A"][0][0]
    d["nu"][0][1] = d["nu"][0][0]
    e = QPBatch(1, n, m, p)
    e.set(d["Q"], d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
    with pytest.raises(SingularException):
        e.reverse(d["dl_dz"])
    e.close()


@pytest.mark.parametrize("n,m,p,phi", [(1, 1, 0, 0.0), (5, 3, 0, 0.5), (7, 0, 2, 0.0), (17, 9, 4, 0.4),
                                       (33, 40, 15, 0.3), (64, 64, 0, 1.0), (96, 31, 31, 0.0)])
def test_small_path_shapes(QPBatch, n, m, p, phi):
    """Ragged shapes around the register tiles' 16-row blocks and the four-step
    groups (N' = 1, not a multiple of 4 or 16, exactly 128, m = 0, p = 0),
    with dense tangents so every forward RHS term is live; batch 2, both
    directions against the oracle, and the path actually taken."""
    from diffopt_amd.synthetic import qp_numpy
    d = qp_numpy(2, n, m, p, phi, 1000 + n + m + p, dense_tangents=True)
    e = QPBatch(2, n, m, p)
    e.set(d["Q"], d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
    rev = e.reverse(d["dl_dz"])
    assert (e.lu_kind() == SMALL).all(), e.lu_kind()
    fwd = e.forward(dQ=d["dQ"], dq=d["dq"], dG=d["dG"] if m else None, dh=d["dh"] if m else None,
                    dA=d["dA"] if p else None, db=d["db"] if p else None)
    e.close()
    for b in range(2):
        args = [d[k][b] for k in ("Q", "G", "h", "A", "z", "lam", "nu")]
        ref_r = np.concatenate(oqp.reverse_differentiate(*args, d["dl_dz"][b]))
        ref_f = np.concatenate(oqp.forward_differentiate(
            *args, dQ=d["dQ"][b], dq=d["dq"][b], dG=d["dG"][b] if m else None, dh=d["dh"][b] if m else None,
            dA=d["dA"][b] if p else None, db=d["db"][b] if p else None))
        assert relfro(rev[b], ref_r) <= RTOL
        assert relfro(fwd[b], ref_f) <= RTOL


def test_small_path_reused_handle(QPBatch):
    """One handle, successive models (the Julia QPModel's pattern): its first
    two calls stage through pageable copies, the later ones through the pinned
    pack and the single read-back of outputs and flags; every model matches a
    fresh handle bit for bit, and a model the path cannot take (Q = 0) on the
    pinned route still falls back to the batched route in the same call."""
    n, m, p = 50, 80, 30
    e = QPBatch(2, n, m, p)
    for it in range(4):
        d = _data(2, n, m, p, 0.2, 9100 + it)
        if it == 3:
            d["Q"][1] = 0.0
        args = [d[k] for k in ("Q", "G", "h", "A", "z", "lam", "nu")]
        e.set(*args)
        rev = e.reverse(d["dl_dz"])
        fwd = e.forward(dq=d["dq"], dh=d["dh"], db=d["db"])
        assert (e.lu_kind() == SMALL).all() == (it < 3)
        f = QPBatch(2, n, m, p)
        f.set(*args)
        np.testing.assert_array_equal(rev, f.reverse(d["dl_dz"]))
        np.testing.assert_array_equal(fwd, f.forward(dq=d["dq"], dh=d["dh"], db=d["db"]))
        f.close()
        for b in range(2):
            ref_r, ref_f = _oracle(d, b, p)
            assert relfro(rev[b], ref_r) <= RTOL
            if not (it == 3 and b == 1):   # (the LSQR branch's forward: as test_small_path_fallbacks, reverse only)
                assert relfro(fwd[b], ref_f) <= RTOL
    e.close()


def test_small_path_csc_handle_reuse(QPBatch):
    """The Julia QPModel's exact sequence on one handle — dopt_qp_set_csc of
    the MOI form, reverse, forward — for successive models: from the third
    call on set_csc validates on the host and returns with its copy queued,
    and the small kernels read the seed from / write the outputs into the
    pinned read-back buffer in place.  Every model against the oracle; a set
    overwritten before any call (the queued copy of the first waits before
    the pinned buffer is written again) solves the second model; a malformed
    CSC raises on the host and leaves no model; a good set afterwards works."""
    import scipy.sparse as sp
    from diffopt_amd import EngineError
    n, m, p = 50, 80, 30
    e = QPBatch(1, n, m, p)

    def put(d):
        e.set_csc([sp.csc_matrix(d["Q"][0])], [sp.csc_matrix(d["G"][0])], d["h"], [sp.csc_matrix(d["A"][0])],
                  d["z"], d["lam"], d["nu"])

    def check(d):
        rev = e.reverse(d["dl_dz"])
        assert (e.lu_kind() == SMALL).all()
        fwd = e.forward(dq=d["dq"], dh=d["dh"], db=d["db"])
        ref_r, ref_f = _oracle(d, 0, p)
        assert relfro(rev[0], ref_r) <= RTOL and relfro(fwd[0], ref_f) <= RTOL

    for it in range(5):
        d = _data(1, n, m, p, 0.2, 9300 + it)
        put(d)
        check(d)
    d1, d2 = _data(1, n, m, p, 0.2, 9400), _data(1, n, m, p, 0.2, 9401)
    put(d1)
    put(d2)               # no call between the two sets
    check(d2)
    bad = sp.csc_matrix(d1["G"][0])
    bad.indices[0] = 999  # row index out of range
    with pytest.raises(EngineError, match="rowval out of range"):
        e.set_csc([sp.csc_matrix(d1["Q"][0])], [bad], d1["h"], [sp.csc_matrix(d1["A"][0])], d1["z"], d1["lam"], d1["nu"])
    with pytest.raises(EngineError):
        e.reverse(d1["dl_dz"])
    put(d1)
    check(d1)
    # matrix tangents on the pinned route (the packed copy in, not the
    # vector-only zero-copy form)
    rng = np.random.default_rng(9500)
    dQ = rng.standard_normal((1, n, n))
    dQ = dQ + dQ.transpose(0, 2, 1)
    dG, dA = rng.standard_normal((1, m, n)), rng.standard_normal((1, p, n))
    e.reverse(d1["dl_dz"])
    fwd = e.forward(dQ=dQ, dq=d1["dq"], dG=dG, dh=d1["dh"], dA=dA, db=d1["db"])
    args = [d1[k][0] for k in ("Q", "G", "h", "A", "z", "lam", "nu")]
    ref = np.concatenate(oqp.forward_differentiate(*args, dQ=dQ[0], dq=d1["dq"][0], dG=dG[0], dh=d1["dh"][0],
                                                   dA=dA[0], db=d1["db"][0]))
    assert relfro(fwd[0], ref) <= RTOL
    e.close()
