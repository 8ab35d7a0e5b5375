"""Sparse QP route (sparse.hip; VERDICT r05 missing 2): the MOI matrix form
kept sparse and `lsqr(LHS, RHS)` / `lsqr(LHS', RHS)` on the implicit full LHS
— the reference's `norm(Q) ≈ 0` branch (QuadraticProgram.jl:333, :486-492),
which never densifies.  Checked against the oracle's sparse restatement
(oracle/qp.py lp_sparse_differentiate: scipy CSC LHS + the IterativeSolvers
LSQR restatement) at north_star's 1e-6 relative Frobenius bar; against the
reference's own LP fixtures (test/linear_program.jl via tests/golden); against
the dense route on the same problems; above the dense route's n + m + p ≤ 8192
cap; and the route's refusals (Q ≠ 0, dense-only calls)."""

import json
import os

import numpy as np
import pytest

from oracle import qp as oqp

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
RTOL = 1e-6


def relfro(a, b):
    return np.linalg.norm(np.asarray(a) - np.asarray(b)) / max(np.linalg.norm(b), 1e-300)


def _batch(d, sparse=True):
    import scipy.sparse as sp
    from diffopt_amd.qp import QPBatch
    B, n = d["z"].shape
    m = d["lam"].shape[1]
    p = d["nu"].shape[1]
    e = QPBatch(B, n, m, p, sparse=sparse)
    Q0 = sp.csc_matrix((n, n))
    e.set_csc([Q0] * B, d["G"] if m else None, d["h"], d["A"] if p else None, d["z"], d["lam"], d["nu"])
    return e


def _oracle(d, b):
    m = d["lam"].shape[1]
    p = d["nu"].shape[1]
    return oqp.lp_sparse_differentiate(d["G"][b] if m else None, d["h"][b], d["A"][b] if p else None, d["z"][b],
                                       d["lam"][b], d["nu"][b], d["dl_dz"][b], d["dq"][b],
                                       d["dh"][b] if m else None, d["db"][b] if p else None)


def _check(d, e=None):
    e = e or _batch(d)
    rev, fwd = e.forward_reverse(d["dl_dz"], dq=d["dq"], dh=d["dh"], db=d["db"])
    stats = e.lsqr_stats()
    worst = 0.0
    for b in range(d["z"].shape[0]):
        orv, ofw, (itr, isr), (itf, isf) = _oracle(d, b)
        worst = max(worst, relfro(rev[b], orv), relfro(fwd[b], ofw))
        assert stats[b, 0, 0] in (1, 2) and stats[b, 1, 0] in (1, 2), stats[b]   # converged, as the oracle
        assert isr in (1, 2) and isf in (1, 2)
    assert worst <= RTOL, worst
    return e, rev, fwd


def test_sparse_lp_batch_vs_oracle():
    from diffopt_amd.synthetic import lp_sparse_numpy
    d = lp_sparse_numpy(3, 300, 20, 200, 4, 101)
    e, rev, fwd = _check(d)
    assert list(e.iterative()) == [True] * 3
    assert list(e.lu_kind()) == [0] * 3                      # LU_KIND_LSQR
    assert list(e.system_size()) == [300 + 480 + 20] * 3
    # separate calls: the same LSQR runs, bit for bit
    r1 = e.reverse(d["dl_dz"])
    f1 = e.forward(dq=d["dq"], dh=d["dh"], db=d["db"])
    np.testing.assert_array_equal(r1, rev)
    np.testing.assert_array_equal(f1, fwd)


def test_sparse_route_matches_dense_route():
    """The same LPs through the dense route's LSQR kernel (K assembled densely)
    and the sparse route: both restate the same LSQR; only the summation order
    of the products differs, so they agree far below the 1e-6 bar."""
    from diffopt_amd.synthetic import lp_sparse_numpy
    d = lp_sparse_numpy(2, 120, 10, 80, 3, 102)
    rs, fs = _batch(d, sparse=True).forward_reverse(d["dl_dz"], dq=d["dq"], dh=d["dh"], db=d["db"])
    rd, fd = _batch(d, sparse=False).forward_reverse(d["dl_dz"], dq=d["dq"], dh=d["dh"], db=d["db"])
    for b in range(2):
        assert relfro(rs[b], rd[b]) <= 1e-7
        assert relfro(fs[b], fd[b]) <= 1e-7


def test_sparse_lp_above_dense_cap():
    """n + m + p = 9 100 > 8 192: the handle takes the sparse route by itself
    (dense dopt_qp_set is refused); reverse and forward against the oracle."""
    from diffopt_amd import _lib
    from diffopt_amd.qp import QPBatch
    from diffopt_amd.synthetic import lp_sparse_numpy
    d = lp_sparse_numpy(1, 4000, 100, 1000, 5, 103)
    m, p = d["lam"].shape[1], d["nu"].shape[1]
    assert 4000 + m + p > 8192
    e = QPBatch(1, 4000, m, p)
    assert e.sparse
    with pytest.raises(_lib.EngineError):
        e.set(np.zeros((1, 4000, 4000)), np.zeros((1, m, 4000)), d["h"], np.zeros((1, p, 4000)), d["z"], d["lam"],
              d["nu"])
    e.close()
    _check(d)


def test_sparse_reference_lp_fixtures():
    """The reference's LP fixtures (test/linear_program.jl, tests/golden) on
    the sparse route: the reference's own expected values at its tolerances,
    and the oracle at 1e-6."""
    import scipy.sparse as sp
    from diffopt_amd.qp import QPBatch
    from test_oracle_golden import qp_outputs
    with open(os.path.join(HERE, "golden", "lp_fixtures.json")) as fh:
        fx = json.load(fh)
    ran = 0
    for f in fx:
        a = {k: np.array(v, dtype=float) for k, v in f.items() if isinstance(v, list)}
        n = a["Q"].shape[0]
        if np.any(a["Q"] != 0):
            continue
        G = a["G"].reshape(-1, n)
        A = a["A"].reshape(-1, n)
        m, p = G.shape[0], A.shape[0]
        fw = {k: np.array(v, dtype=float) for k, v in f["fwd"].items()}
        if any(k in fw and fw[k].size and np.any(fw[k]) for k in ("dQ", "dG", "dA")):
            fwd_mats = True
        else:
            fwd_mats = False
        e = QPBatch(1, n, m, p, sparse=True)
        e.set_csc(sp.csc_matrix(np.zeros((n, n))), sp.csc_matrix(G) if m else None, a["h"][None] if m else None,
                  sp.csc_matrix(A) if p else None, a["z"][None], a["lam"][None] if m else None,
                  a["nu"][None] if p else None)
        rev = e.reverse(a["dzb"][None])[0]
        kw = {k: v[None] for k, v in fw.items() if v.size}
        if "dG" in kw:
            kw["dG"] = kw["dG"].reshape(1, m, n)
        if "dA" in kw:
            kw["dA"] = kw["dA"].reshape(1, p, n)
        fwd = e.forward(**kw)[0]
        got = qp_outputs(dict(a, G=G, A=A), {k: (v.reshape(G.shape) if k == "dG" else v.reshape(A.shape) if k == "dA"
                                                 else v) for k, v in fw.items()},
                         solve_rev=lambda: (rev[:n], rev[n:n + m], rev[n + m:]), solve_fwd=lambda: fwd[:n])
        for k, v in f["expect"].items():
            exp = np.array(v, dtype=float).reshape(np.shape(got[k]))
            np.testing.assert_allclose(got[k], exp, atol=f["atol"], rtol=f["rtol"], err_msg=f"{f['name']} {k}")
        Q = np.zeros((n, n))
        rz, rl, rn = oqp.reverse_differentiate(Q, G, a["h"], A, a["z"], a["lam"], a["nu"], a["dzb"])
        oz, ol, on = oqp.forward_differentiate(Q, G, a["h"], A, a["z"], a["lam"], a["nu"],
                                               **{k: (v.reshape(G.shape) if k == "dG" else
                                                      v.reshape(A.shape) if k == "dA" else v)
                                                  for k, v in fw.items() if v.size})
        assert relfro(rev, np.concatenate([rz, rl, rn])) <= RTOL
        assert relfro(fwd, np.concatenate([oz, ol, on])) <= RTOL, (f["name"], fwd_mats)
        ran += 1
    assert ran >= 1


def test_sparse_route_refusals():
    """Q ≠ 0 needs a sparse direct LU (the reference's UMFPACK), which the
    route does not have: dopt_qp_factor fails with a message; so do the calls
    that need factors or a kept mask."""
    import scipy.sparse as sp
    from diffopt_amd import _lib
    from diffopt_amd.synthetic import lp_sparse_numpy
    d = lp_sparse_numpy(1, 60, 5, 30, 3, 104)
    n, m, p = 60, d["lam"].shape[1], d["nu"].shape[1]
    e = _batch(d)
    with pytest.raises(_lib.EngineError):
        e.kept()
    with pytest.raises(_lib.EngineError):
        e.reverse_k(np.ones((2, 1, n)))
    e.set_csc([sp.identity(n, format="csc")], d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
    assert list(e.iterative()) == [False]
    with pytest.raises(_lib.EngineError, match="sparse direct LU"):
        e.factor()
    # malformed CSC: the dense route's validation
    G = d["G"][0].copy()
    G.indices[0] = m + 5
    with pytest.raises(_lib.EngineError, match="rowval"):
        e.set_csc([sp.csc_matrix((n, n))], [G], d["h"], d["A"], d["z"], d["lam"], d["nu"])


# ---------------------------------------------------------------------------
# The conic back-end on the sparse route: A_moi kept sparse (dopt_set_sparse on
# a conic handle + dopt_conic_set_csc), LSQR on the matrix-free M
# (ConicProgram.jl:243-247, :323, :372) from its CSC / CSR arrays.
# ---------------------------------------------------------------------------
def _conic_run(d, cones, sparse, B):
    import scipy.sparse as sp
    from diffopt_amd.conic import ConicBatch
    n = d["x"].shape[1]
    e = ConicBatch(B, n, cones, sparse=sparse)
    if sparse:
        e.set_csc([sp.csc_matrix(a) for a in d["A"]], d["b"], d["c"], d["x"], d["s"], d["y"])
    else:
        e.set(d["A"], d["b"], d["c"], d["x"], d["s"], d["y"])
    r = e.forward_reverse(d["dx"], d["dA"], d["db"], d["dc"])
    st = e.lsqr_stats()
    e.close()
    return r, st


def _conic_vs_oracle(d, cones, B, res, st, minnorm=False):
    """Every output at 1e-6 of the oracle; with `minnorm` (a converging shape
    whose √eps stopping noise times cond(M) can pass 1e-6 — the dense route's
    converged-shape bar, test_conic_gpu._minnorm_judge) an output above 1e-6
    is held instead to: the engine's LSQR solution of that direction within
    max(2 × the oracle's distance, 1e-8) of the exact minimum-norm solution."""
    from oracle import conic as ocn
    from test_conic_gpu import _errors, _minnorm_judge, _oracle_outputs
    (out, fdx), (g, dA, db, dc) = res
    worst, judged = 0.0, 0
    for b in range(B):
        cache = ocn.Cache(d["A"][b], d["b"][b], d["c"][b], d["x"][b], d["s"][b], d["y"][b], cones)
        ref = _oracle_outputs(cache, d["dA"][b], d["db"][b], d["dc"][b], d["dx"][b])
        fi, ri = ref["info"]
        assert fi[1] in (1, 2) and ri[1] in (1, 2), (b, fi, ri)
        assert st["fwd_istop"][b] in (1, 2) and st["istop"][b] in (1, 2), st
        err = _errors(dict(fwd=out[b], dx=fdx[b], g=g[b], dA=dA[b], db=db[b], dc=dc[b]), ref, cache)
        if minnorm and max(err.values()) > RTOL:
            mn = _minnorm_judge(cache, d, b, out[b], g[b], ref)
            for k, v in err.items():
                if v > RTOL:
                    assert mn["fwd" if k in ("fwd", "dx") else "rev"], (b, k, v)
                    judged += 1
            err = {k: v for k, v in err.items() if v <= RTOL}
        worst = max([worst] + list(err.values()))
    assert worst <= RTOL, worst
    return worst, judged


CONIC_ALL5 = [("m69", 4, 60, [(0, 2), (1, 30), (2, 20), (3, 8), (4, 6), (4, 3)], 42),
              ("m87", 4, 80, [(0, 5), (1, 20), (2, 10), (3, 10), (3, 6), (4, 15), (4, 21)], 41)]


@pytest.mark.parametrize("shape", CONIC_ALL5, ids=[s[0] for s in CONIC_ALL5])
def test_sparse_conic_all_cone_codes_vs_oracle(shape):
    """Every cone code on the converging family (the dense route's
    test_all_cone_codes_converging shapes), A_moi through the sparse route:
    every output at 1e-6 with no relaxed bar, LSQR converged as the oracle's;
    and equal to the dense persistent route's to 1e-7 (same LSQR, only the
    products' summation order differs: both stop at the √eps tests, so the
    two trajectories drift apart by ≈ 1e-9, measured 1.05e-9 on dA)."""
    from diffopt_amd.synthetic import conic_numpy_wellcond
    _, B, n, cones, seed = shape
    d = conic_numpy_wellcond(B, n, cones, seed, pair_norm=1.0)
    res, st = _conic_run(d, cones, True, B)
    _conic_vs_oracle(d, cones, B, res, st)
    import os
    old = os.environ.get("DOPT_CONIC_SPLIT")
    os.environ["DOPT_CONIC_SPLIT"] = "0"
    try:
        dres, _ = _conic_run(d, cones, False, B)
    finally:
        if old is None:
            del os.environ["DOPT_CONIC_SPLIT"]
        else:
            os.environ["DOPT_CONIC_SPLIT"] = old
    for a, b in zip(res[0] + res[1], dres[0] + dres[1]):
        assert relfro(a, b) <= 1e-7


def test_sparse_conic_sparse_pattern():
    """A genuinely sparse A_moi (≈ 5 entries per row, m = 892 ≤ n = 900 — the
    converging side of this family; every cone code): the sparse route against
    the oracle (dense A in the oracle) at 1e-6, LSQR converged as the oracle's;
    an output above 1e-6 (measured: 1.4e-6, LSQR's √eps stopping noise on this
    M) judged by the exact min-norm bar of the dense route's converged shapes."""
    from diffopt_amd.synthetic import conic_numpy_wellcond
    cones = [(0, 10), (3, 20)] * 20 + [(1, 200)] + [(4, 21)] * 2 + [(2, 50)]
    n = 900
    d = conic_numpy_wellcond(2, n, cones, 77, pair_norm=1.0, sparse_k=5)
    assert (d["A"] != 0).mean() < 0.02
    res, st = _conic_run(d, cones, True, 2)
    _, judged = _conic_vs_oracle(d, cones, 2, res, st, minnorm=True)
    assert judged <= 6   # at most half of the 2 × 6 outputs on the min-norm bar


def test_sparse_conic_refusals():
    from diffopt_amd import _lib
    from diffopt_amd.conic import ConicBatch
    from diffopt_amd.synthetic import conic_numpy_wellcond
    cones = [(3, 5), (1, 5)]
    d = conic_numpy_wellcond(1, 8, cones, 5)
    e = ConicBatch(1, 8, cones, sparse=True)
    with pytest.raises(_lib.EngineError, match="dopt_conic_set_csc"):
        e.set(d["A"], d["b"], d["c"], d["x"], d["s"], d["y"])
    e.close()
    big = [(4, 66 * 67 // 2)]
    e = ConicBatch(1, 8, big, sparse=True)
    import scipy.sparse as sp
    m = big[0][1]
    with pytest.raises(_lib.EngineError, match="side 64"):
        e.set_csc(sp.csc_matrix((m, 8)), np.zeros((1, m)), np.zeros((1, 8)), np.zeros((1, 8)), np.zeros((1, m)),
                  np.zeros((1, m)))
    e.close()
