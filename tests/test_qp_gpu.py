"""QP path on the MI355X: HIP engine (through the C-ABI) vs the CPU oracle and
the reference's golden fixtures.  Parity bar (BASELINE.json north_star): 1e-6
relative Frobenius in Float64 on (dz, dλ, dν) forward and reverse; bit-exact
discrete selections (the `iterative` branch and the kept / eliminated
inequality rows, compared as masks).

Both factorisations are covered: the default no-pivot blocked LU with its
threshold test (problems that fail it are re-factorised with partial
pivoting: `lu_kind`), and partial pivoting for every problem (DOPT_LU=0)."""

import json
import os

import numpy as np
import pytest

from oracle import qp as oqp

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
RTOL = 1e-6   # relative Frobenius, north_star
NOPIV, PIVOT, LSQR = 1, 2, 0


def relfro(a, b):
    a = np.asarray(a, dtype=float)
    b = np.asarray(b, dtype=float)
    nb = np.linalg.norm(b)
    return np.linalg.norm(a - b) / (nb if nb > 0 else 1.0)


@pytest.fixture(scope="module")
def QPBatch():
    from diffopt_amd.qp import QPBatch
    return QPBatch


@pytest.fixture(params=["nopiv", "pivot"])
def lu_mode(request, monkeypatch):
    """The factorisation (read by dopt_create): default, or partial pivoting
    for every problem."""
    if request.param == "pivot":
        monkeypatch.setenv("DOPT_LU", "0")
    else:
        monkeypatch.delenv("DOPT_LU", raising=False)
    return request.param


def _fixtures():
    out = []
    for f in ["qp_fixtures.json", "lp_fixtures.json"]:
        with open(os.path.join(HERE, "golden", f)) as fh:
            out += json.load(fh)
    return out


FX = _fixtures()


def _arr(fx):
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


def _engine_solve(QPBatch, a, fw):
    n, m, p = a["Q"].shape[0], a["G"].shape[0], a["A"].shape[0]
    e = QPBatch(1, n, m, p)
    e.set(a["Q"][None], a["G"][None], a["h"][None], a["A"][None], a["z"][None],
          a["lam"][None], a["nu"][None])
    rev = e.reverse(a["dzb"][None])[0]
    kw = {k: v[None] for k, v in fw.items() if v.size}
    fwd = e.forward(**kw)[0]
    it = bool(e.iterative()[0])
    return (rev[:n], rev[n:n + m], rev[n + m:]), (fwd[:n], fwd[n:n + m], fwd[n + m:]), it


@pytest.mark.parametrize("fx", FX, ids=[f["name"] for f in FX])
def test_engine_matches_reference_fixture_and_oracle(QPBatch, lu_mode, fx):
    from test_oracle_golden import qp_outputs
    a, fw = _arr(fx)
    (dz, dl, dn), (fz, fl, fn), it = _engine_solve(QPBatch, a, fw)
    assert it == oqp.is_iterative(a["Q"])            # bit-exact branch selection
    got = qp_outputs(a, fw, solve_rev=lambda: (dz, dl, dn), solve_fwd=lambda: fz)
    for k, v in fx["expect"].items():                 # the reference's own values
        exp = np.array(v, dtype=float).reshape(np.shape(got[k]))
        np.testing.assert_allclose(got[k], exp, atol=fx["atol"], rtol=fx["rtol"], err_msg=k)
    Q, G, h, A, z, lam, nu = (a[k] for k in ["Q", "G", "h", "A", "z", "lam", "nu"])
    rz, rl, rn = oqp.reverse_differentiate(Q, G, h, A, z, lam, nu, a["dzb"])
    oz, ol, on = oqp.forward_differentiate(Q, G, h, A, z, lam, nu, **fw)
    # relative Frobenius per direction on the stacked [dz|dλ|dν] (a block whose
    # exact value is 0 — e.g. dλ of eliminated rows — is measured on that scale)
    for g, r in [((dz, dl, dn), (rz, rl, rn)), ((fz, fl, fn), (oz, ol, on))]:
        assert relfro(np.concatenate(g), np.concatenate(r)) <= RTOL


def _synthetic(batch, n, m, p, phi, seed, dense=False, lam_eps=0.0):
    from diffopt_amd.synthetic import qp_numpy
    return qp_numpy(batch, n, m, p, phi, seed, dense_tangents=dense, lam_eps=lam_eps)


def _oracle_kept(d, b):
    """The reference's elimination set: λ == 0 and (Gz − h) != 0 with Gz − h in
    Julia's sparse mul! order — the rows kept are the complement."""
    s = oqp.gz_minus_h(d["G"][b], d["z"][b], d["h"][b])
    return ~((d["lam"][b] == 0) & (s != 0))


def _check_batch(QPBatch, d, dense=False, kinds=None):
    """GPU vs oracle on every problem; kept-row masks bit-equal; optionally the
    expected factorisation kind per problem.  Returns the engine."""
    B, n = d["z"].shape
    m = d["lam"].shape[1]
    p = d["nu"].shape[1]
    e = QPBatch(B, n, m, p)
    e.set(d["Q"], d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
    fkw = dict(dq=d["dq"], dh=d["dh"], db=d["db"])
    if dense:
        fkw.update(dQ=d["dQ"], dG=d["dG"], dA=d["dA"])
    rev, fwd = e.forward_reverse(d["dl_dz"], **fkw)
    sizes = e.system_size()
    kept = e.kept()
    worst = 0.0
    for b in range(B):
        args = [d[k][b] for k in ["Q", "G", "h", "A", "z", "lam", "nu"]]
        rz, rl, rn = oqp.reverse_differentiate(*args, d["dl_dz"][b])
        fk = {k: v[b] for k, v in fkw.items()}
        oz, ol, on = oqp.forward_differentiate(*args, **fk)
        worst = max(worst, relfro(rev[b], np.concatenate([rz, rl, rn])),
                    relfro(fwd[b], np.concatenate([oz, ol, on])))
        ok = _oracle_kept(d, b)
        np.testing.assert_array_equal(kept[b], ok)   # bit-exact index selection
        assert sizes[b] == n + ok.sum() + p
    assert worst <= RTOL, worst
    if kinds is not None:
        np.testing.assert_array_equal(e.lu_kind(), kinds)
    return e


def test_cfg1_shape_batch(QPBatch, lu_mode):
    _check_batch(QPBatch, _synthetic(4, 50, 80, 30, 0.2, 20250308),
                 kinds=[NOPIV if lu_mode == "nopiv" else PIVOT] * 4)


def test_cfg2_shape_small_batch(QPBatch, lu_mode):
    _check_batch(QPBatch, _synthetic(6, 200, 300, 0, 0.3, 20250309),
                 kinds=[NOPIV if lu_mode == "nopiv" else PIVOT] * 6)


def test_dense_tangents(QPBatch, lu_mode):
    _check_batch(QPBatch, _synthetic(3, 40, 60, 10, 0.5, 7, dense=True), dense=True)


def test_blocked_mid_size(QPBatch, lu_mode):
    """Reduced system 560: several 64-column blocks with a 32-wide tail."""
    _check_batch(QPBatch, _synthetic(2, 300, 400, 20, 0.6, 11))


def test_blocked_cfg3_shape(QPBatch, lu_mode):
    """BASELINE config 3 shape (n=1000, m=1500, 30 % active ⇒ N' = 1450) at batch 2."""
    _check_batch(QPBatch, _synthetic(2, 1000, 1500, 0, 0.3, 20250310))


def test_ragged_shapes(QPBatch, lu_mode):
    for (n, m, p) in [(1, 1, 0), (3, 0, 0), (5, 0, 2), (7, 3, 0), (33, 31, 1), (64, 1, 63),
                      (40, 50, 7), (90, 10, 5)]:
        _check_batch(QPBatch, _synthetic(2, n, m, p, 0.5, 100 + n))


def test_no_elimination_worst_case(QPBatch, lu_mode):
    """Interior-point-like duals: inactive rows get λ = 1e-9 (not exactly 0),
    so nothing is eliminated and N' = n + m (bench.py --lam-eps)."""
    d = _synthetic(3, 200, 300, 0, 0.3, 20250312, lam_eps=1e-9)
    e = _check_batch(QPBatch, d)
    assert (e.system_size() == 500).all()


def _indefinite(d, idx, seed=5):
    """Replace Q of the problems `idx` by a symmetric indefinite matrix with a
    tiny diagonal: the no-pivot LU's first multipliers are ~1e4, so those
    problems fail the threshold test and take partial pivoting.  (z, λ, ν)
    stays a KKT point: the engine never reads q."""
    rng = np.random.default_rng(seed)
    n = d["Q"].shape[1]
    for b in idx:
        S = rng.standard_normal((n, n))
        Q = (S + S.T) / 2
        Q[np.diag_indices(n)] = 1e-4
        d["Q"][b] = Q
    return d


def test_pivot_fallback_mixed_batch(QPBatch, lu_mode):
    """Problems that fail the no-pivot threshold test, interleaved with ones
    that pass: the rejected ones are re-assembled and factorised with partial
    pivoting (their solves run after the speculative no-pivot solves)."""
    d = _indefinite(_synthetic(6, 60, 80, 5, 0.4, 41), [1, 4])
    want = [NOPIV, PIVOT, NOPIV, NOPIV, PIVOT, NOPIV] if lu_mode == "nopiv" else [PIVOT] * 6
    e = _check_batch(QPBatch, d, kinds=want)
    # the split API reuses the same factors.  Not bit-equal to the fused call:
    # there the no-pivot problems' forward sweeps run inside the LU with the
    # 64-block inverses (qp_nopiv.hip fwd_block), the split solves sweep with
    # the 32-block ones — agreement to rounding (measured ≤ 5e-13 relative)
    rev, fwd = e.forward_reverse(d["dl_dz"], dq=d["dq"], dh=d["dh"], db=d["db"])
    e.factor()
    np.testing.assert_allclose(e.reverse(d["dl_dz"]), rev, rtol=1e-11, atol=1e-13)
    np.testing.assert_allclose(e.forward(dq=d["dq"], dh=d["dh"], db=d["db"]), fwd, rtol=1e-11, atol=1e-13)
    np.testing.assert_array_equal(e.lu_kind(), want)


def test_pivot_fallback_every_problem(QPBatch):
    """Every problem rejected (tall blocked systems with several blocks)."""
    d = _indefinite(_synthetic(3, 150, 160, 0, 0.5, 43), [0, 1, 2])
    _check_batch(QPBatch, d, kinds=[PIVOT] * 3)


@pytest.fixture(params=["sym", "general"])
def sym_mode(request, monkeypatch):
    """The no-pivot LU's route for P-symmetric problems (read by dopt_create):
    the P-symmetric one (lower tiles, U12 from L21; default) or the general
    one for every problem (DOPT_SYM=0)."""
    if request.param == "general":
        monkeypatch.setenv("DOPT_SYM", "0")
    else:
        monkeypatch.delenv("DOPT_SYM", raising=False)
    monkeypatch.delenv("DOPT_LU", raising=False)
    return request.param


def test_sym_route_cfg2_shape(QPBatch, sym_mode):
    """The config-2 shape through the P-symmetric route (P = diag(1, λ_k, 1)
    makes P·K symmetric: only the lower trailing tiles are updated, U12 is
    taken from L21) and through the general no-pivot LU: both at the oracle
    bar, and the two agree to rounding."""
    d = _synthetic(4, 200, 300, 0, 0.3, 20250309 + 7)
    e = _check_batch(QPBatch, d, kinds=[NOPIV] * 4)
    np.testing.assert_array_equal(e.info(), 0)


def test_sym_route_32_wide_tail(QPBatch, sym_mode):
    """Reduced size 200, padded to 224 = three 64-blocks + a 32-wide tail: the
    left-looking diagonal launch of the tail block
    forms only the lower 16×16 tiles inside the block (the row-3 tiles and the
    waves past the 32 rows idle), the sweep vectors come through the staged
    strip's padding; every problem at the oracle bar."""
    d = _synthetic(8, 150, 100, 0, 0.5, 20251017)
    e = _check_batch(QPBatch, d, kinds=[NOPIV] * 8)
    np.testing.assert_array_equal(e.info(), 0)
    pads = [(int(s) + 31) // 32 * 32 for s in e.system_size()]
    assert any(p % 64 == 32 and p > 64 for p in pads), pads


def test_sym_and_general_routes_agree(QPBatch, monkeypatch):
    """Same problems (multi-block, with equality rows) through both no-pivot
    routes: equal to ~1e-12 (different rounding, same factors)."""
    d = _synthetic(3, 300, 400, 20, 0.6, 12)
    outs = []
    for mode in ("1", "0"):
        monkeypatch.setenv("DOPT_SYM", mode)
        B, n = d["z"].shape
        e = QPBatch(B, n, d["lam"].shape[1], d["nu"].shape[1])
        e.set(d["Q"], d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
        outs.append(e.forward_reverse(d["dl_dz"], dq=d["dq"], dh=d["dh"], db=d["db"]))
        np.testing.assert_array_equal(e.lu_kind(), [NOPIV] * B)
    for a, b in zip(outs[0], outs[1]):
        assert relfro(a, b) <= 1e-11


def _wilkinson_c(n, c):
    """Wilkinson's growth matrix with multipliers −c: 1 on the diagonal, −c
    below it, 1 in the last column.  Its no-pivot LU keeps every |l| = c but
    the last column grows as (1 + c)^k."""
    W = np.eye(n) - c * np.tril(np.ones((n, n)), -1)
    W[:, -1] = 1.0
    return W


def test_growth_bound_rejects_small_multiplier_growth(QPBatch, monkeypatch):
    """a KKT whose no-pivot LU has small multipliers
    (|l| = 8 ≤ 10, the threshold test passes) but element growth 9^15 ≈ 2e14:
    Q = the Wilkinson-type matrix above (n = 16).  The growth bound |u| ≤
    1e8·max|K| must reject it → partial pivoting, at the oracle bar; a
    well-conditioned neighbour keeps the no-pivot route.  Run on the general
    route (DOPT_SYM=0: Q is not symmetric, so the P-symmetric route would
    reject it earlier, at the assembly's symmetry check — tested below)."""
    d = _synthetic(2, 16, 8, 0, 0.5, 71)
    d["Q"][1] = _wilkinson_c(16, 8.0)
    monkeypatch.setenv("DOPT_SYM", "0")
    monkeypatch.delenv("DOPT_LU", raising=False)
    _check_batch(QPBatch, d, kinds=[NOPIV, PIVOT])


def test_asymmetric_Q_leaves_sym_route(QPBatch, monkeypatch):
    """An asymmetric Q (the reference's Q is always symmetric — its
    quadratic terms are mirrored — but the C-ABI takes any dense Q) under the
    default P-symmetric route: the assembly's symmetry check rejects it and it
    is re-assembled in full and factorised with partial pivoting; results at
    the oracle bar, the symmetric neighbours unaffected."""
    monkeypatch.delenv("DOPT_SYM", raising=False)
    monkeypatch.delenv("DOPT_LU", raising=False)
    d = _synthetic(3, 70, 90, 4, 0.4, 72)
    rng = np.random.default_rng(3)
    d["Q"][1] = d["Q"][1] + 1e-3 * np.triu(rng.standard_normal((70, 70)), 1)
    _check_batch(QPBatch, d, kinds=[NOPIV, PIVOT, NOPIV])


def test_ill_conditioned_Q(QPBatch, sym_mode):
    """Q with condition number 1e8 (eigenvalues log-spaced in [1e-8, 1]).
    Q's own no-pivot LU is harmless (|l| ≤ 1.4), but the kept G rows then
    take multipliers ~ G·U⁻¹ up to 7e6 (measured in numpy on these problems):
    the threshold test rejects every problem — as UMFPACK's threshold pivoting
    would move off those pivots — and partial pivoting matches the oracle at
    1e-6, on both no-pivot routes."""
    d = _synthetic(3, 120, 150, 6, 0.3, 73)
    rng = np.random.default_rng(4)
    for b in range(3):
        V, _ = np.linalg.qr(rng.standard_normal((120, 120)))
        Q = (V * np.logspace(0, -8, 120)) @ V.T
        d["Q"][b] = (Q + Q.T) / 2
    _check_batch(QPBatch, d, kinds=[PIVOT] * 3)


def test_lam_eps_1e12(QPBatch, sym_mode):
    """bench.py --lam-eps at 1e-12: every inactive row kept with λ = 1e-12
    (N' = n + m; the P-symmetric route scales those rows by 1e-12); no-pivot
    route, oracle bar."""
    d = _synthetic(3, 200, 300, 0, 0.3, 20250312, lam_eps=1e-12)
    e = _check_batch(QPBatch, d, kinds=[NOPIV] * 3)
    assert (e.system_size() == 500).all()


def test_reverse_grads_materialised(QPBatch):
    """dopt_qp_reverse_grads: ReverseObjectiveFunction / ReverseConstraintFunction
    of every problem (QuadraticProgram.jl:448-473, :307-314) against the
    oracle's getters, host mode and device mode (bit-identical)."""
    import torch
    d = _synthetic(3, 50, 80, 30, 0.2, 20250308)
    B, n = d["z"].shape
    m, p = d["lam"].shape[1], d["nu"].shape[1]
    e = QPBatch(B, n, m, p)
    e.set(d["Q"], d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
    rev = np.asarray(e.reverse(d["dl_dz"]))
    g = e.reverse_grads(rev)
    for b in range(B):
        dz, dl, dn = rev[b, :n], rev[b, n:n + m], rev[b, n + m:]
        dq, dQ = oqp.reverse_objective(d["z"][b], dz)
        dG, gc = oqp.reverse_constraint_le(d["z"][b], d["lam"][b], dz, dl)
        dA, ac = oqp.reverse_constraint_eq(d["z"][b], d["nu"][b], dz, dn)
        for got, ref in ((g["dq"][b], dq), (g["dQ"][b], dQ), (g["dG"][b], dG),
                         (g["g_const"][b], gc), (g["dA"][b], dA), (g["a_const"][b], ac)):
            np.testing.assert_allclose(got, ref, rtol=1e-14, atol=1e-15)
    dev = {k: torch.as_tensor(v, device="cuda") for k, v in d.items()}
    e2 = QPBatch(B, n, m, p)
    e2.set(dev["Q"], dev["G"], dev["h"], dev["A"], dev["z"], dev["lam"], dev["nu"])
    g2 = e2.reverse_grads(torch.as_tensor(rev, device="cuda"))
    torch.cuda.synchronize()
    for k in g:
        np.testing.assert_array_equal(g2[k].cpu().numpy(), g[k])


def test_csc_staging_matches_dense_and_oracle(QPBatch):
    """dopt_qp_set_csc (MOI matrix form: Julia CSC, Int64, 1-based) densified
    on the device: against the oracle on the same sparse problems, and
    bit-identical to dopt_qp_set with the dense matrices; sparse G/A with an
    empty column; malformed CSC raises."""
    import scipy.sparse as sp
    from diffopt_amd import EngineError
    d = _synthetic(3, 40, 60, 10, 0.5, 77)
    B, n = d["z"].shape
    m, p = 60, 10
    rng = np.random.default_rng(5)
    G = d["G"] * (rng.random(d["G"].shape) < 0.3)
    G[:, :, 3] = 0.0                      # an empty column
    A = d["A"] * (rng.random(d["A"].shape) < 0.5)
    h = np.einsum("bmn,bn->bm", G, d["z"]) - np.einsum("bmn,bn->bm", d["G"], d["z"]) + d["h"]
    e2 = QPBatch(B, n, m, p)
    e2.set_csc([sp.csc_matrix(q) for q in d["Q"]], [sp.csc_matrix(g) for g in G], h,
               [sp.csc_matrix(a) for a in A], d["z"], d["lam"], d["nu"])
    r2, f2 = e2.forward_reverse(d["dl_dz"], dq=d["dq"], dh=d["dh"], db=d["db"])
    for b in range(B):
        args = [d["Q"][b], G[b], h[b], A[b], d["z"][b], d["lam"][b], d["nu"][b]]
        ref_r = np.concatenate(oqp.reverse_differentiate(*args, d["dl_dz"][b]))
        ref_f = np.concatenate(oqp.forward_differentiate(*args, dq=d["dq"][b], dh=d["dh"][b],
                                                         db=d["db"][b]))
        assert relfro(r2[b], ref_r) <= RTOL and relfro(f2[b], ref_f) <= RTOL
    e1 = QPBatch(B, n, m, p)
    e1.set(d["Q"], G, h, A, d["z"], d["lam"], d["nu"])
    r1, f1 = e1.forward_reverse(d["dl_dz"], dq=d["dq"], dh=d["dh"], db=d["db"])
    np.testing.assert_array_equal(r1, r2)
    np.testing.assert_array_equal(f1, f2)
    bad = sp.csc_matrix(G[0])
    bad.indices[0] = 99                   # row index out of range
    with pytest.raises(EngineError):
        e2.set_csc(sp.csc_matrix(d["Q"][0]), bad, h, sp.csc_matrix(A[0]), d["z"], d["lam"], d["nu"])
    # a failed set leaves no model behind: a larger rejected
    # model (dense G: the packed staging buffer grows, freeing the one the
    # previous model's inputs lived in) must not be solved with stale inputs
    big = sp.csc_matrix(d["G"][0] + 1.0)
    big.indices[5] = 99
    with pytest.raises(EngineError):
        e2.set_csc(sp.csc_matrix(d["Q"][0]), big, h, sp.csc_matrix(A[0]), d["z"], d["lam"], d["nu"])
    with pytest.raises(EngineError):
        e2.forward_reverse(d["dl_dz"], dq=d["dq"], dh=d["dh"], db=d["db"])
    with pytest.raises(EngineError):
        e2.reverse(d["dl_dz"])
    # and a good set afterwards works as before
    e2.set_csc([sp.csc_matrix(q) for q in d["Q"]], [sp.csc_matrix(g) for g in G], h,
               [sp.csc_matrix(a) for a in A], d["z"], d["lam"], d["nu"])
    r3, f3 = e2.forward_reverse(d["dl_dz"], dq=d["dq"], dh=d["dh"], db=d["db"])
    np.testing.assert_array_equal(r3, r2)
    np.testing.assert_array_equal(f3, f2)


def test_factor_then_reverse_forward(QPBatch, lu_mode):
    """dopt_qp_factor once, then reverse and forward on the kept factors (the
    reference re-factorises per call): against the oracle, and equal to the
    fused forward_reverse call to rounding (its forward sweeps run inside the
    no-pivot LU; bit-equal under partial pivoting); a second reverse with
    another seed reuses the factorisation."""
    d = _synthetic(5, 30, 40, 5, 0.4, 3)
    B, n = d["z"].shape
    e = QPBatch(B, n, 40, 5)
    e.set(d["Q"], d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
    e.factor()
    r2 = e.reverse(d["dl_dz"])
    f2 = e.forward(dq=d["dq"], dh=d["dh"], db=d["db"])
    seed2 = d["dl_dz"][::-1].copy()
    r3 = e.reverse(seed2)
    for b in range(B):
        args = [d[k][b] for k in ["Q", "G", "h", "A", "z", "lam", "nu"]]
        assert relfro(r2[b], np.concatenate(oqp.reverse_differentiate(*args, d["dl_dz"][b]))) <= RTOL
        assert relfro(r3[b], np.concatenate(oqp.reverse_differentiate(*args, seed2[b]))) <= RTOL
        assert relfro(f2[b], np.concatenate(oqp.forward_differentiate(
            *args, dq=d["dq"][b], dh=d["dh"][b], db=d["db"][b]))) <= RTOL
    r1, f1 = e.forward_reverse(d["dl_dz"], dq=d["dq"], dh=d["dh"], db=d["db"])
    if lu_mode == "nopiv":
        np.testing.assert_allclose(r1, r2, rtol=1e-11, atol=1e-13)
        np.testing.assert_allclose(f1, f2, rtol=1e-11, atol=1e-13)
    else:
        np.testing.assert_array_equal(r1, r2)
        np.testing.assert_array_equal(f1, f2)


def test_large_reduced_system_blocked_route(QPBatch, lu_mode):
    """Reduced systems above the partial-pivoting panel's 1536 rows (here
    1620) take the no-pivot blocked LU (taller solves run in entry chunks);
    with DOPT_LU=0 they take the generic LU."""
    _check_batch(QPBatch, _synthetic(2, 1200, 700, 0, 0.6, 12),
                 kinds=[NOPIV if lu_mode == "nopiv" else PIVOT] * 2)


def test_large_rejected_problem_takes_generic_lu(QPBatch):
    """A tall problem (reduced size > 1536) the no-pivot LU rejects is
    re-assembled and factorised by the generic LU, next to accepted ones and a
    small rejected one (partial-pivoting blocked LU) in the same batch."""
    d = _indefinite(_synthetic(3, 1200, 700, 0, 0.6, 13), [1])
    _check_batch(QPBatch, d, kinds=[NOPIV, PIVOT, NOPIV])


def test_config3_no_elimination_shape(QPBatch):
    """Config 3 with interior-point-like duals (λ = 1e-9 on inactive rows,
    nothing eliminated: N' = 2500, the `--lam-eps` bench case) on the blocked
    route, two problems against the oracle."""
    _check_batch(QPBatch, _synthetic(2, 1000, 1500, 0, 0.3, 14, lam_eps=1e-9), kinds=[NOPIV] * 2)


def test_singular_kkt_raises(QPBatch, lu_mode):
    """λ_i == 0 and s_i == 0 → zero row/column in LHS → SingularException
    (the no-pivot LU rejects the zero pivot; partial pivoting reports it)."""
    from diffopt_amd import SingularException
    Q = np.eye(2)[None]
    G = np.array([[[1.0, 0.0]]])
    z = np.array([[1.0, 2.0]])
    h = np.array([1.0])[None]           # s = Gz − h = 0
    lam = np.zeros((1, 1))
    e = QPBatch(1, 2, 1, 0)
    e.set(Q, G, h, np.zeros((1, 0, 2)), z, lam, np.zeros((1, 0)))
    with pytest.raises(SingularException):
        e.reverse(np.ones((1, 2)))
    assert e.info()[0] > 0


def test_singular_info_in_full_kkt_columns(QPBatch, lu_mode):
    """The zero pivot is reported in the reference LHS's coordinates
    ([z; λ; ν], 1-based), not the reduced system's: row 0 is eliminated
    (λ = 0, s ≠ 0), row 1 (λ = 0, s = 0) is the zero column, reduced column
    3 → LHS column n + 1 + 1 = 4."""
    from diffopt_amd import SingularException
    Q = np.eye(2)[None]
    G = np.array([[[1.0, 0.0], [0.0, 1.0], [1.0, 1.0]]])
    z = np.array([[1.0, 2.0]])
    h = np.array([[3.0, 2.0, 3.0]])     # s = Gz − h = (−2, 0, 0)
    lam = np.array([[0.0, 0.0, 1.0]])
    e = QPBatch(1, 2, 3, 0)
    e.set(Q, G, h, np.zeros((1, 0, 2)), z, lam, np.zeros((1, 0)))
    with pytest.raises(SingularException) as ex:
        e.reverse(np.ones((1, 2)))
    assert e.info()[0] == 4
    assert ex.value.info == 4


def test_lp_iterative_batch_mixed_with_qp(QPBatch, lu_mode):
    """A batch mixing Q == 0 (LSQR branch) and Q != 0 (LU branch)."""
    with open(os.path.join(HERE, "golden", "lp_fixtures.json")) as fh:
        lp = json.load(fh)
    fx = [f for f in lp if f["name"] == "lp_simplex"][0]
    a, fw = _arr(fx)
    n, m = a["Q"].shape[0], a["G"].shape[0]
    Qs = np.stack([a["Q"], np.eye(n)])
    e = QPBatch(2, n, m, 0)
    e.set(Qs, np.stack([a["G"]] * 2), np.stack([a["h"]] * 2), np.zeros((2, 0, n)),
          np.stack([a["z"]] * 2), np.stack([a["lam"]] * 2), np.zeros((2, 0)))
    rev = e.reverse(np.stack([a["dzb"]] * 2))
    assert list(e.iterative()) == [True, False]
    assert e.lu_kind()[0] == LSQR
    for b in range(2):
        rz, rl, rn = oqp.reverse_differentiate(Qs[b], a["G"], a["h"], np.zeros((0, n)),
                                               a["z"], a["lam"], np.zeros(0), a["dzb"])
        assert relfro(rev[b], np.concatenate([rz, rl, rn])) <= RTOL


def test_lsqr_branch_beyond_lds_size(QPBatch):
    """The LSQR branch on a system of n + m + p = 4200 > 4096 unknowns (its
    vectors live in a global workspace; a batch with LU problems too):
    LSQR's own stopping guarantee on the KKT residual, and the LU problem
    against the oracle."""
    rng = np.random.default_rng(9)
    n, m = 200, 4000
    d = _synthetic(2, n, m, 0, 0.02, 31)
    d["Q"][0] = 0.0                              # problem 0: LP → LSQR on the full LHS
    e = QPBatch(2, n, m, 0)
    e.set(d["Q"], d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
    seed = rng.standard_normal((2, n))
    rev = np.asarray(e.reverse(seed))
    assert list(e.iterative()) == [True, False]
    LHS = oqp.create_LHS_matrix(d["z"][0], d["lam"][0], d["Q"][0], d["G"][0], d["h"][0], d["A"][0])
    rhs = np.concatenate([seed[0], np.zeros(m)])
    x = -rev[0]
    r = np.linalg.norm(LHS.T @ (LHS @ x - rhs))   # least-squares optimality (LSQR's test2)
    assert r <= 1e-6 * np.linalg.norm(LHS) ** 2 * np.linalg.norm(x) + 1e-6 * np.linalg.norm(rhs)
    args = [d[k][1] for k in ["Q", "G", "h", "A", "z", "lam", "nu"]]
    assert relfro(rev[1], np.concatenate(oqp.reverse_differentiate(*args, seed[1]))) <= RTOL


def test_device_mode_matches_host_mode(QPBatch):
    import torch
    d = _synthetic(3, 20, 30, 4, 0.3, 5)
    B, n = d["z"].shape
    e = QPBatch(B, n, 30, 4)
    e.set(d["Q"], d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
    r1, f1 = e.forward_reverse(d["dl_dz"], dq=d["dq"], dh=d["dh"], db=d["db"])
    t = {k: torch.tensor(v, device="cuda") for k, v in d.items()}
    e2 = QPBatch(B, n, 30, 4)
    e2.set(t["Q"], t["G"], t["h"], t["A"], t["z"], t["lam"], t["nu"])
    r2, f2 = e2.forward_reverse(t["dl_dz"], dq=t["dq"], dh=t["dh"], db=t["db"])
    np.testing.assert_array_equal(r1, r2.cpu().numpy())
    np.testing.assert_array_equal(f1, f2.cpu().numpy())


def test_output_buffers_are_validated(QPBatch):
    """Caller-supplied outputs of the wrong dtype, shape, layout or memory kind
    raise before any kernel writes."""
    import torch
    d = _synthetic(2, 10, 12, 2, 0.3, 6)
    e = QPBatch(2, 10, 12, 2)
    e.set(d["Q"], d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
    L = 24
    for bad in (np.empty((2, L), np.float32), np.empty((2, L - 1)), np.empty((L, 2)).T,
                torch.empty(2, L, dtype=torch.float64, device="cuda")):
        with pytest.raises(TypeError):
            e.forward_reverse(d["dl_dz"], dq=d["dq"], out_rev=bad, out_fwd=np.empty((2, L)))


@pytest.mark.parametrize("cfg", [(200, 300, 20250309), (1000, 1500, 20250310)],
                         ids=["config2", "config3"])
def test_full_batch_kkt_residual_property(QPBatch, cfg):
    """BASELINE configs 2 and 3 at full batch (1024 × n=200, m=300 and
    1024 × n=1000, m=1500): size-independent check — every solution satisfies
    its KKT system (reverse: LHS x = rhs, forward: LHSᵀ x = rhs) to 1e-9
    relative, computed in fp64 on the GPU; every problem passes the no-pivot
    threshold test; the kept masks equal a GPU recount of λ == 0 ∧ s ≠ 0."""
    import torch
    from diffopt_amd.synthetic import qp_torch
    n, m, seed = cfg
    p = 0
    d = qp_torch(1024, n, m, p, 0.3, seed)
    e = QPBatch(1024, n, m, p)
    e.set(d["Q"], d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
    rev, fwd = e.forward_reverse(d["dl_dz"], dq=d["dq"], dh=d["dh"], db=d["db"])
    torch.cuda.synchronize()
    Q, G, z, lam = d["Q"], d["G"], d["z"], d["lam"]
    s = torch.einsum("bmn,bn->bm", G, z) - d["h"]
    # reverse: −x = rev ; LHS x = [dl; 0]
    xz, xl = -rev[:, :n], -rev[:, n:]
    r1 = torch.einsum("bij,bj->bi", Q, xz) + torch.einsum("bmn,bm->bn", G, lam * xl) - d["dl_dz"]
    r2 = torch.einsum("bmn,bn->bm", G, xz) + s * xl
    res = torch.sqrt((r1 ** 2).sum(1) + (r2 ** 2).sum(1)) / torch.linalg.norm(d["dl_dz"], dim=1)
    assert float(res.max()) < 1e-9
    # forward: LHSᵀ y = [dq; −λ dh]
    yz, yl = -fwd[:, :n], -fwd[:, n:]
    f1 = torch.einsum("bji,bj->bi", Q, yz) + torch.einsum("bmn,bm->bn", G, yl) - d["dq"]
    f2 = lam * torch.einsum("bmn,bn->bm", G, yz) + s * yl - (-lam * d["dh"])
    nrm = torch.sqrt((d["dq"] ** 2).sum(1) + ((lam * d["dh"]) ** 2).sum(1))
    res = torch.sqrt((f1 ** 2).sum(1) + (f2 ** 2).sum(1)) / nrm
    assert float(res.max()) < 1e-9
    assert (e.info() == 0).all()
    assert (e.lu_kind() == NOPIV).all()
    # by construction inactive rows have s = −U(0.5, 1.5), far from 0, so the
    # kept set is exactly the active set whatever the summation order
    kept = ~((lam == 0) & (s != 0)).cpu().numpy()
    np.testing.assert_array_equal(e.kept(), kept)
    np.testing.assert_array_equal(e.system_size(), n + kept.sum(1))
    del d, rev, fwd, Q, G, z, lam, s
    e.close()
    torch.cuda.empty_cache()


def test_profiling_restricted_to_named_phases(QPBatch):
    """set_profiling(phases=[...]) times only the named phases (the bench's
    timed region), set_profiling(True) every phase; results unchanged."""
    d = _synthetic(4, 50, 80, 30, 0.2, 20250311)
    B, n = d["z"].shape
    e = QPBatch(B, n, d["lam"].shape[1], d["nu"].shape[1])
    e.set(d["Q"], d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
    kw = dict(dq=d["dq"], dh=d["dh"], db=d["db"])
    e.set_profiling(True)
    r_all, f_all = e.forward_reverse(d["dl_dz"], **kw)
    e.set_profiling(False)
    every = e.phase_times()
    assert {"qp_assemble", "qp_lu", "qp_rhs", "qp_solve", "qp_output"} <= set(every)
    e.set_profiling(True, phases=["qp_lu"])
    r_one, f_one = e.forward_reverse(d["dl_dz"], **kw)
    e.set_profiling(False)
    one = e.phase_times()
    assert set(one) == {"qp_lu"} and one["qp_lu"][1] == 1 and one["qp_lu"][0] > 0
    np.testing.assert_array_equal(r_one, r_all)
    np.testing.assert_array_equal(f_one, f_all)
    with pytest.raises(ValueError):
        e.set_profiling(True, phases=["no_such_phase"])


@pytest.mark.parametrize("shape", [(6, 40, 60, 4), (3, 150, 200, 10)], ids=["small", "multi-block"])
def test_left_looking_factors_serve_every_solve(QPBatch, monkeypatch, shape):
    """The left-looking P-symmetric route stores only L (U = D·P⁻¹·Lᵀ·P): the
    fused call's backward sweeps go through Lᵀ, later single-direction and
    multi-RHS solves on the same factors materialise U first.  Every result
    against the oracle, and the routes agree with the right-looking LU
    (DOPT_LEFT=0) to rounding."""
    monkeypatch.delenv("DOPT_LEFT", raising=False)
    monkeypatch.delenv("DOPT_LU", raising=False)
    monkeypatch.delenv("DOPT_SYM", raising=False)
    B, n, m, p = shape
    d = _synthetic(B, n, m, p, 0.35, 4242 + n)
    e = QPBatch(B, n, m, p)
    e.set(d["Q"], d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
    fkw = dict(dq=d["dq"], dh=d["dh"], db=d["db"])
    r1, f1 = e.forward_reverse(d["dl_dz"], **fkw)
    assert e.sym_route().all()
    r2 = e.reverse(d["dl_dz"])              # U materialised from L here
    f2 = e.forward(**fkw)
    seeds = np.stack([d["dl_dz"], d["dl_dz"][::-1].copy(), 2.0 * d["dl_dz"]])
    rk = e.reverse_k(seeds)
    for b in range(B):
        args = [d[k][b] for k in ["Q", "G", "h", "A", "z", "lam", "nu"]]
        ref_r = np.concatenate(oqp.reverse_differentiate(*args, d["dl_dz"][b]))
        ref_f = np.concatenate(oqp.forward_differentiate(*args, **{k: v[b] for k, v in fkw.items()}))
        for got in (r1[b], r2[b], rk[0, b], 0.5 * rk[2, b]):
            assert relfro(got, ref_r) <= RTOL
        assert relfro(rk[1, b], np.concatenate(oqp.reverse_differentiate(*args, seeds[1, b]))) <= RTOL
        for got in (f1[b], f2[b]):
            assert relfro(got, ref_f) <= RTOL
    assert relfro(r2, r1) <= 1e-10
    e.close()
    monkeypatch.setenv("DOPT_LEFT", "0")
    g = QPBatch(B, n, m, p)
    g.set(d["Q"], d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
    r3, f3 = g.forward_reverse(d["dl_dz"], **fkw)
    assert relfro(r3, r1) <= 1e-9 and relfro(f3, f1) <= 1e-9
    g.close()


def test_plug_point_adjoint_reuses_factors():
    """MI355XSolver: the reference's second call per model passes LHS' (the
    adjoint of the LHS just solved, QuadraticProgram.jl:335, :438); the solver
    answers it from the same factorisation (dopt_lhs_resolve, transposed),
    against numpy at 1e-10, in both orders, once per factorisation; the same
    array twice, or a new array, is factorised again; a singular LHS' raises
    as LHS did."""
    from diffopt_amd import SingularException
    from diffopt_amd.qp import MI355XSolver
    rng = np.random.default_rng(5)
    rows = 90
    L = rng.standard_normal((rows, rows)) + rows ** 0.5 * np.eye(rows)
    r = rng.standard_normal(rows)
    s = MI355XSolver()
    x = s.solve_system(L, r)
    xt = s.solve_system(L.T, r)
    assert s.resolves == 1
    assert np.linalg.norm(x - np.linalg.solve(L, r)) <= 1e-10 * np.linalg.norm(x)
    assert np.linalg.norm(xt - np.linalg.solve(L.T, r)) <= 1e-10 * np.linalg.norm(xt)
    L2 = rng.standard_normal((rows, rows)) + rows ** 0.5 * np.eye(rows)
    xt2 = s.solve_system(L2.T, r)          # a new array: factorised
    x2 = s.solve_system(L2, r)             # then its parent: reused
    assert s.resolves == 2
    assert np.linalg.norm(x2 - np.linalg.solve(L2, r)) <= 1e-10 * np.linalg.norm(x2)
    assert np.linalg.norm(xt2 - np.linalg.solve(L2.T, r)) <= 1e-10 * np.linalg.norm(xt2)
    s.solve_system(L2, r)                  # one reuse per factorisation: factorised again
    assert s.resolves == 2
    s.solve_system(L2, r)                  # the same array twice: factorised again
    assert s.resolves == 2
    S = L.copy()
    S[:, 3] = 0.0
    with pytest.raises(SingularException):
        s.solve_system(S, r)
    with pytest.raises(SingularException):
        s.solve_system(S.T, r)
    assert s.resolves == 3
    s.close()


def _fma_exact(a, b, c):
    """fma(a, b, c) correctly rounded (exact rational arithmetic)."""
    from fractions import Fraction
    return float(Fraction(a) * Fraction(b) + Fraction(c))


def test_weakly_active_rows_kept_bit_exact(QPBatch, lu_mode):
    """Rows with λ_i = 0 whose h_i is G_i·z summed in Julia's sparse `mul!`
    order (product and sum rounded separately) have s_i = (Gz − h)_i == 0
    exactly: the reference keeps them (QuadraticProgram.jl:256-282 eliminates
    nothing; the engine's exact elimination must keep exactly the rows with
    s ≠ 0).  Such a row makes the KKT column of λ_i all zero, so the reference's
    `LHS \\ RHS` raises SingularException — and so must the engine.  Round 6
    found the prepare kernels' s FMA-contracted (HIP's `__dadd_rn(x,
    __dmul_rn(a, b))` is plain `x + a*b` and fuses): with an FMA, s_i comes out
    ≈ 1e-17 instead of 0 on these rows, the row is eliminated, and the kept
    mask and the singular verdict both differ from the reference's."""
    from diffopt_amd import _lib
    d = _synthetic(2, 40, 60, 5, 0.3, 20251018)
    B, n = d["z"].shape
    m = d["lam"].shape[1]
    teeth = 0
    for b in range(B):
        ina = np.flatnonzero(d["lam"][b] == 0)
        gz = oqp.gz_minus_h(d["G"][b], d["z"][b], np.zeros(m))   # Julia-order G·z
        d["h"][b, ina] = gz[ina]
        for i in ina:   # the FMA form of the same sum: non-zero on most of these rows
            acc = 0.0
            for j in range(n):
                acc = _fma_exact(d["G"][b, i, j], d["z"][b, j], acc)
            teeth += (acc - gz[i]) != 0.0
    assert teeth >= 2, "the construction must separate FMA from Julia-order sums"
    e = QPBatch(B, n, m, 5)
    e.set(d["Q"], d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
    info = e.factor(singular_ok=True)
    assert info > 0                                       # singular, as `LHS \\ RHS`
    kept = e.kept()
    for b in range(B):
        np.testing.assert_array_equal(kept[b], _oracle_kept(d, b))   # bit-exact index selection
        L = oqp.create_LHS_matrix(d["z"][b], d["lam"][b], d["Q"][b], d["G"][b], d["h"][b], d["A"][b])
        assert not np.all(np.any(L != 0, axis=0))          # the oracle's LHS has a zero column
    with pytest.raises(_lib.SingularException):
        e.reverse(d["dl_dz"])
