"""QP path on the MI355X: HIP engine vs the CPU oracle and the reference's
golden fixtures.  Parity bar (BASELINE.json north_star): 1e-6 relative
Frobenius in Float64 on (dz, dλ, dν) forward and reverse; bit-exact discrete
selections (iterative branch, eliminated-row set)."""

import json
import os

import numpy as np
import pytest

from oracle import qp as oqp

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
RTOL = 1e-6   # relative Frobenius, north_star


def relfro(a, b):
    a = np.asarray(a, dtype=float)
    b = np.asarray(b, dtype=float)
    nb = np.linalg.norm(b)
    return np.linalg.norm(a - b) / (nb if nb > 0 else 1.0)


@pytest.fixture(scope="module")
def QPBatch():
    from diffopt_amd.qp import QPBatch
    return QPBatch


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
def test_engine_matches_reference_fixture_and_oracle(QPBatch, fx):
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


def _synthetic(batch, n, m, p, phi, seed, dense=False):
    from diffopt_amd.synthetic import qp_numpy
    return qp_numpy(batch, n, m, p, phi, seed, dense_tangents=dense)


def _check_batch(QPBatch, d, dense=False, fast_max=None):
    B, n = d["z"].shape
    m = d["lam"].shape[1]
    p = d["nu"].shape[1]
    e = QPBatch(B, n, m, p)
    if fast_max is not None:
        e.set_fast_max(fast_max)
    e.set(d["Q"], d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
    fkw = dict(dq=d["dq"], dh=d["dh"], db=d["db"])
    if dense:
        fkw.update(dQ=d["dQ"], dG=d["dG"], dA=d["dA"])
    rev, fwd = e.forward_reverse(d["dl_dz"], **fkw)
    sizes = e.system_size()
    worst = 0.0
    for b in range(B):
        args = [d[k][b] for k in ["Q", "G", "h", "A", "z", "lam", "nu"]]
        rz, rl, rn = oqp.reverse_differentiate(*args, d["dl_dz"][b])
        fk = {k: v[b] for k, v in fkw.items()}
        oz, ol, on = oqp.forward_differentiate(*args, **fk)
        worst = max(worst, relfro(rev[b], np.concatenate([rz, rl, rn])),
                    relfro(fwd[b], np.concatenate([oz, ol, on])))
        # bit-exact elimination set: λ == 0 and (Gz − h) != 0 (Julia summation order)
        s = oqp.gz_minus_h(d["G"][b], d["z"][b], d["h"][b])
        kept = np.count_nonzero(~((d["lam"][b] == 0) & (s != 0)))
        assert sizes[b] == n + kept + p
    assert worst <= RTOL, worst
    return e


def test_cfg1_shape_batch(QPBatch):
    _check_batch(QPBatch, _synthetic(4, 50, 80, 30, 0.2, 20250308))


def test_cfg2_shape_small_batch(QPBatch):
    _check_batch(QPBatch, _synthetic(6, 200, 300, 0, 0.3, 20250309))


def test_dense_tangents(QPBatch):
    _check_batch(QPBatch, _synthetic(3, 40, 60, 10, 0.5, 7, dense=True), dense=True)


def test_blocked_path_mid_size(QPBatch):
    """Reduced system 512 < N' ≤ 1536 (here 560) takes the blocked step path
    (panel / U12 / MFMA trailing-update launches over the whole batch)."""
    _check_batch(QPBatch, _synthetic(2, 300, 400, 20, 0.6, 11))


def test_blocked_path_cfg3_shape(QPBatch):
    """BASELINE config 3 shape (n=1000, m=1500, 30 % active ⇒ N' = 1450, three
    panel rows per thread) at batch 2."""
    _check_batch(QPBatch, _synthetic(2, 1000, 1500, 0, 0.3, 20250310))


def test_fused_path_small_and_ragged(QPBatch):
    """fast_max = 512 routes every LU problem with N' ≤ 512 to the fused
    one-workgroup-per-problem kernel (the default route is the blocked path)."""
    _check_batch(QPBatch, _synthetic(3, 200, 300, 0, 0.3, 20250309), fast_max=512)
    _check_batch(QPBatch, _synthetic(3, 50, 80, 30, 0.2, 20250308), fast_max=512)
    _check_batch(QPBatch, _synthetic(3, 40, 60, 10, 0.5, 7, dense=True), dense=True, fast_max=512)
    for (n, m, p) in [(1, 1, 0), (3, 0, 0), (5, 0, 2), (7, 3, 0), (33, 31, 1), (64, 1, 63)]:
        _check_batch(QPBatch, _synthetic(2, n, m, p, 0.5, 100 + n), fast_max=512)


def test_blocked_path_forced_small_and_ragged(QPBatch):
    """fast_max = 0 forces every LU problem onto the blocked path: config-1/2
    shapes and ragged sizes (p = 0, m = 0, N' not a multiple of 32)."""
    _check_batch(QPBatch, _synthetic(3, 200, 300, 0, 0.3, 20250309), fast_max=0)
    _check_batch(QPBatch, _synthetic(3, 50, 80, 30, 0.2, 20250308), fast_max=0)
    for (n, m, p) in [(1, 1, 0), (3, 0, 0), (7, 3, 0), (33, 31, 1), (64, 1, 63)]:
        _check_batch(QPBatch, _synthetic(2, n, m, p, 0.5, 100 + n), fast_max=0)


@pytest.mark.parametrize("group", ["2", "3", "4"])
def test_blocked_panel_groups(QPBatch, monkeypatch, group):
    """Left-looking panel groups (DOPT_LU_GROUP, read at handle creation):
    separate U12 kernel with the group's pending update, rank-32g trailing
    update; shapes whose panel count is not a multiple of the group."""
    monkeypatch.setenv("DOPT_LU_GROUP", group)
    _check_batch(QPBatch, _synthetic(3, 200, 300, 0, 0.3, 20250309))
    _check_batch(QPBatch, _synthetic(2, 300, 400, 20, 0.6, 11))
    for (n, m, p) in [(7, 3, 0), (33, 31, 1), (64, 1, 63)]:
        _check_batch(QPBatch, _synthetic(2, n, m, p, 0.5, 100 + n))


@pytest.mark.parametrize("ct", ["2", "4"])
def test_blocked_update_strips(QPBatch, monkeypatch, ct):
    """Strip trailing-update kernel (DOPT_UPD_CT column tiles per workgroup,
    prefetched): bit-identical to the one-tile kernel, and oracle parity on
    shapes with ragged column-tile counts."""
    d = _synthetic(2, 300, 400, 20, 0.6, 11)
    B, n = d["z"].shape
    outs = []
    for env in (None, ct):
        if env is None:
            monkeypatch.delenv("DOPT_UPD_CT", raising=False)
        else:
            monkeypatch.setenv("DOPT_UPD_CT", env)
        e = QPBatch(B, n, 400, 20)
        e.set(d["Q"], d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
        outs.append(e.forward_reverse(d["dl_dz"], dq=d["dq"], dh=d["dh"], db=d["db"]))
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    np.testing.assert_array_equal(outs[0][1], outs[1][1])
    _check_batch(QPBatch, _synthetic(2, 200, 300, 0, 0.3, 20250309))
    _check_batch(QPBatch, _synthetic(2, 1000, 1500, 0, 0.3, 20250310))


@pytest.mark.parametrize("B", [16, 12])
def test_solve2_interleaved_order(QPBatch, monkeypatch, B):
    """Both-direction solve with the directions of each group of 8 problems
    adjacent in dispatch order (DOPT_SOLVE_ILV=1, the default; B % 8 != 0
    falls back to the split order): bit-identical to the split order, and
    oracle parity."""
    d = _synthetic(B, 120, 150, 10, 0.4, 20250311)
    n = d["z"].shape[1]
    outs = []
    for env in ("0", "1"):
        monkeypatch.setenv("DOPT_SOLVE_ILV", env)
        e = QPBatch(B, n, 150, 10)
        e.set(d["Q"], d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
        outs.append(e.forward_reverse(d["dl_dz"], dq=d["dq"], dh=d["dh"], db=d["db"]))
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    np.testing.assert_array_equal(outs[0][1], outs[1][1])
    monkeypatch.delenv("DOPT_SOLVE_ILV")
    _check_batch(QPBatch, d)


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


def test_csc_staging_matches_dense(QPBatch):
    """dopt_qp_set_csc (MOI matrix form: Julia CSC, Int64, 1-based) densified
    on the device gives bit-identical sensitivities to dopt_qp_set with the
    same dense matrices; sparse G/A with empty columns; malformed CSC raises."""
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
    e1 = QPBatch(B, n, m, p)
    e1.set(d["Q"], G, h, A, d["z"], d["lam"], d["nu"])
    r1, f1 = e1.forward_reverse(d["dl_dz"], dq=d["dq"], dh=d["dh"], db=d["db"])
    e2 = QPBatch(B, n, m, p)
    e2.set_csc([sp.csc_matrix(q) for q in d["Q"]], [sp.csc_matrix(g) for g in G], h,
               [sp.csc_matrix(a) for a in A], d["z"], d["lam"], d["nu"])
    r2, f2 = e2.forward_reverse(d["dl_dz"], dq=d["dq"], dh=d["dh"], db=d["db"])
    np.testing.assert_array_equal(r1, r2)
    np.testing.assert_array_equal(f1, f2)
    bad = sp.csc_matrix(G[0])
    bad.indices[0] = 99                   # row index out of range
    with pytest.raises(EngineError):
        e2.set_csc(sp.csc_matrix(d["Q"][0]), bad, h, sp.csc_matrix(A[0]), d["z"], d["lam"], d["nu"])


def test_blocked_matches_fused_and_split(QPBatch):
    """Same batch through the fused kernel and the blocked path: agreement to
    rounding (different accumulation order only); blocked split calls
    (factor → reverse → forward) bit-equal to the blocked fused call."""
    d = _synthetic(4, 120, 200, 10, 0.4, 21)
    B, n = d["z"].shape
    e1 = QPBatch(B, n, 200, 10)
    e1.set_fast_max(512)
    e1.set(d["Q"], d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
    r1, f1 = e1.forward_reverse(d["dl_dz"], dq=d["dq"], dh=d["dh"], db=d["db"])
    e2 = QPBatch(B, n, 200, 10)
    e2.set_fast_max(0)
    e2.set(d["Q"], d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
    r2, f2 = e2.forward_reverse(d["dl_dz"], dq=d["dq"], dh=d["dh"], db=d["db"])
    for a, b in ((r1, r2), (f1, f2)):
        assert max(relfro(a[i], b[i]) for i in range(B)) <= 1e-11
    e2.factor()
    r3 = e2.reverse(d["dl_dz"])
    f3 = e2.forward(dq=d["dq"], dh=d["dh"], db=d["db"])
    np.testing.assert_array_equal(r2, r3)
    np.testing.assert_array_equal(f2, f3)


def test_mixed_routes_in_one_batch(QPBatch):
    """One batch whose problems take different paths — fused (N' ≤ fast_max)
    and blocked (N' > fast_max), interleaved — with forward tangents that
    reach eliminated rows (the `full` RHS buffer both paths share).  The LSQR
    branch in a mixed batch: test_lp_iterative_batch_mixed_with_qp."""
    lo = _synthetic(3, 60, 80, 4, 0.2, 31)    # N' = 60 + 16 + 4 = 80
    hi = _synthetic(3, 60, 80, 4, 0.6, 32)    # N' = 60 + 48 + 4 = 112 (48 + 4 < n: LICQ)
    d = {k: np.concatenate([np.stack([lo[k][i], hi[k][i]]) for i in range(3)]) for k in lo}
    _check_batch(QPBatch, d, fast_max=100)


def test_generic_large_system_path(QPBatch):
    """Reduced system > 1536 unknowns takes the generic LU kernel."""
    _check_batch(QPBatch, _synthetic(2, 1200, 700, 0, 0.6, 12))


def test_ragged_shapes(QPBatch):
    for (n, m, p) in [(1, 1, 0), (3, 0, 0), (5, 0, 2), (7, 3, 0), (33, 31, 1), (64, 1, 63)]:
        _check_batch(QPBatch, _synthetic(2, n, m, p, 0.5, 100 + n))


def test_reverse_forward_separately_equal_fused(QPBatch):
    d = _synthetic(5, 30, 40, 5, 0.4, 3)
    B, n = d["z"].shape
    e = QPBatch(B, n, 40, 5)
    e.set(d["Q"], d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
    r1, f1 = e.forward_reverse(d["dl_dz"], dq=d["dq"], dh=d["dh"], db=d["db"])
    e.factor()
    r2 = e.reverse(d["dl_dz"])
    f2 = e.forward(dq=d["dq"], dh=d["dh"], db=d["db"])
    np.testing.assert_array_equal(r1, r2)
    np.testing.assert_array_equal(f1, f2)


@pytest.mark.parametrize("fast_max", [512, 0])
def test_singular_kkt_raises(QPBatch, fast_max):
    """λ_i == 0 and s_i == 0 → zero row/column in LHS → SingularException
    (fused path and blocked path)."""
    from diffopt_amd import SingularException
    Q = np.eye(2)[None]
    G = np.array([[[1.0, 0.0]]])
    z = np.array([[1.0, 2.0]])
    h = np.array([1.0])[None]           # s = Gz − h = 0
    lam = np.zeros((1, 1))
    e = QPBatch(1, 2, 1, 0)
    e.set_fast_max(fast_max)
    e.set(Q, G, h, np.zeros((1, 0, 2)), z, lam, np.zeros((1, 0)))
    with pytest.raises(SingularException):
        e.reverse(np.ones((1, 2)))
    assert e.info()[0] > 0


def test_lp_iterative_batch_mixed_with_qp(QPBatch):
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
    for b in range(2):
        rz, rl, rn = oqp.reverse_differentiate(Qs[b], a["G"], a["h"], np.zeros((0, n)),
                                               a["z"], a["lam"], np.zeros(0), a["dzb"])
        assert relfro(rev[b], np.concatenate([rz, rl, rn])) <= RTOL


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


@pytest.mark.parametrize("cfg", [(200, 300, 20250309), (1000, 1500, 20250310)],
                         ids=["config2", "config3"])
def test_full_batch_kkt_residual_property(QPBatch, cfg):
    """BASELINE configs 2 and 3 at full batch (1024 × n=200, m=300 and
    1024 × n=1000, m=1500): size-independent check — every solution satisfies
    its KKT system (reverse: LHS x = rhs, forward: LHSᵀ x = rhs) to 1e-9
    relative, computed in fp64 on the GPU — plus bit-exact kept-set sizes
    against a GPU recount of λ == 0 ∧ s ≠ 0."""
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
    # by construction inactive rows have s = −U(0.5, 1.5), far from 0, so the
    # kept set is exactly the active set whatever the summation order
    kept = (~((lam == 0) & (s != 0))).sum(1).cpu().numpy()
    np.testing.assert_array_equal(e.system_size(), n + kept)
    del d, rev, fwd, Q, G, z, lam, s
    e.close()
    torch.cuda.empty_cache()
