"""The reference's narrow QP plug point, ``QuadraticProgram.LinearAlgebraSolver``
(QuadraticProgram.jl:475-502; test/moi_wrapper.jl:74-98 plugs a custom
solver): ``solve_system(solver, LHS, RHS, iterative)`` =
``iterative ? lsqr(LHS, RHS) : LHS \\ RHS`` on the device (dopt_lhs_solve,
diffopt_amd.qp.solve_system).  Checked on the reference's own use: the
assembled KKT LHS of a QP (reverse) and its adjoint (forward), against the
oracle's full-KKT solve; LSQR against the oracle's IterativeSolvers
restatement; a singular LHS raises SingularException."""

import numpy as np
import pytest

from oracle import lsqr as olsqr
from oracle import qp as oqp

pytestmark = pytest.mark.gpu


def _kkt(seed, n=40, m=60, p=5):
    from diffopt_amd.synthetic import qp_numpy
    d = qp_numpy(1, n, m, p, 0.4, seed)
    Q, G, h, A, z, lam = (d[k][0] for k in ["Q", "G", "h", "A", "z", "lam"])
    return d, (Q, G, h, A, z, lam), oqp.create_LHS_matrix(z, lam, Q, G, h, A)


def test_reverse_and_forward_systems():
    from diffopt_amd.qp import solve_system
    d, a, LHS = _kkt(5)
    L = np.asarray(LHS.todense() if hasattr(LHS, "todense") else LHS)
    N = L.shape[0]
    rng = np.random.default_rng(1)
    rhs = rng.standard_normal(N)
    x = solve_system(L, rhs)
    np.testing.assert_allclose(x, np.linalg.solve(L, rhs), rtol=1e-10, atol=1e-12)
    xt = solve_system(L.T, rhs)                                   # LHS' (forward, :438)
    np.testing.assert_allclose(xt, np.linalg.solve(L.T, rhs), rtol=1e-10, atol=1e-12)
    R = rng.standard_normal((N, 3))                               # several right-hand sides
    np.testing.assert_allclose(solve_system(L, R), np.linalg.solve(L, R), rtol=1e-10, atol=1e-12)
    # batched: two problems at once
    _, _, L2 = _kkt(6)
    L2 = np.asarray(L2.todense() if hasattr(L2, "todense") else L2)
    if L2.shape == L.shape:
        Xb = solve_system(np.stack([L, L2]), np.stack([rhs, rhs]))
        np.testing.assert_allclose(Xb[1], np.linalg.solve(L2, rhs), rtol=1e-10, atol=1e-12)


def test_iterative_branch_is_lsqr():
    from diffopt_amd.qp import solve_system
    rng = np.random.default_rng(2)
    # well-conditioned (σ ∈ ≈[0.9, 1.1]): LSQR stops at its √eps tests within a
    # few iterations, so the two runs agree far below north_star's 1e-6 bar
    A = np.eye(30) + 0.1 * rng.standard_normal((30, 30)) / np.sqrt(30)
    b = rng.standard_normal(30)
    x = solve_system(A, b, iterative=True)
    ref = olsqr.lsqr_dense(A, b)
    assert np.linalg.norm(x - ref) / np.linalg.norm(ref) <= 1e-6


def test_singular_raises():
    from diffopt_amd import _lib
    from diffopt_amd.qp import solve_system
    rng = np.random.default_rng(3)
    A = rng.standard_normal((20, 20))
    A[:, 7] = 0.0                                                 # a zero column: exactly singular
    with pytest.raises(_lib.SingularException):
        solve_system(A, rng.standard_normal(20))


def test_cached_solver_handle():
    """MI355XSolver keeps one engine handle per (batch, rows) across calls
    (the reference calls solve_system with LHS, then LHS', per
    model, and loops models): the reverse / forward pair and a loop over
    models of two sizes on one solver give exactly the fresh-handle results,
    and a singular system in between does not poison the cached handle.  The
    cached handle's later calls stage through one pinned copy each way (its
    first, like every fresh handle's, through pageable copies): the
    comparisons against fresh handles check the two against each other."""
    from diffopt_amd import _lib
    from diffopt_amd.qp import MI355XSolver, solve_system
    s = MI355XSolver()
    rng = np.random.default_rng(11)
    for seed, shape in ((21, (40, 60, 5)), (22, (40, 60, 5)), (23, (20, 30, 4)), (24, (40, 60, 5))):
        _, _, LHS = _kkt(seed, *shape)
        L = np.asarray(LHS.todense() if hasattr(LHS, "todense") else LHS)
        rhs = rng.standard_normal(L.shape[0])
        for M in (L, L.T):
            got = s.solve_system(M, rhs)
            if M is L:   # factorised here: the fresh-handle result exactly
                np.testing.assert_array_equal(got, solve_system(M, rhs))
            else:        # LHS': a transposed solve on L's factors (dopt_lhs_resolve)
                np.testing.assert_allclose(got, solve_system(M, rhs), rtol=1e-12, atol=1e-14)
            np.testing.assert_allclose(got, np.linalg.solve(M, rhs), rtol=1e-10, atol=1e-12)
        if seed == 22:
            Z = L.copy()
            Z[:, 3] = 0.0
            with pytest.raises(_lib.SingularException):
                s.solve_system(Z, rhs)
    assert s._key == (1, L.shape[0])
    s.close()


def test_factor_reuse_sees_in_place_edit():
    """the LHS' call is answered from the LHS call's
    factors only while the matrix still holds the contents factorised.  An
    edit in place between the two calls (same memory, so the transposed view
    looks identical by address) must refactorise and give ``L'ᵀ \\ rhs`` of
    the EDITED matrix, as the reference's ``LHS' \\ RHS`` does
    (QuadraticProgram.jl:335, :438); an unedited pair still takes the reuse."""
    from diffopt_amd.qp import MI355XSolver
    s = MI355XSolver()
    rng = np.random.default_rng(31)
    _, _, LHS = _kkt(41)
    L = np.array(LHS.todense() if hasattr(LHS, "todense") else LHS, dtype=np.float64, order="C")
    rhs = rng.standard_normal(L.shape[0])
    s.solve_system(L, rhs)
    before = s.resolves
    L[2, 2] += 0.5                        # edited in place: the factors are stale
    L[5, 1] -= 0.25
    got = s.solve_system(L.T, rhs)
    assert s.resolves == before           # no reuse: refactorised
    np.testing.assert_allclose(got, np.linalg.solve(L.T, rhs), rtol=1e-10, atol=1e-12)
    # the unedited pair: reused once, and still exact
    s.solve_system(L, rhs)
    got2 = s.solve_system(L.T, rhs)
    assert s.resolves == before + 1
    np.testing.assert_allclose(got2, np.linalg.solve(L.T, rhs), rtol=1e-10, atol=1e-12)
    s.close()
