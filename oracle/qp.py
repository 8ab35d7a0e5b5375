"""ORACLE (test infrastructure only) — DiffOpt.jl QuadraticProgram back-end.

CPU restatement of ``/root/reference/src/QuadraticProgram/QuadraticProgram.jl``.
Matrix-form problem (OptNet notation, Amos & Kolter 2017):

    min ½ zᵀQz + qᵀz   s.t.  G z ≤ h  (λ ≥ 0),   A z = b  (ν)

with the reference's dual sign convention already applied
(``λ = −dual(LessThan)``, ``ν = −dual(EqualTo)``, QuadraticProgram.jl:164-180).
Every array is dense float64; ``Q`` is the symmetric Hessian as produced by
``sparse_array_representation`` (utils.jl:46-69).
"""

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

from .lsqr import lsqr_dense


def gz_minus_h(G, z, h):
    """``G * z - h`` in Julia's ``SparseMatrixCSC`` mul! order: column by
    column, product and sum rounded separately (no FMA).  Bit-exact with the
    engine, so the exact-zero tests on ``s`` agree."""
    acc = np.zeros(G.shape[0])
    for j in range(G.shape[1]):
        acc = acc + G[:, j] * z[j]
    return acc - h


def create_LHS_matrix(z, lam, Q, G, h, A, sparse=False):
    """``create_LHS_matrix`` (QuadraticProgram.jl:256-282).

    ``LHS = [Q, GᵀD(λ), Aᵀ; G, D(Gz−h), 0; A, 0, 0]`` with block order
    ``[z; λ; ν]`` and the special cases for missing G and/or A.
    """
    n = Q.shape[0]
    m = 0 if G is None else G.shape[0]
    p = 0 if A is None else A.shape[0]
    if m == 0 and p == 0:
        L = np.array(Q, dtype=np.float64)
        return sp.csc_matrix(L) if sparse else L
    if G is not None and A is not None and m and p and G.shape[1] != A.shape[1]:
        raise ValueError("Sizes of A and G do not match")  # :273-275
    N = n + m + p
    L = np.zeros((N, N))
    L[:n, :n] = Q
    if m:
        s = gz_minus_h(G, z, h)
        L[:n, n:n + m] = G.T * lam[None, :]
        L[n:n + m, :n] = G
        L[n:n + m, n:n + m] = np.diag(s)
    if p:
        L[:n, n + m:] = A.T
        L[n + m:, :n] = A
    return sp.csc_matrix(L) if sparse else L


def is_iterative(Q):
    """``iterative = norm(Q) ≈ 0`` (QuadraticProgram.jl:333, 436).

    Julia's ``isapprox(x, 0)`` with default tolerances is ``x == 0`` exactly,
    and Julia's ``norm`` is scaling-safe (no underflow to 0 for tiny entries;
    NaN propagates), so the test is "every entry == 0".
    """
    return bool(np.all(np.asarray(Q) == 0.0))


def solve_system(LHS, RHS, iterative, sparse=False):
    """Default ``solve_system`` (QuadraticProgram.jl:486-492)."""
    if iterative:
        return lsqr_dense(LHS, RHS)
    if sparse:
        return spla.splu(sp.csc_matrix(LHS)).solve(RHS)
    return np.linalg.solve(LHS, RHS)


def reverse_differentiate(Q, G, h, A, z, lam, nu, dl_dz, sparse=False):
    """``reverse_differentiate!`` (QuadraticProgram.jl:316-351).

    Returns ``(dz, dλ, dν) = split(−LHS \\ [dl/dz; 0; 0])``.
    """
    n = Q.shape[0]
    m = 0 if G is None else G.shape[0]
    p = 0 if A is None else A.shape[0]
    LHS = create_LHS_matrix(z, lam, Q, G, h, A, sparse=sparse)
    RHS = np.concatenate([np.asarray(dl_dz, float), np.zeros(m + p)])
    it = is_iterative(Q)
    if it and not np.any(RHS):
        x = np.zeros_like(RHS)  # documented deviation: reference lsqr → NaN
    else:
        x = solve_system(LHS.toarray() if (sparse and it) else LHS, RHS, it,
                         sparse=sparse and not it)
    g = -x
    return g[:n], g[n:n + m], g[n + m:]


def forward_rhs(Q, G, h, A, z, lam, nu, dQ=None, dq=None, dG=None, dh=None,
                dA=None, db=None):
    """Forward right-hand side (QuadraticProgram.jl:429-433).

    ``[dQ z + dq + dGᵀλ + dAᵀν; λ∘(dG z) − λ∘dh; dA z − db]``; ``None`` means
    a zero tangent.
    """
    n = Q.shape[0]
    m = 0 if G is None else G.shape[0]
    p = 0 if A is None else A.shape[0]
    r1 = np.zeros(n)
    if dQ is not None:
        r1 += dQ @ z
    if dq is not None:
        r1 += dq
    r2 = np.zeros(m)
    r3 = np.zeros(p)
    if m:
        if dG is not None:
            r1 += dG.T @ lam
            r2 += lam * (dG @ z)
        if dh is not None:
            r2 -= lam * dh
    if p:
        if dA is not None:
            r1 += dA.T @ nu
            r3 += dA @ z
        if db is not None:
            r3 -= db
    return np.concatenate([r1, r2, r3])


def forward_differentiate(Q, G, h, A, z, lam, nu, dQ=None, dq=None, dG=None,
                          dh=None, dA=None, db=None, sparse=False):
    """``forward_differentiate!`` (QuadraticProgram.jl:357-446).

    Returns ``(dz, dλ, dν) = split(−LHSᵀ \\ RHS)``.
    """
    n = Q.shape[0]
    m = 0 if G is None else G.shape[0]
    LHS = create_LHS_matrix(z, lam, Q, G, h, A, sparse=sparse)
    RHS = forward_rhs(Q, G, h, A, z, lam, nu, dQ, dq, dG, dh, dA, db)
    it = is_iterative(Q)
    LT = LHS.T
    if it and not np.any(RHS):
        x = np.zeros_like(RHS)
    else:
        x = solve_system(LT.toarray() if (sparse and it) else LT, RHS, it,
                         sparse=sparse and not it)
    g = -x
    return g[:n], g[n:n + m], g[n + m:]


# ---- output getters (lazy in the reference, materialised here) ----------

def reverse_objective(z, dz):
    """``ReverseObjectiveFunction`` (QuadraticProgram.jl:448-458):
    ``dq = dz``, ``dQ = (dz zᵀ + z dzᵀ)/2``."""
    return dz.copy(), 0.5 * (np.outer(dz, z) + np.outer(z, dz))


def reverse_constraint_le(z, lam, dz, dlam):
    """``ReverseConstraintFunction`` for LessThan rows, all rows at once
    (``_get_dA`` :467-473, ``_get_db`` :307-311): row i coefficients
    ``λ_i dλ_i z + λ_i dz`` and constant ``λ_i dλ_i``.  The user-facing
    tangent of ``h`` is ``dh = −constant`` (test/utils.jl:210)."""
    dG = (lam * dlam)[:, None] * z[None, :] + lam[:, None] * dz[None, :]
    const = lam * dlam
    return dG, const


def reverse_constraint_eq(z, nu, dz, dnu):
    """``ReverseConstraintFunction`` for EqualTo rows (``_get_dA`` :461-466,
    ``_get_db`` :312-314): coefficients ``dν_i z + ν_i dz``, constant
    ``dν_i`` (user-facing ``db = −dν``)."""
    dA = dnu[:, None] * z[None, :] + nu[:, None] * dz[None, :]
    return dA, dnu.copy()


def create_LHS_sparse(z, lam, G, h, A, n):
    """``create_LHS_matrix`` (QuadraticProgram.jl:256-282) with Q = 0 as the
    reference builds it — a ``SparseMatrixCSC`` (scipy CSC here), never dense:
    ``[0, GᵀD(λ), Aᵀ; G, D(Gz − h), 0; A, 0, 0]``.  G, A: scipy sparse."""
    m = 0 if G is None else G.shape[0]
    p = 0 if A is None else A.shape[0]
    top = [sp.csc_matrix((n, n))]
    if m:
        s = G @ z - h
        top.append(G.T @ sp.diags(lam))
    if p:
        top.append(A.T)
    rows = [top]
    if m:
        rows.append([G, sp.diags(s)] + ([None] if p else []))
    if p:
        rows.append([A] + ([None] if m else []) + [None])
    return sp.bmat(rows, format="csc")


def lp_sparse_differentiate(G, h, A, z, lam, nu, dl_dz, dq=None, dh=None, db=None):
    """Reverse and forward of the LSQR branch (Q = 0) on the sparse LHS:
    ``−lsqr(LHS, [dl/dz; 0; 0])`` (:336-337) and ``−lsqr(LHS', RHS)`` with the
    forward RHS of :429-433 for vector tangents (dQ = dG = dA = 0).  Returns
    (reverse [dz|dλ|dν], forward [dz|dλ|dν], (it_rev, istop_rev), (it_fwd, istop_fwd))."""
    from .lsqr import lsqr
    n = z.shape[0]
    m = 0 if G is None else G.shape[0]
    p = 0 if A is None else A.shape[0]
    L = create_LHS_sparse(z, lam, G, h, A, n)
    N = n + m + p
    r_rev = np.concatenate([dl_dz, np.zeros(m + p)])
    r1 = np.zeros(n) if dq is None else np.array(dq, float)
    r2 = np.zeros(m) if dh is None or not m else -lam * dh
    r3 = np.zeros(p) if db is None or not p else -np.asarray(db, float)
    r_fwd = np.concatenate([r1, r2, r3])
    xr, itr, isr = lsqr(lambda v: L @ v, lambda u: L.T @ u, r_rev, N, return_info=True)
    xf, itf, isf = lsqr(lambda v: L.T @ v, lambda u: L @ u, r_fwd, N, return_info=True)
    return -xr, -xf, (itr, isr), (itf, isf)
