"""ORACLE (test infrastructure only) — DiffOpt.jl NonLinearProgram back-end.

CPU restatement of ``/root/reference/src/NonLinearProgram/nlp_utilities.jl``
and ``NonLinearProgram.jl`` at the level the engine takes over: the
derivatives of the model at the solution are given (the reference gets them
from the MOI Nonlinear evaluator, ``_compute_optimal_hess_jac``,
nlp_utilities.jl:35-92), everything after that is restated here.

Per problem (dense float64, 0-based):

* structure: ``con_kind[c]`` — 0 ``EqualTo``, 1 ``GreaterThan``, 2
  ``LessThan`` in the NLP constraint order (``cons`` sorted by NLP index,
  NonLinearProgram.jl:485); ``has_low[n]`` / ``has_up[n]`` — primal variable
  bounds (``VariableIndex``-in-``GreaterThan`` / ``LessThan``); ``sense`` +1
  MIN, −1 MAX (``_sense_mult``, nlp_utilities.jl:448-450);
* point: ``Hxx[n, n]``, ``Hxp[n, P]`` — Hessian of the Lagrangian
  ``∇²f − sense·Σ y_i ∇²c_i`` (``eval_hessian_lagrangian`` with σ = 1,
  μ = −sense·y, nlp_utilities.jl:48-54) w.r.t. primal × primal and primal ×
  parameter; ``Jx[c, n]``, ``Jp[c, P]`` — constraint Jacobian (:65-77);
  ``x[n]`` primal values; ``cval[c]`` constraint function values and
  ``crhs[c]`` set constants (the slack of an inequality row is
  ``cval − crhs``, :202-206); ``y[c]`` constraint duals, ``yl[n]`` / ``yu[n]``
  bound duals and ``xl[n]`` / ``xu[n]`` bound values, all in MOI's convention
  (``ConstraintDualStart``).

The KKT system follows sIpopt (nlp_utilities.jl:358-387):

    M = [ W   Aᵀ  I_L  I_U ]      N = [ ∇ₓₚL ]
        [ A   0   0    0   ]          [ ∇ₚC  ]
        [ V_L 0   X_lb 0   ]          [ 0    ]
        [ V_U 0   0    X_ub]          [ 0    ]

over ``w = [x; s_geq; s_leq]`` (slack columns −1 in A), and
``∂s = −M⁻¹N`` with per-block sign adjustments (:486-499).
"""

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla


class Layout:
    """Index bookkeeping shared by the build, the sign adjustment and the
    fwd/rev extraction (``_cache_evaluator!``, NonLinearProgram.jl:438-500)."""

    def __init__(self, con_kind, has_low, has_up):
        con_kind = np.asarray(con_kind, dtype=int)
        self.n = len(has_low)
        self.c = len(con_kind)
        # _find_inequalities (nlp_utilities.jl:160-174): ascending NLP index
        self.geq = np.flatnonzero(con_kind == 1)
        self.leq = np.flatnonzero(con_kind == 2)
        self.ng, self.nl = len(self.geq), len(self.leq)
        self.low_p = np.flatnonzero(np.asarray(has_low, dtype=bool))
        self.up_p = np.flatnonzero(np.asarray(has_up, dtype=bool))
        self.num_w = self.n + self.ng + self.nl
        # has_low / has_up extended with the slack indices (:276-277)
        self.has_low = np.concatenate([self.low_p, self.n + np.arange(self.ng)]).astype(int)
        self.has_up = np.concatenate([self.up_p, self.n + self.ng + np.arange(self.nl)]).astype(int)
        self.nlo, self.nup = len(self.has_low), len(self.has_up)
        self.rows = self.num_w + self.c + self.nlo + self.nup
        # index_duals (NonLinearProgram.jl:480-484): constraint duals, primal
        # lower-bound duals, primal upper-bound duals (slack bound duals skipped)
        w, c = self.num_w, self.c
        self.index_duals = np.concatenate([
            w + np.arange(c),
            w + c + np.arange(len(self.low_p)),
            w + c + len(self.low_p) + self.ng + np.arange(len(self.up_p)),
        ]).astype(int)


def solution_and_bounds(L, sense, x, cval, crhs, y, xl, xu, yl, yu):
    """``_compute_solution_and_bounds`` (nlp_utilities.jl:181-279): the
    primal-slack vector X and the bound values / duals over it (dense,
    zeros where a bound is absent)."""
    s_geq = cval[L.geq] - crhs[L.geq]
    s_leq = cval[L.leq] - crhs[L.leq]
    X = np.concatenate([x, s_geq, s_leq])
    V_L = np.zeros(L.num_w)
    X_L = np.zeros(L.num_w)
    V_U = np.zeros(L.num_w)
    X_U = np.zeros(L.num_w)
    V_L[L.low_p] = yl[L.low_p] * sense
    X_L[L.low_p] = xl[L.low_p]
    V_L[L.n + np.arange(L.ng)] = y[L.geq] * sense
    V_U[L.up_p] = yu[L.up_p] * (-sense)
    X_U[L.up_p] = xu[L.up_p]
    V_U[L.n + L.ng + np.arange(L.nl)] = y[L.leq] * (-sense)
    return X, V_L, X_L, V_U, X_U


def build_sensitivity_matrices(L, Hxx, Hxp, Jx, Jp, X, V_L, X_L, V_U, X_U):
    """``_build_sensitivity_matrices`` (nlp_utilities.jl:286-396): dense M, N."""
    n, c, w = L.n, L.c, L.num_w
    P = Hxp.shape[1]
    A = np.zeros((c, w))
    A[:, :n] = Jx
    A[L.geq, n + np.arange(L.ng)] = -1.0
    A[L.leq, n + L.ng + np.arange(L.nl)] = -1.0
    M = np.zeros((L.rows, L.rows))
    M[:n, :n] = Hxx
    M[:w, w:w + c] = A.T
    M[w:w + c, :w] = A
    lo0, up0 = w + c, w + c + L.nlo
    for i, j in enumerate(L.has_low):
        M[lo0 + i, j] = V_L[j]
        M[lo0 + i, lo0 + i] = X[j] - X_L[j]
        M[j, lo0 + i] = -1.0
    for i, j in enumerate(L.has_up):
        M[up0 + i, j] = V_U[j]
        M[up0 + i, up0 + i] = X_U[j] - X[j]
        M[j, up0 + i] = 1.0
    N = np.zeros((L.rows, P))
    N[:n] = Hxp
    N[w:w + c] = Jp
    return M, N


def _lu(J):
    """``SparseArrays.lu(J; check = false)``: None when the factor is exactly
    singular (UMFPACK status 1; SuperLU raises)."""
    try:
        return spla.splu(sp.csc_matrix(J))
    except RuntimeError:
        return None


def inertia_correction(M, num_cons, num_w, st=1e-6, max_corrections=50):
    """``_inertia_correction`` (NonLinearProgram.jl:356-381):
    ``J_k = M + k·st·D``, D = +1 except −1 on the constraint rows, k = 1, 2, …
    Returns ``(factor or None, k)``."""
    d = np.ones(M.shape[0])
    d[num_w:num_w + num_cons] = -1.0
    J = M + st * np.diag(d)
    K = _lu(J)
    k = 1
    while K is None and k < max_corrections:
        J = J + st * np.diag(d)
        K = _lu(J)
        k += 1
    return K, k


def lu_with_inertia_correction(M, num_w, num_cons, st=1e-6, max_corrections=50):
    """``_lu_with_inertia_correction`` (NonLinearProgram.jl:394-422).
    Returns ``(factor or None, corrections)``."""
    K = _lu(M)
    if K is not None:
        return K, 0
    return inertia_correction(M, num_cons, num_w, st=st, max_corrections=max_corrections)


def compute_sensitivity(con_kind, has_low, has_up, sense, Hxx, Hxp, Jx, Jp, x, cval, crhs, y, xl, xu, yl, yu,
                        return_info=False):
    """``_compute_sensitivity`` (nlp_utilities.jl:457-500): ∂s (rows × P) with
    the MOI sign adjustments; zeros when the inertia correction fails
    (``_compute_derivatives_no_relax``, :436-439)."""
    L = Layout(con_kind, has_low, has_up)
    X, V_L, X_L, V_U, X_U = solution_and_bounds(L, sense, x, cval, crhs, y, xl, xu, yl, yu)
    M, N = build_sensitivity_matrices(L, Hxx, Hxp, Jx, Jp, X, V_L, X_L, V_U, X_U)
    K, corr = lu_with_inertia_correction(M, L.num_w, L.c)
    if K is None:
        ds = np.zeros(N.shape)
    else:
        ds = -K.solve(N) if N.shape[1] else np.zeros(N.shape)
        w, c = L.num_w, L.c
        ds[w:w + c] *= -sense
        ds[w + c:w + c + L.nlo] *= sense
        ds[w + c + L.nlo:] *= -sense
    if return_info:
        return ds, L, M, N, (corr if K is not None else -1)
    return ds


def forward(ds, L, dp):
    """``forward_differentiate!`` (NonLinearProgram.jl:502-528): primal and
    dual (constraints, primal lower bounds, primal upper bounds) tangents."""
    return ds[:L.n] @ dp, ds[L.index_duals] @ dp


def reverse(ds, L, dx, ddual):
    """``reverse_differentiate!`` (NonLinearProgram.jl:530-582): Δp = ∂sᵀΔw,
    Δw = Δx on the primal rows and the dual seeds on ``index_duals``."""
    dw = np.zeros(ds.shape[0])
    dw[:L.n] = dx
    dw[L.index_duals] = ddual
    return ds.T @ dw
