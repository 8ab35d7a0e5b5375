"""ORACLE (test infrastructure only) — DiffOpt.jl ConicProgram back-end.

CPU restatement of ``/root/reference/src/ConicProgram/ConicProgram.jl``.
Geometric conic form as stored by the reference (``MatrixOfConstraints`` with a
``ProductOfSets`` row layout): ``A_moi x + b_moi ∈ K``, objective ``c`` (MIN
sense; MAX negates ``c`` only, ConicProgram.jl:206-208).  Primal start ``x``,
constraint primal ``s`` and constraint dual ``y`` (ConicProgram.jl:144-170).
"""

import numpy as np

from . import cones as C
from .lsqr import lsqr


class Cache:
    """``_gradient_cache`` (ConicProgram.jl:172-255)."""

    def __init__(self, A_moi, b_moi, c, x, s, y, cones, max_sense=False,
                 psd_convention="S2JSm2"):
        A_moi = np.asarray(A_moi, dtype=np.float64)
        self.A = -A_moi                       # :179-183 (diffcp sign)
        self.b = np.asarray(b_moi, dtype=np.float64)
        m, n = self.A.shape
        y = np.asarray(y, dtype=np.float64)
        s = np.asarray(s, dtype=np.float64)
        if np.any(np.isnan(y)) or y.shape[0] < m:   # :186-190
            raise ValueError("Some constraints are missing a value for the "
                             "`ConstraintDualStart` attribute.")
        if np.any(np.isnan(s)) or s.shape[0] < m:   # :192-196
            raise ValueError("Some constraints are missing a value for the "
                             "`ConstraintPrimalStart` attribute.")
        c = np.asarray(c, dtype=np.float64)
        self.c = -c if max_sense else c.copy()
        self.x = np.asarray(x, dtype=np.float64)
        self.s = s
        self.y = y
        self.cones = list(cones)
        self.v = y - s                             # :222
        self.blocks = C.dpi_blocks(self.v, self.cones, psd_convention)  # :225
        self._off = C.cone_offsets(self.cones)
        self.vp = C.pi(self.v, self.cones)         # :249
        self.m, self.n = m, n

    @property
    def D(self):
        """Dense ``Dπ`` (the reference's ``BlockDiagonal``, :225)."""
        return C.blockdiag(self.blocks)

    def _dpi(self, v, trans=False):
        """``Dπ·v`` / ``Dπᵀ·v`` block by block, as ``BlockDiagonal`` multiplies."""
        out = np.empty_like(v)
        for k, blk in enumerate(self.blocks):
            a, b = self._off[k], self._off[k + 1]
            out[a:b] = (blk.T if trans else blk) @ v[a:b]
        return out

    def M(self):
        """Dense ``M = [0, AᵀDπ, c; −A, I−Dπ, b; −cᵀ, −bᵀDπ, 0]`` (:243-247)."""
        m, n = self.m, self.n
        N = n + m + 1
        M = np.zeros((N, N))
        D = self.D
        M[:n, n:n + m] = self.A.T @ D
        M[:n, -1] = self.c
        M[n:n + m, :n] = -self.A
        M[n:n + m, n:n + m] = np.eye(m) - D
        M[n:n + m, -1] = self.b
        M[-1, :n] = -self.c
        M[-1, n:n + m] = -(self.b @ D)
        return M

    # matrix-free products, identical to multiplying by M() ---------------
    def matvec(self, z):
        n, m = self.n, self.m
        u, v, w = z[:n], z[n:n + m], z[-1]
        Dv = self._dpi(v)
        return np.concatenate([self.A.T @ Dv + self.c * w,
                               -self.A @ u + v - Dv + self.b * w,
                               [-(self.c @ u) - (self.b @ Dv)]])

    def rmatvec(self, r):
        n, m = self.n, self.m
        p, q, t = r[:n], r[n:n + m], r[-1]
        Ap = self.A @ p
        return np.concatenate([-(self.A.T @ q) - self.c * t,
                               self._dpi(Ap - q - self.b * t, trans=True) + q,
                               [self.c @ p + self.b @ q]])


def forward_rhs(cache, dA=None, db=None, dc=None):
    """RHS of ConicProgram.jl:314-318 (``dA``/``db``/``dc`` are the user
    tangents of the MOI coefficients/constants/objective — NOT negated,
    :270-305)."""
    n, m = cache.n, cache.m
    dA = np.zeros((m, n)) if dA is None else np.asarray(dA, float)
    db = np.zeros(m) if db is None else np.asarray(db, float)
    dc = np.zeros(n) if dc is None else np.asarray(dc, float)
    u, vp = cache.x, cache.vp
    return np.concatenate([dA.T @ vp + dc, -(dA @ u) + db,
                           [-(dc @ u) - (db @ vp)]])


def forward_differentiate(cache, dA=None, db=None, dc=None, return_info=False, stats=None, maxiter=None):
    """``forward_differentiate!`` (ConicProgram.jl:257-334).

    Returns ``(dx, du, dv, dw)`` where ``dx = −(du − x·dw)`` is
    ``ForwardVariablePrimal`` (:403-412).  ``maxiter`` caps LSQR (default:
    IterativeSolvers' max(size(M)); the engine's dopt_conic_set_maxiter).
    """
    RHS = forward_rhs(cache, dA, db, dc)
    N = RHS.shape[0]
    info = (0, 0)
    if np.linalg.norm(RHS) <= 0.0:      # `<= 1e-400` underflows to 0.0 (:320)
        dz = np.zeros(N)
    else:
        dz, it, istop = lsqr(cache.matvec, cache.rmatvec, RHS, N,
                             return_info=True, stats=stats, maxiter=maxiter)
        info = (it, istop)
    n, m = cache.n, cache.m
    du, dv, dw = dz[:n], dz[n:n + m], dz[-1]
    dx = -(du - cache.x * dw)
    out = (dx, du, dv, dw)
    return (out, info) if return_info else out


def reverse_differentiate(cache, dx, return_info=False, stats=None, maxiter=None):
    """``reverse_differentiate!`` (ConicProgram.jl:336-394) with dy = ds = 0.

    Returns ``(g, πz)``; ``lsqr`` is applied to ``M`` (not ``Mᵀ``, :372).
    ``maxiter`` caps LSQR as in ``forward_differentiate``.
    """
    n, m = cache.n, cache.m
    dx = np.asarray(dx, dtype=np.float64)
    dz = np.concatenate([dx, np.zeros(m), [-(cache.x @ dx)]])
    info = (0, 0)
    if np.linalg.norm(dz) <= 1e-4:      # :369-370
        g = np.zeros(n + m + 1)
    else:
        g, it, istop = lsqr(cache.matvec, cache.rmatvec, dz, n + m + 1,
                            return_info=True, stats=stats, maxiter=maxiter)
        info = (it, istop)
    piz = np.concatenate([cache.x, cache.vp, [1.0]])
    return ((g, piz), info) if return_info else (g, piz)


def reverse_outputs(cache, g):
    """Getters (ConicProgram.jl:396-443): ``dc = g_x − g_end·x``;
    ``db_i = g_{n+i} − g_end·vp_i``; ``dA_i = g_{n+i}·xᵀ − vp_i·g_xᵀ``."""
    n, m = cache.n, cache.m
    gx, gv, ge = g[:n], g[n:n + m], g[-1]
    dc = gx - ge * cache.x
    db = gv - ge * cache.vp
    dA = np.outer(gv, cache.x) - np.outer(cache.vp, gx)
    return dA, db, dc
