"""ORACLE (test infrastructure only) — LSQR as called by DiffOpt.jl.

Restates ``IterativeSolvers.lsqr(A, b)`` (IterativeSolvers.jl 0.9, compat
``"0.9"`` at reference ``Project.toml:21``; source not vendored) as reached from
``QuadraticProgram.jl:488`` (``norm(Q) ≈ 0`` branch) and
``ConicProgram.jl:323, 372``.  Defaults used by those call sites:
``x0 = 0``, ``damp = 0``, ``atol = btol = sqrt(eps(Float64))``,
``conlim = 1/sqrt(eps(Float64))``, ``maxiter = maximum(size(A))``.

The iteration is Paige & Saunders (1982) LSQR, Golub–Kahan bidiagonalisation
with the standard convergence tests (istop 1..7).  Zero right-hand side: the
reference divides by ``β = 0`` and returns NaN; the engine (and this oracle)
return the exact minimum-norm solution ``0`` instead — documented deviation
(DESIGN.md §"Reference quirks").
"""

import math

import numpy as np

EPS = np.finfo(np.float64).eps
SQRT_EPS = math.sqrt(EPS)


def lsqr(matvec, rmatvec, b, n, atol=SQRT_EPS, btol=SQRT_EPS,
         conlim=1.0 / SQRT_EPS, maxiter=None, return_info=False, stats=None):
    """Minimum-norm least-squares solve of ``A x = b`` from ``x0 = 0``.

    ``matvec(v)`` computes ``A v`` (length m), ``rmatvec(u)`` computes ``Aᵀ u``
    (length n).  ``maxiter`` defaults to ``max(m, n)``.  A dict passed as
    ``stats`` receives the terminal estimates ``rnorm``, ``arnorm``, ``xnorm``,
    ``anorm`` (0 when the loop does not run).
    """
    b = np.asarray(b, dtype=np.float64)
    m = b.shape[0]
    if maxiter is None:
        maxiter = max(m, n)
    x = np.zeros(n)
    if stats is not None:
        stats.update(rnorm=0.0, arnorm=0.0, xnorm=0.0, anorm=0.0)
    ctol = 1.0 / conlim if conlim > 0 else 0.0
    u = b.copy()
    beta = float(np.linalg.norm(u))
    if beta == 0.0:
        return (x, 0, 0) if return_info else x
    u /= beta
    v = rmatvec(u)
    alpha = float(np.linalg.norm(v))
    if alpha == 0.0:
        return (x, 0, 0) if return_info else x
    v /= alpha
    anorm = 0.0
    acond = 0.0
    ddnorm = 0.0
    res2 = 0.0
    xnorm = 0.0
    xxnorm = 0.0
    z = 0.0
    sn2 = 0.0
    cs2 = -1.0
    rhobar = alpha
    phibar = beta
    bnorm = beta
    w = v.copy()
    istop = 0
    it = 0
    while it < maxiter:
        it += 1
        u = matvec(v) - alpha * u
        beta = float(np.linalg.norm(u))
        if beta > 0:
            u /= beta
            anorm = math.sqrt(anorm * anorm + alpha * alpha + beta * beta)
            v = rmatvec(u) - beta * v
            alpha = float(np.linalg.norm(v))
            if alpha > 0:
                v /= alpha
        # damp = 0: the damping rotation is the identity (cs1 = 1, sn1 = 0)
        rhobar1 = rhobar
        psi = 0.0
        rho = math.hypot(rhobar1, beta)
        cs = rhobar1 / rho
        sn = beta / rho
        theta = sn * alpha
        rhobar = -cs * alpha
        phi = cs * phibar
        phibar = sn * phibar
        tau = sn * phi
        t1 = phi / rho
        t2 = -theta / rho
        dk_norm2 = float(np.dot(w, w)) / (rho * rho)
        x = x + t1 * w
        w = v + t2 * w
        ddnorm += dk_norm2
        delta = sn2 * rho
        gambar = -cs2 * rho
        rhs = phi - delta * z
        zbar = rhs / gambar
        xnorm = math.sqrt(xxnorm + zbar * zbar)
        gamma = math.hypot(gambar, theta)
        cs2 = gambar / gamma
        sn2 = theta / gamma
        z = rhs / gamma
        xxnorm += z * z
        acond = anorm * math.sqrt(ddnorm)
        res1 = phibar * phibar
        res2 += psi * psi
        rnorm = math.sqrt(res1 + res2)
        arnorm = alpha * abs(tau)
        test1 = rnorm / bnorm
        test2 = arnorm / (anorm * rnorm) if anorm * rnorm != 0 else 0.0
        test3 = 1.0 / acond if acond != 0 else 0.0
        t1r = test1 / (1.0 + anorm * xnorm / bnorm)
        rtol = btol + atol * anorm * xnorm / bnorm
        if stats is not None:
            stats.update(rnorm=rnorm, arnorm=arnorm, xnorm=xnorm, anorm=anorm)
        if it >= maxiter:
            istop = 7
        if 1.0 + test3 <= 1.0:
            istop = 6
        if 1.0 + test2 <= 1.0:
            istop = 5
        if 1.0 + t1r <= 1.0:
            istop = 4
        if test3 <= ctol:
            istop = 3
        if test2 <= atol:
            istop = 2
        if test1 <= rtol:
            istop = 1
        if istop != 0:
            break
    return (x, it, istop) if return_info else x


def lsqr_dense(Amat, b, **kw):
    """``IterativeSolvers.lsqr(A, b)`` for an explicit (dense or sparse) A."""
    n = Amat.shape[1]
    return lsqr(lambda v: Amat @ v, lambda u: Amat.T @ u, b, n, **kw)
