"""ORACLE (test infrastructure only) — projections onto the dual cones.

Restates ``DiffOpt.π`` / ``DiffOpt.Dπ`` (reference ``src/diff_opt.jl:491-519``)
which call MathOptSetDistances 0.2.9 (``Project.toml:25``, not vendored)
``projection_on_set`` / ``projection_gradient_on_set`` on ``MOI.dual_set`` of
each constraint set, over the rows of a ``ProductOfSets``
(``src/product_of_sets.jl:15-74``; ``map_rows`` ``diff_opt.jl:521-592``).

Cone codes (shared with ``include/diffopt_mi355x.h``):
  0 Zeros (dual: Reals)            π = id,        Dπ = I
  1 Nonnegatives (self-dual)       π = max(v,0),  Dπ = diag((sign v + 1)/2)
  2 Nonpositives (self-dual)       π = min(v,0),  Dπ = diag((1 − sign v)/2)
  3 SecondOrderCone (self-dual)    case split ‖x‖ ≤ t / ‖x‖ ≤ −t / else
  4 PositiveSemidefiniteConeTriangle (self-dual, MOI unscaled upper triangle,
    column-wise) π = tri(V max(Λ,0) Vᵀ) of smat(v); Dπ = S²·J·S⁻² = Jᵀ with J
    the exact Jacobian of that map in unscaled coordinates and
    S = diag(1 on diagonal entries, √2 off-diagonal) (S·J·S⁻¹ is symmetric, so
    S²JS⁻² is J's transpose).  Of the candidate conventions {J, SJS⁻¹, S²J,
    S²JS⁻²} × {plain, scaled π} only plain π with S²JS⁻² reproduces every PSD
    fixture of the reference (test/conic_program.jl:184-208, 521-525, 618-641,
    841-842) — checked in tests/test_oracle_golden.py.  (SURVEY.md §0 listed
    S²J as also fitting; the PSD+POS fixture, whose LSQR stops at maxiter,
    rules it out: max |Δdx| 4.45 vs 0.019 at atol 0.3.)
  Nonnegatives at exactly v = 0 gives 0.5 (MOSD's formula as recalled; the
  value is parity-unpinned, generators keep a guard band away from 0).
"""

import math

import numpy as np

ZEROS, NONNEG, NONPOS, SOC, PSD = 0, 1, 2, 3, 4
NAMES = {ZEROS: "Zeros", NONNEG: "Nonnegatives", NONPOS: "Nonpositives",
         SOC: "SecondOrderCone", PSD: "PositiveSemidefiniteConeTriangle"}


def psd_side(dim):
    d = int((math.isqrt(8 * dim + 1) - 1) // 2)
    if d * (d + 1) // 2 != dim:
        raise ValueError(f"{dim} is not a triangular number")
    return d


def tri_indices(d):
    """MOI upper-triangle column-wise order: (0,0),(0,1),(1,1),(0,2),…"""
    out = []
    for j in range(d):
        for i in range(j + 1):
            out.append((i, j))
    return out


_TRI_IJ = {}


def _tri_ij(d):
    """Row / column index arrays of tri_indices(d) (cached)."""
    if d not in _TRI_IJ:
        ij = np.array(tri_indices(d), dtype=np.int64).reshape(-1, 2)
        _TRI_IJ[d] = (ij[:, 0], ij[:, 1])
    return _TRI_IJ[d]


def smat(v, d):
    i, j = _tri_ij(d)
    X = np.zeros((d, d))
    X[i, j] = v
    X[j, i] = v
    return X


def tri(X):
    i, j = _tri_ij(X.shape[0])
    return X[i, j].copy()


def psd_scale(d):
    return np.array([1.0 if i == j else math.sqrt(2.0) for (i, j) in tri_indices(d)])


def proj(code, v):
    v = np.asarray(v, dtype=np.float64)
    if code == ZEROS:
        return v.copy()
    if code == NONNEG:
        return np.maximum(v, 0.0)
    if code == NONPOS:
        return np.minimum(v, 0.0)
    if code == SOC:
        t = v[0]
        x = v[1:]
        nx = float(np.linalg.norm(x))
        if nx <= t:
            return v.copy()
        if nx <= -t:
            return np.zeros_like(v)
        out = np.empty_like(v)
        out[0] = 1.0
        out[1:] = x / nx
        return out * ((nx + t) / 2.0)
    if code == PSD:
        d = psd_side(v.shape[0])
        lam, U = np.linalg.eigh(smat(v, d))
        return tri((U * np.maximum(lam, 0.0)) @ U.T)
    raise ValueError(f"unknown cone code {code}")


def psd_jacobian_unscaled(v):
    """Exact Jacobian of v ↦ tri(Π_PSD(smat(v))) (Daleckii–Krein)."""
    d = psd_side(v.shape[0])
    lam, U = np.linalg.eigh(smat(v, d))
    k = v.shape[0]
    if np.all(lam >= 0):
        return np.eye(k)
    lp = np.maximum(lam, 0.0)
    B = np.empty((d, d))
    for i in range(d):
        for j in range(d):
            if lam[i] == lam[j]:
                B[i, j] = 1.0 if lam[i] > 0 else 0.0
            else:
                B[i, j] = (lp[i] - lp[j]) / (lam[i] - lam[j])
    J = np.empty((k, k))
    for c, (i, j) in enumerate(tri_indices(d)):
        E = np.zeros((d, d))
        E[i, j] = 1.0
        E[j, i] = 1.0
        dP = U @ (B * (U.T @ E @ U)) @ U.T
        J[:, c] = tri(dP)
    return J


class PSDStructured:
    """Dπ of a PSD-triangle cone without its dense k × k Jacobian (k = d(d+1)/2,
    e.g. 45 150 at d = 300 — 16 GB dense): J·w = tri(U (B ∘ (Uᵀ smat(w) U)) Uᵀ)
    with the eigendecomposition smat(v) = U Λ Uᵀ and the Daleckii–Krein
    weights B of psd_jacobian_unscaled (the same J, column by column:
    J e_c = tri(dP(E_c)), and smat(w) = Σ_c w_c E_c).  `convention` S2JSm2:
    Dπ·w = S² J (S⁻² w) and Dπᵀ·w = J w (S J S⁻¹ is symmetric).  Used by
    dpi_blocks for sides above STRUCTURED_MIN; equal to the dense blocks to
    rounding (tests/test_oracle_golden.py)."""

    def __init__(self, v, psd_convention="S2JSm2"):
        if psd_convention != "S2JSm2":
            raise ValueError("structured PSD Dπ implements the S2JSm2 convention")
        v = np.asarray(v, dtype=np.float64)
        self.k = v.shape[0]
        self.shape = (self.k, self.k)
        self.d = d = psd_side(self.k)
        lam, self.U = np.linalg.eigh(smat(v, d))
        self.ident = bool(np.all(lam >= 0))
        lp = np.maximum(lam, 0.0)
        dl = lam[:, None] - lam[None, :]
        same = dl == 0.0
        with np.errstate(divide="ignore", invalid="ignore"):
            B = (lp[:, None] - lp[None, :]) / np.where(same, 1.0, dl)
        self.B = np.where(same, (lam[:, None] > 0).astype(float) * np.ones_like(B), B)
        s = psd_scale(d)
        self.s2 = s * s

    def jvec(self, w):
        w = np.asarray(w, dtype=np.float64)
        if self.ident:
            return w.copy()
        U = self.U
        return tri(U @ (self.B * (U.T @ smat(w, self.d) @ U)) @ U.T)

    def __matmul__(self, w):
        return self.s2 * self.jvec(np.asarray(w, dtype=np.float64) / self.s2)

    @property
    def T(self):
        outer = self

        class _T:
            shape = outer.shape

            def __matmul__(self, w):
                return outer.jvec(w)
        return _T()


STRUCTURED_MIN = 128   # PSD sides from here on: PSDStructured instead of a dense block (k > 8256)


def dproj(code, v, psd_convention="S2JSm2"):
    v = np.asarray(v, dtype=np.float64)
    k = v.shape[0]
    if code == ZEROS:
        return np.eye(k)
    if code == NONNEG:
        return np.diag((np.sign(v) + 1.0) / 2.0)
    if code == NONPOS:
        return np.diag((1.0 - np.sign(v)) / 2.0)
    if code == SOC:
        t = v[0]
        x = v[1:]
        nx = float(np.linalg.norm(x))
        if nx <= t:
            return np.eye(k)
        if nx <= -t:
            return np.zeros((k, k))
        R = np.empty((k, k))
        R[0, 0] = nx
        R[0, 1:] = x
        R[1:, 0] = x
        R[1:, 1:] = (nx + t) * np.eye(k - 1) - (t / (nx * nx)) * np.outer(x, x)
        return R / (2.0 * nx)
    if code == PSD:
        J = psd_jacobian_unscaled(v)
        d = psd_side(k)
        S = psd_scale(d)
        if psd_convention == "S2J":
            return (S * S)[:, None] * J
        if psd_convention == "S2JSm2":
            return (S * S)[:, None] * J / (S * S)[None, :]
        if psd_convention == "J":
            return J
        if psd_convention == "SJSinv":
            return S[:, None] * J / S[None, :]
        raise ValueError(psd_convention)
    raise ValueError(f"unknown cone code {code}")


def cone_offsets(cones):
    off = [0]
    for _, dim in cones:
        off.append(off[-1] + dim)
    return off


def pi(v, cones):
    """``DiffOpt.π`` (diff_opt.jl:491-499): flattened projection."""
    off = cone_offsets(cones)
    out = np.empty_like(np.asarray(v, dtype=np.float64))
    for k, (code, dim) in enumerate(cones):
        out[off[k]:off[k + 1]] = proj(code, v[off[k]:off[k + 1]])
    return out


def dpi_blocks(v, cones, psd_convention="S2JSm2", structured_min=STRUCTURED_MIN):
    """``DiffOpt.Dπ`` (diff_opt.jl:509-519): list of diagonal blocks — dense,
    except PSD cones of side ≥ structured_min (PSDStructured: same operator,
    applied through the eigendecomposition)."""
    off = cone_offsets(cones)
    out = []
    for k, (code, dim) in enumerate(cones):
        vk = v[off[k]:off[k + 1]]
        if code == PSD and psd_side(dim) >= structured_min and psd_convention == "S2JSm2":
            out.append(PSDStructured(vk, psd_convention))
        else:
            out.append(dproj(code, vk, psd_convention))
    return out


def blockdiag(blocks):
    m = sum(b.shape[0] for b in blocks)
    D = np.zeros((m, m))
    o = 0
    for b in blocks:
        k = b.shape[0]
        D[o:o + k, o:o + k] = b if isinstance(b, np.ndarray) else np.stack([b @ e for e in np.eye(k)], axis=1)
        o += k
    return D
