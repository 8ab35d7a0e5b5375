"""Seeded synthetic instances with a KKT point by construction.

QP (OptNet sign):  Q = LLᵀ/n + 0.1 I,  G, A ~ N(0,1)/√n,  z ~ N(0,1);
a seeded permutation makes ⌊φ·m⌋ rows active (s_i = 0, λ_i ~ U(0.5,1.5)), the
others inactive (λ_i = 0, s_i ~ −U(0.5,1.5)); ν ~ N(0,1); h = Gz − s; b = Az;
q = −(Qz + Gᵀλ + Aᵀν).  Reverse seed dl/dz ~ N(0,1); forward tangents
dq, dh, db ~ N(0,1) (dQ = dG = dA = 0 unless `dense_tangents`).
`lam_eps` > 0 gives the inactive rows λ_i = lam_eps instead of 0 (interior-
point-like duals: no row is eliminated exactly, N' = n + m + p).
Seeds: 20250307 + config index.  No solver is needed: (z, λ, ν) is the exact
primal–dual optimum of the generated problem.
"""

import math

import numpy as np

SEED0 = 20250307

# BASELINE.json configs (index → shape); p = 0 assumed where unspecified
QP_CONFIGS = {
    1: dict(n=50, m=80, p=30, phi=0.2, batch=1),
    2: dict(n=200, m=300, p=0, phi=0.3, batch=1024),
    3: dict(n=1000, m=1500, p=0, phi=0.3, batch=8192),
}
CONIC_CONFIGS = {
    4: dict(n=500, cones=[(3, 25)] * 20, batch=512),
    5: dict(n=500, cones=[(4, 1275)] * 10, batch=64),
}


def qp_numpy(batch, n, m, p, phi, seed, dense_tangents=False, lam_eps=0.0):
    rng = np.random.default_rng(seed)
    out = {k: [] for k in ["Q", "q", "G", "h", "A", "b", "z", "lam", "nu", "dl_dz",
                           "dq", "dh", "db", "dQ", "dG", "dA"]}
    k_act = int(math.floor(phi * m))
    for _ in range(batch):
        L = rng.standard_normal((n, n))
        Q = L @ L.T / n + 0.1 * np.eye(n)
        Q = 0.5 * (Q + Q.T)   # exactly symmetric (the reference's Q always is)
        G = rng.standard_normal((m, n)) / math.sqrt(n)
        A = rng.standard_normal((p, n)) / math.sqrt(n)
        z = rng.standard_normal(n)
        perm = rng.permutation(m)
        lam = np.full(m, float(lam_eps))
        s = np.zeros(m)
        act, ina = perm[:k_act], perm[k_act:]
        lam[act] = rng.uniform(0.5, 1.5, size=k_act)
        s[ina] = -rng.uniform(0.5, 1.5, size=m - k_act)
        nu = rng.standard_normal(p)
        h = G @ z - s
        b = A @ z
        q = -(Q @ z + G.T @ lam + A.T @ nu)
        out["Q"].append(Q); out["q"].append(q); out["G"].append(G); out["h"].append(h)
        out["A"].append(A); out["b"].append(b); out["z"].append(z); out["lam"].append(lam)
        out["nu"].append(nu)
        out["dl_dz"].append(rng.standard_normal(n))
        out["dq"].append(rng.standard_normal(n))
        out["dh"].append(rng.standard_normal(m))
        out["db"].append(rng.standard_normal(p))
        if dense_tangents:
            S = rng.standard_normal((n, n))
            out["dQ"].append((S + S.T) / 2)
            out["dG"].append(rng.standard_normal((m, n)))
            out["dA"].append(rng.standard_normal((p, n)))
    res = {k: np.stack(v) for k, v in out.items() if v}
    return res


def qp_config_numpy(cfg, batch=None, **kw):
    c = QP_CONFIGS[cfg]
    return qp_numpy(batch or c["batch"], c["n"], c["m"], c["p"], c["phi"], SEED0 + cfg, **kw)


def qp_torch(batch, n, m, p, phi, seed, device="cuda", rank_offset=0, lam_eps=0.0):
    """Same construction on the GPU with torch (for bench-sized batches).
    `rank_offset` shifts the seed so every rank gets distinct problems."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed * 1000003 + rank_offset)
    f64 = dict(dtype=torch.float64, device=device)
    L = torch.randn(batch, n, n, generator=g, **f64)
    Q = L @ L.transpose(1, 2) / n + 0.1 * torch.eye(n, **f64)
    del L
    # exactly symmetric, as the reference's Q always is (its quadratic terms
    # are mirrored): a batched GEMM sums Q_ij and Q_ji in different orders
    Q = 0.5 * (Q + Q.transpose(1, 2))
    G = torch.randn(batch, m, n, generator=g, **f64) / math.sqrt(n)
    A = torch.randn(batch, p, n, generator=g, **f64) / math.sqrt(n)
    z = torch.randn(batch, n, generator=g, **f64)
    k_act = int(math.floor(phi * m))
    keys = torch.rand(batch, m, generator=g, device=device)
    perm = torch.argsort(keys, dim=1)
    act = torch.zeros(batch, m, dtype=torch.bool, device=device)
    act.scatter_(1, perm[:, :k_act], True)
    lam = torch.where(act, 0.5 + torch.rand(batch, m, generator=g, **f64),
                      torch.full((), float(lam_eps), **f64))
    s = torch.where(act, torch.zeros((), **f64), -(0.5 + torch.rand(batch, m, generator=g, **f64)))
    nu = torch.randn(batch, p, generator=g, **f64)
    h = torch.einsum("bmn,bn->bm", G, z) - s
    b = torch.einsum("bpn,bn->bp", A, z)
    q = -(torch.einsum("bij,bj->bi", Q, z) + torch.einsum("bmn,bm->bn", G, lam)
          + torch.einsum("bpn,bp->bn", A, nu))
    return dict(Q=Q, q=q, G=G, h=h, A=A, b=b, z=z, lam=lam, nu=nu,
                dl_dz=torch.randn(batch, n, generator=g, **f64),
                dq=torch.randn(batch, n, generator=g, **f64),
                dh=torch.randn(batch, m, generator=g, **f64),
                db=torch.randn(batch, p, generator=g, **f64))


# ---------------------------------------------------------------------------
# conic: optimal (x, s, y) by construction, complementary boundary pairs
# ---------------------------------------------------------------------------
def _tri(X):
    d = X.shape[0]
    return np.array([X[i, j] for j in range(d) for i in range(j + 1)])


def conic_numpy(batch, n, cones, seed, guard=1e-3):
    """Geometric form A_moi x + b_moi ∈ K with primal slack s ∈ K, dual y ∈ K*,
    ⟨s, y⟩ = 0 per cone (MOI set_dot), dual feasibility c = A_moiᵀ W y with
    W the set_dot weights (2 on PSD off-diagonal triangle entries)."""
    rng = np.random.default_rng(seed)
    m = sum(d for _, d in cones)
    out = {k: [] for k in ["A", "b", "c", "x", "s", "y", "dx", "dA", "db", "dc"]}
    for _ in range(batch):
        s = np.zeros(m)
        y = np.zeros(m)
        wts = np.ones(m)
        o = 0
        for code, dim in cones:
            if code == 0:       # Zeros: s = 0, y free
                y[o:o + dim] = rng.standard_normal(dim)
            elif code in (1, 2):  # Nonneg / Nonpos: complementary, guard band
                sg = 1.0 if code == 1 else -1.0
                act = rng.random(dim) < 0.5
                mag_s = rng.uniform(0.5, 1.5, dim)
                mag_y = rng.uniform(0.5, 1.5, dim)
                s[o:o + dim] = np.where(act, 0.0, sg * mag_s)
                y[o:o + dim] = np.where(act, sg * mag_y, 0.0)
            elif code == 3:     # SOC: s = α(‖u‖, u), y = β(‖u‖, −u)
                u = rng.standard_normal(dim - 1)
                nu_ = np.linalg.norm(u)
                al, be = rng.uniform(0.5, 1.5), rng.uniform(0.5, 1.5)
                s[o] = al * nu_
                s[o + 1:o + dim] = al * u
                y[o] = be * nu_
                y[o + 1:o + dim] = -be * u
            elif code == 4:     # PSD: S = V diag(σ) Vᵀ, Y = V diag(ω) Vᵀ, σ∘ω = 0
                d = int((math.isqrt(8 * dim + 1) - 1) // 2)
                V, _ = np.linalg.qr(rng.standard_normal((d, d)))
                r = d // 2
                sig = np.concatenate([rng.uniform(0.5, 1.5, r), np.zeros(d - r)])
                om = np.concatenate([np.zeros(r), rng.uniform(0.5, 1.5, d - r)])
                s[o:o + dim] = _tri((V * sig) @ V.T)
                y[o:o + dim] = _tri((V * om) @ V.T)
                wts[o:o + dim] = np.array([1.0 if i == j else 2.0
                                           for j in range(d) for i in range(j + 1)])
            o += dim
        A = rng.standard_normal((m, n)) / math.sqrt(n)
        x = rng.standard_normal(n)
        b = s - A @ x                      # A x + b = s ∈ K
        c = A.T @ (wts * y)                # c − A_moiᵀ W y = 0 (MOI dual feasibility)
        out["A"].append(A); out["b"].append(b); out["c"].append(c); out["x"].append(x)
        out["s"].append(s); out["y"].append(y)
        out["dx"].append(rng.standard_normal(n))
        out["dA"].append(rng.standard_normal((m, n)))
        out["db"].append(rng.standard_normal(m))
        out["dc"].append(rng.standard_normal(n))
    return {k: np.stack(v) for k, v in out.items()}


def nlp_numpy(batch, n, c, P, seed, frac_geq=0.4, frac_leq=0.3, frac_low=0.5, frac_up=0.3, active=0.3,
              sense=1):
    """NLP KKT data at a strictly complementary point (nlp_utilities.jl
    conventions, MOI duals): shared structure (row kinds: EqualTo, then
    GreaterThan, then LessThan, shuffled; variable bounds), per problem a
    symmetric Hxx = LLᵀ/n + 0.1I (times `sense`), dense Hxp, Jx ~ N(0,1)/√n,
    Jp ~ N(0,1); a fraction `active` of the inequality rows / bounds is
    active (slack 0, dual ±U(0.5,1.5) by the set's sign), the rest inactive
    (slack ±U(0.5,1.5), dual 0).  Returns (structure dict, point dict, dp,
    dx seed, ddual seed)."""
    rng = np.random.default_rng(seed)
    ng, nl = int(frac_geq * c), int(frac_leq * c)
    kinds = np.array([1] * ng + [2] * nl + [0] * (c - ng - nl), dtype=np.int32)
    rng.shuffle(kinds)
    has_low = (rng.random(n) < frac_low).astype(np.int8)
    has_up = (rng.random(n) < frac_up).astype(np.int8)
    st = dict(con_kind=kinds, has_low=has_low, has_up=has_up, sense=sense)
    keys = ["Hxx", "Hxp", "Jx", "Jp", "x", "cval", "crhs", "y", "xl", "xu", "yl", "yu"]
    pt = {k: [] for k in keys}
    u = lambda size=None: rng.uniform(0.5, 1.5, size)
    for _ in range(batch):
        L = rng.standard_normal((n, n))
        pt["Hxx"].append(sense * (L @ L.T / n + 0.1 * np.eye(n)))
        pt["Hxp"].append(rng.standard_normal((n, P)))
        pt["Jx"].append(rng.standard_normal((c, n)) / math.sqrt(n))
        pt["Jp"].append(rng.standard_normal((c, P)))
        x = rng.standard_normal(n)
        cval = rng.standard_normal(c)
        crhs = cval.copy()
        y = np.zeros(c)
        for k in range(c):
            act = rng.random() < active
            if kinds[k] == 0:
                y[k] = rng.standard_normal()
            elif kinds[k] == 1:   # GreaterThan: slack = cval − crhs ≥ 0, dual ≥ 0
                if act:
                    y[k] = u()
                else:
                    crhs[k] = cval[k] - u()
            else:                 # LessThan: slack ≤ 0, dual ≤ 0
                if act:
                    y[k] = -u()
                else:
                    crhs[k] = cval[k] + u()
        xl, xu, yl, yu = (np.zeros(n) for _ in range(4))
        for j in range(n):
            if has_low[j]:
                if rng.random() < active:
                    xl[j], yl[j] = x[j], u()
                else:
                    xl[j] = x[j] - u()
            if has_up[j]:
                if rng.random() < active and not (has_low[j] and xl[j] == x[j]):
                    xu[j], yu[j] = x[j], -u()
                else:
                    xu[j] = x[j] + u()
        for k, v in zip(keys[4:], (x, cval, crhs, y, xl, xu, yl, yu)):
            pt[k].append(v)
    pt = {k: np.stack(v) for k, v in pt.items()}
    nd = c + int(has_low.sum()) + int(has_up.sum())
    return st, pt, rng.standard_normal((batch, P)), rng.standard_normal((batch, n)), \
        rng.standard_normal((batch, nd))


def _sparse_wellcond(rng, m, n, k, dense=True):
    """A dense m × n array with ≈ k non-zeros per row and singular values
    O(1): the rows of I + 0.3·R/√k (R: k N(0,1) entries per row) for min(m, n)
    of them, k random N(0,1)/√k entries for the rest, rows permuted."""
    import scipy.sparse as sp
    q = min(m, n)
    rows = np.repeat(np.arange(q), k)
    W = sp.identity(n, format="csr")[:q] + sp.csr_matrix(
        (0.3 * rng.standard_normal(q * k) / math.sqrt(k), (rows, rng.integers(0, n, size=q * k))), shape=(q, n))
    if m > q:
        ri = np.repeat(np.arange(m - q), k)
        W = sp.vstack([W, sp.csr_matrix((rng.standard_normal((m - q) * k) / math.sqrt(k),
                                         (ri, rng.integers(0, n, size=(m - q) * k))), shape=(m - q, n))])
    W = W.tocsr()[rng.permutation(m)]
    return W.toarray() if dense else W.tocsc()


def conic_numpy_wellcond(batch, n, cones, seed, f_interior=0.25, f_dual_interior=0.25, sigma=(1.0, 2.0),
                         pair_norm=0.25, sparse_k=None, sparse_out=False):
    """The converging variant of a conic shape: the same
    cone list, but an instance family on which the reference's LSQR converges
    (istop 1–2) well inside maxiter, so parity can be held to 1e-6 on every
    output.  Differences from ``conic_numpy``:

    * A = U·diag(σ)·Vᵀ with Haar-orthogonal U, V and σ ~ U(sigma) — a square
      Gaussian A (config 4: m = n = 500) has σ_min ≈ 1/n and leaves M with
      near-null singular values ~1e-3 beside its structural null space, so
      LSQR crawls to maxiter (istop 7); with σ ∈ [1, 2] the non-zero spectrum
      of M sits in about [0.3, 4];
    * SOC cones draw one of three complementary cases: s strictly interior
      with y = 0 (probability ``f_interior``; Dπ = 0), s = 0 with y strictly
      interior (``f_dual_interior``; Dπ = I), or the boundary pair of
      ``conic_numpy`` (the third, SOC-specific Dπ branch) — every Dπ branch of
      ConicProgram's SOC projection is exercised;
    * the SOC pair vectors have norm ``pair_norm`` and x ~ N(0,1)/√n, so b and
      c (the last row / column of M) stay O(1).

    M is singular at any exact primal–dual point — z = (x, y − s, 1) is always
    in its null space (M·z = (c − A_moiᵀy, A_moi x + b − s, −(cᵀx + bᵀy)) = 0 by
    feasibility and zero gap) — so LSQR returns the minimum-norm least-squares
    solution, which is unique; "converging" means istop 1–2.  Nonnegatives /
    Nonpositives / Zeros rows as in ``conic_numpy`` (Nonneg / Nonpos entries of
    v = y − s on both sides of 0, |v| ≥ 0.5: the guard band).  PSD triangles
    (VERDICT r03 item 2): S = V·diag(σ)·Vᵀ, Y = V·diag(ω)·Vᵀ strictly
    complementary — each eigen-index carries exactly one of σ_i, ω_i, drawn
    from ``pair_norm``·U(0.5, 1.5), at least one of each — so v = Y − S has
    eigenvalues of both signs bounded away from 0 and every Daleckii–Krein
    weight λ⁺/(λ⁺ − λ⁻) lies in [1/4, 3/4]; c uses MOI's set_dot weights (2 on
    the off-diagonal triangle entries)."""
    rng = np.random.default_rng(seed)
    m = sum(d for _, d in cones)
    out = {k: [] for k in ["A", "b", "c", "x", "s", "y", "dx", "dA", "db", "dc"]}
    for _ in range(batch):
        s = np.zeros(m)
        y = np.zeros(m)
        wts = np.ones(m)
        o = 0
        for code, dim in cones:
            if code == 0:
                y[o:o + dim] = rng.standard_normal(dim)
            elif code in (1, 2):
                sg = 1.0 if code == 1 else -1.0
                act = rng.random(dim) < 0.5
                mag_s = rng.uniform(0.5, 1.5, dim)
                mag_y = rng.uniform(0.5, 1.5, dim)
                s[o:o + dim] = np.where(act, 0.0, sg * mag_s)
                y[o:o + dim] = np.where(act, sg * mag_y, 0.0)
            elif code == 3:
                u = rng.standard_normal(dim - 1)
                u *= pair_norm / np.linalg.norm(u)
                al, be, lift = rng.uniform(0.5, 1.5), rng.uniform(0.5, 1.5), rng.uniform(1.5, 2.5)
                r = rng.random()
                if r < f_interior:            # s ∈ int K, y = 0
                    s[o] = al * pair_norm * lift
                    s[o + 1:o + dim] = al * u
                elif r < f_interior + f_dual_interior:   # s = 0, y ∈ int K
                    y[o] = be * pair_norm * lift
                    y[o + 1:o + dim] = -be * u
                else:                          # boundary pair
                    s[o] = al * pair_norm
                    s[o + 1:o + dim] = al * u
                    y[o] = be * pair_norm
                    y[o + 1:o + dim] = -be * u
            elif code == 4:
                d = int((math.isqrt(8 * dim + 1) - 1) // 2)
                V, _ = np.linalg.qr(rng.standard_normal((d, d)))
                on_s = rng.random(d) < 0.5
                on_s[0], on_s[-1] = True, False          # both ranks non-zero
                mag = pair_norm * rng.uniform(0.5, 1.5, d)
                sig, om = np.where(on_s, mag, 0.0), np.where(on_s, 0.0, mag)
                s[o:o + dim] = _tri((V * sig) @ V.T)
                y[o:o + dim] = _tri((V * om) @ V.T)
                wts[o:o + dim] = np.array([1.0 if i == j else 2.0 for j in range(d) for i in range(j + 1)])
            else:
                raise ValueError("conic_numpy_wellcond: cone code %d not generated" % code)
            o += dim
        if sparse_k:   # the sparse route's family: k entries per row, well conditioned
            A = _sparse_wellcond(rng, m, n, sparse_k, dense=not sparse_out)
        else:
            k = min(m, n)
            U, _ = np.linalg.qr(rng.standard_normal((m, m)))
            V, _ = np.linalg.qr(rng.standard_normal((n, n)))
            sv = rng.uniform(sigma[0], sigma[1], k)
            A = (U[:, :k] * sv) @ V[:, :k].T
        x = rng.standard_normal(n) / math.sqrt(n)
        b = s - A @ x
        c = A.T @ (wts * y)
        out["A"].append(A); out["b"].append(b); out["c"].append(c); out["x"].append(x)
        out["s"].append(s); out["y"].append(y)
        out["dx"].append(rng.standard_normal(n))
        if not sparse_out:   # (sparse_out: A stays a list of scipy CSC, no dense dA tangent)
            out["dA"].append(rng.standard_normal((m, n)))
        out["db"].append(rng.standard_normal(m))
        out["dc"].append(rng.standard_normal(n))
    return {k: (v if k == "A" and sparse_out else np.stack(v)) for k, v in out.items() if v}


def lp_sparse_numpy(batch, n, p, m_extra, k, seed):
    """Seeded sparse LPs (Q = 0: the reference's LSQR branch) at a vertex, for
    the sparse route (sparse.hip).  Per problem: n − p active inequality rows
    and the p equality rows together form W = Π·(I + 0.3·R/√k) (R: k random
    N(0,1) entries per row, Π a row permutation) — a well-conditioned square
    matrix, so the full KKT LHS is nonsingular and LSQR converges well before
    maxiter; m_extra inactive rows with k random entries each.  Active rows:
    s = 0, λ ~ U(0.5, 1.5); inactive: λ = 0, s ~ −U(0.5, 1.5).  Returns dict of
    lists: G, A (scipy CSC per problem), h, z, lam, nu, dl_dz, dq, dh, db
    (stacked arrays), with m = n − p + m_extra."""
    import scipy.sparse as sp
    rng = np.random.default_rng(seed)
    m = n - p + m_extra
    out = {key: [] for key in ["G", "A", "h", "z", "lam", "nu", "dl_dz", "dq", "dh", "db"]}
    for _ in range(batch):
        rows = np.repeat(np.arange(n), k)
        cols = rng.integers(0, n, size=n * k)
        vals = 0.3 * rng.standard_normal(n * k) / math.sqrt(k)
        W = (sp.identity(n, format="csr") + sp.csr_matrix((vals, (rows, cols)), shape=(n, n))).tocsr()
        W = W[rng.permutation(n)]
        Ga, A = W[: n - p], W[n - p:]
        ri = np.repeat(np.arange(m_extra), k)
        ci = rng.integers(0, n, size=m_extra * k)
        Gi = sp.csr_matrix((rng.standard_normal(m_extra * k) / math.sqrt(k), (ri, ci)), shape=(m_extra, n))
        G = sp.vstack([Ga, Gi]).tocsr()
        perm = rng.permutation(m)
        G = G[perm]
        act = perm < n - p                       # row i of G is active iff it came from Ga
        lam = np.where(act, rng.uniform(0.5, 1.5, size=m), 0.0)
        s = np.where(act, 0.0, -rng.uniform(0.5, 1.5, size=m))
        z = rng.standard_normal(n)
        out["G"].append(sp.csc_matrix(G))
        out["A"].append(sp.csc_matrix(A))
        out["h"].append(G @ z - s)
        out["z"].append(z)
        out["lam"].append(lam)
        out["nu"].append(rng.standard_normal(p))
        out["dl_dz"].append(rng.standard_normal(n))
        out["dq"].append(rng.standard_normal(n))
        out["dh"].append(rng.standard_normal(m))
        out["db"].append(rng.standard_normal(p))
    for key in ["h", "z", "lam", "nu", "dl_dz", "dq", "dh", "db"]:
        out[key] = np.stack(out[key])
    return out
