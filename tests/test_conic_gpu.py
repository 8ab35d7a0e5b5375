"""ConicProgram sensitivity path on the GPU (via the C-ABI) against the CPU
oracle and the reference's own fixtures (test/conic_program.jl, see
tests/golden/make_golden.py).

Parity bar: north_star's 1e-6 relative Frobenius against the oracle, per
problem and per output.  One exception, counted and capped per test: when M
is numerically singular and LSQR stops at maxiter (istop 7 — the config-4
bench shape, the PSD+POS fixture), the oracle itself moves by ≫ 1e-6 under a
1-ulp perturbation of its inputs, so no implementation can meet 1e-6; such
an output is held to 10× the oracle's own 1-ulp spread instead ("relaxed").
Every test reports how many outputs were judged under the relaxed bar and
asserts its cap (0 for the well-posed shapes)."""

import json
import os

import numpy as np
import pytest

from oracle import conic as ocn

pytestmark = pytest.mark.gpu
RTOL = 1e-6
HERE = os.path.dirname(os.path.abspath(__file__))
SEED0 = 20250307


def relfro(a, b):
    a, b = np.asarray(a, dtype=float).ravel(), np.asarray(b, dtype=float).ravel()
    nb = np.linalg.norm(b)
    return np.linalg.norm(a - b) / nb if nb > 0 else np.linalg.norm(a)


def relcomb(a, b, scale):
    """Relative error of an output derived linearly from the LSQR solution
    (dx = −(du − x·dw), dc = g_x − g_end·x, …), normalised by the bound that
    a 1e-6-relative error of the solution itself propagates to (`scale` =
    ‖solution‖ × the derivation's gain), so a component that cancels to ~0 in
    exact arithmetic is not judged on its rounding noise."""
    a, b = np.asarray(a, dtype=float).ravel(), np.asarray(b, dtype=float).ravel()
    den = max(np.linalg.norm(b), scale)
    return np.linalg.norm(a - b) / den if den > 0 else np.linalg.norm(a)


class Tally:
    """Counts the outputs judged under the relaxed (1-ulp envelope) bar."""

    def __init__(self, name):
        self.name, self.total, self.relaxed, self.worst = name, 0, 0, 0.0

    def check(self, err, envelope_fn, what, minnorm_fn=None):
        """err ≤ RTOL, or (only if the oracle's own envelope exceeds RTOL/10)
        err ≤ 10 × envelope.  `envelope_fn` is evaluated lazily.  For a shape
        whose LSQR converges (istop 1–2) `minnorm_fn` may judge instead: the
        engine at least as close to the EXACT minimum-norm solution as twice
        the oracle (both stop at the reference's √eps tolerances, so their
        mutual difference is stopping noise, not error)."""
        self.total += 1
        self.worst = max(self.worst, err)
        if err <= RTOL:
            return
        if minnorm_fn is not None:
            assert minnorm_fn(), (what, err, "farther from the exact min-norm solution than 2 × the oracle")
            self.relaxed += 1
            return
        env = envelope_fn()
        assert env > RTOL / 10, (what, err, env)
        assert err <= 10.0 * env, (what, err, env)
        self.relaxed += 1

    def report(self, cap):
        """cap None: the shape's relaxed outputs were each judged by the exact
        min-norm bar (check's minnorm_fn), so their count is reported only."""
        bar = "exact min-norm bar, no cap" if cap is None else f"cap {cap}"
        print(f"[parity] {self.name}: {self.total} outputs, {self.relaxed} under the relaxed "
              f"envelope bar ({bar}), worst error {self.worst:.2e}")
        log = os.environ.get("DOPT_PARITY_LOG")
        if log:
            with open(log, "a") as f:
                f.write(json.dumps(dict(test=self.name, outputs=self.total, relaxed=self.relaxed,
                                        cap=cap, worst=self.worst)) + "\n")
        if cap is not None and not os.environ.get("DOPT_PARITY_CALIBRATE"):
            assert self.relaxed <= cap, (self.name, self.relaxed, cap)


def envelope(solve, args, ref, metric, trials=3):
    """Largest change of the oracle's output when its right-hand-side data is
    perturbed by one ulp (relative 2⁻⁵², seeded)."""
    rng = np.random.default_rng(7)
    worst = 0.0
    for _ in range(trials):
        pert = [np.asarray(a, float) * (1.0 + 2.0 ** -52 * rng.standard_normal(np.shape(a)))
                for a in args]
        worst = max(worst, metric(solve(*pert), ref))
    return worst


@pytest.fixture(scope="module")
def ConicBatch():
    from diffopt_amd.conic import ConicBatch
    return ConicBatch


FX = json.load(open(os.path.join(HERE, "golden", "conic_fixtures.json")))
FX_CAP = {"conic_psd_pos": 2}   # LSQR stops at maxiter on cond(M) ≈ 8e16


@pytest.mark.parametrize("fx", FX, ids=[f["name"] for f in FX])
def test_fixture_forward_reverse(ConicBatch, fx):
    A = np.array(fx["A"], dtype=float)
    m, n = A.shape
    cones = [tuple(c) for c in fx["cones"]]
    c = -np.array(fx["c"]) if fx["max_sense"] else np.array(fx["c"], dtype=float)
    cache = ocn.Cache(A, fx["b"], fx["c"], fx["x"], fx["s"], fx["y"], cones, fx["max_sense"])
    e = ConicBatch(1, n, cones)
    e.set(A[None], np.array(fx["b"])[None], c[None], np.array(fx["x"])[None],
          np.array(fx["s"])[None], np.array(fx["y"])[None])
    tally = Tally(fx["name"])
    x = np.array(fx["x"], dtype=float)
    for t in fx["forward"]:
        dA = np.array(t["dA"], dtype=float)
        out, dx = e.forward(dA[None], np.array(t["db"])[None], np.array(t["dc"])[None])
        np.testing.assert_allclose(dx[0], t["dx"], atol=t["atol"], rtol=t["rtol"])
        odx, du, dv, dw = ocn.forward_differentiate(cache, dA, t["db"], t["dc"])
        ref = np.concatenate([du, dv, [dw]])

        def fsolve(dA_, db_, dc_):
            _, a, b_, c_ = ocn.forward_differentiate(cache, dA_, db_, dc_)
            return np.concatenate([a, b_, [c_]])
        env = lambda: envelope(fsolve, [dA, t["db"], t["dc"]], ref, relfro)
        tally.check(relfro(out[0], ref), env, "forward")
        sol = np.linalg.norm(ref)
        tally.check(relcomb(dx[0], odx, sol * (1 + np.linalg.norm(x))), env, "dx")
    for t in fx["reverse"]:
        g, dA, db, dc = e.reverse(np.array(t["dx"], dtype=float)[None])
        np.testing.assert_allclose(db[0][t["rows"]], t["db"], atol=t["atol"], rtol=t["rtol"])
        og, _ = ocn.reverse_differentiate(cache, t["dx"])
        tally.check(relfro(g[0], og), lambda: envelope(
            lambda dx_: ocn.reverse_differentiate(cache, dx_)[0], [t["dx"]], og, relfro), "reverse")
    e.close()
    tally.report(FX_CAP.get(fx["name"], 0))


def _oracle_outputs(cache, dA, db, dc, dx):
    (odx, du, dv, dw), fi = ocn.forward_differentiate(cache, dA, db, dc, return_info=True)
    (og, _), ri = ocn.reverse_differentiate(cache, dx, return_info=True)
    odA, odb, odc = ocn.reverse_outputs(cache, og)
    return dict(fwd=np.concatenate([du, dv, [dw]]), dx=odx, g=og, dA=odA, db=odb, dc=odc,
                info=(fi, ri))


def _errors(got, ref, cache):
    """Per-output error metrics (relfro for the LSQR solutions, relcomb for
    the outputs derived from them)."""
    nx, nvp = np.linalg.norm(cache.x), np.linalg.norm(cache.vp)
    sol, ng = np.linalg.norm(ref["fwd"]), np.linalg.norm(ref["g"])
    return dict(fwd=relfro(got["fwd"], ref["fwd"]),
                dx=relcomb(got["dx"], ref["dx"], sol * (1 + nx)),
                g=relfro(got["g"], ref["g"]),
                dA=relcomb(got["dA"], ref["dA"], ng * (nx + nvp)),
                db=relcomb(got["db"], ref["db"], ng * (1 + nvp)),
                dc=relcomb(got["dc"], ref["dc"], ng * (1 + nx)))


def _minnorm_judge(cache, d, b, out_b, g_b, ref):
    """{direction: engine within max(2 × oracle, 1e-8) of the exact min-norm
    solution} — the converged shapes' bar (test_converged_shapes_vs_exact_minnorm)."""
    frhs = ocn.forward_rhs(cache, d["dA"][b], d["db"][b], d["dc"][b])
    rrhs = np.concatenate([d["dx"][b], np.zeros(cache.m), [-(cache.x @ d["dx"][b])]])
    res = {}
    for what, rhs, eng, orc in (("fwd", frhs, out_b, ref["fwd"]), ("rev", rrhs, g_b, ref["g"])):
        ex = _exact_minnorm(cache, rhs)
        nx = np.linalg.norm(ex)
        res[what] = np.linalg.norm(eng - ex) / nx <= max(2.0 * np.linalg.norm(orc - ex) / nx, 1e-8)
    return res


def _synthetic_check(ConicBatch, B, n, cones, seed, name, cap=0, trials=3, want_dA=True, gen=None,
                     minnorm=False):
    """GPU vs oracle per problem and output (tallied: RTOL, or the relaxed
    envelope bar where the oracle's own 1-ulp spread exceeds RTOL/10; with
    `minnorm` — shapes whose LSQR converges — the exact min-norm bar instead).
    Returns (tally, engine LSQR iteration counts fwd, rev, oracle infos)."""
    from diffopt_amd.synthetic import conic_numpy
    d = (gen or conic_numpy)(B, n, cones, seed)
    e = ConicBatch(B, n, cones)
    e.set(d["A"], d["b"], d["c"], d["x"], d["s"], d["y"])
    out, dx = e.forward(d["dA"], d["db"], d["dc"])
    it_f = e.iterations()
    g, dA, db, dc = e.reverse(d["dx"], want_dA=want_dA)
    it_r = e.iterations()
    e.close()
    tally = Tally(name)
    infos = []
    for b in range(B):
        cache = ocn.Cache(d["A"][b], d["b"][b], d["c"][b], d["x"][b], d["s"][b], d["y"][b], cones)
        args = [d["dA"][b], d["db"][b], d["dc"][b], d["dx"][b]]
        ref = _oracle_outputs(cache, *args)
        infos.append(ref["info"])
        got = dict(fwd=out[b], dx=dx[b], g=g[b], dA=dA[b] if want_dA else ref["dA"], db=db[b], dc=dc[b])
        err = _errors(got, ref, cache)
        env_cache = {}

        def env_of(k):
            if not env_cache:   # one set of perturbed oracle solves serves every output
                rng = np.random.default_rng(7)
                env_cache.update(dict.fromkeys(err, 0.0))
                for _ in range(trials):
                    pert = [a * (1.0 + 2.0 ** -52 * rng.standard_normal(a.shape)) for a in args]
                    pe = _errors(_oracle_outputs(cache, *pert), ref, cache)
                    env_cache.update({kk: max(env_cache[kk], pe[kk]) for kk in env_cache})
            return env_cache[k]
        mn_cache = {}

        def mn_of(k, b=b, cache=cache, ref=ref):
            if not mn_cache:
                mn_cache.update(_minnorm_judge(cache, d, b, out[b], g[b], ref))
            return mn_cache["fwd" if k in ("fwd", "dx") else "rev"]
        for k in err:
            tally.check(err[k], lambda k=k: env_of(k), (b, k), (lambda k=k: mn_of(k)) if minnorm else None)
    tally.report(cap)
    return tally, it_f, it_r, infos


def test_well_posed_batch(ConicBatch):
    # m > n (unique primal) and LSQR converging (istop 1), but stopping at the
    # reference's √eps tolerance, so two correct runs differ by ≈ cond(M)·1.5e-8
    # (4 of the 12 outputs in (1e-6, 2.8e-6], r02): an output above 1e-6 is
    # judged by the exact min-norm bar (engine within 2× the oracle's distance)
    _synthetic_check(ConicBatch, 2, 100, [(3, 10)] * 20, 21, "well-posed SOC", cap=None, minnorm=True)


def test_mixed_cones_batch(ConicBatch):
    # LSQR to maxiter on a singular M: 32–33 of 36 under the 1-ulp envelope bar
    # (r04: 33 with the DPP wave sums' summation order)
    _synthetic_check(ConicBatch, 6, 30, [(0, 3), (1, 10), (3, 6), (2, 4), (4, 6)], 11, "mixed cones",
                     cap=34)


def test_soc_only_batch(ConicBatch):
    _synthetic_check(ConicBatch, 4, 40, [(3, 5)] * 8, 12, "SOC only", cap=24)


def test_psd_blocks_batch(ConicBatch):
    _synthetic_check(ConicBatch, 3, 25, [(4, 10), (4, 15), (1, 5)], 13, "PSD blocks", cap=18)


def test_config4_nondegenerate_shape(ConicBatch):
    # config-4 structure (n=500, 20 SOCs) with cone dim 50, so m = 1000 > n and
    # M is non-singular: LSQR converges; converged at √eps as above (2 of 12
    # outputs in (1e-6, 4.9e-6], r02): the exact min-norm bar above 1e-6
    _synthetic_check(ConicBatch, 2, 500, [(3, 50)] * 20, 14, "config-4 structure, m=1000", cap=None, minnorm=True)


def test_config4_converging_variant(ConicBatch):
    """Config 4's shape (n = 500, 20 × SOC(25), m = n) on the converging
    instance family (synthetic.conic_numpy_wellcond: well-conditioned A, every
    SOC Dπ branch — interior, dual-interior, boundary pair), seed SEED0 + 4 —
    the first problems of `bench.py --config 4 --conic-variant wellcond`.
    LSQR converges (istop 1–2) in ≈ 40–60 iterations in the engine and the
    oracle; every output at 1e-6 relative Frobenius with NO relaxed output
    (cap 0).  LSQR's own scalars: istop equal, the iteration count within one
    (a 1-ulp perturbation of the oracle's inputs moves its own count by one on
    2 of these 4 problems: the stopping test sits at √eps), rnorm and xnorm
    to 1e-6 (converged quantities), anorm to 1e-3 where the counts agree (it
    sums every α_k² + β_k² of the Golub–Kahan sequence, whose later terms
    drift with the vectors' lost orthogonality: 4e-5 measured), arnorm not at
    all (at istop 2 it is the √eps-level stopping residual, noise)."""
    from diffopt_amd.synthetic import conic_numpy_wellcond
    cones = [(3, 25)] * 20
    B, n = 4, 500
    d = conic_numpy_wellcond(B, n, cones, SEED0 + 4)
    e = ConicBatch(B, n, cones)
    e.set(d["A"], d["b"], d["c"], d["x"], d["s"], d["y"])
    (out, fdx), (g, dA, db, dc) = e.forward_reverse(d["dx"], d["dA"], d["db"], d["dc"])
    st = e.lsqr_stats()
    nr = e.lsqr_norms()
    e.close()
    tally = Tally("config-4 converging variant")
    keys = ("rnorm", "arnorm", "xnorm", "anorm")
    for b in range(B):
        cache = ocn.Cache(d["A"][b], d["b"][b], d["c"][b], d["x"][b], d["s"][b], d["y"][b], cones)
        sf, sr = {}, {}
        (odx, du, dv, dw), fi = ocn.forward_differentiate(cache, d["dA"][b], d["db"][b], d["dc"][b],
                                                          return_info=True, stats=sf)
        (og, _), ri = ocn.reverse_differentiate(cache, d["dx"][b], return_info=True, stats=sr)
        odA, odb, odc = ocn.reverse_outputs(cache, og)
        ref = dict(fwd=np.concatenate([du, dv, [dw]]), dx=odx, g=og, dA=odA, db=odb, dc=odc)
        err = _errors(dict(fwd=out[b], dx=fdx[b], g=g[b], dA=dA[b], db=db[b], dc=dc[b]), ref, cache)
        for k, v in err.items():
            tally.check(v, lambda: 0.0, (b, k))   # envelope 0: no relaxed bar
        for (istop, it), (est, ost), oi in (((st["fwd_istop"][b], st["fwd_iterations"][b]), (nr["fwd"][b], sf), fi),
                                            ((st["istop"][b], st["iterations"][b]), (nr["last"][b], sr), ri)):
            assert istop in (1, 2) and istop == oi[1], (b, istop, oi)
            assert abs(int(it) - oi[0]) <= 1, (b, it, oi)
            o = np.array([ost[k] for k in keys])
            for j in (0, 2):
                assert abs(est[j] - o[j]) <= 1e-6 * abs(o[j]), (b, keys[j], est[j], o[j])
            if int(it) == oi[0]:
                assert abs(est[3] - o[3]) <= 1e-3 * abs(o[3]), (b, "anorm", est[3], o[3])
    tally.report(0)


def _ls_quality(M, rhs, x):
    """(‖Mx − rhs‖, ‖Mᵀ(Mx − rhs)‖ / (‖M‖₂‖Mx − rhs‖)) of an LSQR iterate."""
    r = M @ x - rhs
    nr = np.linalg.norm(r)
    return nr, np.linalg.norm(M.T @ r) / (np.linalg.norm(M, 2) * nr)


def test_config4_bench_shape(ConicBatch):
    """The exact config-4 bench shape and generator (20 × SOC(25), n = 500,
    seed SEED0 + 4: the first two problems of bench.py's batch).  M has, besides
    its structural null space, singular values down to ~1e-17 (a square
    Gaussian A): both LSQR directions stop at maxiter = N = 1001 (istop 7) in
    the engine and in the oracle alike, and the final iterate is chaotic —
    measured on the oracle itself, a 1-ulp relative perturbation of the
    right-hand side moves its terminal rnorm by ~3e-3, xnorm and anorm by
    ~1e-2, arnorm by up to 8×, and the true normal-equation residual ratio by
    30× (profiles/r03/conic_cfg4_maxiter_spread.txt).  No implementation can
    match such a run to 1e-6, so parity here is judged on what is stable:

    * istop = 7 and 1001 iterations in both directions, as the oracle;
    * LSQR's terminal estimates rnorm, xnorm, anorm inside the band the
      oracle's own 1-ulp neighbours span (widened by twice that spread), arnorm
      within 4× of that band in log scale;
    * the engine iterate is as good a least-squares point as the oracle's:
      the true ‖M x − b‖ inside the same band and ‖Mᵀ(Mx − b)‖/(‖M‖‖Mx − b‖)
      at most 2× the worst of the oracle's runs.
    The outputs themselves are still reported against the 1-ulp envelope
    (tallied, cap 12) as a sanity bound; the 1e-6 claim for config 4 rests on
    the converging variant above."""
    tally, it_f, it_r, infos = _synthetic_check(ConicBatch, 2, 500, [(3, 25)] * 20, SEED0 + 4,
                                                "config-4 bench shape", cap=12, trials=2)
    assert (it_f == 1001).all() and (it_r == 1001).all()
    assert all(fi == (1001, 7) and ri == (1001, 7) for fi, ri in infos)
    from diffopt_amd.synthetic import conic_numpy
    cones = [(3, 25)] * 20
    d = conic_numpy(2, 500, cones, SEED0 + 4)
    e = ConicBatch(2, 500, cones)
    e.set(d["A"], d["b"], d["c"], d["x"], d["s"], d["y"])
    (out, _), (g, *_r) = e.forward_reverse(d["dx"], d["dA"], d["db"], d["dc"], want_dA=False)
    nr = e.lsqr_norms()
    st = e.lsqr_stats()
    e.close()
    assert (st["istop"] == 7).all() and (st["fwd_istop"] == 7).all()
    keys = ("rnorm", "arnorm", "xnorm", "anorm")
    lines = []
    for b in range(2):
        cache = ocn.Cache(d["A"][b], d["b"][b], d["c"][b], d["x"][b], d["s"][b], d["y"][b], cones)
        M = cache.M()
        frhs = ocn.forward_rhs(cache, d["dA"][b], d["db"][b], d["dc"][b])
        rrhs = np.concatenate([d["dx"][b], np.zeros(cache.m), [-(cache.x @ d["dx"][b])]])
        for name, rhs, x, est in (("fwd", frhs, out[b], nr["fwd"][b]), ("rev", rrhs, g[b], nr["last"][b])):
            rng = np.random.default_rng(7)
            runs = []
            for t in range(5):
                rr = rhs if t == 0 else rhs * (1.0 + 2.0 ** -52 * rng.standard_normal(rhs.shape))
                stt = {}
                from oracle.lsqr import lsqr
                xo, it, istop = lsqr(cache.matvec, cache.rmatvec, rr, len(rr), return_info=True, stats=stt)
                assert (it, istop) == (1001, 7)
                runs.append([stt[k] for k in keys] + list(_ls_quality(M, rhs, xo)))
            runs = np.array(runs)
            lo, hi = runs.min(0), runs.max(0)
            sp = hi - lo
            q = _ls_quality(M, rhs, x)
            got = list(est) + list(q)
            lines.append(f"problem {b} {name}: engine {np.array2string(np.array(got), precision=4)}; "
                         f"oracle min {np.array2string(lo, precision=4)} max {np.array2string(hi, precision=4)}")
            for j in (0, 2, 3, 4):   # rnorm, xnorm, anorm, true ‖Mx − b‖
                assert lo[j] - 2 * sp[j] <= got[j] <= hi[j] + 2 * sp[j], (b, name, j, got[j], lo[j], hi[j])
            assert lo[1] / 4 <= got[1] <= hi[1] * 4, (b, name, "arnorm", got[1], lo[1], hi[1])
            assert got[5] <= 2 * hi[5], (b, name, "normal residual", got[5], hi[5])
    print("[parity] config-4 maxiter quality:\n  " + "\n  ".join(lines))


def test_config5_full_shape(ConicBatch):
    """The full config-5 SDP shape (10 × PSD(50): m = 12 750, n = 500, seed
    SEED0 + 5: bench.py's first problem), batch 1 — 13 251 unknowns, the split
    (row-block) LSQR path.  dA is not materialised (51 MB per problem)."""
    tally, it_f, it_r, infos = _synthetic_check(ConicBatch, 1, 500, [(4, 1275)] * 10, SEED0 + 5,
                                                "config-5 full shape", cap=0, trials=1, want_dA=False)
    print(f"[parity] config-5 LSQR iterations: engine fwd {it_f[0]} rev {it_r[0]}, oracle {infos[0]}")


# every shape converges at √eps (istop 1–2): 1–3 of the outputs land in
# (1e-6, 1.6e-5] depending on the summation order (r02–r04), each judged by the
# exact min-norm bar (engine within 2× the oracle's distance from it)
@pytest.mark.parametrize("shape", [
    ("large PSD (d = 66) + small cones", 2, 60, [(4, 2211), (4, 15), (1, 5)], 17),
    ("large PSD (d = 100)", 1, 60, [(4, 5050)], 18),
    ("large PSD (d = 300)", 1, 40, [(4, 45150)], 19),
], ids=["d66_mixed", "d100", "d300"])
def test_large_psd_sides(ConicBatch, shape):
    """PSD sides above 64 (the LDS eigensolver / Dπ apply limit): the same code
    on global scratch, split LSQR path; d = 300 exceeds the Jacobi rotation
    table (256: chunked rotations, the eigenvalue order in the scratch) and the
    oracle's dense Jacobian (45 150², 16 GB: oracle.cones.PSDStructured).
    Reference: any MOI PSD triangle (ConicProgram.jl:132-142,
    diff_opt.jl:491-519)."""
    name, B, n, cones, seed = shape
    _synthetic_check(ConicBatch, B, n, cones, seed, name, cap=None, minnorm=True)


# ---------------------------------------------------------------------------
# the non-SOC Dπ branches at the 1e-6 bar, and the
# converged-but-capped shapes against the exact minimum-norm solution
# ---------------------------------------------------------------------------
ALL5_SHAPES = [
    # every cone code, m > n, strictly complementary pairs: Zeros, Nonneg /
    # Nonpos entries of v on both sides of 0 (|v| ≥ 0.5), SOC interior / dual-
    # interior / boundary pairs, PSD blocks with eigenvalues of v of both signs
    # (synthetic.conic_numpy_wellcond); LSQR converges (istop 2) in 54–86
    # iterations, the oracle's own 1-ulp spread ≤ 5e-7 (seed 42: ≤ 5e-9)
    ("all five cones, m=69 n=60", 4, 60, [(0, 2), (1, 30), (2, 20), (3, 8), (4, 6), (4, 3)], 42),
    ("all five cones, m=87 n=80", 4, 80, [(0, 5), (1, 20), (2, 10), (3, 10), (3, 6), (4, 15), (4, 21)], 41),
]


@pytest.mark.parametrize("split", ["0", "1"], ids=["persistent", "split"])
@pytest.mark.parametrize("shape", ALL5_SHAPES, ids=["m69", "m87"])
def test_all_cone_codes_converging(ConicBatch, monkeypatch, shape, split):
    """Zeros / Nonnegatives / Nonpositives / SOC / PSD in one M
    (ConicProgram.jl:172-255, diff_opt.jl:491-519), on instances where the
    reference's LSQR converges: every output of every problem at 1e-6
    relative Frobenius with NO relaxed output (cap 0), on the persistent and
    on the split LSQR path, forward (:320-324) and reverse (:369-372)."""
    from diffopt_amd.synthetic import conic_numpy_wellcond
    name, B, n, cones, seed = shape
    monkeypatch.setenv("DOPT_CONIC_SPLIT", split)
    d = conic_numpy_wellcond(B, n, cones, seed, pair_norm=1.0)
    codes = {c for c, _ in cones}
    assert codes == {0, 1, 2, 3, 4}
    e = ConicBatch(B, n, cones)
    e.set(d["A"], d["b"], d["c"], d["x"], d["s"], d["y"])
    (out, fdx), (g, dA, db, dc) = e.forward_reverse(d["dx"], d["dA"], d["db"], d["dc"])
    st = e.lsqr_stats()
    e.close()
    tally = Tally(f"{name} ({'split' if split == '1' else 'persistent'})")
    for b in range(B):
        cache = ocn.Cache(d["A"][b], d["b"][b], d["c"][b], d["x"][b], d["s"][b], d["y"][b], cones)
        # the generator's strict complementarity, as the branches see it
        v = d["y"][b] - d["s"][b]
        o = 0
        for code, dim in cones:
            if code in (1, 2):
                assert np.all(np.abs(v[o:o + dim]) >= 0.5) and (v[o:o + dim] > 0).any() and (v[o:o + dim] < 0).any()
            if code == 4:
                k = int((np.sqrt(8 * dim + 1) - 1) // 2)
                Vm = np.zeros((k, k))
                tri = [(i, j) for j in range(k) for i in range(j + 1)]
                for t_, (i, j) in enumerate(tri):
                    Vm[i, j] = Vm[j, i] = v[o + t_]
                ev = np.linalg.eigvalsh(Vm)
                assert ev.min() < -0.1 and ev.max() > 0.1 and np.abs(ev).min() >= 1e-3
            o += dim
        ref = _oracle_outputs(cache, d["dA"][b], d["db"][b], d["dc"][b], d["dx"][b])
        fi, ri = ref["info"]
        assert fi[1] in (1, 2) and ri[1] in (1, 2), (b, fi, ri)
        assert st["fwd_istop"][b] in (1, 2) and st["istop"][b] in (1, 2)
        err = _errors(dict(fwd=out[b], dx=fdx[b], g=g[b], dA=dA[b], db=db[b], dc=dc[b]), ref, cache)
        for k, val in err.items():
            tally.check(val, lambda: 0.0, (b, k))   # envelope 0: no relaxed bar
    tally.report(0)


def _exact_minnorm(cache, rhs):
    """The exact minimum-norm least-squares solution of M·z = rhs — what
    LSQR from z0 = 0 converges to — by LSQR with its tolerances at 1e-15 on
    the oracle's matrix-free M (scipy.sparse.linalg.lsqr)."""
    import scipy.sparse.linalg as spl
    N = cache.n + cache.m + 1
    op = spl.LinearOperator((N, N), matvec=cache.matvec, rmatvec=cache.rmatvec, dtype=float)
    z, istop = spl.lsqr(op, rhs, atol=1e-15, btol=1e-15, conlim=1e16, iter_lim=50 * N)[:2]
    assert istop in (1, 2), istop
    return z


@pytest.mark.parametrize("shape", [
    ("well-posed SOC", 2, 100, [(3, 10)] * 20, 21),
    ("config-4 structure, m=1000", 2, 500, [(3, 50)] * 20, 14),
    ("large PSD (d = 66) + small cones", 2, 60, [(4, 2211), (4, 15), (1, 5)], 17),
    ("large PSD (d = 100)", 1, 60, [(4, 5050)], 18),
    ("large PSD (d = 300)", 1, 40, [(4, 45150)], 19),
], ids=["soc", "m1000", "d66", "d100", "d300"])
def test_converged_shapes_vs_exact_minnorm(ConicBatch, shape):
    """The shapes whose LSQR converges (istop 1–2) but stops at the
    reference's √eps tolerances, where engine and oracle differ by up to
    1.6e-5 (caps 1–4 above): both are compared with the EXACT minimum-norm
    solution of the same system, and the engine must be at least as close as
    twice the oracle (the reference algorithm itself) — ‖engine − exact‖ ≤
    max(2‖oracle − exact‖, 1e-8‖exact‖), forward and reverse.  That separates
    the √eps stopping noise both share from an error of the engine's own."""
    from diffopt_amd.synthetic import conic_numpy
    name, B, n, cones, seed = shape
    d = conic_numpy(B, n, cones, seed)
    e = ConicBatch(B, n, cones)
    e.set(d["A"], d["b"], d["c"], d["x"], d["s"], d["y"])
    (out, _), (g, *_r) = e.forward_reverse(d["dx"], d["dA"], d["db"], d["dc"], want_dA=False)
    e.close()
    lines = []
    for b in range(B):
        cache = ocn.Cache(d["A"][b], d["b"][b], d["c"][b], d["x"][b], d["s"][b], d["y"][b], cones)
        frhs = ocn.forward_rhs(cache, d["dA"][b], d["db"][b], d["dc"][b])
        rrhs = np.concatenate([d["dx"][b], np.zeros(cache.m), [-(cache.x @ d["dx"][b])]])
        _, du, dv, dw = ocn.forward_differentiate(cache, d["dA"][b], d["db"][b], d["dc"][b])
        og, _ = ocn.reverse_differentiate(cache, d["dx"][b])
        for what, rhs, eng, orc in (("fwd", frhs, out[b], np.concatenate([du, dv, [dw]])), ("rev", rrhs, g[b], og)):
            ex = _exact_minnorm(cache, rhs)
            nx = np.linalg.norm(ex)
            e_eng, e_orc = np.linalg.norm(eng - ex) / nx, np.linalg.norm(orc - ex) / nx
            lines.append(f"problem {b} {what}: engine {e_eng:.2e}, oracle {e_orc:.2e} from the exact min-norm solution")
            assert e_eng <= max(2.0 * e_orc, 1e-8), (name, b, what, e_eng, e_orc)
    print(f"[parity] {name}:\n  " + "\n  ".join(lines))
    log = os.environ.get("DOPT_PARITY_LOG")
    if log:
        with open(log, "a") as f:
            f.write(json.dumps(dict(test=f"exact min-norm: {name}", lines=lines)) + "\n")


def test_zero_rhs_gives_zero(ConicBatch):
    from diffopt_amd.synthetic import conic_numpy
    cones = [(1, 6), (3, 4)]
    d = conic_numpy(2, 8, cones, 15)
    e = ConicBatch(2, 8, cones)
    e.set(d["A"], d["b"], d["c"], d["x"], d["s"], d["y"])
    out, dx = e.forward(None, None, None)          # RHS exactly zero (:320)
    assert np.all(out == 0) and np.all(dx == 0)
    g, _, _, _ = e.reverse(np.full((2, 8), 1e-6))  # ‖dz‖ ≤ 1e-4 (:369-370)
    assert np.all(g == 0)
    e.close()


def test_missing_starts_raise(ConicBatch):
    """NaN in y or s (the reference's marker of a missing start) fails the
    factorisation with ConicProgram.jl:186-196's messages, dual first."""
    from diffopt_amd import EngineError
    from diffopt_amd.synthetic import conic_numpy
    cones = [(1, 6), (3, 4)]
    d = conic_numpy(2, 8, cones, 15)
    for key, word in (("y", "ConstraintDualStart"), ("s", "ConstraintPrimalStart")):
        bad = dict(d)
        bad[key] = d[key].copy()
        bad[key][1, 7] = np.nan
        e = ConicBatch(2, 8, cones)
        e.set(bad["A"], bad["b"], bad["c"], bad["x"], bad["s"], bad["y"])
        with pytest.raises(EngineError, match=word):
            e.factor()
        with pytest.raises(EngineError, match=word):
            e.reverse(d["dx"])
        e.close()


def test_csc_staging_matches_dense_and_oracle(ConicBatch):
    """dopt_conic_set_csc (A_moi as Julia CSC arrays, 1-based, densified on the
    device): against the oracle on the same sparse problems, and bit-identical
    to dopt_conic_set with the dense A; a malformed colptr raises."""
    import scipy.sparse as sp
    from diffopt_amd import EngineError
    from diffopt_amd.synthetic import conic_numpy
    cones = [(0, 3), (1, 10), (3, 6), (4, 6)]
    d = conic_numpy(3, 20, cones, 31)
    A = d["A"].copy()
    A[:, :, 2] = 0.0                      # an empty column
    outs = []
    for mode in ("dense", "csc"):
        e = ConicBatch(3, 20, cones)
        if mode == "dense":
            e.set(A, d["b"], d["c"], d["x"], d["s"], d["y"])
        else:
            e.set_csc([sp.csc_matrix(a) for a in A], d["b"], d["c"], d["x"], d["s"], d["y"])
        out, dx = e.forward(None, d["db"], d["dc"])
        g = e.reverse(d["dx"])[0]
        outs.append((np.asarray(out), np.asarray(dx), np.asarray(g)))
        e.close()
    for a, b in zip(*outs):
        np.testing.assert_array_equal(a, b)
    # every problem here stops at maxiter (istop 7) and the oracle's 1-ulp
    # spread is heavy-tailed: problem 1 (reverse) measured 1.4e-5 as the max
    # of 3 seeded perturbations but 1.6e-3 as the max of 20 — the envelope
    # takes 20
    tally = Tally("CSC staging")
    for b in range(3):
        cache = ocn.Cache(A[b], d["b"][b], d["c"][b], d["x"][b], d["s"][b], d["y"][b], cones)
        _, du, dv, dw = ocn.forward_differentiate(cache, None, d["db"][b], d["dc"][b])
        og, _ = ocn.reverse_differentiate(cache, d["dx"][b])
        ref = np.concatenate([du, dv, [dw]])
        def fsolve(db_, dc_):
            _, a, v, w = ocn.forward_differentiate(cache, None, db_, dc_)
            return np.concatenate([a, v, [w]])
        tally.check(relfro(outs[1][0][b], ref),
                    lambda: envelope(fsolve, [d["db"][b], d["dc"][b]], ref, relfro, trials=20), (b, "fwd"))
        tally.check(relfro(outs[1][2][b], og), lambda: envelope(
            lambda dx_: ocn.reverse_differentiate(cache, dx_)[0], [d["dx"][b]], og, relfro, trials=20),
            (b, "rev"))
    tally.report(6)
    e = ConicBatch(1, 20, cones)
    bad = sp.csc_matrix(A[0])
    bad.indptr[5] = bad.indptr[4] - 1     # non-monotone colptr
    with pytest.raises(EngineError):
        e.set_csc(bad, d["b"][:1], d["c"][:1], d["x"][:1], d["s"][:1], d["y"][:1])
    e.close()


# ---------------------------------------------------------------------------
# split path (row-block × problem grids, conic_split_* kernels): forced with
# DOPT_CONIC_SPLIT=1 on the shapes above, and taken automatically for
# m > 1024 (several row blocks per problem, partial Aᵀ products reduced)
# ---------------------------------------------------------------------------
@pytest.fixture
def SplitConicBatch(ConicBatch, monkeypatch):
    monkeypatch.setenv("DOPT_CONIC_SPLIT", "1")
    return ConicBatch


def test_split_mixed_cones_batch(SplitConicBatch):
    # LSQR to maxiter on a singular M: 32–33 of 36 under the 1-ulp envelope bar
    # (r04: 33 with the fused split iteration's summation order)
    _synthetic_check(SplitConicBatch, 6, 30, [(0, 3), (1, 10), (3, 6), (2, 4), (4, 6)], 11,
                     "split: mixed cones", cap=34)


def test_split_well_posed_batch(SplitConicBatch):
    _synthetic_check(SplitConicBatch, 2, 100, [(3, 10)] * 20, 21, "split: well-posed SOC", cap=None, minnorm=True)


def test_split_psd_blocks_batch(SplitConicBatch):
    _synthetic_check(SplitConicBatch, 3, 25, [(4, 10), (4, 15), (1, 5)], 13, "split: PSD blocks", cap=18)


@pytest.mark.parametrize("shape", [
    ("split six-launch: well-posed SOC", 2, 100, [(3, 10)] * 20, 21, None),
    ("split six-launch: PSD blocks", 3, 25, [(4, 10), (4, 15), (1, 5)], 13, 18),
], ids=lambda s: s[0])
def test_split_six_launch_form(SplitConicBatch, monkeypatch, shape):
    """DOPT_SPLIT_FUSE=0: the six-launch split iteration (separate u / v
    update kernels) against the oracle, as the fused form is held above."""
    monkeypatch.setenv("DOPT_SPLIT_FUSE", "0")
    label, B, n, cones, seed, cap = shape
    _synthetic_check(SplitConicBatch, B, n, cones, seed, label, cap=cap, minnorm=cap is None)


def test_split_zero_rhs_gives_zero(SplitConicBatch):
    test_zero_rhs_gives_zero(SplitConicBatch)


def test_split_matches_persistent_kernel(ConicBatch, monkeypatch):
    # same problems through both LSQR drivers: identical algorithm, different
    # summation order of the A products → agreement to the oracle bar
    from diffopt_amd.synthetic import conic_numpy
    cones = [(3, 10)] * 20
    d = conic_numpy(3, 100, cones, 21)
    res = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("DOPT_CONIC_SPLIT", mode)
        e = ConicBatch(3, 100, cones)
        e.set(d["A"], d["b"], d["c"], d["x"], d["s"], d["y"])
        out, _ = e.forward(d["dA"], d["db"], d["dc"])
        g = e.reverse(d["dx"])[0]
        res[mode] = (np.asarray(out), np.asarray(g), e.iterations())
        e.close()
    assert relfro(res["1"][0], res["0"][0]) <= 1e-5
    assert relfro(res["1"][1], res["0"][1]) <= 1e-5


def test_config5_structure_multi_rowblock(ConicBatch):
    # config-5 structure (PSD(50) cones, m ≫ n) at oracle speed: 3 PSD(50)
    # → m = 3825 = 8 row blocks, auto split path
    _synthetic_check(ConicBatch, 2, 100, [(4, 1275)] * 3, 16, "config-5 structure, 3 cones", cap=None, minnorm=True)


# ---------------------------------------------------------------------------
# co-iterated forward + reverse (dopt_conic_forward_reverse, conic_lsqr2_kernel):
# one sweep over A per M / Mᵀ apply for both directions, per-direction stopping
# rules — bit-identical to the two separate calls, iteration counts included
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("shape", [
    ("mixed cones", 3, 30, [(0, 3), (1, 10), (3, 6), (2, 4), (4, 6)], 11),
    ("well-posed SOC", 2, 100, [(3, 10)] * 20, 21),
    ("config-4 bench shape", 2, 500, [(3, 25)] * 20, 14),
], ids=lambda s: s[0])
def test_forward_reverse_coiterated_bitwise(ConicBatch, shape):
    from diffopt_amd.synthetic import conic_numpy
    _, B, n, cones, seed = shape
    d = conic_numpy(B, n, cones, seed)
    e = ConicBatch(B, n, cones)
    e.set(d["A"], d["b"], d["c"], d["x"], d["s"], d["y"])
    out, fdx = e.forward(d["dA"], d["db"], d["dc"])
    it_f = e.iterations().copy()
    g, dA, db, dc = e.reverse(d["dx"])
    it_r = e.iterations().copy()
    (out2, fdx2), (g2, dA2, db2, dc2) = e.forward_reverse(d["dx"], d["dA"], d["db"], d["dc"])
    for a, b in [(out, out2), (fdx, fdx2), (g, g2), (dA, dA2), (db, db2), (dc, dc2)]:
        np.testing.assert_array_equal(np.asarray(a), np.asarray(b))
    st = e.lsqr_stats()
    np.testing.assert_array_equal(st["fwd_iterations"], it_f)
    np.testing.assert_array_equal(st["iterations"], it_r)
    e.close()


@pytest.mark.parametrize("shape", [
    ("split: mixed cones", 3, 30, [(0, 3), (1, 10), (3, 6), (2, 4), (4, 6)], 11),
    ("split: PSD blocks", 2, 25, [(4, 10), (4, 15), (1, 5)], 13),
], ids=lambda s: s[0])
def test_forward_reverse_coiterated_split_bitwise(SplitConicBatch, shape):
    """The split path (row-block × problem grids) co-iterated: 2B sequences,
    one pass over each row block of A for both live sequences."""
    test_forward_reverse_coiterated_bitwise(SplitConicBatch, shape)


# ---------------------------------------------------------------------------
# Capped LSQR on the istop-7 shapes: dopt_conic_set_maxiter
# against oracle/lsqr.py's maxiter at the same k, every output at the 1e-6 bar
# with no relaxed outputs.  tools/conic_capped_spread.py
# (profiles/r05/conic_capped_spread.txt) measured where the ORACLE's own
# iterate stops being reproducible: on these shapes the Golub–Kahan process
# exhausts its Krylov space after a few steps (β → rounding level), and from
# then on a 1-ulp change of the right-hand side moves the k-th iterate by
# ×≈30 per iteration — past 1e-6 from k = 6 (config-4 bench shape), 8 (mixed
# cones, SOC only) and 9 (PSD blocks, CSC shape).  The caps below sit before
# those thresholds, so the iteration arithmetic (M / Mᵀ applies, every Dπ
# branch, the plane rotations, the co-iteration) is pinned tightly on exactly
# the workloads whose converged outputs only meet the envelope bar.
# ---------------------------------------------------------------------------
CAPPED = [("config-4 bench shape", 2, 500, [(3, 25)] * 20, SEED0 + 4, False, (2, 5)),
          ("mixed cones", 3, 30, [(0, 3), (1, 10), (3, 6), (2, 4), (4, 6)], 11, False, (3, 7)),
          ("SOC only", 2, 40, [(3, 5)] * 8, 12, False, (3, 7)),
          ("PSD blocks", 3, 25, [(4, 10), (4, 15), (1, 5)], 13, False, (4, 8)),
          ("CSC shape", 3, 20, [(0, 3), (1, 10), (3, 6), (4, 6)], 31, True, (4, 8))]


@pytest.mark.parametrize("split", ["0", "1"])
@pytest.mark.parametrize("shape", CAPPED, ids=lambda s: s[0])
def test_capped_lsqr_istop7(ConicBatch, monkeypatch, shape, split):
    import scipy.sparse as sp
    from diffopt_amd.synthetic import conic_numpy
    name, B, n, cones, seed, csc, ks = shape
    monkeypatch.setenv("DOPT_CONIC_SPLIT", split)
    d = conic_numpy(B, n, cones, seed)
    A = d["A"].copy()
    if csc:
        A[:, :, 2] = 0.0
    worst = 0.0
    for k in ks:
        e = ConicBatch(B, n, cones)
        if csc:
            e.set_csc([sp.csc_matrix(a) for a in A], d["b"], d["c"], d["x"], d["s"], d["y"])
        else:
            e.set(A, d["b"], d["c"], d["x"], d["s"], d["y"])
        e.set_maxiter(k)
        (out, dx), (g, dA, db, dc) = e.forward_reverse(d["dx"], d["dA"], d["db"], d["dc"])
        st = e.lsqr_stats()
        e.close()
        for b in range(B):
            cache = ocn.Cache(A[b], d["b"][b], d["c"][b], d["x"][b], d["s"][b], d["y"][b], cones)
            (odx, du, dv, dw), fi = ocn.forward_differentiate(cache, d["dA"][b], d["db"][b], d["dc"][b],
                                                             return_info=True, maxiter=k)
            (og, _), ri = ocn.reverse_differentiate(cache, d["dx"][b], return_info=True, maxiter=k)
            odA, odb, odc = ocn.reverse_outputs(cache, og)
            ref = dict(fwd=np.concatenate([du, dv, [dw]]), dx=odx, g=og, dA=odA, db=odb, dc=odc)
            got = dict(fwd=np.asarray(out)[b], dx=np.asarray(dx)[b], g=np.asarray(g)[b],
                       dA=np.asarray(dA)[b], db=np.asarray(db)[b], dc=np.asarray(dc)[b])
            # the same number of iterations, stopped by the cap as the oracle
            assert (st["fwd_iterations"][b], st["fwd_istop"][b]) == (fi[0], fi[1]) == (k, 7), (b, fi)
            assert (st["iterations"][b], st["istop"][b]) == (ri[0], ri[1]) == (k, 7), (b, ri)
            for key, err in _errors(got, ref, cache).items():
                worst = max(worst, err)
                assert err <= RTOL, f"{name} k={k} problem {b} {key}: {err:.3e}"
    log = os.environ.get("DOPT_PARITY_LOG")
    if log:
        with open(log, "a") as f:
            f.write(json.dumps(dict(test=f"capped LSQR: {name} (split={split})", ks=list(ks), worst=worst)) + "\n")


def test_split_batch_slices_bitwise(SplitConicBatch):
    """The fused split LSQR runs a batch as two slices on two streams (round 5):
    a batch of 3 (slices of 2 and 1 problems) gives bit for bit the outputs and
    iteration counts of each problem solved alone (batch 1, one slice)."""
    from diffopt_amd.synthetic import conic_numpy
    cones = [(4, 10), (4, 15), (1, 5)]
    B, n = 3, 25
    d = conic_numpy(B, n, cones, 13)
    e = SplitConicBatch(B, n, cones)
    e.set(d["A"], d["b"], d["c"], d["x"], d["s"], d["y"])
    (out, fdx), (g, dA, db, dc) = e.forward_reverse(d["dx"], d["dA"], d["db"], d["dc"])
    st = e.lsqr_stats()
    e.close()
    for b in range(B):
        e1 = SplitConicBatch(1, n, cones)
        e1.set(*[d[k][b:b + 1] for k in ("A", "b", "c", "x", "s", "y")])
        (o1, f1), (g1, a1, b1, c1) = e1.forward_reverse(d["dx"][b:b + 1], d["dA"][b:b + 1], d["db"][b:b + 1],
                                                        d["dc"][b:b + 1])
        s1 = e1.lsqr_stats()
        e1.close()
        for x, y in [(out, o1), (fdx, f1), (g, g1), (dA, a1), (db, b1), (dc, c1)]:
            np.testing.assert_array_equal(np.asarray(x)[b], np.asarray(y)[0])
        for k in ("istop", "iterations", "fwd_istop", "fwd_iterations"):
            assert st[k][b] == s1[k][0], (b, k)
