#!/usr/bin/env python3
"""bench.py — KKT sensitivity solves/sec (forward + reverse) on batched dense QPs.

Workload: N = 1 (no torchrun) — BASELINE.json configs[1] = config 2: a batch
of 1024 dense QPs, n = 200 variables, m = 300 inequalities (p = 0), 30 %
active.  N > 1 (torchrun) — configs[2] = config 3, the north_star headline:
n = 1000, m = 1500, 1024 problems per rank (8192 on 8 GPUs).  Synthetic
(seeded, KKT point by construction — SURVEY.md §8(d)), inputs resident in HBM
before the timed region.  One step = for every problem of the batch: KKT
assembly + LU factorisation + reverse solve (dl/dz → dz, dλ, dν) + forward
solve (dq, dh → dz, dλ, dν) — the reference refactorises per call; the engine
factors once per step and reuses it for both directions.  N > 1: one process
per GPU, problems sharded (weak scaling), plus one RCCL all-gather of the
packed sensitivities per step (§8(e)).  `--lam-eps 1e-9` gives the inactive
rows tiny non-zero duals (interior-point-like: no exact elimination, N' = n+m).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...   (driver, N > 1)

Prints ONE JSON line on rank 0 (the driver's contract), with `roofline`
(dominant kernel, timed live with HIP events on the engine's stream) and
`cpu_baseline` (the oracle restatement timed on the host's cores).
"""

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "diffopt.jl_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

PEAK_FP64_TFLOPS = 78.6     # MI355X FP64 matrix/vector dense (spec; probe measured 75.4)
PEAK_HBM_GBS = 8000.0       # MI355X HBM3E spec (MI355X_MICROARCH.md)
QP_CFG = {2: dict(id=2, n=200, m=300, p=0, phi=0.3, batch=1024),
          3: dict(id=3, n=1000, m=1500, p=0, phi=0.3, batch=1024)}
# conic configs (BASELINE.json configs[3], [4]); batch = problems per GPU
# (config 5: 64 SDPs over 4 GPUs = 16 per GPU)
CONIC_CFG = {4: dict(batch=512), 5: dict(batch=16)}
# NLP back-end (§8(f)4; not a BASELINE config — no published number): 1024
# problems, 200 primal variables, 100 constraints (40 ≥, 30 ≤, 30 =), 20
# parameters, 50 % / 30 % of the variables bounded below / above → M of
# about 600 rows
NLP_CFG = {6: dict(batch=1024, n=200, c=100, P=20)}
NLP_KEYS = ["Hxx", "Hxp", "Jx", "Jp", "x", "cval", "crhs", "y", "xl", "xu", "yl", "yu"]
# the sparse route (sparse.hip, §8 beyond BASELINE — VERDICT r05 missing 2;
# no published number): 7 — sparse LPs (Q = 0, the reference's LSQR branch)
# above the dense route's n + m + p <= 8192 cap, ≈ 5 entries per row; 8 —
# sparse conic programs (A_moi kept sparse, every cone code, m <= n)
SPARSE_CFG = {7: dict(batch=256, n=4000, p=100, m_extra=1000, k=5),
              8: dict(batch=256, n=3000, k=5,
                      cones=[(0, 10), (3, 20)] * 50 + [(1, 1000)] + [(4, 21)] * 4 + [(2, 216)])}


def host_cores():
    """(usable, machine) host CPUs: `usable` is what this process may actually
    run on — its affinity mask, capped by a cgroup-v2 CPU quota when one is
    set (the GPU box gives each one-GPU job a share of a larger machine, and
    os.cpu_count() reports the whole machine) — `machine` is os.cpu_count().
    SURVEY.md §8(d): the CPU baseline runs on all usable host cores."""
    machine = os.cpu_count() or 1
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = machine
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            usable = min(usable, max(1, math.ceil(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    return usable, machine


def cpu_workers(args):
    return args.cpu_workers or host_cores()[0]


# --------------------------------------------------------------------------
# CPU baseline: the oracle restatement of the reference algorithm (sparse LU of
# the full KKT via SuperLU, re-factorised for reverse and for forward exactly
# as QuadraticProgram.jl:490 does), one process per core.
# --------------------------------------------------------------------------
def _cpu_worker(args):
    cfg, seed, seconds = args
    os.environ["OPENBLAS_NUM_THREADS"] = "1"
    from diffopt_amd.synthetic import qp_numpy
    from oracle import qp as oqp
    d = qp_numpy(1, cfg["n"], cfg["m"], cfg["p"], cfg["phi"], seed, lam_eps=cfg.get("lam_eps", 0.0))
    a = [d[k][0] for k in ["Q", "G", "h", "A", "z", "lam", "nu"]]
    n_done = 0
    t0 = time.perf_counter()
    while True:
        oqp.reverse_differentiate(*a, d["dl_dz"][0], sparse=True)
        oqp.forward_differentiate(*a, dq=d["dq"][0], dh=d["dh"][0], sparse=True)
        n_done += 1
        if time.perf_counter() - t0 >= seconds:
            break
    return n_done, time.perf_counter() - t0


def cpu_baseline(cfg, seconds, workers):
    import multiprocessing as mp
    ctx = mp.get_context("fork")
    t0 = time.perf_counter()
    with ctx.Pool(workers) as pool:
        res = pool.map(_cpu_worker, [(cfg, 1000 + i, seconds) for i in range(workers)])
    wall = time.perf_counter() - t0
    solves = sum(r[0] for r in res)
    rate = sum(r[0] / r[1] for r in res)
    return dict(value=round(rate, 2), unit="solves/s", cores=workers, machine_cpus=host_cores()[1], kind="port",
                sample=(f"{solves} config-{cfg.get('id', 2)} QP solves (n={cfg['n']}, m={cfg['m']}, fwd+rev, "
                        f"SuperLU re-factorised per direction) on {workers} processes "
                        f"× {seconds:.0f} s (wall {wall:.1f} s)"))


def _nlp_cpu_worker(args):
    cfg, seed, seconds = args
    os.environ["OPENBLAS_NUM_THREADS"] = "1"
    from diffopt_amd.synthetic import nlp_numpy
    from oracle import nlp as onlp
    st, pt, dp, dx, dd = nlp_numpy(2, cfg["n"], cfg["c"], cfg["P"], seed)
    n_done = 0
    t0 = time.perf_counter()
    while True:
        b = n_done % 2
        a = [pt[k][b] for k in NLP_KEYS]
        sk = (st["con_kind"], st["has_low"], st["has_up"], st["sense"])
        # forward_differentiate! and reverse_differentiate! each recompute ∂s
        # (NonLinearProgram.jl:516, 536): two factorisations per fwd+rev
        ds, L, *_ = onlp.compute_sensitivity(*sk, *a, return_info=True)
        onlp.forward(ds, L, dp[b])
        ds, L, *_ = onlp.compute_sensitivity(*sk, *a, return_info=True)
        onlp.reverse(ds, L, dx[b], dd[b])
        n_done += 1
        if time.perf_counter() - t0 >= seconds:
            break
    return n_done, time.perf_counter() - t0


def run_nlp(args, world, rank, local_rank):
    """NLP KKT sensitivities (config 6): one step = for every problem the sIpopt
    KKT assembly, LU with the inertia-correction check, forward (Δp → Δx,
    Δdual) and reverse (Δx, Δdual → Δp) solves."""
    cfg = dict(NLP_CFG[args.config])
    B = args.batch or cfg["batch"]
    n, c, P = cfg["n"], cfg["c"], cfg["P"]
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        import multiprocessing as mp
        workers = cpu_workers(args)
        t0 = time.perf_counter()
        with mp.get_context("fork").Pool(workers) as pool:
            res = pool.map(_nlp_cpu_worker, [(cfg, 3000 + i, args.cpu_seconds) for i in range(workers)])
        wall = time.perf_counter() - t0
        cpu = dict(value=round(sum(r[0] / r[1] for r in res), 2), unit="solves/s", cores=workers,
                   machine_cpus=host_cores()[1], kind="port",
                   sample=(f"{sum(r[0] for r in res)} config-6 NLP solves (n={n}, c={c}, P={P}; ∂s recomputed "
                           f"per direction with SuperLU, as the reference) on {workers} processes × "
                           f"{args.cpu_seconds:.0f} s (wall {wall:.1f} s)"))
    import numpy as np
    import torch
    torch.cuda.set_device(local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local_rank))
    from diffopt_amd.nlp import NLPBatch
    from diffopt_amd.synthetic import SEED0, nlp_numpy
    st, pt, dp, dx, dd = nlp_numpy(B, n, c, P, SEED0 + args.config + 7919 * rank)
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a), device="cuda")
    # the deferred factor return (opt-in, dopt_nlp_set_deferred): the inputs are
    # device tensors that stay untouched across the step, as its contract asks
    eng = NLPBatch(B, n, c, P, device=local_rank, deferred=True)
    eng.set_structure(st["con_kind"], st["has_low"], st["has_up"], st["sense"])
    eng.set(*[t(pt[k]) for k in NLP_KEYS])
    dp_t, dx_t, dd_t = t(dp), t(dx), t(dd)
    rows = eng.layout()["rows"]

    def step():
        eng.factor()
        if args.nlp_separate:   # the reference's two calls: forward_differentiate!, reverse_differentiate!
            eng.forward(dp_t)
            eng.reverse(dx_t, dd_t)
        else:
            eng.forward_reverse(dp_t, dx_t, dd_t)   # forward + reverse, one pass over the factors for both

    for _ in range(args.warmup):
        step()
    breakdown, name = _phase_breakdown(eng, step, 3)
    eng.phase_times()
    eng.set_profiling(True, phases=[name])
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    eng.set_profiling(False)
    phases = eng.phase_times()
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    corr = eng.corrections()
    kinds = eng.lu_kind()
    sizes = eng.system_size().astype(np.float64)   # R (n + c) on the reduced route, M's rows on the full one
    if rank == 0:
        ms_tot, cnt = phases[name]   # live, over the timed region
        avg_s = ms_tot / cnt / 1e3
        if name in ("qp_lu", "qp_lu_pivot"):
            work = float((2.0 / 3.0 * sizes ** 3).sum())   # the general (non-symmetric) LU of each factorised system
            achieved = work / avg_s / 1e12
            roof = dict(bound="mfma", achieved=round(achieved, 3), peak=PEAK_FP64_TFLOPS, unit="TFLOP/s",
                        frac=round(achieved / PEAK_FP64_TFLOPS, 4))
        else:
            work = float((8.0 * sizes * sizes).sum())   # one read of the factors
            achieved = work / avg_s / 1e9
            roof = dict(bound="hbm", achieved=round(achieved, 1), peak=PEAK_HBM_GBS, unit="GB/s",
                        frac=round(achieved / PEAK_HBM_GBS, 4))
        roof["kernel"] = name.replace("qp_", "nlp_")
        roof["traffic"] = _load_pmc(name + "@cfg6")
        roof["avg_launch_ms"] = round(avg_s * 1e3, 4)
        roof["phases_ms_per_step"] = {k.replace("qp_", "nlp_"): v for k, v in breakdown.items()}
        line = {
            "metric": "NLP KKT sensitivity solves/sec (fwd+rev)"
                      + (" [separate forward and reverse calls]" if args.nlp_separate else ""),
            "value": round(world * B * args.steps / elapsed, 1),
            "unit": "solves/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded strictly complementary NLP KKT point, diffopt_amd.synthetic.nlp_numpy)",
            "config": {"workload": "config 6: NLP KKT batch (sIpopt system + inertia correction), fwd+rev",
                       "problems_per_gpu": B, "n": n, "constraints": c, "params": P, "kkt_rows": rows,
                       "factorised_size_mean": round(float(sizes.mean()), 1),
                       "inertia_corrections": int((corr != 0).sum()),
                       "deferred_factor": True,
                       "factorisation": {"no_pivot": int((kinds == 1).sum()),
                                         "partial_pivoting": int((kinds == 2).sum())},
                       "parallelism": f"batch-sharded x{world}"},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


def _conic_gen(variant):
    from diffopt_amd import synthetic
    return synthetic.conic_numpy_wellcond if variant == "wellcond" else synthetic.conic_numpy


def _conic_cpu_worker(args):
    cfg, seed, seconds, variant = args
    os.environ["OPENBLAS_NUM_THREADS"] = "1"
    import numpy as np
    from diffopt_amd.synthetic import CONIC_CONFIGS
    from oracle import conic as ocn
    c = CONIC_CONFIGS[cfg]
    d = _conic_gen(variant)(1, c["n"], c["cones"], seed)
    t0 = time.perf_counter()
    cache = ocn.Cache(d["A"][0], d["b"][0], d["c"][0], d["x"][0], d["s"][0], d["y"][0], c["cones"])
    t_cache = time.perf_counter() - t0
    if cfg == 4:
        n_done = 0
        t0 = time.perf_counter()
        while True:
            ocn.Cache(d["A"][0], d["b"][0], d["c"][0], d["x"][0], d["s"][0], d["y"][0], c["cones"])
            ocn.forward_differentiate(cache, db=d["db"][0], dc=d["dc"][0])
            ocn.reverse_differentiate(cache, d["dx"][0])
            n_done += 1
            if time.perf_counter() - t0 >= seconds:
                break
        return n_done, time.perf_counter() - t0, None
    # config 5: one full solve is minutes of CPU; time LSQR iterations (one
    # matvec + one rmatvec each) for `seconds` and extrapolate with the
    # iteration counts the engine reports
    v = d["db"][0].copy()
    z = np.concatenate([d["dc"][0], d["db"][0], [1.0]])
    k = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        cache.rmatvec(cache.matvec(z))
        k += 1
    t_it = (time.perf_counter() - t0) / k
    return k, t_cache, t_it


def conic_cpu_samples(cfg, seconds, workers, variant="bench"):
    import multiprocessing as mp
    ctx = mp.get_context("fork")
    t0 = time.perf_counter()
    with ctx.Pool(workers) as pool:
        res = pool.map(_conic_cpu_worker, [(cfg, 1000 + i, seconds, variant) for i in range(workers)])
    return res, time.perf_counter() - t0, workers


def conic_cpu_baseline(cfg, seconds, samples, iters_per_solve, variant="bench"):
    res, wall, workers = samples
    if cfg == 4:
        solves = sum(r[0] for r in res)
        rate = sum(r[0] / r[1] for r in res)
        sample = (f"{solves} config-4{' converging-variant' if variant == 'wellcond' else ''} SOCP solves "
                  f"(n=500, 20 SOC(25), Dπ + fwd LSQR + rev LSQR, "
                  f"IterativeSolvers defaults) on {workers} processes × {seconds:.0f} s "
                  f"(wall {wall:.1f} s)")
    else:
        per = [r[1] + iters_per_solve * r[2] for r in res]
        rate = sum(1.0 / t for t in per)
        sample = (f"config-5 SDP (n=500, 10 PSD(50), m=12750): Dπ build timed once and "
                  f"{sum(r[0] for r in res)} LSQR iterations (M·v + Mᵀ·u) timed for "
                  f"{seconds:.0f} s per process on {workers} processes, extrapolated to the "
                  f"engine's {iters_per_solve:.0f} fwd+rev iterations per solve (wall {wall:.1f} s)")
    return dict(value=round(rate, 3), unit="solves/s", cores=workers, machine_cpus=host_cores()[1], kind="port",
                sample=sample)


def make_conic_step(eng, dev, gather, B):
    """One bench step of the conic configs on `eng` (a ConicBatch holding this
    rank's B problems; `dev` its device tensors dx / db / dc): Dπ, the
    co-iterated forward + reverse LSQR, and with `gather` (world > 1) one RCCL
    all-gather of the packed [forward | reverse] solutions of all problems of
    the process group.
    Returns (forward, reverse, gathered or None).  Module level so that
    tests/test_parallel_gpu.py runs this exact step under a world-1 nccl
    group."""
    import torch
    N = eng.N
    packed = torch.empty(B, 2 * N, dtype=torch.float64, device="cuda") if gather else None

    def step():
        eng.factor()                                   # v, π(v), Dπ per cone
        # both directions in one call: the two LSQR runs co-iterated, one sweep
        # over A per M / Mᵀ apply for both (dopt_conic_forward_reverse)
        (fo, fdx), (g, _, rdb, rdc) = eng.forward_reverse(dev["dx"], db=dev["db"], dc=dev["dc"],
                                                          want_dA=False)
        gathered = None
        if packed is not None:
            from diffopt_amd import parallel
            packed[:, :N].copy_(fo)
            packed[:, N:].copy_(g)
            gathered = parallel.all_gather_rows(packed, _group_size() * B)
        return fo, g, gathered
    return step


def run_conic(args, world, rank, local_rank):
    """Configs 4/5: batched conic sensitivities (cone Dπ + forward LSQR +
    reverse LSQR per problem), roofline on the LSQR kernel's algorithmic HBM
    bytes."""
    import numpy as np
    import torch
    from diffopt_amd.conic import ConicBatch
    from diffopt_amd.synthetic import CONIC_CONFIGS, SEED0
    c = CONIC_CONFIGS[args.config]
    variant = args.conic_variant
    if variant == "wellcond" and args.config != 4:
        raise SystemExit("--conic-variant wellcond is defined for config 4 (SOC cones)")
    n, cones = c["n"], c["cones"]
    B = args.batch or CONIC_CFG[args.config]["batch"]
    m = sum(dim for _, dim in cones)
    # the CPU baseline forks worker processes: run it before this process
    # initialises HIP (config 5 extrapolates with the engine's iteration
    # counts, a host computation done after the GPU run)
    cpu_raw = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        workers = cpu_workers(args)
        cpu_raw = conic_cpu_samples(args.config, args.cpu_seconds, workers, variant)
    torch.cuda.set_device(local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", rank=rank, world_size=world,
                                device_id=torch.device("cuda", local_rank))
    d = _conic_gen(variant)(B, n, cones, SEED0 + args.config + 7919 * rank)
    dev = {k: torch.from_numpy(d[k]).cuda() for k in ["A", "b", "c", "x", "s", "y", "dx", "db", "dc"]}
    del d
    eng = ConicBatch(B, n, cones, device=local_rank)
    eng.set(dev["A"], dev["b"], dev["c"], dev["x"], dev["s"], dev["y"])
    step = make_conic_step(eng, dev, world > 1, B)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # iteration counts (deterministic for fixed inputs) for the byte count
    eng.forward_reverse(dev["dx"], db=dev["db"], dc=dev["dc"], want_dA=False)
    stats = eng.lsqr_stats()
    it_f = stats["fwd_iterations"].astype(np.float64)
    it_r = stats["iterations"].astype(np.float64)
    torch.cuda.synchronize()
    eng.phase_times()
    eng.set_profiling(True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    eng.set_profiling(False)
    phases = eng.phase_times()
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    if rank == 0:
        cpu = None
        if cpu_raw is not None:
            cpu = conic_cpu_baseline(args.config, args.cpu_seconds, cpu_raw,
                                     float(it_f.mean() + it_r.mean()), variant)
        plen = 0
        for code, dim in cones:
            if code in (1, 2):
                plen += dim
            elif code == 3:
                plen += 4
            elif code == 4:
                dd = int((math.isqrt(8 * dim + 1) - 1) // 2)
                plen += 2 * dd * dd + 2
        # algorithmic HBM bytes per LSQR iteration: two passes over A (M·v and
        # Mᵀ·u are sequentially dependent; each pass serves both A· and Aᵀ·),
        # the structured Dπ parameters, and the N-vectors
        b_it = 16.0 * m * n + 8.0 * (plen + 4 * (n + m))
        ms_tot, cnt = phases["conic_lsqr"]
        avg_s = ms_tot / cnt / 1e3
        if cnt == args.steps:
            # one co-iterated launch per step: while both directions run, each
            # pair of sweeps over A serves both; the vectors are per direction
            b_vec = 8.0 * (plen + 4 * (n + m))
            per_launch = float((16.0 * m * n * np.maximum(it_f, it_r)).sum() + b_vec * (it_f + it_r).sum())
        else:   # split path: one launch per direction
            per_launch = b_it * float(it_f.sum() + it_r.sum()) / 2.0
        achieved = per_launch / avg_s / 1e9
        roof = dict(bound="hbm", achieved=round(achieved, 1), peak=PEAK_HBM_GBS, unit="GB/s",
                    frac=round(achieved / PEAK_HBM_GBS, 4),
                    traffic=_load_pmc(("conic_lsqr_split" if args.config == 5 else "conic_lsqr")
                                      + ("@wellcond" if variant == "wellcond" else "")),
                    kernel="conic_lsqr", avg_launch_ms=round(avg_s * 1e3, 4),
                    bytes_per_iteration=b_it,
                    lsqr_iterations_mean={"forward": float(it_f.mean()), "reverse": float(it_r.mean())},
                    lsqr_istop={"forward": {str(k): int(v) for k, v in zip(*np.unique(stats["fwd_istop"], return_counts=True))},
                                "reverse": {str(k): int(v) for k, v in zip(*np.unique(stats["istop"], return_counts=True))}},
                    phases_ms_per_step={k: round(v[0] / args.steps, 4) for k, v in sorted(phases.items())})
        value = world * B * args.steps / elapsed
        print(json.dumps({
            "metric": "KKT sensitivity solves/sec (fwd+rev) on batched conic programs",
            "value": round(value, 3), "unit": "solves/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": ("synthetic (seeded complementary cone pairs by construction, SURVEY.md §8(d))" if variant == "bench"
                     else "synthetic converging variant (diffopt_amd.synthetic.conic_numpy_wellcond: well-conditioned "
                          "A, interior / dual-interior / boundary SOC pairs)"),
            "config": {"workload": f"config {args.config}: " + ("SOCP batch, 20 SOC(25)" if args.config == 4
                                                                  else "SDP batch, 10 PSD(50)")
                       + (" — converging variant (LSQR istop 1-2)" if variant == "wellcond" else ""),
                       "problems_per_gpu": B, "n": n, "m_rows": m,
                       "parallelism": f"batch-sharded x{world}" + (" + RCCL all-gather" if world > 1 else "")},
            "roofline": roof, "cpu_baseline": cpu}), flush=True)
    if dist:
        dist.destroy_process_group()



def _sparse_cpu(cfg_id, seconds):
    """CPU baseline of the sparse configs: the oracle's restatement (scipy CSC
    LHS / matrix-free M + the IterativeSolvers LSQR restatement) on one core,
    problems of the same generator until ≈ `seconds` have passed."""
    import numpy as np
    from diffopt_amd import synthetic as syn
    from oracle import qp as oqp
    c = SPARSE_CFG[cfg_id]
    t0, done = time.perf_counter(), 0
    while time.perf_counter() - t0 < seconds or done == 0:
        if cfg_id == 7:
            d = syn.lp_sparse_numpy(1, c["n"], c["p"], c["m_extra"], c["k"], 9000 + done)
            oqp.lp_sparse_differentiate(d["G"][0], d["h"][0], d["A"][0], d["z"][0], d["lam"][0], d["nu"][0],
                                        d["dl_dz"][0], d["dq"][0], d["dh"][0], d["db"][0])
        else:
            from oracle import conic as ocn
            d = syn.conic_numpy_wellcond(1, c["n"], c["cones"], 9000 + done, pair_norm=1.0, sparse_k=c["k"])
            cache = ocn.Cache(d["A"][0], d["b"][0], d["c"][0], d["x"][0], d["s"][0], d["y"][0], c["cones"])
            ocn.forward_differentiate(cache, None, d["db"][0], d["dc"][0])
            ocn.reverse_differentiate(cache, d["dx"][0])
        done += 1
    el = time.perf_counter() - t0
    return dict(value=round(done / el, 3), unit="solves/s", cores=1, kind="port",
                sample=f"{done} problems of the config's generator, one core, {el:.1f} s")


def run_sparse(args, world, rank, local_rank):
    """Configs 7 / 8: the sparse route (sparse.hip; conic.hip's sparse LSQR).
    One step = forward + reverse of every problem, LSQR on the matrix-free KKT
    LHS / M from the CSC and CSR copies.  Roofline: HBM, on the algorithmic
    bytes of the LSQR iterations actually run (the entries once per product
    role, index + value, the N-vectors) — DESIGN.md §4."""
    import numpy as np
    import torch
    c = SPARSE_CFG[args.config]
    B = args.batch or c["batch"]
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = _sparse_cpu(args.config, min(args.cpu_seconds, 20.0))
    torch.cuda.set_device(local_rank)
    from diffopt_amd import synthetic as syn
    seed = SEED0_SPARSE + args.config + 7919 * rank
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a), device="cuda")
    if args.config == 7:
        from diffopt_amd.qp import QPBatch
        import scipy.sparse as sp
        n, p = c["n"], c["p"]
        d = syn.lp_sparse_numpy(B, n, p, c["m_extra"], c["k"], seed)
        m = d["lam"].shape[1]
        N = n + m + p
        eng = QPBatch(B, n, m, p, device=local_rank)
        eng.set_csc([sp.csc_matrix((n, n))] * B, d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
        nnz = float(sum(g.nnz for g in d["G"]) + sum(a.nnz for a in d["A"])) / B
        dl, dq, dh, db = t(d["dl_dz"]), t(d["dq"]), t(d["dh"]), t(d["db"])
        step = lambda: eng.forward_reverse(dl, dq=dq, dh=dh, db=db)
        phase = "qp_lsqr"
        # per LSQR iteration: two products, each reading every entry of G and A
        # in both of its LHS roles (CSC for the z rows, CSR for the λ / ν rows:
        # 12 B index + value), s and λ, the operand and result vectors; then
        # the LSQR vector updates (≈ 16 N-vector passes)
        b_it = 2.0 * (12.0 * 2.0 * nnz + 16.0 * m + 16.0 * N) + 8.0 * 16.0 * N
        workload = (f"config 7: sparse LP batch (Q = 0, LSQR branch) above the dense cap, n={n}, m={m}, p={p}, "
                    f"~{c['k']} entries per row")
    else:
        from diffopt_amd.conic import ConicBatch
        n, cones = c["n"], c["cones"]
        d = syn.conic_numpy_wellcond(B, n, cones, seed, pair_norm=1.0, sparse_k=c["k"], sparse_out=True)
        m = sum(dim for _, dim in cones)
        N = n + m + 1
        eng = ConicBatch(B, n, cones, device=local_rank, sparse=True)
        eng.set_csc(d["A"], d["b"], d["c"], d["x"], d["s"], d["y"])
        nnz = float(sum(a.nnz for a in d["A"])) / B
        dx, db, dc = t(d["dx"]), t(d["db"]), t(d["dc"])
        step = lambda: eng.forward_reverse(dx, db=db, dc=dc, want_dA=False)
        phase = "conic_lsqr"
        plen = 0
        for code, dim in cones:
            if code in (1, 2):
                plen += dim
            elif code == 3:
                plen += 4
            elif code == 4:
                dd = int((math.isqrt(8 * dim + 1) - 1) // 2)
                plen += 2 * dd * dd + 2
        # two M / Mᵀ applies per iteration, each reading A_moi's entries as CSR
        # (A·) and as CSC (Aᵀ·), plus Dπ's parameters and the N-vectors
        b_it = 48.0 * nnz + 8.0 * (plen + 4 * (n + m))
        workload = f"config 8: sparse conic batch (A_moi kept sparse, every cone code), n={n}, m={m}, ~{c['k']} per row"
    del d
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if args.config == 7:
        st = eng.lsqr_stats()
        it_f, it_r = st[:, 1, 1].astype(np.float64), st[:, 0, 1].astype(np.float64)
    else:
        st = eng.lsqr_stats()
        it_f, it_r = st["fwd_iterations"].astype(np.float64), st["iterations"].astype(np.float64)
    eng.phase_times()
    eng.set_profiling(True, phases=[phase])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    eng.set_profiling(False)
    ms_tot, cnt = eng.phase_times()[phase]
    if rank == 0:
        avg_s = ms_tot / cnt / 1e3
        per_step = b_it * float((it_f + it_r).sum())
        achieved = per_step / (ms_tot / 1e3 / args.steps) / 1e9
        roof = dict(bound="hbm", achieved=round(achieved, 1), peak=PEAK_HBM_GBS, unit="GB/s",
                    frac=round(achieved / PEAK_HBM_GBS, 4), traffic=_load_pmc(f"{phase}@cfg{args.config}"),
                    kernel=phase,
                    avg_launch_ms=round(avg_s * 1e3, 4), bytes_per_iteration=b_it, nnz_per_problem=nnz,
                    lsqr_iterations_mean={"forward": float(it_f.mean()), "reverse": float(it_r.mean())})
        print(json.dumps({
            "metric": "KKT sensitivity solves/sec (fwd+rev), sparse route",
            "value": round(world * B * args.steps / elapsed, 3), "unit": "solves/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (seeded, diffopt_amd.synthetic: lp_sparse_numpy / conic_numpy_wellcond sparse_k)",
            "config": {"workload": workload, "problems_per_gpu": B, "N": N, "parallelism": f"batch-sharded x{world}"},
            "roofline": roof, "cpu_baseline": cpu}), flush=True)


SEED0_SPARSE = 20250307


def _phase_breakdown(eng, step, nsteps, drain=None):
    """Per-phase GPU ms per step from an untimed pass with every phase's HIP
    events on, and the dominant phase.  The timed region then records events
    around that phase only: each event pair costs a few microseconds of queue
    time between launches, which the other phases need not add to the clock."""
    import torch
    torch.cuda.synchronize()
    eng.phase_times()                      # reset accumulators
    eng.set_profiling(True)
    for _ in range(nsteps):
        step()
    if drain is not None:
        drain()
    torch.cuda.synchronize()
    eng.set_profiling(False)
    ph = eng.phase_times()
    dom = max(ph.items(), key=lambda kv: kv[1][0])[0]
    return {k: round(v[0] / nsteps, 4) for k, v in sorted(ph.items())}, dom

def _load_pmc(kernel):
    """HBM bytes/launch for `kernel` from the committed rocprofv3 --pmc summary
    (tools/pmc_summary.py → profiles/pmc_latest.json), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_latest.json")
    try:
        with open(path) as f:
            return json.load(f)["kernels"][kernel]["hbm_bytes_per_launch"]
    except Exception:
        return None


def _group_size():
    import torch.distributed as dist
    return dist.get_world_size()


def make_qp_step(eng, d, out_rev, out_fwd, gather, B, pipe=None):
    """One bench step of the QP configs on `eng` (a QPBatch holding this
    rank's B problems; `d` its device tensors): assembly, LU, both solves and
    outputs into out_rev / out_fwd, then with `gather` (world > 1) one RCCL
    all-gather of the packed [rev | fwd] rows of every rank's problems —
    overlapped through `pipe`
    (parallel.GatherPipeline; the result is pipe.result(k)) or blocking.
    Returns the gathered tensor of a blocking gather, else None.  Module level
    so that tests/test_parallel_gpu.py runs this exact step under a world-1
    nccl group."""
    import torch
    from diffopt_amd import parallel
    p = eng.p
    L = out_rev.shape[1]
    packed = torch.empty(B, 2 * L, dtype=torch.float64, device="cuda") if gather and pipe is None else None

    def step():
        eng.forward_reverse(d["dl_dz"], dq=d["dq"], dh=d["dh"], db=d["db"] if p else None,
                            out_rev=out_rev, out_fwd=out_fwd)
        if gather:
            # weak scaling: every rank owns B problems of the world·B batch;
            # one RCCL all-gather of the packed [rev | fwd] sensitivities per
            # step, overlapped with the next step's kernels (GatherPipeline;
            # every gather completes inside the timed region: drain() below)
            if pipe is not None:
                parallel.pack(out_rev, out_fwd, into=pipe.next_buffer())
                pipe.submit()
            else:
                parallel.pack(out_rev, out_fwd, into=packed)
                return parallel.all_gather_rows(packed, _group_size() * B)
        return None
    return step


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=None,
                    choices=sorted(QP_CFG) + sorted(CONIC_CFG) + sorted(NLP_CFG) + sorted(SPARSE_CFG),
                    help="default: 2 at N = 1, 3 (the north_star headline) under torchrun")
    ap.add_argument("--lam-eps", type=float, default=0.0,
                    help="QP: inactive rows get λ = LAM_EPS instead of 0 (no exact elimination)")
    ap.add_argument("--batch", type=int, default=None, help="problems per GPU")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-workers", type=int, default=None,
                    help="CPU-baseline processes (default: every usable host core, host_cores())")
    ap.add_argument("--conic-variant", choices=["bench", "wellcond"], default="bench",
                    help="config 4: the bench generator (LSQR stops at maxiter) or the converging variant")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--nlp-separate", action="store_true",
                    help="config 6: time dopt_nlp_forward and dopt_nlp_reverse as two calls (the reference's "
                         "pattern) instead of the fused dopt_nlp_forward_reverse")
    ap.add_argument("--no-allgather", action="store_true")
    ap.add_argument("--sync-allgather", action="store_true",
                    help="N > 1: blocking all-gather per step instead of the overlapped pipeline")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.config is None:
        args.config = 3 if world > 1 else 2
    if args.config in CONIC_CFG:
        return run_conic(args, world, rank, local_rank)
    if args.config in NLP_CFG:
        return run_nlp(args, world, rank, local_rank)
    if args.config in SPARSE_CFG:
        return run_sparse(args, world, rank, local_rank)
    cfg = dict(QP_CFG[args.config])
    cfg["lam_eps"] = args.lam_eps
    if args.batch:
        cfg["batch"] = args.batch
    B, n, m, p = cfg["batch"], cfg["n"], cfg["m"], cfg["p"]

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        workers = cpu_workers(args)
        cpu = cpu_baseline(cfg, args.cpu_seconds, workers)

    import numpy as np
    import torch
    torch.cuda.set_device(local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", rank=rank, world_size=world,
                                device_id=torch.device("cuda", local_rank))
    from diffopt_amd.qp import QPBatch
    from diffopt_amd.synthetic import SEED0, qp_torch

    d = qp_torch(B, n, m, p, cfg["phi"], SEED0 + args.config, rank_offset=rank, lam_eps=args.lam_eps)
    eng = QPBatch(B, n, m, p, device=local_rank)
    eng.set(d["Q"], d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
    L = n + m + p
    out_rev = torch.empty(B, L, dtype=torch.float64, device="cuda")
    out_fwd = torch.empty(B, L, dtype=torch.float64, device="cuda")
    gathered = None
    pipe = None
    if world > 1 and not args.no_allgather:
        from diffopt_amd import parallel
        gathered = True
        if not args.sync_allgather:
            pipe = parallel.GatherPipeline(B, 2 * L, torch.float64, "cuda")

    step = make_qp_step(eng, d, out_rev, out_fwd, gathered is not None, B, pipe)

    for _ in range(args.warmup):
        step()
    if pipe is not None:
        pipe.drain()
    torch.cuda.synchronize()
    sizes = eng.system_size()
    kinds = eng.lu_kind()
    symr = eng.sym_route()
    breakdown, name = _phase_breakdown(eng, step, 3, pipe.drain if pipe is not None else None)
    eng.phase_times()                      # reset accumulators
    eng.set_profiling(True, phases=[name])
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if pipe is not None:
        pipe.drain()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    eng.set_profiling(False)
    phases = eng.phase_times()
    elapsed = t1 - t0
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    if (eng.info() != 0).any():
        raise RuntimeError("singular KKT in the benchmark batch")

    if rank == 0:
        # dominant kernel and its roofline (algorithmic work per launch ÷ avg
        # launch time measured with HIP events on the engine's stream)
        ms_tot, cnt = phases[name]   # live, over the timed region
        avg_s = ms_tot / cnt / 1e3
        Ns = sizes.astype("float64")
        if name in ("qp_lu", "qp_lu_pivot"):
            # flops the shipped factorisation does: N'³/3 per problem on the
            # P-symmetric route (lower trailing tiles, U from L), 2N'³/3 on the
            # general one; the general LU's (2/3)·N'³ reported beside it
            work = float(np.where(symr == 1, 1.0 / 3.0, 2.0 / 3.0) @ (Ns ** 3))
            work_lu = float((2.0 / 3.0 * Ns ** 3).sum())
            achieved = work / avg_s / 1e12
            roof = dict(bound="mfma", achieved=round(achieved, 3), peak=PEAK_FP64_TFLOPS,
                        unit="TFLOP/s", frac=round(achieved / PEAK_FP64_TFLOPS, 4),
                        flops_per_launch=work, achieved_at_lu_flops=round(work_lu / avg_s / 1e12, 3))
        else:
            if name == "qp_solve":
                # both directions' backward sweeps (the forward sweeps run
                # inside the no-pivot LU): each reads half of K, 8·N'² together
                work = float((8.0 * Ns ** 2).sum())
            elif name == "qp_assemble":
                work = float(B * 8.0 * (n * n + 2 * m * n) + (8.0 * Ns ** 2).sum())
            else:
                work = float(B * 8.0 * (m * n + 2 * L))
            achieved = work / avg_s / 1e9
            roof = dict(bound="hbm", achieved=round(achieved, 1), peak=PEAK_HBM_GBS,
                        unit="GB/s", frac=round(achieved / PEAK_HBM_GBS, 4))
        roof["kernel"] = name
        # PMC bytes per launch measured for this workload (profiles/pmc_latest.json:
        # config 2 unsuffixed, others @cfgN, the --lam-eps worst case @lam), or null
        pkey = name if args.config == 2 else f"{name}@cfg{args.config}"
        roof["traffic"] = _load_pmc(pkey + "@lam" if args.lam_eps > 0 else pkey)
        roof["avg_launch_ms"] = round(avg_s * 1e3, 4)
        roof["phases_ms_per_step"] = breakdown   # untimed pass (_phase_breakdown)
        # the whole step against SURVEY §8(d)'s roofline t_roof = max(B/BW, F/P):
        # B = the algorithmic bytes of a solve (inputs once, both outputs),
        # F = the flops the shipped algorithm does (N'³/3 on the P-symmetric
        # route, 2N'³/3 otherwise; the reference's full-KKT LU beside it)
        b_step = B * 8.0 * (n * n + m * n + p * n + 4 * L + m + n)
        f_step = float(np.where(symr == 1, 1.0 / 3.0, 2.0 / 3.0) @ (Ns ** 3))
        f_ref = B * (2.0 / 3.0 * L ** 3 + 4.0 * L ** 2 + 4.0 * m * n)
        t_hbm, t_fp = b_step / (PEAK_HBM_GBS * 1e9), f_step / (PEAK_FP64_TFLOPS * 1e12)
        ms_step = elapsed / args.steps
        roof["step"] = dict(t_roof_ms=round(1e3 * max(t_hbm, t_fp), 4), hbm_ms=round(1e3 * t_hbm, 4),
                            fp64_ms=round(1e3 * t_fp, 4), bytes=b_step, flops=f_step,
                            frac=round(max(t_hbm, t_fp) / ms_step, 4),
                            reference_flops=f_ref, fp64_ms_at_reference_flops=round(1e3 * f_ref / (PEAK_FP64_TFLOPS * 1e12), 4))
        value = world * B * args.steps / elapsed
        line = {
            "metric": "KKT sensitivity solves/sec (fwd+rev) on batched QPs",
            "value": round(value, 1),
            "unit": "solves/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded KKT point by construction, SURVEY.md §8(d))",
            "config": {"workload": f"config {args.config}: dense QP batch, fwd+rev sensitivities",
                       "problems_per_gpu": B, "n": n, "m_ineq": m, "p_eq": p,
                       "active_fraction": cfg["phi"],
                       "reduced_kkt_size_mean": round(float(Ns.mean()), 1),
                       "inactive_dual": args.lam_eps,
                       "factorisation": {"no_pivot": int((kinds == 1).sum()),
                                         "no_pivot_p_symmetric": int((symr == 1).sum()),
                                         "partial_pivoting": int((kinds == 2).sum())},
                       "parallelism": f"batch-sharded x{world}" + ((" + RCCL all-gather" + (" (overlapped)" if pipe is not None else "")) if gathered is not None else "")},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
