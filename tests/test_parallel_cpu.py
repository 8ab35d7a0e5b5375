"""Batch-sharded multi-process path on CPU (gloo): shard ranges, the one
all-gather of packed sensitivities, ragged splits.  The per-shard solve is
the oracle (test-side checker standing in for the GPU engine, which the
`-m gpu` tests cover); the product's sharding/gather code is what is tested:
gathered results must be bit-identical to the single-process oracle run."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from diffopt_amd import parallel
from diffopt_amd.synthetic import qp_numpy
from oracle import qp as oqp


def test_shard_ranges_cover_batch_contiguously():
    for total in (0, 1, 7, 1024, 8192, 8193):
        for world in (1, 2, 3, 4, 8):
            rs = [parallel.shard(total, world, r) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == total
            for (a, b), (c, d) in zip(rs, rs[1:]):
                assert b == c and b >= a
            sz = parallel.shard_sizes(total, world)
            assert max(sz) - min(sz) <= 1
    with pytest.raises(ValueError):
        parallel.shard(10, 2, 2)


class _OracleEngine:
    """Test stand-in with the QPBatch interface, backed by the CPU oracle."""

    def __init__(self, batch):
        self.batch = batch

    def set(self, Q, G, h, A, z, lam, nu):
        self.args = (Q, G, h, A, z, lam, nu)

    def forward_reverse(self, dl_dz, dQ=None, dq=None, dG=None, dh=None, dA=None, db=None):
        rev, fwd = [], []
        for b in range(self.batch):
            a = [x[b] for x in self.args]
            rev.append(np.concatenate(oqp.reverse_differentiate(*a, dl_dz[b])))
            fwd.append(np.concatenate(oqp.forward_differentiate(
                *a, dq=None if dq is None else dq[b], dh=None if dh is None else dh[b],
                db=None if db is None else db[b])))
        return np.stack(rev), np.stack(fwd)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, total, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        d = qp_numpy(total, 12, 18, 3, 0.3, 77)
        rev, fwd = parallel.sharded_forward_reverse(_OracleEngine, d, total)
        q.put((rank, rev.numpy(), fwd.numpy()))
    finally:
        dist.destroy_process_group()


def _run(world, total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    d = qp_numpy(total, 12, 18, 3, 0.3, 77)
    ref_r, ref_f = _OracleEngine(total), None
    ref_r.set(*[d[k] for k in ["Q", "G", "h", "A", "z", "lam", "nu"]])
    R, F = ref_r.forward_reverse(d["dl_dz"], dq=d["dq"], dh=d["dh"], db=d["db"])
    for _, rev, fwd in res:
        assert rev.shape == R.shape
        assert np.array_equal(rev, R) and np.array_equal(fwd, F)


def test_gloo_world2_even_split():
    _run(2, 6)


def test_gloo_world3_ragged_split():
    _run(3, 7)


def _pipeline_worker(rank, world, port, steps, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rows, width = 3, 5
        pipe = parallel.GatherPipeline(rows, width, torch.float64, "cpu")
        got = {}
        for k in range(steps):
            buf = pipe.next_buffer()
            buf.copy_(torch.full((rows, width), 100.0 * k + rank, dtype=torch.float64)
                      + torch.arange(rows * width, dtype=torch.float64).reshape(rows, width))
            pipe.submit()
            if k >= 1:      # the previous step's gather may complete under this step
                got[k - 1] = pipe.result(k - 1).clone()
        pipe.drain()
        got[steps - 1] = pipe.result(steps - 1).clone()
        q.put((rank, {k: v.numpy() for k, v in got.items()}))
    finally:
        dist.destroy_process_group()


def test_gloo_gather_pipeline_world2():
    """GatherPipeline (bench.py's overlapped all-gather): every step's
    gathered rows are exactly the ranks' packed rows in rank order, with two
    gathers in flight and the buffers reused."""
    world, steps = 2, 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_pipeline_worker, args=(r, world, port, steps, q))
          for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    base = np.arange(15, dtype=np.float64).reshape(3, 5)
    for _, got in res:
        assert sorted(got) == list(range(steps))
        for k, v in got.items():
            ref = np.concatenate([base + 100.0 * k + r for r in range(world)])
            assert np.array_equal(v, ref)
