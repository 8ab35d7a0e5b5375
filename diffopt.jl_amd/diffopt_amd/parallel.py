"""Batch sharding across GPUs.

Independent KKT systems: rank r of G owns the contiguous problem range
``shard(B, G, r)``; assembly, factorisation and both solves run locally with
no collective in the data path.  The only exchange is one all-gather of the
packed per-problem sensitivities ``[rev | fwd]`` (RCCL over xGMI with the
``nccl`` backend on ROCm; ``gloo`` on CPU for the tests).  Ragged splits
(B not divisible by G) are padded to the largest shard for the collective
and trimmed afterwards.
"""

import torch


def shard(total, world, rank):
    """Contiguous [start, stop) of `total` problems for `rank` of `world`
    (the first total % world ranks get one extra problem)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of world {world}")
    base, extra = divmod(int(total), int(world))
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def shard_sizes(total, world):
    return [shard(total, world, r)[1] - shard(total, world, r)[0] for r in range(world)]


def pack(out_rev, out_fwd, into=None):
    """(B, L) reverse + (B, L) forward → (B, 2L) contiguous rows."""
    L = out_rev.shape[1]
    if into is None:
        into = torch.empty(out_rev.shape[0], 2 * L, dtype=out_rev.dtype, device=out_rev.device)
    into[:, :L].copy_(out_rev)
    into[:, L:].copy_(out_fwd)
    return into


def all_gather_rows(local, total, group=None):
    """All-gather the rows of every rank's `local` (its shard of `total`
    problems, in rank order) → (total, …) on every rank.  One collective."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    sizes = shard_sizes(total, world)
    rank = dist.get_rank(group)
    if local.shape[0] != sizes[rank]:
        raise ValueError(f"rank {rank} holds {local.shape[0]} rows, shard is {sizes[rank]}")
    mx = max(sizes)
    tail = tuple(local.shape[1:])
    if all(s == mx for s in sizes):
        out = torch.empty((total,) + tail, dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(out, local.contiguous(), group=group)
        return out
    padded = torch.zeros((mx,) + tail, dtype=local.dtype, device=local.device)
    padded[: local.shape[0]].copy_(local)
    buf = torch.empty((world * mx,) + tail, dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(buf, padded, group=group)
    return torch.cat([buf[r * mx: r * mx + sizes[r]] for r in range(world)], dim=0)


class GatherPipeline:
    """All-gather of per-step packed sensitivities, overlapped with the next
    step's compute (for streams of independent batches).

    Two packed buffers alternate: `next_buffer()` returns the buffer to pack
    step k into (first waiting for the gather that last read it, two steps
    ago), `submit()` starts the asynchronous all-gather of it and returns at
    once, `drain()` waits for every gather in flight.  With the ``nccl``
    backend (RCCL) the waits order torch's current stream after the
    collective without blocking the host, so step k's gather over xGMI runs
    under step k+1's kernels.  Even shards only (every rank `rows` rows).
    `result(k)` is the gathered (world·rows, width) tensor of step k once it
    has completed (the two most recent steps are kept).
    """

    def __init__(self, rows, width, dtype, device, group=None):
        import torch.distributed as dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.bufs = [torch.empty(rows, width, dtype=dtype, device=device) for _ in range(2)]
        self.outs = [torch.empty(self.world * rows, width, dtype=dtype, device=device)
                     for _ in range(2)]
        self.work = [None, None]
        self.step = 0

    def next_buffer(self):
        i = self.step & 1
        if self.work[i] is not None:
            self.work[i].wait()
            self.work[i] = None
        return self.bufs[i]

    def submit(self):
        import torch.distributed as dist
        i = self.step & 1
        self.work[i] = dist.all_gather_into_tensor(self.outs[i], self.bufs[i], group=self.group,
                                                   async_op=True)
        self.step += 1

    def drain(self):
        for i in range(2):
            if self.work[i] is not None:
                self.work[i].wait()
                self.work[i] = None

    def result(self, k):
        if k < self.step - 2 or k >= self.step:
            raise IndexError(f"step {k} is not among the last two submitted")
        if self.work[k & 1] is not None:
            self.work[k & 1].wait()
            self.work[k & 1] = None
        return self.outs[k & 1]


def sharded_forward_reverse(engine_factory, data, total, group=None):
    """Run one batch-sharded fwd+rev sensitivity solve.

    `data` maps QP input names ("Q", "G", "h", "A", "z", "lam", "nu",
    "dl_dz", "dq", "dh", "db", optional "dQ", "dG", "dA") to FULL-batch
    arrays (leading dim `total`) or to this rank's shard already (leading dim
    = shard size).  `engine_factory(batch)` returns an object with
    `set(Q, G, h, A, z, lam, nu)` and `forward_reverse(dl_dz, dQ=…, …)` (a
    `diffopt_amd.qp.QPBatch`).  Returns the gathered (total, L) reverse and
    forward sensitivities on every rank.
    """
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    lo, hi = shard(total, world, rank)

    def local(x):
        if x is None:
            return None
        return x[lo:hi] if x.shape[0] == total and hi - lo != total else x

    d = {k: local(v) for k, v in data.items()}
    eng = engine_factory(hi - lo)
    eng.set(d["Q"], d.get("G"), d.get("h"), d.get("A"), d["z"], d.get("lam"), d.get("nu"))
    rev, fwd = eng.forward_reverse(d["dl_dz"], dQ=d.get("dQ"), dq=d.get("dq"), dG=d.get("dG"),
                                   dh=d.get("dh"), dA=d.get("dA"), db=d.get("db"))
    rev_t, fwd_t = torch.as_tensor(rev), torch.as_tensor(fwd)
    packed = pack(rev_t, fwd_t)
    full = all_gather_rows(packed, total, group)
    L = rev_t.shape[1]
    return full[:, :L], full[:, L:]
