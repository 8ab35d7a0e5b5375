"""The multi-GPU path's collective on the GPU box: the RCCL (`nccl` backend)
all-gather of packed sensitivities that the HIP engine produced, as bench.py
runs it under torchrun, here as a world-size-1 group on one MI355X (the
driver runs the 8-rank case; tests/test_parallel_cpu.py covers world 2/3 with
gloo).  Gathered rows must be bit-identical to the engine's outputs."""

import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def nccl_group():
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    yield dist
    dist.destroy_process_group()


def test_engine_outputs_through_rccl_gather(nccl_group):
    import torch
    from diffopt_amd import parallel
    from diffopt_amd.qp import QPBatch
    from diffopt_amd.synthetic import qp_torch
    B, n, m, p = 64, 40, 60, 0
    e = QPBatch(B, n, m, p)
    L = n + m + p
    pipe = parallel.GatherPipeline(B, 2 * L, torch.float64, "cuda")
    outs = []
    for k in range(3):   # three steps of distinct problems through the overlapped gather
        d = qp_torch(B, n, m, p, 0.3, 1234 + k)
        e.set(d["Q"], d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
        rev, fwd = e.forward_reverse(d["dl_dz"], dq=d["dq"], dh=d["dh"])
        parallel.pack(rev, fwd, into=pipe.next_buffer())
        pipe.submit()
        outs.append(torch.cat([rev, fwd], 1).clone())
        if k >= 1:
            assert torch.equal(pipe.result(k - 1), outs[k - 1])
    pipe.drain()
    torch.cuda.synchronize()
    assert torch.equal(pipe.result(2), outs[2])
    # the blocking form (bench.py --sync-allgather)
    g = parallel.all_gather_rows(outs[2], B)
    assert torch.equal(g, outs[2])
    e.close()


def test_sharded_forward_reverse_on_engine(nccl_group):
    """parallel.sharded_forward_reverse with the HIP engine as the per-shard
    solver: the gathered rows equal a direct engine call."""
    import torch
    from diffopt_amd import parallel
    from diffopt_amd.qp import QPBatch
    from diffopt_amd.synthetic import qp_torch
    B, n, m, p = 32, 30, 40, 4
    d = qp_torch(B, n, m, p, 0.3, 99)
    rev, fwd = parallel.sharded_forward_reverse(lambda b: QPBatch(b, n, m, p), d, B)
    e = QPBatch(B, n, m, p)
    e.set(d["Q"], d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
    r2, f2 = e.forward_reverse(d["dl_dz"], dq=d.get("dq"), dh=d.get("dh"), db=d.get("db"))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(rev.cpu().numpy(), r2.cpu().numpy())
    np.testing.assert_array_equal(fwd.cpu().numpy(), f2.cpu().numpy())
