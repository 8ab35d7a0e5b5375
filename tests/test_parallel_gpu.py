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


def _bench():
    import importlib
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if root not in sys.path:
        sys.path.insert(0, root)
    return importlib.import_module("bench")


@pytest.mark.parametrize("overlapped", [True, False], ids=["pipeline", "blocking"])
def test_bench_qp_step_config3_shape(nccl_group, overlapped):
    """bench.py's QP step (make_qp_step — the function the driver's torchrun
    scaling run executes) at config 3's shape (n = 1000, m = 1500, 4
    problems) with its RCCL gather switched on under the group: the gathered
    [rev | fwd] rows are bit-identical to the engine's outputs, with the
    overlapped GatherPipeline and with the blocking gather."""
    import torch
    from diffopt_amd import parallel
    from diffopt_amd.qp import QPBatch
    from diffopt_amd.synthetic import SEED0, qp_torch
    bench = _bench()
    B, n, m, p = 4, 1000, 1500, 0
    d = qp_torch(B, n, m, p, 0.3, SEED0 + 3)
    eng = QPBatch(B, n, m, p)
    eng.set(d["Q"], d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
    L = n + m + p
    out_rev = torch.empty(B, L, dtype=torch.float64, device="cuda")
    out_fwd = torch.empty(B, L, dtype=torch.float64, device="cuda")
    world = nccl_group.get_world_size()
    pipe = parallel.GatherPipeline(B, 2 * L, torch.float64, "cuda") if overlapped else None
    step = bench.make_qp_step(eng, d, out_rev, out_fwd, True, B, pipe)
    for k in range(2):
        g = step()
        want = torch.cat([out_rev, out_fwd], 1).clone()
        got = pipe.result(k) if overlapped else g
        torch.cuda.synchronize()
        assert got.shape == (world * B, 2 * L)
        assert torch.equal(got, want)
    if pipe is not None:
        pipe.drain()
    assert (eng.info() == 0).all()
    eng.close()


def test_bench_conic_step_config5_shape(nccl_group):
    """bench.py's conic step (make_conic_step, bench.py:run_conic under
    torchrun — config 5 is specified on 4 GPUs) at config 5's full problem
    shape (10 × PSD(50), n = 500, m = 12 750; 2 problems: the split LSQR path,
    co-iterated) with the RCCL gather on: the gathered [forward | reverse]
    rows are bit-identical to the engine's outputs, and equal to a separate
    dopt_conic_forward_reverse call on the same data."""
    import torch
    from diffopt_amd.conic import ConicBatch
    from diffopt_amd.synthetic import CONIC_CONFIGS, SEED0, conic_numpy
    bench = _bench()
    c = CONIC_CONFIGS[5]
    B, n, cones = 2, c["n"], c["cones"]
    d = conic_numpy(B, n, cones, SEED0 + 5)
    dev = {k: torch.from_numpy(d[k]).cuda() for k in ["A", "b", "c", "x", "s", "y", "dx", "db", "dc"]}
    eng = ConicBatch(B, n, cones)
    eng.set(dev["A"], dev["b"], dev["c"], dev["x"], dev["s"], dev["y"])
    step = bench.make_conic_step(eng, dev, True, B)
    fo, g, gathered = step()
    fo, g = fo.clone(), g.clone()
    torch.cuda.synchronize()
    N = eng.N
    assert gathered.shape == (nccl_group.get_world_size() * B, 2 * N)
    assert torch.equal(gathered[:, :N], fo) and torch.equal(gathered[:, N:], g)
    (fo2, _), (g2, *_r) = eng.forward_reverse(dev["dx"], db=dev["db"], dc=dev["dc"], want_dA=False)
    torch.cuda.synchronize()
    assert torch.equal(fo2, fo) and torch.equal(g2, g)
    st = eng.lsqr_stats()
    assert (st["fwd_iterations"] > 0).all() and (st["iterations"] > 0).all()
    eng.close()
