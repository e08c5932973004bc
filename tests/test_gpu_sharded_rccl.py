"""The sharded path on the real backend: a world-1 "nccl" (= RCCL) process
group on the GPU box's one MI355X, with the HIP kernel as the local reduce.

World 1 is the most RCCL allows on one device (it rejects two ranks on the
same GPU); the multi-rank collective logic is covered by
tests/test_sharded_gloo.py and the 8-GPU run belongs to the driver. What this
adds: every collective the sharded entry points issue (all-gather,
all-to-all, reduce-scatter, the size all-reduce) runs through RCCL on device
tensors, and the results match the C oracle (exact paths bit for bit)."""
from __future__ import annotations

import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.fixture(scope="module")
def rccl_world1():
    assert torch.cuda.is_available()
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    yield
    dist.destroy_process_group()


def _expect(xs, w32, dtype):
    from oracle import oracle as orc
    if dtype == torch.float64:
        return torch.from_numpy(orc.wreduce([x.cpu().numpy() for x in xs], np.asarray(w32, np.float64), "f64"))
    if dtype in (torch.bfloat16, torch.float16):
        code = "bf16" if dtype == torch.bfloat16 else "f16"
        rows = [x.cpu().view(torch.int16).numpy().view(np.uint16) for x in xs]
        return torch.from_numpy(orc.wreduce(rows, w32, code).view(np.int16).copy()).view(dtype)
    return torch.from_numpy(orc.wreduce([x.cpu().numpy() for x in xs], w32, "f32"))


def _same(a, b):
    a, b = a.cpu(), b.cpu()
    if a.dtype in (torch.bfloat16, torch.float16):
        return torch.equal(a.view(torch.int16), b.view(torch.int16))
    if a.dtype != b.dtype:
        return False
    return torch.equal(a.view(torch.int64 if a.dtype == torch.float64 else torch.int32),
                       b.view(torch.int64 if b.dtype == torch.float64 else torch.int32))


@pytest.mark.parametrize("n,p,dtype", [(5, 100_003, torch.float32), (8, 1_048_577, torch.float32),
                                       (3, 50_001, torch.bfloat16), (4, 40_003, torch.float64)])
def test_sharded_entry_points_rccl(rccl_world1, n, p, dtype):
    from dasklearn_amd.sharded import ShardedAggregator
    from oracle import oracle as orc

    assert dist.get_backend() == "nccl"
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(11 + n)
    xs = [(torch.randn(p, generator=g, device=dev) * 0.05).to(dtype) for _ in range(n)]
    weights = [float(w) for w in np.random.default_rng(n).dirichlet(np.ones(n))]
    f64 = dtype == torch.float64  # the Python floats stay exact (fedavg.py:25)
    w32 = orc.reference_weights_f64(n, weights) if f64 else orc.reference_weights(n, weights)
    expect = _expect(xs, w32, dtype)

    agg = ShardedAggregator()  # HIP kernel as the local reduce
    b, e = agg.bounds(p)
    assert (b, e) == (0, p)
    assert _same(agg.aggregate_param_sharded([x[b:e] for x in xs], weights, p), expect)
    assert _same(agg.aggregate_param_sharded([x[b:e] for x in xs], weights, p, gather=False), expect)
    # whole models on "different ranks" (all on rank 0 here): all-to-all, exact fold, all-gather
    assert _same(agg.aggregate_model_sharded(xs, [n], weights, exact=True), expect)
    # FAST: partial sums + reduce-scatter + all-gather, tolerance only
    fast = agg.aggregate_model_sharded(xs, [n], weights, exact=False).cpu().double()
    scale = sum(abs(float(w)) * x.cpu().double().abs() for w, x in zip(w32, xs))
    ulp = {torch.bfloat16: 2.0 ** -8, torch.float64: 2.0 ** -52}.get(dtype, 2.0 ** -23)
    assert torch.all((fast - expect.double()).abs() <= (n + 2) * ulp * scale + 1e-300)
    # uniform weights (fedavg.py:14-15)
    wu = orc.reference_weights_f64(n, None) if f64 else orc.reference_weights(n, None)
    assert _same(agg.aggregate_param_sharded(xs, None, p), _expect(xs, wu, dtype))


@pytest.mark.parametrize("n,p,dtype", [(4, 70_001, torch.float32), (3, 50_001, torch.bfloat16),
                                       (5, 30_003, torch.float16), (3, 20_001, torch.float64)])
def test_c_abi_sharded_entry_on_torch_rccl_comm(rccl_world1, n, p, dtype):
    """dlsim_wreduce_sharded driven directly on the process group's own RCCL
    communicator (ProcessGroupNCCL._comm_ptr, RCCL bound from torch/lib):
    gather and no-gather, bit-identical to the oracle."""
    from dasklearn_amd import _native
    from dasklearn_amd.sharded import ShardedAggregator
    from oracle import oracle as orc

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(5 + n)
    xs = [(torch.randn(p, generator=g, device=dev) * 0.05).to(dtype) for _ in range(n)]
    w32 = orc.reference_weights_f64(n, None) if dtype == torch.float64 else orc.reference_weights(n, None)
    expect = _expect(xs, w32, dtype)
    agg = ShardedAggregator()
    comm = agg._rccl_comm(dev)
    assert comm is not None  # the ABI path is the one aggregate_param_sharded takes here
    for gather in (True, False, "allgather"):
        out = torch.full((p,), float("nan"), dtype=dtype, device=dev)
        _native.wreduce_sharded(xs, w32, out, comm, gather=gather)
        assert _same(out, expect)
    # a plan on the real communicator (agreed once; world 1 runs no gather)
    for gather in ("bcast", "allgather"):
        plan = _native.ShardedPlan(comm, p, n, dtype, gather, device=dev)
        for _ in range(3):
            out = torch.full((p,), float("nan"), dtype=dtype, device=dev)
            plan.run(xs, w32, out)
            assert _same(out, expect)
        plan.close()
    # through ShardedAggregator.plan (the C plan on this group's communicator)
    pl = agg.plan(p, n, dtype)
    assert pl._c is not None
    assert _same(pl.run(xs, None), expect)  # uniform weights, as w32
    pl.close()
    # a null communicator and a slice length that is not this rank's shard are
    # argument errors, not launches
    assert _native.load().dlsim_wreduce_sharded(None, 0, 0, None, None, 0, 0, 0, None, 0, None) == -1
    with pytest.raises(_native.DlsimError, match="shard"):
        _native.wreduce_sharded([x[:p - 1] for x in xs], w32, torch.empty(p, dtype=dtype, device=dev), comm)
