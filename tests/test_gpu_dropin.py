"""The drop-in boundary on the GPU: FedAvg.aggregate / ModelManager /
functions.aggregate with nn.Modules, as dasklearn/worker.py would call them
(worker.py:27-31 -> functions.py:89-106 -> model_manager.py:41-43 ->
fedavg.py:12-26)."""
from __future__ import annotations

import copy
import os

import numpy as np
import pytest
import torch
from torch import nn

from conftest import GOLDEN, golden_paths, load_golden
from oracle import oracle as orc
from oracle import fedavg_torch

pytestmark = pytest.mark.gpu

from dasklearn_amd import functions  # noqa: E402
from dasklearn_amd.gradient_aggregation import GradientAggregationMethod  # noqa: E402
from dasklearn_amd.gradient_aggregation.fedavg import FedAvg  # noqa: E402
from dasklearn_amd.model_manager import ModelManager  # noqa: E402


class Ragged(nn.Module):
    def __init__(self, shapes, dtype=torch.float32):
        super().__init__()
        self.ps = nn.ParameterList([nn.Parameter(torch.zeros(*s, dtype=dtype)) for s in shapes])


def modules_from_golden(g):
    meta = g["meta"]
    dt = {"bf16": torch.bfloat16, "f16": torch.float16, "f64": torch.float64}.get(meta["dtype"], torch.float32)
    models = []
    for row in g["inputs"]:
        m = Ragged(meta["shapes"], dt)
        off = 0
        with torch.no_grad():
            for p in m.parameters():
                k = p.numel()
                src = row[off:off + k]
                if meta["dtype"] in ("bf16", "f16"):
                    t = torch.from_numpy(src.view(np.int16).copy()).view(dt)
                else:
                    t = torch.from_numpy(src.copy())
                p.copy_(t.view_as(p))
                off += k
        models.append(m)
    return models


def flat_of(model):
    t = torch.cat([p.detach().reshape(-1).cpu() for p in model.parameters()])
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().view(np.uint16)
    return t.numpy()


class Settings:
    gradient_aggregation = GradientAggregationMethod.FEDAVG
    torch_threads = 4


@pytest.mark.parametrize("path", [p for p in golden_paths() if "buffers" not in p],
                         ids=lambda p: os.path.basename(p)[:-4])
def test_fedavg_modules_match_reference_golden(path):
    g = load_golden(path)
    models = modules_from_golden(g)
    out = FedAvg.aggregate(models, g["weights_arg"])
    assert type(out) is type(models[0])
    assert all(not p.is_cuda for p in out.parameters())  # host in -> host out
    assert orc.same_bits(flat_of(out), g["expected"]), g["meta"]["case"]


def test_buffers_carried_over_from_model0():
    g = load_golden(os.path.join(GOLDEN, "buffers_bn_f32_n3_none.npz"))

    class WithBN(nn.Module):
        def __init__(self):
            super().__init__()
            self.lin = nn.Linear(7, 5)
            self.bn = nn.BatchNorm1d(5)

    models = []
    buf_off = 0
    for i, row in enumerate(g["inputs"]):
        m = WithBN()
        off = 0
        with torch.no_grad():
            for p in m.parameters():
                p.copy_(torch.from_numpy(row[off:off + p.numel()].copy()).view_as(p))
                off += p.numel()
            if i == 0:
                for b in m.buffers():
                    k = b.numel()
                    b.copy_(torch.from_numpy(g["buffers0"][buf_off:buf_off + k]).view_as(b).to(b.dtype))
                    buf_off += k
            else:
                m.bn.running_mean.fill_(100.0 + i)  # must NOT leak into the output
        models.append(m)
    out = FedAvg.aggregate(models, None)
    assert orc.same_bits(flat_of(out), g["expected"])
    got_bufs = np.concatenate([b.detach().reshape(-1).double().numpy() for b in out.buffers()])
    assert np.array_equal(got_bufs, g["expected_buffers"])
    assert [p.requires_grad for p in out.parameters()] == list(g["expected_requires_grad"])
    # inputs untouched (the reference only reads them)
    assert float(models[1].bn.running_mean[0]) == 101.0


def test_fedavg_device_resident_models_zero_copy():
    """CUDA models in, CUDA model out; an output fed back in is an arena (one launch, no packing)."""
    torch.manual_seed(1)
    d = torch.device("cuda", 0)
    models = [nn.Sequential(nn.Linear(64, 32), nn.ReLU(), nn.Linear(32, 10)).to(d) for _ in range(4)]
    out = FedAvg.aggregate(models, [0.1, 0.2, 0.3, 0.4])
    assert all(p.is_cuda for p in out.parameters())
    ref = fedavg_torch.aggregate_modules([copy.deepcopy(m).cpu() for m in models], [0.1, 0.2, 0.3, 0.4])
    assert orc.same_bits(flat_of(out), flat_of(ref))
    # second round: outputs (arena-backed) as inputs
    out2 = FedAvg.aggregate([out, out, models[0]], None)
    ref2 = fedavg_torch.aggregate_modules([copy.deepcopy(out).cpu(), copy.deepcopy(out).cpu(),
                                           copy.deepcopy(models[0]).cpu()], None)
    assert orc.same_bits(flat_of(out2), flat_of(ref2))


def test_mixed_dtype_module_groups():
    torch.manual_seed(2)

    class Mixed(nn.Module):
        def __init__(self):
            super().__init__()
            self.a = nn.Parameter(torch.randn(1001))
            self.b = nn.Parameter(torch.randn(333).to(torch.bfloat16))
            self.c = nn.Parameter(torch.randn(17))

    models = [Mixed() for _ in range(3)]
    out = FedAvg.aggregate(models, [0.5, 0.25, 0.25])
    ref = fedavg_torch.aggregate_modules(models, [0.5, 0.25, 0.25])
    for p, q in zip(out.parameters(), ref.parameters()):
        assert p.dtype == q.dtype
        a = p.detach().cpu()
        b = q.detach()
        if a.dtype == torch.bfloat16:
            assert torch.equal(a.view(torch.int16), b.view(torch.int16))
        else:
            assert orc.same_bits(a.numpy(), b.numpy())


def test_errors_match_reference():
    m = [Ragged([[4]]), Ragged([[4]])]
    with pytest.raises(AssertionError):
        FedAvg.aggregate(m, [0.5])
    with pytest.raises(IndexError):
        FedAvg.aggregate([], None)


def test_model_manager_and_task_function():
    g = load_golden(os.path.join(GOLDEN, "cfg1_gnlenet_f32_n2_none.npz"))
    models = modules_from_golden(g)
    mm = ModelManager(None, Settings(), 0)
    for i, m in enumerate(models):
        mm.process_incoming_trained_model(i, m)
    mm.process_incoming_trained_model(0, models[1])  # duplicate id ignored (model_manager.py:28-30)
    assert orc.same_bits(flat_of(mm.aggregate_trained_models()), g["expected"])

    res = functions.aggregate(Settings(), {"models": models, "round": 1, "peer": 0})
    assert isinstance(res, list) and len(res) == 1
    assert orc.same_bits(flat_of(res[0]), g["expected"])
    res = functions.aggregate(Settings(), {"models": models, "round": 1, "peer": None,
                                           "weights": [0.25, 0.75]})
    exp = orc.wreduce(list(g["inputs"]), orc.reference_weights(2, [0.25, 0.75]), "f32")
    assert orc.same_bits(flat_of(res[0]), exp)


def test_device_resident_option_keeps_result_on_gpu():
    """settings.aggregate_on_device (opt-in): host models in, GPU module out;
    same bits as the host result."""
    g = load_golden(os.path.join(GOLDEN, "cfg1_gnlenet_f32_n2_none.npz"))
    models = modules_from_golden(g)

    class OnDevice(Settings):
        aggregate_on_device = True

    res = functions.aggregate(OnDevice(), {"models": models, "round": 1, "peer": 0})
    assert all(p.is_cuda for p in res[0].parameters())
    assert orc.same_bits(flat_of(res[0]), g["expected"])


def test_host_result_placement_and_stage_timing_works():
    """Host models -> host result: in page-locked memory (round 4: the D2H is
    asynchronous and the output module is built meanwhile; the call returns a
    complete result), small and large; under DLSIM_HOST_RESULT=pageable's
    rule (arena.HOST_RESULT_PINNED False) a small result comes back in
    pageable memory. All exact, the timed variant too."""
    from dasklearn_amd import _native, arena
    from dasklearn_amd.arena import aggregate_modules
    g = load_golden(os.path.join(GOLDEN, "cfg1_gnlenet_f32_n2_none.npz"))
    models = modules_from_golden(g)
    stages = {}
    out = aggregate_modules(models, None, _native.DLSIM_EXACT, timing=stages)
    assert set(stages) >= {"layout", "pipeline", "module"}  # the D2H is part of the pipeline
    assert orc.same_bits(flat_of(out), g["expected"])
    for _ in range(3):  # the deferred wait: read right after the call returns
        out = aggregate_modules(models, None, _native.DLSIM_EXACT)
        p0 = next(out.parameters())
        assert not p0.is_cuda and p0.is_pinned()
        assert orc.same_bits(flat_of(out), g["expected"])
    saved = arena.HOST_RESULT_PINNED
    arena.HOST_RESULT_PINNED = False
    try:
        out = aggregate_modules(models, None, _native.DLSIM_EXACT)
        assert not next(out.parameters()).is_pinned()  # 341 KB < PAGEABLE_RESULT_BYTES
        assert orc.same_bits(flat_of(out), g["expected"])
    finally:
        arena.HOST_RESULT_PINNED = saved
    # past the page-locked budget small results come back pageable,
    # device-model results copied to the host too; exact either way
    saved_budget = arena.PINNED_RESULT_BUDGET
    arena.PINNED_RESULT_BUDGET = 0
    arena.PINNED_BUDGET.calls = 0  # re-read the allocator's statistics now
    try:
        out = aggregate_modules(models, None, _native.DLSIM_EXACT)
        assert not next(out.parameters()).is_pinned()
        assert orc.same_bits(flat_of(out), g["expected"])
        dev_models = [m.cuda() for m in modules_from_golden(g)]
        out = aggregate_modules(dev_models, None, _native.DLSIM_EXACT, to_host=True)
        assert not next(out.parameters()).is_cuda and not next(out.parameters()).is_pinned()
        assert orc.same_bits(flat_of(out), g["expected"])
    finally:
        arena.PINNED_RESULT_BUDGET = saved_budget
        arena.PINNED_BUDGET.calls = 0
    out = aggregate_modules(models, None, _native.DLSIM_EXACT)
    assert next(out.parameters()).is_pinned()
    torch.manual_seed(9)
    big = [Ragged([(arena.PAGEABLE_RESULT_BYTES // 4 + 1000,), (77,)]) for _ in range(3)]
    with torch.no_grad():
        for m in big:
            for q in m.parameters():
                q.normal_()
    out = aggregate_modules(big, [0.2, 0.3, 0.5], _native.DLSIM_EXACT)
    assert next(out.parameters()).is_pinned()
    exp = orc.wreduce([flat_of(m) for m in big], orc.reference_weights(3, [0.2, 0.3, 0.5]), "f32")
    assert orc.same_bits(flat_of(out), exp)


def test_wire_decode_to_device_feeds_aggregate_without_packing():
    """DLSW-decoded device state of a parameters-only model is one dense arena:
    installed as the parameters, the aggregate reads it in place (arena_view,
    one launch) and matches the oracle."""
    from dasklearn_amd import wire
    from dasklearn_amd.arena import ParamLayout
    torch.manual_seed(5)
    make = lambda: nn.Sequential(nn.Linear(33, 17), nn.Linear(17, 5))  # noqa: E731
    models = [make() for _ in range(3)]
    dev_models = []
    for m in models:
        sd = wire.decode_state_dict(wire.serialize_model(m), torch.device("cuda", 0))
        shell = make()
        for name, _ in list(shell.named_parameters()):
            mod, attr = name.rsplit(".", 1)
            setattr(shell.get_submodule(mod), attr, nn.Parameter(sd[name]))
        dev_models.append(shell)
    lay = ParamLayout(dev_models[0])
    assert all(lay.arena_view(list(m.parameters()), torch.float32) is not None for m in dev_models)
    out = FedAvg.aggregate(dev_models, None)
    ref = fedavg_torch.aggregate_modules(models, None)
    assert orc.same_bits(flat_of(out), flat_of(ref))


# ---- chunked host pipeline (arena._host_pipeline) ------------------------------------

class Mixed(nn.Module):
    """fp32, bf16 and fp16 parameter groups, interleaved (three arenas)."""

    def __init__(self, seed):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        self.a = nn.Parameter(torch.randn(300, 37, generator=g) * 0.05)
        self.b = nn.Parameter((torch.randn(1001, generator=g) * 0.05).to(torch.bfloat16))
        self.c = nn.Parameter(torch.randn(4097, generator=g) * 0.05)
        self.d = nn.Parameter((torch.randn(64, 65, generator=g) * 0.05).to(torch.bfloat16))
        self.e = nn.Parameter(torch.randn(3, generator=g))
        self.f = nn.Parameter((torch.randn(777, generator=g) * 0.05).to(torch.float16))


def _expected_by_dtype(models, weights):
    w = orc.reference_weights(len(models), weights)
    out = {}
    for dt, code in ((torch.float32, "f32"), (torch.bfloat16, "bf16"), (torch.float16, "f16")):
        rows = []
        for m in models:
            ps = [p.detach().reshape(-1) for p in m.parameters() if p.dtype == dt]
            t = torch.cat(ps)
            rows.append(t.view(torch.int16).numpy().view(np.uint16) if dt != torch.float32 else t.numpy())
        out[dt] = orc.wreduce(rows, w, code)
    return out


@pytest.mark.parametrize("chunk_bytes", [None, 4096, 50_000])
@pytest.mark.parametrize("to_host", [None, False])
def test_host_pipeline_chunks_are_exact(monkeypatch, chunk_bytes, to_host):
    """Host modules go through the chunked pack/H2D/reduce/D2H pipeline; chunk
    boundaries split tensors (forced small chunks) and both dtype groups:
    bit-identical to the oracle, on the host (default) or on the device."""
    from dasklearn_amd import arena
    if chunk_bytes is not None:
        monkeypatch.setattr(arena, "PIPELINE_CHUNK_BYTES", chunk_bytes)
    models = [Mixed(s) for s in range(5)]
    weights = [0.1, 0.3, 0.2, 0.15, 0.25]
    out = FedAvg.aggregate(models, weights, to_host=to_host)
    assert all(p.is_cuda == (to_host is False) for p in out.parameters())
    exp = _expected_by_dtype(models, weights)
    for dt in (torch.float32, torch.bfloat16, torch.float16):
        t = torch.cat([p.detach().reshape(-1).cpu() for p in out.parameters() if p.dtype == dt])
        got = t.view(torch.int16).numpy().view(np.uint16) if dt == torch.bfloat16 else t.numpy()
        assert orc.same_bits(got, exp[dt]), (dt, chunk_bytes)


def test_host_pipeline_resnet18_shapes_multi_chunk():
    """8 host ResNet-18/CIFAR-10-shaped models (62 tensors, 44.7 MB each, 5
    pipeline chunks): the host path of the north-star workload, bit-exact;
    a second call reuses the staging buffers."""
    import sys
    sys.path.insert(0, GOLDEN)
    from inputs import resnet18_cifar10_shapes
    from dasklearn_amd import arena
    assert arena.pipeline_chunk_elems(arena.ParamLayout(Ragged(resnet18_cifar10_shapes())).totals[torch.float32], 4) > 0
    models = []
    for i in range(8):
        m = Ragged(resnet18_cifar10_shapes())
        g = torch.Generator().manual_seed(50 + i)
        with torch.no_grad():
            for p in m.parameters():
                p.copy_(torch.randn(p.shape, generator=g) * 0.05)
        models.append(m)
    w = list(np.random.default_rng(7).dirichlet(np.ones(8)))
    exp = orc.wreduce_rows_f32(np.stack([flat_of(m) for m in models]), orc.reference_weights(8, w))
    for _ in range(2):
        out = FedAvg.aggregate(models, w)
        assert all(p.is_pinned() for p in out.parameters())
        assert orc.same_bits(flat_of(out), exp)


class _Tied(nn.Module):
    """Weight tying and a shared submodule: parameters() yields each tensor
    once, and deepcopy(models[0]) (fedavg.py:20) keeps the sharing."""

    def __init__(self):
        super().__init__()
        self.a = nn.Linear(3, 4)
        self.tied = nn.Linear(3, 4)
        self.tied.weight = self.a.weight  # tied: one parameter, two attributes
        self.seq = nn.Sequential(nn.Linear(4, 4), nn.ReLU())
        self.again = self.seq  # shared submodule
        self.bn = nn.BatchNorm1d(4)
        self.register_parameter("none_slot", None)


@pytest.mark.parametrize("where", ["host", "device"])
def test_tied_parameters_and_shared_submodules(where):
    """FedAvg.aggregate on modules with a tied weight and a shared submodule:
    each shared tensor is aggregated once, the output keeps the sharing
    (out.tied.weight IS out.a.weight, out.again IS out.seq) as the reference's
    deepcopy does, and every parameter is bit-identical to the reference's op
    sequence (oracle/fedavg_torch.py); buffers come from models[0]."""
    models = []
    for i in range(5):
        torch.manual_seed(100 + i)
        m = _Tied()
        with torch.no_grad():
            m.bn.running_mean.copy_(torch.randn(4))
            m.bn.num_batches_tracked.fill_(i + 3)
        models.append(m)
    w = [float(v) for v in np.random.default_rng(11).dirichlet(np.ones(5))]
    ref = fedavg_torch.aggregate_modules([copy.deepcopy(m) for m in models], w)
    ins = [m.to("cuda") for m in models] if where == "device" else models
    out = FedAvg.aggregate(ins, w)
    assert type(out) is _Tied
    assert out.tied.weight is out.a.weight and out.again is out.seq
    assert len(list(out.parameters())) == len(list(ref.parameters())) == 7
    for (na, pa), (nb, pb) in zip(out.named_parameters(), ref.named_parameters()):
        assert na == nb and pa.is_cuda == (where == "device")
        assert orc.same_bits(pa.detach().cpu().numpy(), pb.detach().numpy()), na
    assert torch.equal(out.bn.running_mean.cpu(), models[0].bn.running_mean.cpu())
    assert int(out.bn.num_batches_tracked) == 3
    assert out.none_slot is None


class _Strided(nn.Module):
    def __init__(self, seed):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        self.w = nn.Parameter(torch.randn(5, 9, generator=g).t())  # transposed: strides (1, 9)
        self.b = nn.Parameter(torch.randn(9, generator=g))
        self.c = nn.Parameter(torch.randn(2, 3, 4, generator=g).permute(2, 0, 1))


@pytest.mark.parametrize("where", ["host", "device"])
def test_non_contiguous_parameters_keep_models0_strides(where):
    """deepcopy(models[0]) (fedavg.py:20) clones a non-contiguous parameter with
    its strides (preserve_format) and add_ works on logical elements: the
    output has models[0]'s strides and the reference's values bit for bit."""
    models = [_Strided(7 + i) for i in range(4)]
    w = [0.1, 0.2, 0.3, 0.4]
    ref = fedavg_torch.aggregate_modules([copy.deepcopy(m) for m in models], w)
    ins = [copy.deepcopy(m).to("cuda") for m in models] if where == "device" else models
    out = FedAvg.aggregate(ins, w)
    for (na, pa), (nb, pb) in zip(out.named_parameters(), ref.named_parameters()):
        assert pa.shape == pb.shape and pa.stride() == pb.stride(), (na, pa.stride(), pb.stride())
        assert pa.is_cuda == (where == "device")
        assert torch.equal(pa.detach().cpu().contiguous().view(torch.int32), pb.detach().contiguous().view(torch.int32)), na


def test_zero_copy_small_host_tasks():
    """Round 5: small host models with a host result
    take dlsim_host_wreduce_zc (the kernel reads the page-locked rows and
    writes the page-locked result over PCIe, no DMA): bit-exact against the
    reference's fixtures, fp32 / bf16 / fp16, one to many models, a
    non-contiguous parameter; larger models, DLSIM_ZERO_COPY=0 and device
    results keep the DMA pipeline; the C entry refuses pageable memory
    before any launch."""
    from dasklearn_amd import _native, arena
    from dasklearn_amd.arena import aggregate_modules
    before = arena.ZC_CALLS[0]
    for name in ("cfg1_gnlenet_f32_n2_none", "cfg2_gnlenet_f32_n8_none",  # 17 x GNLeNet: 5.8 MB, the DMAs
                 "ragged_bf16_n3_list", "ragged_bf16_n17_list", "ragged_f32_n100_list"):
        g = load_golden(os.path.join(GOLDEN, name + ".npz"))
        models = modules_from_golden(g)
        calls = arena.ZC_CALLS[0]
        out = aggregate_modules(models, g["weights_arg"], _native.DLSIM_EXACT)
        assert arena.ZC_CALLS[0] == calls + 1, name
        p0 = next(out.parameters())
        assert not p0.is_cuda and p0.is_pinned()
        assert orc.same_bits(flat_of(out), g["expected"]), name
    # a transposed (non-contiguous) parameter: copied, then packed
    torch.manual_seed(21)
    ms = [torch.nn.Linear(40, 30) for _ in range(3)]
    for m in ms:
        m.weight.data = m.weight.data.t().contiguous().t()
    out = aggregate_modules(ms, [0.5, 0.25, 0.25], _native.DLSIM_EXACT)
    exp = orc.wreduce([np.concatenate([m.weight.detach().numpy().ravel(), m.bias.detach().numpy()]) for m in ms],
                      orc.reference_weights(3, [0.5, 0.25, 0.25]), "f32")
    got = np.concatenate([out.weight.detach().contiguous().numpy().ravel(), out.bias.detach().numpy()])
    assert orc.same_bits(got, exp)
    assert arena.ZC_CALLS[0] > before
    # off switch and size limit: the DMA pipeline, same bits
    g = load_golden(os.path.join(GOLDEN, "cfg1_gnlenet_f32_n2_none.npz"))
    models = modules_from_golden(g)
    for attr, val in (("ZERO_COPY", False), ("ZC_MAX_BYTES", 1000)):
        saved = getattr(arena, attr)
        setattr(arena, attr, val)
        try:
            calls = arena.ZC_CALLS[0]
            out = aggregate_modules(models, None, _native.DLSIM_EXACT)
            assert arena.ZC_CALLS[0] == calls
            assert orc.same_bits(flat_of(out), g["expected"])
        finally:
            setattr(arena, attr, saved)
    # the C entry refuses memory the device does not map (no launch, no fault)
    lib = _native.load()
    import ctypes
    src = torch.randn(64)
    pinned = torch.empty(2, 64, pin_memory=True)
    pageable = torch.empty(2, 64)
    res_pinned = torch.empty(64, pin_memory=True)
    srcs = (ctypes.c_void_p * 2)(src.data_ptr(), src.data_ptr())
    numels = (ctypes.c_size_t * 1)(64)
    w = (ctypes.c_float * 2)(0.5, 0.5)
    for stage, res in ((pageable, res_pinned), (pinned, torch.empty(64))):
        rc = lib.dlsim_host_wreduce_zc(2, 1, srcs, numels, w, stage.data_ptr(), 64, res.data_ptr(),
                                       _native.DLSIM_F32, _native.DLSIM_EXACT, 1,
                                       torch.cuda.current_stream().cuda_stream)
        assert rc == _native.DLSIM_E_ARG, rc
        assert b"page-locked" in lib.dlsim_last_error()
    rc = lib.dlsim_host_wreduce_zc(2, 1, srcs, numels, w, pinned.data_ptr(), 64, res_pinned.data_ptr(),
                                   _native.DLSIM_F32, _native.DLSIM_EXACT, 1, torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    assert orc.same_bits(res_pinned.numpy(), orc.wreduce([src.numpy(), src.numpy()],
                                                         orc.reference_weights(2, [0.5, 0.5]), "f32"))


def test_zero_copy_pipelined_chunks(monkeypatch):
    """dlsim_host_wreduce_zc over chunks of the element axis (tasks of >= 1 MiB
    of rows): the pack of chunk c + 1 overlaps the reduce of chunk c reading
    its rows over PCIe. Chunk boundaries inside parameters of ragged sizes,
    fp32 and bf16, 7 models: bit-exact against the oracle."""
    from dasklearn_amd import _native, arena
    from dasklearn_amd.arena import aggregate_modules
    monkeypatch.setenv("DLSIM_AB", "1")  # the library reads A/B switches only under DLSIM_AB=1
    monkeypatch.setenv("DLSIM_ZC_CHUNK_KB", "16")  # read per call: many small chunks
    for dt in (torch.float32, torch.bfloat16):
        torch.manual_seed(5)
        ms = []
        for _ in range(7):
            m = torch.nn.Sequential(torch.nn.Linear(601, 131), torch.nn.Linear(131, 67), torch.nn.Linear(67, 5))
            ms.append(m.to(dt))
        calls = arena.ZC_CALLS[0]
        w = [0.1, 0.2, 0.05, 0.15, 0.2, 0.1, 0.2]
        out = aggregate_modules(ms, w, _native.DLSIM_EXACT)
        assert arena.ZC_CALLS[0] == calls + 1
        rows = [np.concatenate([p.detach().float().numpy().ravel() for p in m.parameters()]) for m in ms]
        got = np.concatenate([p.detach().float().numpy().ravel() for p in out.parameters()])
        if dt == torch.float32:
            exp = orc.wreduce(rows, orc.reference_weights(7, w), "f32")
            assert orc.same_bits(got, exp)
        else:
            bits = [orc.f32_to_bf16_bits(r.astype(np.float32)) for r in rows]
            exp = orc.bf16_bits_to_f32(orc.wreduce(bits, orc.reference_weights(7, w), "bf16"))
            assert orc.same_bits(got.astype(np.float32), exp.astype(np.float32))


def test_small_host_task_fast_path(monkeypatch):
    """Round 6: once a model class's layout is known,
    a small host task runs arena._host_zc_aggregate -- parameters walked and
    checked in C, one _pyhost call into dlsim_host_wreduce_zc, the module
    built while the kernel runs. Bit-exact against the oracle (fp32, bf16,
    fp16; weights None and a list), the reference's output contract
    (deepcopy of models[0]: buffers and requires_grad from it, page-locked
    host parameters), an output fed back in as an input, and the cases it
    hands to the general path (same bits there): a non-contiguous parameter,
    a model on the GPU, models whose parameter lists differ."""
    from dasklearn_amd import _native, arena
    from dasklearn_amd.gradient_aggregation.fedavg import FedAvg
    real = arena._host_zc_aggregate
    taken = []

    def spy(models, w32, mode):
        r = real(models, w32, mode)
        taken.append(r is not None)
        return r
    monkeypatch.setattr(arena, "_host_zc_aggregate", spy)

    class Net(torch.nn.Module):
        def __init__(self, dt):
            super().__init__()
            self.conv = torch.nn.Conv2d(3, 8, 3)
            self.gn = torch.nn.GroupNorm(2, 8)
            self.fc = torch.nn.Linear(72, 10)
            self.register_buffer("steps", torch.tensor(7))
            self.to(dt)

    def flat(m):
        return np.concatenate([p.detach().float().numpy().ravel() for p in m.parameters()])

    def expect(ms, w, dt):
        rows = [flat(m) for m in ms]
        wf = orc.reference_weights(len(ms), w)
        if dt == torch.float32:
            return orc.wreduce(rows, wf, "f32")
        conv = orc.f32_to_bf16_bits if dt == torch.bfloat16 else orc.f32_to_f16_bits
        back = orc.bf16_bits_to_f32 if dt == torch.bfloat16 else orc.f16_bits_to_f32
        return back(orc.wreduce([conv(r.astype(np.float32)) for r in rows], wf,
                                "bf16" if dt == torch.bfloat16 else "f16")).astype(np.float32)

    for dt in (torch.float32, torch.bfloat16, torch.float16):
        torch.manual_seed(3)
        ms = [Net(dt) for _ in range(4)]
        ms[0].fc.bias.requires_grad_(False)
        for w in (None, [0.4, 0.3, 0.2, 0.1]):
            taken.clear()
            FedAvg.aggregate(ms, w)  # may learn the class layout on the general path
            out = FedAvg.aggregate(ms, w)
            assert taken[-1], dt
            assert orc.same_bits(flat(out).astype(np.float32), expect(ms, w, dt)), (dt, w)
            assert type(out) is Net and out is not ms[0] and int(out.steps) == 7
            assert not out.fc.bias.requires_grad and out.fc.weight.requires_grad
            p0 = next(out.parameters())
            assert not p0.is_cuda and p0.is_pinned() and p0.dtype == dt
        again = FedAvg.aggregate([out, ms[1]], None)  # an output as an input (a registered host arena)
        assert taken[-1]
        assert orc.same_bits(flat(again).astype(np.float32), expect([out, ms[1]], None, dt))
    # handed to the general path, same bits
    torch.manual_seed(4)
    ms = [Net(torch.float32) for _ in range(3)]
    FedAvg.aggregate(ms, None)
    ms[1].fc.weight.data = ms[1].fc.weight.data.t().contiguous().t()  # non-contiguous
    taken.clear()
    out = FedAvg.aggregate(ms, None)
    assert taken == [False] and orc.same_bits(flat(out), expect(ms, None, torch.float32))
    dev_model = Net(torch.float32).cuda()
    taken.clear()
    out = FedAvg.aggregate([ms[0], dev_model], None)
    assert taken == [False]
    assert orc.same_bits(flat(out.cpu()), expect([ms[0], dev_model.cpu()], None, torch.float32))
    other = torch.nn.Sequential(torch.nn.Linear(4, 3))
    taken.clear()
    with pytest.raises(RuntimeError):  # zip over different parameter lists: torch's add_ raises, as the reference
        FedAvg.aggregate([ms[0], other], None)
    assert taken == [False]
