"""Host-side logic of the drop-in boundary that needs no GPU: weight rules
and exception order (fedavg.py:14-17, 20), parameter layouts, arena
detection, the no-CPU-fallback rule, the task-function contract."""
from __future__ import annotations

import numpy as np
import pytest
import torch
from torch import nn

from dasklearn_amd import _native, arena, functions
from dasklearn_amd.gradient_aggregation import GradientAggregation, GradientAggregationMethod
from dasklearn_amd.gradient_aggregation.fedavg import FedAvg
from dasklearn_amd.model_manager import ModelManager


def test_enum_matches_reference_value():
    # session_settings.py:40 default / gradient_aggregation/__init__.py:9
    assert GradientAggregationMethod.FEDAVG == 1
    assert issubclass(FedAvg, GradientAggregation)


def test_fp32_weight_rounding_is_rne_from_double():
    ws = [0.1, 1 / 3, 1e-40, 3.4e38, -0.7, 1.0000000596046448]
    got = _native.fp32_weights(ws)
    exp = torch.tensor(ws, dtype=torch.float64).to(torch.float32).numpy()
    assert np.array_equal(got.view(np.uint32), exp.view(np.uint32))


def test_empty_model_list_raises_index_error():
    with pytest.raises(IndexError):
        FedAvg.aggregate([], None)


def test_weight_count_mismatch_raises_assertion():
    m = [nn.Linear(2, 2), nn.Linear(2, 2)]
    with pytest.raises(AssertionError):
        FedAvg.aggregate(m, [1.0])


def test_no_cpu_fallback_without_gpu():
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    m = [nn.Linear(2, 2), nn.Linear(2, 2)]
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        FedAvg.aggregate(m, None)


def test_unsupported_param_dtype_raises():
    """float32, bfloat16, float16 and float64 parameters run on the GPU;
    others (integer, complex) raise. fp64 is single-task only."""
    arena.ParamLayout(nn.Linear(3, 3).to(torch.float16))
    arena.ParamLayout(nn.Linear(3, 3).to(torch.float64))
    m = nn.Linear(3, 3).to(torch.complex64)
    with pytest.raises(TypeError):
        arena.ParamLayout(m)
    with pytest.raises(TypeError, match="one task at a time"):
        _native.dtype_code(torch.float64)
    assert _native.dtype_code(torch.float64, single_task=True) == _native.DLSIM_F64


def test_weights_per_dtype_follow_the_reference_op():
    """w * p1 (fedavg.py:25): an fp32/bf16/fp16 tensor rounds the Python float
    to fp32; a double tensor keeps it exact."""
    ws = [0.1, 1.0 / 3.0]
    assert _native.weights_for_dtype(ws, torch.float32).dtype == np.float32
    assert _native.weights_for_dtype(ws, torch.bfloat16)[1] == np.float32(1.0 / 3.0)
    w64 = _native.weights_for_dtype(ws, torch.float64)
    assert w64.dtype == np.float64 and w64[0] == 0.1 and w64[1] == 1.0 / 3.0


def test_layout_groups_by_dtype_in_parameters_order():
    class Mixed(nn.Module):
        def __init__(self):
            super().__init__()
            self.a = nn.Parameter(torch.zeros(5))
            self.b = nn.Parameter(torch.zeros(3, dtype=torch.bfloat16))
            self.c = nn.Parameter(torch.zeros(2, 2))

    lay = arena.ParamLayout(Mixed())
    assert list(lay.groups) == [torch.float32, torch.bfloat16]
    assert lay.groups[torch.float32] == [0, 2]
    assert lay.offsets[0] == 0 and lay.offsets[2] == 5 and lay.offsets[1] == 0
    assert lay.totals[torch.float32] == 9 and lay.totals[torch.bfloat16] == 3


def test_arena_view_detects_flat_backed_modules():
    m = nn.Sequential(nn.Linear(4, 3), nn.Linear(3, 2))
    lay = arena.ParamLayout(m)
    assert lay.arena_view(list(m.parameters()), torch.float32) is None  # separate storages
    flat = torch.arange(lay.totals[torch.float32], dtype=torch.float32)
    out = arena.module_from_arenas(m, lay, {torch.float32: flat})
    v = lay.arena_view(list(out.parameters()), torch.float32)
    assert v is not None and v.data_ptr() == flat.data_ptr() and torch.equal(v, flat)


def test_module_from_arenas_has_deepcopy_semantics():
    torch.manual_seed(0)
    m = nn.Sequential(nn.Linear(4, 3), nn.BatchNorm1d(3))
    m[1].running_mean.fill_(7.0)
    m.extra_attribute = {"k": [1, 2]}
    m[0].bias.requires_grad_(False)
    lay = arena.ParamLayout(m)
    flat = torch.full((lay.totals[torch.float32],), 2.0)
    out = arena.module_from_arenas(m, lay, {torch.float32: flat})
    assert type(out) is type(m) and out is not m
    assert torch.equal(out[1].running_mean, m[1].running_mean)
    assert out[1].running_mean.data_ptr() != m[1].running_mean.data_ptr()
    assert out.extra_attribute == m.extra_attribute and out.extra_attribute is not m.extra_attribute
    assert [p.requires_grad for p in out.parameters()] == [p.requires_grad for p in m.parameters()]
    assert all(torch.all(p == 2.0) for p in out.parameters())
    assert all(torch.all(p != 2.0) for p in m.parameters())  # original untouched


class _Tied(nn.Module):
    """Weight tying, a shared submodule, a hook and a non-module attribute."""

    def __init__(self):
        super().__init__()
        self.emb = nn.Linear(6, 6, bias=False)
        self.head = nn.Linear(6, 6)
        self.head.weight = self.emb.weight
        self.block = nn.Sequential(nn.Conv2d(2, 3, 3, padding=1), nn.GroupNorm(1, 3))
        self.again = self.block  # the same submodule twice
        self.table = [torch.ones(2), {"x": (1, 2)}]
        self.register_buffer("steps", torch.tensor(5))
        self.register_forward_hook(lambda mod, i, o: None)


class _CustomCopy(nn.Linear):
    def __deepcopy__(self, memo):  # classes with their own deepcopy keep it
        new = nn.Linear(self.in_features, self.out_features)
        memo[id(self)] = new
        new.marker = "custom"
        return new


def _structure(m):
    return [(name, type(mod).__name__, sorted(k for k in mod.__dict__ if k != "_compiled_call_impl"))
            for name, mod in m.named_modules(remove_duplicate=False)]


@pytest.mark.parametrize("make", [lambda: _Tied(),
                                  lambda: nn.Sequential(nn.Conv2d(3, 4, 3), nn.BatchNorm2d(4), nn.ReLU(),
                                                        nn.Flatten(), nn.Linear(4, 2)),
                                  lambda: nn.ModuleDict({"a": nn.Linear(2, 2), "b": nn.ParameterList(
                                      [nn.Parameter(torch.ones(3)), nn.Parameter(torch.zeros(2, 2))])})])
def test_fast_clone_matches_deepcopy(make):
    """module_from_arenas clones model0 without copy.deepcopy's generic
    machinery (arena._clone_module); the result must look exactly like
    copy.deepcopy(model0) with the parameters replaced."""
    import copy
    m = make()
    lay = arena.ParamLayout(m)
    flat = torch.arange(lay.totals[torch.float32], dtype=torch.float32)
    out = arena.module_from_arenas(m, lay, {torch.float32: flat})
    ref = copy.deepcopy(m)
    assert _structure(out) == _structure(ref)
    assert [n for n, _ in out.named_parameters()] == [n for n, _ in ref.named_parameters()]
    assert [n for n, _ in out.named_buffers()] == [n for n, _ in ref.named_buffers()]
    for (n, b), (_, b0) in zip(out.named_buffers(), m.named_buffers()):
        assert torch.equal(b, b0) and b.data_ptr() != b0.data_ptr(), n
    got = torch.cat([p.detach().reshape(-1) for p in out.parameters()])
    assert torch.equal(got, flat)  # parameters are the arena, in order
    assert all(a.data_ptr() != b.data_ptr() for a, b in zip(out.parameters(), m.parameters()))
    if isinstance(m, _Tied):
        assert out.head.weight is out.emb.weight and out.again is out.block
        assert out.table is not m.table and torch.equal(out.table[0], m.table[0])
        assert len(out._forward_hooks) == 1 and out._forward_hooks is not m._forward_hooks
        x = torch.randn(1, 2, 4, 4)
        assert torch.equal(out.block(x), out.again(x))
    assert arena.registered_arenas(out) is not None


class _GNLeNetTree(nn.Module):
    """The module tree of the reference's default model
    (dasklearn/models/cifar10.py:103-136): 16 modules, 14 parameters, plain
    attributes including a tuple."""

    def __init__(self):
        super().__init__()
        self.model_change = None
        self.gradient = None
        self.input_channel, self.output, self.model_input, self.classifier_input = 3, 10, (24, 24), 576
        self.features = nn.Sequential(
            nn.Conv2d(3, 32, 5, 1, 2), nn.MaxPool2d(3, 2), nn.GroupNorm(2, 32), nn.ReLU(True),
            nn.Conv2d(32, 32, 5, 1, 2), nn.GroupNorm(2, 32), nn.MaxPool2d(3, 2), nn.ReLU(True),
            nn.Conv2d(32, 64, 5, 1, 2), nn.GroupNorm(2, 64), nn.MaxPool2d(3, 2), nn.ReLU(True))
        self.classifier = nn.Sequential(nn.Linear(576, 10))


class _OldState(nn.Linear):
    """A module whose state lacks attributes Module.__setstate__ adds (an old
    pickle): the clone must take the __setstate__ route."""

    def __init__(self):
        super().__init__(2, 2)
        del self._forward_hooks_always_called


def _deep_equal(v, w):
    if type(v) is not type(w):
        return False
    if isinstance(v, torch.Tensor):
        return torch.equal(v, w)
    if isinstance(v, (list, tuple)):
        return len(v) == len(w) and all(_deep_equal(x, y) for x, y in zip(v, w))
    if isinstance(v, dict):
        return list(v.keys()) == list(w.keys()) and all(_deep_equal(v[k], w[k]) for k in v)
    return v == w


def _compare_clones(a, b, m):
    """Two clones of m: same classes, attribute names, attribute values
    (tensors by value), the same sharing among themselves as m has, and no
    mutable object shared with m except what deepcopy shares (atomic values,
    tuples of them)."""
    ma, mb = dict(a.named_modules(remove_duplicate=False)), dict(b.named_modules(remove_duplicate=False))
    assert ma.keys() == mb.keys()
    for name, x in ma.items():
        y = mb[name]
        assert type(x) is type(y)
        assert x.__dict__.keys() == y.__dict__.keys(), name
        for k, v in x.__dict__.items():
            w = y.__dict__[k]
            assert type(v) is type(w), (name, k)
            if k not in ("_modules", "_parameters"):
                assert _deep_equal(v, w), (name, k)
            orig = dict(m.named_modules(remove_duplicate=False))[name].__dict__.get(k)  # __setstate__ may add k
            if isinstance(v, (list, dict, set)) or isinstance(v, torch.Tensor):
                assert (v is orig) == (w is orig), (name, k)


@pytest.mark.parametrize("make", [lambda: _GNLeNetTree(), lambda: _Tied(), lambda: _OldState(),
                                  lambda: nn.Sequential(_CustomCopy(3, 2), nn.BatchNorm1d(2)),
                                  lambda: nn.ModuleDict({"a": nn.Linear(2, 2), "b": nn.ParameterList(
                                      [nn.Parameter(torch.ones(3)), nn.Parameter(torch.zeros(2, 2))])})])
def test_c_clone_matches_python_clone(make):
    """arena._clone_module (csrc/pyhost.cpp) against its Python specification
    arena._clone_module_py, with the same parameter memo."""
    m = make()
    m.extra = {"k": [1, 2]}
    m.ints = [3, 4]
    m.mixed = [torch.ones(1), 2]

    def memo():
        return {id(p): nn.Parameter(p.detach().clone(), requires_grad=p.requires_grad) for p in m.parameters()}

    ma, mb = memo(), memo()
    torch.manual_seed(1)  # _CustomCopy's __deepcopy__ draws a fresh Linear
    a = arena._clone_module(m, ma)
    torch.manual_seed(1)
    b = arena._clone_module_py(m, mb)
    _compare_clones(a, b, m)
    assert a.ints == m.ints and a.ints is not m.ints
    assert a.mixed is not m.mixed and a.mixed[0] is not m.mixed[0]
    for p, q in zip(a.parameters(), b.parameters()):
        assert torch.equal(p, q) and p.requires_grad == q.requires_grad
    if all(arena._plain_module_class(type(x)) for x in m.modules()):  # else deepcopy makes the parameters
        assert [id(p) for p in a.parameters()] == [id(ma[id(p)]) for p in m.parameters()]
    assert ma[id(m)] is a and mb[id(m)] is b
    again = arena._clone_module(m, ma)  # a module already in the memo
    assert again is a


def test_c_clone_propagates_errors():
    class Bad:
        def __deepcopy__(self, memo):
            raise RuntimeError("no copy")

    m = nn.Linear(2, 2)
    m.bad = Bad()
    with pytest.raises(RuntimeError, match="no copy"):
        arena._clone_module(m, {})


def test_c_clone_survives_an_attribute_that_mutates_the_module():
    """an attribute whose __deepcopy__ changes the module's dict
    while the C clone walks it must not leave the walk holding freed
    references; like the Python specification (`for k, v in d.items()`) the
    clone raises RuntimeError, and with the values replaced in place (no size
    change) both finish."""
    class Grow:
        def __init__(self, owner, add):
            self.owner, self.add = owner, add

        def __deepcopy__(self, memo):
            if self.add:
                self.owner.__dict__[f"grown_{len(self.owner.__dict__)}"] = object()
            else:
                for k in list(self.owner.__dict__):
                    if k.startswith("victim"):
                        self.owner.__dict__[k] = [0]  # drops the old value's last reference
            return Grow(None, False)

    for spec in (arena._clone_module, arena._clone_module_py):
        m = nn.Linear(2, 2)
        m.a_grow = Grow(m, True)
        m.z_victim = [object() for _ in range(3)]
        with pytest.raises(RuntimeError, match="changed size"):
            spec(m, {})
        m = nn.Linear(2, 2)
        m.a_swap = Grow(m, False)
        m.victim = [object() for _ in range(3)]
        out = spec(m, {})
        assert isinstance(out.a_swap, Grow)


def test_fast_clone_respects_custom_deepcopy():
    m = nn.Sequential(_CustomCopy(3, 2))
    lay = arena.ParamLayout(m)
    out = arena.module_from_arenas(m, lay, {torch.float32: torch.zeros(lay.totals[torch.float32])})
    assert out[0].marker == "custom"


def test_registered_arenas_invalidated_by_reassignment():
    m = nn.Sequential(nn.Linear(4, 3), nn.Linear(3, 2))
    lay = arena.ParamLayout(m)
    flat = torch.zeros(lay.totals[torch.float32])
    out = arena.module_from_arenas(m, lay, {torch.float32: flat})
    reg = arena.registered_arenas(out)
    assert reg is not None and reg[1][torch.float32] is flat
    assert [p is q for p, q in zip(reg[0].params, out.parameters())] == [True] * 4
    out[1].bias.data = torch.ones(2)  # re-pointed: no longer the arena
    assert arena.registered_arenas(out) is None
    out2 = arena.module_from_arenas(m, lay, {torch.float32: flat.clone()})
    out2[0].weight = nn.Parameter(torch.ones(3, 4))  # replaced
    assert arena.registered_arenas(out2) is None
    assert arena.registered_arenas(m) is None  # never registered
    # same address and shape, other strides (a square weight
    # re-viewed transposed): the arena no longer holds p's logical values
    sq = nn.Sequential(nn.Linear(3, 3))
    lsq = arena.ParamLayout(sq)
    out3 = arena.module_from_arenas(sq, lsq, {torch.float32: torch.arange(float(lsq.totals[torch.float32]))})
    assert arena.registered_arenas(out3) is not None
    out3[0].weight.data = out3[0].weight.data.t()
    assert out3[0].weight.data_ptr() == arena._arena_entry(out3).bases[torch.float32]
    assert arena.registered_arenas(out3) is None


def test_input_arenas_mixes_registered_and_plain():
    m = nn.Sequential(nn.Linear(4, 3), nn.Linear(3, 2))
    lay = arena.ParamLayout(m)
    a = arena.module_from_arenas(m, lay, {torch.float32: torch.zeros(lay.totals[torch.float32])})
    layout, params, views = arena.input_arenas([a, m, a])
    assert views[torch.float32] is None  # m is not an arena
    layout, params, views = arena.input_arenas([a, a])
    assert [v.data_ptr() for v in views[torch.float32]] == [a[0].weight.data_ptr()] * 2
    with pytest.raises(ValueError):
        arena.input_arenas([a, nn.Sequential(nn.Linear(4, 3), nn.Linear(3, 3))])


def test_model_manager_first_model_per_peer_wins():
    mm = ModelManager(None, object(), 0)
    a, b = nn.Linear(1, 1), nn.Linear(1, 1)
    mm.process_incoming_trained_model(3, a)
    mm.process_incoming_trained_model(3, b)
    assert list(mm.incoming_trained_models.values()) == [a]
    mm.reset_incoming_trained_models()
    assert mm.incoming_trained_models == {}


def test_model_manager_method_selection():
    class S:
        gradient_aggregation = GradientAggregationMethod.FEDAVG

    assert ModelManager(None, S(), 0).get_aggregation_method() is FedAvg

    class T:
        gradient_aggregation = 99

    assert ModelManager(None, T(), 0).get_aggregation_method() is None


def test_task_function_is_star_exported():
    ns = {}
    exec("from dasklearn_amd.functions import *", ns)
    assert ns["aggregate"] is functions.aggregate


@pytest.mark.parametrize("numel,esz,expect", [
    (125_000_000, 2, 125_000_064),      # cfg4 bf16: 256 B padding, not a 64 KiB multiple
    (1 << 20, 4, (1 << 20) + 1024),     # 4 MiB stride -> +4 KiB
    (1 << 23, 2, (1 << 23) + 2048),
    (2_795_456, 4, 2_795_456),          # 11 MiB fp32 (< 16 MiB): 256 B rule
    (85_354, 4, 85_376),
    (1, 4, 64),
])
def test_staging_row_stride(numel, esz, expect):
    s = arena.row_stride(numel, esz)
    assert s == expect
    assert (s * esz) % 256 == 0 and s >= numel
    assert (s * esz) % 65536 != 0


@pytest.mark.parametrize("numel,esz,units", [
    (11_181_642, 4, 22),    # the north star's rows: 44.7 MB -> 22 x 2 MiB
    (1 << 22, 4, 9),        # 16 MiB exactly: 8 units -> 9 (8 MiB multiple avoided)
    (6_291_456, 4, 13),     # 24 MiB: 12 -> 13
    (10_000_000, 4, 21),    # 40 MB: 20 units -> 21
    (25_000_000, 4, 49),    # 100 MB: 48 -> 49
    (30_000_000, 4, 58),
    (2_200_000, 8, 9),      # fp64 17.6 MB -> 9 units
    (2_000_000, 8, 0),      # fp64 16.0 MB < 16 MiB: the 256 B rule
])
def test_row_stride_2mib_rule(numel, esz, units):
    """Round 3 (profiles/r03_rowrule/): 4/8-byte rows of >= 16 MiB are whole
    2 MiB units, never a multiple of 8 MiB apart."""
    s = arena.row_stride(numel, esz)
    if numel * esz < arena.ROW_ALIGN_MIN:
        assert s * esz % 256 == 0 and s * esz < arena.ROW_ALIGN_MIN + 4096
        return
    assert s * esz == units * arena.ROW_ALIGN and units % 4 != 0 and s >= numel
    assert arena.base_align(numel * esz, esz) == arena.ROW_ALIGN
    assert arena.base_align(numel * 2, 2) == 256  # 2-byte rows keep the 256 B rule


def test_aligned_empty_starts_on_the_boundary():
    for n in (1, 1000, 3 << 20):
        t = arena.aligned_empty(n, torch.float32, "cpu", arena.ROW_ALIGN)
        assert t.numel() == n and t.data_ptr() % arena.ROW_ALIGN == 0 and t.is_contiguous()
    assert arena.arena_empty(5 << 20, torch.float32, "cpu").data_ptr() % arena.ROW_ALIGN == 0
    assert arena.arena_empty(100, torch.float32, "cpu").numel() == 100


@pytest.mark.parametrize("total,esz", [(1000, 4), (11_181_642, 4), (11_181_642, 2), (3 << 20, 4), (10 ** 9, 4)])
def test_host_pipeline_chunk_elems(total, esz):
    """The host pipeline cuts the parameter axis into at most
    PIPELINE_MAX_CHUNKS chunks of about PIPELINE_CHUNK_BYTES per model
    (0 = one chunk); the chunks cover the arena."""
    c = arena.pipeline_chunk_elems(total, esz)
    if c == 0:
        assert total * esz < 1.5 * arena.PIPELINE_CHUNK_BYTES
        return
    k = -(-total // c)
    assert 2 <= k <= arena.PIPELINE_MAX_CHUNKS and c * k >= total
    assert k == arena.PIPELINE_MAX_CHUNKS or abs(c * esz - arena.PIPELINE_CHUNK_BYTES) < arena.PIPELINE_CHUNK_BYTES


def test_module_params_matches_parameters():
    """arena.module_params restates list(module.parameters()): pre-order
    modules, each once; parameters in registration order, each once; None
    slots skipped."""
    from dasklearn_amd.arena import module_params

    class Odd(nn.Module):
        def __init__(self):
            super().__init__()
            self.a = nn.Linear(3, 4)
            self.shared = nn.Linear(4, 4)
            self.seq = nn.Sequential(nn.Conv2d(2, 3, 3), nn.ReLU(), self.shared, nn.BatchNorm1d(4))
            self.register_parameter("none_slot", None)
            self.tied = nn.Linear(3, 4)
            self.tied.weight = self.a.weight  # shared parameter
            self.w = nn.Parameter(torch.zeros(2))
            self.empty = nn.Module()
            self.shared_again = self.seq  # shared submodule

    for m in (Odd(), nn.Sequential(nn.Linear(2, 2), nn.Linear(2, 2)), nn.Linear(1, 1), nn.Module()):
        from dasklearn_amd.arena import module_params_py
        assert [id(q) for q in module_params_py(m)] == [id(q) for q in m.parameters()]
        got, ref = module_params(m), list(m.parameters())
        assert len(got) == len(ref) and all(a is b for a, b in zip(got, ref))


def test_clone_skips_setstate_only_when_it_is_a_plain_update():
    """arena._clone_module replaces nn.Module.__setstate__ by __dict__.update
    when the state has every attribute __setstate__ would add: the key list
    must be exactly the one of this torch's __setstate__."""
    import inspect
    import re
    src = inspect.getsource(nn.Module.__setstate__)
    keys = set(re.findall(r'"(_\w+)" not in self\.__dict__', src))
    assert keys == set(arena._SETSTATE_KEYS)


def test_pyhost_signature_and_pointer_helpers():
    """csrc/pyhost.cpp: matches() compares count, shapes and dtypes;
    data_ptrs() returns model-major pointers, or None when a tensor is not
    contiguous (the caller then copies it)."""
    from dasklearn_amd import _pyhost
    m = nn.Sequential(nn.Linear(3, 4), nn.Linear(4, 2))
    lay = arena.ParamLayout(m)
    ps = arena.module_params(m)
    assert _pyhost.matches(ps, lay._signature)
    assert not _pyhost.matches(ps[:-1], lay._signature)
    other = nn.Sequential(nn.Linear(3, 4), nn.Linear(4, 3))
    assert not _pyhost.matches(arena.module_params(other), lay._signature)
    assert not _pyhost.matches(arena.module_params(m.double()), lay._signature)
    rows = [ps, ps]
    assert _pyhost.data_ptrs(rows, [0, 2]) == [ps[0].data_ptr(), ps[2].data_ptr()] * 2
    t = [torch.zeros(4, 3).t(), torch.zeros(2)]
    assert _pyhost.data_ptrs([t], [1]) == [t[1].data_ptr()]
    assert _pyhost.data_ptrs([t], [0, 1]) is None


def test_arena_registry_follows_module_lifetime():
    """Registered arenas are keyed by id(module) with a weak reference: the
    entry goes when the module does, and a new object at a reused id is not
    mistaken for the old one."""
    import gc
    m = nn.Sequential(nn.Linear(4, 3))
    lay = arena.ParamLayout(m)
    out = arena.module_from_arenas(m, lay, {torch.float32: torch.zeros(lay.totals[torch.float32])})
    key = id(out)
    assert key in arena._ARENAS and arena.registered_arenas(out) is not None
    del out
    gc.collect()
    assert key not in arena._ARENAS
    import weakref
    other = nn.Sequential(nn.Linear(4, 3))
    arena._ARENAS[id(other)] = (weakref.ref(m), None)  # a slot whose weak ref names another module
    assert arena._arena_entry(other) is None
    del arena._ARENAS[id(other)]


def test_wreduce_rows_validates_without_launching():
    """_native.wreduce_rows (csrc/pyhost.cpp): argument checks, and a
    non-contiguous tensor returns False before anything reaches the library.
    Zero tensors call the library, which returns before any HIP call."""
    rows = [[torch.zeros(4, 3), torch.zeros(3)], [torch.zeros(4, 3).t(), torch.zeros(3)]]
    w = _native.fp32_weights([0.5, 0.5])
    assert _native.wreduce_rows(rows, [0, 1], [12, 3], w, 0, [0, 48], _native.DLSIM_F32, 0, 0) is False  # host
    assert _native.wreduce_rows(rows, [], [], w, 0, [], _native.DLSIM_F32, 0, 0) is True
    with pytest.raises(ValueError, match="one float per model"):
        _native.wreduce_rows(rows, [1], [3], _native.fp32_weights([1.0]), 0, [0], _native.DLSIM_F32, 0, 0)
    with pytest.raises(ValueError, match="differ in length"):
        _native.wreduce_rows(rows, [1], [3, 4], w, 0, [0], _native.DLSIM_F32, 0, 0)


def test_pyhost_checked_params_and_flat_run():
    """checked_params = module_params + matches in one call (None on a
    mismatch); flat_run = the tensors of a dtype group are contiguous and at
    their byte offsets from the group's first tensor."""
    from dasklearn_amd import _pyhost
    m = nn.Sequential(nn.Linear(3, 4), nn.Linear(4, 2))
    lay = arena.ParamLayout(m)
    ps = _pyhost.checked_params(m, lay._signature)
    assert ps is not None and all(a is b for a, b in zip(ps, m.parameters()))
    assert _pyhost.checked_params(nn.Sequential(nn.Linear(3, 4), nn.Linear(4, 3)), lay._signature) is None
    dt = torch.float32
    idx = lay.groups[dt]
    total = lay.totals[dt]
    assert not _pyhost.flat_run(ps, idx, lay.byte_offsets[dt], total)  # separate storages
    out = arena.module_from_arenas(m, lay, {dt: torch.zeros(lay.totals[dt])})
    qs = arena.module_params(out)
    assert _pyhost.flat_run(qs, idx, lay.byte_offsets[dt], total)
    assert not _pyhost.flat_run(qs, idx, lay.byte_offsets[dt], total + 1)  # past the storage
    assert lay.arena_view(qs, dt) is not None and lay.arena_view(ps, dt) is None
    flat = torch.zeros(lay.totals[dt])
    t = [flat[0:12].view(4, 3).t(), flat[12:16], flat[16:24].view(2, 4), flat[24:26]]  # right place, transposed
    assert not _pyhost.flat_run(t, idx, lay.byte_offsets[dt], total)
    with pytest.raises(ValueError, match="differ in length"):
        _pyhost.flat_run(qs, idx, lay.byte_offsets[dt][:-1], total)
    with pytest.raises(TypeError, match="expected a tensor"):
        _pyhost.flat_run([1, 2, 3, 4], idx, lay.byte_offsets[dt], total)


def test_clone_leaves_empty_hook_registries_untracked_until_used():
    """The C clone hands out its fresh empty OrderedDicts untracked by the
    cyclic collector; inserting a hook re-tracks the registry (CPython's dict
    insert path), so a cycle through a hook is still collected."""
    import gc
    import weakref
    m = nn.Sequential(nn.Linear(2, 2))
    lay = arena.ParamLayout(m)
    out = arena.module_from_arenas(m, lay, {torch.float32: torch.zeros(lay.totals[torch.float32])})
    assert not gc.is_tracked(out._forward_hooks) and not gc.is_tracked(out[0]._forward_pre_hooks)
    assert gc.is_tracked(m._forward_hooks)  # the original is untouched

    class Hook:
        def __call__(self, mod, inp, o):
            return None

    h = Hook()
    h.cycle = out  # hook -> module -> registry -> hook
    out.register_forward_hook(h)
    assert gc.is_tracked(out._forward_hooks)
    r = weakref.ref(out)
    del out, h
    gc.collect()
    assert r() is None  # the cycle was found


def test_clone_fresh_containers_are_distinct_working_objects():
    """The clone makes its empty OrderedDict / dict / set attributes through
    the C constructors (PyODict_New, PyDict_New, PySet_New): each is a fresh
    object of the exact type, one per module and attribute, and works as a
    hook registry (hooks run and are removed)."""
    from collections import OrderedDict
    m = nn.Sequential(nn.Linear(3, 3), nn.ReLU())
    lay = arena.ParamLayout(m)
    a = torch.cat([q.detach().reshape(-1) for q in lay.params])  # m's own values
    out = arena.module_from_arenas(m, lay, {torch.float32: a})
    seen = set()
    for src, dst in zip(m.modules(), out.modules()):
        for k, v in src.__dict__.items():
            if type(v) in (OrderedDict, dict, set) and not v and k not in ("_parameters", "_modules"):
                w = dst.__dict__[k]
                assert type(w) is type(v) and not w and w is not v and id(w) not in seen, k
                seen.add(id(w))
    x = torch.ones(1, 3)
    h = out.register_forward_hook(lambda mod, i, o: o * 2)
    p = out[0].register_forward_pre_hook(lambda mod, i: (i[0] * 3,))
    assert torch.equal(out(x), m(x * 3) * 2)
    assert not m._forward_hooks and not m[0]._forward_pre_hooks  # the original is untouched
    h.remove()
    p.remove()
    assert torch.equal(out(x), m(x)) and not out._forward_hooks


@pytest.mark.parametrize("offset", [0, 64])
def test_param_views_match_make_subclass(offset):
    """fill_param_views (C++) builds what torch.Tensor._make_subclass(
    nn.Parameter, arena.as_strided(...), requires_grad) does: Parameters that
    are views of the arena at the layout's offsets, with models[0]'s
    requires_grad, sharing the arena's storage (also at a storage offset)."""
    from dasklearn_amd import _pyhost

    class M(nn.Module):
        def __init__(self):
            super().__init__()
            self.a = nn.Linear(3, 4)
            self.s = nn.Parameter(torch.tensor(2.0))  # 0-dim
            self.e = nn.Parameter(torch.zeros(0, 3))  # empty
            self.c = nn.Conv2d(2, 3, 3)

    m = M()
    m.a.bias.requires_grad_(False)
    lay = arena.ParamLayout(m)
    dt = torch.float32
    buf = torch.arange(offset + lay.totals[dt], dtype=dt)
    a = buf[offset:]
    idx = lay.groups[dt]
    got, exp = {}, {}
    _pyhost.fill_param_views(got, a, lay.view_specs[dt], lay.params, idx)
    arena._param_views_py(exp, a, lay.view_specs[dt], lay.params, idx)
    assert got.keys() == exp.keys() == {id(lay.params[k]) for k in idx}
    for key in exp:
        g, e = got[key], exp[key]
        assert type(g) is nn.Parameter and g.requires_grad == e.requires_grad
        assert g.shape == e.shape and g.stride() == e.stride() and g.data_ptr() == e.data_ptr()
        assert torch.equal(g, e) and g.untyped_storage().data_ptr() == buf.untyped_storage().data_ptr()
    a.add_(1)  # the views see the arena
    assert all(torch.equal(got[k], exp[k]) for k in exp)
    # leaves like the reference's deepcopy parameters: no autograd base, no
    # grad_fn, a version counter of their own, usable in autograd and in place
    for key in exp:
        g = got[key]
        assert g.is_leaf and g.grad_fn is None and g._base is None and not g._is_view()
        assert g._version == 0
    w = got[id(m.a.weight)]
    v0 = got[id(m.c.weight)]._version
    with torch.no_grad():
        w.mul_(2)
    assert w._version == 1 and got[id(m.c.weight)]._version == v0
    loss = (got[id(m.a.weight)] * 3).sum()
    loss.backward()
    assert torch.equal(w.grad, torch.full_like(w, 3.0))
    assert got[id(m.a.bias)].grad is None and not got[id(m.a.bias)].requires_grad


def test_pyhost_torch_version_guard():
    """_pyhost is compiled against one torch's internals;
    the package refuses it under another torch instead of mis-cloning."""
    from dasklearn_amd import _pyhost
    assert _pyhost.BUILT_FOR_TORCH == torch.__version__
    arena.check_pyhost_build(torch.__version__, torch.__version__)
    with pytest.raises(ImportError, match="built for torch 2.1.2"):
        arena.check_pyhost_build("2.1.2", torch.__version__)
    with pytest.raises(ImportError, match="rebuild"):
        arena.check_pyhost_build(torch.__version__, torch.__version__ + "-other")
