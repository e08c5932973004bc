"""dlsim_wreduce_sharded's gather path with W > 1 ranks on one GPU (GPU).

The C ABI binds RCCL at run time (dlsim_rccl_bind). Here it binds a stub
(tests/native/stub_rccl.hip, built by __graft_entry__.build()) whose
communicator says "rank r of W" and whose in-place ncclBroadcast(root) copies
root's slice out of a buffer the test pre-fills with what rank root would hold
(its exact slice, NaN everywhere else). Every rank r of W in {2, 3, 8} then
runs the real entry point: its local reduce lands at its own slice, the
grouped broadcasts fill every other slice, and the assembled output must be
bit-identical to dlsim_wreduce over the whole buffers. Ragged last slices and
empty shards (more ranks than 64-element units) are included; the broadcast
log shows each non-empty slice requested once, with its byte offset and count,
inside one group.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import pytest
import torch

from oracle import oracle as orc

pytestmark = pytest.mark.gpu

from dasklearn_amd import _native  # noqa: E402
from test_gpu_parity import dev, from_dev, make_rows, to_dev  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STUB = os.path.join(ROOT, "tests", "native", "_build", "libstub_rccl.so")


@pytest.fixture(scope="module")
def stub():
    assert os.path.exists(STUB), "stub RCCL not built: run __graft_entry__.build()"
    lib = ctypes.CDLL(STUB)
    vp = ctypes.c_void_p
    lib.stub_comm_create.argtypes = [ctypes.c_int, ctypes.c_int, vp, ctypes.POINTER(vp)]
    lib.stub_comm_create.restype = vp
    lib.stub_comm_destroy.argtypes = [vp]
    lib.stub_comm_calls.argtypes = [vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_size_t),
                                    ctypes.POINTER(ctypes.c_size_t), ctypes.c_int]
    lib.stub_comm_calls.restype = ctypes.c_int
    lib.stub_comm_max_group_depth.argtypes = [vp]
    lib.stub_comm_max_group_depth.restype = ctypes.c_int
    lib.stub_comm_set_peer_words.argtypes = [vp, ctypes.POINTER(ctypes.c_int64), ctypes.c_int]
    lib.stub_comm_allreduces.argtypes = [vp]
    lib.stub_comm_allreduces.restype = ctypes.c_int
    lib.stub_comm_set_gather_sources.argtypes = [vp, ctypes.POINTER(vp)]
    lib.stub_comm_set_out_bytes.argtypes = [vp, ctypes.c_size_t]
    lib.stub_comm_gathers.argtypes = [vp, ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t)]
    lib.stub_comm_gathers.restype = ctypes.c_int
    _native.rccl_bind(STUB)
    yield lib
    _native.rccl_bind()  # back to torch's RCCL for the other tests


def _nan_like(t):
    return torch.full_like(t, float("nan"))


@pytest.mark.parametrize("dtype", ["f32", "bf16", "f16", "f64"])
@pytest.mark.parametrize("world,p", [(2, 64 * 37 * 2 + 13), (3, 64 * 41 * 3 + 50), (8, 64 * 29 * 8 + 63),
                                     (8, 100), (3, 64)])
def test_sharded_gather_assembles_the_whole_output(stub, world, p, dtype):
    """fp64 goes through dlsim_wreduce_sharded_f64 (exact double weights,
    ncclFloat64 broadcasts)."""
    n = 5
    rows = make_rows(n, p, world * 1000 + p, dtype)
    ws = [float(v) for v in np.random.default_rng(world).dirichlet(np.ones(n))]
    w = orc.reference_weights_f64(n, ws) if dtype == "f64" else orc.reference_weights(n, ws)
    xs = to_dev(list(rows), dtype)
    full = torch.empty_like(xs[0])
    _native.wreduce(xs, w, full)
    expected = from_dev(full)
    assert orc.same_bits(expected, orc.wreduce(list(rows), w, dtype))
    esz = xs[0].element_size()
    bounds = [_native.shard_range(p, world, r, 64) for r in range(world)]
    assert bounds[0][0] == 0 and bounds[-1][1] == p
    assert all(bounds[q][1] == bounds[q + 1][0] for q in range(world - 1))
    for r in range(world):
        peers = []
        for q, (b, e) in enumerate(bounds):
            buf = _nan_like(full)
            buf[b:e].copy_(full[b:e])  # what rank q holds after its own reduce
            peers.append(buf)
        out = _nan_like(full)
        comm = stub.stub_comm_create(world, r, out.data_ptr(),
                                     (ctypes.c_void_p * world)(*[t.data_ptr() for t in peers]))
        try:
            b, e = bounds[r]
            _native.wreduce_sharded([x[b:e] for x in xs], w, out, comm, gather=True)
            torch.cuda.synchronize()
            assert orc.same_bits(from_dev(out), expected), f"rank {r} of {world}"
            k = 64
            roots = (ctypes.c_int * k)()
            offs = (ctypes.c_size_t * k)()
            cnts = (ctypes.c_size_t * k)()
            m = stub.stub_comm_calls(comm, roots, offs, cnts, k)
            want = [(q, bq * esz, eq - bq) for q, (bq, eq) in enumerate(bounds) if eq > bq]
            assert [(roots[i], offs[i], cnts[i]) for i in range(m)] == want
            assert stub.stub_comm_max_group_depth(comm) == 1  # one ncclGroupStart/End around them
            assert stub.stub_comm_allreduces(comm) == 1  # the agreement step, before the group
        finally:
            stub.stub_comm_destroy(comm)


def test_sharded_without_gather_writes_only_the_own_slice(stub):
    world, p, n = 4, 64 * 10 * 4 + 7, 3
    rows = make_rows(n, p, 5, "f32")
    w = orc.reference_weights(n, None)
    xs = to_dev(list(rows), "f32")
    expected = orc.wreduce(list(rows), w, "f32")
    peers = [_nan_like(xs[0]) for _ in range(world)]
    for r in range(world):
        b, e = _native.shard_range(p, world, r, 64)
        out = _nan_like(xs[0])
        comm = stub.stub_comm_create(world, r, out.data_ptr(),
                                     (ctypes.c_void_p * world)(*[t.data_ptr() for t in peers]))
        try:
            _native.wreduce_sharded([x[b:e] for x in xs], w, out, comm, gather=False)
            got = from_dev(out)
            assert orc.same_bits(got[b:e], expected[b:e])
            assert np.isnan(np.delete(got, np.arange(b, e))).all()
            assert stub.stub_comm_calls(comm, None, None, None, 0) == 0
        finally:
            stub.stub_comm_destroy(comm)


def test_sharded_rejects_a_slice_of_the_wrong_length(stub):
    world, p = 2, 1000
    x = torch.zeros(p, device=dev())
    out = torch.empty(p, device=dev())
    comm = stub.stub_comm_create(world, 1, out.data_ptr(), (ctypes.c_void_p * 2)(out.data_ptr(), out.data_ptr()))
    try:
        with pytest.raises(_native.DlsimError, match="slices have"):
            _native.wreduce_sharded([x[:500]], orc.reference_weights(1, None), out, comm)
        # the failure was agreed with the other rank before returning, and no
        # broadcast was requested
        assert stub.stub_comm_allreduces(comm) == 1
        assert stub.stub_comm_calls(comm, None, None, None, 0) == 0
    finally:
        stub.stub_comm_destroy(comm)


def _agree_words(world, failed, n_elems, dtype, gather):
    w = [1 if r in failed else 0 for r in range(world)]
    for v in (n_elems, dtype, 1 if gather else 0):
        w += [v, -v]
    return (ctypes.c_int64 * len(w))(*w), len(w)


@pytest.mark.parametrize("case", ["peer_failed", "n_elems", "gather"])
def test_sharded_peer_failure_is_agreed_before_the_group(stub, case):
    """when another rank failed its checks, or the ranks
    disagree on the arguments that shape the broadcast group, this rank
    returns an error without entering the group (no broadcast requested), its
    own slice still reduced."""
    world, p, n = 3, 64 * 20 * 3 + 5, 4
    rows = make_rows(n, p, 77, "f32")
    w = orc.reference_weights(n, None)
    xs = to_dev(list(rows), "f32")
    expected = orc.wreduce(list(rows), w, "f32")
    out = _nan_like(xs[0])
    comm = stub.stub_comm_create(world, 0, out.data_ptr(), (ctypes.c_void_p * world)(*[out.data_ptr()] * world))
    try:
        if case == "peer_failed":
            words, k = _agree_words(world, {2}, p, _native.DLSIM_F32, True)
        elif case == "n_elems":
            words, k = _agree_words(world, set(), p + 64, _native.DLSIM_F32, True)
        else:
            words, k = _agree_words(world, set(), p, _native.DLSIM_F32, False)
        stub.stub_comm_set_peer_words(comm, words, k)
        b, e = _native.shard_range(p, world, 0, 64)
        with pytest.raises(_native.DlsimError) as ei:
            _native.wreduce_sharded([x[b:e] for x in xs], w, out, comm, gather=True)
        if case == "peer_failed":
            assert ei.value.rc == _native.DLSIM_E_PEER and "rank(s) 2 of 3" in str(ei.value)
        else:
            assert ei.value.rc == _native.DLSIM_E_DISAGREE and "disagree" in str(ei.value)
        assert stub.stub_comm_allreduces(comm) == 1
        assert stub.stub_comm_calls(comm, None, None, None, 0) == 0
        assert orc.same_bits(from_dev(out)[b:e], expected[b:e])
    finally:
        stub.stub_comm_destroy(comm)


def test_sharded_failed_rank_joins_the_agreement(stub):
    """A caller whose own checks failed (ShardedAggregator) joins the
    agreement through wreduce_sharded_failed: the library counts it as a
    failed rank and returns its argument error."""
    world, p = 2, 1000
    out = torch.empty(p, device=dev())
    comm = stub.stub_comm_create(world, 1, out.data_ptr(), (ctypes.c_void_p * 2)(out.data_ptr(), out.data_ptr()))
    try:
        with pytest.raises(_native.DlsimError) as ei:
            _native.wreduce_sharded_failed(comm, p, True, dev())
        assert ei.value.rc == _native.DLSIM_E_ARG
        assert stub.stub_comm_allreduces(comm) == 1
        assert stub.stub_comm_calls(comm, None, None, None, 0) == 0
    finally:
        stub.stub_comm_destroy(comm)


# ---- the padded all-gather and plans (next #2) ----------------

def _peer_buffers(full, bounds):
    """What each rank q holds after its own reduce: its exact slice, NaN elsewhere."""
    peers = []
    for b, e in bounds:
        buf = _nan_like(full)
        buf[b:e].copy_(full[b:e])
        peers.append(buf)
    return peers


def _padded_sources(full, bounds):
    """Rank q's all-gather segment: its slice, NaN-padded to the 64-element
    rounded widest slice (what rank q sends)."""
    width = max(e - b for b, e in bounds)
    width = (width + 63) // 64 * 64
    srcs = []
    for b, e in bounds:
        seg = torch.full((width,), float("nan"), dtype=full.dtype, device=full.device)
        seg[:e - b].copy_(full[b:e])
        srcs.append(seg)
    return srcs, width


def _comm(stub, world, r, out, peers, srcs=None):
    comm = stub.stub_comm_create(world, r, out.data_ptr(), (ctypes.c_void_p * world)(*[t.data_ptr() for t in peers]))
    stub.stub_comm_set_out_bytes(comm, out.numel() * out.element_size())
    if srcs is not None:
        stub.stub_comm_set_gather_sources(comm, (ctypes.c_void_p * world)(*[t.data_ptr() for t in srcs]))
    return comm


def _case(world, p, dtype, seed):
    n = 5
    rows = make_rows(n, p, seed, dtype)
    ws = [float(v) for v in np.random.default_rng(seed).dirichlet(np.ones(n))]
    w = orc.reference_weights_f64(n, ws) if dtype == "f64" else orc.reference_weights(n, ws)
    xs = to_dev(list(rows), dtype)
    full = torch.empty_like(xs[0])
    _native.wreduce(xs, w, full)
    assert orc.same_bits(from_dev(full), orc.wreduce(list(rows), w, dtype))
    return xs, w, full, [_native.shard_range(p, world, r, 64) for r in range(world)]


@pytest.mark.parametrize("dtype", ["f32", "bf16", "f64"])
@pytest.mark.parametrize("world,p", [(2, 64 * 37 * 2 + 13), (3, 64 * 41 * 3 + 50), (8, 64 * 29 * 8 + 63),
                                     (8, 100), (3, 64), (4, 64 * 4 * 10)])
def test_sharded_allgather_assembles_the_whole_output(stub, world, p, dtype):
    """DLSIM_GATHER_ALLGATHER: the local reduce lands in this rank's padded
    segment, ONE in-place all-gather of 64-element-rounded equal segments,
    then the unpad kernel: bit-identical to one GPU on every rank, with
    ragged last slices, empty shards (100 elements over 8 ranks) and an even
    split; no broadcast is requested."""
    xs, w, full, bounds = _case(world, p, dtype, world * 7 + p)
    expected = from_dev(full)
    peers = _peer_buffers(full, bounds)
    srcs, width = _padded_sources(full, bounds)
    esz = xs[0].element_size()
    for r in range(world):
        out = _nan_like(full)
        comm = _comm(stub, world, r, out, peers, srcs)
        try:
            b, e = bounds[r]
            _native.wreduce_sharded([x[b:e] for x in xs], w, out, comm, gather="allgather")
            torch.cuda.synchronize()
            assert orc.same_bits(from_dev(out), expected), f"rank {r} of {world}"
            cnt, off = ctypes.c_size_t(), ctypes.c_size_t()
            assert stub.stub_comm_gathers(comm, ctypes.byref(cnt), ctypes.byref(off)) == 1
            assert cnt.value == width and off.value == r * width * esz
            assert stub.stub_comm_calls(comm, None, None, None, 0) == 0
            assert stub.stub_comm_allreduces(comm) == 1
        finally:
            stub.stub_comm_destroy(comm)


@pytest.mark.parametrize("gather", ["bcast", "allgather"])
@pytest.mark.parametrize("world", [2, 8])
def test_plan_agrees_once_over_ten_runs(stub, world, gather):
    """a plan agrees once (one all-reduce at creation);
    ten identical runs add no all-reduce and no host wait, and every run's
    output is bit-identical to one GPU; each run requests its gather."""
    p, dtype = 64 * 23 * world + 29, "f32"
    xs, w, full, bounds = _case(world, p, dtype, 1000 + world)
    expected = from_dev(full)
    peers = _peer_buffers(full, bounds)
    srcs, _ = _padded_sources(full, bounds)
    r = world - 1
    out = _nan_like(full)
    comm = _comm(stub, world, r, out, peers, srcs)
    try:
        plan = _native.ShardedPlan(comm, p, len(xs), torch.float32, gather, device=dev())
        assert stub.stub_comm_allreduces(comm) == 1
        b, e = bounds[r]
        for _ in range(10):
            out.fill_(float("nan"))
            plan.run([x[b:e] for x in xs], w, out)
            assert orc.same_bits(from_dev(out), expected)
        assert stub.stub_comm_allreduces(comm) == 1
        if gather == "bcast":
            assert stub.stub_comm_calls(comm, None, None, None, 0) == 10 * world
        else:
            assert stub.stub_comm_gathers(comm, None, None) == 10
        plan.close()
    finally:
        stub.stub_comm_destroy(comm)


@pytest.mark.parametrize("gather", ["bcast", "allgather"])
def test_plan_run_failure_still_enters_the_gather(stub, gather):
    """A run whose local checks fail (null slices and output: run_failed, or
    a wrong weight count) still enters the plan's gather, so its peers are not
    left waiting, and raises on this rank. The slice it sends is all-ones
    bytes (NaN), never the stale numbers its buffer held."""
    world, p = 3, 64 * 11 * 3 + 5
    xs, w, full, bounds = _case(world, p, "f32", 4242)
    peers = _peer_buffers(full, bounds)
    srcs, _ = _padded_sources(full, bounds)
    out = _nan_like(full)
    comm = _comm(stub, world, 1, out, peers, srcs)
    try:
        plan = _native.ShardedPlan(comm, p, len(xs), torch.float32, gather, device=dev())
        with pytest.raises(_native.DlsimError):
            plan.run_failed(dev())
        torch.cuda.synchronize()
        b, e = bounds[1]
        bad = np.concatenate([w, w[:1]])
        with pytest.raises(AssertionError):  # caught in Python, which still enters the gather
            plan.run([x[b:e] for x in xs], bad, out)
        out[b:e].copy_(full[b:e])  # plausible numbers that must not be sent
        with pytest.raises(_native.DlsimError, match="slices have"):  # the library checks the length
            plan.run([x[b:e - 1] for x in xs], w, out)
        torch.cuda.synchronize()
        assert bool((out[b:e].view(torch.int32) == -1).all()), "a failed rank's slice goes out as NaN"
        entered = stub.stub_comm_calls(comm, None, None, None, 0) if gather == "bcast" \
            else stub.stub_comm_gathers(comm, None, None)
        assert entered == (3 * world if gather == "bcast" else 3)
        assert stub.stub_comm_allreduces(comm) == 1
        # the plan still works after a failed run
        plan.run([x[b:e] for x in xs], w, out)
        assert orc.same_bits(from_dev(out), from_dev(full))
        plan.close()
    finally:
        stub.stub_comm_destroy(comm)


def test_plan_creation_is_agreed(stub):
    """Plan creation is collective: a peer that failed, or disagrees on the
    fan-in, leaves no plan on this rank (DLSIM_E_PEER / DLSIM_E_DISAGREE)."""
    world, p, n = 2, 1000, 3
    out = torch.empty(p, device=dev())
    comm = stub.stub_comm_create(world, 0, out.data_ptr(), (ctypes.c_void_p * 2)(out.data_ptr(), out.data_ptr()))
    try:
        words = [0, 1]  # rank 1 failed
        for v in (p, n, _native.DLSIM_F32, 1):
            words += [v, -v]
        stub.stub_comm_set_peer_words(comm, (ctypes.c_int64 * len(words))(*words), len(words))
        with pytest.raises(_native.DlsimError) as ei:
            _native.ShardedPlan(comm, p, n, torch.float32, True, device=dev())
        assert ei.value.rc == _native.DLSIM_E_PEER
        words = [0, 0]
        for v in (p, n + 1, _native.DLSIM_F32, 1):  # the peer has another fan-in
            words += [v, -v]
        stub.stub_comm_set_peer_words(comm, (ctypes.c_int64 * len(words))(*words), len(words))
        with pytest.raises(_native.DlsimError) as ei:
            _native.ShardedPlan(comm, p, n, torch.float32, True, device=dev())
        assert ei.value.rc == _native.DLSIM_E_DISAGREE
        assert stub.stub_comm_allreduces(comm) == 2
    finally:
        stub.stub_comm_destroy(comm)


@pytest.mark.parametrize("gather", ["bcast", "allgather"])
def test_per_call_cost_plan_vs_agreement(stub, gather):
    """Per-call host time of the agreed call (all-reduce + host wait) against a
    plan's run, W = 2 on the stub (printed for DESIGN §7; the stub's
    all-reduce is host-synchronous like the library's read-back)."""
    import time
    world, p = 2, 64 * 1000 * 2
    xs, w, full, bounds = _case(world, p, "f32", 9)
    peers = _peer_buffers(full, bounds)
    srcs, _ = _padded_sources(full, bounds)
    out = _nan_like(full)
    comm = _comm(stub, world, 0, out, peers, srcs)
    try:
        b, e = bounds[0]
        sl = [x[b:e] for x in xs]
        plan = _native.ShardedPlan(comm, p, len(xs), torch.float32, gather, device=dev())
        reps = 200
        for f in (lambda: _native.wreduce_sharded(sl, w, out, comm, gather=gather), lambda: plan.run(sl, w, out)):
            f()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            _native.wreduce_sharded(sl, w, out, comm, gather=gather)
        torch.cuda.synchronize()
        agreed = (time.perf_counter() - t0) / reps * 1e6
        t0 = time.perf_counter()
        for _ in range(reps):
            plan.run(sl, w, out)
        torch.cuda.synchronize()
        planned = (time.perf_counter() - t0) / reps * 1e6
        print(f"\nPER_CALL_US gather={gather} W=2 p={p}: agreed {agreed:.1f} us, plan {planned:.1f} us")
        assert planned < agreed
        plan.close()
    finally:
        stub.stub_comm_destroy(comm)
