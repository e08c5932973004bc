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
            assert ei.value.rc == _native.DLSIM_E_ARG and "disagree" in str(ei.value)
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
