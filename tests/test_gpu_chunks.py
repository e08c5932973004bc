"""Chunked-model path on the GPU: dlsim_chunk_mean_batched (PyTorch's CPU
order), dlsim_mean (input order) and ChunkManager.reconstruct_model against
the reference's ChunkManager fixtures and the oracle."""
from __future__ import annotations

import os

import numpy as np
import pytest
import torch

from oracle import oracle as orc
from test_chunks_cpu import CHUNK_FIXTURES, Net, load

pytestmark = pytest.mark.gpu

from dasklearn_amd import _native, functions  # noqa: E402
from dasklearn_amd.chunk_manager import ChunkManager  # noqa: E402


def dev():
    return torch.device("cuda", 0)


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 8, 9, 14, 15, 17, 33, 128, 129])
def test_dlsim_mean_vs_oracle(n, dtype):
    rng = np.random.default_rng(n)
    p = 9_001 + n
    x = rng.standard_normal((n, p)).astype(np.float32)
    rows = orc.f32_to_bf16_bits(x) if dtype == "bf16" else x
    if dtype == "bf16":
        xs = [torch.from_numpy(r.view(np.int16).copy()).view(torch.bfloat16).to(dev()) for r in rows]
    else:
        xs = [torch.from_numpy(r.copy()).to(dev()) for r in rows]
    out = torch.empty(p, dtype=xs[0].dtype, device=dev())
    _native.mean(xs, out)
    got = out.cpu()
    got = got.view(torch.int16).numpy().view(np.uint16) if dtype == "bf16" else got.numpy()
    exp = orc.mean(list(rows), dtype)
    if dtype == "bf16" and n > 128:
        # the second pass continues from a bf16-rounded partial sum: tolerance
        g, e = orc.bf16_bits_to_f32(got), orc.bf16_bits_to_f32(exp)
        assert np.all(np.abs(g - e) <= 2.0 ** -7 * np.abs(orc.bf16_bits_to_f32(rows)).mean(0) + 1e-30)
    else:
        assert orc.same_bits(got, exp)


@pytest.mark.parametrize("path", CHUNK_FIXTURES, ids=lambda p: os.path.basename(p)[:-4])
@pytest.mark.parametrize("where", ["host", "device"])
def test_reconstruct_matches_reference(path, where):
    d = load(path)
    k, counts = d["meta"]["num_chunks"], d["meta"]["counts"]
    chunks = [[torch.from_numpy(d[f"chunks_{c}"][p].copy()) for p in range(counts[c])] for c in range(k)]
    if where == "device":
        chunks = [[t.to(dev()) for t in cs] for cs in chunks]
    target = Net(d["meta"]["shapes"])
    if where == "device":
        target = target.to(dev())
    prev = torch.get_num_threads()
    torch.set_num_threads(d["meta"]["torch_threads"])  # the reference worker's threads
    try:
        out = ChunkManager.reconstruct_model(chunks, target)
    finally:
        torch.set_num_threads(prev)
    assert out is target
    assert all(torch.is_tensor(c) for c in chunks)  # replaced in place by the means
    got = ChunkManager.get_flat_params(out).cpu().numpy()
    # bit-exact for every contributor count (PyTorch's CPU order)
    assert orc.same_bits(got, d["expected"]), counts


def test_reconstruct_task_function_uses_factory():
    d = load(CHUNK_FIXTURES[0])
    k, counts = d["meta"]["num_chunks"], d["meta"]["counts"]
    chunks = [[torch.from_numpy(d[f"chunks_{c}"][p].copy()) for p in range(counts[c])] for c in range(k)]

    class S:
        dataset, model = "cifar10", "custom"

    old = functions.model_factory
    functions.model_factory = lambda dataset, architecture=None: Net(d["meta"]["shapes"])
    try:
        res = functions.reconstruct_from_chunks(S(), {"chunks": chunks})
    finally:
        functions.model_factory = old
    assert isinstance(res, list) and len(res) == 1
    got = ChunkManager.get_flat_params(res[0]).numpy()
    if max(counts) <= 4:
        assert orc.same_bits(got, d["expected"])
    chunked = functions.chunk(S(), {"model": res[0], "n": 3})
    assert len(chunked) == 3 and sum(c.numel() for c in chunked) == got.size


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_mean_batched_equals_separate_means(dtype):
    """dlsim_mean_batched: 40 tasks (two kernel-argument batches), fan-in 1..20
    (the > 16 ones run alone), ragged sizes: each task bit-identical to the
    oracle mean (n <= 128: one pass)."""
    rng = np.random.default_rng(3)
    tasks, exp = [], []
    for t in range(40):
        n = 1 + (t * 7) % 20
        p = 1 + int(rng.integers(1, 5000))
        x = rng.standard_normal((n, p)).astype(np.float32)
        rows = orc.f32_to_bf16_bits(x) if dtype == "bf16" else x
        if dtype == "bf16":
            xs = [torch.from_numpy(r.view(np.int16).copy()).view(torch.bfloat16).to(dev()) for r in rows]
        else:
            xs = [torch.from_numpy(r.copy()).to(dev()) for r in rows]
        tasks.append((xs, torch.empty(p, dtype=xs[0].dtype, device=dev())))
        exp.append(orc.mean(list(rows), dtype))
    _native.mean_batched(tasks)
    for (_, out), e in zip(tasks, exp):
        got = out.cpu()
        got = got.view(torch.int16).numpy().view(np.uint16) if dtype == "bf16" else got.numpy()
        assert orc.same_bits(got, e)


@pytest.mark.parametrize("where", ["host", "device"])
def test_mean_chunk_indices_one_launch_per_dtype(where):
    """Every chunk index of a reconstruction in one batched launch, host chunks
    through one staging buffer: same bits as one dlsim_chunk_mean_batched call
    per index; results live where their first chunk lives."""
    rng = np.random.default_rng(9)
    chunks = []
    for c in range(10):
        p = 777 + 13 * c
        dt = torch.bfloat16 if c % 3 == 2 else torch.float32
        cs = [torch.from_numpy(rng.standard_normal(p).astype(np.float32)).to(dt) for _ in range(1 + c % 6)]
        chunks.append([t.to(dev()) for t in cs] if where == "device" else cs)
    means = ChunkManager.mean_chunk_indices(chunks)
    if where == "host":
        # host means of one dtype lie back to back even when the sizes break
        # 16-B alignment (777 + 13c elements): reconstruct_model skips the cat
        from dasklearn_amd.chunk_manager import _span
        f32 = [m for cs, m in zip(chunks, means) if cs[0].dtype == torch.float32]
        assert _span(f32) is not None
    for cs, m in zip(chunks, means):
        assert m.is_cuda == (where == "device") and m.dtype == cs[0].dtype and m.shape == cs[0].shape
        ref = torch.empty(cs[0].numel(), dtype=cs[0].dtype, device=dev())
        _native.chunk_mean_batched([([t.to(dev()).reshape(-1) for t in cs], ref)])
        assert torch.equal(m.cpu().view(torch.int16 if m.dtype == torch.bfloat16 else torch.int32),
                           ref.cpu().view(torch.int16 if m.dtype == torch.bfloat16 else torch.int32))


def _rows_t(rng, m, n, dtype, offset=0):
    """m rows of n elements as device tensors, `offset` elements into their
    buffers (offset 1: not 16-byte aligned)."""
    x = (rng.standard_normal((m, n)) * np.exp(rng.standard_normal((m, n)) * 2))
    x = x if dtype == "f64" else x.astype(np.float32)
    rows = orc.f32_to_bf16_bits(x) if dtype == "bf16" else orc.f32_to_f16_bits(x) if dtype == "f16" else x
    tdt = torch.bfloat16 if dtype == "bf16" else torch.float16
    ts = []
    for r in rows:
        h = torch.from_numpy(r.view(np.int16).copy()).view(tdt) if dtype in ("bf16", "f16") \
            else torch.from_numpy(r.copy())
        buf = torch.empty(n + offset, dtype=h.dtype, device=dev())
        buf[offset:].copy_(h)
        ts.append(buf[offset:])
    return rows, ts


def _bits(t):
    t = t.cpu()
    return t.view(torch.int16).numpy().view(np.uint16) if t.dtype == torch.bfloat16 else t.numpy()


@pytest.mark.parametrize("dtype", ["f32", "bf16", "f16", "f64"])
@pytest.mark.parametrize("threads", [1, 4, 8])
def test_chunk_mean_matches_torch_order(dtype, threads):
    """Every (m, n) class of PyTorch's CPU sum order — cascade blocks, the
    < 32-column ilp tail, the < 8-column scalar groups, the one-element inner
    reduction, the level-1 flush at 16 rows — in batches that cross the
    32-task / 192-input launch limits: each task bit-identical to the
    order-exact oracle (pinned against torch.mean on the CPU)."""
    rng = np.random.default_rng(threads * 10 + ["f32", "bf16", "f16", "f64"].index(dtype))
    tasks, exp = [], []
    for m in (1, 2, 3, 4, 5, 8, 9, 16, 17, 18, 33, 100):
        for n in (1, 2, 3, 5, 7, 8, 9, 31, 33, 65, 1000, 4099, 40001):
            rows, ts = _rows_t(rng, m, n, dtype)
            tasks.append((ts, torch.empty(n, dtype=ts[0].dtype, device=dev())))
            exp.append(orc.chunk_mean(list(rows), dtype, threads))
    _native.chunk_mean_batched(tasks, threads=threads)
    for (ts, out), e in zip(tasks, exp):
        assert orc.same_bits(_bits(out), e), (len(ts), out.numel())


@pytest.mark.parametrize("dtype", ["f32", "bf16", "f16", "f64"])
def test_chunk_mean_unaligned_and_aliased(dtype):
    """Rows one element into their buffers (scalar path), and the output
    aliasing input 0."""
    rng = np.random.default_rng(5)
    for m, n in ((3, 4099), (7, 40001), (20, 100)):
        rows, ts = _rows_t(rng, m, n, dtype, offset=1)
        out = torch.empty(n + 1, dtype=ts[0].dtype, device=dev())[1:]
        _native.chunk_mean_batched([(ts, out)], threads=4)
        e = orc.chunk_mean(list(rows), dtype, 4)
        assert orc.same_bits(_bits(out), e)
        _native.chunk_mean_batched([(ts, ts[0])], threads=4)
        assert orc.same_bits(_bits(ts[0]), e)


@pytest.mark.parametrize("dtype", ["f32", "bf16", "f16", "f64"])
def test_chunk_mean_line_misaligned_heads(dtype):
    """Chunks that start off a 128-B line (slices of equally aligned rows, as
    chunk_model cuts a flat model): block 0 folds the leading columns and the
    tiles start on the line. Every 16-B misalignment, sizes around the point
    where the head is taken, one input (or the output) misaligned differently
    (no head), in one batch: each task bit-identical to the oracle."""
    rng = np.random.default_rng(77 + ["f32", "bf16", "f16", "f64"].index(dtype))
    esz = {"f32": 4, "bf16": 2, "f16": 2, "f64": 8}[dtype]
    tdt = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16, "f64": torch.float64}[dtype]
    for threads in (1, 4):
        tasks, exp = [], []
        for k, mis in enumerate(range(16, 128, 16)):
            off = mis // esz
            for m, n in ((2, 8192 + 64), (4, 3 * 4096 + 5), (7, 40001), (17, 70_000 + k)):
                rows, _ = _rows_t(rng, m, n, dtype)
                ts = []
                odd = int(rng.integers(0, m + 1)) if k % 3 == 2 else -1  # that one elsewhere
                for i, r in enumerate(rows):
                    h = torch.from_numpy(r.view(np.int16).copy()).view(tdt) if dtype in ("bf16", "f16") \
                        else torch.from_numpy(r.copy())
                    o = off + (16 // esz if i == odd else 0)
                    buf = torch.empty(64 + n + 64, dtype=tdt, device=dev())  # caching allocator: 512-B aligned
                    buf[o:o + n].copy_(h)
                    ts.append(buf[o:o + n])
                ob = torch.empty(64 + n + 64, dtype=tdt, device=dev())
                out = ob[off + (16 // esz if odd == m else 0):][:n]
                assert out.data_ptr() % 128 == (mis if odd != m else (mis + 16) % 128)
                tasks.append((ts, out))
                exp.append(orc.chunk_mean(list(rows), dtype, threads))
        _native.chunk_mean_batched(tasks, threads=threads)
        for (ts, out), e in zip(tasks, exp):
            assert orc.same_bits(_bits(out), e), (len(ts), out.numel(), ts[0].data_ptr() % 128)


@pytest.mark.parametrize("dtype", ["f32", "f64"])
@pytest.mark.parametrize("m", [193, 256, 300])
def test_chunk_mean_large_fan_in(m, dtype):
    """More inputs than a kernel-argument batch holds: the device pointer
    array path, with the level-2 flush of the cascade at 256 rows."""
    rng = np.random.default_rng(m)
    for n in (1, 9, 5000):
        rows, ts = _rows_t(rng, m, n, dtype)
        out = torch.empty(n, dtype=ts[0].dtype, device=dev())
        _native.chunk_mean_batched([(ts, out)], threads=4)
        assert orc.same_bits(_bits(out), orc.chunk_mean(list(rows), dtype, 4)), n


def test_chunk_mean_resnet18_chunks_full_size():
    """k = 10 chunks of a ResNet-18-sized flat model (11,181,642 fp32), 12
    contributors each, worker threads 4: every element bit-identical."""
    P, k, m = 11_181_642, 10, 12
    g = torch.Generator(device=dev()).manual_seed(3)
    flats = [torch.randn(P, generator=g, device=dev()) * 0.05 for _ in range(m)]
    size = P // k
    bounds = [(c * size, (c + 1) * size if c < k - 1 else P) for c in range(k)]
    tasks = [([f[b:e] for f in flats], torch.empty(e - b, device=dev())) for b, e in bounds]
    _native.chunk_mean_batched(tasks, threads=4)
    host = [f.cpu().numpy() for f in flats]
    for (b, e), (_, out) in zip(bounds, tasks):
        assert orc.same_bits(out.cpu().numpy(), orc.chunk_mean([h[b:e] for h in host], "f32", 4))


def test_chunk_mean_errors():
    x = torch.zeros(8, device=dev())
    with pytest.raises(IndexError):
        _native.chunk_mean_batched([([], x)])
    with pytest.raises(RuntimeError, match="cpu_threads"):
        _native.chunk_mean_batched([([x], torch.empty(8, device=dev()))], threads=0)


@pytest.mark.parametrize("dtype", ["f32", "bf16", "f16", "f64"])
@pytest.mark.parametrize("threads,cpu_threads,side", [(1, 1, False), (4, 4, True), (8, 8, True), (3, 16, False)])
def test_host_chunk_mean_matches_torch_order(dtype, threads, cpu_threads, side):
    """dlsim_host_chunk_mean (host chunks packed on `threads` library threads,
    per-row H2D, per-task mean and D2H): every task bit-identical to the
    order-exact oracle at cpu_threads, including empty tasks, one-element
    chunks, fan-in 1 and 40, host inputs at odd offsets, with and without the
    side copy streams."""
    from dasklearn_amd.arena import _side_streams
    rng = np.random.default_rng(threads * 100 + cpu_threads)
    tasks, exp, hosts = [], [], []
    for m, n in [(4, 300_001), (1, 7), (40, 4099), (3, 0), (17, 1), (2, 65), (9, 1_000_003), (5, 33)]:
        x = rng.standard_normal((m, n)) * 0.1
        x = x if dtype == "f64" else x.astype(np.float32)
        rows = orc.f32_to_bf16_bits(x) if dtype == "bf16" else orc.f32_to_f16_bits(x) if dtype == "f16" else x
        ts = []
        for i, r in enumerate(rows):
            if dtype in ("f32", "f64"):
                h = torch.from_numpy(r.copy())
            else:
                h = torch.from_numpy(r.view(np.int16).copy()).view(torch.bfloat16 if dtype == "bf16" else torch.float16)
            if i % 2:  # an odd offset into a larger host buffer
                buf = torch.empty(n + 1, dtype=h.dtype)
                buf[1:].copy_(h)
                h = buf[1:]
            ts.append(h)
        out = torch.empty(n + 64, dtype=ts[0].dtype, device=dev())[:n]
        tasks.append((ts, out))
        hosts.append(torch.empty(n, dtype=ts[0].dtype, pin_memory=True))
        exp.append(orc.chunk_mean(list(rows), dtype, cpu_threads) if n else None)
    esz = tasks[0][1].element_size()
    need = _native.staged_rows_elems([t[1].numel() for t in tasks], [len(t[0]) for t in tasks], esz)
    stage = torch.empty(need, dtype=tasks[0][1].dtype, pin_memory=True)
    d_in = torch.empty(need, dtype=tasks[0][1].dtype, device=dev())
    h2d, d2h = _side_streams(dev()) if side else (None, None)
    stream = torch.cuda.current_stream(dev())
    _native.host_chunk_mean(tasks, stage, d_in, host_outs=hosts, threads=threads, cpu_threads=cpu_threads,
                            stream=stream, h2d_stream=h2d, d2h_stream=d2h)
    stream.synchronize()
    for (ts, out), h, e in zip(tasks, hosts, exp):
        if e is None:
            continue
        assert orc.same_bits(_bits(out), e), (len(ts), out.numel())
        assert orc.same_bits(_bits(h), e), (len(ts), out.numel())


def test_host_chunk_mean_rejects_small_staging():
    x = [torch.zeros(100), torch.zeros(100)]
    out = torch.empty(100, device=dev())
    stage = torch.empty(64, pin_memory=True)
    with pytest.raises(ValueError):
        _native.host_chunk_mean([(x, out)], stage, torch.empty(64, device=dev()))


@pytest.mark.parametrize("dtype", ["f32", "bf16", "f64"])
@pytest.mark.parametrize("layout", ["tight", "padded", "gaps", "reversed"])
def test_host_chunk_mean_small_job_one_dma(dtype, layout):
    """a job under 4 MiB (GNLeNet's Conflux reconstruct:
    k = 10 chunk indices of ~8.5 K elements, m = 4) packs every row, sends ONE
    H2D, runs ONE batched launch and, when the outputs lie back to back at the
    same offsets on the device and the host (ChunkManager's layout), ONE D2H;
    every mean bit-identical to the order-exact oracle. Layouts: back to back
    (tight), padded device offsets, equal offsets on both sides with gaps
    between the outputs (the host bytes in the gaps must survive),
    and back to back in reverse task order."""
    rng = np.random.default_rng(17)
    k, m, size = 10, 4, 85_354 // 10
    sizes = [size] * (k - 1) + [85_354 - size * (k - 1)]
    tdt = {"f32": torch.float32, "bf16": torch.bfloat16, "f64": torch.float64}[dtype]
    esz = torch.empty((), dtype=tdt).element_size()
    al = 256 // esz
    gap = 37 if layout == "gaps" else 0
    padded = layout == "padded"
    dev_len = [((n + al - 1) // al * al if padded else n) + gap for n in sizes]
    host_len = [n + gap for n in sizes]
    d_out = torch.empty(sum(dev_len), dtype=tdt, device=dev())
    host = torch.empty(sum(host_len), dtype=tdt, pin_memory=True)
    host.view(torch.uint8).fill_(0xA5)  # the sentinel the gaps must keep
    order = list(range(k))[::-1] if layout == "reversed" else list(range(k))
    doff, hoff = {}, {}
    o = h = 0
    for t in order:
        doff[t], hoff[t] = o, h
        o += dev_len[t]
        h += host_len[t]
    tasks, exp, hosts = [], [], []
    for t, n in enumerate(sizes):
        x = rng.standard_normal((m, n)) * 0.1
        x = x if dtype == "f64" else x.astype(np.float32)
        rows = orc.f32_to_bf16_bits(x) if dtype == "bf16" else x
        ts = [torch.from_numpy(r.view(np.int16).copy()).view(tdt) if dtype == "bf16" else torch.from_numpy(r.copy())
              for r in rows]
        tasks.append((ts, d_out[doff[t]:doff[t] + n]))
        hosts.append(host[hoff[t]:hoff[t] + n])
        exp.append(orc.chunk_mean(list(rows), dtype, 4))
    need = _native.staged_rows_elems(sizes, [m] * k, esz)
    assert need * esz < 4 << 20
    stage = torch.empty(need, dtype=tdt, pin_memory=True)
    d_in = torch.empty(need, dtype=tdt, device=dev())
    stream = torch.cuda.current_stream(dev())
    _native.host_chunk_mean(tasks, stage, d_in, host_outs=hosts, threads=4, cpu_threads=4, stream=stream)
    stream.synchronize()
    for (ts, out), hh, e in zip(tasks, hosts, exp):
        assert orc.same_bits(_bits(out), e)
        assert orc.same_bits(_bits(hh), e)
    if gap:
        raw = host.view(torch.uint8).numpy()
        for t, n in enumerate(sizes):
            g0 = (hoff[t] + n) * esz
            assert (raw[g0:g0 + gap * esz] == 0xA5).all(), f"gap after task {t} overwritten"


CHUNK_FIXTURES_F64 = sorted(__import__("glob").glob(os.path.join(os.path.dirname(CHUNK_FIXTURES[0]), "..",
                                                                   "chunks_f64", "*.npz")))


@pytest.mark.parametrize("path", CHUNK_FIXTURES_F64, ids=lambda p: os.path.basename(p)[:-4])
@pytest.mark.parametrize("where", ["host", "device"])
def test_reconstruct_f64_matches_reference(path, where):
    """ChunkManager.reconstruct_model on double models,
    bit-identical to the reference's own (PyTorch's double order)."""
    d = load(path)
    k, counts = d["meta"]["num_chunks"], d["meta"]["counts"]
    chunks = [[torch.from_numpy(d[f"chunks_{c}"][p].copy()) for p in range(counts[c])] for c in range(k)]
    target = Net(d["meta"]["shapes"]).double()
    if where == "device":
        chunks = [[t.to(dev()) for t in cs] for cs in chunks]
        target = target.to(dev())
    prev = torch.get_num_threads()
    torch.set_num_threads(d["meta"]["torch_threads"])
    try:
        out = ChunkManager.reconstruct_model(chunks, target)
    finally:
        torch.set_num_threads(prev)
    got = ChunkManager.get_flat_params(out).cpu().numpy()
    assert got.dtype == np.float64
    assert np.array_equal(got.view(np.int64), d["expected"].view(np.int64)), counts


class _TiedNet(torch.nn.Module):
    """A tied weight (in state_dict() under two names) and a shared
    submodule (once: named_modules() de-duplicates it)."""

    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(40, 30)
        self.b = torch.nn.Linear(40, 30)
        self.b.weight = self.a.weight
        self.seq = torch.nn.Sequential(torch.nn.Linear(30, 7))
        self.again = self.seq


@pytest.mark.parametrize("where", ["host", "device"])
@pytest.mark.parametrize("k", [3, 7])
def test_reconstruct_tied_parameters_follows_copy_order(where, k):
    """chunk_manager.py:45-52 copies the flat means into the state_dict
    tensors one after another, so a tied tensor (two entries) ends with the
    means at its SECOND position; the device path's multi-tensor copy must not
    race them. Compared with the reference's sequence run on the CPU."""
    torch.manual_seed(5)
    peers = [_TiedNet() for _ in range(4)]
    chunked = [ChunkManager.chunk_model(m, k) for m in peers]
    by_index = [[chunked[i][c] for i in range(4) if (i + c) % 3 != 0] or [chunked[0][c]] for c in range(k)]
    ref = _TiedNet()
    flat = torch.cat([torch.mean(torch.stack(cs), dim=0) for cs in by_index])
    ptr = 0
    with torch.no_grad():
        for t in ref.state_dict().values():
            t.copy_(flat[ptr:ptr + t.numel()].view(t.shape))
            ptr += t.numel()
    target = _TiedNet()
    chunks = [[c.to(dev()) for c in cs] for cs in by_index] if where == "device" else [list(cs) for cs in by_index]
    if where == "device":
        target = target.to(dev())
    out = ChunkManager.reconstruct_model(chunks, target)
    assert out.b.weight is out.a.weight and out.again is out.seq
    for (na, ta), (nb, tb) in zip(out.state_dict().items(), ref.state_dict().items()):
        assert na == nb and orc.same_bits(ta.cpu().numpy(), tb.numpy()), na


@pytest.mark.parametrize("m,k", [(16, 4), (16, 10), (17, 3), (31, 5), (40, 6), (5, 7)])
def test_chunk_mean_deferred_launch(m, k):
    """fp32 chunk launches of >= 20 MB per stream with every task 16-B
    aligned and m >= 16 take the deferred-store kernel (k_chunk_mean_defer:
    512-lane blocks of R rows, the ragged block per task):
    chunks of a 6.3 M-element flat model cut at arbitrary points
    (line-misaligned heads, partial rows, scalar tails), the level-1 flush at
    16 rows (m = 16, 17, 31), launches split at the 192-input limit (m = 40:
    some below 20 MB, tiled), m = 5 tiled: every element bit-identical to the
    order-exact oracle at 4 worker threads. (Round 6: m = 5 now takes the
    fixed-m form, k_chunk_mean_defer_m.)"""
    P = 6_300_001
    g = torch.Generator(device=dev()).manual_seed(m * 100 + k)
    flats = [torch.randn(P, generator=g, device=dev()) * 0.05 for _ in range(m)]
    rng = np.random.default_rng(m + k)
    cuts = sorted(set(int(c) // 4 * 4 for c in rng.integers(1, P - 1, size=k - 1)))
    bounds = list(zip([0] + cuts, cuts + [P]))
    tasks = [([f[b:e] for f in flats], torch.empty(e - b, device=dev())) for b, e in bounds]
    _native.chunk_mean_batched(tasks, threads=4)
    host = [f.cpu().numpy() for f in flats]
    for (b, e), (_, out) in zip(bounds, tasks):
        assert orc.same_bits(out.cpu().numpy(), orc.chunk_mean([h[b:e] for h in host], "f32", 4)), (b, e)
    del flats, tasks
    torch.cuda.empty_cache()


@pytest.mark.parametrize("m,k", [(2, 3), (4, 10), (7, 1), (10, 10), (12, 6), (15, 4)])
def test_chunk_mean_fixed_m_deferred_launch(m, k):
    """Round 6: an fp32 launch whose tasks all have the same m, 4 <= m < 16
    (>= 20 MB per stream, 16-B aligned; m = 2 stays tiled) takes the fixed-m
    deferred kernel
    (k_chunk_mean_defer_m: MF contributors folded straight-line, each task's
    last row block also doing its ragged end). Arbitrary cuts plus a tiny
    chunk (no whole row: only the last-block ragged work), a chunk of whole
    rows exactly, line-misaligned heads and scalar tails: every element
    bit-identical to the order-exact oracle at 4 worker threads."""
    P = 6_300_001 if m < 12 else 3_900_001
    g = torch.Generator(device=dev()).manual_seed(m * 1000 + k)
    flats = [torch.randn(P, generator=g, device=dev()) * 0.05 for _ in range(m)]
    rng = np.random.default_rng(m * 7 + k)
    cuts = set(int(c) // 4 * 4 for c in rng.integers(1, P - 1, size=k - 1))
    if k >= 4:
        c0 = min(cuts)
        cuts |= {c0 + 1000, c0 + 1000 + 4 * 512 * 40}  # a 1,000-element chunk, then 40 whole rows
    cuts = sorted(c for c in cuts if 0 < c < P)
    bounds = list(zip([0] + cuts, cuts + [P]))
    tasks = [([f[b:e] for f in flats], torch.empty(e - b, device=dev())) for b, e in bounds]
    _native.chunk_mean_batched(tasks, threads=4)
    host = [f.cpu().numpy() for f in flats]
    for (b, e), (_, out) in zip(bounds, tasks):
        assert orc.same_bits(out.cpu().numpy(), orc.chunk_mean([h[b:e] for h in host], "f32", 4)), (b, e)
    del flats, tasks
    torch.cuda.empty_cache()
