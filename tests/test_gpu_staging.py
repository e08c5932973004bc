"""arena._Staging (GPU): one grow-only device buffer and one grow-only pinned
buffer per (device, dtype), carved into [n, row_stride] rows per call; the
previous user's event is waited for before the rows are handed out again;
the lock is per key and released by release()."""
from __future__ import annotations

import threading

import pytest
import torch

pytestmark = pytest.mark.gpu

from dasklearn_amd import arena  # noqa: E402


def test_rows_shape_growth_and_reuse():
    st = arena._Staging()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    rows, host = st.acquire(dev, torch.float32, 3, 1000, stream)
    stride = arena.row_stride(1000, 4)
    assert rows.shape == (3, 1000) and host.shape == (3, 1000) and host.is_pinned()
    assert rows.stride(0) == stride == host.stride(0)
    st.release(dev, torch.float32, stream)
    again, host2 = st.acquire(dev, torch.float32, 3, 1000, stream)
    assert again is rows and host2 is host  # the same request: the same views
    st.release(dev, torch.float32, stream)
    small, _ = st.acquire(dev, torch.float32, 2, 500, stream)  # fits: no new buffer
    key = st._key(dev, torch.float32)
    assert small.data_ptr() == rows.data_ptr() and st.dev[key].numel() == 3 * stride
    st.release(dev, torch.float32, stream)
    big, bhost = st.acquire(dev, torch.float32, 5, 4000, stream)  # grows, one buffer per key
    assert st.dev[key].numel() >= 5 * arena.row_stride(4000, 4) and len(st.dev) == 1 and len(st.host) == 1
    st.release(dev, torch.float32, stream)
    dev_only, none = st.acquire(dev, torch.bfloat16, 2, 10, stream, pinned=False)
    assert none is None and dev_only.dtype == torch.bfloat16 and len(st.dev) == 2 and len(st.host) == 1
    st.release(dev, torch.bfloat16, stream)
    st.clear()
    assert not st.dev and not st.host and not st.last_use


def test_acquire_waits_for_the_previous_users_work():
    st = arena._Staging()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    rows, host = st.acquire(dev, torch.float32, 1, 1 << 20, stream)
    host.fill_(1.0)
    rows.copy_(host, non_blocking=True)  # queued work that reads the pinned rows
    torch.cuda._sleep(20_000_000)  # keep the stream busy past release()
    st.release(dev, torch.float32, stream)
    ev = st.last_use[st._key(dev, torch.float32)]
    st.acquire(dev, torch.float32, 1, 1 << 20, stream)
    assert ev.query()  # acquire returned only once that work had completed
    st.release(dev, torch.float32, stream)


def test_lock_is_per_key_and_released():
    st = arena._Staging()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    st.acquire(dev, torch.float32, 1, 16, stream)
    other = []
    t = threading.Thread(target=lambda: other.append(st.acquire(dev, torch.float16, 1, 16, stream)))
    t.start()
    t.join(10)
    assert other, "another key must not wait for this one"
    st.release(dev, torch.float16, stream)
    waiting = threading.Thread(target=lambda: (st.acquire(dev, torch.float32, 1, 16, stream),
                                               st.release(dev, torch.float32, stream)))
    waiting.start()
    waiting.join(0.2)
    assert waiting.is_alive()  # the same key waits for release()
    st.release(dev, torch.float32, stream)
    waiting.join(10)
    assert not waiting.is_alive()


def test_synced_release_leaves_no_event():
    st = arena._Staging()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    st.acquire(dev, torch.float32, 1, 16, stream)
    stream.synchronize()
    st.release(dev, torch.float32, stream, synced=True)
    assert st._key(dev, torch.float32) not in st.last_use
