"""Flat-buffer wire format (dasklearn_amd/wire.py): bit-exact round trips of
every state_dict the reference ships (parameters, BN buffers incl. int64
counters, bf16), header validation, and the reference's load path."""
from __future__ import annotations

import pickle

import pytest
import torch
from torch import nn

from dasklearn_amd import wire


class WithBN(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv = nn.Conv2d(3, 8, 3)
        self.bn = nn.BatchNorm2d(8)
        self.fc = nn.Linear(8, 10)
        self.half_w = nn.Parameter(torch.randn(7, 3).to(torch.bfloat16))
        self.register_buffer("nothing", torch.zeros(0))


def same(a, b):
    if a.dtype != b.dtype or a.shape != b.shape:
        return False
    return torch.equal(a.view(-1).view(torch.uint8), b.reshape(-1).contiguous().view(torch.uint8))


def test_round_trip_bit_exact():
    torch.manual_seed(0)
    m = WithBN()
    m.bn.num_batches_tracked.fill_(12345)
    with torch.no_grad():
        m.bn.running_var.uniform_(0.5, 2)
    buf = wire.serialize_model(m)
    sd = wire.decode_state_dict(buf)
    ref = m.state_dict()
    assert list(sd) == list(ref)
    for k in ref:
        assert same(sd[k], ref[k]), k
    m2 = wire.unserialize_model(buf, WithBN())
    for k, v in m2.state_dict().items():
        assert same(v, ref[k]), k


def test_payload_offsets_aligned_and_zero_copy():
    m = WithBN()
    buf = wire.serialize_model(m)
    header, start = wire._parse(buf)
    assert start % 64 == 0
    for e in header["entries"]:
        assert e["offset"] % torch.tensor([], dtype=wire._DTYPES[e["dtype"]]).element_size() == 0
    sd = wire.decode_state_dict(buf)
    t = sd["fc.weight"]
    t.fill_(0.0)  # views alias the buffer (zero-copy decode)
    assert all(v == 0 for v in wire.decode_state_dict(buf)["fc.weight"].reshape(-1).tolist())


def test_non_contiguous_tensors_encode():
    sd = {"t": torch.arange(12.0).view(3, 4).t()}
    out = wire.decode_state_dict(wire.encode_state_dict(sd))
    assert torch.equal(out["t"], sd["t"])


def test_rejects_foreign_buffers():
    with pytest.raises(ValueError):
        wire.decode_state_dict(bytearray(pickle.dumps({"a": 1})))
    buf = wire.serialize_model(nn.Linear(2, 2))
    buf[4] = 9  # version (little-endian u32 at byte 4)
    with pytest.raises(ValueError):
        wire.decode_state_dict(buf)


def test_unsupported_dtype():
    with pytest.raises(TypeError):
        wire.encode_state_dict({"c": torch.zeros(2, dtype=torch.complex64)})


def test_encoded_bytes_are_deterministic():
    torch.manual_seed(1)
    m = WithBN()
    a = bytes(wire.serialize_model(m))
    b = bytes(wire.serialize_model(m))
    assert a == b  # padding is zeroed, nothing uninitialised leaks
