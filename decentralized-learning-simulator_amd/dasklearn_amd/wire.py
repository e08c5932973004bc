"""Flat-buffer wire format for model state.

The reference moves models as pickles: `serialize_model` pickles the
state_dict (dasklearn/models/__init__.py:9-16) and the broker pickles whole
nn.Modules onto ZeroMQ (broker.py:205,218; communication.py:31-35), about
0.85 GB/s for an 11 M-parameter model. This codec is one header plus one
contiguous payload, so

* encoding an arena-backed model (what this package's aggregate returns)
  copies the arena bytes once; other models are gathered tensor by tensor;
* decoding is zero-copy (`torch.frombuffer` views over the payload), or one
  H2D copy straight into a device arena whose views are the tensors — the
  form the GPU aggregate reads without packing;
* nothing is unpickled: the header is JSON, the payload raw little-endian.

Layout ("DLSW", version 1):
    b"DLSW" | u32 version | u32 header_len | header (UTF-8 JSON) | pad to 64 B | payload
    header = {"entries": [{"name", "dtype", "shape", "offset", "nbytes"}...],
              "payload_bytes": N}
The payload starts 64-byte aligned; entries are packed densely at their
natural alignment (the element size), so a parameters-only state_dict of one
dtype decodes into exactly the flat arena the GPU aggregate reduces in one
launch (dasklearn_amd/arena.py `arena_view`).
"""
from __future__ import annotations

import json
import struct
from collections import OrderedDict
from typing import Dict, Optional

import torch

MAGIC = b"DLSW"
VERSION = 1
ALIGN = 64

_DTYPES = {
    "float32": torch.float32, "bfloat16": torch.bfloat16, "float16": torch.float16,
    "float64": torch.float64, "int64": torch.int64, "int32": torch.int32, "int16": torch.int16,
    "int8": torch.int8, "uint8": torch.uint8, "bool": torch.bool,
}
_NAMES = {v: k for k, v in _DTYPES.items()}


def _round(x: int, a: int = ALIGN) -> int:
    return (x + a - 1) // a * a


def _layout(sd: Dict[str, torch.Tensor]):
    entries, off = [], 0
    for name, t in sd.items():
        if t.dtype not in _NAMES:
            raise TypeError(f"{name}: unsupported dtype {t.dtype}")
        off = _round(off, t.element_size())
        nbytes = t.numel() * t.element_size()
        entries.append({"name": name, "dtype": _NAMES[t.dtype], "shape": list(t.shape),
                        "offset": off, "nbytes": nbytes})
        off += nbytes
    return entries, _round(off)


def encode_state_dict(sd: Dict[str, torch.Tensor]):
    """state_dict (host or device tensors) -> DLSW bytes, as a uint8 numpy
    array (buffer protocol: send it, write it, or hand it to decode_state_dict).
    The buffer is written once: no zero-fill, one copy per tensor."""
    entries, payload = _layout(sd)
    header = json.dumps({"entries": entries, "payload_bytes": payload}).encode()
    pre = MAGIC + struct.pack("<II", VERSION, len(header)) + header
    start = _round(len(pre))
    buf = torch.empty(start + payload, dtype=torch.uint8)
    buf[:len(pre)].copy_(torch.frombuffer(bytearray(pre), dtype=torch.uint8))
    buf[len(pre):start].zero_()
    body = buf[start:]
    end = 0
    for e, t in zip(entries, sd.values()):
        if e["offset"] > end:
            body[end:e["offset"]].zero_()  # alignment padding
        end = e["offset"] + e["nbytes"]
        if e["nbytes"] == 0:
            continue
        src = t.detach().contiguous().reshape(-1).view(torch.uint8)
        body[e["offset"]:end].copy_(src)  # D2H when t is on the GPU
    body[end:].zero_()
    return buf.numpy()


def _parse(buf):
    mv = memoryview(buf)
    if bytes(mv[:4]) != MAGIC:
        raise ValueError("not a DLSW buffer")
    version, hlen = struct.unpack("<II", mv[4:12])
    if version != VERSION:
        raise ValueError(f"unsupported DLSW version {version}")
    header = json.loads(bytes(mv[12:12 + hlen]).decode())
    return header, _round(12 + hlen)


def decode_state_dict(buf, device: Optional[torch.device] = None) -> "OrderedDict[str, torch.Tensor]":
    """DLSW bytes -> state_dict. device=None: zero-copy host views over `buf`
    (keep `buf` alive and unmodified); a CUDA device: one H2D copy of the
    payload into a device arena, tensors are views of it."""
    header, start = _parse(buf)
    payload = header["payload_bytes"]
    body = torch.frombuffer(buf, dtype=torch.uint8, offset=start, count=payload) if payload else \
        torch.empty(0, dtype=torch.uint8)
    if device is not None and torch.device(device).type == "cuda":
        body = body.to(device)
    out = OrderedDict()
    for e in header["entries"]:
        dt = _DTYPES[e["dtype"]]
        raw = body[e["offset"]:e["offset"] + e["nbytes"]]
        out[e["name"]] = raw.view(dt).view(e["shape"]) if e["nbytes"] else \
            torch.empty(e["shape"], dtype=dt, device=body.device)
    return out


def serialize_model(model: torch.nn.Module):
    """DLSW counterpart of the reference's serialize_model (models/__init__.py:9-10)."""
    return encode_state_dict(model.state_dict())


def unserialize_model(buf, model: torch.nn.Module, device=None) -> torch.nn.Module:
    """Load DLSW bytes into `model` (the reference builds it with create_model,
    models/__init__.py:13-16) and return it."""
    model.load_state_dict(decode_state_dict(buf, device))
    return model
