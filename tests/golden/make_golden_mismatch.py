"""Golden vectors for models whose parameter lists differ, from the REFERENCE.

The reference pairs parameters with `zip` (fedavg.py:23-24,
/root/reference/dasklearn/gradient_aggregation/fedavg.py): a model with fewer
parameters than models[0] contributes to the leading ones only, extra
parameters of a model are ignored, and `c1.add_(w * p1)` broadcasts a
parameter whose shape broadcasts to models[0]'s (and raises otherwise).
This script runs the reference's own ``FedAvg.aggregate`` on such models and
writes inputs and outputs as .npz fixtures (``mismatch_*.npz``) next to it.
Only data is written; no reference source is copied. Skips (exit 0) when
/root/reference is absent (e.g. on the GPU box).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_mismatch.py

Fixture layout (np.load(..., allow_pickle=False)):
    meta      0-d unicode array, JSON: case, dtype, shapes (per model, the
              list of parameter shapes in parameters() order), weights_kind,
              error (the exception type name the reference raised, or null)
    inputs    1-D, every model's parameters flattened and concatenated in
              model order (float32 / float64, or uint16 bits for bf16 / f16)
    weights   float64, if weights_kind == "list"
    expected  1-D, the reference's output parameters flattened (absent when
              the reference raised)
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def main() -> int:
    if not os.path.isdir(REF):
        print("reference absent; nothing to do")
        return 0
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    import torch
    from torch import nn
    from dasklearn.gradient_aggregation.fedavg import FedAvg  # the oracle of record

    TDT = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16, "f64": torch.float64}

    class Shaped(nn.Module):
        def __init__(self, shapes, dtype):
            super().__init__()
            self.ps = nn.ParameterList([nn.Parameter(torch.zeros(s, dtype=dtype)) for s in shapes])

    def to_np(t, dtype):
        t = t.detach().contiguous().reshape(-1)
        if dtype in ("bf16", "f16"):
            return t.view(torch.int16).numpy().view(np.uint16).copy()
        return t.numpy().copy()

    rng = np.random.default_rng(4242)
    cases = [
        # (name, dtype, per-model shapes, weights kind)
        ("fewer_f32", "f32", [[[5], [130], [7, 3]], [[5], [130]], [[5], [130], [7, 3]]], "list"),
        ("more_f32", "f32", [[[5], [130]], [[5], [130], [9]], [[5], [130], [9], [2]]], "list"),
        ("mixed_f32_none", "f32", [[[64], [33], [1000]], [[64]], [[64], [33]], [[64], [33], [1000], [4]]], "none"),
        ("fewer_bf16", "bf16", [[[5], [130], [7, 3]], [[5], [130]], [[5], [130], [7, 3]]], "list"),
        ("fewer_f16", "f16", [[[5], [130], [7, 3]], [[5]], [[5], [130], [7, 3]]], "list"),
        ("fewer_f64", "f64", [[[5], [130], [7, 3]], [[5], [130]], [[5], [130], [7, 3]]], "list"),
        ("empty_model_f32", "f32", [[[5], [6]], [], [[5], [6]]], "list"),
        ("broadcast_f32", "f32", [[[4, 6], [3]], [[6], [3]], [[1, 6], [1]]], "list"),
        ("broadcast_bf16", "bf16", [[[4, 6], [3]], [[6], [3]], [[1, 6], [1]]], "none"),
        ("nonbroadcast_f32", "f32", [[[4, 6]], [[5]]], "list"),
        ("samenumel_f32", "f32", [[[4, 6]], [[6, 4]]], "none"),
    ]
    written = []
    for name, dtype, shapes, wk in cases:
        n = len(shapes)
        tdt = TDT[dtype]
        models = []
        for sh in shapes:
            m = Shaped(sh, tdt)
            with torch.no_grad():
                for p in m.parameters():
                    v = rng.standard_normal(p.numel()) * 0.05
                    p.copy_(torch.from_numpy(v).to(tdt).view_as(p))
            models.append(m)
        weights = [float(w) for w in rng.dirichlet(np.ones(n))] if wk == "list" else None
        flat_in = [to_np(p, dtype) for m in models for p in m.parameters()]
        inputs = np.concatenate(flat_in) if flat_in else np.zeros(0, np.float32)
        error, expected = None, None
        try:
            out = FedAvg.aggregate(models, weights)
            expected = np.concatenate([to_np(p, dtype) for p in out.parameters()])
        except Exception as e:  # noqa: BLE001 -- the type is the fixture
            error = type(e).__name__
        meta = dict(case=f"mismatch_{name}", dtype=dtype, shapes=shapes, weights_kind=wk, error=error)
        arrays = dict(meta=np.array(json.dumps(meta)), inputs=inputs)
        if weights is not None:
            arrays["weights"] = np.asarray(weights, dtype=np.float64)
        if expected is not None:
            arrays["expected"] = expected
        path = os.path.join(HERE, meta["case"] + ".npz")
        np.savez_compressed(path, **arrays)
        written.append(os.path.basename(path) + (f" (raises {error})" if error else ""))
    print("\n".join(written))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
