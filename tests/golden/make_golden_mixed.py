"""Golden vectors for models whose parameters at one position differ in dtype,
from the REFERENCE.

fedavg.py:20-25 (/root/reference/dasklearn/gradient_aggregation/fedavg.py)
seeds each output parameter as models[0]'s (`deepcopy`, then `mul_(0)`) and
runs `c1.add_(w * p1)` with torch's type promotion: the product is taken in
p1's dtype, the in-place add in the promoted dtype of (c1, product), rounded
back into c1's dtype. This script runs the reference's own
``FedAvg.aggregate`` on such models and writes inputs and outputs as .npz
fixtures (``mixed_*.npz``) next to it. Only data is written; no reference
source is copied. Skips (exit 0) when /root/reference is absent (e.g. on the
GPU box).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_mixed.py

Fixture layout (np.load(..., allow_pickle=False)):
    meta      0-d unicode array, JSON: case, shapes (per model, its parameter
              shapes in parameters() order), dtypes (per model, the dtype name
              of each parameter: f32 / bf16 / f16 / f64), weights_kind, error
              (the exception type name the reference raised, or null)
    x{i}_{t}  parameter t of model i, flattened (float32 / float64, or uint16
              bits for bf16 / f16)
    weights   float64, if weights_kind == "list"
    y{t}      output parameter t, flattened, in models[0]'s dtype (absent
              when the reference raised)
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
        def __init__(self, shapes, dtypes):
            super().__init__()
            self.ps = nn.ParameterList([nn.Parameter(torch.zeros(s, dtype=TDT[d])) for s, d in zip(shapes, dtypes)])

    def to_np(t):
        t = t.detach().contiguous().reshape(-1)
        if t.dtype in (torch.bfloat16, torch.float16):
            return t.view(torch.int16).numpy().view(np.uint16).copy()
        return t.numpy().copy()

    rng = np.random.default_rng(5151)
    S = [[300], [7, 33], [5]]  # three parameters per model

    def same(d, k=3):
        return [d] * k

    cases = [
        # (name, per-model shapes, per-model dtypes, weights kind, value scale, special values)
        ("f32_bf16_f16", [S, S, S], [same("f32"), same("bf16"), same("f16")], "list", 0.05, False),
        ("bf16_f32", [S, S], [same("bf16"), same("f32")], "list", 0.05, False),
        ("bf16_f32_bf16_none", [S, S, S], [same("bf16"), same("f32"), same("bf16")], "none", 0.05, False),
        ("f16_bf16_f32", [S, S, S], [same("f16"), same("bf16"), same("f32")], "list", 0.05, False),
        ("f32_f64", [S, S, S], [same("f32"), same("f64"), same("f32")], "list", 0.05, False),
        ("f64_f32_bf16", [S, S, S], [same("f64"), same("f32"), same("bf16")], "list", 0.05, False),
        ("bf16_f64", [S, S], [same("bf16"), same("f64")], "list", 0.05, False),
        ("f16_f64_none", [S, S], [same("f16"), same("f64")], "none", 0.05, False),
        ("per_param", [S, S, S], [["f32", "bf16", "f16"], ["bf16", "f32", "f64"], ["f16", "f64", "f32"]], "list",
         0.05, False),
        ("mixed_and_fewer", [S, S[:2], S[:1]], [same("f32"), ["bf16", "f16"], ["f64"]], "list", 0.05, False),
        ("mixed_broadcast", [[[4, 6], [3]], [[6], [1]], [[1, 6], [3]]], [["f32", "bf16"], ["bf16", "f32"],
                                                                           ["f16", "bf16"]], "list", 0.05, False),
        ("big_weights_f16_overflow", [S, S, S], [same("f32"), same("f16"), same("bf16")], "big", 30000.0, False),
        ("specials", [S, S, S], [same("f32"), same("bf16"), same("f16")], "list", 0.05, True),
        ("ten_models", [S] * 10, [same(["f32", "bf16", "f16", "f64"][i % 4]) for i in range(10)], "list", 0.05,
         False),
    ]
    written = []
    for name, shapes, dtypes, wk, scale, special in cases:
        n = len(shapes)
        models = []
        for sh, dts in zip(shapes, dtypes):
            m = Shaped(sh, dts)
            with torch.no_grad():
                for p in m.parameters():
                    v = rng.standard_normal(p.numel()) * scale
                    if special and p.numel() >= 8:
                        v[:8] = [np.inf, -np.inf, np.nan, 0.0, -0.0, 1e-40, 7e4, -3e38]
                    p.copy_(torch.from_numpy(v).to(p.dtype).view_as(p))
            models.append(m)
        if wk == "list":
            weights = [float(w) for w in rng.dirichlet(np.ones(n))]
        elif wk == "big":
            weights = [2.5, -1.75, 3.0][:n]
        else:
            weights = None
        error, outs = None, None
        try:
            out = FedAvg.aggregate(models, weights)
            outs = [to_np(p) for p in out.parameters()]
        except Exception as e:  # noqa: BLE001 -- the type is the fixture
            error = type(e).__name__
        meta = dict(case=f"mixed_{name}", shapes=shapes, dtypes=dtypes, weights_kind=wk, error=error)
        arrays = dict(meta=np.array(json.dumps(meta)))
        for i, m in enumerate(models):
            for t, p in enumerate(m.parameters()):
                arrays[f"x{i}_{t}"] = to_np(p)
        if weights is not None:
            arrays["weights"] = np.asarray(weights, dtype=np.float64)
        if outs is not None:
            for t, y in enumerate(outs):
                arrays[f"y{t}"] = y
        path = os.path.join(HERE, meta["case"] + ".npz")
        np.savez_compressed(path, **arrays)
        written.append(os.path.basename(path) + (f" (raises {error})" if error else ""))
    print("\n".join(written))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
