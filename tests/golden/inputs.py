"""Deterministic synthetic inputs shared by the golden generator, the tests
and bench.py (numpy PCG64 streams: identical here and on the GPU box, which
run the same image). Data only — no reference code."""
from __future__ import annotations

import numpy as np


def flat_inputs(n: int, p: int, seed: int) -> np.ndarray:
    """(n, p) float32 model-parameter-like values: N(0,1) * 0.05."""
    rng = np.random.Generator(np.random.PCG64(seed))
    return rng.standard_normal((n, p), dtype=np.float32) * np.float32(0.05)


def dirichlet_weights(n: int, seed: int) -> np.ndarray:
    """Dirichlet(1) mixing weights (float64 — the Python floats a caller
    would hand to FedAvg.aggregate)."""
    rng = np.random.Generator(np.random.PCG64(seed + 7))
    return rng.dirichlet(np.ones(n))


def resnet18_cifar10_shapes():
    """parameters() shapes of torchvision resnet18(num_classes=10) — the
    reference's `create_model("cifar10", "resnet18")` (models/__init__.py:27-29):
    62 tensors, 11,181,642 parameters (torchvision is not installed here, so
    the shapes are restated)."""
    shapes = [(64, 3, 7, 7), (64,), (64,)]
    cin = 64
    for cout, stride in ((64, 1), (128, 2), (256, 2), (512, 2)):
        for b in range(2):
            s = stride if b == 0 else 1
            shapes += [(cout, cin, 3, 3), (cout,), (cout,), (cout, cout, 3, 3), (cout,), (cout,)]
            if b == 0 and (s != 1 or cin != cout):
                shapes += [(cout, cin, 1, 1), (cout,), (cout,)]
            cin = cout
    shapes += [(10, 512), (10,)]
    return shapes
