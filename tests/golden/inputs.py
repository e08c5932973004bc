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
