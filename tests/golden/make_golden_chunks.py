"""Golden vectors for the chunked-model path (Conflux / Shatter) from the REFERENCE.

Runs the reference's own `ChunkManager.chunk_model` and
`ChunkManager.reconstruct_model`
(/root/reference/dasklearn/simulation/conflux/chunk_manager.py:13-53) — the
`chunk` and `reconstruct_from_chunks` tasks of dasklearn/functions.py:136-146 —
on seeded models, at the worker's 4 torch threads (broker.py:31), and writes
inputs and outputs as .npz data next to this script. Skips when
/root/reference is absent.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_chunks.py

fp64 cases (double models) go to chunks_f64/ with meta dtype "f64".

Per case (np.load(..., allow_pickle=False)):
    meta       JSON: case, num_chunks k, contributors per chunk index, shapes,
               torch_version / cpu_capability of the generating process (the
               summation order of torch.mean is pinned to them)
    flat_<p>   flat state_dict of contributing model p (float32, cat order)
    chunks_<c> (m_c, L_c) chunk c of each contributor, in the order given to
               reconstruct_model
    expected   flat state_dict of the reconstructed model
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
    from dasklearn.simulation.conflux.chunk_manager import ChunkManager

    torch.set_num_threads(4)

    class Net(nn.Module):
        def __init__(self, shapes):
            super().__init__()
            self.ps = nn.ParameterList([nn.Parameter(torch.zeros(*s)) for s in shapes])

    shapes = [[1027], [64, 3], [517], [1]]  # 1,733 parameters
    written = []
    # (num_chunks, contributors per chunk index)
    for k, counts in [(1, [2]), (3, [1, 2, 3]), (4, [4, 4, 4, 4]), (2, [5, 8]), (3, [16, 3, 7])]:
        mmax = max(counts)
        g = torch.Generator().manual_seed(100 + k * 10 + mmax)
        models = []
        for p in range(mmax):
            m = Net(shapes)
            with torch.no_grad():
                for q in m.parameters():
                    q.copy_(torch.randn(q.shape, generator=g) * 0.05)
            models.append(m)
        chunked = [ChunkManager.chunk_model(m, k) for m in models]  # the `chunk` task
        # chunk index c receives chunk c from the first counts[c] peers
        chunks = [[chunked[p][c].clone() for p in range(counts[c])] for c in range(k)]
        chunk_arrays = {f"chunks_{c}": torch.stack(chunks[c]).numpy().copy() for c in range(k)}
        target = Net(shapes)  # reconstruct_from_chunks builds a fresh model (functions.py:144)
        out = ChunkManager.reconstruct_model([list(cs) for cs in chunks], target)
        expected = ChunkManager.get_flat_params(out).numpy().copy()
        case = f"chunks_k{k}_m{'-'.join(map(str, counts))}"
        meta = dict(case=case, num_chunks=k, counts=counts, shapes=shapes, torch_threads=4,
                    source="seeded randn*0.05 models (stored)",
                    # the order torch.mean follows is ATen's cascade_sum of THIS
                    # torch build and CPU dispatch: parity is pinned to them
                    torch_version=torch.__version__,
                    cpu_capability=torch.backends.cpu.get_cpu_capability())
        arrays = dict(meta=np.array(json.dumps(meta)), expected=expected, **chunk_arrays)
        for p in range(mmax):
            arrays[f"flat_{p}"] = ChunkManager.get_flat_params(models[p]).numpy().copy()
        path = os.path.join(HERE, "chunks", case + ".npz")
        os.makedirs(os.path.dirname(path), exist_ok=True)
        np.savez_compressed(path, **arrays)
        written.append(path)
    # fp64 models: the same tasks on double parameters,
    # whose torch.mean runs PyTorch's double order (Vectorized<double>: 4
    # lanes, 16-column blocks and rounding). The last case has enough columns
    # that the worker's 4 threads split them (m * n >= 32768).
    shapes64 = [[9001], [50, 50], [7]]  # 11,508 parameters
    for k, counts, shp in [(1, [2], shapes), (3, [1, 2, 3], shapes), (4, [4, 4, 4, 4], shapes),
                           (2, [5, 8], shapes), (3, [16, 3, 7], shapes), (2, [4, 9], shapes64)]:
        mmax = max(counts)
        g = torch.Generator().manual_seed(700 + k * 10 + mmax)
        models = []
        for p in range(mmax):
            m = Net(shp).double()
            with torch.no_grad():
                for q in m.parameters():
                    q.copy_(torch.randn(q.shape, generator=g, dtype=torch.float64) * 0.05)
            models.append(m)
        chunked = [ChunkManager.chunk_model(m, k) for m in models]
        chunks = [[chunked[p][c].clone() for p in range(counts[c])] for c in range(k)]
        chunk_arrays = {f"chunks_{c}": torch.stack(chunks[c]).numpy().copy() for c in range(k)}
        target = Net(shp).double()
        out = ChunkManager.reconstruct_model([list(cs) for cs in chunks], target)
        expected = ChunkManager.get_flat_params(out).numpy().copy()
        assert expected.dtype == np.float64
        case = f"chunks_f64_k{k}_m{'-'.join(map(str, counts))}"
        meta = dict(case=case, num_chunks=k, counts=counts, shapes=shp, torch_threads=4, dtype="f64",
                    source="seeded randn*0.05 double models (stored)",
                    torch_version=torch.__version__,
                    cpu_capability=torch.backends.cpu.get_cpu_capability())
        arrays = dict(meta=np.array(json.dumps(meta)), expected=expected, **chunk_arrays)
        for p in range(mmax):
            arrays[f"flat_{p}"] = ChunkManager.get_flat_params(models[p]).numpy().copy()
        path = os.path.join(HERE, "chunks_f64", case + ".npz")
        os.makedirs(os.path.dirname(path), exist_ok=True)
        np.savez_compressed(path, **arrays)
        written.append(path)
    print("wrote %d fixtures" % len(written))
    return 0


if __name__ == "__main__":
    sys.exit(main())
