"""Probe (round 4): where one host-chunk reconstruct task's time goes.

The reference's default model (GNLeNet's module tree, 14 state_dict entries),
m = 4 peers' models chunked k = 10 ways (ChunkManager.chunk_model), host
chunks into a host target model, as functions.reconstruct_from_chunks runs
it: ChunkManager.reconstruct_model per call, medians of REPS, then a cProfile
of 300 calls (functions with the most own time) and the CPU reference at 4
threads.

    python scripts/probes/probe_chunk_task.py [reps]
"""
import cProfile
import io
import json
import os
import pstats
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "scripts"), os.path.join(ROOT, "decentralized-learning-simulator_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from bench_rounds import GNLeNetTree  # noqa: E402
from dasklearn_amd.chunk_manager import ChunkManager  # noqa: E402


def cpu_reconstruct(chunks, model):  # the reference's op sequence (chunk_manager.py:34-53)
    for idx in range(len(chunks)):
        chunks[idx] = torch.mean(torch.stack(chunks[idx]), dim=0)
    flat = torch.cat(chunks)
    pointer = 0
    for param in model.state_dict().values():
        numel = param.data.numel()
        param.data.copy_(flat[pointer:pointer + numel].view(param.data.shape))
        pointer += numel
    return model


def med(fn, reps):
    for _ in range(20):
        fn()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    return round(statistics.median(ts) * 1e6, 1)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    torch.set_num_threads(4)
    torch.cuda.set_device(0)
    torch.manual_seed(0)
    m, k = 4, 10
    models = [GNLeNetTree() for _ in range(m)]
    host_chunks = [ChunkManager.chunk_model(mdl, k) for mdl in models]
    by_index = [[host_chunks[i][c] for i in range(m)] for c in range(k)]
    tgt = GNLeNetTree()
    res = {"case": "gnlenet_host_chunks", "m": m, "k": k, "reps": reps}
    res["reconstruct_us"] = med(lambda: ChunkManager.reconstruct_model([list(c) for c in by_index], tgt), reps)
    res["mean_chunk_indices_us"] = med(lambda: ChunkManager.mean_chunk_indices([list(c) for c in by_index]), reps)
    tgt_c = GNLeNetTree()
    res["cpu_ref_4t_us"] = med(lambda: cpu_reconstruct([list(c) for c in by_index], tgt_c), reps)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(300):
        ChunkManager.reconstruct_model([list(c) for c in by_index], tgt)
    pr.disable()
    buf = io.StringIO()
    pstats.Stats(pr, stream=buf).sort_stats("tottime").print_stats(22)
    print(json.dumps(res), flush=True)
    print(buf.getvalue(), flush=True)


if __name__ == "__main__":
    main()
