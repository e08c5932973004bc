"""Chunked-model reconstruction: the mean of every chunk
index over its contributors, as Conflux's `reconstruct_from_chunks` task does
(dasklearn/functions.py:142-146 -> simulation/conflux/chunk_manager.py:38-53),
for a ResNet-18/CIFAR-10-sized flat model (11,181,642 fp32), k = 10 chunks
(ConfluxSettings.chunks_in_sample default, conflux/settings.py:11) and m
contributors per index (success_fraction 1: the sample size).

  kernel      dlsim_chunk_mean_batched (PyTorch's CPU order, the product path)
              over device-resident chunks, every index in one launch: HIP
              events over back-to-back launches, algorithmic bytes
              (m + 1) * P * 4 per reconstruction; seq_kernel: the same with
              dlsim_mean_batched (input order), for comparison
  device      ChunkManager.reconstruct_model on device chunks (wall)
  host        the same on host chunks (PCIe-inclusive wall; the reference's case),
              at the box's default threads and at the worker's 4
  cpu_ref     the reference's arithmetic on the CPU: per index
              torch.mean(torch.stack(chunks), 0), then cat + copy, 4 threads

    python scripts/bench_chunks.py            # flat 11 M model, m = 4 and 10
    python scripts/bench_chunks.py --models   # ResNet-18 and GNLeNet state_dicts
    python scripts/bench_chunks.py --kernel-only [--m 4]
                      # the batched chunk-mean launches alone (for rocprofv3
                      # kernel stats and PMC passes of k_chunk_mean_batch)
"""
from __future__ import annotations

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "decentralized-learning-simulator_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402
from torch import nn  # noqa: E402

from dasklearn_amd import _native  # noqa: E402
from dasklearn_amd.arena import aligned_empty, arena_empty, base_align, row_stride  # noqa: E402
from dasklearn_amd.chunk_manager import ChunkManager  # noqa: E402

P = 11_181_642


class Flat(nn.Module):
    def __init__(self):
        super().__init__()
        self.w = nn.Parameter(torch.zeros(P))


def med(f, reps=10, sync=True):
    f()
    if sync:
        torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        if sync:
            torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2]


def cpu_reconstruct(chunks, model):
    means = [torch.mean(torch.stack(cs), dim=0) for cs in chunks]
    flat = torch.cat(means)
    with torch.no_grad():
        off = 0
        for t in model.state_dict().values():
            t.copy_(flat[off:off + t.numel()].view(t.shape))
            off += t.numel()
    return model


def main(ms=(4, 10), kernel_only=False, reps=50):
    dev = torch.device("cuda", 0)
    k = 10
    for m in ms:
        g = torch.Generator().manual_seed(m)
        flats = [torch.randn(P, generator=g) * 0.05 for _ in range(m)]
        host_chunks = [ChunkManager.chunk_model(_wrap(f), k) for f in flats]  # [model][index]
        by_index = [[host_chunks[i][c] for i in range(m)] for c in range(k)]
        dflats = [f.to(dev) for f in flats]
        dev_chunks = [ChunkManager.chunk_model(_wrap(f), k) for f in dflats]
        dev_by_index = [[dev_chunks[i][c] for i in range(m)] for c in range(k)]
        byts = (m + 1) * P * 4
        # kernel only: one batched launch per reconstruction over rotating
        # sets of inputs and outputs whose footprint is >= 1 GiB, so that no
        # launch finds its chunks in the 256 MiB Infinity Cache
        # (round 3) every set lays the m contributors' flat models out as the
        # rows of one allocation (arena.row_stride), each chunk a slice of its
        # model, the means back to back in one output arena, as
        # ChunkManager.reconstruct_model sees them; round 2 cloned each chunk
        # into its own small allocation, which measured 38-62 us for the same
        # m = 4 launch depending on where the allocator put the clones
        sets = max(3, -(-(1 << 30) // byts))
        # round 5: the outputs rotate over >= 1 GiB too (a multiple of the
        # input sets): a few outputs stay in the Infinity Cache and their
        # writes never reach HBM
        out_sets = -(-max(sets, -(-(1 << 30) // (P * 4))) // sets) * sets
        res = {"k": k, "m": m, "params": P, "bytes": byts, "rotating_sets": sets, "rotating_outputs": out_sets}
        stride = row_stride(P, 4)
        rows = aligned_empty(sets * m * stride, torch.float32, dev, base_align(P * 4, 4)).view(sets, m, stride)
        bounds = [(c * (P // k), (c + 1) * (P // k) if c < k - 1 else P) for c in range(k)]
        in_sets, outs = [], []
        for s_ in range(sets):
            for i in range(m):
                rows[s_, i, :P].copy_(dflats[i])
            in_sets.append([[rows[s_, i, b:e] for i in range(m)] for b, e in bounds])
        for _ in range(out_sets):
            o = arena_empty(P, torch.float32, dev)
            outs.append([o[b:e] for b, e in bounds])
        tasks = [[(cs, o) for cs, o in zip(in_sets[j % sets], outs[j])] for j in range(out_sets)]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        legs = (("kernel", lambda ts: _native.chunk_mean_batched(ts, threads=4)),
                ("seq_kernel", _native.mean_batched))
        for key, fn in legs[:1] if kernel_only else legs:
            for s in range(sets):
                fn(tasks[s])
            torch.cuda.synchronize()
            e0.record()
            for r in range(reps):
                fn(tasks[r % out_sets])
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / reps
            res[key + "_us"] = round(us, 2)
            res[key + "_GBps"] = round(byts / us / 1e3, 1)
            res[key + "_frac_of_8TBps"] = round(byts / us / 1e3 / 8000.0, 4)
        if kernel_only:
            print(json.dumps(res), flush=True)
            del dflats, dev_chunks, dev_by_index, in_sets, outs, tasks
            continue
        # per-index launches (the unbatched form) for comparison
        torch.cuda.synchronize()
        e0.record()
        for r in range(reps):
            for cs, o in tasks[r % out_sets]:
                _native.chunk_mean_batched([(cs, o)], threads=4)
        e1.record()
        torch.cuda.synchronize()
        res["per_index_launches_us"] = round(e0.elapsed_time(e1) * 1e3 / reps, 2)
        tgt_d = Flat().to(dev)
        res["device_ms"] = round(med(lambda: ChunkManager.reconstruct_model([list(c) for c in dev_by_index],
                                                                           tgt_d)) * 1e3, 3)
        tgt_h = Flat()
        res["host_ms"] = round(med(lambda: ChunkManager.reconstruct_model([list(c) for c in by_index],
                                                                         tgt_h)) * 1e3, 3)
        res["host_GBps"] = round(byts / (res["host_ms"] * 1e-3) / 1e9, 2)
        nt = torch.get_num_threads()
        torch.set_num_threads(4)
        res["host_4t_ms"] = round(med(lambda: ChunkManager.reconstruct_model([list(c) for c in by_index],
                                                                            tgt_h)) * 1e3, 3)
        tgt_c = Flat()
        res["cpu_ref_4t_ms"] = round(med(lambda: cpu_reconstruct([list(c) for c in by_index], tgt_c),
                                         reps=5, sync=False) * 1e3, 3)
        res["cpu_ref_4t_GBps"] = round(byts / (res["cpu_ref_4t_ms"] * 1e-3) / 1e9, 2)
        torch.set_num_threads(nt)
        print(json.dumps(res), flush=True)
        del dflats, dev_chunks, dev_by_index, in_sets, outs, tasks


class ResNet18(nn.Module):
    """torchvision resnet18(num_classes=10)'s module structure (the reference's
    create_model("cifar10", "resnet18")): 62 parameters, 60 BatchNorm buffers
    (num_batches_tracked int64), 122 state_dict entries, 11,181,642 params."""

    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        blocks, cin = [], 64
        for cout, stride in ((64, 1), (128, 2), (256, 2), (512, 2)):
            for b in range(2):
                s = stride if b == 0 else 1
                blk = nn.Module()
                blk.conv1 = nn.Conv2d(cin, cout, 3, s, 1, bias=False)
                blk.bn1 = nn.BatchNorm2d(cout)
                blk.conv2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
                blk.bn2 = nn.BatchNorm2d(cout)
                if b == 0 and (s != 1 or cin != cout):
                    blk.downsample = nn.Sequential(nn.Conv2d(cin, cout, 1, s, bias=False), nn.BatchNorm2d(cout))
                blocks.append(blk)
                cin = cout
        self.blocks = nn.ModuleList(blocks)
        self.fc = nn.Linear(512, 10)


def resnet_case(dev, m=4, k=10):
    """Conflux's reconstruct on a real state_dict: m peers' ResNet-18 models
    chunked into k pieces, rebuilt into a fresh model (host and device)."""
    torch.manual_seed(0)
    models = [ResNet18() for _ in range(m)]
    for mdl in models:
        with torch.no_grad():
            for t in mdl.state_dict().values():
                if t.is_floating_point():
                    t.copy_(torch.randn(t.shape) * 0.05)
    host_chunks = [ChunkManager.chunk_model(mdl, k) for mdl in models]
    by_index = [[host_chunks[i][c] for i in range(m)] for c in range(k)]
    dev_by_index = [[c.to(dev) for c in cs] for cs in by_index]
    res = {"case": "resnet18_state_dict", "k": k, "m": m, "entries": len(models[0].state_dict())}
    tgt_d = ResNet18().to(dev)
    res["device_ms"] = round(med(lambda: ChunkManager.reconstruct_model([list(c) for c in dev_by_index],
                                                                       tgt_d)) * 1e3, 3)
    tgt_h = ResNet18()
    res["host_ms"] = round(med(lambda: ChunkManager.reconstruct_model([list(c) for c in by_index], tgt_h)) * 1e3, 3)
    nt = torch.get_num_threads()
    torch.set_num_threads(4)
    tgt_c = ResNet18()
    res["cpu_ref_4t_ms"] = round(med(lambda: cpu_reconstruct([list(c) for c in by_index], tgt_c), reps=5,
                                     sync=False) * 1e3, 3)
    torch.set_num_threads(nt)
    return res


def gnlenet_case(dev, m=4, k=10, reps=200):
    """The same on the reference's default model (GNLeNet's module tree,
    14 state_dict entries, 85,354 params): per-task cost, not bandwidth."""
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    from bench_rounds import GNLeNetTree
    torch.manual_seed(0)
    models = [GNLeNetTree() for _ in range(m)]
    host_chunks = [ChunkManager.chunk_model(mdl, k) for mdl in models]
    by_index = [[host_chunks[i][c] for i in range(m)] for c in range(k)]
    dev_by_index = [[c.to(dev) for c in cs] for cs in by_index]
    res = {"case": "gnlenet_state_dict", "k": k, "m": m, "entries": len(models[0].state_dict())}
    tgt_d = GNLeNetTree().to(dev)
    res["device_us"] = round(med(lambda: ChunkManager.reconstruct_model([list(c) for c in dev_by_index], tgt_d),
                                 reps=reps) * 1e6, 1)
    tgt_h = GNLeNetTree()
    res["host_us"] = round(med(lambda: ChunkManager.reconstruct_model([list(c) for c in by_index], tgt_h),
                               reps=reps) * 1e6, 1)
    nt = torch.get_num_threads()
    torch.set_num_threads(4)
    tgt_c = GNLeNetTree()
    res["cpu_ref_4t_us"] = round(med(lambda: cpu_reconstruct([list(c) for c in by_index], tgt_c), reps=reps,
                                     sync=False) * 1e6, 1)
    torch.set_num_threads(nt)
    return res


def _wrap(flat):
    m = Flat()
    m.w = nn.Parameter(flat, requires_grad=False)
    return m


if __name__ == "__main__":
    if "--kernel-only" in sys.argv:
        ms = [int(sys.argv[sys.argv.index("--m") + 1])] if "--m" in sys.argv else [4, 10]
        reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 200
        main(ms, kernel_only=True, reps=reps)
        sys.exit(0)
    if "--models" in sys.argv:  # the two real module trees only
        d = torch.device("cuda", 0)
        print(json.dumps(resnet_case(d)), flush=True)
        print(json.dumps(gnlenet_case(d)), flush=True)
    else:
        main()
    print(json.dumps(resnet_case(torch.device("cuda", 0))), flush=True)
