"""Probe (round 6): why does one rotating input set of the 8-rank slice run
~20 % faster than the others? In round 6's traces of `bench.py --slice-of 8`
(8 x 1,397,760 fp32, 22 sets carved from one allocation, outputs rotating over
198 buffers) every dispatch on set 0 took 7.4-8.0 us and every other set's
9.6-10.0 (profiles/r06_final/prof/ns_s8_buckets.json, r06_rehearse/).

Here one process builds the slice's sets three ways and times K launches of
each set alone (outputs rotating as in the bench), HIP events:
  bench     the bench's layout: every set in one allocation, set s at
            s * 8 rows (row stride arena.row_stride: 256-B rounding)
  aligned   the same allocation with every set's first row on a 2 MiB boundary
  per_set   each set its own allocation (arena.resident_empty)
Prints one JSON line per layout: the per-set means and their spread.
`--offsets` places one set at 21 offsets into a 4 GiB block instead.

    python scripts/probes/probe_slice_sets.py [K]
    python scripts/probes/probe_slice_sets.py --offsets
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "decentralized-learning-simulator_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402

import bench  # noqa: E402
from dasklearn_amd import _native  # noqa: E402
from dasklearn_amd.arena import arena_empty, resident_empty, row_stride  # noqa: E402

N = 8
dev = torch.device("cuda", 0)


def layouts(p, sets):
    stride = row_stride(p, 4)
    set_elems = N * stride
    al = (2 << 20) // 4
    aligned_set = -(-set_elems // al) * al
    keep = []
    one = resident_empty(sets * set_elems, torch.float32, dev, 256)
    keep.append(one)
    yield "bench", [one[s * set_elems:(s + 1) * set_elems].view(N, stride) for s in range(sets)], keep
    two = resident_empty(sets * aligned_set + al, torch.float32, dev, 2 << 20)
    keep.append(two)
    yield "aligned", [two[s * aligned_set:s * aligned_set + set_elems].view(N, stride) for s in range(sets)], keep
    per = [resident_empty(set_elems, torch.float32, dev, 256).view(N, stride) for _ in range(sets)]
    keep.append(per)
    yield "per_set", per, keep


def main():
    k_steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    b, e = _native.shard_range(bench.RESNET18_P, 8, 0, 64)
    p = e - b
    sets, n_out = 22, 198
    w32 = _native.fp32_weights(bench.weights_for("dirichlet", N))
    outs = [arena_empty(p, torch.float32, dev) for _ in range(n_out)]
    g = torch.Generator(device=dev).manual_seed(1)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for name, rows, keep in layouts(p, sets):
        for r in rows:
            r[:, :p].copy_(torch.randn((N, p), generator=g, device=dev) * 0.05)
        per_set = []
        for s in range(sets):
            plans = [_native.ReducePlan([rows[s][i, :p] for i in range(N)], w32, outs[j]) for j in range(s, n_out, sets)]
            for k in range(10):
                plans[k % len(plans)].launch()
            torch.cuda.synchronize()
            e0.record()
            for k in range(k_steps):
                plans[k % len(plans)].launch()
            e1.record()
            torch.cuda.synchronize()
            per_set.append(round(e0.elapsed_time(e1) * 1e3 / k_steps, 3))
        base = [rows[s].data_ptr() % (2 << 20) for s in range(sets)]
        print(json.dumps({"layout": name, "per_set_us": per_set, "min": min(per_set), "max": max(per_set),
                          "mean": round(sum(per_set) / sets, 3), "base_mod_2MiB": base}), flush=True)
        del keep


def offsets_main(k_steps=200):
    """`--offsets`: one 4 GiB contiguous block, the slice's set placed at every
    192 MiB step into it (2 MiB aligned), each timed alone; does the fast set
    follow the offset into the first allocation (a translation fragment or a
    physical region) or something else? PROBE_ORDER=A0,A10,B0,... visits
    offsets (192 MiB steps) of blocks A, B, ... (each allocated on first use)
    in any order; PROBE_FILL=each (fill a set just before timing it) or all
    (fill a whole block when it is allocated); the token X copies 2 x 1 GiB
    with ordinary loads and stores (evicts the caches) before the next set."""
    b, e = _native.shard_range(bench.RESNET18_P, 8, 0, 64)
    p = e - b
    stride = row_stride(p, 4)
    set_elems = N * stride
    w32 = _native.fp32_weights(bench.weights_for("dirichlet", N))
    outs = [arena_empty(p, torch.float32, dev) for _ in range(9)]
    blocks = {}
    step = (192 << 20) // 4
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = []
    order = os.environ.get("PROBE_ORDER", ",".join(f"A{k}" for k in range(21))).split(",")
    fill = os.environ.get("PROBE_FILL", "each")
    for tok in order:
        if tok == "X":  # stream 2 x 1 GiB through the caches with ordinary copies
            src = torch.empty((1 << 30) // 4, device=dev).normal_()
            dst = torch.empty_like(src)
            for _ in range(2):
                dst.copy_(src)
            torch.cuda.synchronize()
            del src, dst
            res.append(("X", None, None))
            continue
        blk, k = tok[0], int(tok[1:])
        if blk not in blocks:
            blocks[blk] = resident_empty((4 << 30) // 4, torch.float32, dev, 2 << 20)
            if fill == "all":
                blocks[blk].normal_(0, 0.05)
        rows = blocks[blk][k * step:k * step + set_elems].view(N, stride)
        if fill == "each":
            rows[:, :p].normal_(0, 0.05)
        plans = [_native.ReducePlan([rows[i, :p] for i in range(N)], w32, o) for o in outs]
        for j in range(10):
            plans[j % 9].launch()
        torch.cuda.synchronize()
        e0.record()
        for j in range(k_steps):
            plans[j % 9].launch()
        e1.record()
        torch.cuda.synchronize()
        res.append((tok, k * 192, round(e0.elapsed_time(e1) * 1e3 / k_steps, 3)))
    print(json.dumps({"layout": "offsets_in_4GiB", "fill": fill,
                      "base_va_mod_1GiB": {b: t.data_ptr() % (1 << 30) for b, t in blocks.items()},
                      "block_offset_MiB_us": res}), flush=True)


if __name__ == "__main__":
    if "--offsets" in sys.argv:
        offsets_main()
    else:
        main()
