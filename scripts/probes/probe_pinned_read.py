"""Probe: CPU read rate of pinned host memory vs pageable, and D2H landing
options for a reconstructed 44.7 MB model (ChunkManager host path).

    python scripts/probes/probe_pinned_read.py
"""
import json
import time

import torch

P = 11_181_642


def t(f, r=7):
    f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(r):
        t0 = time.perf_counter()
        f()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return round(sorted(ts)[r // 2] * 1e3, 3)


def main():
    dev = torch.device("cuda", 0)
    res = {"threads": torch.get_num_threads()}
    pin = torch.randn(P).pin_memory()
    pag = torch.randn(P)
    dst = torch.empty(P)
    d = torch.randn(P, device=dev)
    res["pageable_from_pinned_ms"] = t(lambda: dst.copy_(pin))
    res["pageable_from_pageable_ms"] = t(lambda: dst.copy_(pag))
    k = 10
    n = P // k
    pviews = [pin[i * n:(i + 1) * n] for i in range(k)]
    gviews = [pag[i * n:(i + 1) * n] for i in range(k)]
    res["cat_pinned_views_ms"] = t(lambda: torch.cat(pviews))
    res["cat_pageable_views_ms"] = t(lambda: torch.cat(gviews))
    res["d2h_pinned_ms"] = t(lambda: pin.copy_(d, non_blocking=True))
    res["d2h_pageable_ms"] = t(lambda: dst.copy_(d))
    # ResNet-18-like split into 62 tensors
    sizes = [P // 62] * 61 + [P - 61 * (P // 62)]
    parts = [torch.empty(s) for s in sizes]

    def d2h_parts():
        o = 0
        for p in parts:
            p.copy_(d[o:o + p.numel()])
            o += p.numel()
    res["d2h_62_pageable_ms"] = t(d2h_parts)

    def pin_to_parts():
        o = 0
        for p in parts:
            p.copy_(pin[o:o + p.numel()])
            o += p.numel()
    res["pinned_to_62_parts_ms"] = t(pin_to_parts)
    torch.set_num_threads(4)
    res["t4_pageable_from_pinned_ms"] = t(lambda: dst.copy_(pin))
    res["t4_pageable_from_pageable_ms"] = t(lambda: dst.copy_(pag))
    res["t4_cat_pinned_views_ms"] = t(lambda: torch.cat(pviews))
    res["t4_cat_pageable_views_ms"] = t(lambda: torch.cat(gviews))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
