"""Host -> device without packing: per call, for 8 host
ResNet-18-shaped models (62 tensors each), wall ms (synchronised per call) of
  pack_pinned   torch.cat into pinned staging + one H2D per model (serial)
  pageable_all  one H2D per tensor straight from pageable memory
  hybrid        H2D straight from pageable memory for tensors >= 64 KiB,
                the small ones packed into pinned staging
  pack_only     the torch.cat into pinned staging alone (no GPU)
  h2d_only      H2D of already packed pinned rows alone"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import torch  # noqa: E402
from inputs import resnet18_cifar10_shapes  # noqa: E402


def med(f, reps=15):
    f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return round(ts[len(ts) // 2] * 1e3, 3)


def main():
    dev = torch.device("cuda", 0)
    n = 8
    shapes = resnet18_cifar10_shapes()
    models = [[torch.randn(s).reshape(-1) for s in shapes] for _ in range(n)]
    sizes = [x.numel() for x in models[0]]
    offs = [0]
    for s in sizes:
        offs.append(offs[-1] + s)
    P = offs[-1]
    pinned = torch.empty((n, P), pin_memory=True)
    d = torch.empty((n, P), device=dev)
    res = {"GB_in": round(n * P * 4 / 1e9, 4)}
    for th in (4, 16):
        torch.set_num_threads(th)

        def pack_pinned():
            for i in range(n):
                torch.cat(models[i], out=pinned[i])
                d[i].copy_(pinned[i], non_blocking=True)
        res[f"pack_pinned_t{th}"] = med(pack_pinned)
        res[f"pack_only_t{th}"] = med(lambda: [torch.cat(models[i], out=pinned[i]) for i in range(n)])
    res["h2d_only"] = med(lambda: [d[i].copy_(pinned[i], non_blocking=True) for i in range(n)])

    def pageable_all():
        for i in range(n):
            for k, x in enumerate(models[i]):
                d[i, offs[k]:offs[k + 1]].copy_(x, non_blocking=True)
    res["pageable_all"] = med(pageable_all)
    for thr in (1 << 16, 1 << 20):
        big = [k for k, s in enumerate(sizes) if s * 4 >= thr]
        small = [k for k, s in enumerate(sizes) if s * 4 < thr]
        nsmall = sum(sizes[k] for k in small)
        stage = torch.empty((n, max(1, nsmall)), pin_memory=True)
        dstage = torch.empty((n, max(1, nsmall)), device=dev)

        def hybrid():
            for i in range(n):
                torch.cat([models[i][k] for k in small], out=stage[i])
                dstage[i].copy_(stage[i], non_blocking=True)
                for k in big:
                    d[i, offs[k]:offs[k + 1]].copy_(models[i][k], non_blocking=True)
        res[f"hybrid_{thr >> 10}KiB"] = med(hybrid)
        res[f"hybrid_{thr >> 10}KiB_nbig"] = len(big)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
