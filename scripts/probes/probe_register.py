"""Probe ("zero-copy hipHostRegister of torch-mp shm
storages"): what registering the shared-memory storages a worker receives
would cost, against the pack-and-copy pipeline the package ships.

A reference worker receives each model through a torch.multiprocessing queue
with the file_system strategy (worker.py:6, broker.py:26): every parameter
storage is its own page-aligned mapping of a /dev/shm file, fresh for every
task. Zero-copy DMA (or a kernel reading host memory) needs those pages
page-locked and mapped for the GPU, i.e. hipHostRegister on each storage, per
task, then hipHostUnregister before the storage can go.

This only registers and unregisters (no copy, no kernel reads the memory):
8 ResNet-18-shaped and 7 GNLeNet-shaped models moved to shared memory the way
the queue moves them. Prints one JSON line per model set.

    python scripts/probes/probe_register.py
"""
from __future__ import annotations

import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "decentralized-learning-simulator_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402
import torch.multiprocessing as tmp  # noqa: E402

from bench import GNLENET_SHAPES, resnet18_shapes  # noqa: E402

hipHostRegisterDefault = 0


def hip():
    lib = ctypes.CDLL("libamdhip64.so")
    lib.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    lib.hipHostRegister.restype = ctypes.c_int
    lib.hipHostUnregister.argtypes = [ctypes.c_void_p]
    lib.hipHostUnregister.restype = ctypes.c_int
    return lib


def shm_models(shapes, n):
    tmp.set_sharing_strategy("file_system")
    models = []
    for i in range(n):
        g = torch.Generator().manual_seed(i)
        ts = [(torch.randn(sh, generator=g) * 0.05) for sh in shapes]
        for t in ts:
            t.share_memory_()  # what the queue's reducer does to each storage
        models.append(ts)
    return models


def main():
    torch.cuda.init()
    lib = hip()
    out = []
    for name, shapes, n in (("resnet18", resnet18_shapes(), 8), ("gnlenet", GNLENET_SHAPES, 7)):
        models = shm_models(shapes, n)
        storages = [t.untyped_storage() for ts in models for t in ts]
        nbytes = sum(s.nbytes() for s in storages)
        page = os.sysconf("SC_PAGE_SIZE")
        aligned = sum(1 for s in storages if s.data_ptr() % page == 0)
        reg, unreg = [], []
        for rep in range(7):
            t0 = time.perf_counter()
            for s in storages:
                rc = lib.hipHostRegister(s.data_ptr(), s.nbytes(), hipHostRegisterDefault)
                if rc != 0:
                    raise RuntimeError(f"hipHostRegister failed: {rc}")
            t1 = time.perf_counter()
            for s in storages:
                rc = lib.hipHostUnregister(s.data_ptr())
                if rc != 0:
                    raise RuntimeError(f"hipHostUnregister failed: {rc}")
            t2 = time.perf_counter()
            if rep:
                reg.append((t1 - t0) * 1e3)
                unreg.append((t2 - t1) * 1e3)
        rec = {"models": name, "n": n, "storages": len(storages), "page_aligned": aligned, "bytes": nbytes,
               "register_ms_median": round(statistics.median(reg), 3),
               "unregister_ms_median": round(statistics.median(unreg), 3),
               "register_GBps": round(nbytes / (statistics.median(reg) * 1e-3) / 1e9, 2),
               "note": "hipHostRegister + hipHostUnregister of every shm parameter storage of one task; "
                       "no copy and no kernel touches the memory"}
        print(json.dumps(rec), flush=True)
        out.append(rec)
    return 0


if __name__ == "__main__":
    sys.exit(main())
