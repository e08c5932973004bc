"""Probe (round 4): what a worker pays to read a model it has just received.

A reference worker receives each model as torch.multiprocessing file_system
shared memory (worker.py:6): its parameter storages are shm files that the
worker maps afresh, so the first read of every 4 KiB page takes a page fault.
Here a forked producer sends GNLeNet models (a deepcopy of one model, 14
parameter storages, as a train task returns them) through an mp.Queue. The
consumer times the first copy of each model's bytes into a buffer three ways:

  touch     copy through the mapping (what the pack does): faults included
  populate  madvise(MADV_POPULATE_READ) on each storage, then the copy
  pread     open each storage's /dev/shm file and preadv it (no mapping read)

plus the same copy again once the pages are mapped (warm). CPU only.

    python scripts/probes/probe_shm_faults.py [models]
"""
import copy
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "scripts"), os.path.join(ROOT, "decentralized-learning-simulator_amd")):
    sys.path.insert(0, p)

import time  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

MADV_POPULATE_READ = 22


def producer(q, n):
    torch.multiprocessing.set_sharing_strategy("file_system")
    from bench_rounds import GNLeNetTree
    base = GNLeNetTree()
    for _ in range(n):
        m = copy.deepcopy(base)
        m.share_memory()
        q.put(m)
    q.put(None)


def as_bytes(st):
    return np.ctypeslib.as_array((ctypes.c_uint8 * st.nbytes()).from_address(st.data_ptr()))


def copy_all(arrs, buf):
    o = 0
    for a in arrs:
        buf[o:o + a.size] = a
        o += a.size


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    mp.set_sharing_strategy("file_system")
    libc = ctypes.CDLL("libc.so.6", use_errno=True)
    libc.madvise.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    ctx = mp.get_context("fork")
    buf = np.empty(1 << 20, dtype=np.uint8)
    res = {"models": n}
    for mode in ("touch", "populate", "pread"):
        q = ctx.Queue()
        pr = ctx.Process(target=producer, args=(q, n))
        pr.start()
        first, warm, nbytes = [], [], 0
        while True:
            m = q.get()
            if m is None:
                break
            sts = [p.detach().untyped_storage() for p in m.parameters()]
            nbytes = sum(s.nbytes() for s in sts)
            arrs = [as_bytes(s) for s in sts]
            names = [s._share_filename_cpu_()[1].decode() for s in sts] if mode == "pread" else None
            t = time.perf_counter()
            if mode == "pread":
                o = 0
                for name, s in zip(names, sts):
                    fd = os.open("/dev/shm" + name, os.O_RDONLY)
                    os.preadv(fd, [memoryview(buf)[o:o + s.nbytes()]], 0)
                    os.close(fd)
                    o += s.nbytes()
            else:
                if mode == "populate":
                    for s in sts:
                        a = s.data_ptr()
                        lo, hi = a & ~4095, (a + s.nbytes() + 4095) & ~4095
                        libc.madvise(lo, hi - lo, MADV_POPULATE_READ)
                copy_all(arrs, buf)
            first.append(time.perf_counter() - t)
            t = time.perf_counter()
            copy_all(arrs, buf)
            warm.append(time.perf_counter() - t)
            del m, sts, arrs
        pr.join()
        res[mode] = {"first_us": round(statistics.median(first) * 1e6, 1),
                     "warm_us": round(statistics.median(warm) * 1e6, 1), "bytes": nbytes, "storages": 14}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
