"""Probe: where the ~500 µs of a small host chunk job goes (GNLeNet, k = 10,
m = 4: 40 rows, 1.36 MB in, 340 KB out). Each part timed alone with a sync,
median wall µs:
  sync_empty        a sync of an idle stream
  pack_t1           dlsim_host_pack of the 40 rows into pinned staging
  h2d_sync          one H2D of the staged rows + sync
  mean_dev_sync     dlsim_chunk_mean_batched on device rows + sync
  d2h_sync          one D2H of the 340 KB of means into pinned memory + sync
  mean_hostin_sync  the same launch reading the pinned staging over PCIe (no DMA)
  mean_hostio_sync  ... and writing the means into pinned host memory
  pin_alloc_in/out  torch.empty(pin_memory=True) of the staging / result size
  dev_alloc_in      torch.empty on the device of the staging size
  host_chunk_mean_prealloc_sync  dlsim_host_chunk_mean + sync, buffers reused
  host_chunk_mean_prealloc_t1_sync  the same, packed on the calling thread only
  pipelined         ChunkManager.mean_chunk_indices
  reconstruct       ChunkManager.reconstruct_model (means + copy into the model)
The host-memory launches run only if hipHostGetDevicePointer maps the pinned
buffers at their host addresses.

    python scripts/probes/probe_small_parts.py
"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "scripts"), os.path.join(ROOT, "decentralized-learning-simulator_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from bench_rounds import GNLeNetTree  # noqa: E402
from dasklearn_amd import _native  # noqa: E402
from dasklearn_amd.chunk_manager import ChunkManager  # noqa: E402


def med(f, reps=400):
    for _ in range(20):
        f()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return round(ts[len(ts) // 2] * 1e6, 1)


def mapped(t):
    hip = ctypes.CDLL("libamdhip64.so")
    dp = ctypes.c_void_p()
    rc = hip.hipHostGetDevicePointer(ctypes.byref(dp), ctypes.c_void_p(t.data_ptr()), 0)
    return rc == 0 and dp.value == t.data_ptr()


def main():
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    torch.manual_seed(0)
    m, k = 4, 10
    models = [GNLeNetTree() for _ in range(m)]
    host_chunks = [ChunkManager.chunk_model(mdl, k) for mdl in models]
    by_index = [[host_chunks[i][c] for i in range(m)] for c in range(k)]
    sizes = [cs[0].numel() for cs in by_index]
    al = 64
    rnd = lambda n: (n + al - 1) // al * al  # noqa: E731
    srcs, offs, rows, n_in = [], [], [], 0
    for cs in by_index:
        r = []
        for c in cs:
            srcs.append(c.reshape(-1))
            offs.append(n_in * 4)
            r.append(n_in)
            n_in += rnd(c.numel())
        rows.append(r)
    n_out = sum(sizes)
    stage = torch.empty(n_in, pin_memory=True)
    d_in = torch.empty(n_in, device=dev)
    d_out = torch.empty(n_out, device=dev)
    h_out = torch.empty(n_out, pin_memory=True)
    out_off = [sum(sizes[:i]) for i in range(k)]
    _native.host_pack(srcs, offs, stage.view(torch.uint8), threads=1)
    lib = _native.load()

    def launch(in_base, out_base):
        fan, ptrs, outs = [], [], []
        for r, n, o in zip(rows, sizes, out_off):
            fan.append(len(r))
            ptrs.extend(in_base + x * 4 for x in r)
            outs.append(out_base + o * 4)
        b = len(fan)
        rc = lib.dlsim_chunk_mean_batched(b, (ctypes.c_int * b)(*fan), (ctypes.c_void_p * len(ptrs))(*ptrs),
                                          (ctypes.c_void_p * b)(*outs), (ctypes.c_size_t * b)(*sizes),
                                          _native.dtype_code(torch.float32), 4, ctypes.c_void_p(st.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"dlsim_chunk_mean_batched rc={rc}")

    res = {"model": "gnlenet", "k": k, "m": m, "bytes_in": n_in * 4, "bytes_out": n_out * 4}
    res["sync_empty"] = med(lambda: st.synchronize())
    res["pack_t1"] = med(lambda: _native.host_pack(srcs, offs, stage.view(torch.uint8), threads=1))
    res["h2d_sync"] = med(lambda: (d_in.copy_(stage, non_blocking=True), st.synchronize()))
    res["mean_dev_sync"] = med(lambda: (launch(d_in.data_ptr(), d_out.data_ptr()), st.synchronize()))
    ref = d_out.cpu()
    res["d2h_sync"] = med(lambda: (h_out.copy_(d_out, non_blocking=True), st.synchronize()))
    res["host_mapped"] = mapped(stage) and mapped(h_out)
    if res["host_mapped"]:
        d_out.zero_()
        res["mean_hostin_sync"] = med(lambda: (launch(stage.data_ptr(), d_out.data_ptr()), st.synchronize()))
        res["hostin_equal"] = bool(torch.equal(d_out.cpu(), ref))
        h_out.zero_()
        res["mean_hostio_sync"] = med(lambda: (launch(stage.data_ptr(), h_out.data_ptr()), st.synchronize()))
        res["hostio_equal"] = bool(torch.equal(h_out, ref))
    res["pin_alloc_in"] = med(lambda: torch.empty(n_in, pin_memory=True))
    res["pin_alloc_out"] = med(lambda: torch.empty(n_out, pin_memory=True))
    res["dev_alloc_in"] = med(lambda: torch.empty(n_in, device=dev))
    tasks = [(cs, d_out[o:o + n]) for cs, n, o in zip(by_index, sizes, out_off)]
    houts = [h_out[o:o + n] for n, o in zip(sizes, out_off)]
    res["host_chunk_mean_prealloc_sync"] = med(lambda: (_native.host_chunk_mean(
        tasks, stage, d_in, host_outs=houts, stream=st), st.synchronize()))
    res["host_chunk_mean_prealloc_t1_sync"] = med(lambda: (_native.host_chunk_mean(
        tasks, stage, d_in, host_outs=houts, threads=1, stream=st), st.synchronize()))
    res["pipelined"] = med(lambda: ChunkManager.mean_chunk_indices([list(c) for c in by_index]))
    tgt = GNLeNetTree()
    res["reconstruct"] = med(lambda: ChunkManager.reconstruct_model([list(c) for c in by_index], tgt))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
