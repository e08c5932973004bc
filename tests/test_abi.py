"""The C ABI (include/dlsim.h) — CPU checks: the library loads, exports every
declared symbol, host-only entry points work, and argument errors are
reported without touching a GPU."""
from __future__ import annotations

import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT
from dasklearn_amd import _native

HEADER = os.path.join(ROOT, "include", "dlsim.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dlsim_[a-z_0-9]+)\s*\(", src)))


def test_header_matches_binding_list():
    assert declared_functions() == sorted(_native.EXPORTS)


def test_library_exports_every_declared_symbol():
    lib = _native.load()
    for name in declared_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", _native.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (dlsim_\w+)", out))
    assert set(declared_functions()) <= exported


def test_library_is_gfx950_code_object():
    data = open(_native.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_version():
    assert _native.version() >> 16 == 1


@pytest.mark.parametrize("n,world", [(0, 1), (1, 1), (100, 3), (11_181_642, 8), (1000, 7), (63, 4)])
def test_shard_range_partitions_exactly(n, world):
    bounds = [_native.shard_range(n, world, r, 64) for r in range(world)]
    assert bounds[0][0] == 0 and bounds[-1][1] == n
    for (b0, e0), (b1, e1) in zip(bounds, bounds[1:]):
        assert e0 == b1
    for b, e in bounds:
        assert b <= e and b % 64 == 0
    widths = [e - b for b, e in bounds[:-1]]
    if widths:
        assert max(widths) - min(widths) <= 64


def test_shard_range_rejects_bad_rank():
    with pytest.raises(_native.DlsimError):
        _native.shard_range(100, 2, 2, 64)


def _raw_call(n, dtype=0, mode=0, out=ctypes.c_void_p(16)):
    lib = _native.load()
    ptrs = (ctypes.c_void_p * max(n, 1))(*([16] * max(n, 1)))
    w = np.ones(max(n, 1), dtype=np.float32)
    return lib.dlsim_wreduce(ptrs, n, w.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), out, 100,
                             dtype, mode, None)


def test_argument_errors_need_no_gpu():
    lib = _native.load()
    assert _raw_call(0) == -1
    assert b"n must be" in lib.dlsim_last_error()
    assert _raw_call(2, dtype=7) == -2
    assert _raw_call(2, mode=9) == -3
    assert _raw_call(2, out=ctypes.c_void_p(0)) == -1
    # partially overlapping output
    ptrs = (ctypes.c_void_p * 2)(4096, 8192)
    w = np.ones(2, dtype=np.float32)
    rc = lib.dlsim_wreduce(ptrs, 2, w.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                           ctypes.c_void_p(4096 + 64), 1000, 0, 0, None)
    assert rc == -1 and b"overlap" in lib.dlsim_last_error()


def test_zero_elements_is_a_noop():
    lib = _native.load()
    ptrs = (ctypes.c_void_p * 2)(16, 32)
    w = np.ones(2, dtype=np.float32)
    assert lib.dlsim_wreduce(ptrs, 2, w.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                             ctypes.c_void_p(64), 0, 0, 0, None) == 0


def _host_call(numels, stride=4096, staging=4096, rows=8192, out=16, srcs=None, dtype=0, mode=0, n=2):
    lib = _native.load()
    t = len(numels)
    srcs = srcs if srcs is not None else [64] * (n * t)
    w = np.ones(n, dtype=np.float32)
    return lib.dlsim_host_wreduce(n, t, (ctypes.c_void_p * max(len(srcs), 1))(*srcs),
                                  (ctypes.c_size_t * max(t, 1))(*numels),
                                  w.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), staging, rows, stride,
                                  out, None, dtype, mode, 0, 4, None, None, None)


def test_host_wreduce_argument_errors_need_no_gpu():
    """dlsim_host_wreduce rejects bad staging before any HIP call; zero
    elements is a no-op."""
    lib = _native.load()
    assert _host_call([0, 0]) == 0
    assert _host_call([10], dtype=5) == -2
    assert _host_call([10], mode=4) == -3
    assert _host_call([10], n=0) == -1
    assert _host_call([100, 28], stride=64) == -1 and b"row_stride" in lib.dlsim_last_error()
    assert _host_call([10], stride=12) == -1 and b"aligned" in lib.dlsim_last_error()
    assert _host_call([10], staging=4100) == -1
    assert _host_call([10], srcs=[64, 0]) == -1 and b"null source" in lib.dlsim_last_error()
    assert _host_call([10], out=0) == -1


def test_host_chunk_mean_argument_errors_need_no_gpu():
    lib = _native.load()

    def call(fan, numels, staging_elems=1 << 20, dtype=0, cpu_threads=4, staging=4096, outs=None):
        b = len(fan)
        ins = (ctypes.c_void_p * max(sum(fan), 1))(*([64] * max(sum(fan), 1)))
        outs = outs if outs is not None else [128] * b
        return lib.dlsim_host_chunk_mean(b, (ctypes.c_int * b)(*fan), ins, (ctypes.c_size_t * b)(*numels),
                                         staging, 8192, staging_elems, (ctypes.c_void_p * b)(*outs), None,
                                         dtype, cpu_threads, 4, None, None, None)
    assert call([], []) == 0
    assert call([2], [0]) == 0  # nothing to stage
    assert call([2], [10], dtype=9) == -2
    assert call([2], [10], cpu_threads=0) == -1
    assert call([0], [10]) == -1 and b"fan-in" in lib.dlsim_last_error()
    assert call([2, 3], [100, 7], staging_elems=100) == -1 and b"needed" in lib.dlsim_last_error()
    assert _native.staged_rows_elems([100, 7], [2, 3], 4) == 2 * 128 + 3 * 64
    assert call([2, 3], [100, 7], staging_elems=2 * 128 + 3 * 64 - 1) == -1
    assert call([2], [10], staging=4100) == -1 and b"aligned" in lib.dlsim_last_error()
    assert call([2], [10], outs=[0]) == -1 and b"null output" in lib.dlsim_last_error()


def test_library_errors_stay_on_the_calling_thread():
    """dlsim_last_error is thread-local: a failing call on one thread does not
    clobber the message another thread reads (argument errors, no GPU)."""
    import threading
    lib = _native.load()
    for _ in range(20):
        barrier = threading.Barrier(2)
        seen = {}

        def fail_with(tag, n):
            barrier.wait()
            rc = lib.dlsim_wreduce(None, n, None, None, 16, 0, 0, None)
            seen[tag] = (rc, lib.dlsim_last_error().decode())

        ts = [threading.Thread(target=fail_with, args=("zero", 0)),
              threading.Thread(target=fail_with, args=("neg", -3))]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert seen["zero"][0] == -1 and "got 0)" in seen["zero"][1], seen
        assert seen["neg"][0] == -1 and "got -3)" in seen["neg"][1], seen


def test_kernel_name_follows_the_dispatch():
    """dlsim_kernel_name (host logic; the library reads the device's CU
    count, 256 when the query fails, as here without a GPU): the
    deferred-store kernel for fp32 fan-in 3-10 and above 14 (grouped) from
    10 MB per stream, 11-14 from 16 rows of 512 vectors per CU; the tiled
    kernel otherwise (dispatch.hpp use_defer). Fixed fan-in deferred launches
    (fp32 up to 14 inputs) take the form with preloaded leading arguments
    (`k_wreduce_defer_pre`, round 6); the grouped form keeps its name."""
    import torch
    f32, bf16 = torch.float32, torch.bfloat16
    d, t = "dlsim::k_wreduce_defer", "dlsim::k_wreduce_tiles"
    dp, tp = d + "_pre", t
    cus = torch.cuda.get_device_properties(0).multi_processor_count if torch.cuda.is_available() else 256

    def wide(nelem):  # fan-in 11-14: defer from 16 rows of 512 float4 vectors per CU
        return dp if nelem // 4 // 512 >= 16 * cus else tp
    assert _native.kernel_name(8, 11_181_642, f32) == dp  # the north star
    assert _native.kernel_name(8, 11_181_642, f32, _native.DLSIM_FAST) == dp
    assert _native.kernel_name(8, 11_181_642, f32, None) == dp  # dlsim_mean
    assert _native.kernel_name(8, 2_499_999, f32) == tp  # below 10 MB
    assert _native.kernel_name(8, 2_500_000, f32) == dp
    assert _native.kernel_name(3, 11_181_642, f32) == dp
    assert _native.kernel_name(2, 11_181_642, f32) == tp
    assert _native.kernel_name(2, 125_000_000, f32) == tp
    assert _native.kernel_name(12, 5_000_000, f32) == wide(5_000_000)  # < 16 rows per CU on 256 CUs
    assert _native.kernel_name(12, 11_181_642, f32) == wide(11_181_642)
    assert _native.kernel_name(14, 8_388_608, f32) == wide(8_388_608)  # exactly 16 rows per CU on 256 CUs
    assert _native.kernel_name(15, 11_181_642, f32) == d  # the grouped form
    assert _native.kernel_name(100, 11_181_642, f32) == d  # cfg5
    assert _native.kernel_name(100, 2_499_999, f32) == t
    assert _native.kernel_name(8, 11_181_642, bf16) == tp
    assert _native.kernel_name(8, 0, f32) == ""
