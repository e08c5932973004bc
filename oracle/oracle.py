"""TEST INFRASTRUCTURE ONLY — the checker, never the product.

Python face of the CPU oracle for the aggregation hot path
(reference: dasklearn/gradient_aggregation/fedavg.py:12-26, FedAvg.aggregate).

* ``wreduce(xs, weights, dtype)`` — the plain-C restatement in
  ``fedavg_oracle.c`` (built by ``oracle/Makefile`` into ``oracle/_build``),
  bit-exact to the reference; pinned against tests/golden/ fixtures that were
  produced by running the reference itself (tests/golden/make_golden.py).
* ``reference_weights(n, weights)`` — fedavg.py:14-17 weight rules
  (None / [] -> float(1./N); otherwise length must match) plus the fp32
  rounding that ``w * p1`` applies (fedavg.py:25).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None


def build() -> str:
    """Compile the C oracle (idempotent)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def _load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB_PATH):
        build()
    lib = ctypes.CDLL(_LIB_PATH)
    pp = ctypes.POINTER(ctypes.c_void_p)
    for name in ("oracle_wreduce_f32", "oracle_wreduce_bf16", "oracle_wreduce_fast_f32",
                 "oracle_wreduce_fast_bf16", "oracle_wreduce_f16", "oracle_wreduce_fast_f16"):
        fn = getattr(lib, name)
        fn.argtypes = [pp, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        fn.restype = ctypes.c_int
    for name in ("oracle_mean_f32", "oracle_mean_bf16", "oracle_mean_f16"):
        fn = getattr(lib, name)
        fn.argtypes = [pp, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t]
        fn.restype = ctypes.c_int
    for name in ("oracle_chunk_mean_f32", "oracle_chunk_mean_bf16", "oracle_chunk_mean_f16", "oracle_chunk_mean_f64"):
        fn = getattr(lib, name)
        fn.argtypes = [pp, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        fn.restype = ctypes.c_int
    lib.oracle_chunk_mean_ilp_begin.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_int]
    lib.oracle_chunk_mean_ilp_begin.restype = ctypes.c_size_t
    lib.oracle_chunk_mean_ilp_begin_f64.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_int]
    lib.oracle_chunk_mean_ilp_begin_f64.restype = ctypes.c_size_t
    for name in ("oracle_wreduce_f64", "oracle_wreduce_fast_f64"):
        fn = getattr(lib, name)
        fn.argtypes = [pp, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        fn.restype = ctypes.c_int
    lib.oracle_wreduce_f32_rows.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_size_t]
    lib.oracle_wreduce_f32_rows.restype = ctypes.c_int
    _lib = lib
    return lib


def reference_weights_f64(n: int, weights: Optional[Sequence[float]]) -> np.ndarray:
    """fedavg.py:14-17 weight rules for a double model: the Python floats,
    exact (a double tensor's `w * p1` keeps them as double scalars)."""
    if not weights:
        weights = [float(1.0 / n) for _ in range(n)]
    else:
        assert len(weights) == n
    return np.asarray([float(w) for w in weights], dtype=np.float64)


def reference_weights(n: int, weights: Optional[Sequence[float]]) -> np.ndarray:
    """fedavg.py:14-17: falsy weights -> [float(1./n)]*n, else len must be n.
    Returned rounded to fp32 (the op converts the Python float with RNE)."""
    if not weights:
        weights = [float(1.0 / n) for _ in range(n)]
    else:
        assert len(weights) == n
    return np.asarray([float(w) for w in weights], dtype=np.float64).astype(np.float32)


def _as_rows(xs, np_dtype):
    # 16-bit rows: float16 arrays are taken by their bits, not converted
    rows = [np.ascontiguousarray(np.asarray(x).view(np.uint16) if np.asarray(x).dtype == np.float16
                                 else x, dtype=np_dtype).reshape(-1) for x in xs]
    p = rows[0].size
    for r in rows:
        if r.size != p:
            raise ValueError("all inputs must have the same element count")
    return rows, p


def wreduce(xs, weights, dtype: str = "f32", mode: str = "exact") -> np.ndarray:
    """N-way weighted reduce of flat arrays, reference rounding order.

    xs: sequence of N arrays — float32 for "f32", float64 for "f64", uint16
    bit patterns for "bf16" and "f16". weights: array-like of length N,
    already resolved: fp32 (reference_weights) for f32/bf16/f16, the exact
    doubles (reference_weights_f64) for f64.
    Returns float32 (f32), float64 (f64) or uint16 bit patterns (bf16, f16).
    """
    lib = _load()
    n = len(xs)
    if n < 1:
        raise IndexError("list index out of range")
    w = np.ascontiguousarray(weights, dtype=np.float64 if dtype == "f64" else np.float32)
    if w.size != n:
        raise AssertionError("weights/models length mismatch")
    if dtype == "f64":
        rows, p = _as_rows(xs, np.float64)
        out = np.empty(p, dtype=np.float64)
        fn = lib.oracle_wreduce_f64 if mode == "exact" else lib.oracle_wreduce_fast_f64
    elif dtype == "f32":
        rows, p = _as_rows(xs, np.float32)
        out = np.empty(p, dtype=np.float32)
        fn = lib.oracle_wreduce_f32 if mode == "exact" else lib.oracle_wreduce_fast_f32
    elif dtype in ("bf16", "f16"):
        rows, p = _as_rows(xs, np.uint16)
        out = np.empty(p, dtype=np.uint16)
        fn = getattr(lib, f"oracle_wreduce_{dtype}" if mode == "exact" else f"oracle_wreduce_fast_{dtype}")
    else:
        raise ValueError(f"unsupported dtype {dtype}")
    ptrs = (ctypes.c_void_p * n)(*[r.ctypes.data for r in rows])
    rc = fn(ctypes.cast(ptrs, ctypes.POINTER(ctypes.c_void_p)), n, w.ctypes.data,
            out.ctypes.data, p)
    if rc != 0:
        raise RuntimeError(f"oracle failed rc={rc}")
    return out.view(np.float16) if dtype == "f16" else out


def mean(xs, dtype: str = "f32") -> np.ndarray:
    """Sequential mean (sum from +0, one division; bf16 rounded once):
    torch.mean(torch.stack(xs), 0) while PyTorch's CPU dim-0 reduction is
    sequential (see chunk_mean for its exact order)."""
    lib = _load()
    n = len(xs)
    if n < 1:
        raise IndexError("list index out of range")
    if dtype == "f32":
        rows, p = _as_rows(xs, np.float32)
        out = np.empty(p, dtype=np.float32)
        fn = lib.oracle_mean_f32
    elif dtype in ("bf16", "f16"):
        rows, p = _as_rows(xs, np.uint16)
        out = np.empty(p, dtype=np.uint16)
        fn = getattr(lib, f"oracle_mean_{dtype}")
    else:
        raise ValueError(f"unsupported dtype {dtype}")
    ptrs = (ctypes.c_void_p * n)(*[r.ctypes.data for r in rows])
    if fn(ctypes.cast(ptrs, ctypes.POINTER(ctypes.c_void_p)), n, out.ctypes.data, p) != 0:
        raise RuntimeError("oracle mean failed")
    return out.view(np.float16) if dtype == "f16" else out


def chunk_mean(xs, dtype: str = "f32", threads: int = 4) -> np.ndarray:
    """torch.mean(torch.stack(xs), 0) exactly as PyTorch's CPU kernels compute
    it at `threads` intra-op threads (simulation/conflux/chunk_manager.py:40
    under broker.py:31's torch.set_num_threads(settings.torch_threads)):
    ATen's cascade_sum column order, then one division (fedavg_oracle.c)."""
    lib = _load()
    n = len(xs)
    if n < 1:
        raise IndexError("list index out of range")
    if dtype == "f32":
        rows, p = _as_rows(xs, np.float32)
        out = np.empty(p, dtype=np.float32)
        fn = lib.oracle_chunk_mean_f32
    elif dtype in ("bf16", "f16"):
        rows, p = _as_rows(xs, np.uint16)
        out = np.empty(p, dtype=np.uint16)
        fn = getattr(lib, f"oracle_chunk_mean_{dtype}")
    elif dtype == "f64":  # Vectorized<double>: 4 lanes, 16-column rounding
        rows, p = _as_rows(xs, np.float64)
        out = np.empty(p, dtype=np.float64)
        fn = lib.oracle_chunk_mean_f64
    else:
        raise ValueError(f"unsupported dtype {dtype}")
    ptrs = (ctypes.c_void_p * n)(*[r.ctypes.data for r in rows])
    if fn(ctypes.cast(ptrs, ctypes.POINTER(ctypes.c_void_p)), n, out.ctypes.data, p, threads) != 0:
        raise RuntimeError("oracle chunk mean failed")
    return out.view(np.float16) if dtype == "f16" else out


def wreduce_zip(params_by_model, weights, dtype: str = "f32", mode: str = "exact"):
    """FedAvg.aggregate over models whose parameter lists may differ
    (fedavg.py:23-24): `zip(center.parameters(), m.parameters())` stops at the
    shorter list, so output parameter t folds, in model order, the models that
    have a t-th parameter (models[0] always; extra parameters are ignored),
    and `c1.add_(w * p1)` broadcasts p1 to c1's shape (numpy's broadcast_to
    stands in for torch's: RuntimeError when it does not reach c1's shape).

    params_by_model: per model, the list of its parameter arrays (float32 /
    float64, or uint16 bits for bf16 / f16). weights: the reference's argument
    (None / [] / list), resolved with fedavg.py:14-17 over all N models.
    Returns the list of output arrays in models[0]'s shapes."""
    n = len(params_by_model)
    if n < 1:
        raise IndexError("list index out of range")
    w = reference_weights_f64(n, weights) if dtype == "f64" else reference_weights(n, weights)
    outs = []
    for t, c in enumerate(params_by_model[0]):
        c = np.asarray(c)
        rows, ws = [], []
        for i, ps in enumerate(params_by_model):
            if len(ps) <= t:
                continue
            q = np.asarray(ps[t])
            if q.shape != c.shape:
                try:
                    q = np.broadcast_to(q, c.shape)
                except ValueError as e:
                    raise RuntimeError(f"output with shape {list(c.shape)} doesn't match the broadcast "
                                       f"shape of {list(q.shape)}") from e
            rows.append(np.ascontiguousarray(q).reshape(-1))
            ws.append(w[i])
        outs.append(wreduce(rows, np.asarray(ws), dtype=dtype, mode=mode).reshape(c.shape)
                    if c.size else c.copy())
    return outs


# ---- parameters of different dtypes at one position (fedavg.py:25 with torch's
# type promotion; pinned by tests/golden/mixed_*.npz) ---------------------------

def _mixed_promote(a: str, b: str) -> str:
    """torch.result_type of two floating tensors: equal -> itself; with a
    double -> double; any other pair of f32 / bf16 / f16 -> float32."""
    if a == b:
        return a
    return "f64" if "f64" in (a, b) else "f32"


def _mixed_to_f64(x, dt: str) -> np.ndarray:
    """Stored values (float32 / float64, or uint16 bits for bf16 / f16) as
    exact doubles."""
    x = np.asarray(x)
    if dt == "bf16":
        return bf16_bits_to_f32(x).astype(np.float64)
    if dt == "f16":
        return f16_bits_to_f32(x).astype(np.float64)
    return x.astype(np.float64)


def _mixed_round_f32(x32: np.ndarray, dt: str) -> np.ndarray:
    """A float32 result cast to dt (RNE), returned as exact doubles."""
    x32 = np.asarray(x32, dtype=np.float32)
    if dt == "bf16":
        return bf16_bits_to_f32(f32_to_bf16_bits(x32)).astype(np.float64)
    if dt == "f16":
        return f32_to_f16_bits(x32).astype(np.float64)
    return x32.astype(np.float64)  # f32 (and f64: exact)


def _mixed_round_f64(x64: np.ndarray, dt: str) -> np.ndarray:
    """A double result cast to dt as c10 does: to float (RNE), and for bf16 /
    f16 from that float (their constructors take a float)."""
    if dt == "f64":
        return x64
    with np.errstate(over="ignore"):
        return _mixed_round_f32(x64.astype(np.float32), dt)


def _mixed_encode(acc: np.ndarray, dt: str) -> np.ndarray:
    if dt == "f64":
        return acc
    x32 = acc.astype(np.float32)
    if dt == "bf16":
        return f32_to_bf16_bits(x32)
    if dt == "f16":
        return f32_to_f16_bits(x32).view(np.uint16)
    return x32


def wreduce_mixed(xs, dtypes, weights_f64, out_dtype: str) -> np.ndarray:
    """One output parameter whose inputs differ in dtype (fedavg.py:20-25):
    acc = models[0]'s parameter * 0 in out_dtype (models[0] defines c1, so
    dtypes[0] == out_dtype), then per input, in order,
      prod = w * x in x's dtype: float(w) * x rounded to float and then to x's
             format for f32 / bf16 / f16, the exact double w times x for f64;
      acc  = add_ in the promoted dtype of (out_dtype, x's dtype): a float sum
             (or a double sum with f64 on either side), cast back to out_dtype.
    xs: flat arrays as stored (uint16 bits for bf16 / f16); weights_f64: the
    Python-float weights. Returns out_dtype's storage (uint16 bits for bf16 /
    f16)."""
    if dtypes[0] != out_dtype:
        raise ValueError("models[0]'s parameter defines the output dtype")
    x0 = _mixed_to_f64(xs[0], out_dtype)
    with np.errstate(all="ignore"):
        if out_dtype == "f64":
            acc = x0 * 0.0
        else:
            acc = (x0.astype(np.float32) * np.float32(0.0)).astype(np.float64)
        for x, dt, w in zip(xs, dtypes, weights_f64):
            xv = _mixed_to_f64(x, dt)
            if dt == "f64":
                prod = np.float64(w) * xv
            else:
                prod = _mixed_round_f32(np.float32(w) * xv.astype(np.float32), dt)
            if _mixed_promote(out_dtype, dt) == "f64":
                acc = _mixed_round_f64(acc + prod, out_dtype)
            else:
                acc = _mixed_round_f32(acc.astype(np.float32) + prod.astype(np.float32), out_dtype)
    return _mixed_encode(acc, out_dtype)


def wreduce_zip_mixed(params_by_model, dtypes_by_model, weights):
    """wreduce_zip for models whose parameters may also differ in dtype:
    the zip pairing and broadcasting of wreduce_zip, each output parameter
    folded by wreduce_mixed in models[0]'s dtype. weights: the reference's
    argument (None / [] / list), resolved with fedavg.py:14-17 as doubles."""
    n = len(params_by_model)
    if n < 1:
        raise IndexError("list index out of range")
    w = reference_weights_f64(n, weights)
    outs = []
    for t, c in enumerate(params_by_model[0]):
        c = np.asarray(c)
        rows, dts, ws = [], [], []
        for i, ps in enumerate(params_by_model):
            if len(ps) <= t:
                continue
            q = np.asarray(ps[t])
            if q.shape != c.shape:
                try:
                    q = np.broadcast_to(q, c.shape)
                except ValueError as e:
                    raise RuntimeError(f"output with shape {list(c.shape)} doesn't match the broadcast "
                                       f"shape of {list(q.shape)}") from e
            rows.append(np.ascontiguousarray(q).reshape(-1))
            dts.append(dtypes_by_model[i][t])
            ws.append(w[i])
        outs.append(wreduce_mixed(rows, dts, ws, dtypes_by_model[0][t]).reshape(c.shape)
                    if c.size else c.copy())
    return outs


def chunk_mean_ilp_begin(m: int, n: int, threads: int, dtype: str = "f32") -> int:
    """First column that PyTorch's CPU sum folds in row_sum (ILP) order."""
    if dtype == "f64":
        return int(_load().oracle_chunk_mean_ilp_begin_f64(m, n, threads))
    return int(_load().oracle_chunk_mean_ilp_begin(m, n, threads))


def wreduce_rows_f32(x: np.ndarray, weights) -> np.ndarray:
    """Full-size fp32 fold over a (N, P) C-contiguous block (same arithmetic as
    ``wreduce``; element loop innermost for speed)."""
    lib = _load()
    x = np.ascontiguousarray(x, dtype=np.float32)
    n, p = x.shape
    w = np.ascontiguousarray(weights, dtype=np.float32)
    out = np.empty(p, dtype=np.float32)
    rc = lib.oracle_wreduce_f32_rows(x.ctypes.data, n, w.ctypes.data, out.ctypes.data, p)
    if rc != 0:
        raise RuntimeError(f"oracle failed rc={rc}")
    return out


def f32_to_bf16_bits(x: np.ndarray) -> np.ndarray:
    """RNE fp32 -> bf16 bit patterns (NaN -> 0x7FC0), numpy restatement."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    nan = (u & 0x7FFFFFFF) > 0x7F800000
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    r[nan] = 0x7FC0
    return r


def f32_to_f16_bits(x: np.ndarray) -> np.ndarray:
    """RNE fp32 -> IEEE binary16 (numpy's conversion), as np.float16 arrays
    (same_bits compares them as binary16)."""
    with np.errstate(over="ignore"):  # overflow to inf is the rounding rule
        return np.asarray(x, dtype=np.float32).astype(np.float16)


def f16_bits_to_f32(h: np.ndarray) -> np.ndarray:
    h = np.asarray(h)
    return (h if h.dtype == np.float16 else h.astype(np.uint16).view(np.float16)).astype(np.float32)


def bf16_bits_to_f32(h: np.ndarray) -> np.ndarray:
    return (np.asarray(h, dtype=np.uint16).astype(np.uint32) << 16).view(np.float32)


def same_bits(a: np.ndarray, b: np.ndarray) -> bool:
    """Bit equality with every NaN treated as equal to every NaN (NaN payloads
    differ between the reference's scalar/vector CPU paths and the GPU).
    16-bit formats: np.float16 arrays are IEEE binary16 (if either side is
    float16, a uint16 other side holds binary16 bits); other uint16 arrays
    are bf16 bit patterns."""
    a = np.asarray(a)
    b = np.asarray(b)
    if a.shape != b.shape:
        return False
    if np.float16 in (a.dtype, b.dtype):
        ia = a.view(np.uint16) if a.dtype == np.float16 else a.astype(np.uint16)
        ib = b.view(np.uint16) if b.dtype == np.float16 else b.astype(np.uint16)
        fa, fb = ia.view(np.float16), ib.view(np.float16)
    elif a.dtype == np.uint16:
        fa, fb = bf16_bits_to_f32(a), bf16_bits_to_f32(b)
        ia, ib = a, b
    elif np.float64 in (a.dtype, b.dtype):
        if a.dtype != b.dtype:
            return False
        fa, fb = a, b
        ia, ib = a.view(np.uint64), b.view(np.uint64)
    else:
        fa, fb = a.astype(np.float32), b.astype(np.float32)
        ia, ib = fa.view(np.uint32), fb.view(np.uint32)
    na, nb = np.isnan(fa), np.isnan(fb)
    if not np.array_equal(na, nb):
        return False
    return bool(np.array_equal(ia[~na], ib[~nb]))
