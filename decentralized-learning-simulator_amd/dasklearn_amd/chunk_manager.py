"""ChunkManager — mirror of dasklearn/simulation/conflux/chunk_manager.py:10-53.

The chunked-model algorithms (Conflux, Shatter) split a model's flat
state_dict into k chunks (`chunk` task, functions.py:136-140), send chunk c to
some peers, and rebuild a model from the received chunks by averaging each
chunk index over its contributors (`reconstruct_from_chunks` task,
functions.py:142-146). That average is a second N-way reduce of the hot path
(SURVEY.md §8f row 2); here it runs on the GPU through `dlsim_chunk_mean_batched`.

* `chunk_model` / `get_flat_params` are pure data movement (a torch.cat of the
  state_dict and slices of it) and are restated with the same tensor ops, on
  whatever device the model lives.
* `reconstruct_model`: per chunk index, `torch.mean(torch.stack(chunks), 0)`
  (chunk_manager.py:38-40) becomes one task of a `dlsim_chunk_mean_batched`
  launch (every chunk index of the reconstruction in one launch), computed in
  PyTorch's own CPU summation order (ATen's cascade_sum column classes at the
  calling process's torch.get_num_threads(), which in the worker is
  settings.torch_threads, broker.py:31) and divided once: bit-identical to the
  reference for every contributor count (tests/test_gpu_chunks.py against the
  reference's fixtures; the order itself is pinned against torch.mean in
  tests/test_chunk_mean_order.py).
  As in the reference, `chunks[c]` is replaced in place by its mean and the
  result is copied into `model.state_dict()` (parameters and buffers).

Scope of that parity claim: the order restated is ATen's CPU cascade_sum of
torch 2.10 with AVX2/AVX512 dispatch (8-float vectors), the build the
reference's chunk fixtures were generated with (their meta records
torch_version and cpu_capability). The reference pins torch~=2.1.2
(requirements.txt:1); a reference worker on another torch or ISA may order
the sum differently, so `order_scope()` names such a process and the first
reconstruction in it warns (ParityScopeWarning).
"""
from __future__ import annotations

import warnings
from typing import List, Optional

import torch
from torch import nn

from . import _native
from .arena import _elem_size, _pyhost, _side_streams, _target_device, arena_empty


ORDER_PINNED_TORCH = "2.10"
ORDER_PINNED_CPU_CAPABILITIES = ("AVX2", "AVX512")


class ParityScopeWarning(UserWarning):
    """The running process is outside the torch build / CPU dispatch the chunk
    mean order was pinned against."""


def order_scope(version: Optional[str] = None, capability: Optional[str] = None) -> Optional[str]:
    """None when this process's torch and CPU dispatch are those the chunk
    mean order is pinned to, else a message saying what differs."""
    version = torch.__version__ if version is None else version
    if capability is None:
        try:
            capability = torch.backends.cpu.get_cpu_capability()
        except Exception:
            capability = "unknown"
    why = []
    if ".".join(version.split("+")[0].split(".")[:2]) != ORDER_PINNED_TORCH:
        why.append(f"torch {version} (order pinned against {ORDER_PINNED_TORCH})")
    if capability not in ORDER_PINNED_CPU_CAPABILITIES:
        why.append(f"CPU capability {capability} (pinned: {'/'.join(ORDER_PINNED_CPU_CAPABILITIES)})")
    if not why:
        return None
    return ("chunk means follow ATen's cascade_sum order of the pinned build; this process runs "
            + " and ".join(why) + ": the reference on this build may sum in another order")


_SCOPE_CHECKED = False


def _check_order_scope() -> None:
    global _SCOPE_CHECKED
    if _SCOPE_CHECKED:
        return
    _SCOPE_CHECKED = True
    msg = order_scope()
    if msg:
        warnings.warn(msg, ParityScopeWarning, stacklevel=3)


class ChunkManager:

    @staticmethod
    def chunk_model(model: nn.Module, num_chunks: int) -> List[torch.Tensor]:
        flat_params = ChunkManager.get_flat_params(model)
        total_elements = flat_params.numel()
        chunk_size = total_elements // num_chunks
        chunks = [flat_params[i * chunk_size:(i + 1) * chunk_size] for i in range(num_chunks)]
        if total_elements % num_chunks != 0:  # the last chunk takes the remainder
            chunks[-1] = torch.cat([chunks[-1], flat_params[num_chunks * chunk_size:]])
        return chunks

    @staticmethod
    def get_flat_params(model: nn.Module) -> torch.Tensor:
        return torch.cat([t.data.view(-1) for t in model.state_dict().values()])

    @staticmethod
    def mean_chunks(chunks_at_idx: List[torch.Tensor], device=None) -> torch.Tensor:
        """torch.mean(torch.stack(chunks_at_idx), dim=0) on the GPU; the result
        lives where the first chunk lives."""
        return ChunkManager.mean_chunk_indices([chunks_at_idx], device)[0]

    @staticmethod
    def mean_chunk_indices(chunks: List[List[torch.Tensor]], device=None) -> List[torch.Tensor]:
        """[torch.mean(torch.stack(cs), dim=0) for cs in chunks]. Device chunks
        are read in place, every chunk index in one batched launch per dtype
        (dlsim_chunk_mean_batched); host chunks (the reference's case) go
        through dlsim_host_chunk_mean (threaded pack into pinned staging,
        per-row H2D, per-index mean and D2H, overlapped). Each result lives
        where its first chunk lives."""
        _check_order_scope()
        fast = _fast_means(chunks, device)
        if fast is not None:
            return fast[0]
        for cs in chunks:
            first = cs[0]
            for c in cs:
                if c.shape != first.shape or c.dtype != first.dtype:
                    raise RuntimeError("stack expects each tensor to be equal size")
        dev = _target_device([cs[0] for cs in chunks], device)
        results: List[torch.Tensor] = [None] * len(chunks)
        with torch.no_grad():
            by_dtype = {}
            for ci, cs in enumerate(chunks):
                by_dtype.setdefault(cs[0].dtype, []).append(ci)
            for dt, idxs in by_dtype.items():
                esz = torch.empty((), dtype=dt).element_size()
                al = 256 // esz
                rnd = lambda k: (k + al - 1) // al * al  # noqa: E731
                # outputs back to back (no padding) when every chunk but the last
                # keeps the next one 16-B aligned: consecutive chunk indices then
                # form one flat buffer that reconstruct_model uses without a cat
                sizes = [chunks[ci][0].numel() for ci in idxs]
                tight = all(k * esz % 16 == 0 for k in sizes[:-1])
                out_off, n_out = [], 0
                for k in sizes:
                    out_off.append(n_out)
                    n_out += k if tight else rnd(k)
                on_dev = all(c.is_cuda and c.device == dev for ci in idxs for c in chunks[ci])
                if on_dev:
                    d_out = arena_empty(max(n_out, 1), dt, dev)  # contiguous from 4 MiB
                    tasks = []
                    for ci, k, o in zip(idxs, sizes, out_off):
                        out = d_out[o:o + k]
                        results[ci] = out.view(chunks[ci][0].shape)
                        if k:
                            tasks.append(([c.reshape(-1).contiguous() for c in chunks[ci]], out))
                    _native.chunk_mean_batched(tasks)
                    continue
                host_out_size = sum(sizes)
                host = torch.empty(max(host_out_size, 1), dtype=dt, pin_memory=True)
                host_off = [0]
                for k in sizes:
                    host_off.append(host_off[-1] + k)
                d_out = torch.empty(max(n_out, 1), dtype=dt, device=dev)
                stream = torch.cuda.current_stream(dev)
                if all(c.get_device() == -1 for ci in idxs for c in chunks[ci]):
                    # host chunks (the reference's case): dlsim_host_chunk_mean
                    # packs the rows on the library's threads, starts each
                    # row's H2D as soon as it is packed, runs each index's mean
                    # once its rows are on the device and copies it back, the
                    # host result back to back (reconstruct_model then uses it
                    # without a cat)
                    fan = [len(chunks[ci]) for ci in idxs]
                    need = _native.staged_rows_elems(sizes, fan, esz)
                    stage = torch.empty(max(need, 1), dtype=dt, pin_memory=True)
                    d_in = torch.empty(max(need, 1), dtype=dt, device=dev)
                    big = need * esz >= PIPELINE_SIDE_STREAM_BYTES
                    h2d, d2h = _side_streams(dev) if big else (None, None)
                    _native.host_chunk_mean(
                        [(chunks[ci], d_out[o:o + k]) for ci, k, o in zip(idxs, sizes, out_off)],
                        stage, d_in, host_outs=[host[h:h + k] for k, h in zip(sizes, host_off)],
                        stream=stream, h2d_stream=h2d, d2h_stream=d2h)
                    stream.synchronize()
                else:
                    _mixed_means(chunks, idxs, sizes, out_off, host, host_off, d_out, dt, dev, rnd, tight)
                for ci, o, h in zip(idxs, out_off, host_off):
                    first = chunks[ci][0]
                    src = host[h:h + first.numel()] if not first.is_cuda else d_out[o:o + first.numel()]
                    results[ci] = src.view(first.shape)
        return results

    @staticmethod
    def reconstruct_model(chunks: List[List[torch.Tensor]], model: nn.Module) -> nn.Module:
        for idx in range(len(chunks)):
            assert chunks[idx], "No chunks received at index %d!" % idx
        _check_order_scope()
        # host chunks: the means' copies are still in flight when this
        # returns; the state_dict walk below runs meanwhile, and nothing reads
        # the means before `pending` is synchronised
        fast = _fast_means(chunks, None, sync=False)
        pending = None
        if fast is not None:
            means, flat_params, pending = fast
        else:
            means, flat_params = ChunkManager.mean_chunk_indices(chunks), None
        try:
            for chunk_idx in range(len(chunks)):
                chunks[chunk_idx] = means[chunk_idx]
            if flat_params is None:
                flat_params = _span(chunks)
            if flat_params is None:
                flat_params = torch.cat(chunks)
            # chunk_manager.py:45-52: copy consecutive slices of the flat
            # means into every state_dict tensor (parameters and buffers, with
            # the dtype conversion of copy_). The copies go out as one
            # torch._foreach_copy_ (a few multi-tensor launches for a device
            # model instead of one per tensor) unless two destinations share
            # memory: a tied parameter is in state_dict() under each of its
            # names, and the reference's copies run in order (the later one
            # wins), which a multi-tensor launch does not guarantee.
            dsts, srcs = [], []
            pointer = 0
            for param in model.state_dict().values():
                numel = param.data.numel()
                dsts.append(param.data)
                srcs.append(flat_params[pointer:pointer + numel].view(param.data.shape))
                pointer += numel
        finally:
            if pending is not None:
                pending[0].synchronize()  # the means are complete (pending[1:] kept their buffers alive)
                pending = None
        with torch.no_grad():
            if dsts and all(d.device == flat_params.device for d in dsts) and not _overlapping(dsts):
                torch._foreach_copy_(dsts, srcs)
            else:
                for d, src in zip(dsts, srcs):
                    d.copy_(src)
        return model


def _fast_means(chunks, device, sync: bool = True):
    """mean_chunk_indices for the common case, validated in one C pass
    (_pyhost.chunk_scan) instead of Python loops over every contributor:
    one dtype, every chunk contiguous and non-empty, all on the host (the
    reference's case: dlsim_host_chunk_mean) or all on the target GPU
    (dlsim_chunk_mean_batched). Returns (means, flat) — flat the means back to
    back as one tensor (torch.cat(means) without the copy), or None when the
    device outputs are padded — or None for any other case (the general path
    below then runs). sync=False: (means, flat, pending) instead, pending None
    or (stream, buffers...) for host chunks whose copies are still in flight:
    the caller synchronises pending[0] before reading the means and keeps
    the tuple (the staging the DMAs read) alive until then."""
    same, place, dix, numels, fans, ptrs = _pyhost.chunk_scan(chunks)  # raises as torch.stack would
    if not chunks or not same or ptrs is None or place == 0 or 0 in numels:
        return None
    first0 = chunks[0][0]
    dt = first0.dtype
    dev = _target_device([first0], device)
    if place == 2 and dev.index != dix:
        return None
    esz = _elem_size(dt)
    al = 256 // esz
    # outputs back to back when every chunk but the last keeps the next one
    # 16-B aligned (as the general path lays them out)
    tight = all(k * esz % 16 == 0 for k in numels[:-1])
    out_off, n_out = [], 0
    for k in numels:
        out_off.append(n_out)
        n_out += k if tight else (k + al - 1) // al * al
    code = _native.dtype_code(dt, single_task=True)
    threads = torch.get_num_threads()
    pending = None
    d_out = arena_empty(n_out, dt, dev)  # contiguous from 4 MiB
    d0 = d_out.data_ptr()
    d_ptrs = [d0 + o * esz for o in out_off]
    with torch.no_grad():
        if place == 2:
            _native.chunk_mean_batched_raw(fans, ptrs, d_ptrs, numels, code, threads,
                                           torch._C._cuda_getCurrentRawStream(dev.index))
            res, offs, flat = d_out, out_off, (d_out if tight else None)
        else:
            total = sum(numels)
            host = torch.empty(total, dtype=dt, pin_memory=True)
            h0 = host.data_ptr()
            offs, h = [], 0
            for k in numels:
                offs.append(h)
                h += k
            need = _native.staged_rows_elems(numels, fans, esz)
            stage = torch.empty(need, dtype=dt, pin_memory=True)
            d_in = torch.empty(need, dtype=dt, device=dev)
            stream = torch.cuda.current_stream(dev)
            h2d, d2h = _side_streams(dev) if need * esz >= PIPELINE_SIDE_STREAM_BYTES else (None, None)
            _native.host_chunk_mean_raw(fans, ptrs, numels, stage.data_ptr(), d_in.data_ptr(), need, d_ptrs,
                                        [h0 + o * esz for o in offs], code, threads, threads, stream.cuda_stream,
                                        None if h2d is None else h2d.cuda_stream,
                                        None if d2h is None else d2h.cuda_stream)
            if sync:
                stream.synchronize()
            else:
                pending = (stream, stage, d_in, d_out)
            res, flat = host, host
    means = []
    for cs, o, k in zip(chunks, offs, numels):
        m = res[o:o + k]
        f = cs[0]
        means.append(m if f.dim() == 1 else m.view(f.shape))
    return (means, flat) if sync else (means, flat, pending)


def _overlapping(ts: List[torch.Tensor]) -> bool:
    """Whether any two of the tensors (on one device) share bytes."""
    spans = sorted((t.data_ptr(), t.data_ptr() + t.numel() * t.element_size()) for t in ts if t.numel())
    return any(b0 < a1 for (_, a1), (b0, _) in zip(spans, spans[1:]))


def _span(ts: List[torch.Tensor]):
    """A flat view equal to torch.cat(ts) when the ts are contiguous and lie
    back to back in one storage (the host means of mean_chunk_indices), else
    None. Saves the cat's fresh allocation, whose first-touch page faults cost
    ~9 ms for a ResNet-18-sized model (scripts/probe_pinned_read.py)."""
    t0 = ts[0]
    if t0.dim() != 1:
        return None
    total, nxt = 0, t0.data_ptr()
    for t in ts:
        if t.dim() != 1 or not t.is_contiguous() or t.dtype != t0.dtype or t.device != t0.device \
                or t.untyped_storage().data_ptr() != t0.untyped_storage().data_ptr() or t.data_ptr() != nxt:
            return None
        nxt += t.numel() * t.element_size()
        total += t.numel()
    return t0.as_strided((total,), (1,))


# Host chunk means go through the side copy streams above this many staged
# bytes (below it the events cost more than the overlap saves).
PIPELINE_SIDE_STREAM_BYTES = 4 << 20


def _mixed_means(chunks, idxs, sizes, out_off, host, host_off, d_out, dt, dev, rnd, tight):
    """Chunk means when some contributors are on a device and some on the
    host: rows at 256-B aligned offsets of one pinned staging buffer (a CUDA
    row copies through it), one H2D per row, one batched launch, then the
    back-to-back host result."""
    in_off, n_in = [], 0
    for ci, k in zip(idxs, sizes):
        offs = []
        for _ in chunks[ci]:
            offs.append(n_in)
            n_in += rnd(k)
        in_off.append(offs)
    stage = torch.empty(max(n_in, 1), dtype=dt, pin_memory=True)
    d_in = torch.empty(max(n_in, 1), dtype=dt, device=dev)
    for ci, offs in zip(idxs, in_off):
        for c, o in zip(chunks[ci], offs):
            k = c.numel()
            stage[o:o + k].copy_(c.reshape(-1))
            d_in[o:o + k].copy_(stage[o:o + k], non_blocking=True)
    tasks = []
    for ci, offs, o in zip(idxs, in_off, out_off):
        k = chunks[ci][0].numel()
        if k:
            tasks.append(([d_in[x:x + k] for x in offs], d_out[o:o + k]))
    _native.chunk_mean_batched(tasks)
    if tight:
        host.copy_(d_out, non_blocking=True)
    else:
        for k, o, h in zip(sizes, out_off, host_off):
            if k:
                host[h:h + k].copy_(d_out[o:o + k], non_blocking=True)
    torch.cuda.current_stream(dev).synchronize()
