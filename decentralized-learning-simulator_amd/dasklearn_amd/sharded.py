"""Parameter-axis sharding of the aggregate across the GPUs of one node.

New (the reference has no multi-device path). One process
per GPU, `torch.distributed` with the "nccl" backend (= RCCL over xGMI on
ROCm). Every output element is independent, so the parameter axis splits into
contiguous slices, one per rank, with boundaries from the C ABI's
`dlsim_shard_range` (aligned to 64 elements = 256 B of fp32, so every slice
starts 16-byte aligned and takes the vector kernel).

Three entry points:

* `aggregate_param_sharded` — rank r already holds slice r of every model
  (e.g. a device-resident arena partitioned at load time): one local exact
  reduce, no data-path collective; optionally an all-gather materialises the
  full output. Bit-identical to the single-GPU (and reference) result. On an
  "nccl" group this is the C ABI's `dlsim_wreduce_sharded` on the group's own
  RCCL communicator (local reduce + grouped in-place broadcasts).
* `aggregate_model_sharded(exact=True)` — whole models live on different
  ranks: an all-to-all moves slice j of every model to rank j (in global
  model order), then the exact local reduce, then an all-gather.
  Bit-identical: each element's N terms are still folded in reference order
  on one GPU.
* `aggregate_model_sharded(exact=False)` — local weighted partial sums (FAST
  mode) + reduce-scatter + all-gather: fewer bytes on xGMI when a rank holds
  more than one model, but a different summation order, so tolerance parity
  only (n * 2^-23 relative in fp32).

`local_reduce` defaults to the HIP kernel; tests inject the CPU oracle to run
the collective logic on `gloo` without a GPU (test infrastructure only).
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

from . import _native

LocalReduce = Callable[[List[torch.Tensor], np.ndarray, torch.Tensor, int], None]


def _hip_reduce(inputs, w32, out, mode):
    _native.wreduce(inputs, w32, out, mode)


class ShardedAggregator:

    def __init__(self, group=None, align_elems: int = 64, local_reduce: Optional[LocalReduce] = None):
        if not dist.is_initialized():
            raise RuntimeError("ShardedAggregator needs torch.distributed to be initialised")
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.align = align_elems
        self.local_reduce = local_reduce or _hip_reduce

    # ---- partition --------------------------------------------------------------
    def bounds(self, n_elems: int, rank: Optional[int] = None) -> Tuple[int, int]:
        r = self.rank if rank is None else rank
        return _native.shard_range(n_elems, self.world, r, self.align)

    def all_bounds(self, n_elems: int) -> List[Tuple[int, int]]:
        return [self.bounds(n_elems, r) for r in range(self.world)]

    def _rccl_comm(self, device) -> Optional[int]:
        """The RCCL communicator behind this group (ProcessGroupNCCL._comm_ptr)
        when the HIP kernel is the local reduce and the group runs on "nccl";
        else None (gloo rehearsals, injected local reduces)."""
        if self.local_reduce is not _hip_reduce or not device.type == "cuda" or self.align != 64 \
                or dist.get_backend(self.group) != "nccl":
            return None
        try:
            pg = self.group if self.group is not None else dist.distributed_c10d._get_default_group()
            ptr = pg._get_backend(device)._comm_ptr()
        except Exception:
            return None
        return int(ptr) or None

    # ---- collectives ------------------------------------------------------------
    def _via_host(self, t: torch.Tensor) -> bool:
        """gloo moves host tensors: device tensors are staged through host
        memory around each gloo collective (a gloo control plane on GPUs,
        e.g. several ranks sharing one GPU); RCCL takes them in place."""
        return t.is_cuda and dist.get_backend(self.group) == "gloo"

    def all_gather(self, shard: torch.Tensor, n_elems: int) -> torch.Tensor:
        """Concatenate every rank's slice into the full vector (ragged last
        slice handled by padding to the largest slice)."""
        bnds = self.all_bounds(n_elems)
        width = max(e - b for b, e in bnds)
        dev = shard.device
        cdev = torch.device("cpu") if self._via_host(shard) else dev
        padded = torch.zeros(width, dtype=shard.dtype, device=cdev)
        padded[:shard.numel()].copy_(shard)
        gathered = torch.empty(width * self.world, dtype=shard.dtype, device=cdev)
        dist.all_gather_into_tensor(gathered, padded, group=self.group)
        if all(e - b == width for b, e in bnds):
            return gathered.to(dev)
        full = torch.empty(n_elems, dtype=shard.dtype, device=dev)
        for r, (b, e) in enumerate(bnds):
            full[b:e].copy_(gathered[r * width:r * width + (e - b)])
        return full

    # ---- entry points -----------------------------------------------------------
    def aggregate_param_sharded(self, shard_inputs: Sequence[torch.Tensor], weights,
                                n_elems: int, gather=True,
                                mode: int = _native.DLSIM_EXACT) -> torch.Tensor:
        """shard_inputs[i] = this rank's slice (self.bounds(n_elems)) of model i.
        gather: False (keep this rank's slice), True / "bcast" (grouped
        in-place broadcasts) or "allgather" (one padded all-gather); on gloo
        both gathers are torch's all_gather_into_tensor.

        Errors are collective: a rank whose arguments fail its checks does not
        raise before the other ranks know, so none of them is left inside a
        collective; every rank then raises the same error (the failing ranks'
        messages, in rank order)."""
        local, code, b, e = None, 0, 0, 0
        g = _native.gather_code(gather)
        c_abi = self._uses_c_abi()
        try:
            if not shard_inputs:
                raise IndexError("list index out of range")  # models[0] of fedavg.py:20
            x0 = shard_inputs[0]
            code = _native.dtype_code(x0.dtype, single_task=True)
            # fp32-rounded weights, or exact doubles for a double model (fedavg.py:25)
            w32 = _resolve(len(shard_inputs), weights, x0.dtype)
            b, e = self.bounds(n_elems)
            for x in shard_inputs:
                if x.numel() != e - b:
                    raise ValueError(f"rank {self.rank}: shard has {x.numel()} elements, expected {e - b}")
                if x.dtype != x0.dtype or x.device != x0.device or not x.is_contiguous():
                    raise ValueError(f"rank {self.rank}: shards must be contiguous tensors of one dtype and device")
                if c_abi and not x.is_cuda:
                    raise ValueError(f"rank {self.rank}: the RCCL path takes device shards")
        except (AssertionError, ValueError, IndexError, TypeError) as ex:
            local = ex
        if c_abi:
            dev = shard_inputs[0].device if local is None else _default_device()
            comm = self._rccl_comm(dev)
            if comm is not None:
                # the C ABI end to end: local reduce into the full buffer, the
                # library's agreement step, then the gather on the caller's
                # RCCL communicator
                full = None
                try:
                    if local is None:
                        full = torch.empty(n_elems, dtype=x0.dtype, device=x0.device)
                        _native.wreduce_sharded(list(shard_inputs), w32, full, comm, g, mode)
                    else:  # join the library's agreement as a failed rank
                        _native.wreduce_sharded_failed(comm, n_elems, g, dev)
                except _native.DlsimError as ex:
                    self._library_failure(local, ex)
                return full if g else full[b:e]
        self._agree(local, [n_elems, 1 if g else 0, code if local is None else 0])
        out = torch.empty(e - b, dtype=x0.dtype, device=x0.device)
        if e > b:
            self.local_reduce(list(shard_inputs), w32, out, mode)
        return self.all_gather(out, n_elems) if g else out

    def plan(self, n_elems: int, n_models: int, dtype: torch.dtype, gather=True) -> "ParamShardPlan":
        """A collective call: every rank agrees ONCE on (n_elems, n_models,
        dtype, gather); the plan's run() then skips the per-call agreement
        and, on RCCL, its host wait."""
        return ParamShardPlan(self, n_elems, n_models, dtype, gather)

    # ---- collective error handling ------------------------------------------------
    def _uses_c_abi(self) -> bool:
        return self.local_reduce is _hip_reduce and self.align == 64 and dist.get_backend(self.group) == "nccl"

    def _agree(self, local: Optional[BaseException], args: Sequence[int]) -> None:
        """One int64 MAX all-reduce of [a failure slot per rank | each argument
        and its negation]: every rank learns which ranks failed and whether the
        arguments that shape the collectives agree, before any of them enters
        one. Raises the same error on every rank if anything is wrong (a
        failed rank's arguments are not compared). The C ABI's
        dlsim_wreduce_sharded runs the same step on RCCL."""
        w = _max_allreduce(self.group, self.world, self.rank, local is not None, args)
        if any(w[:self.world]):
            self._raise_collectively(local)
        if any(w[self.world + 2 * k] != -w[self.world + 2 * k + 1] for k in range(len(args))):
            raise ValueError("ranks disagree on the model size, gather or dtype; no collective was entered")

    def _raise_collectively(self, local: Optional[BaseException]) -> None:
        """Every rank reaches this once some rank has failed (all of them know
        it from the agreement step): gather the failing ranks' messages and
        raise the same error everywhere, typed after the first failing rank's
        (ValueError / AssertionError / IndexError / TypeError, else
        RuntimeError, e.g. a library error)."""
        mine = None if local is None else (type(local).__name__, str(local))
        got: List = [None] * self.world
        dist.all_gather_object(got, mine, group=self.group)
        failed = [(r, g) for r, g in enumerate(got) if g is not None]
        msg = "; ".join(f"rank {r} of {self.world}: {m}" for r, (_, m) in failed)
        kinds = {"ValueError": ValueError, "AssertionError": AssertionError, "IndexError": IndexError,
                 "TypeError": TypeError}
        raise kinds.get(failed[0][1][0] if failed else "", RuntimeError)(msg or "a rank failed")

    def _library_failure(self, local: Optional[BaseException], ex: "_native.DlsimError") -> None:
        """After the library's agreement failed on this rank: the ranks that
        failed their own checks raise collectively with their errors; a rank
        whose only failure is a peer's (DLSIM_E_PEER) joins with none, so the
        type and message come from the failing ranks (the gloo path's rule);
        a disagreement is known to every rank and raised without a gather."""
        if local is None and ex.rc == _native.DLSIM_E_DISAGREE:
            raise ValueError("ranks disagree on the model size, gather or dtype; no collective was entered")
        if local is None and ex.rc == _native.DLSIM_E_PEER:
            self._raise_collectively(None)
        self._raise_collectively(local or ex)

    def aggregate_model_sharded(self, local_models: Sequence[torch.Tensor], counts: Sequence[int],
                                weights, exact: bool = True) -> torch.Tensor:
        """local_models: this rank's whole flat models; counts[r] = how many
        models rank r holds (global model order = rank order, then local
        order). weights: the global list (None/[] -> uniform)."""
        counts = list(counts)
        local = None
        try:
            if len(counts) != self.world or counts[self.rank] != len(local_models):
                raise ValueError("counts must list every rank's model count, this rank's included")
            n_total = sum(counts)
            w32 = _resolve(n_total, weights)
        except (AssertionError, ValueError, TypeError) as ex:
            local = ex
        ref = local_models[0] if local_models and local is None else None
        # every rank checks its arguments before the first collective; the
        # agreement also tells ranks without models the model size and dtype
        n_elems, dtype = _agree_numel(ref, self.group, self, local, with_dtype=True)
        w32 = _resolve(n_total, weights, dtype)  # exact doubles for a double model (fedavg.py:25)
        device = ref.device if ref is not None else _default_device()
        first = sum(counts[:self.rank])
        if exact:
            return self._model_sharded_exact(local_models, counts, w32, n_elems, dtype, device)
        # FAST: partial sums of local models, then sum over ranks
        acc_dt = torch.float64 if dtype == torch.float64 else torch.float32
        partial = torch.zeros(n_elems, dtype=acc_dt, device=device)
        if local_models:
            lw = w32[first:first + len(local_models)]
            acc = torch.empty(n_elems, dtype=dtype, device=device)
            self.local_reduce(list(local_models), lw, acc, _native.DLSIM_FAST)
            partial.copy_(acc)
        bnds = self.all_bounds(n_elems)
        width = max(e - b for b, e in bnds)
        padded = torch.zeros(width * self.world, dtype=acc_dt, device=device)
        for r, (b, e) in enumerate(bnds):
            padded[r * width:r * width + (e - b)].copy_(partial[b:e])
        host = self._via_host(padded)
        if host:
            padded = padded.cpu()
        mine = torch.empty(width, dtype=acc_dt, device=padded.device)
        dist.reduce_scatter_tensor(mine, padded, op=dist.ReduceOp.SUM, group=self.group)
        mine = mine.to(device)
        b, e = bnds[self.rank]
        return self.all_gather(mine[:e - b].to(dtype).contiguous(), n_elems)

    def _model_sharded_exact(self, local_models, counts, w32, n_elems, dtype, device):
        bnds = self.all_bounds(n_elems)
        lens = [e - b for b, e in bnds]
        k = len(local_models)
        # send: for each destination rank j, slice j of every local model
        send = torch.empty(k * n_elems, dtype=dtype, device=device)
        in_splits = []
        off = 0
        for j, (b, e) in enumerate(bnds):
            for m in local_models:
                send[off:off + (e - b)].copy_(m[b:e])
                off += e - b
            in_splits.append(k * (e - b))
        my_len = lens[self.rank]
        out_splits = [counts[r] * my_len for r in range(self.world)]
        if self._via_host(send):
            send = send.cpu()
        recv = torch.empty(sum(out_splits), dtype=dtype, device=send.device)
        dist.all_to_all_single(recv, send, output_split_sizes=out_splits,
                               input_split_sizes=in_splits, group=self.group)
        recv = recv.to(device)
        rows = [recv[i * my_len:(i + 1) * my_len] for i in range(sum(counts))]
        out = torch.empty(my_len, dtype=dtype, device=device)
        if my_len > 0:
            self.local_reduce(rows, w32, out, _native.DLSIM_EXACT)
        return self.all_gather(out, n_elems)


class ParamShardPlan:
    """aggregate_param_sharded for one shape, agreed once (ShardedAggregator.plan).

    On an RCCL group with the HIP reduce this is the C ABI's
    dlsim_sharded_plan; elsewhere (gloo, injected reduces) the agreement runs
    once here and each run is the local reduce plus the all-gather. Every
    rank must run the same sequence of plans. A run whose local checks or
    local reduce fail still enters the gather (so no peer waits forever) and
    raises on that rank only; it sends its slice as NaN, so its peers' copy
    of that slice is NaN rather than plausible numbers."""

    def __init__(self, agg: ShardedAggregator, n_elems: int, n_models: int, dtype: torch.dtype, gather=True):
        self.agg, self.n_elems, self.n, self.dtype = agg, int(n_elems), int(n_models), dtype
        self.gather = _native.gather_code(gather)
        self.bounds = agg.bounds(self.n_elems)
        self._c = None
        local, code = None, 0
        try:
            code = _native.dtype_code(dtype, single_task=True)
            if self.n < 1:
                raise ValueError("a plan needs n_models >= 1")
        except (ValueError, TypeError) as ex:
            local = ex
        comm = agg._rccl_comm(_default_device()) if agg._uses_c_abi() else None
        if comm is not None:
            try:
                if local is None:
                    self._c = _native.ShardedPlan(comm, self.n_elems, self.n, dtype, self.gather,
                                                  device=_default_device())
                else:  # join the agreement as a failed rank
                    _native.wreduce_sharded_failed(comm, self.n_elems, self.gather, _default_device())
            except _native.DlsimError as ex:
                agg._library_failure(local, ex)
            return
        agg._agree(local, [self.n_elems, self.n, code, 1 if self.gather else 0])

    def run(self, shard_inputs: Sequence[torch.Tensor], weights, mode: int = _native.DLSIM_EXACT,
            out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """The full output (gather) or this rank's slice, as
        aggregate_param_sharded; `out` (full size, gather on RCCL) is reused
        when given."""
        b, e = self.bounds
        local = None
        try:
            if len(shard_inputs) != self.n:
                raise ValueError(f"rank {self.agg.rank}: plan has {self.n} models, got {len(shard_inputs)}")
            w = _resolve(self.n, weights, self.dtype)
            for x in shard_inputs:
                if x.numel() != e - b or x.dtype != self.dtype or not x.is_contiguous():
                    raise ValueError(f"rank {self.agg.rank}: shards must be contiguous {self.dtype} slices of "
                                     f"{e - b} elements")
        except (AssertionError, ValueError, TypeError) as ex:
            local = ex
        dev = shard_inputs[0].device if local is None else _default_device()
        if self._c is not None:
            if local is not None:
                try:
                    self._c.run_failed(dev)  # enters the gather; raises the library's error
                except _native.DlsimError:
                    pass
                raise local
            if out is None:
                out = torch.empty(self.n_elems, dtype=self.dtype, device=dev)
            self._c.run(list(shard_inputs), w, out, mode)
            return out if self.gather else out[b:e]
        part = torch.empty(e - b, dtype=self.dtype, device=dev)
        if local is None and e > b:
            try:
                self.agg.local_reduce(list(shard_inputs), w, part, mode)
            except Exception as ex:  # noqa: BLE001 - raised after the gather
                local = ex
        if local is not None:
            part.fill_(float("nan"))  # what the peers receive for this slice
        res = self.agg.all_gather(part, self.n_elems) if self.gather else part
        if local is not None:
            raise local
        return res

    def close(self) -> None:
        if self._c is not None:
            self._c.close()
            self._c = None


def _resolve(n: int, weights, dtype=None) -> np.ndarray:
    # fedavg.py:14-17 rules, then the weight as `w * p1` sees it (fedavg.py:25):
    # rounded to fp32, or an exact double for a double tensor
    if not weights:
        weights = [float(1. / n) for _ in range(n)]
    else:
        assert len(weights) == n
    return _native.weights_for_dtype(weights, dtype) if dtype is not None else _native.fp32_weights(weights)


def _default_device():
    if torch.cuda.is_available():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def _coll_device(group):
    """Where a small control tensor for `group`'s backend lives."""
    if dist.get_backend(group) == "gloo":
        return torch.device("cpu")
    return _default_device()


def _max_allreduce(group, world: int, rank: int, failed: bool, args: Sequence[int]) -> List[int]:
    """[failure slot per rank | arg_0, -arg_0, arg_1, -arg_1, ...] reduced
    with MAX over the group: slot r says rank r failed, and arg_k agrees on
    every rank iff its max equals minus the max of its negation."""
    t = torch.zeros(world + 2 * len(args), dtype=torch.int64, device=_coll_device(group))
    t[rank] = 1 if failed else 0
    for k, v in enumerate(args):
        t[world + 2 * k] = int(v)
        t[world + 2 * k + 1] = -int(v)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return t.tolist()


_DTYPES = {0: torch.float32, 1: torch.bfloat16, 2: torch.float16, 3: torch.float64}  # enum dlsim_dtype


def _agree_numel(ref: Optional[torch.Tensor], group, agg: Optional["ShardedAggregator"] = None,
                 local: Optional[BaseException] = None, with_dtype: bool = False):
    """Every rank must see the same model size (and, with_dtype, element
    type); ranks without models learn them. With `agg`, rank-local argument
    errors are agreed in the same all-reduce (a failure slot per rank) and
    raised on every rank; a size or dtype disagreement is raised on every rank
    too. Returns n, or (n, dtype) with_dtype (fp32 when no rank holds a
    model)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    none = -2 ** 62
    # ranks without models contribute (-1, -2^62): neutral for both maxima
    hi, neg_lo = (ref.numel(), -ref.numel()) if ref is not None else (-1, none)
    code = None
    if ref is not None and local is None:
        try:
            code = _native.dtype_code(ref.dtype, single_task=True)
        except TypeError as ex:  # an unsupported dtype fails this rank, collectively
            local = ex
    t = torch.zeros(world + 4, dtype=torch.int64, device=_coll_device(group))
    t[rank] = 1 if local is not None else 0
    t[world], t[world + 1] = hi, neg_lo
    t[world + 2], t[world + 3] = (code, -code) if code is not None else (-1, none)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    w = t.tolist()
    if any(w[:world]):
        if agg is None:
            raise RuntimeError("a rank failed its checks")
        agg._raise_collectively(local)
    n = int(w[world])
    if w[world + 1] != none and n != -w[world + 1]:
        raise ValueError("models differ in size across ranks")
    if w[world + 3] != none and w[world + 2] != -w[world + 3]:
        raise ValueError("models differ in dtype across ranks")
    if not with_dtype:
        return n
    return n, _DTYPES.get(int(w[world + 2]), torch.float32)
