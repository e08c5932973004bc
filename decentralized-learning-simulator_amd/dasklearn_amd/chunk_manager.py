"""ChunkManager — mirror of dasklearn/simulation/conflux/chunk_manager.py:10-53.

The chunked-model algorithms (Conflux, Shatter) split a model's flat
state_dict into k chunks (`chunk` task, functions.py:136-140), send chunk c to
some peers, and rebuild a model from the received chunks by averaging each
chunk index over its contributors (`reconstruct_from_chunks` task,
functions.py:142-146). That average is a second N-way reduce of the hot path
(SURVEY.md §8f row 2); here it runs on the GPU through `dlsim_mean`.

* `chunk_model` / `get_flat_params` are pure data movement (a torch.cat of the
  state_dict and slices of it) and are restated with the same tensor ops, on
  whatever device the model lives.
* `reconstruct_model`: per chunk index, `torch.mean(torch.stack(chunks), 0)`
  (chunk_manager.py:38-40) becomes one `dlsim_mean` launch over the chunks —
  sum in input order from +0, one division by the contributor count. That is
  bit-identical to the reference while PyTorch's CPU dim-0 reduction is
  sequential (<= 4 contributors per chunk); with more contributors PyTorch
  switches to a size- and thread-dependent order, so parity is a tolerance
  (m * 2^-23 relative to the mean of |x|; tests/test_gpu_chunks.py).
  As in the reference, `chunks[c]` is replaced in place by its mean and the
  result is copied into `model.state_dict()` (parameters and buffers).
"""
from __future__ import annotations

from typing import List

import torch
from torch import nn

from . import _native
from .arena import _target_device


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
        first = chunks_at_idx[0]
        for c in chunks_at_idx:
            if c.shape != first.shape or c.dtype != first.dtype:
                raise RuntimeError("stack expects each tensor to be equal size")
        dev = _target_device([first], device)
        src = [c.reshape(-1) for c in chunks_at_idx]
        with torch.no_grad():
            if first.is_cuda and all(c.device == dev for c in src):
                rows = [c.contiguous() for c in src]
            else:
                stage = torch.empty((len(src), first.numel()), dtype=first.dtype, pin_memory=True)
                for i, c in enumerate(src):
                    stage[i].copy_(c)
                dev_rows = stage.to(dev, non_blocking=True)
                rows = [dev_rows[i] for i in range(len(src))]
            out = torch.empty(first.numel(), dtype=first.dtype, device=dev)
            if out.numel():
                _native.mean(rows, out)
            if not first.is_cuda:
                out = out.cpu()
        return out.view(first.shape)

    @staticmethod
    def reconstruct_model(chunks: List[List[torch.Tensor]], model: nn.Module) -> nn.Module:
        for idx in range(len(chunks)):
            assert chunks[idx], "No chunks received at index %d!" % idx
        for chunk_idx, chunks_at_idx in enumerate(chunks):
            chunks[chunk_idx] = ChunkManager.mean_chunks(chunks_at_idx)
        flat_params = torch.cat(chunks)
        pointer = 0
        with torch.no_grad():
            for param in model.state_dict().values():
                numel = param.data.numel()
                param.data.copy_(flat_params[pointer:pointer + numel].view(param.data.shape))
                pointer += numel
        return model
