"""FedAvg on the MI355X — drop-in for dasklearn/gradient_aggregation/fedavg.py:10-26.

Same contract as the reference `FedAvg.aggregate(models, weights)`:
  * weights None or [] -> float(1./N) each; otherwise len(weights) == N is
    asserted (AssertionError); an empty model list raises IndexError;
  * returns a new module of type(models[0]) with copy.deepcopy(models[0])
    semantics (buffers such as BatchNorm running stats are NOT averaged);
  * inputs are only read;
  * numerically bit-identical to the reference (DLSIM_EXACT): same term
    order, separate fp32 rounding of each product and sum, bf16 rounding of
    each bf16 product and sum.
The arithmetic runs in one HIP kernel over flat parameter arenas
(csrc/wreduce_kernels.hpp); models on the host are staged through pinned
memory, models already on the GPU are read in place (dasklearn_amd/arena.py).
"""
from typing import List, Optional

from torch import nn

from dasklearn_amd import _native
from dasklearn_amd.arena import aggregate_modules
from dasklearn_amd.gradient_aggregation import GradientAggregation


class FedAvg(GradientAggregation):

    @staticmethod
    def aggregate(models: List[nn.Module], weights: Optional[List[float]] = None,
                  to_host: Optional[bool] = None) -> nn.Module:
        """to_host=None (default): the result lives where models[0] lives, as
        in the reference; False keeps it on the GPU for a device-resident
        aggregate -> train chain."""
        return aggregate_modules(models, weights, _native.DLSIM_EXACT, to_host=to_host)


class FedAvgFast(GradientAggregation):
    """Same, with fused multiply-add and fp32 accumulation (DLSIM_FAST):
    not bit-identical to the reference; within n * 2^-23 relative in fp32."""

    @staticmethod
    def aggregate(models: List[nn.Module], weights: Optional[List[float]] = None,
                  to_host: Optional[bool] = None) -> nn.Module:
        return aggregate_modules(models, weights, _native.DLSIM_FAST, to_host=to_host)
