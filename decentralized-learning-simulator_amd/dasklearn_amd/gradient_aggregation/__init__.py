"""Aggregation plugin API — mirrors dasklearn/gradient_aggregation/__init__.py:8-17.

`GradientAggregationMethod` keeps the reference's enum value (FEDAVG = 1,
selected through `SessionSettings.gradient_aggregation`,
dasklearn/session_settings.py:40 and model_manager.py:37-39), so settings
objects built for the reference select the HIP implementation unchanged.
"""
from abc import abstractmethod
from enum import IntEnum
from typing import List, Optional

from torch import nn


class GradientAggregationMethod(IntEnum):
    FEDAVG = 1


class GradientAggregation:

    @staticmethod
    @abstractmethod
    def aggregate(models: List[nn.Module], weights: Optional[List[float]]) -> nn.Module:
        """Return a new module whose parameters are the weighted sum of the
        models' parameters (buffers and attributes copied from models[0])."""
