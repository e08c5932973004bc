"""ModelManager — mirrors dasklearn/model_manager.py:14-43 for the aggregate task.

Collects incoming models keyed by peer id (first one wins, :27-32) and
aggregates them with the method chosen by `settings.gradient_aggregation`
(:37-43). The `dataset` argument is accepted and ignored, as the reference's
aggregate task passes None (functions.py:99).
"""
import logging
from typing import Dict, List, Optional

import torch.nn as nn

from dasklearn_amd.gradient_aggregation import GradientAggregationMethod
from dasklearn_amd.gradient_aggregation.fedavg import FedAvg


class ModelManager:

    def __init__(self, dataset, settings, participant_index: int):
        self.settings = settings
        self.participant_index: int = participant_index
        self.logger = logging.getLogger(self.__class__.__name__)
        self.incoming_trained_models: Dict[int, nn.Module] = {}

    def process_incoming_trained_model(self, peer_id: int, incoming_model: nn.Module):
        if peer_id in self.incoming_trained_models:
            return
        self.incoming_trained_models[peer_id] = incoming_model

    def reset_incoming_trained_models(self):
        self.incoming_trained_models = {}

    def get_aggregation_method(self):
        method = getattr(self.settings, "gradient_aggregation", GradientAggregationMethod.FEDAVG)
        if method == GradientAggregationMethod.FEDAVG:
            return FedAvg
        return None  # the reference returns None for unknown methods too

    def aggregate_trained_models(self, weights: List[float] = None) -> Optional[nn.Module]:
        models = list(self.incoming_trained_models.values())
        method = self.get_aggregation_method()
        # Opt-in (not a reference setting): keep the aggregate on the GPU so a
        # device-resident consumer skips the D2H/H2D round trip.
        if getattr(self.settings, "aggregate_on_device", False):
            return method.aggregate(models, weights=weights, to_host=False)
        return method.aggregate(models, weights=weights)
