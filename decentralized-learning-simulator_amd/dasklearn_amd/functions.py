"""The `aggregate` compute task — drop-in for dasklearn/functions.py:89-106.

`dasklearn/worker.py:27-31` resolves task functions with
`globals()[func_name]` over `from dasklearn.functions import *`; exporting an
`aggregate(settings, params)` with the same contract here is what lets the
worker run the HIP path unchanged (INTEGRATION.md shows the one-line hook).

params: {"models": [nn.Module], "round": int, "peer": int | None,
         optional "weights": [float]}  ->  [nn.Module]   (a list of one, as the
broker requires list/tuple results, broker.py:282-283).
"""
import logging
import time
from typing import Dict, List

from torch import nn

from dasklearn_amd.model_manager import ModelManager

logger = logging.getLogger(__name__)

__all__ = ["aggregate"]


def aggregate(settings, params: Dict) -> List[nn.Module]:
    models = params["models"]
    round_nr = params["round"]
    peer_id = params["peer"]
    weights = params["weights"] if "weights" in params else None
    if peer_id is not None:
        logger.debug("Peer %d aggregating %d models in round %d...", peer_id, len(models), round_nr)
    else:
        logger.debug("Aggregating %d models in round %d...", len(models), round_nr)

    model_manager = ModelManager(None, settings, 0)
    for idx, model in enumerate(models):
        model_manager.process_incoming_trained_model(idx, model)

    start_time = time.time()
    agg_model = model_manager.aggregate_trained_models(weights)
    logger.debug("Model aggregation took %f s.", time.time() - start_time)
    return [agg_model]
