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

__all__ = ["aggregate", "chunk", "reconstruct_from_chunks"]

# The reference builds the model to reconstruct into from its model zoo
# (functions.py:144, dasklearn.models.create_model). Out of scope here, so it
# is looked up lazily when the package runs inside the reference, and can be
# replaced (tests do) by assigning `model_factory`.
model_factory = None


def _create_model(settings):
    global model_factory
    if model_factory is None:
        try:
            from dasklearn.models import create_model  # the reference's model zoo
        except ImportError as exc:  # pragma: no cover - outside the reference
            raise ImportError("reconstruct_from_chunks needs dasklearn.models.create_model "
                              "or dasklearn_amd.functions.model_factory") from exc
        model_factory = create_model
    return model_factory(settings.dataset, architecture=settings.model)


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


def chunk(settings, params: Dict) -> List:
    """functions.py:136-140: split a model's flat state_dict into n chunks."""
    from dasklearn_amd.chunk_manager import ChunkManager
    return ChunkManager.chunk_model(params["model"], params["n"])


def reconstruct_from_chunks(settings, params: Dict) -> List[nn.Module]:
    """functions.py:142-146: average every chunk index over its contributors
    (on the GPU) and load the result into a fresh model."""
    from dasklearn_amd.chunk_manager import ChunkManager
    model = _create_model(settings)
    model = ChunkManager.reconstruct_model(params["chunks"], model)
    return [model]
