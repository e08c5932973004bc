"""dasklearn_amd — MI355X-native aggregation hot path of the decentralized
learning simulator (sacs-epfl/decentralized-learning-simulator).

Mirrors the reference's plugin/task interface for exactly one path:
  dasklearn_amd.functions.aggregate              <- dasklearn/functions.py:89-106
  dasklearn_amd.model_manager.ModelManager       <- dasklearn/model_manager.py:14-43
  dasklearn_amd.gradient_aggregation.fedavg.FedAvg <- dasklearn/gradient_aggregation/fedavg.py:10-26
over a HIP C ABI (include/dlsim.h, lib/libdlsim_hip.so). There is no CPU
fallback: without the built library or a GPU, calls raise.
"""
__version__ = "0.1.0"
