"""Child side of tests/test_gpu_worker_process.py (not a test module).

A restatement of the reference's worker loop (dasklearn/worker.py:21-38): the
task functions are star-imported, resolved with globals()[func_name], and the
result goes back on the result queue; an exception sends ("error", task, None)
and ends the loop. Only the import line differs: it takes the HIP task
functions, as INTEGRATION.md's one-line hook does."""
import time

import torch
import torch.multiprocessing

torch.multiprocessing.set_sharing_strategy("file_system")  # worker.py:6

from dasklearn_amd.functions import *  # noqa: E402,F401,F403


def cache_stats(settings, data):
    """A task of this test worker only: the device cache's counters
    (dasklearn_amd/device_cache.py), or None when it is off."""
    from dasklearn_amd import device_cache
    c = device_cache.active()
    return [None if c is None else dict(c.stats, entries=len(c))]


class Settings:
    gradient_aggregation = 1  # GradientAggregationMethod.FEDAVG
    torch_threads = 4


def worker_main(shared_queue, result_queue, index):
    torch.set_num_threads(Settings.torch_threads)  # broker.py:31
    settings = Settings()
    while True:
        received_time = time.time()
        item = shared_queue.get()
        if item is None:
            break
        task_name, func_name, data = item
        try:
            if func_name not in globals():
                raise RuntimeError("Task function %s not found!" % func_name)
            f = globals()[func_name]
            res = f(settings, data)
            result_queue.put((task_name, res, {"received": received_time, "finished": time.time(),
                                               "worker": index}))
        except Exception:
            result_queue.put(("error", task_name, None))
            break
