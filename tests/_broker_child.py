"""Child side of tests/test_gpu_worker_process.py (not a test module): the
reference broker's process model, run as a fresh Python process that has not
touched the GPU. `python _broker_child.py [fork|spawn]` (default fork, the
reference's start method).

Like dasklearn/broker.py it imports the task functions at top level — here
INTEGRATION.md's hook, `from dasklearn_amd.functions import *` (broker.py:16)
— sets the file_system sharing strategy (broker.py:26) and starts its worker
with torch.multiprocessing.Process under the DEFAULT start method, which is
fork on Linux (broker.py:227-233). The forked worker initialises HIP itself
and runs the restated worker loop (tests/_worker_child.py = worker.py:21-38)
on host models that arrive through shared memory. The parent checks every
result against the oracle bit for bit and prints one JSON line, including the
helper processes torch started (the shm manager) so the caller can wait for
them to exit."""
import json
import os
import sys

if "cache" in sys.argv[2:]:  # the worker's device model cache, before the package is imported
    os.environ["DLSIM_DEVICE_CACHE_MB"] = "256"

import torch
import torch.multiprocessing as multiprocessing

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, ROOT, os.path.join(ROOT, "decentralized-learning-simulator_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

from dasklearn_amd.functions import *  # noqa: E402,F401,F403  (broker.py:16, the hook)

torch.multiprocessing.set_sharing_strategy("file_system")  # broker.py:26

from torch import nn  # noqa: E402

from _worker_child import worker_main  # noqa: E402
from oracle import oracle as orc  # noqa: E402  (the checker)


class Net(nn.Module):
    def __init__(self, seed):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        self.conv = nn.Conv2d(3, 16, 5)
        self.bn = nn.BatchNorm2d(16)
        self.fc = nn.Linear(400, 10)
        with torch.no_grad():
            for q in self.parameters():
                q.copy_(torch.randn(q.shape, generator=g) * 0.05)
            self.bn.running_mean.copy_(torch.randn(16, generator=g))


def flat(m):
    return torch.cat([q.detach().reshape(-1) for q in m.parameters()]).numpy()


def main():
    import psutil
    method = sys.argv[1] if len(sys.argv) > 1 else "fork"
    # fork: the default context, as broker.py uses it; spawn: an explicit one
    ctx = multiprocessing if method == "fork" else multiprocessing.get_context(method)
    out = {"start_method": ctx.get_start_method() if method == "fork" else method}
    shared, results = ctx.Queue(), ctx.Queue()
    proc = ctx.Process(target=worker_main, args=(shared, results, 0))
    out["gpu_initialised_before_fork"] = torch.cuda.is_initialized()
    proc.start()
    ok = True
    try:
        models = [Net(s) for s in range(7)]
        w = [0.05, 0.25, 0.1, 0.2, 0.15, 0.1, 0.15]
        tasks = [("agg_0", models[:2], None), ("agg_1", models, w), ("agg_2", models[2:5], [])]
        for name, ms, ws in tasks:
            data = {"models": ms, "round": 3, "peer": 1}
            if ws is not None:
                data["weights"] = ws
            shared.put((name, "aggregate", data))
        shared.put(("agg_bad", "aggregate", {"models": models[:2], "round": 3, "peer": 2, "weights": [1.0]}))
        got = {}
        for _ in range(4):
            name, res, info = results.get(timeout=120)
            got[name] = (res, info)
        checks = {}
        for name, ms, ws in tasks:
            res, info = got[name]
            m = res[0]
            exp = orc.wreduce([flat(x) for x in ms], orc.reference_weights(len(ms), ws), "f32")
            checks[name] = bool(len(res) == 1 and info["worker"] == 0 and not any(q.is_cuda for q in m.parameters())
                                and orc.same_bits(flat(m), exp)
                                and torch.equal(m.bn.running_mean, ms[0].bn.running_mean))
        checks["error_protocol"] = got.get("error", (None,))[0] == "agg_bad"
        if "cache" in sys.argv[2:]:
            # the worker died on agg_bad (the reference's protocol): a second
            # worker runs the same three tasks, then reports its cache: the
            # models it received before are read from the device
            proc.join(timeout=60)
            proc2 = ctx.Process(target=worker_main, args=(shared, results, 0))
            proc2.start()
            for name, ms, ws in tasks:
                data = {"models": ms, "round": 3, "peer": 1}
                if ws is not None:
                    data["weights"] = ws
                shared.put((name, "aggregate", data))
            shared.put(("stats", "cache_stats", {}))
            shared.put(None)
            got2 = {}
            for _ in range(4):
                name, res, info = results.get(timeout=120)
                got2[name] = res
            for name, ms, ws in tasks:
                exp = orc.wreduce([flat(x) for x in ms], orc.reference_weights(len(ms), ws), "f32")
                checks[name + "_cached"] = orc.same_bits(flat(got2[name][0]), exp)
            out["cache_stats"] = got2["stats"][0]
            # agg_0 sends models 0-1, agg_1 0-6 (0-1 resident), agg_2 2-4 (all resident)
            checks["cache_hits"] = out["cache_stats"] == dict(out["cache_stats"], hits=5, misses=7, uncacheable=0)
            proc2.join(timeout=60)
        out["checks"] = checks
        ok = all(checks.values())
        proc.join(timeout=60)
        out["worker_exitcode"] = proc.exitcode
        ok = ok and proc.exitcode == 0 and not out["gpu_initialised_before_fork"]
    finally:
        if proc.is_alive():
            proc.kill()
            proc.join()
    out["helpers"] = [{"pid": c.pid, "name": c.name()} for c in psutil.Process().children(recursive=True)]
    out["ok"] = ok
    print(json.dumps(out), flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
