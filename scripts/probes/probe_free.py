import sys, time, json
sys.path[:0] = ['/root/repo', '/root/repo/scripts', '/root/repo/decentralized-learning-simulator_amd']
import torch
from bench import resnet18_shapes
from bench_rounds import Shaped
import copy
dev = torch.device('cuda', 0)
res = {}
def mk():
    return [Shaped(resnet18_shapes()).to(dev) for _ in range(20)]
for label, busy in (("idle", False), ("busy", True)):
    ms = mk(); torch.cuda.synchronize()
    if busy:
        torch.cuda._sleep(200_000_000)
    t0 = time.perf_counter(); del ms; t1 = time.perf_counter()
    torch.cuda.synchronize()
    res[label + "_free_20_models_ms"] = round((t1 - t0) * 1e3, 3)
# deepcopy-made models (as train outputs)
base = Shaped(resnet18_shapes()).to(dev)
ms = [copy.deepcopy(base) for _ in range(20)]; torch.cuda.synchronize()
t0 = time.perf_counter(); del ms; t1 = time.perf_counter()
res["deepcopies_free_20_ms"] = round((t1 - t0) * 1e3, 3)
print(json.dumps(res))
