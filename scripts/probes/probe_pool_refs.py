"""Debug probe: storage use counts of the output pool's blocks on the GPU."""
import gc
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "decentralized-learning-simulator_amd")):
    sys.path.insert(0, p)
import torch  # noqa: E402
from dasklearn_amd import arena, _native  # noqa: E402

uc = lambda t: torch._C._storage_Use_Count(t.untyped_storage()._cdata)  # noqa: E731
BIG = (20 << 20) // 4
blk = _native.DeviceBlock(4 << 20, "cuda")
t = blk.tensor()
print("deviceblock tensor alone", uc(t), flush=True)
v = t[10:20]
print("with a view", uc(t), flush=True)
del v
print("view gone", uc(t), flush=True)
c = torch.empty(100, device="cuda")
print("torch cuda tensor alone", uc(c), flush=True)
a = arena.arena_empty(BIG, torch.float32, "cuda")
pool = arena.OUTPUT_POOL
key = [k for k in pool.blocks if k[2] >= BIG * 4][0]
base = pool.blocks[key][-1][0]
print("pool key", key, "blocks", len(pool.blocks[key]))
print("base with a alive", uc(base), flush=True)
del a
gc.collect()
print("base after del a", uc(base), flush=True)
del base
print("in_use flags", [pool._in_use(b) for b in pool.blocks[key]], flush=True)
