import sys, time, torch
sys.path[:0]=['.', 'decentralized-learning-simulator_amd']
from torch import nn
from dasklearn_amd.chunk_manager import ChunkManager
P=11_181_642; k=10; m=4
dev=torch.device('cuda',0)
flats=[torch.randn(P)*0.05 for _ in range(m)]
def chunks_of(f):
    n=P//k; cs=[f[i*n:(i+1)*n] for i in range(k)]; cs[-1]=torch.cat([cs[-1], f[k*n:]]); return cs
hc=[chunks_of(f) for f in flats]
by=[[hc[i][c] for i in range(m)] for c in range(k)]
def t(f, r=5):
    f(); torch.cuda.synchronize(); ts=[]
    for _ in range(r):
        t0=time.perf_counter(); f(); torch.cuda.synchronize(); ts.append(time.perf_counter()-t0)
    return round(sorted(ts)[r//2]*1e3,3)
print("threads", torch.get_num_threads())
print("mean_chunk_indices ms", t(lambda: ChunkManager.mean_chunk_indices([list(c) for c in by])))
stage=torch.empty(m*P+4096, pin_memory=True)
def st():
    o=0
    for cs in by:
        for c in cs:
            stage[o:o+c.numel()].copy_(c); o+=c.numel()
print("stage copies ms", t(st))
d=torch.empty(m*P+4096, device=dev)
print("h2d ms", t(lambda: d.copy_(stage, non_blocking=True)))
means=ChunkManager.mean_chunk_indices([list(c) for c in by])
print("cat ms", t(lambda: torch.cat(means)))
tgt=torch.empty(P)
fl=torch.cat(means)
print("copy ms", t(lambda: tgt.copy_(fl)))
torch.set_num_threads(4)
print("t4 mean_chunk_indices ms", t(lambda: ChunkManager.mean_chunk_indices([list(c) for c in by])))
print("t4 stage copies ms", t(st))
