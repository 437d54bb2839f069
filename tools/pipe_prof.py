"""Phase profile of the pipe kernel (debug build with -DBCE_PIPE_PROF=1), c2 workload."""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bayesian-consensus-engine_amd"))
sys.path.insert(0, ROOT)
from bayesian_engine import _native as N, batch  # noqa: E402
from bench import make_c2  # noqa: E402

M, L, S = 1_000_000, 32, 10_000
off, sid, prob, rel, conf, present = make_c2(M, L, S, 2)
T = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
table = batch.SourceTable.from_arrays(T(rel), T(conf), T(present))
d = [T(off), T(sid), T(prob)]
res = batch._alloc(M, M * L, d[0].device, True, True)
lib = N.lib()
buf = (C.c_ulonglong * 16)()
for _ in range(3):
    batch.consensus(*d, table, max_len=L, out=res)
torch.cuda.synchronize()
lib.bce_pipe_prof_read(buf)
R = 10
for _ in range(R):
    batch.consensus(*d, table, max_len=L, out=res)
torch.cuda.synchronize()
lib.bce_pipe_prof_read(buf)
v = list(buf)
tiles = (M + 63) // 64
names = ["wait_slot", "keys_sort", "walk", "per_market", "copy_out"]
tot = sum(v[:5])
print(f"compute waves {v[5] // R}  tiles {tiles}")
for k, nm in enumerate(names):
    print(f"{nm:12s} {v[k] / R / tiles:10.0f} cyc/tile  {100 * v[k] / tot:5.1f} %")
lnames = ["wait_free_slot", "issue_dma", "wait_landed", "validate_publish"]
ltot = sum(v[8:12])
print("loader wave, per tile:")
for k, nm in enumerate(lnames):
    print(f"{nm:16s} {v[8 + k] / R / tiles:10.0f} cyc/tile  {100 * v[8 + k] / max(ltot, 1):5.1f} %")
