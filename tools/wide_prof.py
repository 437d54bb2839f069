"""Phase profile of consensus_wide_kernel (debug build with -DBCE_PIPE_PROF=1), C3-like bins.

Usage: BCE_LIB=<profiling lib> python tools/wide_prof.py
Per market, s_memtime cycles seen by wave 0 (chain wave when NW > 1) and wave 1.
"""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bayesian-consensus-engine_amd"))
sys.path.insert(0, ROOT)
from bayesian_engine import _native as N, batch  # noqa: E402

S = 1_000_000
rng = np.random.default_rng(3)
lib = N.lib()
buf = (C.c_ulonglong * 16)()
names = ["load", "sort", "leaders", "compute", "round_barrier", "chain", "outputs"]
T = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
rel, conf = rng.uniform(0.1, 1, S), rng.random(S)
present = (rng.random(S) < 0.9).astype(np.uint8)
table = batch.SourceTable.from_arrays(T(rel), T(conf), T(present))
perm = rng.permutation(S).astype(np.int32)


def zipf_trunc(n):
    z = rng.zipf(1.1, n)
    bad = z > S
    while bad.any():
        z[bad] = rng.zipf(1.1, int(bad.sum()))
        bad = z > S
    return z - 1


for lo, hi in [(65, 128), (513, 1024), (1025, 2048), (2049, 4096)]:
    M = max(2000, 20_000_000 // ((lo + hi) // 2))
    lens = rng.integers(lo, hi + 1, M)
    off = np.zeros(M + 1, np.int64)
    off[1:] = np.cumsum(lens)
    n = int(off[-1])
    sid = perm[zipf_trunc(n)]
    prob = rng.random(n)
    d = [T(off), T(sid), T(prob)]
    plan = batch.Plan.build(off)
    res = batch._alloc(M, n, d[0].device, True, True)
    batch.consensus(*d, table, plan=plan, out=res)
    torch.cuda.synchronize()
    lib.bce_pipe_prof_read(buf)
    R = 3
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(R):
        batch.consensus(*d, table, plan=plan, out=res)
    ev[1].record()
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / R
    lib.bce_pipe_prof_read(buf)
    v = list(buf)
    u = res.n_unique.float().mean().item()
    print(f"bin {lo}..{hi}: {M} markets, mean u {u:.0f}, {ms:.3f} ms/launch, {n / ms / 1e6:.2f} G signals/s")
    for w in (0, 1):
        mk = v[w * 8 + 7]
        if not mk:
            continue
        tot = sum(v[w * 8:w * 8 + 7])
        print(f"  wave {w}: {tot / mk:8.0f} cyc/market  " +
              "  ".join(f"{nm} {v[w * 8 + k] / mk:.0f}" for k, nm in enumerate(names)))
