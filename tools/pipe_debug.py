"""Small staged checks of the contiguous short-market kernel (debug tooling)."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bayesian-consensus-engine_amd"))
sys.path.insert(0, ROOT)
from bayesian_engine import batch  # noqa: E402
from oracle import oracle as orc  # noqa: E402


def run(M, L, S, seed, ragged=False):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, L + 1, M) if ragged else np.full(M, L)
    off = np.zeros(M + 1, np.int64)
    off[1:] = np.cumsum(lens)
    n = int(off[-1])
    sid = rng.integers(0, S, n).astype(np.int32)
    prob = rng.random(n)
    rel, conf = rng.uniform(0, 1, S), rng.random(S)
    present = (rng.random(S) < 0.8).astype(np.uint8)
    T = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    table = batch.SourceTable.from_arrays(T(rel), T(conf), T(present))
    t0 = time.time()
    r = batch.consensus(T(off), T(sid), T(prob), table, max_len=L)
    torch.cuda.synchronize()
    dt = time.time() - t0
    exp = orc.consensus_csr(off, sid, prob, rel, conf, present)
    ok = all(np.array_equal(getattr(r, k).cpu().numpy(), exp[k], equal_nan=True)
             for k in ("consensus", "confidence", "total_weight", "n_unique", "err_idx"))
    print(f"M={M} L={L} S={S} ragged={ragged}: {'OK' if ok else 'MISMATCH'} ({dt:.3f}s)", flush=True)


CASES = [(64, 8, 100, False), (1000, 8, 100, False), (64, 16, 100, False), (1000, 16, 100, False),
         (1000, 32, 100, True), (1000, 8, 100, True), (20000, 32, 10000, False), (200000, 32, 10000, True),
         (6_000_000, 2, 1000, True)]

if __name__ == "__main__":
    if len(sys.argv) > 1:
        M, L, S, rg = CASES[int(sys.argv[1])]
        run(M, L, S, 1, rg)
    else:
        import subprocess
        for i in range(len(CASES)):
            r = subprocess.run([sys.executable, "-u", __file__, str(i)], timeout=None if False else 60)
            print(f"case {i} rc={r.returncode}", flush=True)
