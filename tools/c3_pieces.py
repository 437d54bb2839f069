#!/usr/bin/env python3
"""Launch-cost probe for the planned C3 split (GPU box; run under rocprofv3 --kernel-trace and
read with tools/trace_bursts.py): pieces of each wide length bin of the full config-3 plan --
the first (longest) or last (shortest) 1/8, 1/4, 1/2 of the bin, and the whole bin -- are
launched ALONE over the full CSR, REPS times each, with a 60 ms idle gap between pieces so
each piece is its own burst.  Prints one JSON line per piece (bin, side, markets) in burst order.

  rocprofv3 --kernel-trace -d DIR -o run --output-format csv -- python3 tools/c3_pieces.py [--mode fast]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bayesian-consensus-engine_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="fast")
    ap.add_argument("--reps", type=int, default=12)
    ap.add_argument("--bins", default="4,5,6,7,8,9,10,11")
    a = ap.parse_args()
    from bench_extra import make_c3
    from bayesian_engine import _native as N
    from bayesian_engine import batch

    M, off, sid, prob, (rel, conf, pres), _ = make_c3(1, 0)
    dev = torch.device("cuda", 0)
    T = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)  # noqa: E731
    table = batch.SourceTable.from_arrays(T(rel), T(conf), T(pres))
    d_off, d_sid, d_prob = T(off), T(sid), T(prob)
    plan = batch.Plan.build(off, dev)
    res = batch._alloc(M, int(off[-1]), dev, True, True)
    bs = plan.bin_start
    order = plan.order
    pieces = []
    for b in (int(x) for x in a.bins.split(",")):
        n_b = int(bs[b + 1] - bs[b])
        for frac in (8, 4, 2):
            k = n_b // frac
            pieces.append((b, "longest", int(bs[b]), int(bs[b]) + k))
            pieces.append((b, "shortest", int(bs[b + 1]) - k, int(bs[b + 1])))
        pieces.append((b, "whole", int(bs[b]), int(bs[b + 1])))
    for b, side, p0, p1 in pieces:
        # a plan with only [p0, p1) of bin b: the order slice, every other bin empty
        sub = order[p0:p1].contiguous()
        one = np.zeros_like(bs)
        one[b + 1:] = p1 - p0
        p = batch.Plan(sub, one, plan.max_len, plan.scratch)
        for _ in range(a.reps):
            batch.consensus(d_off, d_sid, d_prob, table, plan=p, mode=a.mode, out=res)
        torch.cuda.synchronize()
        time.sleep(0.06)
        print(json.dumps({"bin": b, "side": side, "markets": p1 - p0}), flush=True)
    N.check_faults(dev, "c3_pieces")


if __name__ == "__main__":
    main()
