#!/usr/bin/env python3
"""Per-bin cost of the planned consensus launch on the config-3 batch (GPU box, repo root).

Each length bin of the full batch's plan is launched ALONE (a Plan whose other bins are empty),
timed with HIP events over K steps after a clock ramp, in the requested mode.  The per-market
cost (us per market = bin time / bin market count) is sharding.PLAN_BIN_COST_US, the cost model
of sharding.shard_markets_planned.  Prints one JSON object.

  python3 tools/c3_bins.py [--mode fast|exact] [--steps 20] [--sources 1000000]
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
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--sources", type=int, default=1_000_000)
    a = ap.parse_args()
    from bench_extra import make_c3
    from bayesian_engine import _native as N
    from bayesian_engine import batch

    M, off, sid, prob, (rel, conf, pres), _ = make_c3(1, 0, S=a.sources)
    dev = torch.device("cuda", 0)
    T = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)  # noqa: E731
    table = batch.SourceTable.from_arrays(T(rel), T(conf), T(pres))
    d_off, d_sid, d_prob = T(off), T(sid), T(prob)
    plan = batch.Plan.build(off, dev)
    res = batch._alloc(M, int(off[-1]), dev, True, True)
    bs = plan.bin_start
    lens = np.diff(off)
    out = {"mode": a.mode, "markets": M, "signals": int(off[-1]), "bins": []}

    def timeit(p):
        step = lambda: batch.consensus(d_off, d_sid, d_prob, table, plan=p, mode=a.mode, out=res)  # noqa: E731
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.3:
            step()
            torch.cuda.synchronize()
        for _ in range(3):
            step()
        s = torch.cuda.current_stream(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(s)
        for _ in range(a.steps):
            step()
        e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.steps * 1e3  # us

    full_us = timeit(plan)
    for b in range(len(bs) - 1):
        n_b = int(bs[b + 1] - bs[b])
        if n_b == 0:
            out["bins"].append({"bin": b, "markets": 0})
            continue
        one = np.where(np.arange(len(bs)) <= b, bs[b], bs[b + 1]).astype(np.int64)
        p = batch.Plan(plan.order, one, plan.max_len, plan.scratch)
        us = timeit(p)
        ms = plan.order[int(bs[b]):int(bs[b + 1])].cpu().numpy()
        out["bins"].append({"bin": b, "markets": n_b, "signals": int(lens[ms].sum()), "us": us,
                            "us_per_market": us / n_b, "us_per_1M_signals": us / max(int(lens[ms].sum()), 1) * 1e6})
        print(f"[c3_bins] bin {b}: {n_b} markets {us:.1f} us", file=sys.stderr, flush=True)
    N.check_faults(dev, "c3_bins")
    out["full_us"] = full_us
    out["sum_of_bins_us"] = sum(x.get("us", 0.0) for x in out["bins"])
    print(json.dumps(out))


if __name__ == "__main__":
    main()
