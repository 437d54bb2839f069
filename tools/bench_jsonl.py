"""Throughput of the batched JSON front end on one GPU: payloads/s through
what `consensus-batch` runs (native C++ parse + structure checks + interning, one validation
launch, one consensus launch, native json.dumps(indent=2) rendering), checked byte for byte
against the Python path, whose end-to-end time and phase split are reported beside it.  The
input lines are built before timing (C2-shaped: 32 signals per market over 10k sources).

Usage: python tools/bench_jsonl.py [--markets 100000] [--len 32] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bayesian-consensus-engine_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bayesian_engine import jsonl  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--markets", type=int, default=100_000)
    ap.add_argument("--len", type=int, default=32)
    ap.add_argument("--sources", type=int, default=10_000)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    rng = np.random.default_rng(2)
    sid = rng.integers(0, a.sources, size=(a.markets, a.len))
    prob = np.round(rng.uniform(size=(a.markets, a.len)), 4)
    lines = [json.dumps({"schemaVersion": "1.0.0", "marketId": f"m-{m}",
                         "signals": [{"sourceId": f"src-{s:05d}", "probability": float(p)}
                                     for s, p in zip(sid[m], prob[m])]}) for m in range(a.markets)]
    lines = [ln + "\n" for ln in lines]  # as readlines() hands them to consensus-batch
    jsonl.consensus_jsonl(lines[:1000])  # warm-up (library load, first launches)
    jsonl.consensus_jsonl(lines[:1000], native=False)
    torch.cuda.synchronize()
    best, best_py = None, None
    for _ in range(a.reps):
        t0 = time.perf_counter()
        out, err, failed = jsonl.consensus_jsonl_bytes(lines)  # what consensus-batch writes
        t1 = time.perf_counter()
        if best is None or t1 - t0 < best:
            best = t1 - t0
    assert not failed and not err
    t0 = time.perf_counter()
    payloads, errors, probs, tes = jsonl.parse_batch(lines)
    t1 = time.perf_counter()
    res = jsonl.consensus_many([p["signals"] for p in payloads])
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    texts = [jsonl.render(r) for r in res]
    t3 = time.perf_counter()
    py = jsonl.consensus_jsonl(lines, native=False)
    t4 = time.perf_counter()
    want = "".join(t + "\n" for ok, t in py if ok).encode()
    assert out == want, "native and Python front ends differ"
    assert texts[-1] == json.dumps(res[-1], indent=2)
    ph_py = {"parse_check_s": t1 - t0, "intern_launch_assemble_s": t2 - t1, "render_s": t3 - t2,
             "end_to_end_s": t4 - t3}
    print(json.dumps({"metric": "payloads/sec through consensus-batch's front end (f2)",
                      "value": a.markets / best, "unit": "payloads/s",
                      "signals_per_s": a.markets * a.len / best, "end_to_end_s": best,
                      "output_bytes": len(out), "identical_to_python_path": True,
                      "python_path": {"end_to_end_s": ph_py["end_to_end_s"], "phases": ph_py,
                                      "payloads_per_s": a.markets / ph_py["end_to_end_s"]},
                      "config": {"markets": a.markets, "signals_per_market": a.len, "sources": a.sources,
                                 "host_threads": jsonl._threads()}}))


if __name__ == "__main__":
    main()
