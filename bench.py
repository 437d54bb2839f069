#!/usr/bin/env python3
"""Benchmark: batched consensus (core.compute_consensus + validation range check) on MI355X.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W`` prints ONE JSON line on
rank 0.  N > 1 is launched by torch.distributed.run, one process per GPU; every rank
processes its OWN batch of the headline workload (weak scaling, no data-path collective:
markets shard with zero communication).

Headline workload = BASELINE.json configs[1] / SURVEY.md §8(d) d2: 1,000,000 markets x 32
signals, 10,000 sources; sid ~ U{0..9999}, prob ~ U[0,1) (10% of markets on the
{0.1..0.9} grid), rel ~ U[0.1,1.0], conf ~ U[0,1], present ~ Bernoulli(0.9), PCG64
seed 2 + rank.  A "step" = one full pass of the hot path over the batch with inputs
already resident in HBM: validation + consensus + per-unique outputs (sourceWeights).

Also measured here:
  roofline      algorithmic bytes per launch / the kernel's average
                launch time from HIP events on the launch stream, vs 8.0 TB/s.
  cpu_baseline  the C restatement of the reference (oracle/, kind "port") timed on one
                host core over a bounded sample, rank 0 at N=1 only.
Other configs (--config c3|c4|c5|ns|agg) are secondary bench lines; the default is c2.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "bayesian-consensus-engine_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "signals aggregated/sec (node) at 1M markets×32 signals; % of HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=50)
    p.add_argument("--config", default="c2", choices=["c2", "c3", "c4", "c5", "ns", "agg"])
    p.add_argument("--markets", type=int, default=1_000_000)
    p.add_argument("--len", type=int, default=32)
    p.add_argument("--sources", type=int, default=10_000)
    p.add_argument("--mode", default="exact", choices=["exact", "fast"])
    p.add_argument("--agents", type=int, default=16384, help="config 5 agents")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-sample-markets", type=int, default=1_000_000)
    p.add_argument("--no-parity", action="store_true")
    return p.parse_args()


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    return world, rank, local


def barrier(world):
    if world > 1:
        dist.barrier()


def max_over_ranks(x: float, world: int) -> float:
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x: float, world: int) -> float:
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


# -------------------------------------------------------------------------------------
# config 2 workload
# -------------------------------------------------------------------------------------
def make_c2(M, L, S, seed):
    rng = np.random.default_rng(seed)
    sid = rng.integers(0, S, size=M * L, dtype=np.int32)
    prob = rng.random(M * L)
    grid = np.nonzero(rng.random(M) < 0.1)[0]
    if len(grid):
        g = prob.reshape(M, L)
        g[grid] = rng.integers(1, 10, size=(len(grid), L)) / 10.0
    rel = rng.uniform(0.1, 1.0, S)
    conf = rng.random(S)
    present = (rng.random(S) < 0.9).astype(np.uint8)
    rel = np.where(present == 1, rel, 0.5)
    conf = np.where(present == 1, conf, 0.25)
    offsets = np.arange(0, M * L + 1, L, dtype=np.int64)
    return offsets, sid, prob, rel, conf, present


def cpu_baseline_c2(offsets, sid, prob, rel, conf, present, sample_markets, min_seconds=10.0):
    """The oracle's C restatement (kind 'port') on one core over a bounded sample."""
    sys.path.insert(0, ROOT)
    from oracle import oracle as orc

    M = min(sample_markets, len(offsets) - 1)
    off = offsets[: M + 1]
    n = int(off[-1])
    # repeat the pass until ~10 s of CPU work (the bounded-sample rule), report the mean rate
    t0 = time.perf_counter()
    reps = 0
    while True:
        out = orc.consensus_csr(off, sid[:n], prob[:n], rel, conf, present)
        reps += 1
        dt = time.perf_counter() - t0
        if dt >= min_seconds:
            break
    rate = n * reps / dt
    return rate, dict(value=rate, unit="signals/s", cores=1, kind="port",
                      sample=f"{M} markets x {int(n // max(M, 1))} signals of the same workload "
                             f"(seed-identical), oracle/bce_oracle.c single-threaded, {reps} passes in {dt:.2f} s"), out, M


def bench_c2(args, world, rank):
    from bayesian_engine import _native as N, batch

    M, L, S = args.markets, args.len, args.sources
    offsets, sid, prob, rel, conf, present = make_c2(M, L, S, seed=2 + rank)
    dev = torch.device("cuda", torch.cuda.current_device())
    d_off = torch.from_numpy(offsets).to(dev)
    d_sid = torch.from_numpy(sid).to(dev)
    d_prob = torch.from_numpy(prob).to(dev)
    table = batch.SourceTable.from_arrays(torch.from_numpy(rel).to(dev), torch.from_numpy(conf).to(dev),
                                          torch.from_numpy(present).to(dev))
    res = batch._alloc(M, M * L, dev, True, True)
    stream = torch.cuda.current_stream(dev)

    def step():
        batch.consensus(d_off, d_sid, d_prob, table, max_len=L, mode=args.mode, out=res)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        step()
        ev[i][1].record(stream)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier(world)
    torch.cuda.synchronize()
    wall = t1 - t0
    kern_ms = [a.elapsed_time(b) for a, b in ev]
    avg_kernel_s = float(np.mean(kern_ms)) / 1e3
    wall_max = max_over_ranks(wall, world)

    # algorithmic bytes per launch
    sum_u = int(res.n_unique.sum().item())
    n_sig = M * L
    bytes_per_launch = 12 * n_sig + (8 * (M + 1)) + 32 * M + 20 * sum_u + 16 * S + (S + 7) // 8
    achieved_gbs = bytes_per_launch / avg_kernel_s / 1e9

    total_signals = sum_over_ranks(float(n_sig * args.steps), world)
    value = total_signals / wall_max
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "signals/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": wall_max / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (SURVEY.md d2 distributions, PCG64 seed 2+rank)",
        "config": {"workload": f"c2: {M} markets x {L} signals, {S} sources, batched consensus + "
                               f"validation + sourceWeights outputs, mode={args.mode}",
                   "markets_per_gpu": M, "signals_per_market": L, "sources": S,
                   "parallelism": f"markets sharded, {world} independent rank(s), no collective"},
        "roofline": {"bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved_gbs / HBM_PEAK_GBS, "traffic": None,
                     "kernel": "consensus_pipe_kernel<32>" if L <= 32 else "consensus_seg_kernel<64,*>",
                     "bytes_per_launch": bytes_per_launch, "avg_launch_ms": avg_kernel_s * 1e3},
        "cpu_baseline": None,
    }
    pmc = os.path.join(ROOT, "profiles", "pmc_c2.json")
    if os.path.exists(pmc):
        try:
            with open(pmc) as f:
                j = json.load(f)
            if j.get("markets") == M and j.get("signals_per_market") == L:
                out["roofline"]["traffic"] = j.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            pass
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu_val, cb, cpu_out, Ms = cpu_baseline_c2(offsets, sid, prob, rel, conf, present,
                                                   args.cpu_sample_markets)
        out["cpu_baseline"] = cb
        if not args.no_parity:
            n = int(offsets[Ms])
            ok = (np.array_equal(res.consensus[:Ms].cpu().numpy(), cpu_out["consensus"])
                  and np.array_equal(res.total_weight[:Ms].cpu().numpy(), cpu_out["total_weight"])
                  and np.array_equal(res.n_unique[:Ms].cpu().numpy(), cpu_out["n_unique"])
                  and np.array_equal(res.err_idx[:Ms].cpu().numpy(), cpu_out["err_idx"]))
            out["parity_vs_oracle_sample"] = bool(ok)
            del n
    return out


def main():
    args = parse()
    world, rank, _ = dist_setup(args)
    if args.config != "c2":
        from bench_extra import run_extra  # secondary configs

        out = run_extra(args, world, rank)
    else:
        out = bench_c2(args, world, rank)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
