#!/usr/bin/env python3
"""Benchmark: batched consensus (core.compute_consensus + validation range check) on MI355X.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W`` prints ONE JSON line on
rank 0.  One process per GPU: the driver may start the ranks itself with
``torch.distributed.run``; when it does not (``--gpus N`` with no WORLD_SIZE in the
environment) this script starts them -- a child ``torch.distributed.run`` with N ranks,
launched before anything touches the GPU -- and exits with its status.  Every rank
processes its OWN batch of the headline workload (weak scaling, no data-path collective:
markets shard with zero communication); the line reports the world
size the process group saw and every rank's shard.

Headline workload = BASELINE.json configs[1] / SURVEY.md §8(d) d2: 1,000,000 markets x 32
signals, 10,000 sources; sid ~ U{0..9999}, prob ~ U[0,1) (10% of markets on the
{0.1..0.9} grid), rel ~ U[0.1,1.0], conf ~ U[0,1], present ~ Bernoulli(0.9), PCG64
seed 2 + rank.  A "step" = one full pass of the hot path over the batch with inputs
already resident in HBM: validation + consensus + per-unique outputs (sourceWeights).

Also measured here:
  roofline      algorithmic bytes per launch / the kernel's average
                launch time from HIP events on the launch stream, vs 8.0 TB/s; traffic =
                the HBM bytes per launch from rocprofv3 FETCH_SIZE/WRITE_SIZE passes
                (measurements/pmc_c2.json, written by tools/gpu_profile_c2.sh).
  cpu_baseline  the C restatement of the reference (oracle/, kind "port"), on all the host
                cores this process may use, over the same workload, rank 0 at N=1 only;
                its outputs are also the full-size parity check (all eight outputs).
Before the W warmup steps the device runs the step for --prewarm-s seconds so the clocks
have ramped (a 20-step run then matches a 200-step one); that time is reported.
Other configs (--config c3|c4|c5|ns|agg|tb) are secondary bench lines; the default is c2,
and at N=1 the default run also appends c3 (pre-planned), c3_fresh (planned on the GPU in the
step), c3_shard8 (the 8-rank split's shards timed one by one: predicted strong scaling), c3 over
a 10M-source table, c4, tb, tb_ragged, ns (f3), agg (f4) and c5 (reduced steps, each with its
roofline, CPU baseline where a restatement exists and full-size parity) under "secondary"
(--no-secondary skips them).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "bayesian-consensus-engine_amd"))

import torch  # noqa: E402  (importing torch does not touch the GPU)
import torch.distributed as dist  # noqa: E402

METRIC = "signals aggregated/sec (node) at 1M markets×32 signals; % of HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=50)
    p.add_argument("--prewarm-s", type=float, default=1.0, help="clock ramp before the warmup steps")
    p.add_argument("--config", default="c2", choices=["c2", "c3", "c4", "c5", "ns", "agg", "tb"])
    p.add_argument("--markets", type=int, default=1_000_000)
    p.add_argument("--len", type=int, default=32)
    p.add_argument("--ragged", action="store_true", help="tb: market lengths uniform on 1..--len")
    p.add_argument("--tb-contiguous", action="store_true",
                   help="tb: contiguous tiles only (no length-bucket plan), the A/B for batch.tiebreak_plan")
    p.add_argument("--tb-buckets", action="store_true",
                   help="tb: always the length-bucket plan (batch.tiebreak_plan force=True), the other side of that A/B")
    p.add_argument("--sources", type=int, default=10_000)
    p.add_argument("--mode", default=None, choices=["exact", "fast", "mfma"],
                   help="consensus summation mode (default: exact for c2, where it costs nothing; fast -- "
                        "the north star's fixed-order trees within 1e-9 -- for c3, with the exact-mode "
                        "time reported beside it); c5 only: mfma = the matrix-core pass 1")
    p.add_argument("--c3-sources", type=int, default=1_000_000,
                   help="c3: Zipf source universe (SURVEY d3: 1M; 2M / 10M = the large-table lines)")
    p.add_argument("--agents", type=int, default=16384, help="config 5 agents")
    p.add_argument("--compact", action="store_true",
                   help="c2: scalars only (consensus, confidence, total weight, uniqueSources, validation) -- "
                        "no per-unique sourceWeights outputs (SURVEY.md d2 compact mode, 0.420e9 B)")
    p.add_argument("--events", default="region", choices=["step", "region"],
                   help="one HIP event pair around the timed region (default: per-step average "
                        "incl. the launch boundaries), or a pair around every step (~6 us per step)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=2.0, help="wall-clock budget of the CPU baseline")
    p.add_argument("--no-parity", action="store_true")
    p.add_argument("--backend", default="nccl", choices=["nccl", "gloo"])
    p.add_argument("--shard-only", action="store_true",
                   help="with --shard: time the shard(s) only, not the full batch (kernel traces)")
    p.add_argument("--shard", default=None,
                   help="c3 only: R/N or all/N -- time rank R's (or every rank's) market shard of an N-rank "
                        "run in this one process, no process group (predicted strong scaling)")
    p.add_argument("--split", default="planned", choices=["planned", "contiguous"],
                   help="c3 with N > 1 ranks or --shard: planned = sharding.shard_markets_planned (the plan "
                        "order cut at equal measured cost: whole length classes per rank), contiguous = "
                        "sharding.shard_markets (market ranges at equal signal counts)")
    p.add_argument("--single-mode", action="store_true",
                   help="c3 / c5: time only the line's own summation mode (profiling runs: every "
                        "dispatch of a kernel then belongs to that mode)")
    p.add_argument("--fresh", action="store_true",
                   help="c3: plan every step's batch on the GPU inside the timed step (a fresh batch: "
                        "bce_plan_bins_device + one stream synchronisation) instead of a plan built once")
    p.add_argument("--graph", action="store_true",
                   help="c3: replay each step as a captured HIP graph (one launch per step)")
    p.add_argument("--no-secondary", action="store_true",
                   help="c2 at N=1 only: skip the secondary lines (c3, c4, c5, tb) the default run appends "
                        "under 'secondary' (each a reduced-step run of its own --config line)")
    p.add_argument("--stub", action="store_true",
                   help="launcher self-test: a CPU no-op step under gloo (no GPU, no library)")
    return p.parse_args(argv)


# -------------------------------------------------------------------------------------
# process launch: one rank per GPU
# -------------------------------------------------------------------------------------
def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args, argv) -> int:
    """Start N ranks with torch.distributed.run as a CHILD process (this process has not
    touched the GPU) and return its exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.stub:
        if world > 1:
            dist.init_process_group("gloo")
    elif world > 1:
        # one rank per GPU; more ranks than GPUs only for a gloo rehearsal on a small box
        local = local % max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(local)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    else:
        torch.cuda.set_device(0)
    if world > 1 and dist.get_world_size() != args.gpus:
        raise SystemExit(f"bench.py: process group has {dist.get_world_size()} ranks, expected {args.gpus}")
    return world, rank, local


def _dev(args):
    return torch.device("cpu") if (args.stub or args.backend == "gloo") else torch.device("cuda")


def barrier(world):
    if world > 1:
        dist.barrier()


def max_over_ranks(x: float, world: int, dev=None) -> float:
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=dev or "cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x: float, world: int, dev=None) -> float:
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=dev or "cuda")
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def gather_ranks(info: dict, world: int) -> list:
    """Every rank's shard description, on every rank (rank order)."""
    if world == 1:
        return [info]
    out = [None] * world
    dist.all_gather_object(out, info)
    return out


def synchronize(args):
    if not args.stub:
        torch.cuda.synchronize()


def timed_loop(step, args, world, stream=None):
    """Prewarm (clock ramp), W warmup steps, then EXACTLY K timed steps bracketed by a
    barrier + synchronize on both sides.  Returns (max-over-ranks wall seconds,
    mean per-step kernel seconds from HIP events on `stream`, prewarm seconds)."""
    t0 = time.perf_counter()
    n_pre = 0
    while time.perf_counter() - t0 < args.prewarm_s:
        for _ in range(10):
            step()
            n_pre += 1
        synchronize(args)
    prewarm = time.perf_counter() - t0
    for _ in range(args.warmup):
        step()
    synchronize(args)
    barrier(world)
    synchronize(args)
    ev = None
    region = getattr(args, "events", "step") == "region"
    if stream is not None:
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(1 if region else args.steps)]
    t0 = time.perf_counter()
    if ev and region:
        ev[0][0].record(stream)
    for i in range(args.steps):
        if ev and not region:
            ev[i][0].record(stream)
        step()
        if ev and not region:
            ev[i][1].record(stream)
    if ev and region:
        ev[0][1].record(stream)
    synchronize(args)
    t1 = time.perf_counter()
    barrier(world)
    synchronize(args)
    if ev and region:  # launches + the boundaries between them, per step
        per = ev[0][0].elapsed_time(ev[0][1]) / 1e3 / max(args.steps, 1)
    else:
        per = float(np.mean([a.elapsed_time(b) for a, b in ev])) / 1e3 if ev else (t1 - t0) / max(args.steps, 1)
    return max_over_ranks(t1 - t0, world, _dev(args)), per, prewarm


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


def host_threads() -> int:
    """Cores this process may run on (the GPU box's share is 16; nproc shows the host)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def cpu_consensus_threaded(offsets, sid, prob, rel, conf, present, threads):
    """The oracle's C restatement over market chunks on `threads` threads (ctypes releases
    the GIL).  Returns the outputs in the engine's layout."""
    sys.path.insert(0, ROOT)
    from concurrent.futures import ThreadPoolExecutor

    from oracle import oracle as orc

    M = len(offsets) - 1
    cuts = np.linspace(0, M, threads + 1).astype(np.int64)

    def part(i):
        m0, m1 = int(cuts[i]), int(cuts[i + 1])
        a, b = int(offsets[m0]), int(offsets[m1])
        return m0, a, orc.consensus_csr(offsets[m0:m1 + 1] - a, sid[a:b], prob[a:b], rel, conf, present)

    with ThreadPoolExecutor(threads) as ex:
        parts = list(ex.map(part, range(threads)))
    N = int(offsets[-1])
    out = {k: np.zeros(M, v.dtype) for k, v in parts[0][2].items() if k in
           ("consensus", "confidence", "total_weight", "n_unique", "err_idx")}
    for k in ("usid", "weight", "nweight"):
        out[k] = np.zeros(N, parts[0][2][k].dtype)
    for m0, a, o in parts:
        mm = len(o["consensus"])
        for k in ("consensus", "confidence", "total_weight", "n_unique", "err_idx"):
            out[k][m0:m0 + mm] = o[k]
        for k in ("usid", "weight", "nweight"):
            out[k][a:a + len(o[k])] = o[k]
    return out


def cpu_baseline_c2(offsets, sid, prob, rel, conf, present, budget_s):
    threads = host_threads()
    t0 = time.perf_counter()
    reps, out = 0, None
    while True:
        o = cpu_consensus_threaded(offsets, sid, prob, rel, conf, present, threads)
        out = out or o
        reps += 1
        dt = time.perf_counter() - t0
        if dt >= budget_s:
            break
    n = int(offsets[-1])
    rate = n * reps / dt
    M = len(offsets) - 1
    return dict(value=rate, unit="signals/s", cores=threads, kind="port", label="restatement",
                sample=f"the full workload ({M} markets x {n // max(M, 1)} signals, seed-identical), "
                       f"oracle/bce_oracle.c on {threads} threads, {reps} passes in {dt:.2f} s"), out


def parity_all_outputs(res, cpu, offsets, unique=True):
    """All eight outputs vs the CPU restatement, bit for bit (per-unique slots < n_unique);
    the five per-market ones in compact mode."""
    keys = ("consensus", "confidence", "total_weight", "n_unique", "err_idx")
    got = {k: getattr(res, k).cpu().numpy() for k in keys + (("usid", "weight", "nweight") if unique else ())}
    ok = {}
    for k in ("n_unique", "err_idx"):
        ok[k] = bool(np.array_equal(got[k], cpu[k]))
    for k in ("consensus", "confidence", "total_weight"):
        ok[k] = bool(np.array_equal(got[k], cpu[k], equal_nan=True))
    if not unique:
        return ok
    u = cpu["n_unique"].astype(np.int64)
    pos = np.repeat(offsets[:-1], u) + (np.arange(int(u.sum())) - np.repeat(np.cumsum(u) - u, u))
    for k in ("usid", "weight", "nweight"):
        ok[k] = bool(np.array_equal(got[k][pos], cpu[k][pos], equal_nan=True))
    return ok


def read_pmc(name, **match):
    """HBM bytes per launch from a committed rocprofv3 PMC summary (None if absent or
    collected on another shape)."""
    path = os.path.join(ROOT, "measurements", name)
    try:
        with open(path) as f:
            j = json.load(f)
    except (OSError, ValueError):
        return None, None
    if any(j.get(k) != v for k, v in match.items()):
        return None, None
    return j.get("hbm_bytes_per_launch"), j.get("kernel")


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
    uniq = not args.compact
    res = batch._alloc(M, M * L, dev, uniq, True)
    stream = torch.cuda.current_stream(dev)

    def step():
        batch.consensus(d_off, d_sid, d_prob, table, max_len=L, mode=args.mode or "exact", out=res,
                        unique_outputs=uniq)

    wall, avg_kernel_s, prewarm = timed_loop(step, args, world, stream)
    N.check_faults(dev, "c2 timed steps")  # a kernel that gave up would leave stale outputs

    # algorithmic bytes per launch
    sum_u = int(res.n_unique.sum().item())
    n_sig = M * L
    bytes_per_launch = (12 * n_sig + (8 * (M + 1)) + 32 * M + (20 * sum_u if uniq else 0) + 16 * S
                        + (S + 7) // 8)
    achieved_gbs = bytes_per_launch / avg_kernel_s / 1e9
    # the kernel bce_consensus_csr picks (consensus.hip launch_seg_for_len)
    kernel = ("consensus_tab32_kernel" if 16 < L <= 32 and S <= 10112 else
              "consensus_tab32_kernel<hybrid>" if 16 < L <= 32 and S <= (1 << 18) else
              "consensus_pipe_kernel" if L <= 32 and uniq else
              "consensus_flat_kernel" if L <= 32 else "consensus_seg_kernel")
    traffic, _ = (read_pmc("pmc_c2.json", markets=M, signals_per_market=L, sources=S, kernel=kernel)
                  if uniq else (None, None))

    total_signals = sum_over_ranks(float(n_sig * args.steps), world)
    value = total_signals / wall
    ranks = gather_ranks({"rank": rank, "device": torch.cuda.get_device_name(dev), "markets": M,
                          "signals": n_sig, "kernel_ms": avg_kernel_s * 1e3}, world)
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "signals/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": wall / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (SURVEY.md d2 distributions, PCG64 seed 2+rank)",
        "config": {"workload": f"c2: {M} markets x {L} signals, {S} sources, batched consensus + "
                               f"validation{' + sourceWeights outputs' if uniq else ' (compact: scalars only)'}, "
                               f"mode={args.mode or 'exact'}",
                   "markets_per_gpu": M, "signals_per_market": L, "sources": S,
                   "parallelism": f"markets sharded, {world} independent rank(s), no collective"},
        "world_size": world,
        "ranks": ranks,
        "prewarm_s": round(prewarm, 3),
        "roofline": {"bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved_gbs / HBM_PEAK_GBS, "traffic": traffic, "kernel": kernel,
                     "bytes_per_launch": bytes_per_launch, "avg_launch_ms": avg_kernel_s * 1e3},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cb, cpu_out = cpu_baseline_c2(offsets, sid, prob, rel, conf, present, args.cpu_seconds)
        out["cpu_baseline"] = cb
        if not args.no_parity:
            ok = parity_all_outputs(res, cpu_out, offsets, uniq)
            out["parity_vs_oracle"] = {"all_equal": all(ok.values()), "outputs": ok}
    if world > 1 and not args.no_parity:
        # every rank checks its own shard (a bounded prefix of its batch) against the
        # restatement, after the timed region
        out["parity_ranks"] = gather_ranks(rank_parity(res, offsets, sid, prob, rel, conf, present, uniq,
                                                       rank), world)
    return out


def rank_parity(res, offsets, sid, prob, rel, conf, present, unique, rank, m_sample=20000):
    """This rank's outputs for its first m_sample markets vs the C restatement run on them
    (all eight outputs bit for bit; N > 1 lines, where the full-size check runs on no rank)."""
    sys.path.insert(0, ROOT)
    from oracle import oracle as orc

    m = min(m_sample, len(offsets) - 1)
    sub = offsets[:m + 1]
    n = int(sub[-1])
    cpu = orc.consensus_csr(sub - sub[0], sid[:n], prob[:n], rel, conf, present)
    keys = ("consensus", "confidence", "total_weight", "n_unique", "err_idx")
    got = {k: getattr(res, k)[:m].cpu().numpy() for k in keys}
    ok = {k: bool(np.array_equal(got[k], cpu[k], equal_nan=True)) for k in keys}
    if unique:
        u = cpu["n_unique"].astype(np.int64)
        pos = np.repeat(sub[:-1], u) + (np.arange(int(u.sum())) - np.repeat(np.cumsum(u) - u, u))
        for k in ("usid", "weight", "nweight"):
            ok[k] = bool(np.array_equal(getattr(res, k)[:n].cpu().numpy()[pos], cpu[k][pos], equal_nan=True))
    return {"rank": rank, "markets": m, "signals": n, "all_equal": all(ok.values())}


# (line, config, steps, warmup, clock ramp s, extra args): the clock ramp as in each config's own
# line; c3_fresh = config 3 planned on the GPU inside every step (a fresh batch); c3_shard8 = the
# 8-rank planned split's shards timed one by one + the full batch (predicted strong scaling);
# c3_S10M = config 3 over C4's 10M-source table (64-bit sort keys); tb_ragged = the tie-break
# over 1M markets of 1..32 agents; ns / agg = SURVEY §8(f) f3 / f4
SECONDARY = (("c3", "c3", 20, 3, 1.0, {}), ("c3_fresh", "c3", 20, 3, 0.5, {"fresh": True, "single_mode": True}),
             ("c3_shard8", "c3", 20, 3, 0.3, {"shard": "all/8", "single_mode": True}),
             ("c3_S10M", "c3", 10, 2, 0.5, {"c3_sources": 10_000_000}),
             ("c4", "c4", 100, 10, 1.0, {}), ("tb", "tb", 10, 2, 1.0, {}),
             ("tb_ragged", "tb", 10, 2, 0.5, {"ragged": True}), ("ns", "ns", 50, 5, 0.5, {}),
             ("agg", "agg", 50, 5, 0.5, {}), ("c5", "c5", 4, 1, 0.5, {}))


def run_secondary(args, world, rank) -> dict:
    """The other BASELINE.json configs, each timed exactly like its own ``--config`` line
    (reduced steps, same CPU baseline and full-size parity), summarised under the headline
    line so the default run measures every config.  N = 1 only: configs 4 and 5 exchange
    per-source flags / per-agent counts over RCCL when N > 1 (``--config c4|c5 --gpus N``)."""
    import copy
    import gc

    from bench_extra import run_extra

    out = {}
    for line, cfg, steps, warmup, ramp, extra in SECONDARY:
        a2 = copy.copy(args)
        a2.config, a2.steps, a2.warmup, a2.prewarm_s, a2.mode = cfg, steps, warmup, ramp, None
        for k, v in extra.items():
            setattr(a2, k, v)
        t0 = time.perf_counter()
        try:
            if getattr(a2, "shard", None):
                from bench_extra import c3_shards
                j = c3_shards(a2)
                out[line] = {k: j.get(k) for k in ("metric", "value", "unit", "mode", "world", "max_ms", "mean_ms",
                                                  "max_over_mean", "predicted_efficiency", "split", "full_batch")}
                out[line]["shards"] = [{k: x[k] for k in ("rank", "markets", "signals", "kernel_ms")}
                                       for x in j["shards"]]
                out[line]["steps"] = steps
                out[line]["wall_s"] = round(time.perf_counter() - t0, 1)
                gc.collect()
                torch.cuda.empty_cache()
                print(f"[bench] secondary {line}: {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
                continue
            j = run_extra(a2, world, rank)
            r = j.get("roofline") or {}
            cb = j.get("cpu_baseline") or {}
            par = j.get("parity_vs_oracle")
            out[line] = {"metric": j["metric"], "value": j["value"], "unit": j["unit"], "steps": steps,
                        "ms_per_step": j["ms_per_step"], "dtype": j.get("dtype"), "config": j.get("config"),
                        "roofline": {k: r.get(k) for k in ("bound", "achieved", "peak", "unit", "frac", "traffic",
                                                           "kernel", "bytes_per_launch", "avg_launch_ms", "mfma",
                                                           "exact_mode", "fast_mode") if k in r},
                        "cpu_baseline": cb or None, "parity_vs_oracle": par,
                        "wall_s": round(time.perf_counter() - t0, 1)}
        except Exception as exc:  # a secondary line never takes the headline down
            out[line] = {"error": f"{type(exc).__name__}: {exc}"}
        gc.collect()
        torch.cuda.empty_cache()
        print(f"[bench] secondary {line}: {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
    return out


def bench_stub(args, world, rank):
    """Launcher self-test (tests/test_bench_launcher.py): same timing skeleton, CPU no-op step."""
    wall, per, prewarm = timed_loop(lambda: None, args, world)
    ranks = gather_ranks({"rank": rank, "pid": os.getpid()}, world)
    return {"metric": "stub", "value": world * args.steps / max(wall, 1e-9), "unit": "steps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": wall / max(args.steps, 1) * 1e3,
            "world_size": world, "ranks": ranks, "prewarm_s": round(prewarm, 3)}


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.mode == "mfma" and args.config != "c5":
        raise SystemExit("bench.py: --mode mfma is the config-5 matrix-core pass (--config c5)")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args, argv))
    world, rank, _ = dist_setup(args)
    if args.stub:
        out = bench_stub(args, world, rank)
    elif args.shard:
        from bench_extra import c3_shards

        out = c3_shards(args)
    elif args.config != "c2":
        from bench_extra import run_extra  # secondary configs

        out = run_extra(args, world, rank)
    else:
        out = bench_c2(args, world, rank)
        if world == 1 and not args.no_secondary:
            out["secondary"] = run_secondary(args, world, rank)
    if rank == 0:
        if isinstance(out.get("roofline"), dict):  # how avg_launch_ms was taken
            out["roofline"]["timing"] = ("HIP events around the timed region / steps (launches + boundaries)"
                                         if args.events == "region" else "HIP events around every step")
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
