"""Secondary bench lines for BASELINE.json configs 3-5 (``python bench.py --config c3|c4|c5``).

Same contract as the headline (bench.timed_loop): inputs resident in HBM before timing, a
clock ramp, W untimed warmup steps, K timed steps bracketed by barrier + synchronize, max
over ranks, one JSON line; cpu_baseline = the oracle's C restatement on the host cores this
process may use (kind "port"), over a bounded sample of the same workload, rank 0 at N=1.

  c3  100M signals ragged CSR (lengths log-uniform on [1, 4096], Zipf(1.1) sources over
      1e6 ranks), markets sharded over N ranks at equal signal counts (strong scaling:
      the 100M total is fixed).  Step = one planned consensus pass (all length bins).
  c4  10M-source reliability table, T replay steps (decayed view + outcome update per
      step, participation 0.1, correct 0.6).  Sources are owned by sharding.owner_of (a
      multiplicative hash); the table is interned in owner-grouped order so each owner's
      sources are one contiguous block.  With N > 1 every rank's market shard produces
      2-bit outcome flags over ALL sources (each (source, step) outcome from exactly one
      shard: disjoint) and one RCCL reduce-scatter delivers each owner its block.
      Step = one replay step (+ the reduce-scatter).
  c5  dense A x M re-estimation (default 16384 x 1e6 fp64 = 131 GB), markets sharded by
      column over N ranks; per iteration pass 1 (consensus), pass 2 (agreement), an
      all-reduce of the per-agent counts, the weight update.  Step = one iteration.
  ns  SURVEY §8(f) f3: namespaced fallback over a 10M-source rank space (market, domain,
      global scopes, each holding a row for ~50% of sources, 10% unparseable stamps),
      decay on.  Step = one bce_namespace_resolve launch producing the packed consensus
      table.  Sources shard by owner (weak scaling), no collective.
  tb  SURVEY §8(a) a8: DeterministicTieBreaker.resolve over the config-2 batch (1M markets
      x 32 agents, 10% of markets on the {0.1..0.9} grid so their groups tie): prediction =
      the signal's probability, confidence / reliability = its source's table row, weight =
      the reliability.  Step = one batched tie-break (winner, label, group count, variance,
      per-group diagnostics and every agent's group ordinal).
  agg SURVEY §8(f) f4: aggregate_consensus over 10k member groups of 1000 markets each
      (contiguous pattern-matched ranges of a 1M-market batch, 20% without consensus).
      Step = one bce_aggregate_groups launch (weighted_average, majority, confidence;
      median in the config string's second figure).  Groups shard over ranks (weak).
"""
from __future__ import annotations

import ctypes as C
import os
import time

import numpy as np
import torch
import torch.distributed as dist

HBM_PEAK_GBS = 8000.0
ROOT = os.path.dirname(os.path.abspath(__file__))


def _timed(step, args, world, stream, barrier=None, max_over=None):
    from bench import timed_loop

    wall, per, _ = timed_loop(step, args, world, stream)
    return wall, per


def _threads():
    from bench import host_threads

    return host_threads()


def _pmc(name, **match):
    from bench import read_pmc

    return read_pmc(name, **match)[0]


def run_extra(args, world, rank):
    from bench import barrier, max_over_ranks, sum_over_ranks  # noqa: E402

    fn = {"c3": _c3, "c4": _c4, "c5": _c5, "ns": _ns, "agg": _agg, "tb": _tb}[args.config]
    return fn(args, world, rank, barrier, max_over_ranks, sum_over_ranks)


# ---------------------------------------------------------------------------------------
# CPU baselines: the oracle's C restatement (test infrastructure, oracle/) on host threads
# ---------------------------------------------------------------------------------------
def _cpu_c3(off, sid, prob, table_host, args):
    """(cpu_baseline dict, the restatement's outputs of the first pass) or (None, None)."""
    if args.no_cpu_baseline:
        return None, None
    from bench import cpu_consensus_threaded

    rel, conf, present = table_host
    T = _threads()
    t0, reps, out = time.perf_counter(), 0, None
    while True:
        o = cpu_consensus_threaded(off, sid, prob, rel, conf, present, T)
        out = out or o
        reps += 1
        dt = time.perf_counter() - t0
        if dt >= args.cpu_seconds:
            break
    n = int(off[-1])
    return ({"value": n * reps / dt, "unit": "signals/s", "cores": T, "kind": "port", "label": "restatement",
             "sample": f"this rank's whole shard ({len(off) - 1} markets, {n} signals), oracle/bce_oracle.c on "
                       f"{T} threads, {reps} passes in {dt:.2f} s"}, out)


def _parity_c3(res, cpu, off, exact, tol=1e-9):
    """Every output at full size vs the restatement: integer outputs, usid and weight bit for
    bit; consensus / confidence / total weight / normalizedWeight bit for bit in exact mode,
    within the north star's 1e-9 absolute in fast mode (tree-ordered totals).  Returns
    ({output: ok}, max abs deviation over the float outputs)."""
    got = {k: getattr(res, k).cpu().numpy() for k in
           ("consensus", "confidence", "total_weight", "n_unique", "err_idx", "usid", "weight", "nweight")}
    u = cpu["n_unique"].astype(np.int64)
    pos = np.repeat(off[:-1], u) + (np.arange(int(u.sum())) - np.repeat(np.cumsum(u) - u, u))
    ok, dev = {}, 0.0
    for k in ("n_unique", "err_idx"):
        ok[k] = bool(np.array_equal(got[k], cpu[k]))
    for k in ("usid", "weight"):
        ok[k] = bool(np.array_equal(got[k][pos], cpu[k][pos], equal_nan=True))
    for k in ("consensus", "confidence", "total_weight", "nweight"):
        a, b = (got[k][pos], cpu[k][pos]) if k == "nweight" else (got[k], cpu[k])
        if exact:
            ok[k] = bool(np.array_equal(a, b, equal_nan=True))
        else:
            fin = np.isfinite(a) & np.isfinite(b)
            d = float(np.max(np.abs(a[fin] - b[fin]))) if fin.any() else 0.0
            dev = max(dev, d)
            ok[k] = bool(d <= tol and np.array_equal(np.isnan(a), np.isnan(b)))
    return ok, dev


def _cpu_c4(args, S_sample=2_000_000):
    """decay view + outcome update (reliability.py:104-183) per source-step, on a 2M-source
    sample of the config-4 distributions (same per-source work), over host threads."""
    if args.no_cpu_baseline:
        return None
    import sys
    from concurrent.futures import ThreadPoolExecutor

    sys.path.insert(0, ROOT)
    from oracle import oracle as orc

    rng = np.random.default_rng(4)
    now0, day = 1_772_323_200_000_000, 86_400_000_000
    rel, conf = rng.random(S_sample), rng.random(S_sample)
    t_us = now0 - (rng.random(S_sample) * 90 * day).astype(np.int64)
    present = np.ones(S_sample, np.uint8)
    flags = [((rng.random(S_sample) < 0.1).astype(np.uint8) | ((rng.random(S_sample) < 0.6).astype(np.uint8) << 1))
             for _ in range(4)]
    T = _threads()
    cuts = np.linspace(0, S_sample, T + 1).astype(np.int64)
    state = [[rel[a:b].copy(), conf[a:b].copy(), t_us[a:b].copy(), present[a:b].copy()]
             for a, b in zip(cuts[:-1], cuts[1:])]

    def part(i, k):
        a, b = int(cuts[i]), int(cuts[i + 1])
        r, c, t, pr = state[i]
        orc.decay_view(r, t, pr, now0 + k * day)
        state[i] = list(orc.outcome_update(r, c, t, pr, flags[k % 4][a:b], now0 + k * day))

    t0, k = time.perf_counter(), 0
    with ThreadPoolExecutor(T) as ex:
        while True:
            list(ex.map(lambda i: part(i, k), range(T)))
            k += 1
            dt = time.perf_counter() - t0
            if dt >= args.cpu_seconds:
                break
    return {"value": S_sample * k / dt, "unit": "source-steps/s", "cores": T, "kind": "port",
            "label": "restatement",
            "sample": f"{S_sample} sources x {k} replay steps (config-4 distributions), orc_decay_view + "
                      f"orc_outcome_update on {T} threads in {dt:.2f} s"}


def _cpu_c5(P, args, m_sample=1024):
    """One re-estimation iteration (consensus over all agents + agreement counts) on the
    first m_sample market columns of this rank's P, over host threads."""
    if args.no_cpu_baseline:
        return None
    import sys
    from concurrent.futures import ThreadPoolExecutor

    sys.path.insert(0, ROOT)
    from oracle import oracle as orc

    A = P.shape[0]
    m = min(m_sample, P.shape[1])
    Ph = P[:, :m].cpu().numpy()
    T = _threads()
    cuts = np.linspace(0, m, T + 1).astype(np.int64)
    chunks = [np.ascontiguousarray(Ph[:, a:b]) for a, b in zip(cuts[:-1], cuts[1:]) if b > a]
    t0, reps = time.perf_counter(), 0
    with ThreadPoolExecutor(T) as ex:
        while True:
            list(ex.map(lambda c: orc.reestimate(c, 1), chunks))
            reps += 1
            dt = time.perf_counter() - t0
            if dt >= args.cpu_seconds:
                break
    return {"value": A * m * reps / dt, "unit": "cells/s", "cores": T, "kind": "port", "label": "restatement",
            "sample": f"{A} agents x {m} markets (the first columns of this rank's P), one iteration per pass, "
                      f"orc_reestimate on {T} threads, {reps} passes in {dt:.2f} s"}


# ---------------------------------------------------------------------------------------
_C3_CACHE = {}


def make_c3_full(total=100_000_000, S=1_000_000):
    """Config 3, the whole batch: ragged CSR with log-uniform lengths on
    [1, 4096] and Zipf(1.1) sources over S ranks.  Returns (offsets, sid, prob, table arrays
    (rel, conf, present) as interned on the host).  Cached per process (one batch at a time)."""
    key = (total, S)
    if key in _C3_CACHE:
        return _C3_CACHE[key]
    _C3_CACHE.clear()
    rng = np.random.default_rng(3)
    lens = np.floor(np.exp(rng.uniform(0, np.log(4097), size=total // 400))).astype(np.int64)
    cs = np.cumsum(lens)
    M = int(np.searchsorted(cs, total) + 1)
    lens = lens[:M]
    lens[-1] -= int(cs[M - 1] - total)
    offsets = np.zeros(M + 1, np.int64)
    offsets[1:] = np.cumsum(lens)
    n = int(offsets[-1])
    r2 = np.random.default_rng(1000)
    perm = np.random.default_rng(33).permutation(S).astype(np.int32)
    # Zipf(1.1) truncated to S ranks (rejection: redraw values > S; clamping them to rank S
    # would pile the ~24% tail mass onto one artificial hot source)
    z = r2.zipf(1.1, size=n)
    bad = np.nonzero(z > S)[0]
    while bad.size:
        z[bad] = r2.zipf(1.1, size=bad.size)
        bad = bad[z[bad] > S]
    sid = perm[z - 1]
    del z
    prob = r2.random(n)
    rt = np.random.default_rng(34)
    rel, conf = rt.uniform(0.1, 1.0, S), rt.random(S)
    present = (rt.random(S) < 0.9).astype(np.uint8)
    rel_h, conf_h = np.where(present == 1, rel, 0.5), np.where(present == 1, conf, 0.25)
    _C3_CACHE[key] = (offsets, sid, prob, (rel_h, conf_h, present))
    return _C3_CACHE[key]


def make_c3(world=1, rank=0, total=100_000_000, S=1_000_000, split="planned", mode="fast"):
    """This rank's market shard of the config-3 batch as its own CSR: (M of the whole batch,
    offsets, sid, prob, table arrays, the shard's market indices).  ``split`` = "planned"
    (sharding.shard_markets_planned: the plan order cut at equal measured cost, whole length
    classes per rank) or "contiguous" (sharding.shard_markets: market ranges at equal signal
    counts)."""
    from bayesian_engine.sharding import gather_csr, shard_markets, shard_markets_planned

    offsets, sid, prob, table = make_c3_full(total, S)
    M = len(offsets) - 1
    if world <= 1:
        return M, offsets, sid, prob, table, np.arange(M, dtype=np.int64)
    if split == "planned":
        # A/B hook for the split's model (tools/gpu_lines.sh env: steps): a per-bin cost vector
        # in place of sharding's measured one
        kw = {}
        if os.environ.get("BCE_C3_SHARD_COST"):
            kw["cost_us"] = np.array([float(x) for x in os.environ["BCE_C3_SHARD_COST"].split(",")])
        mk = shard_markets_planned(offsets, world, rank, mode=mode, **kw)
    else:
        m0, m1 = shard_markets(offsets, world, rank)
        mk = np.arange(m0, m1, dtype=np.int64)
    loc, _, s, p = gather_csr(offsets, mk, sid, prob)
    return M, loc, s, p, table, mk


def _graphed(step, dev):
    """The step captured once as a HIP graph (torch.cuda.CUDAGraph over the library's
    launches on the current stream, the side stream joined by its fork/join events) and
    replayed: one graph launch per step instead of ~13 kernel launches and 4 event calls."""
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        for _ in range(3):
            step()
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    torch.cuda.synchronize()
    return g.replay


def _c3(args, world, rank, barrier, max_over, sum_over):
    from bayesian_engine import batch

    S = getattr(args, "c3_sources", 1_000_000)
    total = 100_000_000
    split = getattr(args, "split", "planned")
    M, off, sid, prob, table_host, mk = make_c3(world, rank, total, S, split=split, mode=args.mode or "fast")
    n = int(off[-1])
    rel_h, conf_h, present = table_host
    dev = torch.device("cuda", torch.cuda.current_device())
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    table = batch.SourceTable.from_arrays(T(rel_h), T(conf_h), T(present))
    d_off, d_sid, d_prob = T(off), T(sid), T(prob)
    plan = batch.Plan.build(off, dev)
    res = batch._alloc(len(off) - 1, n, dev, True, True)

    mode = args.mode or "fast"
    other = "exact" if mode == "fast" else "fast"
    fresh = getattr(args, "fresh", False)

    def step():
        # fresh: every step plans its batch on the GPU (batch.consensus(plan=None) ->
        # bce_plan_bins_device + one stream synchronisation), as for an incoming batch
        if fresh:  # planned on the device, no host sync (the caller's bound: C3 markets <= 4096)
            batch.consensus(d_off, d_sid, d_prob, table, max_len=4096, mode=mode, out=res)
        else:
            batch.consensus(d_off, d_sid, d_prob, table, plan=plan, mode=mode, out=res)

    def step_other():
        batch.consensus(d_off, d_sid, d_prob, table, plan=plan, mode=other, out=res)

    if getattr(args, "graph", False):
        step, step_other = _graphed(step, dev), _graphed(step_other, dev)

    # the other summation mode, timed the same way on fewer steps, reported beside the line
    import copy
    a2 = copy.copy(args)
    a2.steps, a2.warmup, a2.prewarm_s = max(5, args.steps // 4), 3, 0.0
    wall2 = per2 = None
    if not getattr(args, "single_mode", False) and not fresh:
        wall2, per2 = _timed(step_other, a2, world, torch.cuda.current_stream(dev), barrier, max_over)
    wall, per = _timed(step, args, world, torch.cuda.current_stream(dev), barrier, max_over)
    from bayesian_engine import _native as N

    N.check_faults(dev, "c3 timed steps")
    Mloc = len(off) - 1
    sum_u = int(res.n_unique.sum().item())
    touched = int(np.unique(sid).size)
    bytes_step = 12 * n + 8 * (Mloc + 1) + 32 * Mloc + 20 * sum_u + 17 * touched
    achieved = bytes_step / per / 1e9
    sig = sum_over(float(n * args.steps), world)
    cpu_line, parity = None, None
    if rank == 0 and world == 1:
        cpu_line, cpu_out = _cpu_c3(off, sid, prob, table_host, args)
        if cpu_out is not None and not args.no_parity:
            # full-size parity of both modes: res holds the timed mode's last step; one more
            # step in the other mode into a second result
            res2 = batch._alloc(len(off) - 1, n, dev, True, True)
            batch.consensus(d_off, d_sid, d_prob, table, plan=plan, mode=other, out=res2)
            torch.cuda.synchronize()
            parity = {}
            for md, r in ((mode, res), (other, res2)):
                ok, dv = _parity_c3(r, cpu_out, off, exact=(md == "exact"))
                parity[md] = {"all_ok": all(ok.values()), "outputs": ok,
                              "tolerance": "bit-exact" if md == "exact" else "1e-9 abs (float outputs)",
                              "max_abs_dev": dv}
            del res2
    parity_ranks = None
    if world > 1 and not args.no_parity:
        # every rank checks its whole shard (the timed mode's last step) against the
        # restatement on its share of the host cores, after the timed region
        from bench import cpu_consensus_threaded, gather_ranks

        cpu = cpu_consensus_threaded(off, sid, prob, *table_host, max(1, _threads() // world))
        ok, dv = _parity_c3(res, cpu, off, exact=(mode == "exact"))
        parity_ranks = gather_ranks({"rank": rank, "markets": len(off) - 1, "signals": n, "mode": mode,
                                     "all_ok": all(ok.values()), "max_abs_dev": dv}, world)
    return {
        "metric": "signals aggregated/sec (node), 100M-signal ragged CSR (config 3)",
        "value": sig / wall, "unit": "signals/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "f64", "data": "synthetic (SURVEY.md d3: log-uniform lengths, Zipf 1.1)",
        "config": {"workload": f"c3: {M} markets, {total} signals total, Zipf over {S} sources, mode={mode}, "
                               f"{'fresh batch (planned on the GPU in the step)' if fresh else 'pre-planned'}",
                   "launch": "one captured HIP graph per step" if getattr(args, "graph", False) else
                             "stream launches (plan: one kernel per length bin)",
                   "markets_this_rank": Mloc, "signals_this_rank": n, "unique_per_market_mean": sum_u / max(Mloc, 1),
                   "bins": plan.bin_start.tolist(),
                   "plan": ("planned on the GPU inside every timed step, no host sync (bce_plan_bins_device_async + "
                            "bce_consensus_planned_device: a fresh batch)" if fresh else
                            "pre-planned (Plan.build once, outside the timed steps)"),
                   "parallelism": f"markets sharded over {world} rank(s), no collective" +
                                  (f" (split: {'sharding.shard_markets_planned, whole length classes per rank' if split == 'planned' else 'sharding.shard_markets, contiguous ranges'})" if world > 1 else "")},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": (_pmc("pmc_c3.json", signals_this_rank=n) if S == 1_000_000 else
                                 _pmc(f"pmc_c3_S{S // 1_000_000}M.json", signals_this_rank=n, sources=S)),
                     "kernel": "consensus (all bins, one step)",
                     "bytes_per_launch": bytes_step, "avg_launch_ms": per * 1e3,
                     f"{other}_mode": ({"ms_per_step": wall2 / a2.steps * 1e3, "avg_launch_ms": per2 * 1e3,
                                        "frac": bytes_step / per2 / 1e9 / HBM_PEAK_GBS} if per2 else None)},
        "cpu_baseline": cpu_line,
        "parity_vs_oracle": parity,
        "parity_ranks": parity_ranks,
    }


# ---------------------------------------------------------------------------------------
def _c4(args, world, rank, barrier, max_over, sum_over):
    from bayesian_engine import batch
    from bayesian_engine.sharding import owner_of, pack_owner_flags

    S_total = 10_000_000
    dev = torch.device("cuda", torch.cuda.current_device())
    gid = np.arange(S_total, dtype=np.int64)
    owner = owner_of(gid, world)                           # sharding.owner_of: hash ownership
    counts = np.bincount(owner, minlength=world)
    blk = int((counts.max() + 3) // 4 * 4)                 # padded owner block (4 sources/byte)
    local = np.empty(S_total, np.int64)                    # index inside the owner's block
    for r in range(world):
        sel = np.nonzero(owner == r)[0]
        local[sel] = np.arange(len(sel))
    pos = torch.from_numpy(owner.astype(np.int64) * blk + local).to(dev)
    # the market shard that resolves each source's outcome (another hash): flags cross ranks
    contrib = torch.from_numpy(((gid * 0x2545F491) >> 7) % max(world, 1)).to(dev)
    S = int(counts[rank])                                   # sources this rank owns
    g = torch.Generator(device=dev)
    g.manual_seed(4 + rank)
    now0 = 1_772_323_200_000_000  # 2026-03-01T00:00:00Z in microseconds
    day = 86_400_000_000
    pad = blk
    rel = torch.rand(pad, generator=g, device=dev, dtype=torch.float64)
    conf = torch.rand(pad, generator=g, device=dev, dtype=torch.float64)
    t_us = now0 - (torch.rand(pad, generator=g, device=dev, dtype=torch.float64) * 90 * day).to(torch.int64)
    present = torch.ones(pad, dtype=torch.uint8, device=dev)
    view = torch.empty(pad, dtype=torch.float64, device=dev)
    POOL = 16
    nbytes = blk // 4

    def flags_for(k_seed):
        gg = torch.Generator(device=dev)
        gg.manual_seed(k_seed)
        part = torch.rand(S_total, generator=gg, device=dev) < 0.1
        corr = torch.rand(S_total, generator=gg, device=dev) < 0.6
        # this rank's market shard resolved the sources with contrib == rank (disjoint
        # across ranks); both flag bits are masked so the SUM reduce-scatter equals an OR
        return pack_owner_flags(part, corr, contrib == rank, pos, world, blk)

    pool = [flags_for(1000 + k) for k in range(POOL)]
    recv = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    state = {"k": 0}

    def step():
        k = state["k"]
        fl = pool[k % POOL]
        if world > 1:
            # every owner receives the sum of all shards' 2-bit flags for its block;
            # contributions are disjoint per (source, step), so SUM == OR
            dist.reduce_scatter_tensor(recv, fl, op=dist.ReduceOp.SUM)
            f2 = recv
        else:
            f2 = fl
        batch.replay_step(rel[:S], conf[:S], t_us[:S], present[:S], f2, now0 + k * day, view[:S])
        state["k"] = k + 1

    wall, per = _timed(step, args, world, torch.cuda.current_stream(dev), barrier, max_over)
    from bayesian_engine import _native as N

    N.check_faults(dev, "c4 timed steps")
    parity = _parity_c4(step, state, pool, (rel, conf, t_us, present, view), S, now0, day, args) \
        if rank == 0 and world == 1 else None
    p = 0.1
    bps = 24 + 0.25 + 8 + p * (8 + 24 + 1)
    achieved = bps * S / per / 1e9
    total_ss = sum_over(float(S * args.steps), world)
    return {
        "metric": "source-steps/sec (node), 10M-source decay + outcome replay (config 4)",
        "value": total_ss / wall, "unit": "source-steps/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (SURVEY.md d4: participation 0.1, correct 0.6, 16-step flag pool)",
        "config": {"workload": f"c4: {S_total} sources, replay_step per step", "sources_this_rank": S,
                   "parallelism": f"sources owned by sharding.owner_of over {world} rank(s); per-step outcome "
                                  f"flags from every market shard reduce-scattered to the owners"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": _pmc("pmc_c4.json", sources_this_rank=S),
                     "kernel": "replay_step_kernel", "bytes_per_launch": bps * S, "avg_launch_ms": per * 1e3},
        "cpu_baseline": _cpu_c4(args) if rank == 0 and world == 1 else None,
        "parity_vs_oracle": parity,
    }


def _parity_c4(step, state, pool, arrays, S, now0, day, args):
    """One more replay step on all S sources vs the restatement on a host snapshot of the
    table: rel / conf / t / present and the decayed view bit for bit (the view's 2.0 ** x
    is glibc pow restated)."""
    if args.no_parity or args.no_cpu_baseline:
        return None
    import sys

    sys.path.insert(0, ROOT)
    from oracle import oracle as orc

    rel, conf, t_us, present, view = arrays
    snap = [x[:S].cpu().numpy() for x in (rel, conf, t_us, present)]
    k = state["k"]
    step()
    torch.cuda.synchronize()
    fl = pool[k % len(pool)].cpu().numpy()
    flags = ((fl[:, None] >> (2 * np.arange(4, dtype=np.uint8))) & 3).reshape(-1)[:S].astype(np.uint8)
    now = now0 + k * day
    v_exp = orc.decay_view(snap[0], snap[2], snap[3], now)
    r2, c2, t2, p2 = orc.outcome_update(snap[0], snap[1], snap[2], snap[3], flags, now)
    v = view[:S].cpu().numpy()
    ulps = np.abs(v - v_exp) / np.spacing(np.abs(v_exp))
    ok = {"rel": bool(np.array_equal(rel[:S].cpu().numpy(), r2)),
          "conf": bool(np.array_equal(conf[:S].cpu().numpy(), c2)),
          "t_us": bool(np.array_equal(t_us[:S].cpu().numpy(), t2)),
          "present": bool(np.array_equal(present[:S].cpu().numpy(), p2)),
          "view": bool(np.array_equal(v, v_exp))}
    return {"all_ok": all(ok.values()), "outputs": ok, "sources": S, "participants": int((flags & 1).sum()),
            "view_bit_exact_share": float(np.mean(v == v_exp)), "view_max_ulps": float(ulps.max())}


# ---------------------------------------------------------------------------------------
def _c5(args, world, rank, barrier, max_over, sum_over):
    from bayesian_engine import _native as N

    A = getattr(args, "agents", 16384) or 16384
    M_total = args.markets if args.markets != 1_000_000 else 1_000_000
    Mloc = M_total // world + (1 if rank < M_total % world else 0)
    dev = torch.device("cuda", torch.cuda.current_device())
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    truth = torch.rand(Mloc, generator=g, device=dev) < 0.5
    P = torch.empty((A, Mloc), dtype=torch.float64, device=dev)
    CH = 256
    for a0 in range(0, A, CH):
        a1 = min(A, a0 + CH)
        u = torch.rand((3, a1 - a0, Mloc), generator=g, device=dev, dtype=torch.float64)
        P[a0:a1] = u.median(dim=0).values  # median of 3 uniforms ~ Beta(2, 2)
        del u
    oracle = torch.nonzero(torch.rand(A, generator=g, device=dev) < 0.1).flatten().tolist()
    for a in oracle:
        u = torch.rand((6, Mloc), generator=g, device=dev, dtype=torch.float64).sort(dim=0).values
        P[a] = torch.where(truth, u[4], u[1])  # Beta(5,2) / Beta(2,5) order statistics
    L = N.require_gpu()
    w = torch.full((A,), 0.5, dtype=torch.float64, device=dev)
    cons = torch.empty(Mloc, dtype=torch.float64, device=dev)
    nul = torch.empty(max(Mloc, 1), dtype=torch.uint8, device=dev)
    cnt = torch.zeros(A + 1, dtype=torch.int64, device=dev)  # agreement[A] | resolved
    K = (Mloc + 63) // 64
    votes = torch.empty((K, A), dtype=torch.int64, device=dev)  # one vote bit per cell
    words = torch.empty((2, K), dtype=torch.int64, device=dev)  # consensus votes, resolved masks
    st = N.stream(dev)
    ld = P.stride(0)
    ev_k = []
    nb = int(L.bce_reestimate_mfma_scratch_bytes(Mloc))
    scratch = torch.empty((nb + 7) // 8, dtype=torch.int64, device=dev)
    # the line's mode: the agent-order vector pass ("exact"; "fast" runs it too, batch.reestimate)
    # unless --mode mfma (w^T P on the matrix cores: votes and counts identical, consensus within
    # 4*A*2^-53); the other form is timed beside it for the MFMA utilisation report
    mode = {"m": "mfma" if args.mode == "mfma" else "exact"}

    def pass1():
        if mode["m"] == "mfma":  # w^T P on the matrix cores (near-0.5 markets redone exactly)
            N.check(L.bce_reestimate_consensus_votes_mfma(N.ptr(P), A, Mloc, ld, N.ptr(w), N.ptr(cons), N.ptr(nul),
                                                          N.ptr(votes), N.ptr(words[0]), N.ptr(words[1]),
                                                          N.ptr(scratch), scratch.numel() * 8, st), "c5 p1 mfma")
        else:
            N.check(L.bce_reestimate_consensus_votes(N.ptr(P), A, Mloc, ld, N.ptr(w), N.ptr(cons), N.ptr(nul),
                                                     N.ptr(votes), N.ptr(words[0]), N.ptr(words[1]), st), "c5 p1")

    def step():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        pass1()
        cnt.zero_()
        N.check(L.bce_reestimate_agreement_votes(N.ptr(votes), A, Mloc, N.ptr(words[0]), N.ptr(words[1]),
                                                 N.ptr(cnt[:A]), N.ptr(cnt[A:]), st), "c5 p2")
        e1.record()
        ev_k.append((e0, e1))
        if world > 1:
            dist.all_reduce(cnt, op=dist.ReduceOp.SUM)  # per-agent counts over market shards (e4)
        N.check(L.bce_reestimate_weights(A, N.ptr(cnt[:A]), N.ptr(cnt[A:]), N.ptr(w), st), "c5 w")

    w_init = w.clone()
    wall, per = _timed(step, args, world, torch.cuda.current_stream(dev), barrier, max_over)
    kern = float(np.mean([a.elapsed_time(b) for a, b in ev_k[-args.steps:]])) / 1e3
    # the other pass-1 mode, same loop on fewer steps, from the same starting weights
    import copy
    main_mode = mode["m"]
    other_m = "exact" if main_mode == "mfma" else "mfma"
    other, kern2 = {"mode": other_m, "skipped": "--single-mode"}, None
    if not getattr(args, "single_mode", False):
        mode["m"] = other_m
        w.copy_(w_init)
        a2 = copy.copy(args)
        a2.steps, a2.warmup, a2.prewarm_s = max(2, args.steps // 2), 1, 0.0
        ev_k.clear()
        wall2, _ = _timed(step, a2, world, torch.cuda.current_stream(dev), barrier, max_over)
        kern2 = float(np.mean([a.elapsed_time(b) for a, b in ev_k[-a2.steps:]])) / 1e3
        other = {"mode": mode["m"], "ms_per_step": wall2 / a2.steps * 1e3, "avg_launch_ms": kern2 * 1e3,
                 "frac": (8 * A * Mloc + 16 * A + 9 * Mloc) / kern2 / 1e9 / HBM_PEAK_GBS,
                 "traffic": _pmc("pmc_c5_mfma.json" if mode["m"] == "mfma" else "pmc_c5.json",
                                 markets_this_rank=Mloc)}
        mode["m"] = main_mode
    t_mfma = kern if main_mode == "mfma" else (kern2 or float("nan"))
    parity = None
    if rank == 0 and world == 1 and not args.no_parity and not args.no_cpu_baseline:
        parity = _parity_c5(P, L, N, st, args)
        parity["mfma_mode_votes"] = _parity_c5_mfma(P, L, N, st)
    # algorithmic: P once, w, agreement counts, consensus + null out (the vote bits, A*M/8
    # written and read back, are this implementation's intermediate -- in `traffic`)
    bytes_iter = 8 * A * Mloc + 16 * A + 9 * Mloc
    achieved = bytes_iter / kern / 1e9
    cells = sum_over(float(A * Mloc * args.steps), world)
    tflops = 2.0 * A * Mloc / kern / 1e12  # the w^T P contraction (mul + add per cell)
    return {
        "metric": "agent-market cells re-estimated/sec (node), dense consensus<->reliability (config 5)",
        "value": cells / wall, "unit": "cells/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (SURVEY.md d5: Beta(2,2) via order statistics, 10% oracle agents)",
        "config": {"workload": f"c5: {A} agents x {M_total} markets fp64, 1 iteration per step",
                   "markets_this_rank": Mloc,
                   "parallelism": f"markets sharded by column over {world} rank(s); per-agent counts all-reduced"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": _pmc("pmc_c5_mfma.json" if main_mode == "mfma" else "pmc_c5.json",
                                                  markets_this_rank=Mloc),
                     "kernel": "reestimate_consensus_votes + reestimate_agreement_votes (one iteration)",
                     "bytes_per_launch": bytes_iter, "avg_launch_ms": kern * 1e3,
                     f"{other['mode']}_mode": other,
                     "mfma": {"used": "mode='mfma' pass 1 (v_mfma_f64_4x4x4_4b_f64, one agent row of 64 "
                                      "markets per MFMA on a diagonal A operand: each lane's D accumulates "
                                      "its own cell)",
                              "mode_of_this_line": main_mode,
                              "mfma_ms_per_iteration": t_mfma * 1e3,
                              "contraction_tflops_mfma": 2.0 * A * Mloc / t_mfma / 1e12,
                              "fp64_matrix_peak_tflops": 78.6,
                              "utilisation_useful": 2.0 * A * Mloc / t_mfma / 1e12 / 78.6,
                              "utilisation_issued": 8.0 * A * Mloc / t_mfma / 1e12 / 78.6,
                              "why": "w^T P is a GEMV at 0.25 flop/B: both forms stream P at the HBM rate; the "
                                     "MFMA form issues 4x the useful flops (3 of 4 products per D element are "
                                     "zeros) and runs 1.3-1.8% behind the agent-order VALU pass, so mode='fast' "
                                     "runs the VALU kernel"}},
        "cpu_baseline": _cpu_c5(P, args) if rank == 0 and world == 1 else None,
        "parity_vs_oracle": parity,
    }


def _parity_c5_mfma(P, L, N, st, m=65536):
    """The MFMA pass 1 against the exact one on the first m market columns (from w = 0.5 and
    from a random weight vector): vote bits, consensus votes, resolved masks, null flags and
    agreement counts identical; consensus within 4*A*2^-53."""
    A = P.shape[0]
    m = min(m, P.shape[1])
    dev = P.device
    K = (m + 63) // 64
    nb = int(L.bce_reestimate_mfma_scratch_bytes(m))
    scratch = torch.empty((nb + 7) // 8, dtype=torch.int64, device=dev)
    ok, dmax = True, 0.0
    for w in (torch.full((A,), 0.5, dtype=torch.float64, device=dev),
              torch.rand(A, dtype=torch.float64, device=dev)):
        outs = []
        for fast in (False, True):
            c = torch.empty(m, dtype=torch.float64, device=dev)
            nu = torch.empty(m, dtype=torch.uint8, device=dev)
            votes = torch.empty((K, A), dtype=torch.int64, device=dev)
            words = torch.empty((2, K), dtype=torch.int64, device=dev)
            g = torch.zeros(A + 1, dtype=torch.int64, device=dev)
            if fast:
                N.check(L.bce_reestimate_consensus_votes_mfma(N.ptr(P), A, m, P.stride(0), N.ptr(w), N.ptr(c), N.ptr(nu),
                                                              N.ptr(votes), N.ptr(words[0]), N.ptr(words[1]),
                                                              N.ptr(scratch), scratch.numel() * 8, st), "mfma")
            else:
                N.check(L.bce_reestimate_consensus_votes(N.ptr(P), A, m, P.stride(0), N.ptr(w), N.ptr(c), N.ptr(nu),
                                                         N.ptr(votes), N.ptr(words[0]), N.ptr(words[1]), st), "exact")
            N.check(L.bce_reestimate_agreement_votes(N.ptr(votes), A, m, N.ptr(words[0]), N.ptr(words[1]),
                                                     N.ptr(g[:A]), N.ptr(g[A:]), st), "agree")
            outs.append((c, nu, votes, words, g))
        torch.cuda.synchronize()
        (ce, ne, ve, we, ge), (cf, nf, vf, wf, gf) = outs
        ok = ok and bool(torch.equal(ne, nf) and torch.equal(ve, vf) and torch.equal(we, wf) and torch.equal(ge, gf))
        dmax = max(dmax, float((cf - ce).abs().max().item()))
    return {"all_equal": ok, "consensus_max_abs_dev": dmax, "bound": 4 * (A + 2) * 2.0 ** -53,
            "sample": f"{A} agents x the first {m} market columns, w = 0.5 and random w"}


def _parity_c5(P, L, N, st, args, m=4096):
    """The single-read iteration on the first m market columns of this rank's P (a strided
    view: ld = the full row) from w = 0.5 vs the restatement's first iteration on the same
    columns: consensus, null flags, per-agent agreement counts and resolved count, bit for bit."""
    import sys

    sys.path.insert(0, ROOT)
    from oracle import oracle as orc

    A, Mloc = P.shape
    m = min(m, Mloc)
    dev = P.device
    w = torch.full((A,), 0.5, dtype=torch.float64, device=dev)
    cons = torch.empty(m, dtype=torch.float64, device=dev)
    nul = torch.empty(m, dtype=torch.uint8, device=dev)
    cnt = torch.zeros(A + 1, dtype=torch.int64, device=dev)
    K = (m + 63) // 64
    votes = torch.empty((K, A), dtype=torch.int64, device=dev)
    words = torch.empty((2, K), dtype=torch.int64, device=dev)
    N.check(L.bce_reestimate_consensus_votes(N.ptr(P), A, m, P.stride(0), N.ptr(w), N.ptr(cons), N.ptr(nul),
                                             N.ptr(votes), N.ptr(words[0]), N.ptr(words[1]), st), "c5 parity p1")
    N.check(L.bce_reestimate_agreement_votes(N.ptr(votes), A, m, N.ptr(words[0]), N.ptr(words[1]),
                                             N.ptr(cnt[:A]), N.ptr(cnt[A:]), st), "c5 parity p2")
    torch.cuda.synchronize()
    _, c_exp, n_exp, a_exp = orc.reestimate(P[:, :m].cpu().numpy(), 1)
    resolved_exp = int(np.sum(n_exp[0] == 0))
    ok = {"consensus": bool(np.array_equal(cons.cpu().numpy(), c_exp[0])),
          "null": bool(np.array_equal(nul.cpu().numpy(), n_exp[0])),
          "agreement": bool(np.array_equal(cnt[:A].cpu().numpy(), a_exp[0])),
          "resolved": int(cnt[A].item()) == resolved_exp}
    return {"all_ok": all(ok.values()), "outputs": ok, "sample": f"{A} agents x the first {m} market columns"}


# ---------------------------------------------------------------------------------------
def _ns(args, world, rank, barrier, max_over, sum_over):
    from bayesian_engine import _native as N
    from bayesian_engine import batch
    from bayesian_engine.timeutil import NO_TIMESTAMP

    S = 10_000_000
    dev = torch.device("cuda", torch.cuda.current_device())
    g = torch.Generator(device=dev)
    g.manual_seed(40 + rank)
    now_us = 1_772_323_200_000_000
    day = 86_400_000_000
    scopes = []
    for q in range(3):
        rel = torch.rand(S, generator=g, device=dev, dtype=torch.float64)
        conf = torch.rand(S, generator=g, device=dev, dtype=torch.float64)
        t = now_us - (torch.rand(S, generator=g, device=dev, dtype=torch.float64) * 200 * day).to(torch.int64)
        t[torch.rand(S, generator=g, device=dev) < 0.1] = NO_TIMESTAMP
        has = (torch.rand(S, generator=g, device=dev) < 0.5).to(torch.uint8)
        scopes.append(batch.ScopeTable(rel, conf, t, has))
    relconf = torch.empty((S, 2), dtype=torch.float64, device=dev)
    bits = torch.empty((S + 31) // 32, dtype=torch.int32, device=dev)
    code = torch.empty(S, dtype=torch.uint8, device=dev)
    L = N.require_gpu()
    st = torch.cuda.current_stream(dev)
    ptrs = [N.ptr(a) for sc in scopes for a in (sc.rel, sc.conf, sc.t_us, sc.has)]

    def step():
        N.check(L.bce_namespace_resolve(S, *ptrs, 1, now_us, 30.0, 0.1, 0.5, 0.25, 1, N.ptr(relconf), N.ptr(bits),
                                        N.ptr(code), C.c_void_p(st.cuda_stream)), "bce_namespace_resolve")

    wall, per = _timed(step, args, world, st, barrier, max_over)
    N.check_faults(dev, "ns timed steps")
    cpu_line, parity = (_cpu_ns(scopes, relconf, code, now_us, args) if rank == 0 and world == 1
                        else (None, None))
    # per source: 3 has bytes + the chosen scope's rel/conf/t (24 B, non-cold only) +
    # relconf 16 B + scope code 1 B + 1/8 B present bit
    noncold = float((code != 3).float().mean().item())
    bps = 3 + 24 * noncold + 17.125
    achieved = bps * S / per / 1e9
    tot = sum_over(float(S * args.steps), world)
    return {
        "metric": "sources resolved/sec (node), namespaced fallback market->domain->global->cold (SURVEY f3)",
        "value": tot / wall, "unit": "sources/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64", "data": "synthetic (3 scopes, 50% rows each, 10% unparseable stamps)",
        "config": {"workload": f"ns: {S} sources x 3 scopes per rank, decay on, mark_cold",
                   "noncold_fraction": noncold, "parallelism": f"sources sharded over {world} rank(s), no collective"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": _pmc("pmc_ns.json", sources=S),
                     "kernel": "namespace_resolve_kernel", "bytes_per_launch": bps * S, "avg_launch_ms": per * 1e3},
        "cpu_baseline": cpu_line,
        "parity_vs_oracle": parity,
    }


def _agg(args, world, rank, barrier, max_over, sum_over):
    from bayesian_engine import _native as N

    M, G, K = 1_000_000, 10_000, 1000
    dev = torch.device("cuda", torch.cuda.current_device())
    rng = np.random.default_rng(50 + rank)
    cons = torch.from_numpy(rng.random(M)).to(dev)
    conf = torch.from_numpy(rng.random(M)).to(dev)
    has = torch.from_numpy((rng.random(M) < 0.8).astype(np.uint8)).to(dev)
    starts = rng.integers(0, M - K, G)
    members = torch.from_numpy((starts[:, None] + np.arange(K)[None, :]).reshape(-1).astype(np.int64)).to(dev)
    goff = torch.from_numpy(np.arange(G + 1, dtype=np.int64) * K).to(dev)
    f64 = dict(dtype=torch.float64, device=dev)
    wavg, med, maj, mc = (torch.empty(G, **f64) for _ in range(4))
    nin = torch.empty(G, dtype=torch.int64, device=dev)
    L = N.require_gpu()
    st = torch.cuda.current_stream(dev)

    def launch(with_median):
        N.check(L.bce_aggregate_groups(N.ptr(goff), G, N.ptr(members), M, N.ptr(cons), N.ptr(conf), N.ptr(has),
                                       N.ptr(wavg), N.ptr(med) if with_median else None, N.ptr(maj), N.ptr(mc),
                                       N.ptr(nin), C.c_void_p(st.cuda_stream)), "bce_aggregate_groups")

    wall, per = _timed(lambda: launch(False), args, world, st, barrier, max_over)
    per_med = float("nan")
    if not getattr(args, "single_mode", False):  # (--single-mode: the line's launches only, for rocprof)
        _, per_med = _timed(lambda: launch(True), args, world, st, barrier, max_over)
    cpu_line, parity = (_cpu_agg(goff, members, cons, conf, has, (wavg, med, maj, mc, nin), args)
                        if rank == 0 and world == 1 else (None, None))
    # per-group latency chain (the kernel is not HBM-bound): one workgroup
    # holds a group from its first index load to its last ordered sum
    groups_per_wave_slot = G / torch.cuda.get_device_properties(dev).multi_processor_count
    bpm = 8 + 1 + 16  # member index, has byte, consensus + confidence
    achieved = bpm * G * K / per / 1e9
    tot = sum_over(float(G * K * args.steps), world)
    return {
        "metric": "market results aggregated/sec (node), aggregate_consensus over member groups (SURVEY f4)",
        "value": tot / wall, "unit": "members/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64", "data": "synthetic (1M markets, 80% with consensus)",
        "config": {"workload": f"agg: {G} groups x {K} members over {M} markets per rank; "
                               f"weighted_average+majority+confidence {per * 1e3:.4f} ms, +median {per_med * 1e3:.4f} ms",
                   "parallelism": f"groups sharded over {world} rank(s), no collective"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": _pmc("pmc_agg.json", groups=G),
                     "kernel": "aggregate_kernel", "bytes_per_launch": bpm * G * K, "avg_launch_ms": per * 1e3,
                     "latency": {"note": "latency-chain bound: per group, index loads -> gathers -> "
                                         "compaction -> three ordered sums of ~800 dependent fp64 adds",
                                 "groups_per_cu": groups_per_wave_slot,
                                 "us_per_group_per_cu": per * 1e6 / groups_per_wave_slot,
                                 "dependent_adds_per_group": int(3 * 0.8 * K)}},
        "cpu_baseline": cpu_line,
        "parity_vs_oracle": parity,
    }


# ---------------------------------------------------------------------------------------
def _cpu_tb(off, pred, conf, weight, rel, args):
    """orc_tiebreak_csr (libm pow / round like the reference) over market chunks on host
    threads.  Returns (cpu_baseline dict, outputs of the first pass) or (None, None)."""
    if args.no_cpu_baseline:
        return None, None
    import sys
    from concurrent.futures import ThreadPoolExecutor

    sys.path.insert(0, ROOT)
    from oracle import oracle as orc

    T = _threads()
    M = len(off) - 1
    cuts = np.linspace(0, M, T + 1).astype(np.int64)

    def part(i):
        m0, m1 = int(cuts[i]), int(cuts[i + 1])
        a, b = int(off[m0]), int(off[m1])
        return m0, a, orc.tiebreak_csr(off[m0:m1 + 1] - a, pred[a:b], conf[a:b], weight[a:b], rel[a:b])

    t0, reps, first = time.perf_counter(), 0, None
    with ThreadPoolExecutor(T) as ex:
        while True:
            parts = list(ex.map(part, range(T)))
            first = first or parts
            reps += 1
            dt = time.perf_counter() - t0
            if dt >= args.cpu_seconds:
                break
    N = int(off[-1])
    out = {k: np.zeros(M, parts[0][2][k].dtype) for k in ("winner", "label", "n_groups", "variance")}
    for k in ("g_key", "g_count", "g_total", "g_avgconf", "g_maxrel"):
        out[k] = np.zeros(N, parts[0][2][k].dtype)
    for m0, a, o in first:
        mm = len(o["winner"])
        for k in ("winner", "label", "n_groups", "variance"):
            out[k][m0:m0 + mm] = o[k]
        for k in ("g_key", "g_count", "g_total", "g_avgconf", "g_maxrel"):
            out[k][a:a + len(o[k])] = o[k]
    return ({"value": N * reps / dt, "unit": "signals/s", "cores": T, "kind": "port", "label": "restatement",
             "sample": f"the full workload ({M} markets x {N // max(M, 1)} agents, seed-identical), "
                       f"orc_tiebreak_csr on {T} threads, {reps} passes in {dt:.2f} s"}, out)


def _tb(args, world, rank, barrier, max_over, sum_over):
    from bayesian_engine import _native as N
    from bayesian_engine import batch
    from bench import make_c2

    M, L, S = args.markets, args.len, args.sources
    off, sid, prob, rel_t, conf_t, present = make_c2(M, L, S, seed=2 + rank)
    ragged = bool(getattr(args, "ragged", False))
    if ragged:  # lengths uniform on 1..L: the general (non-FULL) lane kernel takes every tile
        lens = np.random.default_rng(20 + rank).integers(1, L + 1, M).astype(np.int64)
        off = np.zeros(M + 1, np.int64)
        off[1:] = np.cumsum(lens)
        sid, prob = sid[:off[-1]], prob[:off[-1]]
    pred, conf, rel = prob, conf_t[sid], rel_t[sid]
    weight = rel
    dev = torch.device("cuda", torch.cuda.current_device())
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    d = [T(off), T(pred), T(conf), T(weight), T(rel)]
    # the length buckets of a ragged batch are planned once, outside the timed region (a
    # uniform batch gets no buckets: contiguous tiles, the FULL-tile kernel)
    plan = (batch.tiebreak_plan(off, dev, force=getattr(args, "tb_buckets", False))
            if L <= 32 and not getattr(args, "tb_contiguous", False) else None)
    res = batch.tiebreak(*d, offsets_host=off, plan=plan)

    def step():  # every market has L <= 64 agents: no per-step host scan of the offsets
        batch.tiebreak(*d, offsets_host=off, out=res, max_len=L, plan=plan)

    wall, per = _timed(step, args, world, torch.cuda.current_stream(dev), barrier, max_over)
    n = int(off[-1])
    ng = res.n_groups.cpu().numpy().astype(np.int64)
    sum_g = int(ng.sum())
    # in: pred, conf, weight, rel (32 B per agent) + offsets; out per market: winner,
    # variance (8 B each), label, n_groups (4 B each); per group: key, density, avg
    # confidence, max reliability (8 B each), count (4 B); per agent: group ordinal (4 B)
    bytes_step = 32 * n + 8 * (M + 1) + 24 * M + 36 * sum_g + 4 * n
    achieved = bytes_step / per / 1e9
    parity, cpu_line = None, None
    if rank == 0 and world == 1:
        cpu_line, cpu = _cpu_tb(off, pred, conf, weight, rel, args)
        if cpu is not None and not args.no_parity:
            got = {k: getattr(res, k).cpu().numpy() for k in ("winner", "label", "n_groups", "variance", "g_key",
                                                            "g_count", "g_avgconf", "g_maxrel")}
            pos = np.repeat(off[:-1], ng) + (np.arange(sum_g) - np.repeat(np.cumsum(ng) - ng, ng))
            ok = {k: bool(np.array_equal(got[k], cpu[k], equal_nan=True))
                  for k in ("winner", "label", "n_groups", "variance")}
            for k in ("g_key", "g_count", "g_avgconf", "g_maxrel"):
                ok[k] = bool(np.array_equal(got[k][pos], cpu[k][pos], equal_nan=True))
            lab = got["label"]
            parity = {"all_equal": all(ok.values()), "outputs": ok,
                      "labels": {"unanimous": int((lab == 0).sum()), "weight_density": int((lab == 1).sum()),
                                 "prediction_value_smallest": int((lab == 2).sum())},
                      "round6_variance_equal": bool(np.array_equal(np.round(got["variance"], 6),
                                                                   np.round(cpu["variance"], 6)))}
    N.check_faults(dev, "tb timed steps")
    tot = sum_over(float(n * args.steps), world)
    return {
        "metric": ("signals tie-broken/sec (node), DeterministicTieBreaker.resolve over 1M ragged markets"
                   if ragged else "signals tie-broken/sec (node), DeterministicTieBreaker.resolve over 1M markets x 32 agents"),
        "value": tot / wall, "unit": "signals/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64", "data": "synthetic (the c2 batch; 10% grid markets force ties)",
        "config": {"workload": (f"tb: {M} markets x 1..{L} agents (ragged), precision 6" if ragged else
                                f"tb: {M} markets x {L} agents, precision 6"), "groups_per_market_mean": sum_g / M,
                   "parallelism": f"markets sharded over {world} rank(s), no collective"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "traffic": (_pmc("pmc_tb_ragged.json", markets=M, ragged=1) if ragged else
                                 _pmc("pmc_tb.json", markets=M)),
                     "kernel": ("tiebreak_lpm_kernel<gather, 8 / 16 / 32 positions> (length buckets)"
                                if plan is not None and plan.buckets is not None else
                                "tiebreak_lpm_kernel (contiguous tiles: FULL + general body)" if L <= 32
                                else "tiebreak_wave_kernel"),
                     "bytes_per_launch": bytes_step, "avg_launch_ms": per * 1e3},
        "cpu_baseline": cpu_line,
        "parity_vs_oracle": parity,
    }


# ---------------------------------------------------------------------------------------
def c3_shards(args):
    """8-GPU C3 strong scaling predicted on one GPU (``bench.py --config c3 --shard all/N``):
    every rank's market shard of make_c3(world=N, rank=R) (--split: sharding.shard_markets_planned
    by default, or sharding.shard_markets) is
    timed in turn in this one process, no process group, with the bench's own loop, then
    the full batch.  Predicted efficiency = t_full / (N * max_R t_R): a rank's step on its
    own GPU is its shard alone, and the step ends with the slowest rank."""
    from bayesian_engine import _native as N
    from bayesian_engine import batch
    import copy

    spec = args.shard.split("/")
    world = int(spec[1])
    ranks = range(world) if spec[0] == "all" else [int(spec[0])]
    dev = torch.device("cuda", torch.cuda.current_device())
    mode = args.mode or "fast"
    a2 = copy.copy(args)

    split = getattr(args, "split", "planned")

    def time_one(w, r):
        M, off, sid, prob, (rel_h, conf_h, present), _ = make_c3(w, r, S=getattr(args, "c3_sources", 1_000_000),
                                                                 split=split, mode=mode)
        T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
        table = batch.SourceTable.from_arrays(T(rel_h), T(conf_h), T(present))
        d_off, d_sid, d_prob = T(off), T(sid), T(prob)
        plan = batch.Plan.build(off, dev)
        res = batch._alloc(len(off) - 1, int(off[-1]), dev, True, True)

        def step():
            batch.consensus(d_off, d_sid, d_prob, table, plan=plan, mode=mode, out=res)

        if getattr(args, "graph", False):
            step = _graphed(step, dev)
        wall, per = _timed(step, a2, 1, torch.cuda.current_stream(dev))
        N.check_faults(dev, f"c3 shard {r}/{w}")
        lens = np.diff(off)
        bins = np.searchsorted([8, 16, 32, 64, 128, 256, 512, 1024, 1536, 2048, 3072, 4096], lens, side="left")
        out = {"rank": r, "markets": int(len(lens)), "signals": int(off[-1]), "kernel_ms": per * 1e3,
               "wall_ms": wall / a2.steps * 1e3, "signals_per_bin": np.bincount(bins, weights=lens,
                                                                              minlength=13).astype(int).tolist()}
        del table, d_off, d_sid, d_prob, plan, res
        torch.cuda.empty_cache()
        return out

    import sys
    shards = []
    for r in ranks:
        shards.append(time_one(world, r))
        print(f"[c3 shards] {r}/{world}: {shards[-1]['kernel_ms']:.4f} ms", file=sys.stderr, flush=True)
    full = None if getattr(args, "shard_only", False) else time_one(1, 0)
    ms = [s["kernel_ms"] for s in shards]
    eff = full["kernel_ms"] / (world * max(ms)) if spec[0] == "all" and full else None
    out = {"metric": f"c3 predicted {world}-GPU strong-scaling efficiency (full-batch step / ({world} x slowest "
                     f"shard step), each shard timed alone on this GPU)",
           "value": eff, "unit": "fraction of linear", "mode": mode, "world": world,
           "shards": shards, "full_batch": full,
           "max_ms": max(ms), "mean_ms": float(np.mean(ms)), "max_over_mean": max(ms) / float(np.mean(ms)),
           "predicted_efficiency": eff,
           "split": ("sharding.shard_markets_planned (plan order cut at equal measured cost)" if split == "planned"
                     else "sharding.shard_markets (equal signal counts)")}
    return out


def _cpu_ns(scopes, relconf, code, now_us, args, S_sample=2_000_000):
    """orc_namespace_resolve on host threads over the first S_sample sources of the three
    scopes (same per-source work as the kernel), plus parity of the kernel's table and scope
    codes on that sample.  Returns (cpu_baseline, parity) or (None, None)."""
    if args.no_cpu_baseline:
        return None, None
    import sys
    from concurrent.futures import ThreadPoolExecutor

    sys.path.insert(0, ROOT)
    from oracle import oracle as orc

    n = min(S_sample, int(relconf.shape[0]))
    host = [tuple(x[:n].cpu().numpy() for x in (sc.rel, sc.conf, sc.t_us, sc.has)) for sc in scopes]
    T = _threads()
    cuts = np.linspace(0, n, T + 1).astype(np.int64)

    def part(i):
        a, b = int(cuts[i]), int(cuts[i + 1])
        return orc.namespace_resolve([tuple(x[a:b] for x in sc) for sc in host], True, now_us)

    t0, reps, first = time.perf_counter(), 0, None
    with ThreadPoolExecutor(T) as ex:
        while True:
            parts = list(ex.map(part, range(T)))
            first = first or parts
            reps += 1
            dt = time.perf_counter() - t0
            if dt >= args.cpu_seconds:
                break
    rel_o = np.concatenate([p[0] for p in first])
    conf_o = np.concatenate([p[1] for p in first])
    scope_o = np.concatenate([p[2] for p in first])
    rc = relconf[:n].cpu().numpy()
    ok = {"rel": bool(np.array_equal(rc[:, 0], rel_o)), "conf": bool(np.array_equal(rc[:, 1], conf_o)),
          "scope": bool(np.array_equal(code[:n].cpu().numpy(), scope_o))}
    return ({"value": n * reps / dt, "unit": "sources/s", "cores": T, "kind": "port", "label": "restatement",
             "sample": f"the first {n} sources of the 3 scopes (decay on), orc_namespace_resolve on {T} threads, "
                       f"{reps} passes in {dt:.2f} s"},
            {"all_equal": all(ok.values()), "outputs": ok, "sample": f"first {n} sources, bit for bit"})


def _cpu_agg(goff, members, cons, conf, has, outs, args):
    """orc_aggregate_groups on host threads over every group (same work as the kernel, the
    median included), plus full-size parity of the kernel's outputs."""
    if args.no_cpu_baseline:
        return None, None
    import sys
    from concurrent.futures import ThreadPoolExecutor

    sys.path.insert(0, ROOT)
    from oracle import oracle as orc

    go, mem = goff.cpu().numpy(), members.cpu().numpy()
    c, f, h = cons.cpu().numpy(), conf.cpu().numpy(), has.cpu().numpy()
    G = len(go) - 1
    T = _threads()
    cuts = np.linspace(0, G, T + 1).astype(np.int64)

    def part(i):
        g0, g1 = int(cuts[i]), int(cuts[i + 1])
        return orc.aggregate_groups(go[g0:g1 + 1] - go[g0], mem[go[g0]:go[g1]], c, f, h)

    t0, reps, first = time.perf_counter(), 0, None
    with ThreadPoolExecutor(T) as ex:
        while True:
            parts = list(ex.map(part, range(T)))
            first = first or parts
            reps += 1
            dt = time.perf_counter() - t0
            if dt >= args.cpu_seconds:
                break
    exp = {k: np.concatenate([p[k] for p in first]) for k in ("wavg", "median", "majority", "mean_conf", "n_included")}
    wavg, med, maj, mc, nin = (x.cpu().numpy() for x in outs)
    ok = {"wavg": bool(np.array_equal(wavg, exp["wavg"], equal_nan=True)),
          "median": bool(np.array_equal(med, exp["median"], equal_nan=True)),
          "majority": bool(np.array_equal(maj, exp["majority"], equal_nan=True)),
          "mean_conf": bool(np.array_equal(mc, exp["mean_conf"], equal_nan=True)),
          "n_included": bool(np.array_equal(nin, exp["n_included"]))}
    n = int(go[-1])
    return ({"value": n * reps / dt, "unit": "members/s", "cores": T, "kind": "port", "label": "restatement",
             "sample": f"all {G} groups ({n} members, median included), orc_aggregate_groups on {T} threads, "
                       f"{reps} passes in {dt:.2f} s"},
            {"all_equal": all(ok.values()), "outputs": ok, "sample": "every group, bit for bit"})
