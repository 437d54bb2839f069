"""Multi-GPU partitioning: one process per GPU, torch.distributed over
RCCL/xGMI (backend "nccl"; "gloo" for CPU tests).

* Markets (configs 2/3) shard with ZERO communication, source table replicated (e1): either
  contiguous market ranges at equal signal counts (:func:`shard_markets`), or -- the config-3
  split -- the length-binned plan order cut at equal measured cost (:func:`shard_markets_planned`),
  so each rank launches whole length classes; :func:`gather_csr` builds a rank's own CSR.
* Sources (config 4) shard by an owner hash; the only exchange is the per-source outcome
  flags produced by market shards, combined with one SUM all-reduce (e2) whose packing
  keeps the participate and correct counts apart, so a source flagged by two shards in
  one step is detected (:class:`FlagCollision`) instead of being silently mis-read.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist


def shard_markets(offsets_host: np.ndarray, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous market range [m0, m1) of ``rank`` so every rank gets ~N/world signals."""
    off = np.asarray(offsets_host, np.int64)
    M = len(off) - 1
    if world <= 1:
        return 0, M
    total = int(off[-1] - off[0])
    targets = off[0] + (total * np.arange(world + 1, dtype=np.float64) / world)
    cuts = np.searchsorted(off, targets, side="left")
    cuts[0], cuts[-1] = 0, M
    cuts = np.maximum.accumulate(np.clip(cuts, 0, M))
    return int(cuts[rank]), int(cuts[rank + 1])


# Length bins of the planned consensus launch (consensus.hip kBinMax, BCE_NBINS = 13): bins 0..3
# (n <= 64) run lane/segment kernels on the side stream, 4..11 the wide kernels, 12 (> 4096) the
# long kernel.
BIN_MAX = np.array([8, 16, 32, 64, 128, 256, 512, 1024, 1536, 2048, 3072, 4096], np.int64)
_WIDE_LO, _WIDE_HI = 4, 11

# Measured cost of one market in each bin's launch, config-3 batch (microseconds per market).
# Wide bins 4..11: kernel durations from rocprofv3 traces (tools/c3_pieces.py: pieces of 1/8 .. 1/1
# of each bin launched alone are linear in their market count with a few us of ramp,
# profiles/r06d/; bins 4..6 from the full step's kernel durations, profiles/r06c/); the wide
# kernels' per-market cost is set by the bin's sort size, not by the market's own length, so a
# per-market figure per bin is the model.  Side bins 0..3: the full step's lane / segment kernel
# durations.  EXACT: the wide bins scaled by the exact / fast ratio of tools/c3_bins.py
# (profiles/r06a/).  Bin 12 (> 4096, the long kernel: not in config 3) is an estimate.
PLAN_BIN_COST_US = np.array([0.00053, 0.0020, 0.0029, 0.0031,
                             0.00172, 0.00282, 0.00462, 0.0088, 0.0155, 0.0206, 0.0390, 0.0441,
                             0.2], np.float64)
PLAN_BIN_COST_US_EXACT = np.array([0.00053, 0.0020, 0.0029, 0.0031,
                                   0.0018, 0.0030, 0.0051, 0.0117, 0.0218, 0.0277, 0.0533, 0.0647,
                                   0.3], np.float64)
_SIDE_LAST = 3  # bins 0..3 run on the planned launch's side stream, under the wide bins


def market_bins(offsets_host: np.ndarray) -> np.ndarray:
    """Length bin of every market (bce_plan_bins' bin_of)."""
    lens = np.diff(np.asarray(offsets_host, np.int64))
    return np.searchsorted(BIN_MAX, lens, side="left").astype(np.int64)


def plan_order(offsets_host: np.ndarray):
    """(order int32[M], bin_start int64[14]) exactly as bce_plan_bins builds them: markets grouped
    by length bin in bin order, market order inside bins 0..3 and 12, longest first (LPT, ties
    by market order) inside the wide bins 4..11 (consensus.hip bce_plan_bins)."""
    off = np.asarray(offsets_host, np.int64)
    lens = np.diff(off)
    if len(lens) and int(lens.min()) < 0:
        raise ValueError("plan_order: offsets not monotone")
    b = market_bins(off)
    wide = (b >= _WIDE_LO) & (b <= _WIDE_HI)
    sec = np.where(wide, -lens, 0)
    order = np.lexsort((np.arange(len(lens)), sec, b)).astype(np.int32)
    bin_start = np.zeros(len(BIN_MAX) + 2, np.int64)
    bin_start[1:] = np.cumsum(np.bincount(b, minlength=len(BIN_MAX) + 1))
    return order, bin_start


def _equal_cost_cut(c: np.ndarray, world: int) -> np.ndarray:
    """Cut points of a cumulative cost array into ``world`` pieces of equal cost."""
    n = len(c)
    total = float(c[-1]) if n else 0.0
    cuts = np.searchsorted(c, total * np.arange(world + 1, dtype=np.float64) / world, side="left")
    cuts[0], cuts[-1] = 0, n
    return np.maximum.accumulate(np.clip(cuts, 0, n))


# The launch model of bce_consensus_planned's main stream (consensus.hip), for pricing a rank's
# wide / long markets: resident workgroups of each wide bin's kernel on one MI355X (256 CUs; the
# grid sizes in the traces, profiles/r06k/), the merge rules (kMergeRounds = 6: FAST merges the
# non-power-of-two bins 1025..1536 / 2049..3072 into the launch of the bin above and the 65..512
# bins into one 1-wave launch when a launch would fill fewer than 6 resident rounds; EXACT always
# merges the non-power-of-two bins), the cost per market of a bin's markets run on the wider
# kernel of a merged launch (profiles/r06d/ pieces), and a per-launch ramp + tail.  Linear in the
# market count: a model that charged whole rounds of resident workgroups (ceil(n / R)) balanced
# worse (0.84 against 0.91 of linear, profiles/r06l/) -- the workgroups of a persistent launch
# drift apart and its LPT order ends it on its cheapest markets, so partial rounds cost little.
_RESIDENT = {4: 5120, 5: 4096, 6: 4096, 7: 2048, 8: 1280, 9: 1024, 10: 512, 11: 512}
_MERGE_ROUNDS = 6.0
_LAUNCH_US = 6.0
_MERGED_COST_US = {"fast": {4: 0.0029, 5: 0.0033, 8: 0.0190, 10: 0.0416},
                   "exact": {4: 0.0031, 5: 0.0035, 8: 0.0218, 10: 0.0647}}


def _rank_main_us(cnt: np.ndarray, mode: str, cost: np.ndarray) -> float:
    """Modelled main-stream time (us) of a rank holding cnt[b] markets of each bin."""
    c = lambda b0, b1: float(cnt[b0:b1 + 1].sum())  # noqa: E731
    few = lambda b0, b1: 0 < c(b0, b1) < _MERGE_ROUNDS * _RESIDENT[b1]  # noqa: E731
    lo = {b: b for b in range(4, 13)}
    for b in (9, 11):
        if mode == "exact" or few(b - 1, b):
            lo[b] = b - 1
    if few(4, 6):
        lo[6] = 4
    merged = {k for b in lo for k in range(lo[b], b)}
    mc = _MERGED_COST_US["exact" if mode == "exact" else "fast"]
    t = 0.0
    for b in range(4, 13):
        if b in merged or c(lo[b], b) == 0:
            continue
        t += _LAUNCH_US + cnt[b] * cost[b] + sum(cnt[k] * mc.get(k, cost[k]) for k in range(lo[b], b))
    return t


def shard_markets_planned(offsets_host: np.ndarray, world: int, rank: int, mode: str = "fast",
                          cost_us: Optional[np.ndarray] = None) -> np.ndarray:
    """The markets of ``rank`` when the plan order (:func:`plan_order`: length bins, longest
    first inside the wide bins) is cut into ``world`` pieces of equal modelled time (the
    mode's measured cost per market of each bin, ``cost_us``, run through the library's launch
    and merge rules, :func:`_rank_main_us`).  Every rank then holds whole length classes -- one
    to four full-size launches of its resident grid -- instead of every bin at 1/world of its
    size (:func:`shard_markets`), which pays each launch's ramp and tail ``world`` times over.

    The short bins (n <= 64) run on the planned launch's side stream underneath the wide bins,
    so they are cut separately: rank r gets the r-th equal-cost piece of the short markets AND
    the r-th piece of the wide / long ones, and its short launches overlap its wide ones as
    they do in the full batch.  The wide cut is the smallest time T for which a greedy walk of
    the plan order fills ``world`` ranks of modelled time <= T (bisection on T).  Returns the
    market indices in ascending order (int64); :func:`gather_csr` builds the rank's own CSR from
    them and the outputs scatter back by market index."""
    off = np.asarray(offsets_host, np.int64)
    M = len(off) - 1
    if world <= 1:
        return np.arange(M, dtype=np.int64)
    cost = np.asarray(cost_us if cost_us is not None else
                      (PLAN_BIN_COST_US_EXACT if mode == "exact" else PLAN_BIN_COST_US), np.float64)
    order, bin_start = plan_order(off)
    bins = market_bins(off)
    s0 = int(bin_start[_SIDE_LAST + 1])
    # the short markets cut at equal cost: each rank's side stream runs one or two of the short
    # bins' kernels, whole or cut.  (Every short bin in world equal parts put four small side
    # launches on every rank and made the side stream the critical path of most ranks: predicted
    # 0.69-0.70 of linear against 0.90, profiles/r06h/.)
    side = order[:s0]
    cuts = _equal_cost_cut(np.cumsum(cost[bins[side]]), world)
    mine = [side[cuts[rank]:cuts[rank + 1]]]
    wide = order[s0:]
    wb = bins[wide]
    nb = len(BIN_MAX) + 1
    # plan order is bin-sorted: a piece [p0, p1) of it holds a run of bins; its per-bin counts
    # come from the bin boundaries
    wstart = bin_start[_SIDE_LAST + 1:] - s0

    def counts(p0: int, p1: int) -> np.ndarray:
        cnt = np.zeros(nb, np.float64)
        for b in range(_SIDE_LAST + 1, nb):
            a0, a1 = max(p0, int(wstart[b - _SIDE_LAST - 1])), min(p1, int(wstart[b - _SIDE_LAST]))
            if a1 > a0:
                cnt[b] = a1 - a0
        return cnt

    def pack(T: float):
        """Greedy: each rank takes the longest prefix of the rest whose modelled time <= T."""
        cut, p = [0], 0
        for _ in range(world - 1):
            lo_, hi_ = p, len(wide)
            while lo_ < hi_:  # largest q with time(p, q) <= T (time is monotone in q)
                q = (lo_ + hi_ + 1) // 2
                if _rank_main_us(counts(p, q), mode, cost) <= T:
                    lo_ = q
                else:
                    hi_ = q - 1
            p = lo_
            cut.append(p)
        cut.append(len(wide))
        return cut, _rank_main_us(counts(p, len(wide)), mode, cost)

    lo_t, hi_t = 0.0, _rank_main_us(counts(0, len(wide)), mode, cost)
    best = pack(hi_t)[0]
    for _ in range(40):
        mid = 0.5 * (lo_t + hi_t)
        cut, last = pack(mid)
        if last <= mid:
            hi_t, best = mid, cut
        else:
            lo_t = mid
    mine.append(wide[best[rank]:best[rank + 1]])
    assert wb is not None
    return np.sort(np.concatenate(mine)).astype(np.int64)


def gather_csr(offsets_host: np.ndarray, markets: np.ndarray, *arrays):
    """A market subset as its own CSR: (local offsets int64[m+1], signal index int64[n] into the
    full arrays, each of ``arrays`` gathered).  Per-unique outputs of market j of the subset sit
    at local offsets[j]; they belong at offsets_host[markets[j]] of the full batch."""
    off = np.asarray(offsets_host, np.int64)
    mk = np.asarray(markets, np.int64)
    lens = off[mk + 1] - off[mk]
    loc = np.zeros(len(mk) + 1, np.int64)
    np.cumsum(lens, out=loc[1:])
    idx = np.repeat(off[mk] - loc[:-1], lens) + np.arange(int(loc[-1]), dtype=np.int64)
    return (loc, idx) + tuple(np.asarray(a)[idx] for a in arrays)


def owner_of(source_ids: np.ndarray, world: int) -> np.ndarray:
    """Owner rank of each source rank id (multiplicative hash, stable across ranks)."""
    h = (np.asarray(source_ids, np.uint64) * np.uint64(0x9E3779B97F4A7C15)) >> np.uint64(40)
    return (h % np.uint64(max(world, 1))).astype(np.int32)


class FlagCollision(ValueError):
    """Two market shards resolved an outcome for the same source in one step."""


def combine_flags(local_flags: torch.Tensor) -> torch.Tensor:
    """All-reduce per-source outcome flags produced by market shards (e2).

    ``local_flags`` uint8[S]: bit0 participates, bit1 correct, zero where this rank's
    markets produced no outcome.  ``outcome_update`` applies at most one outcome per
    source per call, as the reference's one ``update_reliability`` call per outcome does
    (reliability.py:185-233), so two shards flagging one source in the same step is an
    error, not something to OR together: the caller must split that step in two.

    One SUM all-reduce over int32 words that keep the two bits apart (participation count
    in the low 16 bits, correct count above), then a collision check on the counts.
    Raises :class:`FlagCollision` naming the first colliding sources.
    """
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return local_flags
    f = local_flags.to(torch.int32)
    t = (f & 1) | (((f >> 1) & 1) << 16)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    part = t & 0xFFFF
    bad = torch.nonzero(part > 1).flatten()
    if bad.numel():
        raise FlagCollision(f"{bad.numel()} source(s) got outcomes from more than one market shard in "
                            f"one step (first: {bad[:8].tolist()}); split the step")
    corr = (t >> 16) > 0
    return (part | (corr.to(torch.int32) << 1)).to(torch.uint8)


def pack_owner_flags(part: torch.Tensor, corr: torch.Tensor, mine: torch.Tensor, pos: torch.Tensor,
                     world: int, blk: int) -> torch.Tensor:
    """This market shard's 2-bit outcome flags over ALL sources, laid out by owner block
    (``pos[s]`` = owner(s) * blk + index inside the owner's block) and packed 4 sources per
    byte (source j of a byte in bits 2j, 2j+1): the send buffer of the per-step
    reduce-scatter that hands each owner its block (e2).

    ``mine`` masks the sources whose outcome this shard resolved; the correct bit is set only
    with the participate bit.  Both bits are masked,
    so a rank contributes an all-zero 2-bit field for every source it did not resolve; with
    each (source, step) outcome resolved by exactly one shard the uint8 SUM of the ranks'
    buffers then never carries between fields and equals their OR.
    """
    p = (part & mine).to(torch.uint8)
    c = (part & corr & mine).to(torch.uint8)
    f = torch.zeros(world * blk, dtype=torch.uint8, device=part.device)
    f[pos] = p | (c << 1)
    f = f.view(-1, 4)
    return (f[:, 0] | (f[:, 1] << 2) | (f[:, 2] << 4) | (f[:, 3] << 6)).contiguous()


def allreduce_counts(correct: torch.Tensor, total: torch.Tensor) -> None:
    """Sum per-source agreement counts over market shards (summarize_sources, market.py:293-304)."""
    if dist.is_initialized() and dist.get_world_size() > 1:
        both = torch.stack([correct, total])
        dist.all_reduce(both, op=dist.ReduceOp.SUM)
        correct.copy_(both[0])
        total.copy_(both[1])
