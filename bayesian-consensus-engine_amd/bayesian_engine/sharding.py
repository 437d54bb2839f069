"""Multi-GPU partitioning: one process per GPU, torch.distributed over
RCCL/xGMI (backend "nccl"; "gloo" for CPU tests).

* Markets (configs 2/3) shard with ZERO communication: contiguous market ranges split at
  equal signal counts (prefix sum of the CSR offsets), source table replicated (e1).
* Sources (config 4) shard by an owner hash; the only exchange is the per-source outcome
  flags produced by market shards, combined with one SUM all-reduce (e2) whose packing
  keeps the participate and correct counts apart, so a source flagged by two shards in
  one step is detected (:class:`FlagCollision`) instead of being silently mis-read.
"""
from __future__ import annotations

from typing import Tuple

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
