"""Batched entry points over millions of markets.

All array arguments are device tensors (torch, ``cuda:N``); results stay in HBM.  Each
function is one or a few launches of the HIP kernels in ``libbce_hip.so`` on the current
stream -- there is no CPU fallback (see :mod:`bayesian_engine._native`).

Layout (include/bce.h):
  markets  CSR  offsets int64[M+1], sid int32[N] (interned source ranks in Python
           ``sorted()`` order), prob fp64[N]
  sources  dense table over ranks: rel fp64[S], conf fp64[S] (cold-start defaults baked
           in), present u8[S]; optional t_us int64[S] for decay
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Iterable, List, Optional, Sequence

import numpy as np
import torch

from . import _native as N
from .config import DECAY_HALF_LIFE_DAYS, DECAY_MINIMUM, DEFAULT_CONFIDENCE, DEFAULT_RELIABILITY

_MODES = {"exact": N.MODE_EXACT, "fast": N.MODE_FAST}


# ---------------------------------------------------------------------------------------
# host-side interning and table building
# ---------------------------------------------------------------------------------------
def intern(ids: Iterable[str]) -> Dict[str, int]:
    """Rank ids in Python ``sorted()`` (code-point) order: integer order == str order."""
    return {s: i for i, s in enumerate(sorted(set(ids)))}


@dataclass
class SourceTable:
    """Dense per-source table resident in HBM, in the consensus kernel's layout.

    relconf [S, 2] fp64: interleaved {reliability, confidence} -> one 16-B gather per
    unique source; bits [ceil(S/32)] int32: present bitmask ("sourceId is a key of the
    reliability dict", core.py:167-170).  Cold-start defaults are baked into relconf.
    """

    relconf: torch.Tensor
    bits: torch.Tensor
    names: List[str]
    t_us: Optional[torch.Tensor] = None

    @property
    def n(self) -> int:
        return len(self.names)

    @property
    def rel(self) -> torch.Tensor:
        return self.relconf[:, 0]

    @property
    def conf(self) -> torch.Tensor:
        return self.relconf[:, 1]

    @classmethod
    def from_arrays(cls, rel: torch.Tensor, conf: torch.Tensor, present: Optional[torch.Tensor],
                    names: Optional[Sequence[str]] = None, t_us: Optional[torch.Tensor] = None) -> "SourceTable":
        """Pack device arrays with bce_table_pack (one launch)."""
        L = N.require_gpu()
        S = rel.numel()
        dev = rel.device
        relconf = torch.empty((max(S, 1), 2), dtype=torch.float64, device=dev)
        bits = torch.zeros(max((S + 31) // 32, 1), dtype=torch.int32, device=dev)
        rel = rel.to(torch.float64).contiguous()
        conf = conf.to(torch.float64).contiguous()
        pres = present.to(torch.uint8).contiguous() if present is not None else None
        N.check(L.bce_table_pack(S, N.ptr(rel), N.ptr(conf), N.ptr(pres), N.ptr(relconf), N.ptr(bits),
                                 N.stream(dev)), "bce_table_pack")
        return cls(relconf, bits, list(names) if names is not None else [""] * S, t_us)

    @classmethod
    def from_dict(cls, names: Sequence[str], source_reliability: Optional[dict], device=None) -> "SourceTable":
        """core.py:110-112 semantics: a key present (even with a partial dict) is not cold."""
        S = len(names)
        rel = np.full(max(S, 1), DEFAULT_RELIABILITY, np.float64)
        conf = np.full(max(S, 1), DEFAULT_CONFIDENCE, np.float64)
        present = np.zeros(max(S, 1), np.uint8)
        sr = source_reliability or {}
        for i, n in enumerate(names):
            if n in sr:
                present[i] = 1
                d = sr.get(n, {})  # a None value raises AttributeError, as core.py:110-111 does
                r = d.get("reliability", DEFAULT_RELIABILITY)
                c = d.get("confidence", DEFAULT_CONFIDENCE)
                acc = 0.0
                acc += r  # same TypeError as core.py:120 for non-numbers
                rel[i] = float(r)
                conf[i] = float(c)
        dev = device or N.device()
        T = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
        return cls.from_arrays(T(rel[:S]), T(conf[:S]), T(present[:S]), names)


@dataclass
class ReliabilityTable:
    """Store-side table (SoA) for the streaming decay / outcome-update kernels.

    rel, conf fp64[S], t_us int64[S] (updated_at as microseconds, NO_TIMESTAMP if
    falsy/unparseable), present u8[S] (a row exists).  Absent rows hold the baked
    cold-start values (0.5, 0.25, NO_TIMESTAMP), reliability.py:133-140.
    """

    rel: torch.Tensor
    conf: torch.Tensor
    t_us: torch.Tensor
    present: torch.Tensor
    names: List[str]

    @property
    def n(self) -> int:
        return len(self.names)

    def view(self, now_us: int) -> torch.Tensor:
        """get_reliability(apply_decay=True).reliability of every source."""
        return decay_view(self.rel, self.t_us, now_us, present=self.present)

    def consensus_table(self, now_us: Optional[int] = None, all_present: bool = True) -> "SourceTable":
        """Packed consensus table; reliability decayed at ``now_us`` when given.  Callers that
        fetch every source through get_reliability (market.py:209-219, cli.py:37-44) put
        every sourceId in the dict, hence ``all_present``."""
        rel = self.view(now_us) if now_us is not None else self.rel
        return SourceTable.from_arrays(rel, self.conf, None if all_present else self.present, self.names)


# ---------------------------------------------------------------------------------------
# consensus
# ---------------------------------------------------------------------------------------
@dataclass
class Plan:
    """Markets binned by length (bce_plan_bins), reusable across calls on the same CSR."""

    order: torch.Tensor
    bin_start: np.ndarray
    max_len: int
    scratch: Optional[torch.Tensor]

    @classmethod
    def build(cls, offsets_host: np.ndarray, device=None) -> "Plan":
        L = N.lib()
        off = np.ascontiguousarray(offsets_host, np.int64)
        M = len(off) - 1
        order = np.zeros(max(M, 1), np.int32)
        bins = np.zeros(N.NBINS + 1, np.int64)
        mx = np.zeros(1, np.int32)
        N.check(L.bce_plan_bins(N.ptr(off), M, N.ptr(order), N.ptr(bins), N.ptr(mx)), "plan_bins")
        sb = int(L.bce_consensus_scratch_bytes(N.ptr(off), N.ptr(order), N.ptr(bins)))
        dev = device or N.device()
        scratch = torch.empty(sb, dtype=torch.uint8, device=dev) if sb > 0 else None
        return cls(torch.from_numpy(order).to(dev), bins, int(mx[0]), scratch)

    @classmethod
    def build_device(cls, offsets: torch.Tensor) -> "Plan":
        """The same plan built on the GPU from the device offsets (bce_plan_bins_device: a
        stable radix sort by bin and LPT key, no D2H copy of the CSR).  One stream
        synchronisation returns the bin boundaries to the host."""
        L = N.require_gpu()
        dev = offsets.device
        M = offsets.numel() - 1
        order = torch.empty(max(M, 1), dtype=torch.int32, device=dev)
        sb = int(L.bce_plan_device_scratch_bytes(M))
        work = torch.empty(max(sb, 1), dtype=torch.uint8, device=dev)
        bins = np.zeros(N.NBINS + 1, np.int64)
        mx = np.zeros(1, np.int32)
        lsb = np.zeros(1, np.int64)
        N.check(L.bce_plan_bins_device(N.ptr(offsets), M, N.ptr(order), N.ptr(bins), N.ptr(mx), N.ptr(lsb),
                                       N.ptr(work), sb, N.stream(dev)), "plan_bins_device")
        scratch = torch.empty(int(lsb[0]), dtype=torch.uint8, device=dev) if lsb[0] > 0 else None
        return cls(order, bins, int(mx[0]), scratch)

    @classmethod
    def for_markets(cls, offsets_host: np.ndarray, markets: np.ndarray, device=None) -> "Plan":
        """The plan of a market subset over the FULL CSR (a rank's markets of
        sharding.shard_markets_planned left in place): the subset binned and LPT-ordered as
        bce_plan_bins would, its order holding the full batch's market indices, so outputs land
        at those markets and per-unique outputs at their absolute CSR offsets."""
        from .sharding import gather_csr, plan_order
        L = N.lib()
        off = np.ascontiguousarray(offsets_host, np.int64)
        mk = np.asarray(markets, np.int64)
        loc = gather_csr(off, mk)[0]
        lorder, bins = plan_order(loc)
        order = np.ascontiguousarray(mk[lorder].astype(np.int32))
        lens = np.diff(loc)
        sb = int(L.bce_consensus_scratch_bytes(N.ptr(off), N.ptr(order), N.ptr(bins)))
        dev = device or N.device()
        scratch = torch.empty(sb, dtype=torch.uint8, device=dev) if sb > 0 else None
        return cls(torch.from_numpy(order).to(dev), bins, int(lens.max(initial=0)), scratch)


@dataclass
class ConsensusResult:
    consensus: torch.Tensor      # fp64[M]  (0.0 where null)
    confidence: torch.Tensor     # fp64[M]
    total_weight: torch.Tensor   # fp64[M]
    n_unique: torch.Tensor       # int32[M]
    err_idx: Optional[torch.Tensor]   # int32[M]: first out-of-range signal, -1 if none
    usid: Optional[torch.Tensor]      # int32[N]: rank | cold<<31 at CSR offsets
    weight: Optional[torch.Tensor]    # fp64[N]
    nweight: Optional[torch.Tensor]   # fp64[N]

    def is_null(self, offsets: torch.Tensor) -> torch.Tensor:
        """consensus is None: empty market (core.py:88) or total weight == 0 (core.py:131)."""
        return (self.total_weight == 0) | (offsets[1:] == offsets[:-1])


def _alloc(M: int, Nsig: int, dev, unique: bool, validate: bool) -> ConsensusResult:
    f64 = dict(dtype=torch.float64, device=dev)
    i32 = dict(dtype=torch.int32, device=dev)
    return ConsensusResult(
        torch.empty(M, **f64), torch.empty(M, **f64), torch.empty(M, **f64), torch.empty(M, **i32),
        torch.empty(M, **i32) if validate else None,
        torch.empty(max(Nsig, 1), **i32) if unique else None,
        torch.empty(max(Nsig, 1), **f64) if unique else None,
        torch.empty(max(Nsig, 1), **f64) if unique else None)


def consensus(offsets: torch.Tensor, sid: torch.Tensor, prob: torch.Tensor, table: SourceTable, *,
              plan: Optional[Plan] = None, max_len: Optional[int] = None, mode: str = "exact",
              unique_outputs: bool = True, validate: bool = True, check: bool = False,
              out: Optional[ConsensusResult] = None) -> ConsensusResult:
    """core.compute_consensus for every CSR market (+ the validation range check).

    Pass ``max_len`` (<= 64: one launch, no planning) or a prebuilt :class:`Plan` for
    ragged batches.  Without a plan, the batch is planned on the GPU: with a ``max_len`` bound
    of 65..4096 entirely on the device, with no host synchronisation
    (bce_plan_bins_device_async + bce_consensus_planned_device; a market longer than the bound
    raises the device fault word), else by :meth:`Plan.build_device` (one stream
    synchronisation returns the bin boundaries).  A caller that reruns the same CSR should
    build the Plan once.

    ``mode="fast"`` (fixed-order trees, <= 1e-9 absolute vs the reference order) is
    deterministic per call shape but not invariant to batch composition: a small call (e.g. a
    market shard) may run a length bin in the wider launch of the bin above it, which sums the
    partial totals in another fixed order, so the same market's float outputs can differ in the
    last bits between a full batch and a shard (within 1e-9; include/bce.h BCE_MODE_FAST).
    ``mode="exact"`` is bit-identical in every launch shape.

    Raw CSR is trusted for speed: a ``sid`` outside ``[0, table.n)`` has its row read
    clamped and a market longer than ``max_len`` is left unprocessed; either raises the
    device fault word.  ``check=True`` synchronises and raises :class:`BCEError` for it
    (otherwise call ``_native.check_faults()`` when convenient).
    """
    L = N.require_gpu()
    M = offsets.numel() - 1
    Nsig = sid.numel()
    dev = offsets.device
    res = out or _alloc(M, Nsig, dev, unique_outputs, validate)
    common = (N.ptr(offsets), M, N.ptr(sid), N.ptr(prob), Nsig, N.ptr(table.relconf), N.ptr(table.bits),
              table.n)
    outs = (N.ptr(res.consensus), N.ptr(res.confidence), N.ptr(res.total_weight), N.ptr(res.n_unique),
            N.ptr(res.err_idx), N.ptr(res.usid), N.ptr(res.weight), N.ptr(res.nweight))
    md = _MODES[mode]
    if plan is None and max_len is not None and 0 < max_len <= 64:
        rc = L.bce_consensus_csr(*common, N.ptr(None), 0, int(max_len), md, *outs, N.stream(dev))
        N.check(rc, "bce_consensus_csr")
        if check:
            N.check_faults(dev, "consensus")
        return res
    if plan is None and max_len is not None and 64 < max_len <= 4096 and table.n <= (1 << 25):
        # a fresh ragged batch under the caller's bound: planned on the device and launched with
        # no host synchronisation (bce_plan_bins_device_async + bce_consensus_planned_device)
        order = torch.empty(max(M, 1), dtype=torch.int32, device=dev)
        sb = int(L.bce_plan_device_scratch_bytes(M))
        work = torch.empty(max(sb, 1), dtype=torch.uint8, device=dev)
        bins = torch.empty(N.NBINS + 1, dtype=torch.int64, device=dev)
        st = N.stream(dev)
        N.check(L.bce_plan_bins_device_async(N.ptr(offsets), M, N.ptr(order), N.ptr(bins), N.ptr(work), sb, st),
                "bce_plan_bins_device_async")
        N.check(L.bce_consensus_planned_device(*common, N.ptr(order), N.ptr(bins), md, *outs, st),
                "bce_consensus_planned_device")
        if check:
            N.check_faults(dev, "consensus")
        return res
    if plan is None:
        plan = Plan.build_device(offsets)
    sb = plan.scratch.numel() if plan.scratch is not None else 0
    rc = L.bce_consensus_planned(*common, N.ptr(plan.order), N.ptr(plan.bin_start), md, *outs,
                                 N.ptr(plan.scratch), sb, N.stream(dev))
    N.check(rc, "bce_consensus_planned")
    if check:
        N.check_faults(dev, "consensus")
    return res


def validate(offsets: torch.Tensor, prob: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """validate_input_payload's range check for every market: first bad index or -1."""
    L = N.require_gpu()
    M = offsets.numel() - 1
    err = out if out is not None else torch.empty(max(M, 1), dtype=torch.int32, device=offsets.device)
    N.check(L.bce_validate_csr(N.ptr(offsets), M, N.ptr(prob), N.ptr(err), N.stream(offsets.device)),
            "bce_validate_csr")
    return err[:M]


# ---------------------------------------------------------------------------------------
# decay / outcome update
# ---------------------------------------------------------------------------------------
def decay_view(rel: torch.Tensor, t_us: torch.Tensor, now_us: int, present: Optional[torch.Tensor] = None,
               half_life_days: float = DECAY_HALF_LIFE_DAYS, min_rel: float = DECAY_MINIMUM,
               default_rel: float = DEFAULT_RELIABILITY, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """get_reliability(apply_decay=True) for a whole table (reliability.py:110-131)."""
    L = N.require_gpu()
    n = rel.numel()
    view = out if out is not None else torch.empty(max(n, 2), dtype=torch.float64, device=rel.device)
    N.check(L.bce_decay_view(n, N.ptr(rel), N.ptr(t_us), N.ptr(present), int(now_us), float(half_life_days),
                             float(min_rel), float(default_rel), N.ptr(view), N.stream(rel.device)),
            "bce_decay_view")
    return view[:n]


def decay_apply(rel: Optional[torch.Tensor], elapsed_days: torch.Tensor,
                half_life_days: float = DECAY_HALF_LIFE_DAYS, min_rel: float = DECAY_MINIMUM,
                want_factor: bool = False):
    """decay.compute_decay_factor / apply_reliability_decay on arrays (decay.py:31-100)."""
    L = N.require_gpu()
    n = elapsed_days.numel()
    dev = elapsed_days.device
    out = torch.empty(n, dtype=torch.float64, device=dev) if rel is not None else None
    fac = torch.empty(n, dtype=torch.float64, device=dev) if want_factor else None
    N.check(L.bce_decay_apply(n, N.ptr(rel), N.ptr(elapsed_days), float(half_life_days), float(min_rel),
                              N.ptr(out), N.ptr(fac), N.stream(dev)), "bce_decay_apply")
    return out, fac


def outcome_update(rel: torch.Tensor, conf: torch.Tensor, t_us: torch.Tensor, present: torch.Tensor,
                   flags: torch.Tensor, now_us: int, default_rel: float = DEFAULT_RELIABILITY,
                   default_conf: float = DEFAULT_CONFIDENCE) -> None:
    """In-place update_reliability math for every participant (reliability.py:142-183).

    flags u8[S]: bit0 participates, bit1 correct (at most one outcome per source per call).
    """
    L = N.require_gpu()
    N.check(L.bce_outcome_update(rel.numel(), N.ptr(rel), N.ptr(conf), N.ptr(t_us), N.ptr(present),
                                 N.ptr(flags), int(now_us), float(default_rel), float(default_conf),
                                 N.stream(rel.device)), "bce_outcome_update")


def replay_step(rel, conf, t_us, present, flags2, now_us: int, view: torch.Tensor,
                half_life_days: float = DECAY_HALF_LIFE_DAYS, min_rel: float = DECAY_MINIMUM) -> None:
    """Config-4 step: decayed view at ``now_us`` then the outcome update, fused.

    flags2: 2 bits per source (bit0 participates, bit1 correct), 4 sources per byte.
    Absent rows must hold the baked cold-start values (rel 0.5, conf 0.25, t = NO_TIMESTAMP).
    """
    L = N.require_gpu()
    N.check(L.bce_replay_step(rel.numel(), N.ptr(rel), N.ptr(conf), N.ptr(t_us), N.ptr(present),
                              N.ptr(flags2), int(now_us), float(half_life_days), float(min_rel),
                              DEFAULT_RELIABILITY, DEFAULT_CONFIDENCE, N.ptr(view), N.stream(rel.device)),
            "bce_replay_step")


def pack_flags2(participate: np.ndarray, correct: np.ndarray) -> np.ndarray:
    """Host helper: (participate, correct) bool arrays -> the 2-bit packed flags2 layout."""
    S = len(participate)
    f = participate.astype(np.uint8) | (correct.astype(np.uint8) << 1)
    pad = (-S) % 4
    f = np.concatenate([f, np.zeros(pad, np.uint8)]).reshape(-1, 4)
    return (f[:, 0] | (f[:, 1] << 2) | (f[:, 2] << 4) | (f[:, 3] << 6)).astype(np.uint8)


# ---------------------------------------------------------------------------------------
# tie-break, agreement statistics, re-estimation
# ---------------------------------------------------------------------------------------
@dataclass
class TieBreakResult:
    winner: torch.Tensor
    label: torch.Tensor
    n_groups: torch.Tensor
    variance: torch.Tensor
    g_key: torch.Tensor
    g_count: torch.Tensor
    g_density: torch.Tensor
    g_avgconf: torch.Tensor
    g_maxrel: torch.Tensor
    g_of: torch.Tensor      # int32[N]: each signal's group ordinal (first-seen order)


@dataclass
class TiePlan:
    """Markets of <= 32 agents bucketed by length for the lane-per-market tie-break: lists of the
    markets with <= 8, 9..16 and 17..32 agents, each run by a kernel walking 8 / 16 / 32
    positions per lane over rows gathered into LDS (tiebreak.hip GATHER) -- or None when
    bucketing would not pay (a uniform batch: contiguous tiles, the FULL-tile kernel)."""

    buckets: Optional[list]  # [(device int32 list, max_len)], or None: contiguous tiles


# relative cost of a 64-market tile, measured (kernel traces, 1M markets, profiles/r06gb/):
# contiguous FULL (every market 32 agents: 42 ns per tile) / contiguous ragged (the general
# 32-position body: 45.4 ns) / gathered buckets of 8 / 16 / 32 positions (20.7 / 34.9 / 58.3 ns,
# since round 6's batched row loads: 20 / 40 / 70 before, profiles/archive/r05f/).  The lane
# kernels are latency-bound by their stage -> compute -> flush phases, so fewer positions per
# lane save less than the arithmetic suggests; a uniform 1..32 ragged batch is now bucketed
# (0.674-0.680 vs 0.721 ms contiguous), a uniform 32 batch stays contiguous.
_TILE_COST = {"full": 0.92, "ragged": 1.0, 8: 0.46, 16: 0.77, 32: 1.28}
_BUCKET_GAIN = 0.97  # bucket when the model saves >= 3% (one launch more per call)


def tiebreak_plan(offsets_host: np.ndarray, device=None, force: bool = False) -> TiePlan:
    """Length buckets for batch.tiebreak (markets of <= 32 agents), when they cost less than
    the contiguous tiles by the kernels' relative tile costs (_TILE_COST), or always (force)."""
    lens = np.diff(np.asarray(offsets_host, np.int64))
    if len(lens) == 0 or int(lens.max()) > 32 or int(lens.min()) < 0:
        # a negative length (decreasing offsets) falls in no bucket: the contiguous kernel
        # records it as a device fault (kFaultTooLong) instead of leaving outputs unwritten
        return TiePlan(None)
    M = len(lens)
    pad = (-M) % 64
    t = np.concatenate([lens, np.full(pad, 32)]).reshape(-1, 64)
    full = (t == 32).all(axis=1)
    contig = _TILE_COST["full"] * int(full.sum()) + _TILE_COST["ragged"] * int((~full).sum())
    edges = ((0, 8), (9, 16), (17, 32))
    idx = [np.nonzero((lens >= lo) & (lens <= hi))[0].astype(np.int32) for lo, hi in edges]
    bucket = sum(_TILE_COST[hi] * ((len(i) + 63) // 64) for (lo, hi), i in zip(edges, idx))
    if bucket >= _BUCKET_GAIN * contig and not force:
        return TiePlan(None)
    dev = device or N.device()
    return TiePlan([(torch.from_numpy(i).to(dev), hi) for (lo, hi), i in zip(edges, idx) if len(i)])


def tiebreak(offsets: torch.Tensor, pred: torch.Tensor, conf: torch.Tensor, weight: torch.Tensor,
             rel: torch.Tensor, *, precision: int = 6, offsets_host: Optional[np.ndarray] = None,
             out: Optional[TieBreakResult] = None, max_len: Optional[int] = None,
             plan: Optional[TiePlan] = None) -> TieBreakResult:
    """DeterministicTieBreaker(precision).resolve for every CSR market (tiebreak.py:73-152).

    Any market length (> 4096 agents sort in a global scratch slice).  ``precision`` as
    CPython round() for every int, bit for bit (exact big integers where 10^|precision| is
    not a double); a rounded key too large for a double raises OverflowError, as CPython's
    round() does (precision <= -16 only, checked with one stream synchronisation).

    ``max_len`` (optional, <= 64): the caller's bound on every market's length; the host then
    skips its length scan of the offsets and does not synchronise.  A market longer than the
    bound is left unprocessed and recorded in the device fault word, as the C ABI does --
    ``_native.check_faults`` raises it (the bench and tests call it after their steps).

    ``plan`` (optional, :func:`tiebreak_plan`): length buckets of a ragged batch of <= 32-agent
    markets, reused across calls on the same CSR (no host scan per call).  Without one, a
    ragged batch scanned on the host is bucketed the same way when that pays -- an O(M) host
    pass and up to three host-to-device list copies on EVERY call: a caller that reruns the
    same CSR should build the TiePlan once with :func:`tiebreak_plan` and pass it in."""
    L = N.require_gpu()
    M = offsets.numel() - 1
    Nsig = pred.numel()
    dev = offsets.device
    f64 = dict(dtype=torch.float64, device=dev)
    i32 = dict(dtype=torch.int32, device=dev)
    r = out or TieBreakResult(torch.empty(M, **f64), torch.empty(M, **i32), torch.empty(M, **i32),
                              torch.empty(M, **f64), torch.empty(max(Nsig, 1), **f64),
                              torch.empty(max(Nsig, 1), **i32), torch.empty(max(Nsig, 1), **f64),
                              torch.empty(max(Nsig, 1), **f64), torch.empty(max(Nsig, 1), **f64),
                              torch.empty(max(Nsig, 1), **i32))
    outs = (N.ptr(r.winner), N.ptr(r.label), N.ptr(r.n_groups), N.ptr(r.variance), N.ptr(r.g_key),
            N.ptr(r.g_count), N.ptr(r.g_density), N.ptr(r.g_avgconf), N.ptr(r.g_maxrel), N.ptr(r.g_of))
    ins = (N.ptr(pred), N.ptr(conf), N.ptr(weight), N.ptr(rel))
    st = N.stream(dev)

    def run_buckets(buckets):
        for lst, hi in buckets:
            N.check(L.bce_tiebreak_csr(N.ptr(offsets), M, N.ptr(lst), lst.numel(), *ins, int(hi), int(precision),
                                       *outs, st), "bce_tiebreak_csr")
        return _round_overflow_check(r, precision, dev)

    if plan is not None and plan.buckets is not None:
        return run_buckets(plan.buckets)
    if max_len is not None and 0 < int(max_len) <= 64:
        N.check(L.bce_tiebreak_csr(N.ptr(offsets), M, N.ptr(None), 0, *ins, int(max_len), int(precision), *outs, st),
                "bce_tiebreak_csr")
        return _round_overflow_check(r, precision, dev)
    offh = offsets_host if offsets_host is not None else offsets.cpu().numpy()
    lens = np.diff(offh)
    if len(lens) and int(lens.max()) <= 32:
        tp = tiebreak_plan(offh, dev)
        if tp.buckets is not None:
            return run_buckets(tp.buckets)
    long_ = np.nonzero(lens > 64)[0]
    if len(long_) == 0:
        N.check(L.bce_tiebreak_csr(N.ptr(offsets), M, N.ptr(None), 0, *ins, int(max(int(lens.max(initial=1)), 1)),
                                   int(precision), *outs, st), "bce_tiebreak_csr")
        return _round_overflow_check(r, precision, dev)
    # n <= 32: the lane-per-market kernel; 33..64: wave per market; longer: workgroup per market
    for lo, hi in ((0, 32), (33, 64)):
        short = np.nonzero((lens >= lo) & (lens <= hi))[0].astype(np.int32)
        if len(short):
            sl = torch.from_numpy(short).to(dev)
            N.check(L.bce_tiebreak_csr(N.ptr(offsets), M, N.ptr(sl), len(short), *ins, hi, int(precision), *outs,
                                       st), "bce_tiebreak_csr")
    ll = torch.from_numpy(long_.astype(np.int32)).to(dev)
    N.check(L.bce_tiebreak_csr_long(N.ptr(offsets), M, N.ptr(ll), len(long_), int(precision), *ins,
                                    int(lens[long_].max()), *outs, st), "bce_tiebreak_csr_long")
    return _round_overflow_check(r, precision, dev)


def _round_overflow_check(r, precision: int, dev):
    """round(x, n) with -308 <= n <= -16 can exceed DBL_MAX (CPython: OverflowError,
    "rounded value too large to represent"); the kernels record that as device fault 6."""
    if -308 <= int(precision) <= -16:
        try:
            N.check_faults(dev, "tiebreak round()")
        except N.BCEError as exc:
            if "too large to represent" in str(exc):
                raise OverflowError("rounded value too large to represent") from None
            raise
    return r


def agreement_stats(offsets, sid, prob, outcome, n_sources: int, correct=None, total=None):
    """summarize_sources counts (market.py:279-304): outcome int8[M] (-1 skip, 0, 1)."""
    L = N.require_gpu()
    dev = offsets.device
    if correct is None:
        correct = torch.zeros(max(n_sources, 1), dtype=torch.int32, device=dev)
    if total is None:
        total = torch.zeros(max(n_sources, 1), dtype=torch.int32, device=dev)
    N.check(L.bce_agreement_stats(N.ptr(offsets), offsets.numel() - 1, N.ptr(sid), N.ptr(prob),
                                  N.ptr(outcome), N.ptr(correct), N.ptr(total), N.stream(dev)),
            "bce_agreement_stats")
    return correct, total


# ---------------------------------------------------------------------------------------
# namespaced fallback (reliability_abstraction.py:119-188) and cross-market aggregation
# ---------------------------------------------------------------------------------------
@dataclass
class ScopeTable:
    """One namespace scope of the store (rows of one market_id key) over a rank space:
    rel, conf fp64[S], t_us int64[S] (NO_TIMESTAMP = unparseable), has u8[S] = a row with a
    truthy updated_at exists (the ``if record.updated_at`` test)."""

    rel: torch.Tensor
    conf: torch.Tensor
    t_us: torch.Tensor
    has: torch.Tensor


NS_MARKET, NS_DOMAIN, NS_GLOBAL, NS_COLD = 0, 1, 2, 3


def namespace_resolve(scopes: Sequence[Optional[ScopeTable]], now_us: int, apply_decay: bool = True,
                      mark_cold: bool = False, names: Optional[Sequence[str]] = None,
                      half_life_days: float = DECAY_HALF_LIFE_DAYS, min_rel: float = DECAY_MINIMUM):
    """Fallback chain market -> domain -> global -> cold start for every source in one launch
    (bce_namespace_resolve).  ``scopes`` = [market, domain, global], None = not requested.
    Returns (SourceTable ready for :func:`consensus`, scope u8[S] with NS_* codes)."""
    L = N.require_gpu()
    sc = list(scopes) + [None] * (3 - len(scopes))
    live = [x for x in sc if x is not None]
    if live:
        S = live[0].rel.numel()
        dev = live[0].rel.device
    else:
        S = len(names) if names is not None else 0
        dev = N.device()
    relconf = torch.empty((max(S, 1), 2), dtype=torch.float64, device=dev)
    bits = torch.zeros(max((S + 31) // 32, 1), dtype=torch.int32, device=dev)
    scope = torch.empty(max(S, 1), dtype=torch.uint8, device=dev)
    args, keep = [], []
    for x in sc:
        if x is None:
            args += [None] * 4
        else:
            assert x.rel.numel() == S and x.conf.numel() == S and x.has.numel() == S, "scope sizes differ"
            arrs = (x.rel.to(torch.float64).contiguous(), x.conf.to(torch.float64).contiguous(),
                    x.t_us.to(torch.int64).contiguous(), x.has.to(torch.uint8).contiguous())
            keep.append(arrs)  # alive until the launch is enqueued
            args += [N.ptr(a) for a in arrs]
    N.check(L.bce_namespace_resolve(S, *args, int(bool(apply_decay)), int(now_us), float(half_life_days),
                                    float(min_rel), DEFAULT_RELIABILITY, DEFAULT_CONFIDENCE, int(bool(mark_cold)),
                                    N.ptr(relconf), N.ptr(bits), N.ptr(scope), N.stream(dev)),
            "bce_namespace_resolve")
    table = SourceTable(relconf, bits, list(names) if names is not None else [""] * S)
    return table, scope[:S]


@dataclass
class AggregateResult:
    """Per group: weighted_average, median, majority, mean confidence (NaN where no member
    has a consensus) and the number of members with a consensus."""

    wavg: torch.Tensor
    median: torch.Tensor
    majority: torch.Tensor
    mean_conf: torch.Tensor
    n_included: torch.Tensor


def aggregate(group_offsets: torch.Tensor, members: torch.Tensor, consensus: torch.Tensor,
              confidence: torch.Tensor, has_consensus: torch.Tensor, median: bool = True) -> AggregateResult:
    """CrossMarketAggregator.aggregate_consensus (market.py:340-408) for many member groups
    in one launch (bce_aggregate_groups); sums in list order, bit-exact."""
    L = N.require_gpu()
    dev = consensus.device
    G = group_offsets.numel() - 1
    f64 = dict(dtype=torch.float64, device=dev)
    r = AggregateResult(torch.empty(max(G, 1), **f64), torch.empty(max(G, 1), **f64),
                        torch.empty(max(G, 1), **f64), torch.empty(max(G, 1), **f64),
                        torch.empty(max(G, 1), dtype=torch.int64, device=dev))
    N.check(L.bce_aggregate_groups(N.ptr(group_offsets), G, N.ptr(members), consensus.numel(), N.ptr(consensus),
                                   N.ptr(confidence), N.ptr(has_consensus), N.ptr(r.wavg),
                                   N.ptr(r.median) if median else None, N.ptr(r.majority), N.ptr(r.mean_conf),
                                   N.ptr(r.n_included), N.stream(dev)), "bce_aggregate_groups")
    return AggregateResult(*(t[:G] for t in (r.wavg, r.median, r.majority, r.mean_conf, r.n_included)))


def reestimate(P: torch.Tensor, iters: int, w0: float = 0.5, w: Optional[torch.Tensor] = None,
               keep_history: bool = False, mode: str = "exact"):
    """Config 5: ``iters`` rounds of consensus <-> reliability on agent-major P [A, M].

    Each round reads P once: the consensus pass records every cell's vote as one bit and the
    agreement pass counts from those bits (bce_reestimate_consensus_votes /
    bce_reestimate_agreement_votes; A*ceil(M/64)*8 bytes of scratch).  ``mode="exact"`` sums
    in agent order on the vector ALUs (bit-identical to the reference); ``mode="fast"`` runs the
    same kernel -- it streams P at the HBM rate and is the fastest form.  ``mode="mfma"`` runs
    the consensus pass on the matrix cores (bce_reestimate_consensus_votes_mfma,
    v_mfma_f64_4x4x4_4b_f64: consensus within 4*A*2^-53, votes, agreement counts and weights
    identical to exact) -- the config-5 MFMA contraction, 1.3-1.8% behind the vector pass
    (DESIGN.md §4.6).  Its summation order needs every weight finite and >= 0; the library
    checks that on the device and runs the exact kernel for an iteration whose weights break
    it."""
    L = N.require_gpu()
    A, M = P.shape
    dev = P.device
    ld = P.stride(0)
    assert P.stride(1) == 1
    w = torch.full((A,), w0, dtype=torch.float64, device=dev) if w is None else w
    cons = torch.empty(M, dtype=torch.float64, device=dev)
    nul = torch.empty(max(M, 1), dtype=torch.uint8, device=dev)
    agree = torch.zeros(A, dtype=torch.int64, device=dev)
    resolved = torch.zeros(1, dtype=torch.int64, device=dev)
    K = max((M + 63) // 64, 1)
    votes = torch.empty((K, A), dtype=torch.int64, device=dev)
    words = torch.empty((2, K), dtype=torch.int64, device=dev)  # cvote, ok
    hist = []
    st = N.stream(dev)
    if mode not in _MODES and mode != "mfma":
        raise ValueError(f"mode must be one of {sorted([*_MODES, 'mfma'])}")
    scratch = None
    if mode == "mfma":
        nb = int(L.bce_reestimate_mfma_scratch_bytes(M))
        scratch = torch.empty((nb + 7) // 8, dtype=torch.int64, device=dev)
    for _ in range(iters):
        if scratch is None:
            N.check(L.bce_reestimate_consensus_votes(N.ptr(P, row_strided=True), A, M, ld, N.ptr(w), N.ptr(cons),
                                                     N.ptr(nul), N.ptr(votes), N.ptr(words[0]), N.ptr(words[1]),
                                                     st), "bce_reestimate_consensus_votes")
        else:
            N.check(L.bce_reestimate_consensus_votes_mfma(N.ptr(P, row_strided=True), A, M, ld, N.ptr(w),
                                                          N.ptr(cons), N.ptr(nul), N.ptr(votes), N.ptr(words[0]),
                                                          N.ptr(words[1]), N.ptr(scratch), scratch.numel() * 8, st),
                    "bce_reestimate_consensus_votes_mfma")
        agree.zero_()
        resolved.zero_()
        N.check(L.bce_reestimate_agreement_votes(N.ptr(votes), A, M, N.ptr(words[0]), N.ptr(words[1]),
                                                 N.ptr(agree), N.ptr(resolved), st), "bce_reestimate_agreement_votes")
        N.check(L.bce_reestimate_weights(A, N.ptr(agree), N.ptr(resolved), N.ptr(w), st),
                "bce_reestimate_weights")
        if keep_history:
            hist.append((cons.clone(), nul[:M].clone(), agree.clone(), w.clone()))
    return w, cons, nul[:M], agree, hist
