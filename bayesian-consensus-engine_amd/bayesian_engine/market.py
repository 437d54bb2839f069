"""Drop-in for ``bayesian_engine.market`` (reference src/bayesian_engine/market.py).

The multi-market layer is where the batched engine pays off:

* ``MarketStore.compute_all_consensus`` (market.py:200-221) -- instead of a Python loop of
  per-market ``compute_consensus`` calls, ALL open markets become one CSR batch and one
  consensus launch.  With a reliability store, every (source, market) pair the batch
  needs is fetched in bulk and decayed on the GPU in one launch (the reference's
  per-signal ``get_reliability(..., apply_decay=True)``, market.py:208-219).  Ranks are
  interned over (market position, sourceId) so each market's rank order is Python
  ``sorted()`` order of its sourceIds -- results are identical to the reference's.
* ``CrossMarketAggregator.summarize_sources`` (market.py:256-321) -- the per-source
  correct/total counts run in the ``bce_agreement_stats`` kernel (exact int atomics).

* ``CrossMarketAggregator.aggregate_consensus`` (market.py:340-408) --
  weighted_average / median / majority over member groups in the ``bce_aggregate_groups``
  kernel (list-order sums, exact radix-select median); ``aggregate_many`` does many
  pattern lists in one launch.

Metadata (MarketId glob matching, status, category summaries) is host Python with the
reference's semantics.
"""
from __future__ import annotations

import fnmatch
from dataclasses import dataclass, field
from datetime import datetime, timezone
from enum import Enum
from typing import Any, Dict, List, Optional

import numpy as np
import torch

from . import _native as N
from . import batch
from .config import DEFAULT_CONFIDENCE, DEFAULT_RELIABILITY, SCHEMA_VERSION
from .core import compute_consensus
from .reliability import SQLiteReliabilityStore
from . import decay as _decay
from .timeutil import NO_TIMESTAMP, dt_to_us, iso_to_us

__all__ = ["MarketId", "MarketStatus", "Market", "MarketStore", "SourcePerformance", "CrossMarketAggregator"]


@dataclass(frozen=True)
class MarketId:
    """Unique identifier for a market or question (market.py:41-82)."""

    value: str

    def __post_init__(self):
        if not self.value or not self.value.strip():
            raise ValueError("Market ID cannot be empty")

    def __str__(self) -> str:
        return self.value

    def __repr__(self) -> str:
        return f"MarketId({self.value!r})"

    @property
    def category(self) -> Optional[str]:
        if ":" in self.value:
            return self.value.split(":")[0]
        return None

    @property
    def parts(self) -> List[str]:
        return self.value.split(":")

    def matches(self, pattern: str) -> bool:
        return fnmatch.fnmatch(self.value, pattern)


class MarketStatus(str, Enum):
    OPEN = "open"
    CLOSED = "closed"
    RESOLVED = "resolved"


@dataclass
class Market:
    """A market with metadata and signals (market.py:93-134)."""

    id: MarketId
    status: MarketStatus = MarketStatus.OPEN
    signals: List[Dict[str, Any]] = field(default_factory=list)
    consensus_result: Optional[Dict[str, Any]] = None
    outcome: Optional[bool] = None
    created_at: str = field(default_factory=lambda: datetime.now(timezone.utc).isoformat())
    resolved_at: Optional[str] = None
    metadata: Dict[str, Any] = field(default_factory=dict)

    def add_signal(self, signal: Dict[str, Any]) -> None:
        if self.status != MarketStatus.OPEN:
            raise ValueError(f"Cannot add signal to {self.status} market")
        self.signals.append(signal)

    def compute_consensus(self, source_reliability: Optional[Dict[str, Dict[str, float]]] = None) -> Dict[str, Any]:
        if not self.signals:
            return _empty_market_result(self)
        result = compute_consensus(self.signals, source_reliability)
        result["marketId"] = str(self.id)
        self.consensus_result = result
        return result

    def resolve(self, outcome: bool) -> None:
        self.outcome = outcome
        self.status = MarketStatus.RESOLVED
        self.resolved_at = datetime.now(timezone.utc).isoformat()


def _empty_market_result(market: Market) -> Dict[str, Any]:
    return {"schemaVersion": "1.0.0", "consensus": None, "confidence": 0.0, "marketId": str(market.id)}


class MarketStore:
    """In-memory store for markets (market.py:137-221)."""

    def __init__(self):
        self._markets: Dict[str, Market] = {}

    def create_market(self, market_id: MarketId, metadata: Optional[Dict[str, Any]] = None) -> Market:
        key = str(market_id)
        if key in self._markets:
            raise ValueError(f"Market {market_id} already exists")
        market = Market(id=market_id, metadata=metadata or {})
        self._markets[key] = market
        return market

    def get_market(self, market_id: MarketId) -> Optional[Market]:
        return self._markets.get(str(market_id))

    def get_or_create(self, market_id: MarketId) -> Market:
        market = self.get_market(market_id)
        if market is None:
            market = self.create_market(market_id)
        return market

    def add_signal(self, market_id: MarketId, signal: Dict[str, Any]) -> Market:
        market = self.get_or_create(market_id)
        market.add_signal(signal)
        return market

    def list_markets(self, status: Optional[MarketStatus] = None, pattern: Optional[str] = None) -> List[Market]:
        markets = list(self._markets.values())
        if status is not None:
            markets = [m for m in markets if m.status == status]
        if pattern is not None:
            markets = [m for m in markets if m.id.matches(pattern)]
        return markets

    def compute_all_consensus(self, reliability_store: Optional[SQLiteReliabilityStore] = None
                              ) -> Dict[str, Dict[str, Any]]:
        """Consensus for all open markets in ONE batched launch (market.py:200-221)."""
        markets = self.list_markets(status=MarketStatus.OPEN)
        busy = [m for m in markets if m.signals]
        computed: Dict[str, Dict[str, Any]] = {}
        if busy:
            computed = _batched_consensus(busy, reliability_store)
        results: Dict[str, Dict[str, Any]] = {}
        for market in markets:
            key = str(market.id)
            if not market.signals:
                results[key] = _empty_market_result(market)
            else:
                res = computed[key]
                market.consensus_result = res
                results[key] = res
        return results


def _batched_consensus(markets: List[Market], store: Optional[SQLiteReliabilityStore]) -> Dict[str, Dict[str, Any]]:
    """CSR over the markets, ranks over (market position, sorted sourceId)."""
    per_market_ids = []
    key_names: List[str] = []
    offsets = [0]
    sid_list: List[int] = []
    prob_list: List[float] = []
    base = 0
    for mpos, market in enumerate(markets):
        ids = sorted({s["sourceId"] for s in market.signals})
        rank = {sid: base + i for i, sid in enumerate(ids)}
        per_market_ids.append((base, ids))
        key_names.extend(ids)
        for s in market.signals:
            sid_list.append(rank[s["sourceId"]])
            p = s["probability"]
            if not isinstance(p, (int, float)):
                0 + p  # noqa: B018  -- builtin sum()'s TypeError (core.py:116)
            prob_list.append(float(p))
        offsets.append(len(sid_list))
        base += len(ids)
    S = base
    dev = N.device()
    N.require_gpu()
    rel = np.full(max(S, 2), DEFAULT_RELIABILITY)
    conf = np.full(max(S, 2), DEFAULT_CONFIDENCE)
    present = np.zeros(max(S, 2), np.uint8)
    if store is not None:
        # every sourceId gets a dict entry (market.py:209-219): none is cold-start
        present[:S] = 1
        pairs = [(sid, str(m.id)) for m, (_, ids) in zip(markets, per_market_ids) for sid in ids]
        rows = store.fetch_pairs(pairs)
        t_us = np.full(max(S, 2), NO_TIMESTAMP, np.int64)
        k = 0
        for m, (_, ids) in zip(markets, per_market_ids):
            for sid in ids:
                row = rows.get((sid, str(m.id)))
                if row is not None:
                    rel[k], conf[k], t_us[k] = row[0], row[1], iso_to_us(row[2])
                k += 1
        T = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
        rt = batch.ReliabilityTable(T(rel[:S]), T(conf[:S]), T(t_us[:S]), T(present[:S]), key_names)
        # get_reliability(apply_decay=True) for every pair, "now" read like decay.py:136-137
        table = rt.consensus_table(dt_to_us(_decay.datetime.now(timezone.utc)))
    else:
        T = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
        table = batch.SourceTable.from_arrays(T(rel[:S]), T(conf[:S]), T(present[:S]), key_names)
    off = np.array(offsets, np.int64)
    T = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
    res = batch.consensus(T(off), T(np.array(sid_list, np.int32)), T(np.array(prob_list, np.float64)), table,
                          validate=False, check=True)
    cons = res.consensus.cpu().numpy()
    confd = res.confidence.cpu().numpy()
    tot = res.total_weight.cpu().numpy()
    usid = res.usid.cpu().numpy()
    weight = res.weight.cpu().numpy()
    nweight = res.nweight.cpu().numpy()
    out = {}
    for mpos, market in enumerate(markets):
        b, ids = per_market_ids[mpos]
        a = offsets[mpos]
        u = len(ids)
        null = tot[mpos] == 0
        sw = [{"sourceId": ids[j], "weight": float(weight[a + j]), "normalizedWeight": float(nweight[a + j])}
              for j in range(u)]
        out[str(market.id)] = {
            "schemaVersion": SCHEMA_VERSION,
            "consensus": None if null else float(cons[mpos]),
            "confidence": 0.0 if null else float(confd[mpos]),
            "sourceWeights": sw,
            "normalization": {"totalWeight": float(tot[mpos]), "sourceCount": u},
            "diagnostics": {
                "status": "computed",
                "sources": len(market.signals),
                "uniqueSources": u,
                "coldStartSources": [ids[j] for j in range(u) if usid[a + j] < 0],
            },
            "marketId": str(market.id),
        }
    return out


@dataclass
class SourcePerformance:
    """Aggregated performance of a source across markets (market.py:224-241)."""

    source_id: str
    total_markets: int
    correct_predictions: int
    wrong_predictions: int
    reliability: float
    markets: List[str] = field(default_factory=list)

    @property
    def accuracy(self) -> float:
        total = self.correct_predictions + self.wrong_predictions
        if total == 0:
            return 0.0
        return self.correct_predictions / total


class CrossMarketAggregator:
    """Aggregate data across multiple markets (market.py:244-408)."""

    def __init__(self, market_store: MarketStore):
        self._store = market_store

    def summarize_sources(self, patterns: Optional[List[str]] = None) -> Dict[str, SourcePerformance]:
        markets = self._store.list_markets(status=MarketStatus.RESOLVED)
        if patterns:
            markets = [m for m in markets if any(m.id.matches(p) for p in patterns)]
        markets = [m for m in markets if m.outcome is not None]
        order: Dict[str, int] = {}
        names: List[str] = []
        market_lists: List[List[str]] = []
        offsets = [0]
        sid_list: List[int] = []
        prob_list: List[float] = []
        outcome: List[int] = []
        for market in markets:
            for signal in market.signals:
                sid = signal["sourceId"]
                if sid not in order:
                    order[sid] = len(names)
                    names.append(sid)
                    market_lists.append([])
                market_lists[order[sid]].append(str(market.id))
                prob = signal.get("probability", 0.5)
                if not isinstance(prob, (int, float)):
                    prob >= 0.5  # noqa: B015  -- the reference's TypeError (market.py:299)
                sid_list.append(order[sid])
                prob_list.append(float(prob))
            offsets.append(len(sid_list))
            outcome.append(1 if market.outcome else 0)
        results: Dict[str, SourcePerformance] = {}
        if not names:
            return results
        N.require_gpu()
        dev = N.device()
        T = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
        correct, total = batch.agreement_stats(T(np.array(offsets, np.int64)), T(np.array(sid_list, np.int32)),
                                               T(np.array(prob_list, np.float64)), T(np.array(outcome, np.int8)),
                                               len(names))
        correct = correct.cpu().numpy()
        total = total.cpu().numpy()
        for i, sid in enumerate(names):
            c, t = int(correct[i]), int(total[i])
            w = t - c
            results[sid] = SourcePerformance(sid, t, c, w, c / (c + w) if (c + w) > 0 else 0.5, market_lists[i])
        return results

    def summarize_category(self, category: str) -> Dict[str, Any]:
        markets = self._store.list_markets(pattern=f"{category}:*")
        resolved = [m for m in markets if m.status == MarketStatus.RESOLVED]
        open_markets = [m for m in markets if m.status == MarketStatus.OPEN]
        return {"category": category, "total_markets": len(markets), "resolved": len(resolved),
                "open": len(open_markets), "markets": [str(m.id) for m in markets]}

    def aggregate_consensus(self, patterns: List[str], method: str = "weighted_average") -> Dict[str, Any]:
        """Cross-market aggregation (market.py:338-408), computed by bce_aggregate_groups."""
        return self.aggregate_many([patterns], method)[0]

    def aggregate_many(self, pattern_lists: List[List[str]], method: str = "weighted_average") -> List[Dict[str, Any]]:
        """aggregate_consensus for many pattern lists in ONE kernel launch: each list is a
        member group (markets in list_markets order per pattern, duplicates kept,
        market.py:355-357); the sums run in that order on the GPU (bit-exact)."""
        groups: List[List[int]] = []
        index: Dict[str, int] = {}
        cons: List[float] = []
        conf: List[float] = []
        has: List[int] = []
        for patterns in pattern_lists:
            members: List[int] = []
            for pattern in patterns:
                for market in self._store.list_markets(pattern=pattern):
                    key = str(market.id)
                    if key not in index:
                        index[key] = len(cons)
                        res = market.consensus_result
                        ok = bool(res) and res.get("consensus") is not None  # market.py:369-370
                        cons.append(float(res["consensus"]) if ok else 0.0)
                        conf.append(float(res.get("confidence", 0.5)) if ok else 0.0)
                        has.append(1 if ok else 0)
                    members.append(index[key])
            groups.append(members)
        empty = {"schemaVersion": "1.0.0", "consensus": None, "confidence": 0.0}
        if not any(has[m] for g in groups for m in g):
            return [dict(empty, marketsIncluded=len(g)) for g in groups]
        if method not in ("weighted_average", "median", "majority"):
            for g in groups:  # the reference raises only once a group has consensuses
                if any(has[m] for m in g):
                    raise ValueError(f"Unknown aggregation method: {method}")
        N.require_gpu()
        dev = N.device()
        T = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
        goff = np.zeros(len(groups) + 1, np.int64)
        goff[1:] = np.cumsum([len(g) for g in groups])
        flat = np.array([m for g in groups for m in g], np.int64)
        r = batch.aggregate(T(goff), T(flat if flat.size else np.zeros(1, np.int64)), T(np.array(cons, np.float64)),
                            T(np.array(conf, np.float64)), T(np.array(has, np.uint8)), median=method == "median")
        pick = {"weighted_average": r.wavg, "median": r.median, "majority": r.majority}[method].cpu().numpy()
        mconf = r.mean_conf.cpu().numpy()
        k = r.n_included.cpu().numpy()
        out = []
        for gi, g in enumerate(groups):
            if not g:
                out.append(dict(empty, marketsIncluded=0))
            elif k[gi] == 0:
                out.append(dict(empty, marketsIncluded=len(g)))
            else:
                out.append({"schemaVersion": "1.0.0", "consensus": float(pick[gi]), "confidence": float(mconf[gi]),
                            "marketsIncluded": int(k[gi]), "method": method})
        return out
