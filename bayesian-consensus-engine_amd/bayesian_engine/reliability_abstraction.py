"""Drop-in for ``bayesian_engine.reliability_abstraction`` (reference
src/bayesian_engine/reliability_abstraction.py): namespace-aware reliability with the
fallback chain market -> domain -> global -> cold start.

The per-source API (``get_reliability``, ``update_reliability``, ``set_global_reliability``)
keeps the reference's names, arguments, records and fallback order, on top of this
package's :class:`SQLiteReliabilityStore` (whose decay runs on the GPU).  The batched
path, :meth:`NamespacedReliabilityStore.resolve`, loads the three scopes of a whole rank
space from SQLite once and resolves every source in ONE launch of
``bce_namespace_resolve`` (decay + precedence + consensus-table packing fused), so the
table a consensus batch gathers from is built without a per-source Python loop.
"""
from __future__ import annotations

import sqlite3
from dataclasses import dataclass
from datetime import datetime, timezone
from enum import Enum
from typing import List, Optional, Protocol, Sequence, Tuple, runtime_checkable

import numpy as np
import torch

from . import _native as N
from . import batch
from .config import DEFAULT_CONFIDENCE, DEFAULT_RELIABILITY
from .reliability import SQLiteReliabilityStore
from .timeutil import NO_TIMESTAMP, dt_to_us, iso_to_us

__all__ = ["ReliabilityNamespace", "NamespacedReliabilityRecord", "ReliabilityProvider",
           "NamespacedReliabilityStore"]


class ReliabilityNamespace(str, Enum):
    """Namespace levels for reliability tracking (reliability_abstraction.py:33-38)."""

    GLOBAL = "global"
    DOMAIN = "domain"
    MARKET = "market"


@dataclass(frozen=True)
class NamespacedReliabilityRecord:
    """Reliability record with namespace context (reliability_abstraction.py:41-51)."""

    source_id: str
    namespace: ReliabilityNamespace
    namespace_value: str
    reliability: float
    confidence: float
    updated_at: str
    is_fallback: bool


@runtime_checkable
class ReliabilityProvider(Protocol):
    """Protocol for reliability data providers (reliability_abstraction.py:54-81)."""

    def get_reliability(self, source_id: str, namespace: ReliabilityNamespace,
                        namespace_value: str) -> Optional[NamespacedReliabilityRecord]:
        ...

    def update_reliability(self, source_id: str, namespace: ReliabilityNamespace, namespace_value: str,
                           outcome_correct: bool) -> NamespacedReliabilityRecord:
        ...


# scope code (bce_namespace_resolve) -> (namespace, is_fallback)
_SCOPE_NS = {batch.NS_MARKET: (ReliabilityNamespace.MARKET, False),
             batch.NS_DOMAIN: (ReliabilityNamespace.DOMAIN, True),
             batch.NS_GLOBAL: (ReliabilityNamespace.GLOBAL, True)}


class NamespacedReliabilityStore:
    """Reliability store with namespace-aware fallback chain (reliability_abstraction.py:84-291).

    Fallback order: market-specific, domain-specific, global, cold-start defaults.
    """

    GLOBAL_MARKET_ID = "__global__"

    def __init__(self, db_path: str = ":memory:"):
        self._store = SQLiteReliabilityStore(db_path)

    # ------------------------------------------------------------------ reference API
    def get_reliability(self, source_id: str, market_id: Optional[str] = None, domain: Optional[str] = None,
                        apply_decay: bool = True) -> NamespacedReliabilityRecord:
        """reliability_abstraction.py:119-188."""
        if market_id:
            record = self._store.get_reliability(source_id, market_id, apply_decay)
            if record.updated_at:
                return NamespacedReliabilityRecord(source_id, ReliabilityNamespace.MARKET, market_id,
                                                   record.reliability, record.confidence, record.updated_at, False)
        if domain:
            record = self._store.get_reliability(source_id, f"__domain__:{domain}", apply_decay)
            if record.updated_at:
                return NamespacedReliabilityRecord(source_id, ReliabilityNamespace.DOMAIN, domain,
                                                   record.reliability, record.confidence, record.updated_at, True)
        record = self._store.get_reliability(source_id, self.GLOBAL_MARKET_ID, apply_decay)
        if record.updated_at:
            return NamespacedReliabilityRecord(source_id, ReliabilityNamespace.GLOBAL, "global",
                                               record.reliability, record.confidence, record.updated_at, True)
        return NamespacedReliabilityRecord(source_id, ReliabilityNamespace.GLOBAL, "cold-start",
                                           DEFAULT_RELIABILITY, DEFAULT_CONFIDENCE, "", True)

    def update_reliability(self, source_id: str, outcome_correct: bool, market_id: Optional[str] = None,
                           domain: Optional[str] = None, update_global: bool = False) -> NamespacedReliabilityRecord:
        """reliability_abstraction.py:190-240."""
        if market_id:
            namespace, namespace_value, target = ReliabilityNamespace.MARKET, market_id, market_id
        elif domain:
            namespace, namespace_value, target = ReliabilityNamespace.DOMAIN, domain, f"__domain__:{domain}"
        else:
            namespace, namespace_value, target = ReliabilityNamespace.GLOBAL, "global", self.GLOBAL_MARKET_ID
        record = self._store.update_reliability(source_id, target, outcome_correct)
        if update_global and namespace != ReliabilityNamespace.GLOBAL:
            self._store.update_reliability(source_id, self.GLOBAL_MARKET_ID, outcome_correct)
        return NamespacedReliabilityRecord(source_id, namespace, namespace_value, record.reliability,
                                           record.confidence, record.updated_at, False)

    def set_global_reliability(self, source_id: str, reliability: float,
                               confidence: float) -> NamespacedReliabilityRecord:
        """reliability_abstraction.py:242-283: upsert through a fresh connection to the
        same path (as the reference does; for ":memory:" that is a separate database)."""
        now = datetime.now(timezone.utc).isoformat()
        conn = sqlite3.connect(self._store._db_path)
        conn.execute(
            "INSERT INTO sources (source_id, market_id, reliability, confidence, updated_at) "
            "VALUES (?, ?, ?, ?, ?) ON CONFLICT(source_id, market_id) "
            "DO UPDATE SET reliability = excluded.reliability, confidence = excluded.confidence, "
            "updated_at = excluded.updated_at",
            (source_id, self.GLOBAL_MARKET_ID, reliability, confidence, now),
        )
        conn.commit()
        conn.close()
        return NamespacedReliabilityRecord(source_id, ReliabilityNamespace.GLOBAL, "global", reliability,
                                           confidence, now, False)

    def close(self) -> None:
        self._store.close()

    def __enter__(self) -> "NamespacedReliabilityStore":
        return self

    def __exit__(self, *exc_info: object) -> None:
        self.close()

    # ------------------------------------------------------------------ batched path (f3)
    def _scope(self, key: str, names: Sequence[str], dev) -> Tuple[batch.ScopeTable, List[str]]:
        rows = self._store._conn.execute(
            "SELECT source_id, reliability, confidence, updated_at FROM sources WHERE market_id = ?",
            (key,)).fetchall()
        idx = {n: i for i, n in enumerate(names)}
        S = len(names)
        rel = np.full(S, DEFAULT_RELIABILITY)
        conf = np.full(S, DEFAULT_CONFIDENCE)
        t_us = np.full(S, NO_TIMESTAMP, np.int64)
        has = np.zeros(S, np.uint8)
        stamps = [""] * S
        for sid, r, c, ts in rows:
            i = idx.get(sid)
            if i is None or not ts:  # the reference only takes rows with a truthy updated_at
                continue
            rel[i], conf[i], t_us[i], has[i], stamps[i] = r, c, iso_to_us(ts), 1, ts
        T = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
        return batch.ScopeTable(T(rel), T(conf), T(t_us), T(has)), stamps

    def resolve(self, names: Sequence[str], market_id: Optional[str] = None, domain: Optional[str] = None,
                apply_decay: bool = True, now: Optional[datetime] = None, mark_cold: bool = False,
                device=None):
        """get_reliability(sid, market_id, domain, apply_decay) for every sid of ``names`` in
        one kernel launch.  Returns (SourceTable for batch.consensus, scope codes u8[S],
        per-source updated_at strings of the chosen rows)."""
        N.require_gpu()
        dev = device or N.device()
        names = list(names)
        keys = [market_id if market_id else None, f"__domain__:{domain}" if domain else None,
                self.GLOBAL_MARKET_ID]
        scopes, stamps = [], []
        for key in keys:
            if key is None:
                scopes.append(None)
                stamps.append(None)
            else:
                sc, st = self._scope(key, names, dev)
                scopes.append(sc)
                stamps.append(st)
        now_us = dt_to_us(now or datetime.now(timezone.utc))
        table, scope = batch.namespace_resolve(scopes, now_us, apply_decay=apply_decay, mark_cold=mark_cold,
                                               names=names)
        code = scope.cpu().numpy()
        chosen = [stamps[c][i] if c < 3 else "" for i, c in enumerate(code)]
        return table, scope, chosen

    def get_reliability_many(self, names: Sequence[str], market_id: Optional[str] = None,
                             domain: Optional[str] = None, apply_decay: bool = True,
                             now: Optional[datetime] = None) -> List[NamespacedReliabilityRecord]:
        """Records identical to per-source get_reliability, from one resolve() launch."""
        table, scope, stamps = self.resolve(names, market_id, domain, apply_decay, now)
        rc = table.relconf[:len(names)].cpu().numpy()
        code = scope.cpu().numpy()
        out = []
        for i, sid in enumerate(names):
            c = int(code[i])
            if c == batch.NS_COLD:
                out.append(NamespacedReliabilityRecord(sid, ReliabilityNamespace.GLOBAL, "cold-start",
                                                       DEFAULT_RELIABILITY, DEFAULT_CONFIDENCE, "", True))
                continue
            ns, fb = _SCOPE_NS[c]
            value = market_id if c == batch.NS_MARKET else domain if c == batch.NS_DOMAIN else "global"
            out.append(NamespacedReliabilityRecord(sid, ns, value, float(rc[i, 0]), float(rc[i, 1]), stamps[i], fb))
        return out
