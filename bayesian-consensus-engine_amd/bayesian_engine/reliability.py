"""Drop-in for ``bayesian_engine.reliability`` (reference src/bayesian_engine/reliability.py).

SQLite stays on the host as the system of record (same schema, same SQL, autocommit,
WAL: reliability.py:36-79, 221-264).  The arithmetic of the hot path runs on the GPU:

* ``get_reliability(..., apply_decay=True)`` -- decay of the stored value via
  ``bce_decay_apply`` (reliability.py:114-123);
* ``compute_update`` / ``update_reliability`` -- the capped +-MAX_UPDATE_STEP step and
  the confidence growth via ``bce_outcome_update`` (reliability.py:161-173).

Bulk paths for millions of sources:

* :meth:`SQLiteReliabilityStore.load_table` -- ``SELECT ... ORDER BY source_id`` (SQLite
  BINARY collation == code-point order == the engine's rank order) into a dense HBM
  table (rel, conf, updated_at as int64 microseconds, present);
* :meth:`SQLiteReliabilityStore.decayed_view` -- ``get_reliability(apply_decay=True)``
  for every row of a scope in one launch;
* :meth:`SQLiteReliabilityStore.apply_outcomes` -- one outcome per source: one GPU launch,
  then one ``executemany`` upsert in a single transaction (``dry_run`` = no write-back).
"""
from __future__ import annotations

import sqlite3
from dataclasses import dataclass
from datetime import datetime, timezone
from pathlib import Path
from typing import Dict, List, Mapping, Optional, Sequence, Union

import numpy as np
import torch

from . import _native as N
from . import batch
from .config import (
    BASE_LEARNING_RATE,
    DECAY_HALF_LIFE_DAYS,
    DECAY_MINIMUM,
    DEFAULT_CONFIDENCE,
    DEFAULT_RELIABILITY,
    MAX_UPDATE_STEP,
)
from .decay import apply_reliability_decay, days_since_update
from .timeutil import NO_TIMESTAMP, dt_to_us, iso_to_us, iso_to_us_many, us_to_iso

__all__ = ["ReliabilityRecord", "SQLiteReliabilityStore", "DEFAULT_RELIABILITY", "DEFAULT_CONFIDENCE",
           "MAX_UPDATE_STEP", "DECAY_HALF_LIFE_DAYS", "DECAY_MINIMUM"]

_BASE_LEARNING_RATE: float = BASE_LEARNING_RATE

_CREATE_TABLE_SQL = """
CREATE TABLE IF NOT EXISTS sources (
    source_id   TEXT    NOT NULL,
    market_id   TEXT    NOT NULL,
    reliability REAL    NOT NULL DEFAULT 0.5,
    confidence  REAL    NOT NULL DEFAULT 0.5,
    updated_at  TEXT    NOT NULL,
    PRIMARY KEY (source_id, market_id)
);
"""

_UPSERT_SQL = """
INSERT INTO sources (source_id, market_id, reliability, confidence, updated_at)
VALUES (?, ?, ?, ?, ?)
ON CONFLICT(source_id, market_id)
DO UPDATE SET reliability = excluded.reliability,
              confidence  = excluded.confidence,
              updated_at  = excluded.updated_at
"""


@dataclass(frozen=True)
class ReliabilityRecord:
    """Immutable snapshot of a source's reliability data (reliability.py:48-56)."""

    source_id: str
    market_id: str
    reliability: float
    confidence: float
    updated_at: str


def _update_one_gpu(r: float, c: float, correct: bool) -> tuple:
    """reliability.py:163-173 for one row, through the batched update kernel."""
    N.require_gpu()
    dev = N.device()
    rel = torch.tensor([float(r)], dtype=torch.float64, device=dev)
    conf = torch.tensor([float(c)], dtype=torch.float64, device=dev)
    t = torch.zeros(1, dtype=torch.int64, device=dev)
    pres = torch.ones(2, dtype=torch.uint8, device=dev)
    flags = torch.tensor([1 | (2 if correct else 0)], dtype=torch.uint8, device=dev)
    batch.outcome_update(rel, conf, t, pres, flags, 0)
    return float(rel[0].item()), float(conf[0].item())


class SQLiteReliabilityStore:
    """SQLite-backed store for per-source, per-market reliability scores."""

    def __init__(self, db_path: Union[str, Path] = ":memory:") -> None:
        self._db_path = str(db_path)
        self._conn: sqlite3.Connection = sqlite3.connect(self._db_path, isolation_level=None)
        self._conn.execute("PRAGMA journal_mode=WAL")
        self._conn.execute("PRAGMA foreign_keys=ON")
        self._conn.row_factory = sqlite3.Row
        self._ensure_schema()

    # ------------------------------------------------------------------ reference API
    def get_reliability(self, source_id: str, market_id: str, apply_decay: bool = False) -> ReliabilityRecord:
        row = self._conn.execute(
            "SELECT source_id, market_id, reliability, confidence, updated_at "
            "FROM sources WHERE source_id = ? AND market_id = ?",
            (source_id, market_id),
        ).fetchone()
        if row is not None:
            reliability = row["reliability"]
            updated_at = row["updated_at"]
            if apply_decay and updated_at:
                elapsed_days = days_since_update(updated_at)
                if elapsed_days > 0:
                    reliability = apply_reliability_decay(reliability, elapsed_days, DECAY_HALF_LIFE_DAYS,
                                                          DECAY_MINIMUM)
            return ReliabilityRecord(row["source_id"], row["market_id"], reliability, row["confidence"],
                                     updated_at)
        return ReliabilityRecord(source_id, market_id, DEFAULT_RELIABILITY, DEFAULT_CONFIDENCE, "")

    def compute_update(self, source_id: str, market_id: str, outcome_correct: bool) -> ReliabilityRecord:
        current = self.get_reliability(source_id, market_id)
        new_r, new_c = _update_one_gpu(current.reliability, current.confidence, bool(outcome_correct))
        now = datetime.now(timezone.utc).isoformat()
        return ReliabilityRecord(source_id, market_id, new_r, new_c, now)

    def update_reliability(self, source_id: str, market_id: str, outcome_correct: bool,
                           dry_run: bool = False) -> ReliabilityRecord:
        result = self.compute_update(source_id, market_id, outcome_correct)
        if dry_run:
            return result
        self._conn.execute(_UPSERT_SQL, (source_id, market_id, result.reliability, result.confidence,
                                         result.updated_at))
        return result

    def list_sources(self, market_id: Optional[str] = None) -> List[ReliabilityRecord]:
        if market_id is not None:
            rows = self._conn.execute(
                "SELECT source_id, market_id, reliability, confidence, updated_at "
                "FROM sources WHERE market_id = ? ORDER BY source_id",
                (market_id,),
            ).fetchall()
        else:
            rows = self._conn.execute(
                "SELECT source_id, market_id, reliability, confidence, updated_at "
                "FROM sources ORDER BY source_id, market_id",
            ).fetchall()
        return [ReliabilityRecord(r["source_id"], r["market_id"], r["reliability"], r["confidence"],
                                  r["updated_at"]) for r in rows]

    def close(self) -> None:
        self._conn.close()

    def __enter__(self) -> "SQLiteReliabilityStore":
        return self

    def __exit__(self, *exc_info: object) -> None:
        self.close()

    def _ensure_schema(self) -> None:
        self._conn.executescript(_CREATE_TABLE_SQL)

    # ------------------------------------------------------------------ bulk paths (f1)
    def load_table(self, market_id: str, names: Optional[Sequence[str]] = None,
                   device=None) -> batch.ReliabilityTable:
        """Dense HBM table for one scope.  ``names`` (sorted) fixes the rank space (e.g. all
        sourceIds of a batch); absent rows get the baked cold-start values."""
        rows = self._conn.execute(
            "SELECT source_id, reliability, confidence, updated_at FROM sources "
            "WHERE market_id = ? ORDER BY source_id", (market_id,)).fetchall()
        if names is None:
            names = [r[0] for r in rows]
        idx = {n: i for i, n in enumerate(names)}
        S = len(names)
        rel = np.full(S, DEFAULT_RELIABILITY)
        conf = np.full(S, DEFAULT_CONFIDENCE)
        t_us = np.full(S, NO_TIMESTAMP, np.int64)
        present = np.zeros(S, np.uint8)
        if rows:
            pos = np.fromiter((idx.get(r[0], -1) for r in rows), np.int64, len(rows))
            keep = pos >= 0
            cols = list(zip(*rows))
            p = pos[keep]
            rel[p] = np.asarray(cols[1], np.float64)[keep]
            conf[p] = np.asarray(cols[2], np.float64)[keep]
            t_us[p] = iso_to_us_many(cols[3])[keep]
            present[p] = 1
        dev = device or N.device()
        T = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
        return batch.ReliabilityTable(T(rel), T(conf), T(t_us), T(present), list(names))

    def decayed_view(self, table: batch.ReliabilityTable, now: Optional[datetime] = None) -> torch.Tensor:
        """get_reliability(apply_decay=True).reliability for every source of ``table``."""
        return table.view(dt_to_us(now or datetime.now(timezone.utc)))

    def apply_outcomes(self, market_id: str, outcomes: Mapping[str, bool], dry_run: bool = False,
                       now: Optional[datetime] = None) -> Dict[str, ReliabilityRecord]:
        """update_reliability for many sources at once (one outcome each)."""
        names = sorted(outcomes)
        table = self.load_table(market_id, names)
        S = len(names)
        flags = np.zeros(S, np.uint8)
        for i, n in enumerate(names):
            flags[i] = 1 | (2 if outcomes[n] else 0)
        now_us = dt_to_us(now or datetime.now(timezone.utc))
        dflags = torch.from_numpy(flags).to(table.rel.device)
        batch.outcome_update(table.rel, table.conf, table.t_us, table.present, dflags, now_us)
        rel = table.rel[:S].cpu().numpy()
        conf = table.conf[:S].cpu().numpy()
        stamp = us_to_iso(now_us)
        out = {n: ReliabilityRecord(n, market_id, float(rel[i]), float(conf[i]), stamp) for i, n in enumerate(names)}
        if not dry_run and S:
            with self._conn:  # one transaction
                self._conn.execute("BEGIN")
                self._conn.executemany(_UPSERT_SQL, [(n, market_id, float(rel[i]), float(conf[i]), stamp)
                                                     for i, n in enumerate(names)])
        return out

    def fetch_pairs(self, pairs: Sequence[tuple]) -> Dict[tuple, tuple]:
        """Rows for (source_id, market_id) pairs -> {(sid, mid): (rel, conf, updated_at)}."""
        out = {}
        by_market: Dict[str, List[str]] = {}
        for s, m in pairs:
            by_market.setdefault(m, []).append(s)
        for m, sids in by_market.items():
            for k in range(0, len(sids), 900):
                chunk = sids[k:k + 900]
                q = ("SELECT source_id, reliability, confidence, updated_at FROM sources WHERE market_id = ? "
                     f"AND source_id IN ({','.join('?' * len(chunk))})")
                for sid, r, c, ts in self._conn.execute(q, [m, *chunk]):
                    out[(sid, m)] = (r, c, ts)
        return out
