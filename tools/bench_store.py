"""Throughput of the SQLite <-> HBM bulk path on one GPU: one scope of S
sources loaded into a dense HBM table (ORDER BY source_id, ISO stamp -> int64 us), the
decayed view of every source (one launch), and a bulk outcome update with its write-back
(one launch + one upsert transaction).  The database is built in a temp dir before timing.

Usage: python tools/bench_store.py [--sources 1000000]
"""
import argparse
import json
import os
import sys
import tempfile
import time
from datetime import datetime, timedelta, timezone

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bayesian-consensus-engine_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bayesian_engine.reliability import SQLiteReliabilityStore  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sources", type=int, default=1_000_000)
    a = ap.parse_args()
    S = a.sources
    rng = np.random.default_rng(4)
    now = datetime(2026, 6, 1, tzinfo=timezone.utc)
    names = [f"src-{i:07d}" for i in range(S)]
    ages = rng.uniform(0, 120, S)
    rows = [(n, "m", float(r), float(c), (now - timedelta(days=float(d))).isoformat())
            for n, r, c, d in zip(names, rng.uniform(0.1, 1, S), rng.uniform(0, 1, S), ages)]
    with tempfile.TemporaryDirectory() as d:
        db = os.path.join(d, "rel.db")
        with SQLiteReliabilityStore(db) as st:
            with st._conn:
                st._conn.executemany("INSERT INTO sources (source_id, market_id, reliability, confidence, updated_at)"
                                     " VALUES (?, ?, ?, ?, ?)", rows)
            st.load_table("m", names[:1000])  # warm-up
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            table = st.load_table("m")
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            view = st.decayed_view(table, now=now)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            outcomes = {n: bool(b) for n, b in zip(names, rng.integers(0, 2, S))}
            t3 = time.perf_counter()
            st.apply_outcomes("m", outcomes, now=now)
            t4 = time.perf_counter()
            assert table.n == S and view.numel() >= S
    print(json.dumps({"metric": "sources/sec through the SQLite<->HBM bulk path (f1, host-bound)",
                      "config": {"sources": S},
                      "load_table_s": t1 - t0, "load_sources_per_s": S / (t1 - t0),
                      "decayed_view_s": t2 - t1,
                      "apply_outcomes_with_writeback_s": t4 - t3, "apply_sources_per_s": S / (t4 - t3)}))


if __name__ == "__main__":
    main()
