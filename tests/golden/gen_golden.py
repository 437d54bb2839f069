#!/usr/bin/env python3
"""Generate golden input/output vectors by running the REFERENCE Python.

Test infrastructure only.  Run in the build container (where the read-only
reference lives at /root/reference):

    PYTHONPATH=/root/reference/src python3 tests/golden/gen_golden.py

It imports ``bayesian_engine`` from the reference, freezes the wall clock
(the reference reads ``datetime.now`` in ``reliability.py:175`` and
``decay.py:136-137``; recipe from SURVEY.md §8(c) c5) and writes small JSON /
NPZ fixtures next to this file.  Only the fixtures (data) and this script are
committed; the reference itself never travels to the GPU box.

Fixture map:
  consensus_cases.json    core.compute_consensus single-market cases      (core.py:63-179)
  validate_cases.json     core.validate_input_payload messages            (core.py:24-60)
  decay_cases.json        decay.* grids                                    (decay.py:31-185)
  update_traces.json      SQLiteReliabilityStore update traces            (reliability.py:142-233)
  tiebreak_cases.json     DeterministicTieBreaker.resolve                 (tiebreak.py:73-152)
  summarize_cases.json    CrossMarketAggregator.summarize_sources         (market.py:256-321)
  market_cases.json       MarketStore.compute_all_consensus w/ store      (market.py:200-221)
  c2_slice.npz            config-2-shaped CSR slice (2000 x 32, 10k src)
  c3_slice.npz            config-3-shaped ragged Zipf slice
  c4_replay.npz           config-4-shaped decay + outcome replay (S=2000, T=30)
  c5_reestimate.npz       config-5-shaped re-estimation (A=64, M=512, k=3)
  cli_cases.json          CLI stdout/rc (config 1 = examples/sample_input.json)
  namespace_cases.json    NamespacedReliabilityStore.get_reliability      (reliability_abstraction.py:119-188)
  aggregate_cases.json    CrossMarketAggregator.aggregate_consensus       (market.py:340-408)

  python3 tests/golden/gen_golden.py [name ...]   regenerates only the named fixtures
"""

from __future__ import annotations

import json
import math
import os
import subprocess
import sys
from datetime import datetime, timedelta, timezone

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_SRC = "/root/reference/src"
if REF_SRC not in sys.path:
    sys.path.insert(0, REF_SRC)

import bayesian_engine.decay as ref_decay  # noqa: E402
import bayesian_engine.reliability as ref_rel  # noqa: E402
from bayesian_engine.core import (  # noqa: E402
    ValidationError,
    compute_consensus,
    validate_input_payload,
)
from bayesian_engine.market import (  # noqa: E402
    CrossMarketAggregator,
    MarketId,
    MarketStore,
)
from bayesian_engine.tiebreak import AgentSignal, DeterministicTieBreaker  # noqa: E402

assert ref_rel.__file__.startswith(REF_SRC), "must import the reference, not the build"

EPOCH = datetime(1970, 1, 1, tzinfo=timezone.utc)


# ---------------------------------------------------------------------------
# frozen clock
# ---------------------------------------------------------------------------
class _FrozenDT(datetime):
    _now = datetime(2026, 3, 1, 12, 0, 0, tzinfo=timezone.utc)

    @classmethod
    def now(cls, tz=None):  # noqa: D401
        n = cls._now
        return n if tz is None else n.astimezone(tz)


def freeze(now: datetime) -> None:
    _FrozenDT._now = now
    ref_decay.datetime = _FrozenDT
    ref_rel.datetime = _FrozenDT


def to_us(dt: datetime) -> int:
    d = dt - EPOCH
    return (d.days * 86400 + d.seconds) * 1_000_000 + d.microseconds


def dump(name: str, obj) -> None:
    path = os.path.join(HERE, name)
    with open(path, "w", encoding="utf-8") as f:
        json.dump(obj, f, indent=1, sort_keys=False)
    print("wrote", path, os.path.getsize(path), "bytes")


# ---------------------------------------------------------------------------
# consensus single-market cases
# ---------------------------------------------------------------------------
def gen_consensus_cases(rng: np.random.Generator) -> None:
    cases = []

    def add(name, signals, rel=None):
        res = compute_consensus(signals, rel)
        cases.append({"name": name, "signals": signals, "source_reliability": rel, "expected": res})

    add("empty", [])
    add("golden", [
        {"sourceId": "agent-alpha", "probability": 0.72},
        {"sourceId": "agent-beta", "probability": 0.65},
        {"sourceId": "agent-gamma", "probability": 0.72},
    ])
    add("two_avg", [{"sourceId": "agent-a", "probability": 0.7}, {"sourceId": "agent-b", "probability": 0.8}])
    add("dups_input_order", [
        {"sourceId": "b", "probability": 0.1}, {"sourceId": "a", "probability": 0.3},
        {"sourceId": "b", "probability": 0.7}, {"sourceId": "b", "probability": 0.2},
        {"sourceId": "a", "probability": 0.9},
    ], {"a": {"reliability": 0.9, "confidence": 0.8}})
    add("partial_dicts", [
        {"sourceId": "x", "probability": 0.4}, {"sourceId": "y", "probability": 0.6},
        {"sourceId": "z", "probability": 0.5},
    ], {"x": {"reliability": 0.7}, "y": {"confidence": 0.9}, "z": {}})
    add("zero_total", [{"sourceId": "a", "probability": 0.4}, {"sourceId": "b", "probability": 0.6}],
        {"a": {"reliability": 0.0, "confidence": 0.5}, "b": {"reliability": 0.0, "confidence": 0.5}})
    add("negative_total", [{"sourceId": "a", "probability": 0.4}, {"sourceId": "b", "probability": 0.6}],
        {"a": {"reliability": -0.5, "confidence": 0.5}, "b": {"reliability": 0.2, "confidence": 0.5}})
    add("int_weights", [{"sourceId": "a", "probability": 0.4}, {"sourceId": "b", "probability": 1}],
        {"a": {"reliability": 1, "confidence": 1}, "b": {"reliability": 0.5, "confidence": 0}})
    add("bool_probability", [{"sourceId": "a", "probability": True}, {"sourceId": "b", "probability": False}])
    add("unicode_ids", [
        {"sourceId": "éclair", "probability": 0.3}, {"sourceId": "Zeta", "probability": 0.5},
        {"sourceId": "alpha", "probability": 0.6}, {"sourceId": "中文", "probability": 0.9},
        {"sourceId": "\U0001f600smile", "probability": 0.1}, {"sourceId": "_under", "probability": 0.2},
        {"sourceId": "Alpha", "probability": 0.7}, {"sourceId": "Ａfullwidth", "probability": 0.8},
    ], {"alpha": {"reliability": 0.8, "confidence": 0.6}})
    add("single", [{"sourceId": "solo", "probability": 0.42}])
    add("neg_zero_prob", [{"sourceId": "a", "probability": -0.0}, {"sourceId": "b", "probability": 0.0}])
    add("nan_probability", [{"sourceId": "a", "probability": float("nan")}, {"sourceId": "b", "probability": 0.5}])
    add("out_of_range_prob", [{"sourceId": "a", "probability": 1.5}, {"sourceId": "b", "probability": -0.25}])
    add("extra_fields", [{"sourceId": "a", "probability": 0.3, "weightHint": 4}, {"sourceId": "b", "probability": 0.6}])
    add("unused_rel_keys", [{"sourceId": "a", "probability": 0.3}],
        {"a": {"reliability": 0.6, "confidence": 0.3}, "zz": {"reliability": 0.9}})
    # long single market with duplicates (exercises the long-market path)
    for n, u in ((65, 40), (200, 150), (1000, 300), (3000, 2500)):
        ids = [f"s{int(k):05d}" for k in rng.integers(0, u, size=n)]
        probs = rng.random(n).tolist()
        sig = [{"sourceId": i, "probability": p} for i, p in zip(ids, probs)]
        rel = {f"s{k:05d}": {"reliability": float(rng.uniform(0.1, 1.0)), "confidence": float(rng.random())}
               for k in range(0, u, 2)}
        add(f"long_{n}", sig, rel)
    # random short markets with duplicates and partial dicts
    for k in range(40):
        n = int(rng.integers(1, 65))
        pool = int(rng.integers(1, 80))
        ids = [f"src-{int(x):03d}" for x in rng.integers(0, pool, size=n)]
        if rng.random() < 0.3:
            probs = (rng.integers(1, 10, size=n) / 10.0).tolist()
        else:
            probs = rng.random(n).tolist()
        rel = {}
        for sid in sorted(set(ids)):
            r = rng.random()
            if r < 0.6:
                rel[sid] = {"reliability": float(rng.uniform(0, 1)), "confidence": float(rng.random())}
            elif r < 0.7:
                rel[sid] = {"reliability": float(rng.uniform(0, 1))}
            elif r < 0.75:
                rel[sid] = {"confidence": float(rng.random())}
        add(f"rand_{k}", [{"sourceId": i, "probability": p} for i, p in zip(ids, probs)],
            rel if rng.random() < 0.85 else None)
    dump("consensus_cases.json", cases)


# ---------------------------------------------------------------------------
# validation messages
# ---------------------------------------------------------------------------
def gen_validate_cases() -> None:
    good = {"schemaVersion": "1.0.0", "marketId": "m-1",
            "signals": [{"sourceId": "a", "probability": 0.6}, {"sourceId": "b", "probability": 0.4}]}

    def var(**kw):
        p = json.loads(json.dumps(good))
        p.update(kw)
        return p

    payloads = [
        ("valid", good),
        ("missing_schema", {k: v for k, v in good.items() if k != "schemaVersion"}),
        ("schema_mismatch", var(schemaVersion="2.0.0")),
        ("schema_int", var(schemaVersion=1)),
        ("missing_market", {k: v for k, v in good.items() if k != "marketId"}),
        ("blank_market", var(marketId="   ")),
        ("int_market", var(marketId=7)),
        ("missing_signals", {k: v for k, v in good.items() if k != "signals"}),
        ("signals_not_list", var(signals={"a": 1})),
        ("signal_not_obj", var(signals=[{"sourceId": "a", "probability": 0.1}, 5])),
        ("missing_source", var(signals=[{"probability": 0.1}])),
        ("blank_source", var(signals=[{"sourceId": "a", "probability": 0.1}, {"sourceId": " ", "probability": 0.2}])),
        ("int_source", var(signals=[{"sourceId": 3, "probability": 0.2}])),
        ("missing_prob", var(signals=[{"sourceId": "a"}])),
        ("string_prob", var(signals=[{"sourceId": "a", "probability": "0.5"}])),
        ("null_prob", var(signals=[{"sourceId": "a", "probability": None}])),
        ("bool_prob_ok", var(signals=[{"sourceId": "a", "probability": True}])),
        ("prob_high", var(signals=[{"sourceId": "a", "probability": 0.5}, {"sourceId": "b", "probability": 1.2}])),
        ("prob_low", var(signals=[{"sourceId": "a", "probability": -0.01}])),
        ("prob_nan_ok", var(signals=[{"sourceId": "a", "probability": float("nan")}])),
        ("prob_inf", var(signals=[{"sourceId": "a", "probability": float("inf")}])),
        ("prob_int_ok", var(signals=[{"sourceId": "a", "probability": 1}, {"sourceId": "b", "probability": 0}])),
        ("prob_int_2", var(signals=[{"sourceId": "a", "probability": 2}])),
        ("empty_signals_ok", var(signals=[])),
        ("first_error_wins", var(signals=[{"sourceId": "a", "probability": 3.0}, {"sourceId": "", "probability": 0.5}])),
        ("many_ok", var(signals=[{"sourceId": f"s{i}", "probability": i / 2000} for i in range(1500)])),
        ("unknown_fields_ok", var(extra=1, signals=[{"sourceId": "a", "probability": 0.5, "weightHint": 3}])),
    ]
    out = []
    for name, p in payloads:
        try:
            validate_input_payload(p)
            err = None
        except ValidationError as exc:
            err = str(exc)
        out.append({"name": name, "payload": p, "error": err})
    dump("validate_cases.json", out)


# ---------------------------------------------------------------------------
# decay grids
# ---------------------------------------------------------------------------
def gen_decay_cases(rng: np.random.Generator) -> None:
    from bayesian_engine.decay import (
        apply_reliability_decay,
        compute_decay_factor,
        days_since_update,
        decay_reliability_if_needed,
    )
    factor = []
    for e in [0, -1, -100, 1e-9, 0.5, 1, 15, 29.999, 30, 60, 90, 1000, 1e6] + rng.uniform(0, 200, 200).tolist():
        for h in (30, 15, 1, 7.5):
            factor.append([e, h, compute_decay_factor(e, h)])
    apply = []
    rs = [0.0, 0.05, 0.1, 0.5, 0.8, 0.99, 1.0, 1.5] + rng.random(60).tolist()
    es = [0, -10, 0.5, 1, 10, 30, 1000] + rng.uniform(0, 120, 40).tolist()
    for r in rs:
        for e in es:
            for h, m in ((30, 0.1), (1, 0.1), (30, 0.0), (10, 0.3)):
                apply.append([r, e, h, m, apply_reliability_decay(r, e, h, m)])
    now = datetime(2026, 2, 21, 12, 0, 0, tzinfo=timezone.utc)
    days = []
    stamps = [None, "", "not-a-date", now.isoformat(), (now - timedelta(days=1)).isoformat(),
              (now - timedelta(hours=12)).isoformat(), "2026-02-20T12:00:00", "2026-02-20T12:00:00+00:00",
              "2026-02-20T13:30:00+01:30", (now + timedelta(days=3)).isoformat(),
              "2025-11-03T07:15:42.123456+00:00", "2026-02-21", "2026-02-20 06:00:00"]
    for k in range(60):
        dt = now - timedelta(microseconds=int(rng.integers(0, 200 * 86400 * 10**6)))
        stamps.append(dt.isoformat())
    for s in stamps:
        days.append([s, to_us(now), days_since_update(s, now=now)])
    ifneeded = []
    for s in stamps:
        for r in (0.8, 0.1, 0.55):
            v, changed = decay_reliability_if_needed(r, s, now=now)
            ifneeded.append([r, s, to_us(now), v, changed])
    dump("decay_cases.json", {"factor": factor, "apply": apply, "days": days, "if_needed": ifneeded})


# ---------------------------------------------------------------------------
# update traces through the real SQLite store, frozen clock
# ---------------------------------------------------------------------------
def gen_update_traces(rng: np.random.Generator) -> None:
    traces = []
    base = datetime(2026, 3, 1, 12, 0, 0, tzinfo=timezone.utc)
    seqs = [[True] * 12, [False] * 12, [True, False] * 6,
            [bool(x) for x in rng.integers(0, 2, 25)], [bool(x) for x in rng.integers(0, 2, 25)]]
    for si, seq in enumerate(seqs):
        store = ref_rel.SQLiteReliabilityStore(":memory:")
        steps = []
        for k, ok in enumerate(seq):
            now = base + timedelta(hours=k, microseconds=k * 7)
            freeze(now)
            dry = store.compute_update("src", "m", ok)
            rec = store.update_reliability("src", "m", ok, dry_run=(k == 3))
            steps.append({"correct": ok, "now_us": to_us(now), "dry_run": k == 3,
                          "reliability": rec.reliability, "confidence": rec.confidence,
                          "updated_at": rec.updated_at, "compute_update_r": dry.reliability,
                          "compute_update_c": dry.confidence})
        traces.append({"name": f"seq{si}", "start": "cold", "steps": steps})
        store.close()
    # start from explicit rows (raw SQL insert = test harness only)
    for k in range(30):
        r0 = float(rng.random()) if k % 5 else [0.0, 1.0, 0.95, 0.05, 0.5][k // 5 % 5]
        c0 = float(rng.random()) if k % 7 else 1.0
        store = ref_rel.SQLiteReliabilityStore(":memory:")
        store._conn.execute("INSERT INTO sources VALUES (?,?,?,?,?)", ("s", "m", r0, c0, "2026-01-01T00:00:00+00:00"))
        steps = []
        for j in range(6):
            ok = bool(rng.integers(0, 2))
            freeze(base + timedelta(days=j))
            rec = store.update_reliability("s", "m", ok)
            steps.append({"correct": ok, "reliability": rec.reliability, "confidence": rec.confidence})
        traces.append({"name": f"row{k}", "start": [r0, c0], "steps": steps})
        store.close()
    dump("update_traces.json", traces)


# ---------------------------------------------------------------------------
# tie-break
# ---------------------------------------------------------------------------
def _tb_case(agents):
    tb = DeterministicTieBreaker()
    groups = tb._group_by_prediction(agents)
    raw = [[k, tb._calculate_group_metrics(v)] for k, v in groups.items()]
    pred, diag = tb.resolve(agents)
    return {
        "agents": [[a.agent_id, a.prediction, a.confidence, a.weight, a.reliability_score] for a in agents],
        "winner": pred,
        "method": diag.method,
        "tie_resolved_by": diag.tie_resolved_by,
        "selected_group": diag.selected_group,
        "confidence_variance": diag.confidence_variance,
        "groups": [[k, v] for k, v in diag.groups.items()],
        "raw_groups": [[k, {kk: vv for kk, vv in m.items() if kk != "agents"}] for k, m in raw],
    }


def gen_tiebreak_cases(rng: np.random.Generator) -> None:
    A = AgentSignal
    cases = []
    fixed = [
        [A("a1", 0.75, 0.8)],
        [A("a1", 0.75, 0.8, 0.9, 0.7), A("a2", 0.75, 0.75, 0.85, 0.6), A("a3", 0.75, 0.70, 0.80, 0.5)],
        [A("a1", 0.75, 0.85, 0.9, 0.82), A("a2", 0.75, 0.80, 0.85, 0.78), A("a3", 0.25, 0.70, 0.6, 0.65),
         A("a4", 0.25, 0.65, 0.55, 0.70), A("a5", 0.25, 0.60, 0.50, 0.60)],
        [A("a1", 0.75, 0.8, 1.0, 0.5), A("a2", 0.25, 0.8, 1.0, 0.9)],
        [A("a1", 0.75, 0.8, 1.0, 0.9), A("a2", 0.25, 0.8, 1.0, 0.9)],
        [A("a1", 0.75, 0.8, 0.9, 0.7), A("a2", 0.25, 0.6, 0.5, 0.5)],
        [A("a", 0.0078125, 0.5), A("b", 0.007812, 0.5, 2.0), A("c", 0.007813, 0.5)],
        [A("a", -0.0, 0.5, 1.0, 0.2), A("b", 0.0, 0.5, 3.0, 0.9), A("c", 0.5, 0.5, 2.0, 0.5)],
        [A("a", 0.1234565, 0.1), A("b", 0.1234575, 0.2), A("c", 0.12345650000000001, 0.3)],
        [A("a", 0.3, 0.2, 0.0, 0.0), A("b", 0.6, 0.2, 0.0, 0.0)],
        [A("a", 1.5, 0.2, 1.0, 0.1), A("b", -2.0, 0.9, 1.0, 0.1)],
        [A("a", 0.5, 0.0, -1.0, 0.3), A("b", 0.4, 1.0, -1.0, 0.3), A("c", 0.4, 1.0, 0.5, 0.3)],
    ]
    for ag in fixed:
        cases.append(_tb_case(ag))
    grid = [0.1, 0.2, 0.25, 0.3, 0.5, 0.7, 0.75, 0.9]
    for k in range(150):
        n = int(rng.integers(2, 40))
        agents = []
        for i in range(n):
            if k % 3 == 0:
                p = float(rng.choice(grid))
            elif k % 3 == 1:
                p = float(rng.integers(0, 8)) / 8.0 + float(rng.choice([0.0, 1e-7, 4e-7, 5e-7, 6e-7]))
            else:
                p = float(rng.random())
            w = float(rng.choice([1.0, 0.5, 2.0])) if k % 2 else float(rng.random() * 2)
            rel = float(rng.choice([0.5, 0.9])) if k % 4 < 2 else float(rng.random())
            agents.append(A(f"ag{i}", p, float(rng.random()), w, rel))
        cases.append(_tb_case(agents))
    dump("tiebreak_cases.json", cases)


# ---------------------------------------------------------------------------
# summarize_sources
# ---------------------------------------------------------------------------
def gen_summarize_cases(rng: np.random.Generator) -> None:
    cases = []
    for k in range(10):
        store = MarketStore()
        mk = []
        for m in range(int(rng.integers(1, 30))):
            mid = f"cat{m % 3}:mk{m}"
            market = store.create_market(MarketId(mid))
            sig = []
            for _ in range(int(rng.integers(0, 12))):
                s = {"sourceId": f"a{int(rng.integers(0, 9))}"}
                if rng.random() < 0.9:
                    s["probability"] = float(rng.choice([0.5, 0.49999999999999994, 0.2, 0.8])) \
                        if rng.random() < 0.3 else float(rng.random())
                sig.append(s)
                market.add_signal(s)
            state = rng.random()
            outcome = None
            if state < 0.8:
                outcome = bool(rng.integers(0, 2))
                market.resolve(outcome)
            mk.append({"marketId": mid, "signals": sig, "resolved": outcome is not None, "outcome": outcome})
        perf = CrossMarketAggregator(store).summarize_sources()
        exp = {sid: {"total": p.total_markets, "correct": p.correct_predictions, "wrong": p.wrong_predictions,
                     "reliability": p.reliability, "markets": p.markets} for sid, p in perf.items()}
        cases.append({"markets": mk, "expected": exp, "order": list(perf.keys())})
    dump("summarize_cases.json", cases)


# ---------------------------------------------------------------------------
# MarketStore.compute_all_consensus through a reliability store, frozen clock
# ---------------------------------------------------------------------------
def gen_market_cases(rng: np.random.Generator) -> None:
    now = datetime(2026, 3, 1, 12, 0, 0, tzinfo=timezone.utc)
    cases = []
    for k in range(4):
        store = ref_rel.SQLiteReliabilityStore(":memory:")
        rows = []
        for s in range(12):
            for m in range(5):
                if rng.random() < 0.5:
                    t = now - timedelta(microseconds=int(rng.integers(0, 60 * 86400 * 10**6)))
                    ts = t.isoformat() if rng.random() < 0.9 else ""
                    row = (f"a{s}", f"mk{m}", float(rng.random()), float(rng.random()), ts)
                    store._conn.execute("INSERT INTO sources VALUES (?,?,?,?,?)", row)
                    rows.append(list(row))
        ms = MarketStore()
        markets = []
        for m in range(5):
            mid = f"mk{m}"
            market = ms.create_market(MarketId(mid))
            sig = [{"sourceId": f"a{int(rng.integers(0, 12))}", "probability": float(rng.random())}
                   for _ in range(int(rng.integers(0, 10)))]
            for s in sig:
                market.add_signal(s)
            closed = m == 4 and k % 2 == 1
            if closed:
                market.resolve(True)
            markets.append({"marketId": mid, "signals": sig, "resolved": closed})
        freeze(now)
        res = ms.compute_all_consensus(store)
        res_nostore = ms.compute_all_consensus(None)
        cases.append({"now_us": to_us(now), "rows": rows, "markets": markets, "expected": res,
                      "expected_no_store": res_nostore})
        store.close()
    dump("market_cases.json", cases)


# ---------------------------------------------------------------------------
# CSR slices (config 2 / config 3 shaped)
# ---------------------------------------------------------------------------
def _run_csr(offsets, sid, prob, names, rel, conf, present, has_rel, has_conf):
    M = len(offsets) - 1
    N = len(sid)
    rdict = {}
    for s in np.nonzero(present)[0]:
        d = {}
        if has_rel[s]:
            d["reliability"] = float(rel[s])
        if has_conf[s]:
            d["confidence"] = float(conf[s])
        rdict[names[s]] = d
    name_to_idx = {n: i for i, n in enumerate(names)}
    out = {
        "consensus": np.zeros(M), "is_null": np.zeros(M, np.uint8), "confidence": np.zeros(M),
        "total_weight": np.zeros(M), "n_unique": np.zeros(M, np.int32), "err_idx": np.full(M, -1, np.int32),
        "usid": np.full(N, -1, np.int32), "weight": np.zeros(N), "nweight": np.zeros(N),
        "cold": np.zeros(N, np.uint8),
    }
    for m in range(M):
        a, b = int(offsets[m]), int(offsets[m + 1])
        sig = [{"sourceId": names[int(sid[i])], "probability": float(prob[i])} for i in range(a, b)]
        try:
            validate_input_payload({"schemaVersion": "1.0.0", "marketId": f"m{m}", "signals": sig})
        except ValidationError as exc:
            msg = str(exc)
            out["err_idx"][m] = int(msg.split("[")[1].split("]")[0])
        r = compute_consensus(sig, rdict)
        if b == a:
            out["is_null"][m] = 1
            continue
        if r["consensus"] is None:
            out["is_null"][m] = 1
        else:
            out["consensus"][m] = r["consensus"]
        out["confidence"][m] = r["confidence"]
        out["total_weight"][m] = r["normalization"]["totalWeight"]
        out["n_unique"][m] = r["diagnostics"]["uniqueSources"]
        cold = set(r["diagnostics"]["coldStartSources"])
        for j, sw in enumerate(r["sourceWeights"]):
            out["usid"][a + j] = name_to_idx[sw["sourceId"]]
            out["weight"][a + j] = sw["weight"]
            out["nweight"][a + j] = sw["normalizedWeight"]
            out["cold"][a + j] = sw["sourceId"] in cold
    return out


def _table(rng, S, p_present=0.9):
    rel = rng.uniform(0.1, 1.0, S)
    conf = rng.random(S)
    present = (rng.random(S) < p_present).astype(np.uint8)
    has_rel = np.ones(S, np.uint8)
    has_conf = np.ones(S, np.uint8)
    u = rng.random(S)
    has_conf[(u < 0.05)] = 0
    has_rel[(u >= 0.05) & (u < 0.08)] = 0
    # zero-weight and negative-weight sources (edge semantics core.py:131,151)
    rel[:8] = 0.0
    rel[8:12] = -0.3
    present[:12] = 1
    has_rel[:12] = 1
    # bake defaults into the dense table (config.py:17-18 / core.py:111-112)
    rel_t = np.where(present & has_rel, rel, 0.5)
    conf_t = np.where(present & has_conf, conf, 0.25)
    return rel, conf, present, has_rel, has_conf, rel_t, conf_t


def gen_c2_slice(rng: np.random.Generator) -> None:
    M, L, S = 2000, 32, 10000
    names = [f"src-{i:05d}" for i in range(S)]
    sid = rng.integers(0, S, size=M * L).astype(np.int32)
    prob = rng.random(M * L)
    grid = rng.random(M) < 0.1
    for m in np.nonzero(grid)[0]:
        prob[m * L:(m + 1) * L] = rng.integers(1, 10, L) / 10.0
    # forced duplicates in 5% of markets
    for m in np.nonzero(rng.random(M) < 0.05)[0]:
        k = int(rng.integers(2, 6))
        pos = rng.choice(L, size=k, replace=False) + m * L
        sid[pos] = sid[pos[0]]
    # zero / negative-total markets
    sid[0:L] = rng.integers(0, 8, L)
    sid[L:2 * L] = rng.integers(0, 12, L)
    sid[2 * L:3 * L] = rng.integers(8, 12, L)
    # out-of-range probabilities (validation error index, core.py:59-60)
    for m in (5, 17, 333):
        prob[m * L + (m % L)] = 1.5 if m % 2 else -0.25
    prob[7 * L + 3] = np.nan
    offsets = np.arange(0, M * L + 1, L, dtype=np.int64)
    rel, conf, present, has_rel, has_conf, rel_t, conf_t = _table(rng, S)
    out = _run_csr(offsets, sid, prob, names, rel, conf, present, has_rel, has_conf)
    np.savez_compressed(os.path.join(HERE, "c2_slice.npz"), offsets=offsets, sid=sid, prob=prob,
                        rel=rel_t, conf=conf_t, present=present, **out)
    print("wrote c2_slice.npz")


def gen_c3_slice(rng: np.random.Generator) -> None:
    S = 20000
    names = [f"z{i:06d}" for i in range(S)]
    lens = []
    while len(lens) < 48:
        lens.append(int(np.floor(np.exp(rng.uniform(0, np.log(4097))))))
    lens[:6] = [1, 2, 64, 65, 4096, 4095]
    perm = rng.permutation(S)
    zipf = rng.zipf(1.1, size=sum(lens))
    zipf = np.minimum(zipf, S) - 1
    sid = perm[zipf].astype(np.int32)
    prob = rng.random(len(sid))
    offsets = np.zeros(len(lens) + 1, np.int64)
    offsets[1:] = np.cumsum(lens)
    rel, conf, present, has_rel, has_conf, rel_t, conf_t = _table(rng, S)
    out = _run_csr(offsets, sid, prob, names, rel, conf, present, has_rel, has_conf)
    np.savez_compressed(os.path.join(HERE, "c3_slice.npz"), offsets=offsets, sid=sid, prob=prob,
                        rel=rel_t, conf=conf_t, present=present, **out)
    print("wrote c3_slice.npz", len(sid), "signals")


# ---------------------------------------------------------------------------
# config-4-shaped replay through the real store (frozen clock)
# ---------------------------------------------------------------------------
def gen_c4_replay(rng: np.random.Generator) -> None:
    S, T = 2000, 30
    scope = "__global__"
    now0 = datetime(2026, 3, 1, 0, 0, 0, tzinfo=timezone.utc)
    store = ref_rel.SQLiteReliabilityStore(":memory:")
    names = [f"src-{i:05d}" for i in range(S)]
    present = (rng.random(S) < 0.85).astype(np.uint8)
    r0 = rng.random(S)
    c0 = rng.random(S)
    t0_us = np.zeros(S, np.int64)
    ts_kind = np.zeros(S, np.uint8)  # 0 valid, 1 empty string, 2 invalid text, 3 future
    NOTS = np.iinfo(np.int64).min
    for s in range(S):
        if not present[s]:
            t0_us[s] = NOTS
            continue
        u = rng.random()
        if u < 0.02:
            ts, ts_kind[s], t0_us[s] = "", 1, NOTS
        elif u < 0.03:
            ts, ts_kind[s], t0_us[s] = "garbage", 2, NOTS
        elif u < 0.05:
            t = now0 + timedelta(microseconds=int(rng.integers(1, 40 * 86400 * 10**6)))
            ts, ts_kind[s], t0_us[s] = t.isoformat(), 3, to_us(t)
        else:
            t = now0 - timedelta(microseconds=int(rng.integers(0, 90 * 86400 * 10**6)))
            ts, t0_us[s] = t.isoformat(), to_us(t)
        store._conn.execute("INSERT INTO sources VALUES (?,?,?,?,?)", (names[s], scope, float(r0[s]), float(c0[s]), ts))
    flags = np.zeros((T, S), np.uint8)
    views = np.zeros((T, S))
    for k in range(T):
        now = now0 + timedelta(days=k)
        freeze(now)
        part = rng.random(S) < 0.1
        corr = rng.random(S) < 0.6
        flags[k] = part.astype(np.uint8) | (corr.astype(np.uint8) << 1)
        for s in range(S):
            views[k, s] = store.get_reliability(names[s], scope, apply_decay=True).reliability
        for s in np.nonzero(part)[0]:
            store.update_reliability(names[s], scope, bool(corr[s]))
    final = {r.source_id: r for r in store.list_sources(scope)}
    fr = np.zeros(S)
    fc = np.zeros(S)
    ft = np.full(S, NOTS, np.int64)
    fp = np.zeros(S, np.uint8)
    for s in range(S):
        rec = final.get(names[s])
        if rec is None:
            continue
        fp[s] = 1
        fr[s], fc[s] = rec.reliability, rec.confidence
        try:
            ft[s] = to_us(datetime.fromisoformat(rec.updated_at)) if rec.updated_at else NOTS
        except ValueError:
            ft[s] = NOTS
    np.savez_compressed(os.path.join(HERE, "c4_replay.npz"), now0_us=np.int64(to_us(now0)), step_us=np.int64(86400 * 10**6),
                        present=present, r0=r0, c0=c0, t0_us=t0_us, ts_kind=ts_kind, flags=flags, views=views,
                        final_r=fr, final_c=fc, final_t_us=ft, final_present=fp)
    store.close()
    print("wrote c4_replay.npz")


# ---------------------------------------------------------------------------
# config-5-shaped re-estimation, composed from the reference's own functions
# ---------------------------------------------------------------------------
def gen_c5(rng: np.random.Generator) -> None:
    A, M, K = 64, 512, 3
    truth = rng.random(M) < 0.5
    P = rng.beta(2, 2, size=(A, M))
    oracle = rng.random(A) < 0.1
    for a in np.nonzero(oracle)[0]:
        P[a] = np.where(truth, rng.beta(5, 2, M), rng.beta(2, 5, M))
    names = [f"agent-{a:05d}" for a in range(A)]
    w = np.full(A, 0.5)
    cons = np.zeros((K, M))
    cnull = np.zeros((K, M), np.uint8)
    ws = np.zeros((K, A))
    agree = np.zeros((K, A), np.int64)
    for k in range(K):
        rdict = {names[a]: {"reliability": float(w[a])} for a in range(A)}
        ms = MarketStore()
        for m in range(M):
            mk = ms.create_market(MarketId(f"m{m}"))
            for a in range(A):
                mk.add_signal({"sourceId": names[a], "probability": float(P[a, m])})
        for m in range(M):
            mk = ms.get_market(MarketId(f"m{m}"))
            r = mk.compute_consensus(rdict)
            c = r["consensus"]
            if c is None:
                cnull[k, m] = 1
            else:
                cons[k, m] = c
                mk.resolve(c >= 0.5)
        perf = CrossMarketAggregator(ms).summarize_sources()
        for a in range(A):
            p = perf[names[a]]
            agree[k, a] = p.correct_predictions
            w[a] = p.reliability
        ws[k] = w
    np.savez_compressed(os.path.join(HERE, "c5_reestimate.npz"), P=P, consensus=cons, is_null=cnull,
                        weights=ws, agree=agree, iters=np.int64(K))
    print("wrote c5_reestimate.npz")


# ---------------------------------------------------------------------------
# CLI (config 1)
# ---------------------------------------------------------------------------
def gen_cli_cases() -> None:
    env = dict(os.environ, PYTHONPATH=REF_SRC)
    cases = []

    def run(args, stdin=None):
        p = subprocess.run([sys.executable, "-m", "bayesian_engine.cli"] + args, capture_output=True,
                           text=True, input=stdin, env=env, cwd="/tmp")
        cases.append({"args": args, "stdin": stdin, "rc": p.returncode, "stdout": p.stdout, "stderr": p.stderr})

    sample = json.load(open("/root/reference/examples/sample_input.json"))
    cases_inputs = {"sample_input.json": sample,
                    "golden.json": json.load(open("/root/reference/tests/fixtures/golden_regression.json"))["input"]}
    tmp = "/tmp/bce_cli_fixture"
    os.makedirs(tmp, exist_ok=True)
    for name, payload in cases_inputs.items():
        with open(os.path.join(tmp, name), "w") as f:
            json.dump(payload, f)
    run(["--dry-run", "--input", os.path.join(tmp, "sample_input.json")])
    run(["--input", os.path.join(tmp, "golden.json")])
    run(["consensus", "--input", os.path.join(tmp, "golden.json")])
    run(["--dry-run", "consensus"], stdin=json.dumps(cases_inputs["golden.json"]))
    run(["--input", os.path.join(tmp, "golden.json"), "consensus"], stdin="")
    run(["consensus"], stdin=json.dumps({"marketId": "x", "signals": []}))
    run(["consensus"], stdin=json.dumps({"schemaVersion": "1.0.0", "marketId": "x",
                                          "signals": [{"sourceId": "a", "probability": 1.2}]}))
    for c in cases:
        c["args"] = [a.replace(tmp + "/", "{DIR}/") for a in c["args"]]
    dump("cli_cases.json", {"inputs": cases_inputs, "cases": cases})


def gen_namespace_cases(rng: np.random.Generator) -> None:
    """Rows are inserted with chosen updated_at strings (set_global_reliability stamps the
    real wall clock, reliability_abstraction.py:233-235), then every (market_id, domain)
    query shape is resolved through the reference's fallback chain with decay on and off."""
    from bayesian_engine.reliability_abstraction import NamespacedReliabilityStore

    now = datetime(2026, 3, 1, 12, 0, 0, tzinfo=timezone.utc)
    freeze(now)
    S = 48
    names = sorted(f"src-{i:03d}" for i in range(S)) + ["\u00e9t\u00e9", "Zed", "a b"]
    names = sorted(names)
    scopes = {"market": "m1", "domain": "__domain__:crypto", "global": "__global__"}
    stamp_kinds = ["", "not-a-date", "aware", "naive", "future", "aware_old"]
    rows = []
    store = NamespacedReliabilityStore(":memory:")
    conn = store._store._conn
    for sid in names:
        for scope, mid in scopes.items():
            if rng.random() < 0.35:
                continue  # no row in this scope
            kind = stamp_kinds[int(rng.integers(0, len(stamp_kinds)))]
            age = float(rng.uniform(0, 200))
            if kind in ("", "not-a-date"):
                ts = kind
            elif kind == "aware":
                ts = (now - timedelta(days=age)).isoformat()
            elif kind == "naive":
                ts = (now - timedelta(days=age)).replace(tzinfo=None).isoformat()
            elif kind == "future":
                ts = (now + timedelta(days=age)).isoformat()
            else:
                ts = (now - timedelta(days=1000 + age)).isoformat()
            r = float(rng.choice([0.0, 0.05, 1.0, 1.3, float(rng.random())]))
            c = float(rng.random())
            conn.execute("INSERT INTO sources (source_id, market_id, reliability, confidence, updated_at) "
                         "VALUES (?, ?, ?, ?, ?)", (sid, mid, r, c, ts))
            rows.append([sid, mid, r, c, ts])
    queries = [("m1", "crypto"), (None, "crypto"), ("m1", None), (None, None), ("m2", "sports"), ("", "")]
    results = []
    for mid, dom in queries:
        for decay in (True, False):
            out = []
            for sid in names:
                rec = store.get_reliability(sid, market_id=mid, domain=dom, apply_decay=decay)
                out.append([rec.namespace.value, rec.namespace_value, rec.reliability, rec.confidence,
                            rec.updated_at, rec.is_fallback])
            results.append({"market_id": mid, "domain": dom, "apply_decay": decay, "records": out})
    store.close()
    dump("namespace_cases.json", {"now": now.isoformat(), "now_us": to_us(now), "names": names, "rows": rows,
                                  "queries": results})


def gen_aggregate_cases(rng: np.random.Generator) -> None:
    """Markets in several categories; some with consensus, some never computed, some empty
    (Market.compute_consensus on an empty market sets no result, market.py:117-123), some
    with a null consensus (all-zero weights); aggregate_consensus over pattern lists that
    overlap (duplicated members) for every method, plus an unknown method."""
    store = MarketStore()
    cats = ["crypto", "sports", "politics"]
    ids = []
    for i in range(60):
        cat = cats[i % 3]
        mid = MarketId(f"{cat}:m{i:02d}")
        m = store.create_market(mid)
        ids.append(str(mid))
        kind = rng.random()
        if kind < 0.1:
            continue  # no signals, never computed
        n = int(rng.integers(1, 9))
        grid = rng.random() < 0.4
        for j in range(n):
            p = float(rng.choice([0.1, 0.5, 0.5, 0.9, 0.3])) if grid else float(rng.random())
            m.add_signal({"sourceId": f"s{int(rng.integers(0, 6))}", "probability": p})
        rel = {f"s{k}": {"reliability": float(rng.choice([0.0, 0.2, 0.7, 1.0])),
                         "confidence": float(rng.choice([0.0, 0.25, 0.6]))} for k in range(6)}
        if rng.random() < 0.1:
            rel = {f"s{k}": {"reliability": 0.0, "confidence": 0.5} for k in range(6)}  # null consensus
        if kind < 0.9:
            m.compute_consensus(rel if rng.random() < 0.7 else None)
    agg = CrossMarketAggregator(store)
    pattern_sets = [["crypto:*"], ["sports:*"], ["*"], ["crypto:*", "*"], ["politics:m0*", "politics:*"],
                    ["nothing:*"], ["crypto:m00"], ["sports:m01", "sports:m04"]]
    cases = []
    for pats in pattern_sets:
        for method in ("weighted_average", "median", "majority", "bogus"):
            try:
                res = agg.aggregate_consensus(pats, method=method)
                cases.append({"patterns": pats, "method": method, "result": res})
            except ValueError as e:
                cases.append({"patterns": pats, "method": method, "error": str(e)})
    markets = []
    for key in ids:
        m = store.get_market(MarketId(key))
        markets.append({"id": key, "signals": m.signals,
                        "result": None if m.consensus_result is None else
                        {"consensus": m.consensus_result["consensus"],
                         "confidence": m.consensus_result["confidence"]}})
    dump("aggregate_cases.json", {"markets": markets, "cases": cases})


def main() -> None:
    only = set(sys.argv[1:])
    if only:
        freeze(datetime(2026, 3, 1, 12, 0, 0, tzinfo=timezone.utc))
        if "namespace" in only:
            gen_namespace_cases(np.random.default_rng(17))
        if "aggregate" in only:
            gen_aggregate_cases(np.random.default_rng(18))
        return
    freeze(datetime(2026, 3, 1, 12, 0, 0, tzinfo=timezone.utc))
    gen_consensus_cases(np.random.default_rng(11))
    gen_validate_cases()
    gen_decay_cases(np.random.default_rng(12))
    gen_update_traces(np.random.default_rng(13))
    gen_tiebreak_cases(np.random.default_rng(14))
    gen_summarize_cases(np.random.default_rng(15))
    gen_market_cases(np.random.default_rng(16))
    gen_c2_slice(np.random.default_rng(2))
    gen_c3_slice(np.random.default_rng(3))
    gen_c4_replay(np.random.default_rng(4))
    gen_c5(np.random.default_rng(5))
    gen_cli_cases()
    gen_namespace_cases(np.random.default_rng(17))
    gen_aggregate_cases(np.random.default_rng(18))


if __name__ == "__main__":
    main()
