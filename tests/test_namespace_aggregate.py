"""Namespaced fallback and cross-market aggregation (f4).

Fixtures: tests/golden/namespace_cases.json and aggregate_cases.json, produced by running
the reference's NamespacedReliabilityStore.get_reliability
(reliability_abstraction.py:119-188) and CrossMarketAggregator.aggregate_consensus
(market.py:340-408) with a frozen clock (tests/golden/gen_golden.py).

CPU tests pin the oracle (oracle/bce_oracle.c) to those fixtures; GPU tests check the
bce_namespace_resolve / bce_aggregate_groups kernels against the oracle on random inputs
and the drop-in modules against the fixtures.  Everything is bit-exact, decayed
reliabilities included: 2.0 ** x (decay.py:58) is glibc pow, restated on the GPU
(csrc/glibc_pow.hpp).
"""
import fnmatch
import math
import os
import tempfile
from datetime import datetime, timezone

import numpy as np
import pytest

from golden_util import load_json
from oracle import oracle as orc

NS_NAMES = {0: "market", 1: "domain", 2: "global", 3: "global"}


def _scopes_from_rows(fx, market_id, domain):
    """Scope arrays (rel, conf, t_us, has) per the fixture rows; None = not requested."""
    from bayesian_engine.timeutil import NO_TIMESTAMP, iso_to_us

    names = fx["names"]
    idx = {n: i for i, n in enumerate(names)}
    keys = [market_id or None, f"__domain__:{domain}" if domain else None, "__global__"]
    out = []
    for key in keys:
        if key is None:
            out.append(None)
            continue
        S = len(names)
        rel, conf = np.full(S, 0.5), np.full(S, 0.25)
        t, has = np.full(S, NO_TIMESTAMP, np.int64), np.zeros(S, np.uint8)
        for sid, mid, r, c, ts in fx["rows"]:
            if mid == key and ts:
                i = idx[sid]
                rel[i], conf[i], t[i], has[i] = r, c, iso_to_us(ts), 1
        out.append((rel, conf, t, has))
    return out


def _check_records(q, rel, conf, code, decay_tol):
    for i, rec in enumerate(q["records"]):
        ns, value, r, c, ts, fb = rec
        assert NS_NAMES[int(code[i])] == ns
        if int(code[i]) == 3:
            assert value == "cold-start" and fb is True
        assert float(conf[i]) == c
        assert float(rel[i]) == r, (i, rel[i], r)


def test_oracle_namespace_golden():
    fx = load_json("namespace_cases.json")
    for q in fx["queries"]:
        scopes = _scopes_from_rows(fx, q["market_id"], q["domain"])
        rel, conf, code = orc.namespace_resolve(scopes, q["apply_decay"], fx["now_us"])
        _check_records(q, rel, conf, code, decay_tol=False)  # pow(2, x) == CPython bit for bit


def _aggregate_groups_from_fixture(fx):
    ids = [m["id"] for m in fx["markets"]]
    cons = np.array([m["result"]["consensus"] if m["result"] and m["result"]["consensus"] is not None else 0.0
                     for m in fx["markets"]])
    conf = np.array([m["result"]["confidence"] if m["result"] and m["result"]["consensus"] is not None else 0.0
                     for m in fx["markets"]])
    has = np.array([1 if m["result"] and m["result"]["consensus"] is not None else 0 for m in fx["markets"]],
                   np.uint8)
    groups = []
    for case in fx["cases"]:
        members = [i for p in case["patterns"] for i, mid in enumerate(ids) if fnmatch.fnmatch(mid, p)]
        groups.append(members)
    goff = np.zeros(len(groups) + 1, np.int64)
    goff[1:] = np.cumsum([len(g) for g in groups])
    flat = np.array([m for g in groups for m in g] or [0], np.int64)
    return goff, flat, cons, conf, has, groups


def _check_aggregate(fx, groups, out):
    key = {"weighted_average": "wavg", "median": "median", "majority": "majority"}
    for gi, case in enumerate(fx["cases"]):
        k = int(out["n_included"][gi])
        if "error" in case:
            assert k > 0 and case["method"] not in key
            continue
        res = case["result"]
        if res["consensus"] is None:
            assert k == 0 and res["marketsIncluded"] == len(groups[gi])
            continue
        assert k == res["marketsIncluded"]
        assert float(out[key[case["method"]]][gi]) == res["consensus"], case
        assert float(out["mean_conf"][gi]) == res["confidence"], case


def test_oracle_aggregate_golden():
    fx = load_json("aggregate_cases.json")
    goff, flat, cons, conf, has, groups = _aggregate_groups_from_fixture(fx)
    out = orc.aggregate_groups(goff, flat, cons, conf, has)
    _check_aggregate(fx, groups, out)


def test_namespaced_record_is_frozen():
    """reference tests/test_reliability_abstraction.py::TestNamespacedReliabilityRecord."""
    from bayesian_engine.reliability_abstraction import NamespacedReliabilityRecord, ReliabilityNamespace

    rec = NamespacedReliabilityRecord("agent-a", ReliabilityNamespace.GLOBAL, "global", 0.8, 0.6, "2024-01-01", False)
    with pytest.raises(Exception):
        rec.reliability = 0.9
    assert ReliabilityNamespace("domain") is ReliabilityNamespace.DOMAIN


# ---------------------------------------------------------------------------------------
# GPU
# ---------------------------------------------------------------------------------------
def _dev():
    import torch

    return torch.device("cuda", 0)


@pytest.mark.gpu
@pytest.mark.parametrize("S,present", [(1, (1, 1, 1)), (63, (1, 0, 1)), (64, (0, 0, 1)), (1000, (1, 1, 1)),
                                       (100_003, (1, 1, 1)), (4097, (0, 1, 1))])
@pytest.mark.parametrize("apply_decay", [True, False])
def test_namespace_kernel_vs_oracle(S, present, apply_decay):
    import torch

    from bayesian_engine import batch
    from bayesian_engine.timeutil import NO_TIMESTAMP

    rng = np.random.default_rng(S + 7 * apply_decay)
    now_us = 1_772_366_400_000_000
    scopes_np, scopes_dev = [], []
    for q in range(3):
        if not present[q]:
            scopes_np.append(None)
            scopes_dev.append(None)
            continue
        rel = rng.choice([0.0, 0.05, 1.0, 1.3, 0.5], S) * (rng.random(S) < 0.3) + rng.random(S) * (rng.random(S) >= 0.3)
        conf = rng.random(S)
        t = now_us - rng.integers(-5 * 86_400_000_000, 400 * 86_400_000_000, S)
        t[rng.random(S) < 0.1] = NO_TIMESTAMP
        has = (rng.random(S) < 0.5).astype(np.uint8)
        scopes_np.append((rel, conf, t, has))
        T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(_dev())  # noqa: E731
        scopes_dev.append(batch.ScopeTable(T(rel), T(conf), T(t), T(has)))
    rel_o, conf_o, code_o = orc.namespace_resolve(scopes_np, apply_decay, now_us)
    for mark_cold in (False, True):
        table, code = batch.namespace_resolve(scopes_dev, now_us, apply_decay=apply_decay, mark_cold=mark_cold)
        torch.cuda.synchronize()
        rc = table.relconf[:S].cpu().numpy()
        code_g = code.cpu().numpy()
        assert np.array_equal(code_g, code_o)
        assert np.array_equal(rc[:, 1], conf_o)
        assert np.array_equal(rc[:, 0], rel_o)
        bits = table.bits.cpu().numpy().view(np.uint32)
        got = np.array([(bits[s >> 5] >> (s & 31)) & 1 for s in range(S)], np.uint8)
        exp = (code_o != 3).astype(np.uint8) if mark_cold else np.ones(S, np.uint8)
        assert np.array_equal(got, exp)


@pytest.mark.gpu
def test_namespace_store_golden(tmp_path):
    """The drop-in store: per-row get_reliability (frozen clock) and the one-launch bulk
    path both reproduce the reference's records."""
    import bayesian_engine.decay as dmod
    from bayesian_engine.reliability_abstraction import NamespacedReliabilityStore

    fx = load_json("namespace_cases.json")
    now = datetime.fromisoformat(fx["now"])
    store = NamespacedReliabilityStore(str(tmp_path / "ns.db"))
    conn = store._store._conn
    conn.executemany("INSERT INTO sources (source_id, market_id, reliability, confidence, updated_at) "
                     "VALUES (?, ?, ?, ?, ?)", [tuple(r) for r in fx["rows"]])

    class _Frozen(datetime):
        @classmethod
        def now(cls, tz=None):
            return now if tz is None else now.astimezone(tz)

    old = dmod.datetime
    dmod.datetime = _Frozen
    try:
        for q in fx["queries"]:
            bulk = store.get_reliability_many(fx["names"], q["market_id"], q["domain"], q["apply_decay"], now=now)
            for sid, rec, b in zip(fx["names"], q["records"], bulk):
                ns, value, r, c, ts, fb = rec
                one = store.get_reliability(sid, q["market_id"], q["domain"], q["apply_decay"])
                for got in (one, b):
                    assert (got.source_id, got.namespace.value, got.namespace_value, got.confidence,
                            got.updated_at, got.is_fallback) == (sid, ns, value, c, ts, fb)
                    assert got.reliability == r
                assert one.reliability == b.reliability  # per-row and bulk share one decay function
    finally:
        dmod.datetime = old
        store.close()


@pytest.mark.gpu
def test_namespace_reference_flows():
    """Restates the reference's tests/test_reliability_abstraction.py flows."""
    from bayesian_engine.config import DEFAULT_CONFIDENCE, DEFAULT_RELIABILITY
    from bayesian_engine.reliability_abstraction import NamespacedReliabilityStore, ReliabilityNamespace

    with tempfile.NamedTemporaryFile(suffix=".db", delete=False) as f:
        path = f.name
    try:
        store = NamespacedReliabilityStore(path)
        rec = store.get_reliability("unknown-source")
        assert (rec.namespace, rec.reliability, rec.confidence, rec.is_fallback) == (
            ReliabilityNamespace.GLOBAL, DEFAULT_RELIABILITY, DEFAULT_CONFIDENCE, True)
        r1 = store.get_reliability("agent-a", market_id="m1", domain="crypto")
        assert r1.namespace_value == "cold-start"
        store.set_global_reliability("agent-a", 0.7, 0.5)
        r2 = store.get_reliability("agent-a", market_id="m1", domain="crypto")
        assert r2.namespace == ReliabilityNamespace.GLOBAL and r2.reliability == pytest.approx(0.7)
        store.update_reliability("agent-a", True, domain="crypto")
        r3 = store.get_reliability("agent-a", market_id="m1", domain="crypto")
        assert r3.namespace == ReliabilityNamespace.DOMAIN and r3.is_fallback is True
        store.update_reliability("agent-a", True, market_id="m1")
        r4 = store.get_reliability("agent-a", market_id="m1", domain="crypto")
        assert (r4.namespace, r4.namespace_value, r4.is_fallback) == (ReliabilityNamespace.MARKET, "m1", False)
        wrong = store.update_reliability("agent-b", outcome_correct=False, domain="crypto", update_global=True)
        assert wrong.reliability < DEFAULT_RELIABILITY
        assert store.get_reliability("agent-b").reliability < DEFAULT_RELIABILITY
        # the bulk path agrees with the per-row chain on the same store
        names = ["agent-a", "agent-b", "agent-c"]
        now = datetime.now(timezone.utc)
        bulk = store.get_reliability_many(names, market_id="m1", domain="crypto", now=now)
        assert [b.namespace for b in bulk] == [ReliabilityNamespace.MARKET, ReliabilityNamespace.DOMAIN,
                                               ReliabilityNamespace.GLOBAL]
        assert bulk[2].namespace_value == "cold-start"
        store.close()
    finally:
        os.unlink(path)


@pytest.mark.gpu
def test_aggregate_store_golden():
    """MarketStore + CrossMarketAggregator.aggregate_consensus through the kernel vs the
    reference's results (markets rebuilt from the fixture's signals and results)."""
    from bayesian_engine.market import CrossMarketAggregator, MarketId, MarketStore

    fx = load_json("aggregate_cases.json")
    store = MarketStore()
    for m in fx["markets"]:
        mk = store.create_market(MarketId(m["id"]))
        for s in m["signals"]:
            mk.add_signal(s)
        if m["result"] is not None:
            mk.consensus_result = {"schemaVersion": "1.0.0", "consensus": m["result"]["consensus"],
                                   "confidence": m["result"]["confidence"]}
    agg = CrossMarketAggregator(store)
    for case in fx["cases"]:
        if "error" in case:
            with pytest.raises(ValueError, match="Unknown aggregation method"):
                agg.aggregate_consensus(case["patterns"], method=case["method"])
            continue
        got = agg.aggregate_consensus(case["patterns"], method=case["method"])
        assert got == case["result"], case
    ok = [c for c in fx["cases"] if "error" not in c and c["method"] == "median"]
    many = agg.aggregate_many([c["patterns"] for c in ok], method="median")
    assert many == [c["result"] for c in ok]


@pytest.mark.gpu
@pytest.mark.parametrize("G,maxlen", [(1, 0), (7, 1), (300, 40), (50, 3000), (3, 200_000), (5000, 40), (3000, 2500),
                                      (9000, 3)])
def test_aggregate_kernel_vs_oracle(G, maxlen):
    """Many more groups than workgroups (each workgroup pipelines its groups as one chunk
    stream, across group boundaries), empty groups, multi-chunk groups."""
    import torch

    from bayesian_engine import batch

    rng = np.random.default_rng(G * 31 + maxlen)
    M = 5000
    cons = rng.random(M)
    cons[rng.random(M) < 0.2] = 0.5  # ties at the vote threshold and in the median
    cons[rng.random(M) < 0.05] = 1.0
    cons[rng.random(M) < 0.05] = 0.0
    conf = rng.random(M)
    conf[rng.random(M) < 0.3] = 0.0
    has = (rng.random(M) < 0.8).astype(np.uint8)
    lens = rng.integers(0, maxlen + 1, G)
    goff = np.zeros(G + 1, np.int64)
    goff[1:] = np.cumsum(lens)
    members = rng.integers(0, M, max(int(goff[-1]), 1)).astype(np.int64)
    if G >= 7:  # a group whose members all have zero confidence (sum(conf) == 0 branch)
        conf[members[goff[1]:goff[2]]] = 0.0
    exp = orc.aggregate_groups(goff, members, cons, conf, has)
    T = lambda a: torch.from_numpy(a).to(_dev())  # noqa: E731
    r = batch.aggregate(T(goff), T(members), T(cons), T(conf), T(has))
    torch.cuda.synchronize()
    assert np.array_equal(r.n_included.cpu().numpy(), exp["n_included"])
    for k in ("wavg", "median", "majority", "mean_conf"):
        assert np.array_equal(getattr(r, k).cpu().numpy(), exp[k], equal_nan=True), k
