"""GPU parity of the drop-in modules against the reference's golden vectors.

Every fixture under tests/golden/ was produced by the reference itself
(tests/golden/gen_golden.py).  Consensus, validation, decay, outcome updates, tie-break and
agreement statistics are compared with Python ``==`` (bit-exact): the reference's
``2.0 ** x`` and ``d ** 2`` are glibc pow, which the kernels restate (csrc/glibc_pow.hpp).
"""
import json
import math
import os
import subprocess
import sys
import tempfile
from datetime import datetime, timedelta, timezone

import numpy as np
import pytest

from golden_util import load_json, load_npz

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "bayesian-consensus-engine_amd")
EPOCH = datetime(1970, 1, 1, tzinfo=timezone.utc)


def _eq(a, b):
    """Python == with NaN == NaN, recursively, and the same JSON types (int vs float)."""
    if isinstance(a, float) and isinstance(b, float) and math.isnan(a) and math.isnan(b):
        return True
    if isinstance(a, dict) and isinstance(b, dict):
        return list(a) == list(b) and all(_eq(a[k], b[k]) for k in a)
    if isinstance(a, list) and isinstance(b, list):
        return len(a) == len(b) and all(_eq(x, y) for x, y in zip(a, b))
    return type(a) is type(b) and a == b


@pytest.mark.parametrize("case", load_json("consensus_cases.json"), ids=lambda c: c["name"])
def test_compute_consensus_golden(case):
    from bayesian_engine.core import compute_consensus
    got = compute_consensus(case["signals"], case["source_reliability"])
    assert _eq(got, case["expected"]), (got, case["expected"])


def test_reference_golden_regression_fixture():
    """The reference's own golden fixture (tests/fixtures/golden_regression.json, == on floats)."""
    from bayesian_engine.core import compute_consensus, validate_input_payload
    case = [c for c in load_json("consensus_cases.json") if c["name"] == "golden"][0]
    payload = {"schemaVersion": "1.0.0", "marketId": "golden-regression-1", "signals": case["signals"]}
    validate_input_payload(payload)
    r = compute_consensus(payload["signals"])
    assert r["consensus"] == 0.6966666666666667
    assert [w["normalizedWeight"] for w in r["sourceWeights"]] == [0.3333333333333333] * 3
    assert r == case["expected"]
    assert all(compute_consensus(payload["signals"]) == r for _ in range(3))


@pytest.mark.parametrize("case", load_json("validate_cases.json"), ids=lambda c: c["name"])
def test_validate_input_payload_golden(case):
    from bayesian_engine.core import ValidationError, validate_input_payload
    if case["error"] is None:
        validate_input_payload(case["payload"])
    else:
        with pytest.raises(ValidationError) as ei:
            validate_input_payload(case["payload"])
        assert str(ei.value) == case["error"]


def test_decay_golden():
    from bayesian_engine.decay import apply_reliability_decay, compute_decay_factor, decay_reliability_if_needed
    d = load_json("decay_cases.json")
    for e, h, f in d["factor"]:
        g = compute_decay_factor(e, h)
        assert g == f, (e, h, g, f)
    for r, e, h, m, v in d["apply"]:
        g = apply_reliability_decay(r, e, h, m)
        assert g == v, (r, e, h, m, g, v)
    for r, stamp, now_us, v, changed in d["if_needed"]:
        now = EPOCH + timedelta(microseconds=now_us)
        g, c = decay_reliability_if_needed(r, stamp, now=now)
        assert g == v and c == changed


def test_decay_vectorized_matches_scalar():
    import torch
    from bayesian_engine.decay import apply_reliability_decay, compute_decay_factor
    rng = np.random.default_rng(0)
    e = rng.uniform(-5, 200, 10000)
    r = rng.random(10000)
    f = compute_decay_factor(e)
    v = apply_reliability_decay(r, e)
    for i in range(0, 10000, 997):
        assert f[i] == compute_decay_factor(float(e[i])) or e[i] <= 0
        assert v[i] == apply_reliability_decay(float(r[i]), float(e[i]))
    tv = apply_reliability_decay(torch.tensor(r), torch.tensor(e))
    assert np.array_equal(tv.cpu().numpy(), v)


def test_update_traces_golden():
    from bayesian_engine.reliability import SQLiteReliabilityStore
    for tr in load_json("update_traces.json"):
        store = SQLiteReliabilityStore(":memory:")
        if tr["start"] != "cold":
            store._conn.execute("INSERT INTO sources VALUES (?,?,?,?,?)",
                                ("s", "m", tr["start"][0], tr["start"][1], "2026-01-01T00:00:00+00:00"))
        sid = "src" if tr["start"] == "cold" else "s"
        for st in tr["steps"]:
            rec = store.update_reliability(sid, "m", st["correct"], dry_run=st.get("dry_run", False))
            assert rec.reliability == st["reliability"] and rec.confidence == st["confidence"], (tr["name"], st)
        store.close()


def test_reliability_store_semantics(tmp_path):
    """Restates the reference's tests/test_reliability.py assertions."""
    from bayesian_engine.reliability import (DEFAULT_CONFIDENCE, DEFAULT_RELIABILITY, MAX_UPDATE_STEP,
                                             SQLiteReliabilityStore)
    s = SQLiteReliabilityStore(":memory:")
    assert s.update_reliability("a", "m", True).reliability > DEFAULT_RELIABILITY
    assert s.update_reliability("b", "m", False).reliability < DEFAULT_RELIABILITY
    assert abs(s.get_reliability("a", "m").reliability - DEFAULT_RELIABILITY) <= MAX_UPDATE_STEP + 1e-9
    for _ in range(20):
        s.update_reliability("lo", "m", False)
        s.update_reliability("hi", "m", True)
    assert s.get_reliability("lo", "m").reliability == 0.0
    assert s.get_reliability("hi", "m").reliability == 1.0
    c1 = s.get_reliability("a", "m").confidence
    s.update_reliability("a", "m", False)
    assert s.get_reliability("a", "m").confidence > c1
    s.update_reliability("x", "m1", True)
    s.update_reliability("x", "m2", False)
    assert s.get_reliability("x", "m1").reliability > DEFAULT_RELIABILITY > s.get_reliability("x", "m2").reliability
    ids = [r.source_id for r in s.list_sources()]
    assert ids == sorted(ids)
    assert len(s.list_sources("m1")) == 1
    s.close()
    db = tmp_path / "p.db"
    with SQLiteReliabilityStore(db) as st:
        st.update_reliability("src-a", "m-1", True)
    with SQLiteReliabilityStore(db) as st:
        rec = st.get_reliability("src-a", "m-1")
        assert rec.reliability > DEFAULT_RELIABILITY and rec.confidence > DEFAULT_CONFIDENCE


def test_bulk_store_paths_match_per_row(tmp_path):
    from bayesian_engine import decay as dmod
    from bayesian_engine.reliability import SQLiteReliabilityStore
    from bayesian_engine.timeutil import dt_to_us
    rng = np.random.default_rng(3)
    s = SQLiteReliabilityStore(":memory:")
    now = datetime(2026, 3, 1, tzinfo=timezone.utc)
    names = [f"s{i:04d}" for i in range(300)]
    for n in names[::2]:
        t = now - timedelta(microseconds=int(rng.integers(0, 90 * 86400 * 10**6)))
        s._conn.execute("INSERT INTO sources VALUES (?,?,?,?,?)", (n, "g", float(rng.random()),
                                                                   float(rng.random()), t.isoformat()))
    table = s.load_table("g", names)
    view = s.decayed_view(table, now=now).cpu().numpy()

    class _Frozen(datetime):
        @classmethod
        def now(cls, tz=None):
            return now

    old = dmod.datetime
    dmod.datetime = _Frozen
    try:
        for i, n in enumerate(names):
            assert view[i] == s.get_reliability(n, "g", apply_decay=True).reliability
    finally:
        dmod.datetime = old
    outcomes = {n: bool(rng.integers(0, 2)) for n in names[::3]}
    per_row = {n: s.compute_update(n, "g", c) for n, c in outcomes.items()}
    bulk = s.apply_outcomes("g", outcomes, now=now)
    for n, rec in bulk.items():
        assert (rec.reliability, rec.confidence) == (per_row[n].reliability, per_row[n].confidence)
        assert s.get_reliability(n, "g").reliability == rec.reliability
    assert dt_to_us(now) > 0
    s.close()


def test_tiebreak_golden():
    from bayesian_engine.tiebreak import AgentSignal, DeterministicTieBreaker
    cases = load_json("tiebreak_cases.json")
    tb = DeterministicTieBreaker()
    markets = []
    for case in cases:
        agents = [AgentSignal(a[0], a[1], a[2], a[3], a[4]) for a in case["agents"]]
        markets.append(agents)
        pred, diag = tb.resolve(agents)
        assert pred == case["winner"]
        assert diag.method == case["method"]
        assert diag.tie_resolved_by == case["tie_resolved_by"]
        assert diag.selected_group == case["selected_group"]
        assert diag.confidence_variance == case["confidence_variance"]
        assert [[k, v] for k, v in diag.groups.items()] == case["groups"]
    # the batched entry point gives the same answers in one launch
    batch = tb.resolve_many(markets)
    for (pred, diag), case in zip(batch, cases):
        assert pred == case["winner"] and diag.tie_resolved_by == case["tie_resolved_by"]


def test_tiebreak_long_markets_vs_oracle():
    import torch
    from bayesian_engine import batch
    from oracle import oracle as orc
    rng = np.random.default_rng(9)
    lens = np.array([65, 100, 1000, 4096, 2, 64, 300], np.int64)
    off = np.zeros(len(lens) + 1, np.int64)
    off[1:] = np.cumsum(lens)
    n = int(off[-1])
    pred = np.where(rng.random(n) < 0.5, rng.integers(0, 9, n) / 8.0, rng.random(n))
    pred[rng.random(n) < 0.05] = -0.0
    conf, weight, rel = rng.random(n), rng.choice([0.5, 1.0, 2.0], n), rng.choice([0.5, 0.9], n)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    r = batch.tiebreak(T(off), T(pred), T(conf), T(weight), T(rel), offsets_host=off)
    exp = orc.tiebreak_csr(off, pred, conf, weight, rel)
    assert np.array_equal(r.winner.cpu().numpy(), exp["winner"])
    assert np.array_equal(r.label.cpu().numpy(), exp["label"])
    assert np.array_equal(r.n_groups.cpu().numpy(), exp["n_groups"])
    assert np.array_equal(r.variance.cpu().numpy(), exp["variance"])  # libm pow restated (glibc_pow.hpp)
    for m in range(len(lens)):
        a, g = int(off[m]), int(exp["n_groups"][m])
        sl = slice(a, a + g)
        assert np.array_equal(r.g_key.cpu().numpy()[sl], exp["g_key"][sl])
        assert np.array_equal(r.g_count.cpu().numpy()[sl], exp["g_count"][sl])
        assert np.array_equal(r.g_density.cpu().numpy()[sl], exp["g_total"][sl] / exp["g_count"][sl])
        assert np.array_equal(r.g_maxrel.cpu().numpy()[sl], exp["g_maxrel"][sl])


def test_summarize_sources_golden():
    from bayesian_engine.market import CrossMarketAggregator, MarketId, MarketStore
    for case in load_json("summarize_cases.json"):
        store = MarketStore()
        for mk in case["markets"]:
            m = store.create_market(MarketId(mk["marketId"]))
            for s in mk["signals"]:
                m.add_signal(s)
            if mk["resolved"]:
                m.resolve(mk["outcome"])
        perf = CrossMarketAggregator(store).summarize_sources()
        assert list(perf) == case["order"]
        for sid, e in case["expected"].items():
            p = perf[sid]
            assert (p.total_markets, p.correct_predictions, p.wrong_predictions, p.reliability, p.markets) == \
                (e["total"], e["correct"], e["wrong"], e["reliability"], e["markets"])


def test_compute_all_consensus_golden():
    from bayesian_engine import decay as dmod
    from bayesian_engine.market import MarketId, MarketStore
    from bayesian_engine.reliability import SQLiteReliabilityStore
    for case in load_json("market_cases.json"):
        store = SQLiteReliabilityStore(":memory:")
        for row in case["rows"]:
            store._conn.execute("INSERT INTO sources VALUES (?,?,?,?,?)", tuple(row))
        ms = MarketStore()
        for mk in case["markets"]:
            m = ms.create_market(MarketId(mk["marketId"]))
            for s in mk["signals"]:
                m.add_signal(s)
            if mk["resolved"]:
                m.resolve(True)
        now = EPOCH + timedelta(microseconds=case["now_us"])

        class _Frozen(datetime):
            @classmethod
            def now(cls, tz=None):
                return now

        old = dmod.datetime
        dmod.datetime = _Frozen
        try:
            got = ms.compute_all_consensus(store)
        finally:
            dmod.datetime = old
        exp = case["expected"]
        assert list(got) == list(exp)
        for k in exp:
            g, e = got[k], exp[k]
            assert list(g) == list(e)
            assert _eq(g, e), (k, g, e)  # decayed weights included: bit-exact
        assert _eq(ms.compute_all_consensus(None), case["expected_no_store"])
        store.close()


def test_multi_market_reference_assertions():
    """Restates the reference's tests/test_multi_market.py numeric assertions."""
    from bayesian_engine.market import CrossMarketAggregator, Market, MarketId, MarketStore
    m = Market(id=MarketId("test-1"))
    m.add_signal({"sourceId": "agent-a", "probability": 0.7})
    m.add_signal({"sourceId": "agent-b", "probability": 0.8})
    assert m.compute_consensus()["consensus"] == 0.75
    store = MarketStore()
    m1 = store.create_market(MarketId("crypto:btc:1"))
    m1.add_signal({"sourceId": "agent-a", "probability": 0.8})
    m1.add_signal({"sourceId": "agent-b", "probability": 0.7})
    m1.resolve(True)
    m2 = store.create_market(MarketId("crypto:btc:2"))
    m2.add_signal({"sourceId": "agent-a", "probability": 0.6})
    m2.add_signal({"sourceId": "agent-b", "probability": 0.3})
    m2.resolve(True)
    perf = CrossMarketAggregator(store).summarize_sources()
    assert perf["agent-a"].correct_predictions == 2 and perf["agent-a"].accuracy == 1.0
    assert perf["agent-b"].correct_predictions == 1 and perf["agent-b"].accuracy == 0.5
    for market in store.list_markets():
        market.compute_consensus()
    agg = CrossMarketAggregator(store)
    assert agg.aggregate_consensus(["crypto:*"])["marketsIncluded"] == 2
    assert agg.aggregate_consensus(["crypto:*"], method="majority")["method"] == "majority"


def test_reestimate_c5_slice():
    import torch
    from bayesian_engine import batch
    g = load_npz("c5_reestimate.npz")
    K = int(g["iters"])
    P = torch.from_numpy(g["P"]).cuda()
    w, cons, nul, agree, hist = batch.reestimate(P, K, keep_history=True)
    for k in range(K):
        assert np.array_equal(hist[k][0].cpu().numpy(), g["consensus"][k])
        assert np.array_equal(hist[k][1].cpu().numpy(), g["is_null"][k])
        assert np.array_equal(hist[k][2].cpu().numpy(), g["agree"][k])
        assert np.array_equal(hist[k][3].cpu().numpy(), g["weights"][k])


@pytest.mark.parametrize("A,M,ld_pad", [(600, 5000, 0), (257, 2049, 3), (5, 700, 1)])
def test_reestimate_vs_oracle_tiles(A, M, ld_pad):
    """Several agent tiles (256) and market tiles (2048), ragged edges, padded rows."""
    import torch
    from bayesian_engine import batch
    from oracle import oracle as orc
    rng = np.random.default_rng(A * 7 + M)
    P = rng.beta(2, 2, size=(A, M))
    P[:, rng.random(M) < 0.02] = 0.5
    K = 2
    w_exp, c_exp, n_exp, a_exp = orc.reestimate(P, K)
    full = np.zeros((A, M + ld_pad))
    full[:, :M] = P
    Pt = torch.from_numpy(full).cuda()[:, :M]
    for mode in ("exact", "fast", "mfma"):
        # exact / fast: agent-order sums, bit-identical; mfma (the matrix-core pass): votes,
        # counts and weights identical, consensus within 4*A*2^-53 (batch.reestimate)
        w, cons, nul, agree, _ = batch.reestimate(Pt, K, mode=mode)
        if mode != "mfma":
            assert np.array_equal(cons.cpu().numpy(), c_exp[-1]), mode
        else:
            assert np.abs(cons.cpu().numpy() - c_exp[-1]).max() <= 4 * (A + 2) * 2.0 ** -53, mode
        assert np.array_equal(nul.cpu().numpy(), n_exp[-1]), mode
        assert np.array_equal(agree.cpu().numpy(), a_exp[-1]), mode
        assert np.array_equal(w.cpu().numpy(), w_exp), mode
    with pytest.raises(ValueError):
        batch.reestimate(Pt, 1, mode="tree")


@pytest.mark.parametrize("A,M", [(13, 1), (64, 63), (9, 129), (300, 4097), (13, 2), (64, 64), (9, 130), (300, 4096), (17, 190)])
def test_reestimate_votes_match_two_pass(A, M):
    """The single-read path (vote bits) gives the counts of the two-pass path that
    re-reads P: ragged word edges, A not a multiple of 16, NaN cells, zero weights."""
    import torch
    from bayesian_engine import _native as N
    rng = np.random.default_rng(A + M)
    P = rng.beta(2, 2, size=(A, M))
    P[rng.random((A, M)) < 0.01] = np.nan
    P[:, rng.random(M) < 0.05] = 0.5
    Pt = torch.from_numpy(P).cuda()
    L = N.lib()
    st = N.stream(Pt.device)
    for w0 in (0.5, 0.0):
        w = torch.full((A,), w0, dtype=torch.float64, device="cuda")
        w[::3] = 0.25 if w0 else 0.0
        c1, c2 = torch.empty(M, dtype=torch.float64, device="cuda"), torch.empty(M, dtype=torch.float64, device="cuda")
        n1, n2 = torch.empty(M, dtype=torch.uint8, device="cuda"), torch.empty(M, dtype=torch.uint8, device="cuda")
        g1, g2 = torch.zeros(A + 1, dtype=torch.int64, device="cuda"), torch.zeros(A + 1, dtype=torch.int64, device="cuda")
        K = (M + 63) // 64
        votes = torch.empty((K, A), dtype=torch.int64, device="cuda")
        words = torch.empty((2, K), dtype=torch.int64, device="cuda")
        N.check(L.bce_reestimate_consensus(N.ptr(Pt), A, M, M, N.ptr(w), N.ptr(c1), N.ptr(n1), st))
        N.check(L.bce_reestimate_agreement(N.ptr(Pt), A, M, M, N.ptr(c1), N.ptr(n1), N.ptr(g1[:A]), N.ptr(g1[A:]), st))
        N.check(L.bce_reestimate_consensus_votes(N.ptr(Pt), A, M, M, N.ptr(w), N.ptr(c2), N.ptr(n2), N.ptr(votes),
                                                 N.ptr(words[0]), N.ptr(words[1]), st))
        N.check(L.bce_reestimate_agreement_votes(N.ptr(votes), A, M, N.ptr(words[0]), N.ptr(words[1]),
                                                 N.ptr(g2[:A]), N.ptr(g2[A:]), st))
        torch.cuda.synchronize()
        assert torch.equal(n1, n2)
        assert np.array_equal(c1.cpu().numpy(), c2.cpu().numpy(), equal_nan=True)
        assert torch.equal(g1, g2), (w0, g1[-1].item(), g2[-1].item())
        # the vote bits themselves
        vb = votes.cpu().numpy().view(np.uint64)
        bits = ((vb[:, :, None] >> np.arange(64, dtype=np.uint64)) & np.uint64(1)).astype(bool)  # [K, A, 64]
        exp = np.zeros((K * 64, A), bool)
        exp[:M] = (P >= 0.5).T
        assert np.array_equal(bits.transpose(0, 2, 1).reshape(K * 64, A), exp)


def test_c4_replay_slice():
    """Config-4 replay through the fused replay_step kernel vs the reference trace."""
    import torch
    from bayesian_engine import batch
    g = load_npz("c4_replay.npz")
    pres = g["present"].copy()
    r = np.where(pres == 1, g["r0"], 0.5)
    c = np.where(pres == 1, g["c0"], 0.25)
    t = g["t0_us"].copy()
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    dr, dc, dt, dp = T(r), T(c), T(t), T(pres)
    view = torch.empty_like(dr)
    for k in range(g["flags"].shape[0]):
        now = int(g["now0_us"]) + k * int(g["step_us"])
        f = g["flags"][k]
        f2 = batch.pack_flags2((f & 1) == 1, (f & 2) == 2)
        batch.replay_step(dr, dc, dt, dp, T(f2), now, view)
        v = view.cpu().numpy()
        exp = g["views"][k]
        assert np.array_equal(v, exp), k
    fp = g["final_present"] == 1
    assert np.array_equal(dp.cpu().numpy() == 1, fp)
    assert np.array_equal(dr.cpu().numpy()[fp], g["final_r"][fp])
    assert np.array_equal(dc.cpu().numpy()[fp], g["final_c"][fp])


def _cli(args, stdin=None, cwd=None):
    env = dict(os.environ, PYTHONPATH=PKG)
    return subprocess.run([sys.executable, "-m", "bayesian_engine.cli"] + args, capture_output=True, text=True,
                          input=stdin, env=env, cwd=cwd, timeout=600)


def test_cli_cases_golden():
    fx = load_json("cli_cases.json")
    with tempfile.TemporaryDirectory() as d:
        for name, payload in fx["inputs"].items():
            with open(os.path.join(d, name), "w") as f:
                json.dump(payload, f)
        for case in fx["cases"]:
            p = _cli([a.replace("{DIR}", d) for a in case["args"]], stdin=case["stdin"], cwd=d)
            assert p.returncode == case["rc"], (case["args"], p.stderr)
            assert p.stdout == case["stdout"], case["args"]
            if case["rc"]:
                assert p.stderr.strip().splitlines()[-1] == case["stderr"].strip().splitlines()[-1]


def test_cli_dry_run_and_db_reliability():
    """Restates the reference's tests/test_dry_run.py flows."""
    with tempfile.TemporaryDirectory() as d:
        db = os.path.join(d, "t.db")
        p = _cli(["--db", db, "--dry-run", "report-outcome", "--source-id", "agent-a", "--market-id", "market-1",
                  "--correct"])
        out = json.loads(p.stdout)
        assert p.returncode == 0 and out["dryRun"] is True and out["reliability"] > 0.5
        assert json.loads(_cli(["--db", db, "list-sources"]).stdout)["count"] == 0
        assert json.loads(_cli(["--db", db, "--dry-run", "report-outcome", "--source-id", "a", "--market-id",
                                "m"]).stdout)["reliability"] < 0.5
        p = _cli(["--db", db, "report-outcome", "--source-id", "agent-a", "--market-id", "market-1", "--correct"])
        assert json.loads(p.stdout)["dryRun"] is False
        ls = json.loads(_cli(["--db", db, "list-sources", "--market-id", "market-1"]).stdout)
        assert ls["count"] == 1 and ls["sources"][0]["sourceId"] == "agent-a"
        payload = {"schemaVersion": "1.0.0", "marketId": "market-1",
                   "signals": [{"sourceId": "agent-a", "probability": 0.6}, {"sourceId": "agent-b", "probability": 0.4}]}
        p = _cli(["--db", db, "consensus"], stdin=json.dumps(payload))
        w = {x["sourceId"]: x["weight"] for x in json.loads(p.stdout)["sourceWeights"]}
        assert w["agent-a"] > w["agent-b"]


def _tb_inputs(lens, seed):
    rng = np.random.default_rng(seed)
    off = np.zeros(len(lens) + 1, np.int64)
    off[1:] = np.cumsum(lens)
    n = int(off[-1])
    kind = rng.integers(0, 6, n)
    pred = rng.random(n)
    pred = np.where(kind == 1, rng.integers(0, 9, n) / 8.0, pred)                        # exact binary grid
    pred = np.where(kind == 2, (rng.integers(-2000, 2000, n) + 0.5) * 10.0 ** rng.integers(-6, 4, n), pred)  # near-ties
    pred = np.where(kind == 3, rng.normal(0, 1e9, n), pred)                              # large magnitudes
    pred = np.where(kind == 4, rng.integers(-300, 300, n) * 50.0, pred)                  # multiples of 50
    pred[rng.random(n) < 0.02] = -0.0
    conf, weight, rel = rng.random(n), rng.choice([0.5, 1.0, 2.0], n), rng.choice([0.5, 0.9], n)
    return off, pred, conf, weight, rel


def _tb_check(r, exp, off):
    assert np.array_equal(r.winner.cpu().numpy(), exp["winner"])
    assert np.array_equal(r.label.cpu().numpy(), exp["label"])
    assert np.array_equal(r.n_groups.cpu().numpy(), exp["n_groups"])
    assert np.array_equal(r.variance.cpu().numpy(), exp["variance"])  # libm pow restated (glibc_pow.hpp)
    gk, gc, gd, gm = (r.g_key.cpu().numpy(), r.g_count.cpu().numpy(), r.g_density.cpu().numpy(),
                      r.g_maxrel.cpu().numpy())
    for m in range(len(off) - 1):
        a, g = int(off[m]), int(exp["n_groups"][m])
        sl = slice(a, a + g)
        assert np.array_equal(gk[sl], exp["g_key"][sl]), m
        assert np.array_equal(gc[sl], exp["g_count"][sl]), m
        assert np.array_equal(gd[sl], exp["g_total"][sl] / exp["g_count"][sl]), m
        assert np.array_equal(gm[sl], exp["g_maxrel"][sl]), m


@pytest.mark.parametrize("precision", [0, 2, 6, 10, 17, 22, -1, -2, -7, -15, 400, -400])
def test_tiebreak_any_precision_vs_python_round(precision):
    """Group keys are CPython round(pred, precision) (tiebreak.py:54) for any precision the
    reference accepts that the build restates: the oracle groups by Python's own round()."""
    import torch
    from bayesian_engine import batch
    from oracle import oracle as orc
    lens = np.array([40, 64, 2, 100, 700, 3], np.int64)
    off, pred, conf, weight, rel = _tb_inputs(lens, 1000 + precision)
    keys = np.array([round(float(x), precision) for x in pred], np.float64)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    r = batch.tiebreak(T(off), T(pred), T(conf), T(weight), T(rel), precision=precision, offsets_host=off)
    exp = orc.tiebreak_csr(off, pred, conf, weight, rel, keys=keys)
    _tb_check(r, exp, off)


def test_tiebreak_precision_30_is_supported():
    """precision=30 (10^30 is not a double) used to return BCE_EUNSUPPORTED; it now runs the
    exact big-integer round() like every other int precision (tiebreak.py:46-47,54)."""
    import torch
    from bayesian_engine import batch
    off, pred, conf, weight, rel = _tb_inputs(np.array([5, 6], np.int64), 3)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    r = batch.tiebreak(T(off), T(pred), T(conf), T(weight), T(rel), precision=30, offsets_host=off)
    torch.cuda.synchronize()
    gk = r.g_key.cpu().numpy()
    for m in range(2):
        a = int(off[m])
        first = round(float(pred[a]), 30)
        assert gk[a] == first


def test_tiebreak_markets_longer_than_4096_vs_oracle():
    """The reference has no length limit: 5000 and 12000 agents sort in a global scratch
    slice (4097 and shorter markets in the same batch)."""
    import torch
    from bayesian_engine import batch
    from oracle import oracle as orc
    lens = np.array([5000, 70, 12000, 4097, 1, 64], np.int64)
    off, pred, conf, weight, rel = _tb_inputs(lens, 77)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    for precision in (6, 2, 0, 10):
        keys = np.array([round(float(x), precision) for x in pred], np.float64)
        r = batch.tiebreak(T(off), T(pred), T(conf), T(weight), T(rel), precision=precision, offsets_host=off)
        exp = orc.tiebreak_csr(off, pred, conf, weight, rel, keys=keys)
        _tb_check(r, exp, off)


def test_tiebreak_int_predictions_keep_int_keys():
    """round(int, 6) is an int: the reference's group keys and winner are ints then."""
    from bayesian_engine.tiebreak import AgentSignal, DeterministicTieBreaker
    agents = [AgentSignal("a", 1, 0.9, 2.0, 0.9), AgentSignal("b", 0, 0.5, 1.0, 0.5),
              AgentSignal("c", 1.0, 0.7, 1.0, 0.6), AgentSignal("d", 0.25, 0.5, 1.0, 0.4)]
    pred, diag = DeterministicTieBreaker().resolve(agents)
    assert pred == 1 and type(pred) is int
    assert [type(k) for k in diag.groups] == [int, int, float]
    pred2, diag2 = DeterministicTieBreaker(precision=-1).resolve(agents)
    assert list(diag2.groups) == [0] and type(pred2) is int  # every prediction rounds to the tens: 0


def test_tiebreak_variance_bit_exact_1m_markets():
    """confidence_variance = round(sum((c - mean) ** 2) / n, 6) (tiebreak.py:108-110,149):
    ``** 2`` is libm pow, which differs from d*d for ~0.08% of d, so the kernels restate
    glibc's pow (csrc/glibc_pow.hpp).  1M markets of 2..64 agents with random confidences,
    plus markets whose confidences sit on a 2^-28 grid (every square an exact midpoint
    candidate, where glibc rounds ~18% of squares away from d*d): the raw variance equals
    the oracle's (libm pow) bit for bit, and so does round(variance, 6)."""
    import torch
    from bayesian_engine import batch
    from oracle import oracle as orc
    rng = np.random.default_rng(110)
    M = 1_000_000
    lens = rng.integers(2, 65, M).astype(np.int64)
    lens[:2000] = rng.integers(65, 300, 2000)  # the block kernel's path too
    off = np.zeros(M + 1, np.int64)
    off[1:] = np.cumsum(lens)
    n = int(off[-1])
    conf = rng.random(n)
    grid = np.repeat(rng.random(M) < 0.3, lens)
    conf[grid] = rng.integers(0, 1 << 28, int(grid.sum())) * 2.0 ** -28
    pred = rng.integers(0, 9, n) / 8.0
    weight, rel = rng.random(n), rng.random(n)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    r = batch.tiebreak(T(off), T(pred), T(conf), T(weight), T(rel), offsets_host=off)
    exp = orc.tiebreak_csr(off, pred, conf, weight, rel)
    got = r.variance.cpu().numpy()
    assert np.array_equal(got, exp["variance"])
    assert [round(float(x), 6) for x in got] == [round(float(x), 6) for x in exp["variance"]]
    # the case this test exists for: d*d would have differed somewhere in this batch
    dd = np.zeros(M)
    for m in range(0, M, 997):
        c = conf[off[m]:off[m + 1]]
        mu = sum(c.tolist()) / len(c)
        dd[m] = sum((x - mu) * (x - mu) for x in c.tolist()) / len(c)
    sel = np.arange(0, M, 997)
    assert np.any(dd[sel] != exp["variance"][sel]), "no market where d*d differs: test lost its teeth"


@pytest.mark.parametrize("A,M", [(5, 70), (17, 190), (300, 4097), (4100, 1000)])
def test_reestimate_mfma_fast_mode_matches_exact_votes(A, M):
    """mode="mfma" pass 1 on the matrix cores (bce_reestimate_consensus_votes_mfma):
    consensus within 4*A*2^-53 of the agent-order value (<= 1e-9), and -- because markets
    within 8*A*2^-53 of 0.5 (or with NaN cells) are redone in agent order -- vote bits, consensus votes,
    resolved masks, null flags and agreement counts identical to the exact pass.  Columns
    of mirrored pairs (x, 1-x) put the consensus at 0.5 up to rounding, so the redo runs."""
    import torch
    from bayesian_engine import _native as N
    rng = np.random.default_rng(A * 31 + M)
    P = rng.beta(2, 2, size=(A, M))
    mir = rng.random(M) < 0.2
    half = A // 2
    P[half:2 * half, mir] = 1.0 - P[:half, mir]
    if A % 2:
        P[-1, mir] = 0.5
    P[rng.random((A, M)) < 0.003] = np.nan
    Pt = torch.from_numpy(P).cuda()
    L = N.lib()
    st = N.stream(Pt.device)
    K = (M + 63) // 64
    nb = int(L.bce_reestimate_mfma_scratch_bytes(M))
    scratch = torch.empty((nb + 7) // 8, dtype=torch.int64, device="cuda")
    for wmode in ("half", "mixed", "zero"):
        w = torch.full((A,), 0.5, dtype=torch.float64, device="cuda")
        if wmode == "mixed":
            w = torch.from_numpy(rng.random(A)).cuda()
        elif wmode == "zero":
            w.zero_()
        out = []
        for fn in ("bce_reestimate_consensus_votes", "bce_reestimate_consensus_votes_mfma"):
            c = torch.empty(M, dtype=torch.float64, device="cuda")
            nu = torch.empty(M, dtype=torch.uint8, device="cuda")
            votes = torch.empty((K, A), dtype=torch.int64, device="cuda")
            words = torch.empty((2, K), dtype=torch.int64, device="cuda")
            g = torch.zeros(A + 1, dtype=torch.int64, device="cuda")
            extra = (N.ptr(scratch), scratch.numel() * 8) if fn.endswith("mfma") else ()
            N.check(getattr(L, fn)(N.ptr(Pt), A, M, M, N.ptr(w), N.ptr(c), N.ptr(nu), N.ptr(votes), N.ptr(words[0]),
                                   N.ptr(words[1]), *extra, st), fn)
            N.check(L.bce_reestimate_agreement_votes(N.ptr(votes), A, M, N.ptr(words[0]), N.ptr(words[1]),
                                                     N.ptr(g[:A]), N.ptr(g[A:]), st))
            torch.cuda.synchronize()
            out.append((c.cpu().numpy(), nu.cpu().numpy(), votes.cpu().numpy(), words.cpu().numpy(), g.cpu().numpy()))
        (ce, ne, ve, we, ge), (cf, nf, vf, wf, gf) = out
        assert np.array_equal(ne, nf) and np.array_equal(ve, vf) and np.array_equal(we, wf), wmode
        assert np.array_equal(ge, gf), wmode
        fin = np.isfinite(ce)
        assert np.array_equal(fin, np.isfinite(cf))
        dev = np.abs(cf[fin] - ce[fin])
        assert dev.max(initial=0.0) <= 4 * (A + 2) * 2.0 ** -53 and dev.max(initial=0.0) <= 1e-9, wmode
        near = fin & (np.abs(ce - 0.5) <= 4 * (A + 2) * 2.0 ** -53)
        assert np.array_equal(cf[near], ce[near])  # the redone markets are exact
        assert np.array_equal(np.isnan(cf), np.isnan(ce))  # NaN columns redone too


def _votes_both_modes(P, w):
    """(exact, mfma) outputs of one single-read iteration on the same P and weights."""
    import torch
    from bayesian_engine import _native as N
    A, M = P.shape
    Pt = P if isinstance(P, torch.Tensor) else torch.from_numpy(P).cuda()
    wt = w if isinstance(w, torch.Tensor) else torch.from_numpy(w).cuda()
    L = N.lib()
    st = N.stream(Pt.device)
    K = (M + 63) // 64
    nb = int(L.bce_reestimate_mfma_scratch_bytes(M))
    scratch = torch.empty((nb + 7) // 8, dtype=torch.int64, device="cuda")
    out = []
    for fn in ("bce_reestimate_consensus_votes", "bce_reestimate_consensus_votes_mfma"):
        c = torch.empty(M, dtype=torch.float64, device="cuda")
        nu = torch.empty(M, dtype=torch.uint8, device="cuda")
        votes = torch.empty((K, A), dtype=torch.int64, device="cuda")
        words = torch.empty((2, K), dtype=torch.int64, device="cuda")
        g = torch.zeros(A + 1, dtype=torch.int64, device="cuda")
        extra = (N.ptr(scratch), scratch.numel() * 8) if fn.endswith("mfma") else ()
        N.check(getattr(L, fn)(N.ptr(Pt), A, M, M, N.ptr(wt), N.ptr(c), N.ptr(nu), N.ptr(votes), N.ptr(words[0]),
                               N.ptr(words[1]), *extra, st), fn)
        N.check(L.bce_reestimate_agreement_votes(N.ptr(votes), A, M, N.ptr(words[0]), N.ptr(words[1]),
                                                 N.ptr(g[:A]), N.ptr(g[A:]), st))
        torch.cuda.synchronize()
        out.append((c.cpu().numpy(), nu.cpu().numpy(), votes.cpu().numpy(), words.cpu().numpy(), g.cpu().numpy()))
    return out


@pytest.mark.parametrize("wkind", ["negative", "nan", "inf", "neg_zero"])
def test_reestimate_mfma_weights_outside_precondition_fall_back_to_exact(wkind):
    """The MFMA order's error bound and null test assume finite w >= 0 (stats.hip).  Weights
    that break it make bce_reestimate_consensus_votes_mfma run the exact kernel (device-side
    check): every output identical to the exact pass, bit for bit.  -0.0 is >= 0 and stays
    on the MFMA path (consensus within the bound, votes identical)."""
    rng = np.random.default_rng(7)
    A, M = 300, 5000
    P = rng.beta(2, 2, size=(A, M))
    w = rng.random(A)
    if wkind == "negative":
        w[rng.random(A) < 0.3] *= -1.0  # mixed signs: totals can cancel
    elif wkind == "nan":
        w[17] = np.nan
    elif wkind == "inf":
        w[3] = np.inf
    else:
        w[::2] = -0.0
    (ce, ne, ve, we, ge), (cf, nf, vf, wf, gf) = _votes_both_modes(P, w)
    assert np.array_equal(ne, nf) and np.array_equal(ve, vf) and np.array_equal(we, wf)
    assert np.array_equal(ge, gf)
    if wkind == "neg_zero":
        assert np.abs(cf - ce).max() <= 4 * (A + 2) * 2.0 ** -53
    else:
        assert np.array_equal(cf, ce, equal_nan=True)


def test_reestimate_mfma_nan_cells_match_exact_without_redo_cliff():
    """10% NaN cells: every column holds a NaN, so every consensus is NaN in any order -- the
    MFMA pass must match exact (votes, words, counts) without redoing the columns one by one
    (it stays within 2x of the exact pass's time)."""
    import time
    import torch
    rng = np.random.default_rng(11)
    A, M = 2048, 65536
    P = rng.beta(2, 2, size=(A, M))
    P[rng.random((A, M)) < 0.1] = np.nan
    Pt = torch.from_numpy(P).cuda()
    w = torch.from_numpy(rng.random(A)).cuda()
    (ce, ne, ve, we, ge), (cf, nf, vf, wf, gf) = _votes_both_modes(Pt, w)
    assert np.array_equal(ne, nf) and np.array_equal(ve, vf) and np.array_equal(we, wf)
    assert np.array_equal(ge, gf)
    assert np.array_equal(np.isnan(cf), np.isnan(ce)) and np.isnan(ce).all()
    from bayesian_engine import batch
    times = {}
    for mode in ("exact", "mfma"):
        batch.reestimate(Pt, 1, mode=mode)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        batch.reestimate(Pt, 3, mode=mode)
        torch.cuda.synchronize()
        times[mode] = time.perf_counter() - t0
    assert times["mfma"] <= 2.0 * times["exact"], times


def test_reestimate_mfma_out_of_range_cells_redone_exactly():
    """Finite cells outside [0, 1] void the MFMA error bound: those columns are redone in agent
    order by the lane-per-market fixup kernel -- consensus bit-exact there, votes identical."""
    rng = np.random.default_rng(12)
    A, M = 1000, 20000
    P = rng.beta(2, 2, size=(A, M))
    odd = rng.random(M) < 0.3
    P[rng.integers(0, A, odd.sum()), np.nonzero(odd)[0]] = rng.uniform(-5, 5, odd.sum())
    w = rng.random(A)
    (ce, ne, ve, we, ge), (cf, nf, vf, wf, gf) = _votes_both_modes(P, w)
    assert np.array_equal(ne, nf) and np.array_equal(ve, vf) and np.array_equal(we, wf)
    assert np.array_equal(ge, gf)
    hit = odd & ((P < 0) | (P > 1)).any(axis=0)
    assert hit.sum() > 1000
    assert np.array_equal(cf[hit], ce[hit])


@pytest.mark.parametrize("nd", [23, 30, 100, 300, 323, -16, -100, -308])
def test_tiebreak_every_precision_matches_python_round(nd):
    """DeterministicTieBreaker(precision=nd) for the precisions whose 10^|nd| is not an exact
    double (tiebreak.py:46-47,54 accept any int): the EXOTIC kernels' big-integer round()
    against CPython's round() on random, tiny, subnormal and huge predictions, in markets of
    every kernel's length range (lane per market, wave per market, workgroup per market).
    All outputs bit-exact against the oracle fed Python's own round() keys."""
    import struct
    import torch
    from bayesian_engine import batch
    from oracle import oracle as orc
    rng = np.random.default_rng(500 + nd)
    lens = np.array([2, 5, 17, 32, 33, 48, 64, 65, 200, 31, 8] * 6, np.int64)
    off = np.zeros(len(lens) + 1, np.int64)
    off[1:] = np.cumsum(lens)
    n = int(off[-1])
    kind = rng.integers(0, 5, n)
    pred = rng.random(n)
    pred[kind == 1] = rng.random((kind == 1).sum()) * 10.0 ** rng.integers(-320, -5, (kind == 1).sum())
    sub = np.nonzero(kind == 2)[0]
    pred[sub] = [struct.unpack("<d", struct.pack("<q", int(b)))[0] for b in rng.integers(1, 1 << 52, len(sub))]
    pred[kind == 3] = rng.random((kind == 3).sum()) * 10.0 ** rng.integers(10, 300, (kind == 3).sum())
    pred[kind == 4] = np.round(rng.random((kind == 4).sum()) * 8) / 8.0  # forced ties
    pred[rng.random(n) < 0.3] *= -1.0
    if nd < 0:  # whole markets whose keys collapse to one multiple of 10^-nd
        pred[off[3]:off[4]] = 10.0 ** (-nd) * 3.0
    keys = np.array([round(float(p), nd) for p in pred])
    conf, weight, rel = rng.random(n), rng.random(n), rng.random(n)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    r = batch.tiebreak(T(off), T(pred), T(conf), T(weight), T(rel), precision=nd, offsets_host=off)
    torch.cuda.synchronize()
    exp = orc.tiebreak_csr(off, pred, conf, weight, rel, keys=keys)
    for k in ("winner", "label", "n_groups", "variance"):
        assert np.array_equal(getattr(r, k).cpu().numpy(), exp[k]), (nd, k)
    gk = r.g_key.cpu().numpy()
    for m in range(len(lens)):
        a, ng = int(off[m]), int(exp["n_groups"][m])
        assert gk[a:a + ng].tobytes() == exp["g_key"][a:a + ng].tobytes(), (nd, m)


def test_tiebreak_round_overflow_raises_like_cpython():
    """round(1.7e308, -308) is 2e308: CPython raises OverflowError ("rounded value too large
    to represent"); the batched tie-break raises the same error (device fault 6)."""
    import torch
    from bayesian_engine import batch
    with pytest.raises(OverflowError):
        round(1.7e308, -308)
    off = np.array([0, 3], np.int64)
    pred = np.array([0.5, 1.7e308, 0.25])
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    ones = np.ones(3)
    with pytest.raises(OverflowError, match="too large"):
        batch.tiebreak(T(off), T(pred), T(ones * 0.5), T(ones), T(ones * 0.5), precision=-308, offsets_host=off)
    # the fault word is cleared by the check: a valid call afterwards succeeds
    r = batch.tiebreak(T(off), T(pred[[0, 2, 0]]), T(ones * 0.5), T(ones), T(ones * 0.5), precision=-308,
                       offsets_host=off)
    torch.cuda.synchronize()
    assert float(r.winner[0].item()) == 0.0


@pytest.mark.parametrize("n_agents", [3, 40, 100])
def test_tiebreak_signed_zero_group_key_is_first_member(n_agents):
    """round(-1e-9, 6) is -0.0 and round(1e-9, 6) is 0.0: one dict slot (== compares them
    equal) whose key is the FIRST member's (tiebreak.py:54-55).  Every kernel (lane, wave and
    workgroup per market) reports that key's sign for the group and the winner."""
    import struct
    import torch
    from bayesian_engine import batch
    from oracle import oracle as orc
    rng = np.random.default_rng(n_agents)
    markets = []
    for first in (-1e-9, 1e-9, -0.0, 0.0):
        p = list(rng.choice([1e-9, -1e-9, 0.0, -0.0, 2e-9], n_agents - 1)) + []
        markets.append([first] + p)
    lens = np.array([len(m) for m in markets], np.int64)
    off = np.zeros(len(lens) + 1, np.int64)
    off[1:] = np.cumsum(lens)
    pred = np.concatenate(markets)
    n = len(pred)
    conf, weight, rel = rng.random(n), np.ones(n), np.ones(n)  # one group: it must win
    keys = np.array([round(float(p), 6) for p in pred])
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    r = batch.tiebreak(T(off), T(pred), T(conf), T(weight), T(rel), precision=6, offsets_host=off)
    torch.cuda.synchronize()
    exp = orc.tiebreak_csr(off, pred, conf, weight, rel, keys=keys)
    sign = lambda x: struct.pack("<d", float(x))[7] >> 7  # noqa: E731
    gk, win = r.g_key.cpu().numpy(), r.winner.cpu().numpy()
    for m in range(len(markets)):
        a = int(off[m])
        assert sign(gk[a]) == sign(keys[a]) == sign(exp["g_key"][a]), (m, gk[a], keys[a])
        assert sign(win[m]) == sign(exp["winner"][m]), (m, win[m], exp["winner"][m])


@pytest.mark.parametrize("precision", [6, 0, 2, 10, 22])
def test_tiebreak_full_tiles_vs_oracle(precision):
    """Tiles of 64 markets of exactly 32 agents run a kernel specialised for them
    (tiebreak_lpm_kernel PART 1: n a compile-time 32, selects instead of branches, the
    division by 10^precision as a reciprocal product with one FMA correction); every other
    tile runs the general body (PART 2).  A batch of both kinds -- full tiles around ragged
    ones, adversarial predictions (exact halves at the precision, -0.0, huge, NaN, inf),
    weights with 0 and inf -- matches the oracle bit for bit in every output, the group
    ordinals and per-group mean confidences included."""
    import torch
    from bayesian_engine import batch
    from oracle import oracle as orc
    rng = np.random.default_rng(900 + precision)
    lens = np.full(64 * 40, 32, np.int64)
    lens[64 * 17 + 5] = 31                        # one ragged tile among full ones
    lens[64 * 30:64 * 31] = rng.integers(0, 33, 64)  # a tile of mixed lengths, empty markets included
    off, pred, conf, weight, rel = _tb_inputs(lens, 4000 + precision)
    n = len(pred)
    half = (rng.integers(-5000, 5000, n) + 0.5) * 10.0 ** -precision  # exact ties at the precision
    pred = np.where(rng.random(n) < 0.1, half, pred)
    pred[rng.random(n) < 0.003] = np.nan
    pred[rng.random(n) < 0.003] = np.inf
    pred[rng.random(n) < 0.003] = -np.inf
    weight[rng.random(n) < 0.01] = 0.0
    weight[rng.random(n) < 0.002] = np.inf
    keys = np.array([round(float(x), precision) for x in pred], np.float64)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    r = batch.tiebreak(T(off), T(pred), T(conf), T(weight), T(rel), precision=precision, offsets_host=off)
    torch.cuda.synchronize()
    exp = orc.tiebreak_csr(off, pred, conf, weight, rel, keys=keys)
    for k in ("winner", "label", "n_groups", "variance"):
        assert getattr(r, k).cpu().numpy().tobytes() == exp[k].astype(getattr(r, k).cpu().numpy().dtype).tobytes(), k
    gk, gc, gd, ga, gm, go = (x.cpu().numpy() for x in (r.g_key, r.g_count, r.g_density, r.g_avgconf,
                                                          r.g_maxrel, r.g_of))
    with np.errstate(invalid="ignore"):
        dens = exp["g_total"] / np.maximum(exp["g_count"], 1)
    for m in range(len(lens)):
        a, b, g = int(off[m]), int(off[m + 1]), int(exp["n_groups"][m])
        if b == a:
            continue
        sl = slice(a, a + g)
        assert gk[sl].tobytes() == exp["g_key"][sl].tobytes(), m
        assert np.array_equal(gc[sl], exp["g_count"][sl]), m
        assert gd[sl].tobytes() == dens[sl].tobytes(), m
        assert ga[sl].tobytes() == exp["g_avgconf"][sl].tobytes(), m
        assert gm[sl].tobytes() == exp["g_maxrel"][sl].tobytes(), m
        uniq, ords = [], []
        for k in map(float, keys[a:b]):
            # first-seen ordinal under ==: -0.0 joins 0.0, a NaN key is never equal (own group)
            j = next((i for i, x in enumerate(uniq) if x == k), None)
            if j is None:
                uniq.append(k)
                j = len(uniq) - 1
            ords.append(j)
        assert list(go[a:b]) == ords, m


def test_tiebreak_max_len_skips_host_scan():
    """batch.tiebreak(max_len=L): the caller's bound replaces the host scan of the offsets
    (the bench's per-step path); outputs identical to the scanned call, and a market longer
    than the bound is reported by the device fault word, not silently truncated."""
    import torch
    from bayesian_engine import _native as N
    from bayesian_engine import batch
    lens = np.full(64 * 6, 32, np.int64)
    lens[100] = 7
    off, pred, conf, weight, rel = _tb_inputs(lens, 31)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    d = [T(off), T(pred), T(conf), T(weight), T(rel)]
    r1 = batch.tiebreak(*d, offsets_host=off)
    r2 = batch.tiebreak(*d, max_len=32)
    torch.cuda.synchronize()
    for k in ("winner", "label", "n_groups", "variance", "g_key", "g_count", "g_density", "g_avgconf",
              "g_maxrel", "g_of"):
        assert getattr(r1, k).cpu().numpy().tobytes() == getattr(r2, k).cpu().numpy().tobytes(), k
    N.check_faults(torch.device("cuda", 0), "max_len ok")
    lens = np.array([32, 40, 3], np.int64)
    off, pred, conf, weight, rel = _tb_inputs(lens, 32)
    batch.tiebreak(T(off), T(pred), T(conf), T(weight), T(rel), max_len=32)
    with pytest.raises(N.BCEError, match="longer than"):
        N.check_faults(torch.device("cuda", 0), "max_len too small")


def test_tiebreak_wave_kernel_reports_market_longer_than_64():
    """max_len=64 selects the wave-per-market kernel; a 100-agent market inside the batch is
    left with the empty marker and reported by the fault word -- never computed from wrapped
    lanes.  The 64-agent market beside it is still computed."""
    import torch
    from bayesian_engine import _native as N
    from bayesian_engine import batch
    lens = np.array([64, 100, 5], np.int64)
    off, pred, conf, weight, rel = _tb_inputs(lens, 33)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    r = batch.tiebreak(T(off), T(pred), T(conf), T(weight), T(rel), max_len=64)
    with pytest.raises(N.BCEError, match="longer than"):
        N.check_faults(torch.device("cuda", 0), "max_len 64, a 100-agent market")
    assert int(r.n_groups[1].item()) == -1 and int(r.label[1].item()) == -1
    assert int(r.n_groups[0].item()) >= 1 and int(r.n_groups[2].item()) >= 1


def test_tiebreak_exotic_single_agent_huge_prediction_does_not_raise():
    """precision -308 with a huge prediction alone in its market: the reference returns
    agents[0].prediction unrounded (tiebreak.py:89-96) and raises nothing, so the lane kernel
    must not report round()'s overflow for 1-agent (or empty) markets."""
    import torch
    from bayesian_engine import _native as N
    from bayesian_engine import batch
    off = np.array([0, 1, 3, 3], np.int64)  # a 1-agent market, a 2-agent market, an empty one
    pred = np.array([1.7e308, 0.5, 0.25])
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    ones = np.ones(3)
    r = batch.tiebreak(T(off), T(pred), T(ones * 0.5), T(ones), T(ones * 0.5), precision=-308, offsets_host=off)
    torch.cuda.synchronize()
    N.check_faults(torch.device("cuda", 0), "exotic precision, single huge agent")
    assert float(r.winner[0].item()) == 1.7e308
    assert float(r.winner[1].item()) == round(0.5, -308)


@pytest.mark.parametrize("precision", [6, 0, -2, 30])
def test_tiebreak_ragged_lane_kernel_vs_oracle(precision):
    """Markets of 0..32 agents (every tile ragged: the general lane-per-market body, PART 2 of
    the split launch or the only launch for the exotic precisions) with adversarial values:
    every output bit-exact against the oracle fed Python's own round() keys."""
    import torch
    from bayesian_engine import batch
    from oracle import oracle as orc
    rng = np.random.default_rng(1200 + precision)
    lens = rng.integers(0, 33, 64 * 24).astype(np.int64)
    off, pred, conf, weight, rel = _tb_inputs(lens, 1300 + precision)
    n = len(pred)
    pred = np.where(rng.random(n) < 0.1, (rng.integers(-500, 500, n) + 0.5) * 10.0 ** -max(precision, 0), pred)
    pred[rng.random(n) < 0.005] = np.nan
    weight[rng.random(n) < 0.01] = 0.0
    keys = np.array([round(float(x), precision) for x in pred], np.float64)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    r = batch.tiebreak(T(off), T(pred), T(conf), T(weight), T(rel), precision=precision, max_len=32)
    torch.cuda.synchronize()
    exp = orc.tiebreak_csr(off, pred, conf, weight, rel, keys=keys)
    for k in ("winner", "label", "n_groups", "variance"):
        got = getattr(r, k).cpu().numpy()
        assert got.tobytes() == exp[k].astype(got.dtype).tobytes(), k
    gk, gc, ga, gm = (x.cpu().numpy() for x in (r.g_key, r.g_count, r.g_avgconf, r.g_maxrel))
    for m in range(len(lens)):
        a, g = int(off[m]), int(exp["n_groups"][m])
        if lens[m] == 0:
            continue
        sl = slice(a, a + g)
        assert gk[sl].tobytes() == exp["g_key"][sl].tobytes(), m
        assert np.array_equal(gc[sl], exp["g_count"][sl]), m
        assert ga[sl].tobytes() == exp["g_avgconf"][sl].tobytes(), m
        assert gm[sl].tobytes() == exp["g_maxrel"][sl].tobytes(), m


@pytest.mark.parametrize("precision", [6, 0, -2, 30, -308])
def test_tiebreak_length_buckets_vs_oracle(precision):
    """batch.tiebreak_plan: a ragged batch of 0..32-agent markets bucketed by length (<= 8,
    9..16, 17..32) and run by the gather-staged kernels walking 8 / 16 / 32 positions per lane
    (tiebreak.hip GATHER), the bucket edges 8 / 9 / 16 / 17 / 32 and empty / single-agent
    markets included: every output bit-exact against the oracle, and identical to the
    contiguous-tile launch (max_len=32) on every defined slot.  Exotic precisions take the
    EXOTIC gather kernels."""
    import torch
    from bayesian_engine import _native as N
    from bayesian_engine import batch
    from oracle import oracle as orc
    rng = np.random.default_rng(2200 + precision)
    lens = rng.integers(0, 33, 64 * 30).astype(np.int64)
    lens[:12] = [0, 1, 2, 7, 8, 9, 15, 16, 17, 31, 32, 1]
    off, pred, conf, weight, rel = _tb_inputs(lens, 2300 + precision)
    n = len(pred)
    pred = np.where(rng.random(n) < 0.1, (rng.integers(-500, 500, n) + 0.5) * 10.0 ** -max(precision, 0), pred)
    pred[rng.random(n) < 0.005] = np.nan
    if precision <= -16:
        pred = np.clip(pred, -1e300, 1e300)  # keep round() finite: its overflow has its own test
    keys = np.array([round(float(x), precision) for x in pred], np.float64)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    d = [T(off), T(pred), T(conf), T(weight), T(rel)]
    plan = batch.tiebreak_plan(off, force=True)
    assert plan.buckets is not None and [hi for _, hi in plan.buckets] == [8, 16, 32]
    # the cost model buckets a large uniform 0..32 batch (since round 6's batched gather
    # staging) and a batch of short markets
    big = np.zeros(64001, np.int64)
    big[1:] = np.cumsum(rng.integers(0, 33, 64000))
    assert batch.tiebreak_plan(big).buckets is not None
    short = np.zeros(3001, np.int64)
    short[1:] = np.cumsum(rng.integers(0, 11, 3000))
    assert batch.tiebreak_plan(short).buckets is not None
    r = batch.tiebreak(*d, precision=precision, plan=plan)
    c = batch.tiebreak(*d, precision=precision, max_len=32)
    torch.cuda.synchronize()
    N.check_faults(torch.device("cuda", 0), "length buckets")
    exp = orc.tiebreak_csr(off, pred, conf, weight, rel, keys=keys)
    for k in ("winner", "label", "n_groups", "variance"):
        got = getattr(r, k).cpu().numpy()
        assert got.tobytes() == exp[k].astype(got.dtype).tobytes(), k
        assert got.tobytes() == getattr(c, k).cpu().numpy().tobytes(), k
    assert r.g_of.cpu().numpy()[:n].tobytes() == c.g_of.cpu().numpy()[:n].tobytes()
    ng = exp["n_groups"].astype(np.int64)
    ng[lens == 0] = 0
    pos = np.repeat(off[:-1], ng) + (np.arange(int(ng.sum())) - np.repeat(np.cumsum(ng) - ng, ng))
    for k in ("g_key", "g_count", "g_density", "g_avgconf", "g_maxrel"):
        got = getattr(r, k).cpu().numpy()[pos]
        assert got.tobytes() == getattr(c, k).cpu().numpy()[pos].tobytes(), k
        if k in exp:
            assert got.tobytes() == exp[k][pos].astype(got.dtype).tobytes(), k


def test_tiebreak_market_list_gather_bounds():
    """bce_tiebreak_csr with a market list and max_len 5 / 12 / 30 (the 8 / 16 / 32-position
    gather kernels): results identical to the whole-batch call for the listed markets, and a
    listed market longer than the bound is left with the empty marker and reported."""
    import torch
    from bayesian_engine import _native as N
    from bayesian_engine import batch
    rng = np.random.default_rng(77)
    lens = rng.integers(0, 33, 700).astype(np.int64)
    off, pred, conf, weight, rel = _tb_inputs(lens, 78)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    d = [T(off), T(pred), T(conf), T(weight), T(rel)]
    ref = batch.tiebreak(*d, max_len=32)
    L = N.lib()
    for bound in (5, 12, 30):
        sel = np.nonzero(lens <= bound)[0].astype(np.int32)
        r = batch.tiebreak(*d, max_len=32)  # fresh outputs, then overwrite the listed markets' rows
        for k in ("winner", "label", "n_groups", "variance"):
            getattr(r, k).fill_(-7)
        lst = T(sel)
        outs = [N.ptr(getattr(r, k)) for k in ("winner", "label", "n_groups", "variance", "g_key", "g_count",
                                               "g_density", "g_avgconf", "g_maxrel", "g_of")]
        rc = L.bce_tiebreak_csr(N.ptr(d[0]), len(lens), N.ptr(lst), len(sel), *[N.ptr(x) for x in d[1:]], bound, 6,
                                *outs, N.stream(d[0].device))
        assert rc == 0, L.bce_last_error()
        torch.cuda.synchronize()
        N.check_faults(torch.device("cuda", 0), f"list bound {bound}")
        for k in ("winner", "label", "n_groups", "variance"):
            assert getattr(r, k).cpu().numpy()[sel].tobytes() == getattr(ref, k).cpu().numpy()[sel].tobytes(), (bound, k)
    # arrays 8-B but not 16-B aligned: the per-lane row path, same results
    U = lambda a: torch.from_numpy(np.concatenate([[0.0], a])).cuda()[1:]  # noqa: E731
    du = [d[0], U(pred), U(conf), U(weight), U(rel)]
    sel = np.nonzero(lens <= 30)[0].astype(np.int32)
    r = batch.tiebreak(*d, max_len=32)
    outs = [N.ptr(getattr(r, k)) for k in ("winner", "label", "n_groups", "variance", "g_key", "g_count",
                                           "g_density", "g_avgconf", "g_maxrel", "g_of")]
    assert L.bce_tiebreak_csr(N.ptr(d[0]), len(lens), N.ptr(T(sel)), len(sel), *[N.ptr(x) for x in du[1:]], 30, 6,
                              *outs, N.stream(d[0].device)) == 0
    torch.cuda.synchronize()
    for k in ("winner", "label", "n_groups", "variance"):
        assert getattr(r, k).cpu().numpy()[sel].tobytes() == getattr(ref, k).cpu().numpy()[sel].tobytes(), k
    # a listed market longer than the bound
    sel = np.array([0, int(np.argmax(lens)), 1], np.int32)
    r = batch.tiebreak(*d, max_len=32)
    outs = [N.ptr(getattr(r, k)) for k in ("winner", "label", "n_groups", "variance", "g_key", "g_count",
                                           "g_density", "g_avgconf", "g_maxrel", "g_of")]
    assert L.bce_tiebreak_csr(N.ptr(d[0]), len(lens), N.ptr(T(sel)), 3, *[N.ptr(x) for x in d[1:]], 8, 6, *outs,
                              N.stream(d[0].device)) == 0
    with pytest.raises(N.BCEError, match="longer than"):
        N.check_faults(torch.device("cuda", 0), "list longer than its bound")
    assert int(r.n_groups[int(sel[1])].item()) == -1


@pytest.mark.parametrize("precision", [0, 1, 6, 15, 22])
def test_tiebreak_full_tiles_round_edges(precision):
    """The FULL kernel's round(): rint of x * 10^p, an exact redo only for flagged halves, and
    k / 10^p as a reciprocal product with one FMA correction.  Full tiles of predictions at the
    edges -- exact decimal halves, values one ulp either side of them, magnitudes around the
    threshold past which round() returns x itself, subnormals, +-0.0 -- give the group keys
    Python's round() gives, bit for bit."""
    import math
    import torch
    from bayesian_engine import batch
    from oracle import oracle as orc
    rng = np.random.default_rng(700 + precision)
    M = 64 * 12
    n = M * 32
    scale = 10.0 ** precision
    k = rng.integers(-10**6, 10**6, n).astype(np.float64)
    halves = (k + 0.5) / scale
    pred = halves.copy()
    sel = rng.random(n)
    pred = np.where(sel < 0.2, np.nextafter(halves, np.inf), pred)
    pred = np.where((sel >= 0.2) & (sel < 0.4), np.nextafter(halves, -np.inf), pred)
    E = math.floor(52.0 - precision * 3.321928094887362) + 1  # the restatement's threshold 2^E
    big = np.ldexp(1.0, E) * rng.uniform(0.5, 2.0, n) * np.where(rng.random(n) < 0.5, -1.0, 1.0)
    pred = np.where((sel >= 0.4) & (sel < 0.55), big, pred)
    pred = np.where((sel >= 0.55) & (sel < 0.6), rng.random(n) * 1e-310, pred)     # subnormal
    pred = np.where((sel >= 0.6) & (sel < 0.63), -0.0, pred)
    pred = np.where((sel >= 0.63) & (sel < 0.7), rng.random(n), pred)
    # repeat some values inside markets so groups form
    dup = rng.random(n) < 0.25
    pred[dup] = pred[np.maximum(np.nonzero(dup)[0] - 1, 0)]
    off = np.arange(0, n + 1, 32, dtype=np.int64)
    conf, weight, rel = rng.random(n), rng.random(n), rng.random(n)
    keys = np.array([round(float(x), precision) for x in pred], np.float64)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    r = batch.tiebreak(T(off), T(pred), T(conf), T(weight), T(rel), precision=precision, max_len=32)
    torch.cuda.synchronize()
    exp = orc.tiebreak_csr(off, pred, conf, weight, rel, keys=keys)
    for key in ("winner", "label", "n_groups", "variance"):
        got = getattr(r, key).cpu().numpy()
        assert got.tobytes() == exp[key].astype(got.dtype).tobytes(), key
    gk = r.g_key.cpu().numpy()
    for m in range(M):
        a, g = int(off[m]), int(exp["n_groups"][m])
        assert gk[a:a + g].tobytes() == exp["g_key"][a:a + g].tobytes(), m


def test_tiebreak_plan_declines_decreasing_offsets():
    """a market with a negative length (decreasing offsets) in a batch of
    <= 32-agent markets is not dropped by the length buckets: tiebreak_plan declines to bucket
    and the contiguous lane kernel records the device fault."""
    import torch
    from bayesian_engine import _native as N
    from bayesian_engine import batch
    lens = np.full(64 * 8, 5, np.int64)
    off, pred, conf, weight, rel = _tb_inputs(lens, 4242)
    assert batch.tiebreak_plan(off, force=True).buckets is not None
    bad = off.copy()
    bad[100] = bad[99] - 2  # market 99 has length -2, market 100 a longer one
    assert batch.tiebreak_plan(bad, force=True).buckets is None
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    N.check_faults(torch.device("cuda", 0), "clean slate")
    batch.tiebreak(T(bad), T(pred), T(conf), T(weight), T(rel))
    with pytest.raises(N.BCEError):
        N.check_faults(torch.device("cuda", 0), "decreasing offsets")
