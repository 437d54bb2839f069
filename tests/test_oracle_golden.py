"""Pin the CPU oracle (oracle/bce_oracle.c) to golden vectors generated from the reference.

CPU-only.  Every comparison is bit-exact (Python == on floats), matching the reference's
own golden test (tests/test_golden_fixtures.py:48-60 in the reference).
"""
import math

import numpy as np
import pytest

from golden_util import case_to_csr, load_json, load_npz, same_float
from oracle import oracle as orc


def _check_case(case):
    exp = case["expected"]
    names, offsets, sid, prob, rel, conf, present = case_to_csr(case["signals"], case["source_reliability"])
    out = orc.consensus_csr(offsets, sid, prob, rel, conf, present)
    if not case["signals"]:
        assert exp["diagnostics"]["status"] == "no_signals"
        assert out["total_weight"][0] == 0.0 and out["n_unique"][0] == 0
        return
    u = int(out["n_unique"][0])
    assert u == exp["diagnostics"]["uniqueSources"] == exp["normalization"]["sourceCount"]
    tot = float(out["total_weight"][0])
    assert same_float(tot, exp["normalization"]["totalWeight"])
    if exp["consensus"] is None:
        assert tot == 0
    else:
        assert same_float(float(out["consensus"][0]), exp["consensus"])
    assert same_float(float(out["confidence"][0]), exp["confidence"])
    cold = []
    for j, sw in enumerate(exp["sourceWeights"]):
        us = int(out["usid"][j])
        assert names[us & 0x7FFFFFFF] == sw["sourceId"]
        assert float(out["weight"][j]) == float(sw["weight"])
        assert same_float(float(out["nweight"][j]), sw["normalizedWeight"])
        if us < 0:
            cold.append(sw["sourceId"])
    assert cold == exp["diagnostics"]["coldStartSources"]


@pytest.mark.parametrize("case", load_json("consensus_cases.json"), ids=lambda c: c["name"])
def test_consensus_cases(case):
    _check_case(case)


@pytest.mark.parametrize("name", ["c2_slice.npz", "c3_slice.npz"])
def test_consensus_csr_slices(name):
    g = load_npz(name)
    out = orc.consensus_csr(g["offsets"], g["sid"], g["prob"], g["rel"], g["conf"], g["present"])
    M = len(g["offsets"]) - 1
    assert np.array_equal(out["n_unique"], g["n_unique"])
    assert np.array_equal(out["err_idx"], g["err_idx"])
    null = out["total_weight"] == 0
    assert np.array_equal(null.astype(np.uint8), g["is_null"])
    for k in ("consensus", "confidence", "total_weight"):
        assert np.array_equal(out[k], g[k], equal_nan=True), k
    for m in range(M):
        a, u = int(g["offsets"][m]), int(g["n_unique"][m])
        sl = slice(a, a + u)
        us = out["usid"][sl]
        assert np.array_equal(us & 0x7FFFFFFF, g["usid"][sl])
        assert np.array_equal((us < 0).astype(np.uint8), g["cold"][sl])
        assert np.array_equal(out["weight"][sl], g["weight"][sl])
        assert np.array_equal(out["nweight"][sl], g["nweight"][sl], equal_nan=True)


def test_decay_factor_and_apply():
    d = load_json("decay_cases.json")
    for e, h, f in d["factor"]:
        assert orc.decay_factor(e, h) == f
    for r, e, h, m, v in d["apply"]:
        assert orc.apply_decay(r, e, h, m) == v


def test_days_since():
    from bayesian_engine.timeutil import iso_to_us  # host-side ISO parser (product host code)
    d = load_json("decay_cases.json")
    for stamp, now_us, days in d["days"]:
        t = iso_to_us(stamp)
        assert orc.days_since(now_us, t) == days, stamp


def test_update_traces():
    for tr in load_json("update_traces.json"):
        if tr["start"] == "cold":
            r, c, present = np.array([0.5]), np.array([0.25]), np.array([0], np.uint8)
        else:
            r, c, present = np.array([tr["start"][0]]), np.array([tr["start"][1]]), np.array([1], np.uint8)
        t = np.array([0], np.int64)
        for st in tr["steps"]:
            flags = np.array([1 | (2 if st["correct"] else 0)], np.uint8)
            nr, nc, nt, npres = orc.outcome_update(r, c, t, present, flags, 0)
            assert nr[0] == st["reliability"] and nc[0] == st["confidence"]
            if not st.get("dry_run"):
                r, c, t, present = nr, nc, nt, npres


def test_round_decimal():
    for x in [0.0078125, 0.1234565, 0.1234575, -1e-7, 1e-7, 0.5, 2.5e-6, -0.0, 1.0000005, 0.9999995]:
        assert orc.round_decimal(x, 6) == round(x, 6)
    rng = np.random.default_rng(0)
    for x in rng.random(20000):
        assert orc.round_decimal(x, 6) == round(float(x), 6)
    for k in rng.integers(0, 10**7, 20000):  # exact-half-ish cases
        x = (int(k) + 0.5) / 1e6
        assert orc.round_decimal(x, 6) == round(x, 6)


def test_tiebreak_cases():
    label_names = {0: "unanimous", 1: "weight_density", 2: "prediction_value_smallest", 3: "unanimous"}
    for case in load_json("tiebreak_cases.json"):
        ag = case["agents"]
        offsets = np.array([0, len(ag)], np.int64)
        pred, conf, weight, rel = (np.array([a[i] for a in ag], np.float64) for i in (1, 2, 3, 4))
        out = orc.tiebreak_csr(offsets, pred, conf, weight, rel)
        assert out["winner"][0] == case["winner"]
        assert label_names[int(out["label"][0])] == case["tie_resolved_by"]
        assert (out["label"][0] == 3) == (case["method"] == "single_agent")
        if len(ag) > 1:
            assert round(float(out["variance"][0]), 6) == case["confidence_variance"]
            ng = int(out["n_groups"][0])
            assert ng == len(case["raw_groups"])
            for j, (key, m) in enumerate(case["raw_groups"]):
                assert out["g_key"][j] == key
                assert out["g_count"][j] == m["count"]
                assert out["g_total"][j] == m["total_weight"]
                assert out["g_avgconf"][j] == m["avg_confidence"]
                assert out["g_maxrel"][j] == m["max_reliability"]


def test_summarize_counts():
    for case in load_json("summarize_cases.json"):
        names = sorted({s["sourceId"] for mk in case["markets"] for s in mk["signals"]})
        idx = {n: i for i, n in enumerate(names)}
        offsets, sid, prob, outcome = [0], [], [], []
        for mk in case["markets"]:
            for s in mk["signals"]:
                sid.append(idx[s["sourceId"]])
                prob.append(float(s.get("probability", 0.5)))
            offsets.append(len(sid))
            outcome.append(-1 if not mk["resolved"] else int(mk["outcome"]))
        correct, total = orc.agreement_stats(np.array(offsets), np.array(sid), np.array(prob),
                                             np.array(outcome), max(len(names), 1))
        for n, e in case["expected"].items():
            i = idx[n]
            assert total[i] == e["total"] and correct[i] == e["correct"]
            assert total[i] - correct[i] == e["wrong"]
        seen = {n for n in case["expected"]}
        for n in names:
            if n not in seen:
                assert total[idx[n]] == 0


def test_c4_replay():
    g = load_npz("c4_replay.npz")
    r, c, t, pres = g["r0"].copy(), g["c0"].copy(), g["t0_us"].copy(), g["present"].copy()
    r = np.where(pres == 1, r, 0.5)
    c = np.where(pres == 1, c, 0.25)
    T = g["flags"].shape[0]
    for k in range(T):
        now = int(g["now0_us"]) + k * int(g["step_us"])
        view = orc.decay_view(r, t, pres, now)
        assert np.array_equal(view, g["views"][k]), k
        r, c, t, pres = orc.outcome_update(r, c, t, pres, g["flags"][k], now)
    fp = g["final_present"] == 1
    assert np.array_equal(pres == 1, fp)
    assert np.array_equal(r[fp], g["final_r"][fp])
    assert np.array_equal(c[fp], g["final_c"][fp])
    upd = fp & (g["final_t_us"] != orc.NO_TIMESTAMP)
    assert np.array_equal(t[upd], g["final_t_us"][upd])


def test_c5_reestimate():
    g = load_npz("c5_reestimate.npz")
    K = int(g["iters"])
    w, cons, null, agree = orc.reestimate(g["P"], K)
    assert np.array_equal(null, g["is_null"])
    assert np.array_equal(cons, g["consensus"])
    assert np.array_equal(agree, g["agree"])
    assert np.array_equal(w, g["weights"][-1])


def test_oracle_tiebreak_variance_is_cpython_pow():
    """tiebreak.py:108-110 evaluates `sum((c - mean_conf) ** 2 for c in ...) / n` with
    CPython's float ** (libm pow, not d*d).  The oracle must reproduce it bit for bit on
    markets whose confidences sit on a 2^-28 grid, where pow and d*d disagree most often
    (GCC folds a literal pow(x, 2.0) into x*x, so the oracle calls libm through a pointer)."""
    rng = np.random.default_rng(110)
    M = 4000
    lens = rng.integers(2, 65, M)
    off = np.zeros(M + 1, np.int64)
    off[1:] = np.cumsum(lens)
    n = int(off[-1])
    conf = rng.integers(0, 1 << 28, n) * 2.0 ** -28
    pred = rng.integers(0, 9, n) / 8.0
    e = orc.tiebreak_csr(off, pred, conf, rng.random(n), rng.random(n))
    differs = 0
    for m in range(M):
        c = conf[off[m]:off[m + 1]].tolist()
        mean_conf = sum(c) / len(c)
        v = sum((x - mean_conf) ** 2 for x in c) / len(c)  # the reference's expression
        assert v == e["variance"][m], m
        differs += v != sum((x - mean_conf) * (x - mean_conf) for x in c) / len(c)
    assert differs > 5  # the case matters: d*d would have failed this test
