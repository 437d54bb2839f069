"""CPU tests of the host-side logic around the kernels (no GPU needed)."""
import json
import os
import subprocess
import sys
from datetime import datetime, timedelta, timezone

import numpy as np
import pytest

from golden_util import load_json

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "bayesian-consensus-engine_amd")


def test_iso_to_us_matches_reference_days():
    from bayesian_engine.decay import days_since_update
    from bayesian_engine.timeutil import NO_TIMESTAMP, iso_to_us
    d = load_json("decay_cases.json")
    for stamp, now_us, days in d["days"]:
        now = datetime(1970, 1, 1, tzinfo=timezone.utc) + timedelta(microseconds=now_us)
        assert days_since_update(stamp, now=now) == days
        t = iso_to_us(stamp)
        if days == 0.0 and t != NO_TIMESTAMP:
            assert t >= now_us - 0  # future or same instant
    assert iso_to_us(None) == NO_TIMESTAMP and iso_to_us("") == NO_TIMESTAMP
    assert iso_to_us("garbage") == NO_TIMESTAMP


def test_validation_structural_errors_without_gpu():
    from bayesian_engine.core import ValidationError, validate_input_payload
    for case in load_json("validate_cases.json"):
        p = case["payload"]
        sig = p.get("signals")
        needs_gpu = isinstance(sig, list) and any(
            isinstance(s, dict) and isinstance(s.get("probability"), (int, float)) for s in sig[:1])
        if needs_gpu or case["error"] is None:
            continue
        with pytest.raises(ValidationError) as ei:
            validate_input_payload(p)
        assert str(ei.value) == case["error"], case["name"]


def test_compute_consensus_empty_is_host_only():
    from bayesian_engine.core import compute_consensus
    exp = [c for c in load_json("consensus_cases.json") if c["name"] == "empty"][0]["expected"]
    assert compute_consensus([]) == exp


def test_intern_is_python_sorted_order():
    from bayesian_engine.batch import intern
    ids = ["éclair", "Zeta", "alpha", "中文", "\U0001f600x", "_u", "Alpha", "Ａf", "a", "퟿"]
    r = intern(ids)
    assert [k for k, _ in sorted(r.items(), key=lambda kv: kv[1])] == sorted(set(ids))


def test_pack_flags2_layout():
    from bayesian_engine.batch import pack_flags2
    rng = np.random.default_rng(1)
    S = 1001
    p = rng.random(S) < 0.3
    c = rng.random(S) < 0.5
    f = pack_flags2(p, c)
    assert len(f) == (S + 3) // 4
    for s in range(S):
        bits = (f[s // 4] >> (2 * (s % 4))) & 3
        assert bits == (int(p[s]) | (int(c[s]) << 1))


def test_shard_markets_balanced_and_complete():
    from bayesian_engine.sharding import shard_markets
    rng = np.random.default_rng(2)
    lens = rng.integers(1, 4097, 5000)
    off = np.zeros(len(lens) + 1, np.int64)
    off[1:] = np.cumsum(lens)
    for world in (1, 2, 3, 8):
        ranges = [shard_markets(off, world, r) for r in range(world)]
        assert ranges[0][0] == 0 and ranges[-1][1] == len(lens)
        for (a0, a1), (b0, b1) in zip(ranges, ranges[1:]):
            assert a1 == b0
        sig = [off[b] - off[a] for a, b in ranges]
        assert max(sig) - min(sig) <= 2 * 4096 + 1


def test_owner_of_stable_and_spread():
    from bayesian_engine.sharding import owner_of
    o = owner_of(np.arange(100000), 8)
    assert o.min() == 0 and o.max() == 7
    counts = np.bincount(o, minlength=8)
    assert counts.min() > 0.9 * counts.mean()
    assert np.array_equal(o, owner_of(np.arange(100000), 8))


def test_agent_signal_validation_and_host_shortcuts():
    from bayesian_engine.tiebreak import AgentSignal, DeterministicTieBreaker
    with pytest.raises(ValueError, match="confidence must be in"):
        AgentSignal("a", 0.5, 1.5)
    with pytest.raises(ValueError, match="reliability_score must be in"):
        AgentSignal("a", 0.5, 0.5, 1.0, -0.1)
    with pytest.raises(ValueError, match="empty agent list"):
        DeterministicTieBreaker().resolve([])
    pred, diag = DeterministicTieBreaker().resolve([AgentSignal("a1", 0.75, 0.8)])
    assert pred == 0.75 and diag.method == "single_agent" and diag.tie_resolved_by == "unanimous"
    assert diag.confidence_variance == 0.0 and diag.groups == {0.75: {"count": 1}}


def test_market_metadata_host():
    from bayesian_engine.market import CrossMarketAggregator, Market, MarketId, MarketStatus, MarketStore
    assert MarketId("crypto:btc:1").category == "crypto"
    assert MarketId("simple").category is None
    assert MarketId("a:b:c").parts == ["a", "b", "c"]
    assert MarketId("crypto:btc:1").matches("crypto:*")
    with pytest.raises(ValueError):
        MarketId(" ")
    m = Market(id=MarketId("t"), status=MarketStatus.CLOSED)
    with pytest.raises(ValueError):
        m.add_signal({"sourceId": "a", "probability": 0.5})
    store = MarketStore()
    store.create_market(MarketId("x:1"))
    with pytest.raises(ValueError):
        store.create_market(MarketId("x:1"))
    assert store.compute_all_consensus() == {"x:1": {"schemaVersion": "1.0.0", "consensus": None,
                                                     "confidence": 0.0, "marketId": "x:1"}}
    assert CrossMarketAggregator(store).summarize_sources() == {}
    assert CrossMarketAggregator(store).summarize_category("x")["total_markets"] == 1


def test_dropin_api_surface():
    """Every public name the reference's callers and tests use."""
    import bayesian_engine
    from bayesian_engine import cli, config, core, decay, market, reliability, tiebreak
    assert bayesian_engine.__version__ == "0.1.0"
    for mod, names in {
        core: ["ValidationError", "validate_input_payload", "compute_consensus", "SCHEMA_VERSION"],
        decay: ["compute_decay_factor", "apply_reliability_decay", "days_since_update",
                "decay_reliability_if_needed"],
        reliability: ["ReliabilityRecord", "SQLiteReliabilityStore", "DEFAULT_CONFIDENCE", "DEFAULT_RELIABILITY",
                      "MAX_UPDATE_STEP"],
        tiebreak: ["AgentSignal", "DeterministicTieBreaker", "TieBreakDiagnostics"],
        market: ["MarketId", "MarketStatus", "Market", "MarketStore", "CrossMarketAggregator",
                 "SourcePerformance"],
        cli: ["main"],
        config: ["DEFAULT_RELIABILITY", "DEFAULT_CONFIDENCE", "MAX_UPDATE_STEP", "TIE_TOLERANCE",
                 "DECAY_HALF_LIFE_DAYS", "DECAY_MINIMUM", "SCHEMA_VERSION", "MIN_SOURCE_ID_LENGTH",
                 "MAX_SOURCE_ID_LENGTH", "MAX_SIGNALS_PER_REQUEST"],
    }.items():
        for n in names:
            assert hasattr(mod, n), (mod.__name__, n)
    assert (config.DEFAULT_RELIABILITY, config.DEFAULT_CONFIDENCE, config.MAX_UPDATE_STEP) == (0.5, 0.25, 0.1)
    assert (config.DECAY_HALF_LIFE_DAYS, config.DECAY_MINIMUM, config.SCHEMA_VERSION) == (30, 0.1, "1.0.0")
    assert config.TIE_TOLERANCE == 1e-9 and config.MAX_SIGNALS_PER_REQUEST == 1000


def test_sqlite_store_host_paths(tmp_path):
    from bayesian_engine.reliability import ReliabilityRecord, SQLiteReliabilityStore
    db = tmp_path / "r.db"
    with SQLiteReliabilityStore(db) as s:
        rec = s.get_reliability("ghost", "m")
        assert rec == ReliabilityRecord("ghost", "m", 0.5, 0.25, "")
        assert s.list_sources() == []
    import sqlite3
    c = sqlite3.connect(str(db))
    assert c.execute("SELECT name FROM sqlite_master WHERE type='table' AND name='sources'").fetchone()
    c.close()
    with pytest.raises(AttributeError):
        rec.reliability = 0.9


def test_cli_config1_matches_reference_stdout():
    """BASELINE.json configs[0]: examples/sample_input.json via --dry-run (empty signals)."""
    fx = load_json("cli_cases.json")
    case = fx["cases"][0]
    assert case["args"][0] == "--dry-run"
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        with open(os.path.join(d, "sample_input.json"), "w") as f:
            json.dump(fx["inputs"]["sample_input.json"], f)
        args = [a.replace("{DIR}", d) for a in case["args"]]
        env = dict(os.environ, PYTHONPATH=PKG)
        p = subprocess.run([sys.executable, "-m", "bayesian_engine.cli"] + args, capture_output=True, text=True,
                           env=env, timeout=300)
    assert p.returncode == case["rc"] == 0
    assert p.stdout == case["stdout"]


def test_glibc_pow2_restatement_matches_libm(tmp_path):
    """csrc/glibc_pow.hpp restates this libm's pow(x, 2.0) (the tie-break variance's
    `(c - mean) ** 2`, tiebreak.py:110) and pow(2.0, y) (the decay factor, decay.py:58) bit
    for bit: 4M inputs each incl. exact-midpoint squares, subnormals, huge and underflowing
    values, decay exponents from float and integer-microsecond elapsed times
    (tools/pow2_check.cpp)."""
    import subprocess
    exe = str(tmp_path / "pow2_check")
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-DBCE_POW_HOST_TEST", "-w",
                    "-I", os.path.join(ROOT, "bayesian-consensus-engine_amd", "csrc"),
                    os.path.join(ROOT, "tools", "pow2_check.cpp"), "-o", exe, "-lm"], check=True)
    out = subprocess.run([exe, "1000000"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout
    f = {t.split("=")[0]: int(t.split("=")[1]) for t in out.stdout.split()}
    assert f["tested"] > 3_900_000 and f["mismatches"] == 0
    assert f["d_mul_differs"] > 1000  # d*d alone would not do: libm's pow is not correctly rounded
    # pow(2.0, y) of the decay factor (decay.py:58) too: bit-exact where exp2 is not
    assert f["pow2_tested"] > 3_900_000 and f["pow2_mismatches"] == 0
    assert f["exp2_differs"] > 100


def _py_round_host(x, nd):
    import ctypes as C
    from bayesian_engine import _native as N
    o = C.c_int32(0)
    r = N.lib().bce_debug_py_round(float(x), int(nd), C.byref(o))
    return r, bool(o.value)


def _ref_round(x, nd):
    try:
        return round(x, nd), False
    except OverflowError:
        return None, True


@pytest.mark.parametrize("nd", [23, 24, 30, 53, 100, 200, 300, 322, 323, -16, -17, -22, -23, -100, -200, -300, -307,
                                -308, 1, 6, 17, 22, -1, -5, -15])
def test_big_integer_round_matches_cpython(nd):
    """tiebreak.py:54 round(prediction, precision) for the precisions whose 10^|nd| is not an
    exact double: the exact big-integer restatement (py_round_big.hpp, the code the EXOTIC
    tie-break kernels run) against CPython's round() on random, subnormal, tie and huge
    values, bit for bit (including -0.0 and OverflowError)."""
    import math
    import struct
    rng = np.random.default_rng(1000 + nd)
    xs = list(rng.random(300))
    xs += list(rng.random(200) * 10.0 ** rng.integers(-320, 300, 200))
    bits = rng.integers(1, 1 << 52, 200, dtype=np.int64)
    xs += [struct.unpack("<d", struct.pack("<q", int(b)))[0] for b in bits]  # subnormals
    xs += [5e-324, 2.5e-323, 1e-300, 1e-200, 1e-30, 1e-24, 1.5e-23, 0.5, 0.125, 1.0, 2.5, 1e22, 1e23,
           5e15, 4e15, 1.5e16, 2.5e16, 1e300, 1.7976931348623157e308, 8.98846567431158e307, 0.0, -0.0,
           3.5e307, 4.5e307, 5e307, 1.0000000000000002, 0.1, 0.3]
    # exact decimal ties at this precision: k + 1/2 units of 10^-nd where representable
    if 0 < nd <= 330:
        xs += [float(f"{k}.5e-{nd}") for k in range(0, 40)]
    if nd < 0:
        xs += [float(f"{k}.5e{-nd}") for k in range(0, 40)]
    xs = [float(x) for x in xs]  # Python floats: numpy's own round() is not CPython's
    xs += [-x for x in xs]
    bad = []
    for x in xs:
        got, govf = _py_round_host(x, nd)
        exp, eovf = _ref_round(x, nd)
        if eovf or govf:
            if eovf != govf:
                bad.append((x, got, exp, govf, eovf))
            continue
        same = (struct.pack("<d", got) == struct.pack("<d", exp)) or (math.isnan(got) and math.isnan(exp))
        if not same:
            bad.append((x, got, exp))
    assert not bad, bad[:5]


def test_markstein_quotients_match_ieee_division(tmp_path):
    """The tie-break FULL kernel's divisions without a divide (tiebreak.hip tb_div_small,
    bce_device.hpp py_round_nd_sel): RN(x * RN(1/c)) with one FMA correction equals the IEEE
    quotient -- for k / 10^nd (integer k < 2^53, nd 0..22) and for x / c (c = 1..32, |x| in
    [2^-1000, 2^1000]).  tools/check_markstein.c at 1/100 of its full sample (the full run,
    3.1e9 quotients, is recorded in DESIGN.md §4.9)."""
    import shutil
    import subprocess
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    exe = tmp_path / "check_markstein"
    src = os.path.join(os.path.dirname(__file__), "..", "tools", "check_markstein.c")
    subprocess.run([cc, "-O2", "-ffp-contract=off", "-o", str(exe), src, "-lm"], check=True)
    out = subprocess.run([str(exe), "100"], check=True, capture_output=True, text=True).stdout
    assert out.strip().startswith("0 of "), out


def test_tiebreak_plan_buckets_by_measured_tile_costs():
    """batch.tiebreak_plan (host only): buckets of <= 8 / 9..16 / 17..32 agents exactly when
    they cost less than contiguous tiles by the measured per-tile costs (profiles/r06gb/): a
    uniform 1..32 ragged batch and a batch of short markets are bucketed, a uniform 32 batch
    stays contiguous, a batch with a market past 32 agents is never bucketed; every market lands
    in exactly one bucket."""
    import torch
    from bayesian_engine import batch
    rng = np.random.default_rng(5)
    cpu = torch.device("cpu")

    def off(lens):
        o = np.zeros(len(lens) + 1, np.int64)
        o[1:] = np.cumsum(lens)
        return o

    assert batch.tiebreak_plan(off(rng.integers(1, 33, 20000)), cpu).buckets is not None
    assert batch.tiebreak_plan(off(np.full(20000, 32)), cpu).buckets is None
    assert batch.tiebreak_plan(off(rng.integers(20, 33, 20000)), cpu).buckets is None  # mostly long
    assert batch.tiebreak_plan(off(np.append(rng.integers(0, 5, 1000), 33)), cpu).buckets is None
    lens = rng.integers(0, 13, 20000)
    p = batch.tiebreak_plan(off(lens), cpu)
    assert p.buckets is not None
    seen = np.concatenate([b.numpy() for b, _ in p.buckets])
    assert np.array_equal(np.sort(seen), np.arange(len(lens)))
    for b, hi in p.buckets:
        assert lens[b.numpy()].max() <= hi
    forced = batch.tiebreak_plan(off(rng.integers(1, 33, 500)), cpu, force=True)
    assert [hi for _, hi in forced.buckets] == [8, 16, 32]
