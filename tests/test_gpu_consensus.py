"""GPU parity: batched consensus kernels vs the oracle and the reference's golden vectors.

Bit-exact in BCE_MODE_EXACT (Python == on every float); BCE_MODE_FAST
(tree sums for long markets) within the north-star tolerance 1e-9 absolute.
"""
import numpy as np
import pytest
import torch

from golden_util import case_to_csr, load_json, load_npz
from oracle import oracle as orc

pytestmark = pytest.mark.gpu


def _dev(a, dt=None):
    return torch.from_numpy(np.ascontiguousarray(a if dt is None else a.astype(dt))).cuda()


def _run(g, mode="exact", max_len=None, plan=True):
    from bayesian_engine import batch
    table = batch.SourceTable.from_arrays(_dev(g["rel"]), _dev(g["conf"]), _dev(g["present"]))
    off = _dev(g["offsets"])
    r = batch.consensus(off, _dev(g["sid"], np.int32), _dev(g["prob"]), table, mode=mode,
                        max_len=max_len, plan=None)
    torch.cuda.synchronize()
    return {k: (getattr(r, k).cpu().numpy() if getattr(r, k) is not None else None)
            for k in ("consensus", "confidence", "total_weight", "n_unique", "err_idx", "usid", "weight",
                      "nweight")}


def _compare(out, exp, offsets, exact=True, tol=1e-9):
    M = len(offsets) - 1
    assert np.array_equal(out["n_unique"], exp["n_unique"])
    assert np.array_equal(out["err_idx"], exp["err_idx"])
    for k in ("consensus", "confidence", "total_weight"):
        if exact:
            assert np.array_equal(out[k], exp[k], equal_nan=True), k
        else:
            np.testing.assert_allclose(out[k], exp[k], rtol=0, atol=tol)
    for m in range(M):
        a, u = int(offsets[m]), int(exp["n_unique"][m])
        sl = slice(a, a + u)
        assert np.array_equal(out["usid"][sl], exp["usid"][sl]), m
        assert np.array_equal(out["weight"][sl], exp["weight"][sl]), m
        if exact:
            assert np.array_equal(out["nweight"][sl], exp["nweight"][sl], equal_nan=True), m
        else:
            np.testing.assert_allclose(out["nweight"][sl], exp["nweight"][sl], rtol=0, atol=tol)


@pytest.mark.parametrize("name", ["c2_slice.npz", "c3_slice.npz"])
def test_slices_vs_oracle_and_reference(name):
    g = load_npz(name)
    exp = orc.consensus_csr(g["offsets"], g["sid"], g["prob"], g["rel"], g["conf"], g["present"])
    out = _run(g)
    _compare(out, exp, g["offsets"])
    # and straight against the reference's own outputs captured in the fixture
    assert np.array_equal(out["consensus"], g["consensus"], equal_nan=True)
    assert np.array_equal(out["err_idx"], g["err_idx"])


def test_c2_direct_launch_max_len():
    g = load_npz("c2_slice.npz")
    exp = orc.consensus_csr(g["offsets"], g["sid"], g["prob"], g["rel"], g["conf"], g["present"])
    _compare(_run(g, max_len=32), exp, g["offsets"])


def test_c3_fast_mode_tolerance():
    g = load_npz("c3_slice.npz")
    exp = orc.consensus_csr(g["offsets"], g["sid"], g["prob"], g["rel"], g["conf"], g["present"])
    _compare(_run(g, mode="fast"), exp, g["offsets"], exact=False)


@pytest.mark.parametrize("L,S,M", [(1, 5, 3000), (7, 3, 500), (8, 1000, 4000), (13, 20, 2000), (16, 10000, 3000),
                                   (31, 40, 1000), (32, 10000, 5000), (33, 100, 700), (64, 64, 1000),
                                   (64, 100000, 800), (65, 30, 100), (500, 200, 40), (4096, 5000, 6),
                                   (5000, 3000, 3), (9000, 20000, 2)])
def test_random_uniform_lengths(L, S, M):
    rng = np.random.default_rng(L * 1000 + S)
    sid = rng.integers(0, S, M * L).astype(np.int32)
    prob = rng.random(M * L)
    prob[rng.random(M * L) < 0.01] = 1.25
    off = np.arange(0, M * L + 1, L, dtype=np.int64)
    rel = rng.uniform(0, 1, S)
    conf = rng.random(S)
    present = (rng.random(S) < 0.7).astype(np.uint8)
    rel[present == 0] = 0.5
    conf[present == 0] = 0.25
    g = dict(offsets=off, sid=sid, prob=prob, rel=rel, conf=conf, present=present)
    exp = orc.consensus_csr(off, sid, prob, rel, conf, present)
    _compare(_run(g), exp, off)


def test_ragged_with_empty_and_huge_markets():
    rng = np.random.default_rng(7)
    lens = np.concatenate([[0, 0, 1, 64, 65, 4096, 4097, 0, 12000], rng.integers(0, 300, 400)])
    rng.shuffle(lens)
    off = np.zeros(len(lens) + 1, np.int64)
    off[1:] = np.cumsum(lens)
    S = 3000
    n = int(off[-1])
    sid = (rng.zipf(1.3, n) % S).astype(np.int32)
    prob = rng.random(n)
    rel = rng.uniform(0, 1, S)
    conf = rng.random(S)
    present = (rng.random(S) < 0.8).astype(np.uint8)
    g = dict(offsets=off, sid=sid, prob=prob, rel=rel, conf=conf, present=present)
    exp = orc.consensus_csr(off, sid, prob, rel, conf, present)
    _compare(_run(g), exp, off)


@pytest.mark.parametrize("case", load_json("consensus_cases.json"), ids=lambda c: c["name"])
def test_single_market_cases(case):
    if not case["signals"]:
        pytest.skip("empty market handled on host (core.py:88-96)")
    names, offsets, sid, prob, rel, conf, present = case_to_csr(case["signals"], case["source_reliability"])
    g = dict(offsets=offsets, sid=sid, prob=prob, rel=rel, conf=conf, present=present)
    exp = orc.consensus_csr(offsets, sid, prob, rel, conf, present)
    _compare(_run(g), exp, offsets)


def _compare_vec(out, exp, offsets, exact=True, tol=1e-9):
    """Vectorised comparison (large M): per-unique slots j < n_unique only.  Bit-exact, or
    (exact=False, BCE_MODE_FAST) within the north-star tolerance on the reduced outputs;
    usid / weight are bit-exact in both modes."""
    for k in ("n_unique", "err_idx"):
        assert np.array_equal(out[k], exp[k]), k
    for k in ("consensus", "confidence", "total_weight"):
        if exact:
            assert np.array_equal(out[k], exp[k], equal_nan=True), k
        else:
            np.testing.assert_allclose(out[k], exp[k], rtol=0, atol=tol, equal_nan=True, err_msg=k)
    M = len(offsets) - 1
    u = exp["n_unique"].astype(np.int64)
    pos = np.repeat(offsets[:-1], u) + (np.arange(int(u.sum())) - np.repeat(np.cumsum(u) - u, u))
    for k in ("usid", "weight", "nweight"):
        if exact or k != "nweight":
            assert np.array_equal(out[k][pos], exp[k][pos], equal_nan=True), k
        else:
            np.testing.assert_allclose(out[k][pos], exp[k][pos], rtol=0, atol=tol, equal_nan=True, err_msg=k)
    assert M == len(u)


def test_many_tiles_per_wave():
    """6M tiny markets (> 64 tiles per wave of the persistent short-market kernels)."""
    rng = np.random.default_rng(11)
    M, S = 6_000_000, 1000
    lens = rng.integers(0, 3, M)
    off = np.zeros(M + 1, np.int64)
    off[1:] = np.cumsum(lens)
    n = int(off[-1])
    sid = rng.integers(0, S, n).astype(np.int32)
    prob = rng.random(n)
    rel, conf = rng.uniform(0, 1, S), rng.random(S)
    present = (rng.random(S) < 0.8).astype(np.uint8)
    g = dict(offsets=off, sid=sid, prob=prob, rel=rel, conf=conf, present=present)
    exp = orc.consensus_csr(off, sid, prob, rel, conf, present)
    _compare_vec(_run(g, max_len=2), exp, off)


@pytest.mark.parametrize("maxlen,S,M,seed", [(32, 10000, 20000, 1), (32, 7, 3000, 2), (16, 500, 9000, 3),
                                             (8, 20000, 5000, 4), (31, 100, 4000, 5), (3, 3, 7000, 6)])
def test_short_ragged_unaligned(maxlen, S, M, seed):
    """Ragged lengths 0..maxlen (odd offsets, empty markets, duplicates) on the contiguous
    short-market path, with an offset view (offsets[0] != 0) like a shard."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, maxlen + 1, M)
    lens[rng.random(M) < 0.05] = 0
    base = 13
    off = np.zeros(M + 1, np.int64)
    off[1:] = np.cumsum(lens)
    off += base
    n = int(off[-1])
    sid = rng.integers(0, S, n).astype(np.int32)
    prob = rng.random(n)
    prob[rng.random(n) < 0.02] = -0.5
    prob[rng.random(n) < 0.01] = np.nan
    rel, conf = rng.uniform(-0.2, 1, S), rng.random(S)
    rel[rng.random(S) < 0.05] = 0.0
    present = (rng.random(S) < 0.7).astype(np.uint8)
    g = dict(offsets=off, sid=sid, prob=prob, rel=rel, conf=conf, present=present)
    exp = orc.consensus_csr(off, sid, prob, rel, conf, present)
    _compare_vec(_run(g, max_len=maxlen), exp, off)


def _c2_like(M, S, seed, L=32, base=0):
    rng = np.random.default_rng(seed)
    sid = rng.integers(0, S, M * L).astype(np.int32)
    prob = rng.random(M * L)
    prob[rng.random(M * L) < 0.003] = 1.5
    off = np.arange(0, M * L + 1, L, dtype=np.int64) + base
    sid = np.concatenate([np.zeros(base, np.int32), sid])
    prob = np.concatenate([np.zeros(base), prob])
    rel = rng.uniform(0.1, 1.0, S)
    conf = rng.random(S)
    present = (rng.random(S) < 0.9).astype(np.uint8)
    rel[present == 0] = 0.5
    conf[present == 0] = 0.25
    return dict(offsets=off, sid=sid, prob=prob, rel=rel, conf=conf, present=present)


@pytest.mark.parametrize("S", [10000, 10112, 10113, 12000, 16384, 20000, 100000, 262144, 262145, 1000000])
def test_c2_shape_every_table_size(S):
    """n = 32 contiguous markets: LDS-table kernel (S <= 10112), hybrid LDS + global table
    (S <= 2^18: the first ~10k rows in LDS beside the whole bitmask), pipe kernel beyond
    (present bits from global memory past 16384 sources) -- all bit-exact, all eight outputs."""
    g = _c2_like(20000, S, S)
    exp = orc.consensus_csr(g["offsets"], g["sid"], g["prob"], g["rel"], g["conf"], g["present"])
    _compare_vec(_run(g, max_len=32), exp, g["offsets"])


@pytest.mark.parametrize("kind", ["extreme_in_range", "outside_range"])
def test_c2_normalized_weight_division_paths(kind):
    """LDS-table kernel with table weights spread over the whole exponent range (totals
    that overflow the range of their terms' magnitudes), and tables holding tiny, huge,
    negative, -0.0 and NaN weights: every output bit-exact against the oracle.  (Kept from
    a measured-and-dropped reciprocal-based normalizedWeight division)"""
    g = _c2_like(20000, 9000, 77 if kind == "extreme_in_range" else 78)
    rng = np.random.default_rng(5)
    S = len(g["rel"])
    if kind == "extreme_in_range":
        g["rel"] = np.ldexp(rng.random(S) + 0.5, rng.integers(-399, 399, S))
        g["rel"][rng.random(S) < 0.3] = np.ldexp(1.0, 399)  # totals of several of these leave the range
        g["rel"][rng.random(S) < 0.05] = 0.0
    else:
        pick = rng.random(S)
        g["rel"][pick < 0.02] = 1e-200
        g["rel"][(pick >= 0.02) & (pick < 0.04)] = -0.3
        g["rel"][(pick >= 0.04) & (pick < 0.05)] = -0.0
        g["rel"][(pick >= 0.05) & (pick < 0.06)] = 1e200
        g["rel"][(pick >= 0.06) & (pick < 0.061)] = np.nan
    g["present"][:] = 1
    exp = orc.consensus_csr(g["offsets"], g["sid"], g["prob"], g["rel"], g["conf"], g["present"])
    _compare_vec(_run(g, max_len=32), exp, g["offsets"])


@pytest.mark.parametrize("S,L,base", [(10000, 32, 0), (10000, 32, 4), (10000, 32, 1), (12000, 32, 0),
                                      (30000, 32, 0), (5000, 16, 0), (40000, 8, 3)])
def test_compact_mode(S, L, base):
    """unique_outputs=False (usid/weight/nweight NULL): per-market outputs only, on every
    contiguous short-market kernel; offset views with aligned and unaligned bases."""
    from bayesian_engine import batch
    g = _c2_like(9000, S, S + L, L=L, base=base)
    exp = orc.consensus_csr(g["offsets"], g["sid"], g["prob"], g["rel"], g["conf"], g["present"])
    table = batch.SourceTable.from_arrays(_dev(g["rel"]), _dev(g["conf"]), _dev(g["present"]))
    r = batch.consensus(_dev(g["offsets"]), _dev(g["sid"], np.int32), _dev(g["prob"]), table, max_len=L,
                        unique_outputs=False)
    torch.cuda.synchronize()
    assert r.usid is None and r.weight is None and r.nweight is None
    for k in ("n_unique", "err_idx"):
        assert np.array_equal(getattr(r, k).cpu().numpy(), exp[k]), k
    for k in ("consensus", "confidence", "total_weight"):
        assert np.array_equal(getattr(r, k).cpu().numpy(), exp[k], equal_nan=True), k


def test_tab_kernel_mixed_regular_and_ragged_tiles():
    """Mostly 32-signal markets with a few short ones and empty ones scattered: regular
    tiles take the transposed path, the others the per-lane path, same results."""
    rng = np.random.default_rng(21)
    M, S = 30000, 9000
    lens = np.full(M, 32)
    lens[rng.integers(0, M, 40)] = rng.integers(0, 32, 40)
    off = np.zeros(M + 1, np.int64)
    off[1:] = np.cumsum(lens)
    n = int(off[-1])
    sid = rng.integers(0, S, n).astype(np.int32)
    prob = rng.random(n)
    rel, conf = rng.uniform(0, 1, S), rng.random(S)
    present = (rng.random(S) < 0.8).astype(np.uint8)
    g = dict(offsets=off, sid=sid, prob=prob, rel=rel, conf=conf, present=present)
    exp = orc.consensus_csr(off, sid, prob, rel, conf, present)
    _compare_vec(_run(g, max_len=32), exp, off)


@pytest.mark.parametrize("S", [1, 2, 7, 40])
def test_tab_kernel_heavy_duplicates(S):
    """Tiny tables: nearly every market is all duplicates (many averaging / compaction
    rounds per wave, runs of up to 32)."""
    g = _c2_like(6000, S, 100 + S)
    exp = orc.consensus_csr(g["offsets"], g["sid"], g["prob"], g["rel"], g["conf"], g["present"])
    _compare_vec(_run(g, max_len=32), exp, g["offsets"])


def test_fault_word_reports_bad_sid_and_long_market():
    from bayesian_engine import _native as N, batch
    g = _c2_like(3000, 500, 5)
    table = batch.SourceTable.from_arrays(_dev(g["rel"]), _dev(g["conf"]), _dev(g["present"]))
    N.check_faults()  # clean
    sid = g["sid"].copy()
    sid[777] = 500  # == n_sources
    batch.consensus(_dev(g["offsets"]), _dev(sid, np.int32), _dev(g["prob"]), table, max_len=32)
    with pytest.raises(N.BCEError, match="n_sources"):
        N.check_faults()
    N.check_faults()  # the word was cleared
    off = g["offsets"].copy()
    off[10] += 5  # market 9 has 37 signals, launched as max_len 32
    batch.consensus(_dev(off), _dev(g["sid"], np.int32), _dev(g["prob"]), table, max_len=32)
    with pytest.raises(N.BCEError, match="max_len"):
        N.check_faults()


@pytest.mark.parametrize("mode", ["exact", "fast"])
def test_fault_word_wide_kernel(mode):
    """The wide kernel (64 < n <= 4096) reports a bad sid and a market longer than the
    launch's max_len; batch.consensus(check=True) raises it directly."""
    from bayesian_engine import _native as N, batch
    rng = np.random.default_rng(77)
    lens = rng.integers(65, 900, 50)
    off = np.zeros(len(lens) + 1, np.int64)
    off[1:] = np.cumsum(lens)
    S = 3000
    sid = rng.integers(0, S, off[-1]).astype(np.int32)
    prob = rng.random(off[-1])
    table = batch.SourceTable.from_arrays(_dev(rng.random(S)), _dev(rng.random(S)), _dev(np.ones(S, np.uint8)))
    N.check_faults()
    bad = sid.copy()
    bad[int(off[7]) + 3] = S + 5
    with pytest.raises(N.BCEError, match="n_sources"):
        batch.consensus(_dev(off), _dev(bad, np.int32), _dev(prob), table, max_len=1024, mode=mode, check=True)
    N.check_faults()  # cleared
    # markets of 900 > 512: launched as one wide launch sized for 512
    L = N.lib()
    d_off, d_sid, d_prob = _dev(off), _dev(sid, np.int32), _dev(prob)
    res = batch._alloc(len(lens), int(off[-1]), d_off.device, True, True)
    rc = L.bce_consensus_csr(N.ptr(d_off), len(lens), N.ptr(d_sid), N.ptr(d_prob), int(off[-1]),
                             N.ptr(table.relconf), N.ptr(table.bits), table.n, N.ptr(None), 0, 512,
                             N.MODE_FAST if mode == "fast" else N.MODE_EXACT, N.ptr(res.consensus),
                             N.ptr(res.confidence), N.ptr(res.total_weight), N.ptr(res.n_unique),
                             N.ptr(res.err_idx), N.ptr(res.usid), N.ptr(res.weight), N.ptr(res.nweight),
                             N.stream(d_off.device))
    assert rc == 0
    with pytest.raises(N.BCEError, match="max_len"):
        N.check_faults()


def test_pipe_kernel_spin_cap_reports_fault():
    """A persistent wave that exhausts its bounded wait records a fault instead of silently
    leaving its tiles unwritten (forced with a tiny cap on the pipe kernel: markets of 16,
    which the LDS-table kernel does not take)."""
    from bayesian_engine import _native as N, batch
    L = N.lib()
    g = _c2_like(50000, 12000, 9, L=16)
    table = batch.SourceTable.from_arrays(_dev(g["rel"]), _dev(g["conf"]), _dev(g["present"]))
    args = (_dev(g["offsets"]), _dev(g["sid"], np.int32), _dev(g["prob"]), table)
    N.check_faults()
    try:
        N.check(L.bce_debug_set_spin_cap(1))
        batch.consensus(*args, max_len=16)
        with pytest.raises(N.BCEError, match="timed out"):
            N.check_faults()
    finally:
        L.bce_debug_set_spin_cap(0)
    exp = orc.consensus_csr(g["offsets"], g["sid"], g["prob"], g["rel"], g["conf"], g["present"])
    _compare_vec(_run(g, max_len=16), exp, g["offsets"])
    N.check_faults()


@pytest.mark.parametrize("S", [12000, 40000])
def test_c2_hybrid_table_ragged_and_compact(S):
    """Hybrid LDS/global table on irregular tiles (lengths 17..32, duplicates, cold sources,
    a shard that starts mid-batch) and in compact mode (no per-unique outputs): bit-exact."""
    from bayesian_engine import batch
    rng = np.random.default_rng(S)
    M = 5000
    lens = rng.integers(17, 33, M)
    off = np.zeros(M + 1, np.int64)
    off[1:] = np.cumsum(lens)
    n = int(off[-1])
    hot = rng.integers(0, S, 64)
    sid = np.where(rng.random(n) < 0.3, hot[rng.integers(0, 64, n)], rng.integers(0, S, n)).astype(np.int32)
    prob = rng.random(n)
    rel, conf = rng.uniform(0.1, 1.0, S), rng.random(S)
    present = (rng.random(S) < 0.8).astype(np.uint8)
    rel[present == 0], conf[present == 0] = 0.5, 0.25
    g = dict(offsets=off, sid=sid, prob=prob, rel=rel, conf=conf, present=present)
    exp = orc.consensus_csr(off, sid, prob, rel, conf, present)
    _compare_vec(_run(g, max_len=32), exp, off)
    table = batch.SourceTable.from_arrays(_dev(rel), _dev(conf), _dev(present))
    r = batch.consensus(_dev(off), _dev(sid), _dev(prob), table, max_len=32, unique_outputs=False, check=True)
    for k in ("consensus", "confidence", "total_weight", "n_unique", "err_idx"):
        assert np.array_equal(getattr(r, k).cpu().numpy(), exp[k], equal_nan=True), k
