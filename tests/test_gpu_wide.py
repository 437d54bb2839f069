"""GPU parity for the wide-market kernel (64 < n <= 4096) vs the oracle.

consensus_wide_kernel<NW, R> packs (sid, input index) into 32 bits, so these cases sit on
its edges: every length bin boundary, Zipf-heavy duplicate runs (C3's source law), one
source for a whole 4096-signal market, the largest table the packed key allows
(S = 2^20 at P = 4096) and past it (64-bit keys: up to 16M sources in every bin), NaN /
out-of-range probabilities and non-positive reliabilities.  Bit-exact (==) in
BCE_MODE_EXACT; BCE_MODE_FAST (fixed-order tree totals) within 1e-9 absolute on consensus,
confidence, total weight and normalizedWeight, bit-exact on everything else.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as orc
from test_gpu_consensus import _compare_vec, _dev, _run

pytestmark = pytest.mark.gpu


def test_lane_exchange_selftest():
    """The wide kernel's VALU lane exchanges (DPP rotations/mirrors, v_permlane16/32_swap)
    and its DPP wave scan, checked lane by lane before any sort runs on them."""
    from bayesian_engine import _native as N
    out = torch.zeros(13 * 64, dtype=torch.int32, device="cuda")
    N.check(N.lib().bce_debug_lane_selftest(N.ptr(out), N.stream(out.device)))
    torch.cuda.synchronize()
    o = out.cpu().numpy().astype(np.int64).reshape(13, 64)
    lane = np.arange(64)
    for q, M in enumerate([1, 2, 3, 4, 7, 8, 15, 16, 31, 32, 63]):
        assert np.array_equal(o[q], lane ^ M), (M, o[q].tolist())
    assert np.array_equal(o[11], (lane + 1) * (lane + 2) // 2), o[11].tolist()
    assert o[12][0] == 0 and np.array_equal(o[12][1:], lane[1:] + 99), o[12].tolist()


def _zipf_case(lens, S, seed, a=1.1, base=0, bad=True):
    rng = np.random.default_rng(seed)
    off = np.zeros(len(lens) + 1, np.int64)
    off[1:] = np.cumsum(lens)
    off += base
    n = int(off[-1])
    perm = rng.permutation(S).astype(np.int32)
    z = rng.zipf(a, n)
    sid = perm[(z - 1) % S]
    prob = rng.random(n)
    if bad:
        prob[rng.random(n) < 0.001] = 1.5
        prob[rng.random(n) < 0.001] = np.nan
    rel = rng.uniform(-0.1, 1.0, S)
    conf = rng.random(S)
    present = (rng.random(S) < 0.8).astype(np.uint8)
    return dict(offsets=off, sid=sid, prob=prob, rel=rel, conf=conf, present=present)


def _check(g, mode="exact", **kw):
    exp = orc.consensus_csr(g["offsets"], g["sid"], g["prob"], g["rel"], g["conf"], g["present"])
    _compare_vec(_run(g, mode=mode, **kw), exp, g["offsets"], exact=(mode == "exact"))


EDGES = [65, 127, 128, 129, 255, 256, 257, 511, 512, 513, 1023, 1024, 1025, 1535, 1536, 1537, 2047, 2048, 2049,
         3071, 3072, 3073, 4095, 4096]


MODES = ["exact", "fast"]


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("S,seed", [(1_000_000, 1), (5000, 2), (40, 3)])
def test_wide_bins_zipf(S, seed, mode):
    rng = np.random.default_rng(100 + seed)
    lens = np.exp(rng.uniform(np.log(65), np.log(4096), 400)).astype(np.int64)
    lens = np.concatenate([lens, EDGES, [0, 3, 64]])
    rng.shuffle(lens)
    _check(_zipf_case(lens, S, seed, base=7), mode)


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("S", [1, 2])
def test_wide_single_long_run(S, mode):
    """All 4096 signals on one or two sources: run sums of thousands of terms."""
    _check(_zipf_case(np.array([4096, 4000, 3000, 2048, 1500, 700, 300, 100]), S, 5, bad=False), mode)


def test_wide_fast_mode_c3_shaped():
    """A generated C3-shaped batch (log-uniform lengths 1..4096, Zipf 1.1 over 1M sources,
    ~2M signals) in BCE_MODE_FAST against the oracle's reference-order sums."""
    rng = np.random.default_rng(303)
    lens = np.floor(np.exp(rng.uniform(0, np.log(4097), 4000))).astype(np.int64)
    g = _zipf_case(lens, 1_000_000, 303, bad=False)
    _check(g, "fast")
    out = _run(g, mode="fast")
    # deterministic: a second launch reproduces every bit
    again = _run(g, mode="fast")
    for k in ("consensus", "confidence", "total_weight", "nweight"):
        assert np.array_equal(out[k], again[k], equal_nan=True), k


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("top", [1536, 3072])
def test_wide_non_power_of_two_bins_direct(top, mode):
    """bce_consensus_csr with max_len 1536 / 3072 launches the 3- / 6-wave kernels whose
    sort network has missing +inf waves (every market at most `top` long, hot sources,
    NaN and out-of-range probabilities, empty markets)."""
    rng = np.random.default_rng(top)
    lens = rng.integers(top // 2 + 1, top + 1, 150)
    lens[:6] = [top, top - 1, top // 2 + 1, 0, 65, 1]
    g = _zipf_case(lens, 300_000, top, base=5)
    _check(g, mode, max_len=top)


def test_wide_key_limit_and_fallback():
    """S = 2^20 is the largest table the 32-bit key takes at P = 4096 (top sid at the last
    index); S = 2^20 + 1 sends the 2049..4096 bin to the 64-bit-key instantiation."""
    for S in (1 << 20, (1 << 20) + 1):
        lens = np.array([4096, 4096, 3000, 2500, 2048, 1000, 200])
        g = _zipf_case(lens, S, 9, a=1.05)
        g["sid"][int(g["offsets"][1]) - 1] = S - 1
        g["sid"][int(g["offsets"][0])] = S - 1
        _check(g)
        _check(g, "fast")


@pytest.mark.parametrize("mode", MODES)
def test_wide_nweight_without_weight_output(mode):
    """normalizedWeight requested without the weight output (w[j] parked in LDS instead of
    read back from the weight array)."""
    from bayesian_engine import _native as N, batch
    rng = np.random.default_rng(31)
    lens = rng.integers(65, 4097, 60)
    g = _zipf_case(lens, 50000, 31, bad=False)
    exp = orc.consensus_csr(g["offsets"], g["sid"], g["prob"], g["rel"], g["conf"], g["present"])
    table = batch.SourceTable.from_arrays(_dev(g["rel"]), _dev(g["conf"]), _dev(g["present"]))
    M, n = len(lens), int(g["offsets"][-1])
    off, sid, prob = _dev(g["offsets"]), _dev(g["sid"], np.int32), _dev(g["prob"])
    res = batch._alloc(M, n, off.device, True, True)
    L = N.lib()
    rc = L.bce_consensus_csr(N.ptr(off), M, N.ptr(sid), N.ptr(prob), n, N.ptr(table.relconf), N.ptr(table.bits),
                             table.n, N.ptr(None), 0, int(lens.max()), N.MODE_FAST if mode == "fast" else N.MODE_EXACT,
                             N.ptr(res.consensus), N.ptr(res.confidence), N.ptr(res.total_weight), N.ptr(res.n_unique),
                             N.ptr(res.err_idx), N.ptr(res.usid), N.ptr(None), N.ptr(res.nweight), N.stream(off.device))
    assert rc == 0, L.bce_last_error()
    torch.cuda.synchronize()
    out = {k: getattr(res, k).cpu().numpy() for k in ("consensus", "confidence", "total_weight", "n_unique",
                                                      "err_idx", "usid", "nweight")}
    out["weight"] = exp["weight"]  # not written by this launch
    _compare_vec(out, exp, g["offsets"], exact=(mode == "exact"))


def test_wide_direct_csr_unplanned():
    """bce_consensus_csr with max_len in (64, 4096]: every market (short ones too) goes
    through one wide launch sized by max_len."""
    from bayesian_engine import _native as N, batch
    rng = np.random.default_rng(21)
    lens = rng.integers(0, 3000, 120)
    lens[:5] = [0, 1, 64, 65, 2999]
    g = _zipf_case(lens, 20000, 21, base=3)
    exp = orc.consensus_csr(g["offsets"], g["sid"], g["prob"], g["rel"], g["conf"], g["present"])
    table = batch.SourceTable.from_arrays(_dev(g["rel"]), _dev(g["conf"]), _dev(g["present"]))
    M = len(lens)
    n = int(g["offsets"][-1])
    off, sid, prob = _dev(g["offsets"]), _dev(g["sid"], np.int32), _dev(g["prob"])
    res = batch._alloc(M, n, off.device, True, True)
    L = N.lib()
    rc = L.bce_consensus_csr(N.ptr(off), M, N.ptr(sid), N.ptr(prob), n, N.ptr(table.relconf), N.ptr(table.bits),
                             table.n, N.ptr(None), 0, int(lens.max()), N.MODE_EXACT, N.ptr(res.consensus),
                             N.ptr(res.confidence), N.ptr(res.total_weight), N.ptr(res.n_unique),
                             N.ptr(res.err_idx), N.ptr(res.usid), N.ptr(res.weight), N.ptr(res.nweight),
                             N.stream(off.device))
    assert rc == 0, L.bce_last_error()
    torch.cuda.synchronize()
    out = {k: getattr(res, k).cpu().numpy() for k in ("consensus", "confidence", "total_weight", "n_unique",
                                                      "err_idx", "usid", "weight", "nweight")}
    _compare_vec(out, exp, g["offsets"])


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("pattern", ["descending", "ascending", "sawtooth", "max_sid"])
def test_wide_ordered_inputs(pattern, mode):
    """Market inputs already ordered (or reversed, or a sawtooth with every other sid
    repeated), and sids at the top of the key range, at every bin edge: the register
    network's lane stages (DPP-fused compares, bank-masked min/max, permlane swap pairs, the
    flip-31 reversal) and the uniform wave-crossing min/max see every compare go the same
    way, and +inf padding ties real keys when sid = 2^(32 - IB) - 1."""
    lens = np.array(EDGES * 2, np.int64)
    off = np.zeros(len(lens) + 1, np.int64)
    off[1:] = np.cumsum(lens)
    n = int(off[-1])
    S = 1 << 20  # the largest table a 4096-key bin packs into 32-bit keys
    sid = np.zeros(n, np.int32)
    for m, L in enumerate(lens):
        i = np.arange(L)
        if pattern == "descending":
            v = S - 1 - 3 * i
        elif pattern == "ascending":
            v = 5 + 7 * i
        elif pattern == "sawtooth":
            v = (i // 2) * 11 + (i % 2) * 5 * (L - i)
        else:  # the largest sids, with duplicates
            v = S - 1 - (i % 97)
        sid[off[m]:off[m + 1]] = np.clip(v, 0, S - 1)
    rng = np.random.default_rng(7)
    prob = rng.random(n)
    rel = rng.uniform(0.1, 1.0, S)
    conf = rng.random(S)
    present = (rng.random(S) < 0.8).astype(np.uint8)
    _check(dict(offsets=off, sid=sid, prob=prob, rel=rel, conf=conf, present=present), mode)


@pytest.mark.parametrize("mode", MODES)
def test_wide_planned_every_bin_vs_oracle(mode):
    """One planned call over every wide bin (65..128 .. 3073..4096, the non-power-of-two 1536 /
    3072 bins included) plus short markets, one bin empty: within 1e-9 of the oracle in FAST and
    bit-exact in EXACT, and a second call reproduces every bit."""
    rng = np.random.default_rng(77)
    lens = np.concatenate([rng.integers(65, 129, 37), rng.integers(129, 257, 9), rng.integers(513, 1025, 7),
                           rng.integers(1025, 1537, 3), rng.integers(1537, 2049, 5), rng.integers(3073, 4097, 3),
                           rng.integers(0, 65, 50), [4096, 65, 512, 1024, 2048]])
    rng.shuffle(lens)
    g = _zipf_case(lens, 200_000, 77, base=11)
    exp = orc.consensus_csr(g["offsets"], g["sid"], g["prob"], g["rel"], g["conf"], g["present"])
    out = _run(g, mode=mode)
    _compare_vec(out, exp, g["offsets"], exact=(mode == "exact"))
    again = _run(g, mode=mode)
    for k in ("consensus", "confidence", "total_weight", "n_unique", "usid", "weight", "nweight"):
        assert np.array_equal(again[k], out[k], equal_nan=True), k


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("S", [(1 << 21) + 3, 10_000_000, (1 << 24) - 1])
def test_wide_64bit_keys_large_tables(S, mode):
    """Tables past the packed 32-bit key (S > 2^(32 - IB)): every wide bin runs its 64-bit-key
    instantiation (the one-buffer wave-crossing stages, 64-bit permlane swap pairs and lane
    stages).  Zipf markets at every bin edge, the largest sids at the top of each market, sids
    that agree in their low 20 bits (a 32-bit key would merge them), against the oracle."""
    rng = np.random.default_rng(S % 1000)
    lens = np.concatenate([np.exp(rng.uniform(np.log(65), np.log(4096), 150)).astype(np.int64), EDGES, [0, 1, 64]])
    rng.shuffle(lens)
    g = _zipf_case(lens, S, S % 977, base=3)
    off = g["offsets"] - g["offsets"][0]
    for m in range(0, len(lens), 3):
        a, b = int(off[m]), int(off[m + 1])
        if b - a >= 4:
            g["sid"][a] = S - 1
            g["sid"][a + 1] = (S - 1) & 0xFFFFF        # same low 20 bits as S - 1
            g["sid"][a + 2] = ((S - 1) & 0xFFFFF) | (1 << 20)
            g["sid"][b - 1] = S - 1
    _check(g, mode)


@pytest.mark.parametrize("mode", MODES)
def test_wide_64bit_keys_ordered_and_single_source(mode):
    """64-bit keys (S = 2^22) on ordered, reversed and single-source markets at every bin edge:
    every compare of a stage goes the same way, and runs thousands of terms long."""
    S = 1 << 22
    lens = np.array(EDGES * 2 + [4096, 3000], np.int64)
    off = np.zeros(len(lens) + 1, np.int64)
    off[1:] = np.cumsum(lens)
    n = int(off[-1])
    sid = np.zeros(n, np.int32)
    for m, L in enumerate(lens):
        i = np.arange(L)
        v = [S - 1 - 3 * i, 5 + 4099 * i, np.full(L, S - 2)][m % 3]
        sid[off[m]:off[m + 1]] = np.clip(v, 0, S - 1)
    rng = np.random.default_rng(8)
    g = dict(offsets=off, sid=sid, prob=rng.random(n), rel=rng.uniform(0.1, 1.0, S), conf=rng.random(S),
             present=(rng.random(S) < 0.8).astype(np.uint8))
    _check(g, mode)
