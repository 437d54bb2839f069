"""CPU checks of the planned market split (sharding.shard_markets_planned, the C3 split of the
N > 1 bench line): the numpy plan order is bce_plan_bins' (the library's host planner), the
split is a partition of the markets at equal modelled cost in which every rank holds whole
length classes, and gather_csr rebuilds a rank's own CSR."""
import numpy as np
import pytest

from bayesian_engine import _native as N
from bayesian_engine.sharding import (BIN_MAX, PLAN_BIN_COST_US, gather_csr, market_bins, plan_order,
                                      shard_markets_planned)

EDGE = [0, 1, 8, 9, 16, 17, 32, 33, 64, 65, 128, 129, 256, 257, 512, 513, 1024, 1025, 1536, 1537, 2048,
        2049, 3072, 3073, 4096, 4097, 9000]


def _offsets(seed, M=20000, edges=True):
    rng = np.random.default_rng(seed)
    lens = np.floor(np.exp(rng.uniform(0, np.log(4097), size=M))).astype(np.int64)
    if edges:
        lens = np.concatenate([lens, EDGE, EDGE[::-1]])
        rng.shuffle(lens)
    off = np.zeros(len(lens) + 1, np.int64)
    off[1:] = np.cumsum(lens)
    return off


def _host_plan(off):
    L = N.load_library()
    M = len(off) - 1
    order = np.zeros(max(M, 1), np.int32)
    bins = np.zeros(N.NBINS + 1, np.int64)
    mx = np.zeros(1, np.int32)
    N.check(L.bce_plan_bins(N.ptr(off), M, N.ptr(order), N.ptr(bins), N.ptr(mx)), "plan_bins")
    return order[:M], bins


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_plan_order_is_bce_plan_bins(seed):
    off = _offsets(seed)
    order, bins = plan_order(off)
    o2, b2 = _host_plan(off)
    assert np.array_equal(bins, b2)
    assert np.array_equal(order, o2)


def test_plan_order_rejects_decreasing_offsets():
    with pytest.raises(ValueError):
        plan_order(np.array([0, 5, 3], np.int64))


@pytest.mark.parametrize("mode", ["fast", "exact"])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_planned_split_is_a_balanced_partition_of_length_classes(world, mode):
    from bayesian_engine.sharding import PLAN_BIN_COST_US_EXACT, _rank_main_us
    off = _offsets(7, M=60000, edges=False)
    M = len(off) - 1
    b = market_bins(off)
    cost = PLAN_BIN_COST_US_EXACT if mode == "exact" else PLAN_BIN_COST_US
    seen = np.zeros(M, np.int64)
    main, side, bins_of = [], [], []
    for r in range(world):
        mk = shard_markets_planned(off, world, r, mode=mode)
        assert np.all(np.diff(mk) > 0), "ascending market indices"
        seen[mk] += 1
        cnt = np.bincount(b[mk], minlength=13).astype(np.float64)
        main.append(_rank_main_us(cnt, mode, cost))
        side.append(float((cost[:4] * cnt[:4]).sum()))
        bins_of.append(set(np.unique(b[mk]).tolist()))
    assert (seen == 1).all()
    # the short bins at equal cost up to one market; the wide ones at equal modelled time up to
    # one market's and one launch's worth
    assert max(side) - min(side) <= 2 * cost[:4].max()
    if world > 1:
        assert max(main) - min(main) <= 2 * cost.max() + 8.0, main
    if world == 8:
        # length classes: a rank holds a few whole (or cut) bins, not a slice of every bin
        assert all(len([x for x in s if x <= 3]) <= 2 and len([x for x in s if x > 3]) <= 4 for s in bins_of), bins_of


def test_gather_csr_rebuilds_the_rank_batch():
    off = _offsets(3, M=3000)
    rng = np.random.default_rng(3)
    n = int(off[-1])
    sid = rng.integers(0, 100, n).astype(np.int32)
    prob = rng.random(n)
    mk = np.sort(rng.choice(len(off) - 1, 700, replace=False)).astype(np.int64)
    loc, idx, s, p = gather_csr(off, mk, sid, prob)
    assert loc[0] == 0 and len(loc) == len(mk) + 1
    for j, m in enumerate(mk[:50]):
        a, b = int(off[m]), int(off[m + 1])
        assert np.array_equal(s[loc[j]:loc[j + 1]], sid[a:b])
        assert np.array_equal(p[loc[j]:loc[j + 1]], prob[a:b])
        assert np.array_equal(idx[loc[j]:loc[j + 1]], np.arange(a, b))


def test_bin_table_matches_library():
    assert len(BIN_MAX) + 1 == N.NBINS
    assert len(PLAN_BIN_COST_US) == N.NBINS
