"""Sharded consensus (markets shard over ranks with no communication),
run on one GPU exactly as each rank of an N-rank job runs its shard, against the unsharded run
and the oracle.

Each rank r of ``sharding.shard_markets(offsets, N, r)`` gets the market range [m0, m1):
  * rebased: its own CSR copy (offsets[m0:m1+1] - offsets[m0], the sid / prob slices), its own
    plan (bench.py / bench_extra.make_c3 build a rank's batch this way);
  * offset view: offsets[m0:m1+1] unrebased over the full sid / prob arrays (batch.consensus
    accepts offsets[0] != 0; per-unique outputs land at the absolute CSR positions).
Concatenated in rank order, every output must equal the single unsharded call: bit for bit in
EXACT (and the oracle's), and in FAST bit for bit on the integer outputs, usid and weight and
within the north star's 1e-9 on consensus / confidence / total weight / normalizedWeight -- a
small call (a shard) may run a length bin in the launch of the bin above it (fewer, fuller
launches, bce_consensus_planned's kMergeRounds), whose wider workgroup sums the FAST partial
totals in another fixed order.  This is what the driver's 8-GPU SCALE run relies on.
"""
import numpy as np
import pytest
import torch

from golden_util import load_npz
from oracle import oracle as orc
from test_gpu_consensus import _compare_vec, _dev

pytestmark = pytest.mark.gpu

KEYS_M = ("consensus", "confidence", "total_weight", "n_unique", "err_idx")
KEYS_U = ("usid", "weight", "nweight")


def _c3_like(total, S, seed):
    """make_c3's law at a smaller size: log-uniform lengths on [1, 4096], Zipf(1.1)."""
    rng = np.random.default_rng(seed)
    lens = np.floor(np.exp(rng.uniform(0, np.log(4097), size=total // 300 + 10))).astype(np.int64)
    cs = np.cumsum(lens)
    M = int(np.searchsorted(cs, total) + 1)
    lens = lens[:M]
    lens[-1] -= int(cs[M - 1] - total)
    off = np.zeros(M + 1, np.int64)
    off[1:] = np.cumsum(lens)
    z = rng.zipf(1.1, size=total)
    bad = np.nonzero(z > S)[0]
    while bad.size:
        z[bad] = rng.zipf(1.1, size=bad.size)
        bad = bad[z[bad] > S]
    sid = rng.permutation(S).astype(np.int32)[z - 1]
    prob = rng.random(total)
    prob[rng.random(total) < 1e-4] = 1.5
    rel, conf = rng.uniform(0.1, 1.0, S), rng.random(S)
    present = (rng.random(S) < 0.9).astype(np.uint8)
    return dict(offsets=off, sid=sid, prob=prob, rel=rel, conf=conf, present=present)


def _c2_like(M, L, S, seed):
    rng = np.random.default_rng(seed)
    off = np.arange(0, M * L + 1, L, dtype=np.int64)
    sid = rng.integers(0, S, M * L, dtype=np.int32)
    prob = rng.random(M * L)
    rel, conf = rng.uniform(0.1, 1.0, S), rng.random(S)
    present = (rng.random(S) < 0.9).astype(np.uint8)
    return dict(offsets=off, sid=sid, prob=prob, rel=rel, conf=conf, present=present)


def _case(name):
    if name == "c3_slice":
        d = load_npz("c3_slice.npz")
        return {k: d[k] for k in ("offsets", "sid", "prob", "rel", "conf", "present")}
    if name == "c3_like":
        return _c3_like(3_000_000, 1_000_000, 5)
    return _c2_like(1_000_000, 32, 10_000, 6)


def _call(off_h, sid_d, prob_d, table, N_sig, mode, uniform, dev):
    from bayesian_engine import batch
    off_d = torch.from_numpy(np.ascontiguousarray(off_h)).to(dev)
    res = batch._alloc(len(off_h) - 1, N_sig, dev, True, True)
    if uniform:
        batch.consensus(off_d, sid_d, prob_d, table, max_len=32, mode=mode, out=res)
    else:
        batch.consensus(off_d, sid_d, prob_d, table, plan=batch.Plan.build(off_h, dev), mode=mode, out=res)
    torch.cuda.synchronize()
    return {k: getattr(res, k).cpu().numpy() for k in KEYS_M + KEYS_U}


@pytest.mark.timeout(600)
@pytest.mark.parametrize("mode", ["exact", "fast"])
@pytest.mark.parametrize("name", ["c3_slice", "c3_like", "c2_1M"])
def test_sharded_consensus_matches_unsharded_and_oracle(name, mode):
    from bayesian_engine import _native as N
    from bayesian_engine import batch
    from bayesian_engine.sharding import shard_markets
    g = _case(name)
    off = g["offsets"]
    M, n = len(off) - 1, int(off[-1])
    uniform = name == "c2_1M"
    dev = torch.device("cuda", 0)
    table = batch.SourceTable.from_arrays(_dev(g["rel"]), _dev(g["conf"]), _dev(g["present"]))
    sid_d, prob_d = _dev(g["sid"], np.int32), _dev(g["prob"])
    full = _call(off, sid_d, prob_d, table, n, mode, uniform, dev)
    exp = orc.consensus_csr(off, g["sid"], g["prob"], g["rel"], g["conf"], g["present"])
    _compare_vec(full, exp, off, exact=(mode == "exact"))
    u = exp["n_unique"].astype(np.int64)
    pos = np.repeat(off[:-1], u) + (np.arange(int(u.sum())) - np.repeat(np.cumsum(u) - u, u))
    for world in (2, 8):
        cat = {k: np.zeros_like(full[k]) for k in KEYS_M + KEYS_U}
        view = {k: np.zeros_like(full[k]) for k in KEYS_M + KEYS_U}
        for r in range(world):
            m0, m1 = shard_markets(off, world, r)
            a, b = int(off[m0]), int(off[m1])
            # rebased: the rank's own batch
            loc = off[m0:m1 + 1] - a
            o = _call(loc, _dev(g["sid"][a:b], np.int32), _dev(g["prob"][a:b]), table, b - a, mode, uniform, dev)
            for k in KEYS_M:
                cat[k][m0:m1] = o[k][:m1 - m0]
            for k in KEYS_U:
                cat[k][a:b] = o[k][:b - a]
            # offset view over the full arrays (absolute CSR positions)
            o = _call(off[m0:m1 + 1], sid_d, prob_d, table, n, mode, uniform, dev)
            for k in KEYS_M:
                view[k][m0:m1] = o[k][:m1 - m0]
            for k in KEYS_U:
                view[k][a:b] = o[k][a:b]
        N.check_faults(dev, f"{name} {world} shards")
        floats = ("consensus", "confidence", "total_weight", "nweight")
        for got, how in ((cat, "rebased"), (view, "offset view")):
            for k in KEYS_M + KEYS_U:
                a_, b_ = (got[k][pos], full[k][pos]) if k in KEYS_U else (got[k], full[k])
                if mode == "fast" and k in floats:
                    np.testing.assert_allclose(a_, b_, rtol=0, atol=1e-9, equal_nan=True, err_msg=f"{world} {how} {k}")
                else:
                    assert a_.tobytes() == b_.tobytes(), (world, how, k)
            # the shards against the oracle as well (FAST: the same 1e-9)
            _compare_vec(got, exp, off, exact=(mode == "exact"))


def _call_list(off_h, sid_d, prob_d, table, N_sig, mode, markets, dev):
    """One rank's markets of a planned split left in place: a plan over the full CSR."""
    from bayesian_engine import batch
    off_d = torch.from_numpy(np.ascontiguousarray(off_h)).to(dev)
    res = batch._alloc(len(off_h) - 1, N_sig, dev, True, True)
    batch.consensus(off_d, sid_d, prob_d, table, plan=batch.Plan.for_markets(off_h, markets, dev), mode=mode,
                    out=res)
    torch.cuda.synchronize()
    return {k: getattr(res, k).cpu().numpy() for k in KEYS_M + KEYS_U}


@pytest.mark.timeout(600)
@pytest.mark.parametrize("mode", ["exact", "fast"])
@pytest.mark.parametrize("name", ["c3_slice", "c3_like", "c2_1M"])
def test_planned_shards_match_unsharded_and_oracle(name, mode):
    """sharding.shard_markets_planned (the plan order cut at equal measured cost: whole length
    classes per rank, the C3 split of the N > 1 bench line) for N = 2 and 8, as each rank's own
    gathered CSR (sharding.gather_csr, its own plan; outputs scattered back by market index) and
    as a market subset of the full CSR (batch.Plan.for_markets): EXACT bit for bit, FAST within
    1e-9 on the float outputs, against the unsharded call and the oracle."""
    from bayesian_engine import _native as N
    from bayesian_engine import batch
    from bayesian_engine.sharding import gather_csr, shard_markets_planned
    g = _case(name)
    off = g["offsets"]
    M, n = len(off) - 1, int(off[-1])
    uniform = name == "c2_1M"
    dev = torch.device("cuda", 0)
    table = batch.SourceTable.from_arrays(_dev(g["rel"]), _dev(g["conf"]), _dev(g["present"]))
    sid_d, prob_d = _dev(g["sid"], np.int32), _dev(g["prob"])
    full = _call(off, sid_d, prob_d, table, n, mode, uniform, dev)
    exp = orc.consensus_csr(off, g["sid"], g["prob"], g["rel"], g["conf"], g["present"])
    u = exp["n_unique"].astype(np.int64)
    pos = np.repeat(off[:-1], u) + (np.arange(int(u.sum())) - np.repeat(np.cumsum(u) - u, u))
    for world in (2, 8):
        cat = {k: np.zeros_like(full[k]) for k in KEYS_M + KEYS_U}
        view = {k: np.zeros_like(full[k]) for k in KEYS_M + KEYS_U}
        seen = np.zeros(M, np.int64)
        for r in range(world):
            mk = shard_markets_planned(off, world, r)
            seen[mk] += 1
            loc, idx, s, p = gather_csr(off, mk, g["sid"], g["prob"])
            o = _call(loc, _dev(s, np.int32), _dev(p), table, len(idx), mode, uniform, dev)
            for k in KEYS_M:
                cat[k][mk] = o[k][:len(mk)]
            for k in KEYS_U:
                cat[k][idx] = o[k][:len(idx)]
            o = _call_list(off, sid_d, prob_d, table, n, mode, mk, dev)
            for k in KEYS_M:
                view[k][mk] = o[k][mk]
            for k in KEYS_U:
                view[k][idx] = o[k][idx]
        assert (seen == 1).all(), "every market on exactly one rank"
        N.check_faults(dev, f"{name} {world} planned shards")
        floats = ("consensus", "confidence", "total_weight", "nweight")
        for got, how in ((cat, "gathered"), (view, "market subset")):
            for k in KEYS_M + KEYS_U:
                a_, b_ = (got[k][pos], full[k][pos]) if k in KEYS_U else (got[k], full[k])
                if mode == "fast" and k in floats:
                    np.testing.assert_allclose(a_, b_, rtol=0, atol=1e-9, equal_nan=True, err_msg=f"{world} {how} {k}")
                else:
                    assert a_.tobytes() == b_.tobytes(), (world, how, k)
            _compare_vec(got, exp, off, exact=(mode == "exact"))
