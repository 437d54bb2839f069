"""The device planner (bce_plan_bins_device, batch.Plan.build_device) against the host planner
bce_plan_bins (the test oracle for the plan): order and bin boundaries identical, edge lengths,
several radix chunks, decreasing offsets rejected; and consensus through the device plan equal
to consensus through the host plan (and the oracle)."""
import numpy as np
import pytest
import torch

from golden_util import load_npz
from oracle import oracle as orc
from test_gpu_consensus import _compare_vec, _dev

pytestmark = pytest.mark.gpu

EDGE = [0, 1, 8, 9, 16, 17, 32, 33, 63, 64, 65, 128, 129, 256, 257, 512, 513, 1024, 1025, 1536, 1537, 2048,
        2049, 3072, 3073, 4095, 4096, 4097, 5000, 9000]


def _host_plan(off):
    from bayesian_engine import _native as N
    L = N.lib()
    M = len(off) - 1
    order = np.zeros(max(M, 1), np.int32)
    bins = np.zeros(N.NBINS + 1, np.int64)
    mx = np.zeros(1, np.int32)
    N.check(L.bce_plan_bins(N.ptr(off), M, N.ptr(order), N.ptr(bins), N.ptr(mx)), "plan_bins")
    sb = int(L.bce_consensus_scratch_bytes(N.ptr(off), N.ptr(order), N.ptr(bins)))
    return order[:M], bins, int(mx[0]), sb


def _offsets(lens):
    off = np.zeros(len(lens) + 1, np.int64)
    off[1:] = np.cumsum(np.asarray(lens, np.int64))
    return off


def _cases():
    rng = np.random.default_rng(11)
    yield "c3_slice", load_npz("c3_slice.npz")["offsets"]
    yield "edges", _offsets(EDGE + EDGE[::-1] + EDGE)
    lens = np.floor(np.exp(rng.uniform(0, np.log(4097), 300_000))).astype(np.int64)
    yield "loguniform_300k", _offsets(lens)
    lens = rng.choice(EDGE, 5000)
    yield "edges_shuffled", _offsets(lens)
    yield "one", _offsets([77])
    yield "empty_markets", _offsets([0] * 2049)
    yield "uniform_32", _offsets([32] * 70000)
    yield "base_offset", _offsets(rng.integers(0, 300, 3000)) + 12345
    # > 1024 radix chunks of 1024 markets: the planner's digit-major scan path
    lens = np.where(rng.random(1_200_000) < 0.01, rng.integers(65, 4097, 1_200_000), rng.integers(0, 65, 1_200_000))
    yield "many_markets_1p2M", _offsets(lens)


@pytest.mark.parametrize("name,off", list(_cases()), ids=[c[0] for c in _cases()])
def test_device_plan_identical_to_host_plan(name, off):
    from bayesian_engine import batch
    order, bins, mx, sb = _host_plan(off)
    p = batch.Plan.build_device(_dev(off))
    M = len(off) - 1
    assert np.array_equal(p.bin_start, bins), (p.bin_start, bins)
    assert np.array_equal(p.order[:M].cpu().numpy(), order)
    assert p.max_len == mx
    assert (p.scratch.numel() if p.scratch is not None else 0) == sb


def test_device_plan_zero_markets():
    from bayesian_engine import batch
    p = batch.Plan.build_device(_dev(np.zeros(1, np.int64)))
    assert not p.bin_start.any() and p.max_len == 0


def test_device_plan_rejects_decreasing_offsets():
    from bayesian_engine import _native as N
    from bayesian_engine import batch
    off = _offsets([5, 70, 3, 9] * 700)
    off[1500] = off[1499] - 1  # market 1499 has a negative length
    with pytest.raises(N.BCEError, match="not monotone at market 1499"):
        batch.Plan.build_device(_dev(off))


@pytest.mark.parametrize("mode", ["exact", "fast"])
def test_consensus_without_plan_uses_device_plan(mode):
    """batch.consensus(plan=None) plans on the GPU: same outputs as the host plan, oracle-exact."""
    from bayesian_engine import batch
    g = load_npz("c3_slice.npz")
    off = g["offsets"]
    n = int(off[-1])
    table = batch.SourceTable.from_arrays(_dev(g["rel"]), _dev(g["conf"]), _dev(g["present"]))
    args = (_dev(off), _dev(g["sid"], np.int32), _dev(g["prob"]), table)
    a = batch.consensus(*args, mode=mode, check=True)
    b = batch.consensus(*args, plan=batch.Plan.build(off), mode=mode, check=True)
    torch.cuda.synchronize()
    u = b.n_unique.cpu().numpy().astype(np.int64)
    pos = np.repeat(off[:-1], u) + (np.arange(int(u.sum())) - np.repeat(np.cumsum(u) - u, u))
    for k in ("consensus", "confidence", "total_weight", "n_unique", "err_idx", "usid", "weight", "nweight"):
        x, y = getattr(a, k).cpu().numpy(), getattr(b, k).cpu().numpy()
        if k in ("usid", "weight", "nweight"):
            x, y = x[pos], y[pos]
        assert x.tobytes() == y.tobytes(), k
    exp = orc.consensus_csr(off, g["sid"], g["prob"], g["rel"], g["conf"], g["present"])
    _compare_vec({k: getattr(a, k).cpu().numpy() for k in exp if hasattr(a, k)}, exp, off, exact=(mode == "exact"))
    assert n > 0


@pytest.mark.parametrize("mode", ["exact", "fast"])
def test_sync_free_fresh_batch_matches_host_plan(mode):
    """batch.consensus(plan=None, max_len=4096): planned on the device and launched from the
    device-resident bin boundaries (bce_plan_bins_device_async + bce_consensus_planned_device),
    no host synchronisation -- identical outputs to the host-planned call (EXACT bit for bit;
    FAST: the full-batch launch structure, so bit for bit as well on a batch whose bins are not
    merged, and within 1e-9 in any case), and oracle-exact / within 1e-9."""
    from bayesian_engine import batch
    for g in (load_npz("c3_slice.npz"), _edge_batch()):
        off = g["offsets"]
        table = batch.SourceTable.from_arrays(_dev(g["rel"]), _dev(g["conf"]), _dev(g["present"]))
        args = (_dev(off), _dev(g["sid"], np.int32), _dev(g["prob"]), table)
        a = batch.consensus(*args, max_len=4096, mode=mode, check=True)
        b = batch.consensus(*args, plan=batch.Plan.build(off), mode=mode, check=True)
        torch.cuda.synchronize()
        u = b.n_unique.cpu().numpy().astype(np.int64)
        pos = np.repeat(off[:-1], u) + (np.arange(int(u.sum())) - np.repeat(np.cumsum(u) - u, u))
        for k in ("n_unique", "err_idx", "usid", "weight"):
            x, y = getattr(a, k).cpu().numpy(), getattr(b, k).cpu().numpy()
            if k in ("usid", "weight"):
                x, y = x[pos], y[pos]
            assert x.tobytes() == y.tobytes(), k
        exp = orc.consensus_csr(off, g["sid"], g["prob"], g["rel"], g["conf"], g["present"])
        _compare_vec({k: getattr(a, k).cpu().numpy() for k in exp if hasattr(a, k)}, exp, off,
                     exact=(mode == "exact"))


def _edge_batch():
    rng = np.random.default_rng(21)
    lens = np.concatenate([rng.choice(EDGE[:-3], 3000), [0] * 50])  # up to 4096
    rng.shuffle(lens)
    off = _offsets(lens)
    n, S = int(off[-1]), 5000
    prob = rng.random(n)
    prob[rng.random(n) < 1e-3] = -0.5
    rel, conf = rng.uniform(0.1, 1.0, S), rng.random(S)
    present = (rng.random(S) < 0.8).astype(np.uint8)
    return dict(offsets=off, sid=rng.integers(0, S, n).astype(np.int32), prob=prob, rel=rel, conf=conf,
                present=present)


def test_sync_free_fresh_batch_faults():
    """The sync-free path reports what it cannot compute through the device fault word: a market
    longer than 4096 signals, and decreasing offsets (nothing computed)."""
    from bayesian_engine import _native as N
    from bayesian_engine import batch
    rng = np.random.default_rng(5)
    dev = torch.device("cuda", 0)
    S = 100
    table = batch.SourceTable.from_arrays(_dev(rng.random(S)), _dev(rng.random(S)), _dev(np.ones(S, np.uint8)))
    N.check_faults(dev, "clean slate")
    off = _offsets([100, 5000, 70])
    n = int(off[-1])
    with pytest.raises(N.BCEError, match="longer than"):
        batch.consensus(_dev(off), _dev(rng.integers(0, S, n).astype(np.int32)), _dev(rng.random(n)), table,
                        max_len=4096, check=True)
    bad = _offsets([100, 70, 80, 90])
    bad[2] = bad[1] - 5
    with pytest.raises(N.BCEError, match="not monotone"):
        batch.consensus(_dev(bad), _dev(rng.integers(0, S, 400).astype(np.int32)), _dev(rng.random(400)), table,
                        max_len=4096, check=True)
