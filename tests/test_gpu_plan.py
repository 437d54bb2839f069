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
