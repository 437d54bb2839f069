"""CPU checks of the drop-in boundary: the C ABI library loads and exports exactly what
include/bce.h declares; host-side entry points (planning, argument checks) work without
a GPU; compute entry points refuse to run without one (no CPU fallback)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from bayesian_engine import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "bce.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(bce_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    lib = N.load_library()
    declared = _declared()
    assert len(declared) >= 18
    for name in declared:
        assert hasattr(lib, name), name
    assert set(declared) == set(N.EXPORTED), "ctypes signature table out of sync with bce.h"


def test_abi_version_and_device_count():
    lib = N.load_library()
    assert lib.bce_abi_version() == 3
    assert lib.bce_device_count() >= 0


def test_argument_errors_need_no_gpu():
    lib = N.load_library()
    rc = lib.bce_consensus_csr(None, 5, None, None, 0, None, None, 0, None, 0, 32, 0,
                               None, None, None, None, None, None, None, None, None)
    assert rc == -1
    assert b"offsets" in lib.bce_last_error()
    rc = lib.bce_tiebreak_csr(None, 3, None, 0, None, None, None, None, 8, 99, *([None] * 11))
    assert rc == -1


def test_plan_bins_host():
    lib = N.load_library()
    rng = np.random.default_rng(0)
    lens = np.concatenate([[0, 8, 9, 16, 17, 32, 33, 64, 65, 128, 129, 256, 257, 512, 513, 1024, 1025, 1536,
                            1537, 2048, 2049, 3072, 3073, 4096, 4097], rng.integers(0, 6000, 300)])
    off = np.zeros(len(lens) + 1, np.int64)
    off[1:] = np.cumsum(lens)
    order = np.zeros(len(lens), np.int32)
    bins = np.zeros(N.NBINS + 1, np.int64)
    mx = np.zeros(1, np.int32)
    assert lib.bce_plan_bins(N.ptr(off), len(lens), N.ptr(order), N.ptr(bins), N.ptr(mx)) == 0
    edges = [0, 8, 16, 32, 64, 128, 256, 512, 1024, 1536, 2048, 3072, 4096, 1 << 62]
    assert N.NBINS == 13
    for b in range(N.NBINS):
        ms = order[bins[b]:bins[b + 1]]
        ln = lens[ms]
        if 4 <= b <= 11:  # wide bins: longest first, ties in market order (LPT)
            assert np.all(np.diff(ln) <= 0)
            assert np.all(np.diff(ms)[np.diff(ln) == 0] > 0)
        else:
            assert np.all(np.diff(ms) > 0)  # ascending inside a bin
        assert np.all((ln <= edges[b + 1]) & ((ln > edges[b]) if b else True))
    assert sorted(order.tolist()) == list(range(len(lens)))
    assert mx[0] == lens.max()
    sb = lib.bce_consensus_scratch_bytes(N.ptr(off), N.ptr(order), N.ptr(bins))
    n_huge = int(bins[13] - bins[12])
    P = 1 << int(np.ceil(np.log2(lens[lens > 4096].max())))
    assert sb == min(n_huge, 512) * 4 * P * 8


@pytest.mark.skipif(N.torch.cuda.is_available(), reason="checks the no-GPU path")
def test_compute_refuses_without_gpu():
    from bayesian_engine import core
    with pytest.raises(N.NativeUnavailable):
        core.compute_consensus([{"sourceId": "a", "probability": 0.5}])
