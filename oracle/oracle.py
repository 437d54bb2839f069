"""ctypes wrapper over the CPU restatement (oracle/bce_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the shipped package.  Every function
mirrors one reference function; see bce_oracle.h for the file:line map.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None

NO_TIMESTAMP = np.iinfo(np.int64).min


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = C.CDLL(_LIB_PATH)
        _lib.orc_decay_factor.restype = C.c_double
        _lib.orc_decay_factor.argtypes = [C.c_double, C.c_double]
        _lib.orc_apply_decay.restype = C.c_double
        _lib.orc_apply_decay.argtypes = [C.c_double] * 4
        _lib.orc_days_since.restype = C.c_double
        _lib.orc_days_since.argtypes = [C.c_int64, C.c_int64]
        _lib.orc_round_decimal.restype = C.c_double
        _lib.orc_round_decimal.argtypes = [C.c_double, C.c_int]
    return _lib


def _p(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return C.c_void_p(a.ctypes.data)


def consensus_csr(offsets, sid, prob, rel, conf, present):
    offsets = np.ascontiguousarray(offsets, np.int64)
    sid = np.ascontiguousarray(sid, np.int32)
    prob = np.ascontiguousarray(prob, np.float64)
    rel = np.ascontiguousarray(rel, np.float64)
    conf = np.ascontiguousarray(conf, np.float64)
    present = np.ascontiguousarray(present, np.uint8)
    M, N = len(offsets) - 1, len(sid)
    out = dict(
        consensus=np.zeros(M), confidence=np.zeros(M), total_weight=np.zeros(M),
        n_unique=np.zeros(M, np.int32), err_idx=np.zeros(M, np.int32),
        usid=np.full(N, -1, np.int32), weight=np.zeros(N), nweight=np.zeros(N),
    )
    rc = lib().orc_consensus_csr(
        _p(offsets), C.c_int64(M), _p(sid), _p(prob), _p(rel), _p(conf), _p(present),
        C.c_int32(len(rel)), _p(out["consensus"]), _p(out["confidence"]), _p(out["total_weight"]),
        _p(out["n_unique"]), _p(out["err_idx"]), _p(out["usid"]), _p(out["weight"]), _p(out["nweight"]))
    if rc != 0:
        raise RuntimeError(f"orc_consensus_csr rc={rc}")
    return out


def decay_factor(e, h=30.0):
    return lib().orc_decay_factor(float(e), float(h))


def apply_decay(r, e, h=30.0, m=0.10):
    return lib().orc_apply_decay(float(r), float(e), float(h), float(m))


def days_since(now_us, t_us):
    return lib().orc_days_since(int(now_us), int(t_us))


def round_decimal(x, nd=6):
    return lib().orc_round_decimal(float(x), int(nd))


def decay_view(rel, t_us, present, now_us, half_life=30.0, min_rel=0.10, default_rel=0.50):
    rel = np.ascontiguousarray(rel, np.float64)
    t_us = np.ascontiguousarray(t_us, np.int64)
    present = np.ascontiguousarray(present, np.uint8)
    view = np.zeros(len(rel))
    lib().orc_decay_view(C.c_int64(len(rel)), _p(rel), _p(t_us), _p(present), C.c_int64(int(now_us)),
                         C.c_double(half_life), C.c_double(min_rel), C.c_double(default_rel), _p(view))
    return view


def outcome_update(rel, conf, t_us, present, flags, now_us, default_rel=0.50, default_conf=0.25):
    """In-place on copies; returns (rel, conf, t_us, present)."""
    rel = np.array(rel, np.float64)
    conf = np.array(conf, np.float64)
    t_us = np.array(t_us, np.int64)
    present = np.array(present, np.uint8)
    flags = np.ascontiguousarray(flags, np.uint8)
    lib().orc_outcome_update(C.c_int64(len(rel)), _p(rel), _p(conf), _p(t_us), _p(present), _p(flags),
                             C.c_int64(int(now_us)), C.c_double(default_rel), C.c_double(default_conf))
    return rel, conf, t_us, present


def agreement_stats(offsets, sid, prob, outcome, n_sources):
    offsets = np.ascontiguousarray(offsets, np.int64)
    sid = np.ascontiguousarray(sid, np.int32)
    prob = np.ascontiguousarray(prob, np.float64)
    outcome = np.ascontiguousarray(outcome, np.int8)
    correct = np.zeros(n_sources, np.int32)
    total = np.zeros(n_sources, np.int32)
    lib().orc_agreement_stats(_p(offsets), C.c_int64(len(offsets) - 1), _p(sid), _p(prob), _p(outcome),
                              _p(correct), _p(total))
    return correct, total


def tiebreak_csr(offsets, pred, conf, weight, rel, keys=None):
    """tiebreak.py:73-152 per market; group keys round(pred, 6), or ``keys`` (the caller's
    own round(pred, precision) for other precisions)."""
    offsets = np.ascontiguousarray(offsets, np.int64)
    pred, conf, weight, rel = (np.ascontiguousarray(x, np.float64) for x in (pred, conf, weight, rel))
    keys = None if keys is None else np.ascontiguousarray(keys, np.float64)
    M, N = len(offsets) - 1, len(pred)
    out = dict(winner=np.zeros(M), label=np.zeros(M, np.int32), n_groups=np.zeros(M, np.int32),
               variance=np.zeros(M), g_key=np.zeros(N), g_count=np.zeros(N, np.int32),
               g_total=np.zeros(N), g_avgconf=np.zeros(N), g_maxrel=np.zeros(N))
    rc = lib().orc_tiebreak_csr(_p(offsets), C.c_int64(M), _p(pred), _p(conf), _p(weight), _p(rel),
                                _p(keys) if keys is not None else C.c_void_p(0),
                                *[_p(out[k]) for k in ("winner", "label", "n_groups", "variance", "g_key",
                                                        "g_count", "g_total", "g_avgconf", "g_maxrel")])
    if rc != 0:
        raise RuntimeError(f"orc_tiebreak_csr rc={rc}")
    return out


def reestimate(P, iters, w0=0.5):
    P = np.ascontiguousarray(P, np.float64)
    A, M = P.shape
    w = np.full(A, w0, np.float64)
    cons = np.zeros((iters, M))
    null = np.zeros((iters, M), np.uint8)
    agree = np.zeros((iters, A), np.int64)
    lib().orc_reestimate(_p(P), C.c_int64(A), C.c_int64(M), C.c_int(iters), _p(w), _p(cons), _p(null),
                         _p(agree))
    return w, cons, null, agree


def namespace_resolve(scopes, apply_decay, now_us, half_life=30.0, min_rel=0.10, default_rel=0.50,
                      default_conf=0.25):
    """scopes: 3 entries (market, domain, global), each None or (rel, conf, t_us, has)."""
    n = next(len(sc[0]) for sc in scopes if sc is not None) if any(sc is not None for sc in scopes) else 0
    keep = []
    ptrs = {k: (C.c_void_p * 3)() for k in ("rel", "conf", "t", "has")}
    for q, sc in enumerate(scopes):
        if sc is None:
            continue
        arrs = (np.ascontiguousarray(sc[0], np.float64), np.ascontiguousarray(sc[1], np.float64),
                np.ascontiguousarray(sc[2], np.int64), np.ascontiguousarray(sc[3], np.uint8))
        keep.append(arrs)
        for k, a in zip(("rel", "conf", "t", "has"), arrs):
            ptrs[k][q] = a.ctypes.data
    rel, conf, scope = np.zeros(n), np.zeros(n), np.zeros(n, np.uint8)
    lib().orc_namespace_resolve(C.c_int64(n), ptrs["rel"], ptrs["conf"], ptrs["t"], ptrs["has"],
                                C.c_int(int(apply_decay)), C.c_int64(int(now_us)), C.c_double(half_life),
                                C.c_double(min_rel), C.c_double(default_rel), C.c_double(default_conf),
                                _p(rel), _p(conf), _p(scope))
    return rel, conf, scope


def aggregate_groups(goff, members, cons, conf, has):
    goff = np.ascontiguousarray(goff, np.int64)
    members = np.ascontiguousarray(members, np.int64)
    cons = np.ascontiguousarray(cons, np.float64)
    conf = np.ascontiguousarray(conf, np.float64)
    has = np.ascontiguousarray(has, np.uint8)
    G = len(goff) - 1
    out = dict(wavg=np.zeros(G), median=np.zeros(G), majority=np.zeros(G), mean_conf=np.zeros(G),
               n_included=np.zeros(G, np.int64))
    lib().orc_aggregate_groups(_p(goff), C.c_int64(G), _p(members), _p(cons), _p(conf), _p(has),
                               _p(out["wavg"]), _p(out["median"]), _p(out["majority"]), _p(out["mean_conf"]),
                               _p(out["n_included"]))
    return out
