"""Shared helpers for parity tests: load fixtures, intern single-market cases to CSR."""
from __future__ import annotations

import json
import math
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_json(name):
    with open(os.path.join(GOLDEN, name), encoding="utf-8") as f:
        return json.load(f)


def load_npz(name):
    return dict(np.load(os.path.join(GOLDEN, name), allow_pickle=False))


def same_float(a, b) -> bool:
    """Bit-level equality for floats (NaN == NaN, 0.0 != -0.0 is NOT required)."""
    if isinstance(a, float) and math.isnan(a):
        return isinstance(b, float) and math.isnan(b)
    return a == b


def case_to_csr(signals, rel_dict):
    """One market -> CSR arrays + baked table, names in Python sorted() order."""
    names = sorted({s["sourceId"] for s in signals})
    idx = {n: i for i, n in enumerate(names)}
    rel_dict = rel_dict or {}
    S = max(len(names), 1)
    rel = np.full(S, 0.5)
    conf = np.full(S, 0.25)
    present = np.zeros(S, np.uint8)
    for n, i in idx.items():
        if n in rel_dict:
            present[i] = 1
            d = rel_dict[n]
            rel[i] = float(d.get("reliability", 0.5))
            conf[i] = float(d.get("confidence", 0.25))
    offsets = np.array([0, len(signals)], np.int64)
    sid = np.array([idx[s["sourceId"]] for s in signals], np.int32)
    prob = np.array([float(s["probability"]) for s in signals], np.float64)
    return names, offsets, sid, prob, rel, conf, present
