"""Drop-in for ``bayesian_engine.core`` (reference src/bayesian_engine/core.py:1-179).

Same names, signatures, return dicts and error messages; the arithmetic runs in the HIP
kernels of libbce_hip.so:

* :func:`validate_input_payload` -- the structural/type checks (core.py:34-58) inspect
  the caller's Python objects on the host (that is where they live); the numeric range
  check ``0 <= p <= 1`` (core.py:59-60) runs on the GPU (``bce_validate_csr``).  The
  first failing signal index wins, exactly as in the reference's sequential loop.
* :func:`compute_consensus` -- sorted-source interning on the host (core.py:103: Python
  ``sorted`` order), then one launch of the batched consensus kernel for this market
  (bit-exact: same summation order and rounding as the reference).  Weights are
  returned as the caller's own objects (an int reliability stays an int, core.py:119).

For many markets at once use :mod:`bayesian_engine.batch` (one launch for the batch).
"""
from __future__ import annotations

from typing import Any

import numpy as np
import torch

from . import _native as N
from . import batch
from .config import DEFAULT_CONFIDENCE, DEFAULT_RELIABILITY, SCHEMA_VERSION

__all__ = ["ValidationError", "validate_input_payload", "check_structure", "compute_consensus", "SCHEMA_VERSION",
           "DEFAULT_RELIABILITY", "DEFAULT_CONFIDENCE"]


class ValidationError(ValueError):
    """Raised when input payload fails schema validation (core.py:14-15)."""


def _require(payload: dict[str, Any], key: str) -> Any:
    if key not in payload:
        raise ValidationError(f"{key} is required")
    return payload[key]


def _as_float(p) -> float:
    try:
        return float(p)
    except OverflowError:  # an int beyond float range: still out of [0, 1]
        return float("inf") if p > 0 else float("-inf")


def validate_input_payload(payload: dict[str, Any]) -> None:
    """Validate the v1.0.0 input contract (core.py:24-60), same order and messages."""
    probs, type_error = check_structure(payload)
    if probs:  # range check of the signals before the first type error, on the GPU
        N.require_gpu()
        dev = N.device()
        off = torch.tensor([0, len(probs)], dtype=torch.int64, device=dev)
        p = torch.tensor(probs, dtype=torch.float64, device=dev)
        k = int(batch.validate(off, p)[0].item())
        if k >= 0:
            raise ValidationError(f"signals[{k}].probability must be between 0 and 1")
    if type_error is not None:
        raise type_error


def check_structure(payload: dict[str, Any]) -> tuple[list[float], ValidationError | None]:
    """Host half of validate_input_payload (core.py:34-58): raises the header errors; returns
    the probabilities before the first signal-level type error, and that error (or None).
    The numeric range check (core.py:59-60) over the returned probabilities is the caller's
    GPU launch -- one per payload here, one per batch in :mod:`bayesian_engine.jsonl`."""
    schema_version = _require(payload, "schemaVersion")
    if schema_version != SCHEMA_VERSION:
        raise ValidationError(f"schemaVersion must be '{SCHEMA_VERSION}' (got '{schema_version}')")

    market_id = _require(payload, "marketId")
    if not isinstance(market_id, str) or not market_id.strip():
        raise ValidationError("marketId must be a non-empty string")

    signals = _require(payload, "signals")
    if not isinstance(signals, list):
        raise ValidationError("signals must be an array")

    probs: list[float] = []
    type_error = None
    for idx, signal in enumerate(signals):
        if not isinstance(signal, dict):
            type_error = ValidationError(f"signals[{idx}] must be an object")
            break
        if "sourceId" not in signal:
            type_error = ValidationError("sourceId is required")
            break
        source_id = signal["sourceId"]
        if not isinstance(source_id, str) or not source_id.strip():
            type_error = ValidationError(f"signals[{idx}].sourceId must be a non-empty string")
            break
        if "probability" not in signal:
            type_error = ValidationError("probability is required")
            break
        probability = signal["probability"]
        if not isinstance(probability, (int, float)):
            type_error = ValidationError(f"signals[{idx}].probability must be a number")
            break
        probs.append(probability if type(probability) is float else _as_float(probability))
    return probs, type_error


def _no_signals() -> dict[str, Any]:
    return {
        "schemaVersion": SCHEMA_VERSION,
        "consensus": None,
        "confidence": 0.0,
        "sourceWeights": [],
        "normalization": {"totalWeight": 0.0, "sourceCount": 0},
        "diagnostics": {"status": "no_signals", "sources": 0},
    }


def _check_number(x, other) -> None:
    """Raise the reference's TypeError for a non-numeric operand (core.py:116/120/142)."""
    if not isinstance(x, (int, float)):
        acc = 0.0
        acc += x  # same exception the reference raises at ``total_weight += weight``


def compute_consensus(
    signals: list[dict[str, Any]],
    source_reliability: dict[str, dict[str, float]] | None = None,
) -> dict[str, Any]:
    """Reliability-weighted consensus of one market (core.py:63-179), on the GPU."""
    if not signals:
        return _no_signals()
    if source_reliability is None:
        source_reliability = {}

    source_ids = sorted({s["sourceId"] for s in signals})  # core.py:103
    rank = {sid: i for i, sid in enumerate(source_ids)}
    S = len(source_ids)
    rel_objs = []
    rel = np.empty(S, np.float64)
    conf = np.empty(S, np.float64)
    present = np.zeros(max(S, 2), np.uint8)
    for i, sid in enumerate(source_ids):
        rel_data = source_reliability.get(sid, {})
        r = rel_data.get("reliability", DEFAULT_RELIABILITY)
        c = rel_data.get("confidence", DEFAULT_CONFIDENCE)
        _check_number(r, None)
        if not isinstance(c, (int, float)):
            c * r  # noqa: B018  -- the reference's TypeError at core.py:142
        rel_objs.append(r)
        rel[i] = float(r)
        conf[i] = float(c)
        present[i] = sid in source_reliability
    n = len(signals)
    sid = np.empty(n, np.int32)
    prob = np.empty(n, np.float64)
    for i, s in enumerate(signals):
        sid[i] = rank[s["sourceId"]]
        p = s["probability"]
        if not isinstance(p, (int, float)):
            0 + p  # noqa: B018  -- builtin sum()'s TypeError (core.py:116)
        prob[i] = _as_float(p)

    N.require_gpu()
    dev = N.device()
    T = lambda a: torch.from_numpy(a).to(dev, non_blocking=False)  # noqa: E731
    table = batch.SourceTable.from_arrays(T(rel), T(conf), T(present[:S]), source_ids)
    off = torch.tensor([0, n], dtype=torch.int64, device=dev)
    res = batch.consensus(off, T(sid), T(prob), table, max_len=n if n <= 64 else None, validate=False,
                          check=True)
    cons = float(res.consensus[0].item())
    total = float(res.total_weight[0].item())
    confidence = float(res.confidence[0].item())
    usid = res.usid[:S].cpu().numpy()
    nweight = res.nweight[:S].cpu().numpy()

    null = total == 0  # core.py:131
    source_weights = [
        {"sourceId": source_ids[j], "weight": rel_objs[j], "normalizedWeight": float(nweight[j])}
        for j in range(S)
    ]
    return {
        "schemaVersion": SCHEMA_VERSION,
        "consensus": None if null else cons,
        "confidence": 0.0 if null else confidence,
        "sourceWeights": source_weights,
        "normalization": {"totalWeight": total, "sourceCount": S},
        "diagnostics": {
            "status": "computed",
            "sources": n,
            "uniqueSources": S,
            "coldStartSources": [source_ids[j] for j in range(S) if usid[j] < 0],
        },
    }
