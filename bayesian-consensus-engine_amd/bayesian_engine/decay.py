"""Drop-in for ``bayesian_engine.decay`` (reference src/bayesian_engine/decay.py:1-185).

The half-life pull toward ``DECAY_MINIMUM`` runs in the ``bce_decay_apply`` kernel
(decay.py:52-58, 90-100: ``2 ** (-t/h)``, ``m + (r-m)*f``, CPython min/max clamping, no
FMA contraction).  ``days_since_update`` parses timestamps, which are host objects
(ISO text / datetime), exactly as the reference does (decay.py:125-145).

Scalars in -> Python floats out; numpy arrays / torch tensors in -> arrays out (one launch).
The early returns for ``elapsed <= 0`` hand back the caller's own object, as the
reference does (decay.py:52-53, 90-91).

Parity note: the reference's ``2.0 ** x`` is glibc ``pow``, which is not correctly
rounded (it differs from a correctly rounded 2^x for ~0.1% of inputs); the GPU restates
glibc's pow(2.0, y) itself (csrc/glibc_pow.hpp), so decayed values are bit-identical to
the reference's.  See DESIGN.md §3.
"""
from __future__ import annotations

from datetime import datetime, timezone
from typing import Union

import numpy as np
import torch

from . import _native as N
from . import batch
from .config import DECAY_HALF_LIFE_DAYS, DECAY_MINIMUM

__all__ = ["compute_decay_factor", "apply_reliability_decay", "days_since_update",
           "decay_reliability_if_needed", "DECAY_HALF_LIFE_DAYS", "DECAY_MINIMUM"]


def _is_array(x) -> bool:
    return isinstance(x, (np.ndarray, torch.Tensor))


def _to_dev(x) -> torch.Tensor:
    if isinstance(x, torch.Tensor):
        return x.to(device=N.device(), dtype=torch.float64).contiguous()
    return torch.as_tensor(np.ascontiguousarray(x, np.float64)).to(N.device())


def _gpu(rel, elapsed, half_life_days, min_rel, want_factor):
    N.require_gpu()
    e = _to_dev(elapsed).reshape(-1)
    r = _to_dev(rel).reshape(-1) if rel is not None else None
    out, fac = batch.decay_apply(r, e, float(half_life_days), float(min_rel), want_factor=want_factor)
    return out, fac


def compute_decay_factor(
    elapsed_days: float,
    half_life_days: float = DECAY_HALF_LIFE_DAYS,
) -> float:
    """2^(-elapsed/half_life); 1.0 for elapsed <= 0 (decay.py:31-58)."""
    if _is_array(elapsed_days):
        _, fac = _gpu(None, elapsed_days, half_life_days, DECAY_MINIMUM, True)
        return fac if isinstance(elapsed_days, torch.Tensor) else fac.cpu().numpy()
    if elapsed_days <= 0:
        return 1.0
    _, fac = _gpu(None, [elapsed_days], half_life_days, DECAY_MINIMUM, True)
    return float(fac[0].item())


def apply_reliability_decay(
    current_reliability: float,
    elapsed_days: float,
    half_life_days: float = DECAY_HALF_LIFE_DAYS,
    min_reliability: float = DECAY_MINIMUM,
) -> float:
    """Decay toward the floor, clamped to [min_reliability, 1] (decay.py:61-100)."""
    if _is_array(elapsed_days) or _is_array(current_reliability):
        e = elapsed_days
        r = current_reliability
        if not _is_array(r):
            r = np.full(np.shape(e), float(r))
        if not _is_array(e):
            e = np.full(np.shape(r), float(e))
        out, _ = _gpu(r, e, half_life_days, min_reliability, False)
        return out if isinstance(elapsed_days, torch.Tensor) else out.cpu().numpy()
    if elapsed_days <= 0:
        return current_reliability
    out, _ = _gpu([current_reliability], [elapsed_days], half_life_days, min_reliability, False)
    return float(out[0].item())


def days_since_update(
    last_updated_at: Union[str, datetime, None],
    now: Union[datetime, None] = None,
) -> float:
    """Days elapsed since a timestamp; 0.0 for falsy/invalid input (decay.py:103-145)."""
    if not last_updated_at:
        return 0.0
    if isinstance(last_updated_at, str):
        try:
            last_updated = datetime.fromisoformat(last_updated_at)
        except ValueError:
            return 0.0
    else:
        last_updated = last_updated_at
    if now is None:
        now = datetime.now(timezone.utc)
    if last_updated.tzinfo is None:
        last_updated = last_updated.replace(tzinfo=timezone.utc)
    elapsed = now - last_updated
    return max(0.0, elapsed.total_seconds() / 86400.0)


def decay_reliability_if_needed(
    current_reliability: float,
    last_updated_at: Union[str, datetime, None],
    now: Union[datetime, None] = None,
    half_life_days: float = DECAY_HALF_LIFE_DAYS,
    min_reliability: float = DECAY_MINIMUM,
) -> tuple[float, bool]:
    """(decayed, was_decayed) (decay.py:148-185)."""
    elapsed = days_since_update(last_updated_at, now)
    if elapsed <= 0:
        return current_reliability, False
    decayed = apply_reliability_decay(current_reliability, elapsed, half_life_days, min_reliability)
    return decayed, decayed != current_reliability
