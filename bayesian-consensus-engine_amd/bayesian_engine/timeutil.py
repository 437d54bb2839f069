"""Host-side timestamp handling: ISO-8601 text <-> int64 microseconds since the Unix epoch.

The reference stores ``updated_at`` as ISO text and parses it on every read
(``decay.py:140-145``, ``reliability.py:115-116``).  The engine parses once at bulk
load and keeps int64 microseconds in HBM; elapsed days are then
``(double)(now_us - t_us) / 1e6 / 86400.0`` on the GPU, which equals
``timedelta.total_seconds() / 86400.0`` bit for bit (int-microseconds / 10**6 is
correctly rounded in both).
"""
from __future__ import annotations

from datetime import datetime, timezone
from typing import Sequence, Union

import numpy as np

NO_TIMESTAMP = -(2**63)  # "falsy or unparseable" -> days_since_update returns 0.0
_EPOCH = datetime(1970, 1, 1, tzinfo=timezone.utc)


def dt_to_us(dt: datetime) -> int:
    if dt.tzinfo is None:  # decay.py:139-141: naive means UTC
        dt = dt.replace(tzinfo=timezone.utc)
    d = dt - _EPOCH
    return (d.days * 86400 + d.seconds) * 1_000_000 + d.microseconds


def iso_to_us(value: Union[str, datetime, None]) -> int:
    """Mirror of decay.days_since_update's parsing (decay.py:125-141)."""
    if not value:
        return NO_TIMESTAMP
    if isinstance(value, str):
        try:
            value = datetime.fromisoformat(value)
        except ValueError:
            return NO_TIMESTAMP
    return dt_to_us(value)


def iso_to_us_many(values: Sequence[Union[str, datetime, None]]) -> np.ndarray:
    """``[iso_to_us(v) for v in values]`` as int64.  (A numpy datetime64 parse of the UTC
    stamps was measured slower than CPython's C ``fromisoformat``: 0.73 vs 0.58 s per 1M.)"""
    return np.fromiter(map(iso_to_us, values), np.int64, len(values))


def us_to_iso(us: int) -> str:
    """Inverse used for write-back: datetime.now(timezone.utc).isoformat() style."""
    from datetime import timedelta

    return (_EPOCH + timedelta(microseconds=int(us))).isoformat()


def now_us() -> int:
    return dt_to_us(datetime.now(timezone.utc))
