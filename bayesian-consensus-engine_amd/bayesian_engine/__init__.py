"""MI355X-native drop-in for the ``bayesian_engine`` package (reference __init__.py:1-4).

Modules mirror the reference: ``core``, ``decay``, ``reliability``, ``tiebreak``,
``market``, ``cli``, ``config``.  ``batch`` is the new batched entry point over millions
of markets; ``_native`` binds the C ABI of ``lib/libbce_hip.so`` (include/bce.h).
Importing the package never touches the GPU; the first compute call does, and raises
``NativeUnavailable`` when the HIP library or a GPU is missing (no CPU fallback).
"""

__version__ = "0.1.0"
