"""ctypes binding of libbce_hip.so (the C ABI declared in include/bce.h).

PyTorch is only plumbing here: it owns device memory and the current HIP stream.  The
library is loaded AFTER ``import torch`` so both share one HIP runtime (torch ships
libamdhip64.so.7 with the same SONAME the library links against).

There is no CPU fallback.  Every compute entry point calls :func:`require_gpu`, which
raises :class:`NativeUnavailable` when the built library or a GPU is missing.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import torch

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("BCE_LIB", os.path.join(_PKG_ROOT, "lib", "libbce_hip.so"))

BCE_OK = 0
MODE_EXACT = 0
MODE_FAST = 1
NBINS = 13  # include/bce.h BCE_NBINS
NO_TIMESTAMP = -(2**63)
TB_LABELS = {0: "unanimous", 1: "weight_density", 2: "prediction_value_smallest", 3: "unanimous"}


class NativeUnavailable(RuntimeError):
    """The HIP engine cannot run here (library not built, or no GPU)."""


class BCEError(RuntimeError):
    """A library call returned a non-zero status."""


_lib = None
_lock = threading.Lock()

_vp = C.c_void_p
_i64 = C.c_int64
_i32 = C.c_int32
_f64 = C.c_double

_SIGS = {
    "bce_abi_version": (C.c_int, []),
    "bce_last_error": (C.c_char_p, []),
    "bce_device_count": (C.c_int, []),
    "bce_fault_check": (C.c_int, [_vp]),
    "bce_debug_set_spin_cap": (C.c_int, [C.c_int]),
    "bce_debug_lane_selftest": (C.c_int, [_vp, _vp]),
    "bce_debug_py_round": (_f64, [_f64, _i32, _vp]),
    "bce_jsonl_parse": (C.c_int, [_vp, _i64, _i32, _vp]),
    "bce_jsonl_counts": (C.c_int, [_vp, _vp]),
    "bce_jsonl_arrays": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "bce_jsonl_render": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _i32, _vp,
                                   _vp, _vp, _vp]),
    "bce_jsonl_free": (None, [_vp]),
    "bce_debug_float_repr": (_i32, [_f64, _vp, _i32]),
    "bce_consensus_csr": (C.c_int, [_vp, _i64, _vp, _vp, _i64, _vp, _vp, _i32, _vp, _i64, _i32,
                                    _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "bce_table_pack": (C.c_int, [_i64, _vp, _vp, _vp, _vp, _vp, _vp]),
    "bce_validate_csr": (C.c_int, [_vp, _i64, _vp, _vp, _vp]),
    "bce_plan_bins": (C.c_int, [_vp, _i64, _vp, _vp, _vp]),
    "bce_consensus_scratch_bytes": (C.c_int64, [_vp, _vp, _vp]),
    "bce_plan_bins_device": (C.c_int, [_vp, _i64, _vp, _vp, _vp, _vp, _vp, _i64, _vp]),
    "bce_plan_device_scratch_bytes": (_i64, [_i64]),
    "bce_plan_bins_device_async": (C.c_int, [_vp, _i64, _vp, _vp, _vp, _i64, _vp]),
    "bce_consensus_planned_device": (C.c_int, [_vp, _i64, _vp, _vp, _i64, _vp, _vp, _i32, _vp, _vp, _i32,
                                               _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "bce_consensus_planned": (C.c_int, [_vp, _i64, _vp, _vp, _i64, _vp, _vp, _i32, _vp, _vp, _i32,
                                        _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp]),
    "bce_decay_view": (C.c_int, [_i64, _vp, _vp, _vp, _i64, _f64, _f64, _f64, _vp, _vp]),
    "bce_decay_apply": (C.c_int, [_i64, _vp, _vp, _f64, _f64, _vp, _vp, _vp]),
    "bce_outcome_update": (C.c_int, [_i64, _vp, _vp, _vp, _vp, _vp, _i64, _f64, _f64, _vp]),
    "bce_replay_step": (C.c_int, [_i64, _vp, _vp, _vp, _vp, _vp, _i64, _f64, _f64, _f64, _f64, _vp, _vp]),
    "bce_tiebreak_csr": (C.c_int, [_vp, _i64, _vp, _i64, _vp, _vp, _vp, _vp, _i32, _i32, _vp, _vp, _vp, _vp,
                                   _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "bce_tiebreak_csr_long": (C.c_int, [_vp, _i64, _vp, _i64, _i32, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp,
                                        _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "bce_agreement_stats": (C.c_int, [_vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp]),
    "bce_reestimate_consensus": (C.c_int, [_vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp]),
    "bce_reestimate_agreement": (C.c_int, [_vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp]),
    "bce_reestimate_weights": (C.c_int, [_i64, _vp, _vp, _vp, _vp]),
    "bce_reestimate_consensus_votes": (C.c_int, [_vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "bce_reestimate_agreement_votes": (C.c_int, [_vp, _i64, _i64, _vp, _vp, _vp, _vp, _vp]),
    "bce_reestimate_consensus_votes_mfma": (C.c_int, [_vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                                      _i64, _vp]),
    "bce_reestimate_mfma_scratch_bytes": (_i64, [_i64]),
    "bce_namespace_resolve": (C.c_int, [_i64] + [_vp] * 12 + [_i32, _i64, _f64, _f64, _f64, _f64, _i32,
                                                               _vp, _vp, _vp, _vp]),
    "bce_aggregate_groups": (C.c_int, [_vp, _i64, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
}

EXPORTED = tuple(_SIGS)


def load_library(path: str = LIB_PATH) -> C.CDLL:
    """dlopen the library and declare every signature (works without a GPU)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(path):
                raise NativeUnavailable(
                    f"libbce_hip.so not built at {path}: run __graft_entry__.build() "
                    "(hipcc --offload-arch=gfx950)")
            lib = C.CDLL(path)
            for name, (res, args) in _SIGS.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = lib
    return _lib


def lib() -> C.CDLL:
    return _lib if _lib is not None else load_library()


def require_gpu() -> C.CDLL:
    """The engine's only entry gate: native library + a visible GPU, or raise."""
    L = lib()
    if not torch.cuda.is_available():
        raise NativeUnavailable("bayesian_engine (MI355X build) needs a ROCm GPU; none is visible")
    return L


def check(rc: int, what: str = "") -> None:
    if rc != BCE_OK:
        msg = lib().bce_last_error().decode(errors="replace")
        raise BCEError(f"{what or 'bce call'} failed (status {rc}): {msg}")


def check_faults(device=None, what: str = "") -> None:
    """Synchronise the current stream and raise :class:`BCEError` if a kernel recorded a
    device fault (bce_fault_check): a persistent wave that gave up waiting, a sid >=
    n_sources, a market longer than the max_len it was launched with."""
    check(lib().bce_fault_check(stream(device)), what or "device fault check")


def ptr(t, row_strided: bool = False) -> C.c_void_p:
    """Device (or host numpy) pointer of a contiguous buffer; None -> NULL.

    ``row_strided``: a 2-D tensor whose rows are contiguous but may be padded (the
    callee takes the leading dimension separately)."""
    if t is None:
        return C.c_void_p(0)
    if isinstance(t, torch.Tensor):
        if row_strided:
            assert t.dim() == 2 and t.stride(1) == 1 and t.stride(0) >= t.shape[1], "rows must be contiguous"
        else:
            assert t.is_contiguous(), "tensor must be contiguous"
        return C.c_void_p(t.data_ptr())
    return C.c_void_p(t.ctypes.data)  # numpy (host arrays for planning calls)


def stream(device=None) -> C.c_void_p:
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def device() -> torch.device:
    return torch.device("cuda", torch.cuda.current_device())
