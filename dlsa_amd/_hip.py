"""ctypes binding of libdlsa_hip.so (C-ABI declared in include/dlsa_hip.h).

The shared library is built in-tree (``python -m dlsa_amd.build`` or
``__graft_entry__.build()``) and loaded from this package directory.  There is
no fallback: if the library is missing or fails to load, every product entry
point raises ``DlsaHipError`` -- the HIP kernels are the only implementation of
the map stage.
"""

from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# DLSA_LIB: profiling variants (tools/build_variants.sh); default the in-tree build
LIB_PATH = os.environ.get("DLSA_LIB") or os.path.join(_HERE, "libdlsa_hip.so")

DLSA_OK = 0
STATUS_NAMES = {0: "ok", 1: "maxiter", 2: "singular", 3: "empty", 4: "nonfinite", 5: "missing_level"}
HESSIAN_MIXED = 0
HESSIAN_FP64 = 1
HESSIAN_MIXED_F32 = 2
EXACT_AUTO = 0   # exact (Sig_inv) pass on the int8 cores where it applies
EXACT_FP64 = 1   # exact pass on the fp64 MFMA
MAX_P_FUSED = 192
MAX_P = 512


class DlsaHipError(RuntimeError):
    """Raised when libdlsa_hip.so is unavailable or a call fails."""


class FitOptions(ctypes.Structure):
    _fields_ = [
        ("hessian_mode", ctypes.c_int32),
        ("record_timing", ctypes.c_int32),
        ("switch_tol", ctypes.c_double),
        ("workspace", ctypes.c_void_p),
        ("workspace_bytes", ctypes.c_int64),
        ("rows_per_chunk", ctypes.c_int32),
        ("warm_start", ctypes.c_int32),
        ("exact_pass", ctypes.c_int32),
        ("exact_waves", ctypes.c_int32),
        ("oz_max_bytes", ctypes.c_int64),
        ("reserved", ctypes.c_int32 * 2),
    ]


class FitStats(ctypes.Structure):
    _fields_ = [
        ("iterations", ctypes.c_int32),
        ("passes_fp32", ctypes.c_int32),
        ("passes_fp64", ctypes.c_int32),
        ("n_chunks", ctypes.c_int32),
        ("ms_pass_fp32", ctypes.c_double),
        ("ms_pass_fp64", ctypes.c_double),
        ("ms_solve", ctypes.c_double),
        ("ms_total", ctypes.c_double),
        ("rows_fp32", ctypes.c_int64),
        ("rows_fp64", ctypes.c_int64),
        ("ms_wide_row", ctypes.c_double),
        ("ms_wide_gram", ctypes.c_double),
        ("ms_wide_assemble", ctypes.c_double),
        ("passes_f32x", ctypes.c_int32),
        ("polish_partitions", ctypes.c_int32),
        ("passes_oz", ctypes.c_int32),
        ("oz_fallbacks", ctypes.c_int32),
        ("oz_stale_partitions", ctypes.c_int32),
    ]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64
_F64 = ctypes.c_double

# name -> (restype, argtypes); every symbol include/dlsa_hip.h declares
SIGNATURES = {
    "dlsa_fit_options_default": (None, [ctypes.POINTER(FitOptions)]),
    "dlsa_logistic_workspace_bytes": (_I64, [_P, _I32, _I32, _I32, _I32]),
    "dlsa_logistic_fit_batched": (
        ctypes.c_int,
        [_P, _P, _P, _I32, _I32, _I32, _P, _P, _I32, _F64, _P, _P, _P, _P, _P, _P, _P]),
    "dlsa_logistic_fit_batched_ex": (
        ctypes.c_int,
        [_P, _P, _P, _I32, _I32, _I32, _P, _P, _I32, _F64, _P, _P, _P, _P, _P, _P,
         ctypes.POINTER(FitOptions), _P]),
    "dlsa_ols_fit_batched": (
        ctypes.c_int,
        [_P, _P, _P, _I32, _I32, _I32, _P, _P, _P, _P, _P, _P, _P, ctypes.POINTER(FitOptions),
         _P]),
    "dlsa_logistic_loglik_batched": (
        ctypes.c_int, [_P, _P, _P, _I32, _I32, _I32, _P, _P, _P, _I32, _P, _P]),
    "dlsa_logistic_fit_categorical": (
        ctypes.c_int,
        [_P, _P, _P, _P, _I32, _I32, _I32, _P, _I32, _P, _P, _I32, _F64, _P, _P, _P, _P, _P, _P,
         ctypes.POINTER(FitOptions), _P]),
    "dlsa_partition_rows": (ctypes.c_int, [_P, _I64, _I32, _I32, _P, _P, _P, _P, _P, _P]),
    "dlsa_last_fit_stats": (ctypes.c_int, [ctypes.POINTER(FitStats)]),
    "dlsa_reduce_partitions": (ctypes.c_int, [_P, _P, _P, _I32, _I32, _P, _P]),
    "dlsa_simulate_logistic": (ctypes.c_int, [_P, _P, _I64, _I32, ctypes.c_uint64, _I64, _P]),
    "dlsa_column_moments": (ctypes.c_int, [_P, _I64, _I32, _P, _P]),
    "dlsa_lars_lsa": (ctypes.c_int, [_P, _P, _I32, _I32, _F64, _I32, _F64, _I32, _P, _P, _P,
                                     _P, _P]),
    "dlsa_last_error": (ctypes.c_char_p, []),
    "dlsa_build_info": (ctypes.c_char_p, []),
}

_lib = None
_lock = threading.Lock()


def load():
    """Load libdlsa_hip.so (once).  Raises DlsaHipError if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise DlsaHipError(
                f"{LIB_PATH} not found: build it with `python -m dlsa_amd.build` "
                "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
        try:
            lib = ctypes.CDLL(LIB_PATH)
        except OSError as e:  # pragma: no cover - environment dependent
            raise DlsaHipError(f"cannot load {LIB_PATH}: {e}") from e
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def last_error() -> str:
    return load().dlsa_last_error().decode()


def check(rc: int, what: str):
    if rc != DLSA_OK:
        raise DlsaHipError(f"{what} failed ({rc}): {last_error()}")


def default_options() -> FitOptions:
    opt = FitOptions()
    load().dlsa_fit_options_default(ctypes.byref(opt))
    return opt


def last_fit_stats() -> dict:
    st = FitStats()
    check(load().dlsa_last_fit_stats(ctypes.byref(st)), "dlsa_last_fit_stats")
    return st.as_dict()
