"""ctypes binding of libqkdldpc_hip.so (include/qkd_ldpc_hip.h).

The shared library is the product: HIP kernels for gfx950 plus the C ABI.  This
module only marshals numpy arrays / torch device pointers into it.  If the
library is missing the import of any entry point raises: there is no CPU
fallback anywhere in the package.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libqkdldpc_hip.so")
# Alternative builds are selected only under the diagnostic switch QLDPC_DIAG=1
# (the library reads its A/B knobs under the same switch): without it the
# product library is loaded whatever else the environment holds.
DIAG = os.environ.get("QLDPC_DIAG") == "1"
_AB_BUILD = os.environ.get("QLDPC_AB_BUILD") if DIAG else None
if DIAG and os.environ.get("QLDPC_DIAG_STAMPS") == "1":  # diagnostic phase-stamp build (Makefile target `stamps`)
    LIB_PATH = os.path.join(_HERE, "diag", "libqkdldpc_hip.so")
if _AB_BUILD:  # A/B experiments: an alternative in-tree build, qkd_ldpc_v_amd/ab/<name>/
    LIB_PATH = os.path.join(_HERE, "ab", _AB_BUILD, "libqkdldpc_hip.so")
if DIAG and os.environ.get("QLDPC_ASAN") == "1":  # `make asan`: host code under ASan + UBSan (build/asan/)
    LIB_PATH = os.path.join(os.path.dirname(_HERE), "build", "asan", "libqkdldpc_hip.so")

QLDPC_OK = 0
ERROR_NAMES = {-1: "EINVAL", -2: "EHIP", -3: "EIO", -4: "ENOMEM", -5: "EUNSUP"}

SPA, SPA_LIN, NMSA, OMSA, ANMSA, AOMSA = range(6)
ALGORITHM_NAMES = {SPA: "SPA", SPA_LIN: "SPA(lin approx)", NMSA: "NMSA", OMSA: "OMSA", ANMSA: "ANMSA", AOMSA: "AOMSA"}
MAT_UNCOMPRESSED, MAT_ALIST, MAT_SPARSE_1, MAT_SPARSE_2 = range(4)


class QLDPCError(RuntimeError):
    """A C-ABI call failed; carries the code and qldpc_last_error()."""

    def __init__(self, code: int, where: str, message: str):
        super().__init__(f"{where}: {ERROR_NAMES.get(code, code)}: {message}")
        self.code = code


class qldpc_params(ctypes.Structure):
    _fields_ = [
        ("algorithm", ctypes.c_int32),
        ("max_iterations", ctypes.c_int32),
        ("thr_enabled", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
        ("thr", ctypes.c_double),
        ("primary", ctypes.c_double),
        ("secondary", ctypes.c_double),
    ]


_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_PI32 = ctypes.POINTER(ctypes.c_int32)

# name -> (restype, argtypes)
_SIGNATURES = {
    "qldpc_load_matrix": (_I32, [ctypes.c_char_p, _I32, _PI32, _PI32, _PI32, _P, _P, _P, _P, _PI32]),
    "qldpc_graph_create": (_I32, [_I32, _I32, _P, _P, _I32, ctypes.POINTER(_P)]),
    "qldpc_graph_create_checked": (_I32, [_I32, _I32, _P, _P, _P, _P, _I32, ctypes.POINTER(_P)]),
    "qldpc_graph_create_on": (_I32, [_I32, _I32, _P, _P, _P, _I32, ctypes.POINTER(_P)]),
    "qldpc_graph_create_checked_on": (_I32, [_I32, _I32, _P, _P, _P, _P, _P, _I32, ctypes.POINTER(_P)]),
    "qldpc_graph_create_host": (_I32, [_I32, _I32, _P, _P, ctypes.POINTER(_P)]),
    "qldpc_graph_labels": (_I32, [_P, _P, _P]),
    "qldpc_graph_destroy": (None, [_P]),
    "qldpc_set_kernel_timing": (_I32, [_P, _I32]),
    "qldpc_last_decode_kernel_ms": (_I32, [_P, _I32, _P, ctypes.POINTER(ctypes.c_float)]),
    "qldpc_last_claim_order": (_I32, [_P, _I32, _P, _P, _P, _I32, _PI32]),
    "qldpc_graph_info": (_I32, [_P, _PI32, _PI32, _PI32, _PI32]),
    "qldpc_graph_plan": (_I32, [_P, _I32, _I32, _PI32, _PI32, _PI32, _PI32, ctypes.POINTER(ctypes.c_char_p)]),
    "qldpc_graph_split_plan": (_I32, [_P, _PI32, _PI32, _PI32]),
    "qldpc_decode_batch": (_I32, [_P, ctypes.POINTER(qldpc_params), _I32, _P, _P, _P, _P, _P, _P]),
    "qldpc_decode_batch_device": (_I32, [_P, _I32, ctypes.POINTER(qldpc_params), _I32, _P, _P, _P, _P, _P, _P, _P]),
    "qldpc_build_frames_device": (_I32, [_P, _I32, _I32, _P, _P, _P, _P, _P, _P]),
    "qldpc_log_p": (ctypes.c_double, [ctypes.c_double]),
    "qldpc_keys_match_device": (_I32, [_I32, _I32, _P, _P, _P, _P]),
    "qldpc_qkd_ldpc_batch_device": (
        _I32,
        [_P, _I32, ctypes.POINTER(qldpc_params), _I32, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P],
    ),
    "qldpc_selftest_math_device": (_I32, [_I32, _I32, _P, _P, _P]),
    "qldpc_trial_seeds": (_I32, [ctypes.c_uint64, _I32, _P]),
    "qldpc_xoshiro_jump": (_I32, [ctypes.c_uint64, ctypes.c_uint64, _P]),
    "qldpc_xoshiro_state": (_I32, [ctypes.c_uint64, _P]),
    "qldpc_sort_permutation": (_I32, [_P, _I32, _P]),
    "qldpc_bits_to_remove": (_I32, [_I32, _I32, _P, _P, _I32, _P, _I32, _P, _I32, _P, _PI32]),
    "qldpc_adapt_code_rate": (_I32, [_I32, _I32, ctypes.c_double, ctypes.c_double, ctypes.c_double, _I32, _P, _I32,
                                     _P, _P, _PI32, _P, _PI32, ctypes.POINTER(ctypes.c_double)]),
    "qldpc_select_punctured_untainted": (_I32, [_I32, _I32, _P, _P, _P, _P, _P, _P, _PI32]),
    "qldpc_rate_plan_create": (_I32, [_P, _I32, _P, _I32, _P, ctypes.POINTER(_P)]),
    "qldpc_rate_plan_destroy": (None, [_P]),
    "qldpc_trials_rate_adapt_device": (_I32, [_I32, ctypes.c_double, _I32, _P, ctypes.c_uint64, _I32, _P, _P, _P,
                                              _P, ctypes.POINTER(ctypes.c_double), _P]),
    "qldpc_build_frames_rate_adapt_device": (_I32, [_P, _P, _I32, _I32, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "qldpc_qkd_ldpc_rate_adapt_batch_device": (_I32, [_P, _P, _I32, ctypes.POINTER(qldpc_params), _I32, _P, _P, _P,
                                                      _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "qldpc_trials_device": (_I32, [_I32, ctypes.c_double, _I32, _P, ctypes.c_uint64, _P, _P,
                                   ctypes.POINTER(ctypes.c_double), _P]),
    "qldpc_run_trials": (_I32, [_P, _P, ctypes.POINTER(qldpc_params), ctypes.c_double, _I32, _P, ctypes.c_uint64,
                                _P, _P, _P, _P, ctypes.POINTER(ctypes.c_double)]),
    "qldpc_run_trials_submit": (_I32, [_P, _P, ctypes.POINTER(qldpc_params), ctypes.c_double, _I32, _P,
                                       ctypes.c_uint64, _P, _P, _P, _P, ctypes.POINTER(ctypes.c_double),
                                       ctypes.POINTER(_P)]),
    "qldpc_run_trials_wait": (_I32, [_P]),
    "qldpc_shard_range": (_I32, [_I32, _I32, _I32, _PI32, _PI32]),
    "qldpc_device_count": (_I32, [_PI32]),
    "qldpc_last_error": (ctypes.c_char_p, []),
    "qldpc_version": (ctypes.c_char_p, []),
}

_lib = None


def lib() -> ctypes.CDLL:
    """Load the HIP library once; raise loudly when it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with `make` (or __graft_entry__.build()); "
                "qkd_ldpc_v_amd has no CPU fallback"
            )
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(L, name, None)
            if fn is None and _AB_BUILD:
                continue  # an older A/B build may predate an entry point
            if fn is None:
                raise ImportError(f"{LIB_PATH} does not export {name}: rebuild it (make)")
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def exported_symbols() -> list[str]:
    return list(_SIGNATURES)


def check(rc: int, where: str) -> None:
    if rc != QLDPC_OK:
        raise QLDPCError(rc, where, lib().qldpc_last_error().decode(errors="replace"))


def ptr(a: np.ndarray | None) -> int | None:
    if a is None:
        return None
    if not a.flags.c_contiguous:
        raise ValueError("arrays passed to the C ABI must be C-contiguous")
    return a.ctypes.data


def version() -> str:
    return lib().qldpc_version().decode()


def log_p(qber: float) -> float:
    """log((1-q)/q) evaluated by the host C library (reference :1043)."""
    return lib().qldpc_log_p(float(qber))


@dataclass
class Params:
    """Decoder parameters (qldpc_params)."""

    algorithm: int = SPA
    max_iterations: int = 50
    thr_enabled: bool = True
    thr: float = 100.0
    primary: float = 0.0
    secondary: float = 0.0

    def c(self) -> qldpc_params:
        return qldpc_params(
            int(self.algorithm), int(self.max_iterations), 1 if self.thr_enabled else 0, 0,
            float(self.thr), float(self.primary), float(self.secondary),
        )
