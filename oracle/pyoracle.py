"""ctypes binding of the CPU ORACLE (oracle/libqkdldpc_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker / baseline — never by the product
package.  See ldpc_oracle.h for what it restates and how it is pinned.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libqkdldpc_oracle.so")
if os.environ.get("QLDPC_ASAN") == "1":  # `make asan`: the oracle under ASan + UBSan (build/asan/)
    LIB_PATH = os.path.join(os.path.dirname(_HERE), "build", "asan", "libqkdldpc_oracle.so")
if os.environ.get("QLO_LIB_PATH"):  # tools/oracle_speed.py's timing-split build
    LIB_PATH = os.environ["QLO_LIB_PATH"]


class _Params(ctypes.Structure):
    _fields_ = [("alg", ctypes.c_int32), ("max_iterations", ctypes.c_int32), ("thr_enabled", ctypes.c_int32),
                ("thr", ctypes.c_double), ("primary", ctypes.c_double), ("secondary", ctypes.c_double)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            subprocess.run(["make", "-C", _HERE], check=True, capture_output=True)
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        L.qlo_graph_new.restype = P
        L.qlo_graph_new.argtypes = [ctypes.c_int32, ctypes.c_int32, P, P, P, P]
        L.qlo_graph_free.argtypes = [P]
        L.qlo_syndrome.argtypes = [P, P, P]
        L.qlo_decode.restype = ctypes.c_int32
        L.qlo_decode.argtypes = [P, ctypes.POINTER(_Params), P, P, P, P, P]
        L.qlo_decode_trace.restype = ctypes.c_int32
        L.qlo_decode_trace.argtypes = [P, ctypes.POINTER(_Params), P, P, P, P, P, P]
        L.qlo_decode_batch.argtypes = [P, ctypes.POINTER(_Params), ctypes.c_int32, P, P, P, P, P, P, ctypes.c_int32]
        L.qlo_build_frame.argtypes = [P, P, P, ctypes.c_double, P, P]
        L.qlo_xoshiro.argtypes = [ctypes.c_uint64, ctypes.c_int32, P]
        L.qlo_trial_seeds.argtypes = [ctypes.c_uint64, ctypes.c_int32, P]
        L.qlo_trial.restype = ctypes.c_double
        L.qlo_trial.argtypes = [ctypes.c_int32, ctypes.c_double, ctypes.c_uint64, P, P]
        L.qlo_adapt_code_rate.restype = ctypes.c_int32
        L.qlo_adapt_code_rate.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_double, ctypes.c_double,
                                          ctypes.c_double, ctypes.c_int32, P, ctypes.c_int32, P, P,
                                          ctypes.POINTER(ctypes.c_int32), P, ctypes.POINTER(ctypes.c_int32)]
        L.qlo_trial_rate_adapt.restype = ctypes.c_double
        L.qlo_trial_rate_adapt.argtypes = [ctypes.c_int32, ctypes.c_double, ctypes.c_uint64, ctypes.c_int32, P,
                                           ctypes.c_int32, P, P, P]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data


class Oracle:
    """CPU restatement of the reference decoders for one H matrix."""

    def __init__(self, H):
        self.n, self.m = int(H.n), int(H.m)
        self._keep = [np.ascontiguousarray(x, np.int32) for x in (H.row_ptr, H.col_idx, H.col_ptr, H.row_idx)]
        g = lib().qlo_graph_new(self.n, self.m, *[_p(x) for x in self._keep])
        if not g:
            raise ValueError("inconsistent adjacency lists")
        self._g = ctypes.c_void_p(g)

    def __del__(self):
        try:
            lib().qlo_graph_free(self._g)
        except Exception:
            pass

    @staticmethod
    def params(alg, max_iterations=50, thr_enabled=True, thr=100.0, primary=0.0, secondary=0.0) -> _Params:
        return _Params(int(alg), int(max_iterations), 1 if thr_enabled else 0, float(thr), float(primary),
                       float(secondary))

    def syndrome(self, bits) -> np.ndarray:
        b = np.ascontiguousarray(bits, np.uint8)
        s = np.empty(self.m, np.uint8)
        lib().qlo_syndrome(self._g, _p(b), _p(s))
        return s

    def build_frame(self, alice, bob, qber):
        a = np.ascontiguousarray(alice, np.uint8)
        b = np.ascontiguousarray(bob, np.uint8)
        llr = np.empty(self.n, np.float64)
        s = np.empty(self.m, np.uint8)
        lib().qlo_build_frame(self._g, _p(a), _p(b), float(qber), _p(llr), _p(s))
        return llr, s

    def decode(self, p: _Params, llr, synd, trace: bool = False):
        """-> (bits, iterations, synd_ok, posterior[, trace_posteriors])"""
        l = np.ascontiguousarray(llr, np.float64)
        s = np.ascontiguousarray(synd, np.uint8)
        out = np.empty(self.n, np.uint8)
        post = np.empty(self.n, np.float64)
        ok = ctypes.c_int32()
        if trace:
            tr = np.full((max(int(p.max_iterations), 1), self.n), np.nan)
            it = lib().qlo_decode_trace(self._g, ctypes.byref(p), _p(l), _p(s), _p(out), _p(post), ctypes.byref(ok),
                                        _p(tr))
            return out, int(it), bool(ok.value), post, tr
        it = lib().qlo_decode(self._g, ctypes.byref(p), _p(l), _p(s), _p(out), _p(post), ctypes.byref(ok))
        return out, int(it), bool(ok.value), post

    def decode_batch(self, p: _Params, llr, synd, threads: int = 1, posterior: bool = False):
        l = np.ascontiguousarray(llr, np.float64)
        s = np.ascontiguousarray(synd, np.uint8)
        batch = l.shape[0]
        out = np.empty((batch, self.n), np.uint8)
        it = np.empty(batch, np.uint32)
        ok = np.empty(batch, np.uint8)
        post = np.empty((batch, self.n), np.float64) if posterior else None
        lib().qlo_decode_batch(self._g, ctypes.byref(p), batch, _p(l), _p(s), _p(out), _p(it), _p(ok), _p(post),
                               int(threads))
        return out, it, ok, post


# ---- trial generator (trials_oracle.cpp) ------------------------------------
def xoshiro(seed: int, count: int) -> np.ndarray:
    out = np.empty(count, np.uint64)
    lib().qlo_xoshiro(seed, count, out.ctypes.data)
    return out


def trial_seeds(simulation_seed: int, count: int) -> np.ndarray:
    out = np.empty(count, np.uint64)
    lib().qlo_trial_seeds(simulation_seed, count, out.ctypes.data)
    return out


def trial(n: int, qber: float, seed: int):
    """-> (alice u8[n], bob u8[n], accurate_qber) as run_trial generates them."""
    a = np.empty(n, np.uint8)
    b = np.empty(n, np.uint8)
    q = lib().qlo_trial(n, qber, int(seed) & 0xFFFFFFFFFFFFFFFF, a.ctypes.data, b.ctypes.data)
    return a, b, q


def adapt_code_rate(n, m, qber, delta, efficiency, untainted, state):
    """-> (punctured, shortened) and advances `state` (np.uint64[4]) in place."""
    unt = None if untainted is None else np.ascontiguousarray(untainted, np.int32)
    p = np.empty(n, np.int32)
    s = np.empty(n, np.int32)
    npn, nsn = ctypes.c_int32(0), ctypes.c_int32(0)
    lib().qlo_adapt_code_rate(n, m, qber, delta, efficiency, 0 if unt is None else 1, _p(unt),
                              0 if unt is None else unt.size, state.ctypes.data, p.ctypes.data, ctypes.byref(npn),
                              s.ctypes.data, ctypes.byref(nsn))
    return p[:npn.value].copy(), s[:nsn.value].copy()


def trial_rate_adapt(n, qber, seed, punct, short):
    """-> (alice_ext u8[n], llr f64[n], accurate_qber) of QKD_LDPC_RATE_ADAPT."""
    pa = np.ascontiguousarray(punct, np.int32)
    sh = np.ascontiguousarray(short, np.int32)
    a = np.empty(n, np.uint8)
    llr = np.empty(n, np.float64)
    q = lib().qlo_trial_rate_adapt(n, qber, int(seed) & 0xFFFFFFFFFFFFFFFF, pa.size, pa.ctypes.data, sh.size,
                                   sh.ctypes.data, a.ctypes.data, llr.ctypes.data)
    return a, llr, q
