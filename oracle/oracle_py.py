"""oracle_py — ctypes binding of the CPU oracle (oracle/_build/liboracle.so).

TEST INFRASTRUCTURE ONLY.  Imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the product.  See icp_oracle.h for what the oracle restates
(reference src/cpu.cc) and how it is pinned.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
CLI_PATH = os.path.join(_HERE, "_build", "icp_oracle")

NN_SQUARED = 0
NN_CPU_SQRT = 1

_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


class Alignment(C.Structure):
    _fields_ = [("s", C.c_double), ("R", C.c_double * 9), ("t", C.c_double * 3),
                ("err", C.c_double), ("mu_p", C.c_double * 3), ("mu_y", C.c_double * 3),
                ("S", C.c_double * 9), ("Nm", C.c_double * 16), ("evals", C.c_double * 4),
                ("pick", C.c_int), ("d_caps", C.c_double), ("sp", C.c_double)]


class Trace(C.Structure):
    _fields_ = [("err", C.POINTER(C.c_double)), ("s", C.POINTER(C.c_double)),
                ("R", C.POINTER(C.c_double)), ("t", C.POINTER(C.c_double)),
                ("idx0", C.POINTER(C.c_int32))]


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        dp = C.POINTER(C.c_double)
        ip = C.POINTER(C.c_int32)
        sz = C.c_size_t
        L.oracle_closest.argtypes = [dp, sz, dp, sz, C.c_int, ip, dp]
        L.oracle_closest_range.argtypes = [dp, sz, sz, dp, sz, C.c_int, ip, dp]
        L.oracle_closest_range_blocked.argtypes = [dp, sz, sz, dp, sz, ip, dp]
        L.oracle_max_element_index.argtypes = [dp]
        L.oracle_eig_sym4.argtypes = [dp, dp, dp]
        L.oracle_find_alignment.argtypes = [dp, dp, sz, C.POINTER(Alignment)]
        L.oracle_err_compute.argtypes = [dp, dp, sz, C.c_double, dp, dp]
        L.oracle_err_compute.restype = C.c_double
        L.oracle_err_compute_alignment.argtypes = [dp, dp, sz, C.c_double, dp, dp]
        L.oracle_err_compute_alignment.restype = C.c_double
        L.oracle_icp.argtypes = [dp, sz, dp, sz, C.c_int, C.c_double, C.c_int, C.c_int, C.POINTER(Trace)]
        L.oracle_load_matrix.argtypes = [C.c_char_p, C.POINTER(sz)]
        L.oracle_load_matrix.restype = C.c_void_p
        L.oracle_write_matrix.argtypes = [C.c_char_p, dp, sz]
        _lib = L
    return _lib


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _cloud(a):
    a = np.ascontiguousarray(a, dtype=np.float64)
    assert a.ndim == 2 and a.shape[1] == 3
    return a


def closest(p, m, nn_mode: int = NN_SQUARED, j0: int = 0, j1: int | None = None):
    """cpu.cc:5-27 -> (Y, idx) for scene rows [j0, j1)."""
    p = _cloud(p); m = _cloud(m)
    j1 = p.shape[0] if j1 is None else j1
    idx = np.zeros(p.shape[0], dtype=np.int32)
    y = np.zeros_like(p)
    lib().oracle_closest_range(_dp(p), j0, j1, _dp(m), m.shape[0], nn_mode,
                               idx.ctypes.data_as(C.POINTER(C.c_int32)), _dp(y))
    return y[j0:j1], idx[j0:j1]


def closest_blocked(p, m, j0: int = 0, j1: int | None = None):
    """closest(p, m, NN_SQUARED, j0, j1), SIMD-blocked (icp_oracle_fast.c; finite inputs)."""
    p = _cloud(p); m = _cloud(m)
    j1 = p.shape[0] if j1 is None else j1
    idx = np.zeros(p.shape[0], dtype=np.int32)
    y = np.zeros_like(p)
    lib().oracle_closest_range_blocked(_dp(p), j0, j1, _dp(m), m.shape[0],
                                       idx.ctypes.data_as(C.POINTER(C.c_int32)), _dp(y))
    return y[j0:j1], idx[j0:j1]


def find_alignment(p, y) -> Alignment:
    p = _cloud(p); y = _cloud(y)
    out = Alignment()
    lib().oracle_find_alignment(_dp(p), _dp(y), p.shape[0], C.byref(out))
    return out


def err_compute(p, Y, s, R, t):
    """cpu.cc:29-40: returns (err, p_after)."""
    p = _cloud(p).copy(); Y = _cloud(Y)
    R = np.ascontiguousarray(R, dtype=np.float64).reshape(9); t = np.ascontiguousarray(t, dtype=np.float64)
    e = lib().oracle_err_compute(_dp(p), _dp(Y), p.shape[0], float(s), _dp(R), _dp(t))
    return e, p


def err_compute_alignment(p, y, s, R, t):
    p = _cloud(p); y = _cloud(y)
    R = np.ascontiguousarray(R, dtype=np.float64).reshape(9); t = np.ascontiguousarray(t, dtype=np.float64)
    return lib().oracle_err_compute_alignment(_dp(p), _dp(y), p.shape[0], float(s), _dp(R), _dp(t))


def max_element_index(ev) -> int:
    ev = np.ascontiguousarray(ev, dtype=np.float64)
    return lib().oracle_max_element_index(_dp(ev))


def eig_sym4(N):
    N = np.ascontiguousarray(N, dtype=np.float64).reshape(16)
    ev = np.zeros(4); V = np.zeros(16)
    lib().oracle_eig_sym4(_dp(N), _dp(ev), _dp(V))
    return ev, V.reshape(4, 4).T  # columns = eigenvectors


def icp(m, p, max_iter: int, threshold: float = 1e-5, nn_mode: int = NN_SQUARED,
        allow_unequal: bool = False, want_idx0: bool = False):
    """cpu.cc:55-79 -> dict(iterations, new_p, err, s, R, t[, idx0]); raises on the
    reference's fatal checks (np != nm -> 'size', np < 4 -> 'few')."""
    m = _cloud(m); p = _cloud(p).copy()
    n = max(max_iter, 1)
    err = np.zeros(n); s = np.zeros(n); R = np.zeros((n, 9)); t = np.zeros((n, 3))
    idx0 = np.zeros(p.shape[0], dtype=np.int32) if want_idx0 else None
    tr = Trace(_dp(err), _dp(s), _dp(R), _dp(t),
               idx0.ctypes.data_as(C.POINTER(C.c_int32)) if want_idx0 else None)
    it = lib().oracle_icp(_dp(m), m.shape[0], _dp(p), p.shape[0], max_iter, threshold, nn_mode,
                          1 if allow_unequal else 0, C.byref(tr))
    if it == -1:
        raise ValueError("size")
    if it == -2:
        raise ValueError("few")
    out = dict(iterations=it, new_p=p, err=err[:it], s=s[:it], R=R[:it].reshape(-1, 3, 3), t=t[:it])
    if want_idx0:
        out["idx0"] = idx0
    return out


def load_matrix(path: str) -> np.ndarray:
    n = C.c_size_t(0)
    ptr = lib().oracle_load_matrix(path.encode(), C.byref(n))
    if not ptr:
        raise FileNotFoundError(path)
    arr = np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_double)), shape=(max(n.value, 1) * 3,))
    out = arr[: n.value * 3].copy().reshape(n.value, 3)
    C.CDLL(None).free(C.c_void_p(ptr))
    return out
