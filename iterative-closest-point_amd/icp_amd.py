"""icp_amd — Python mirror of the reference's src/GPU interface over libicp_hip.so.

The product is the C-ABI library (include/icp_capi.h) built from csrc/; this module only
binds it with ctypes so tests, bench.py and the graft entry point can drive it.  Names
follow the reference (yassram/iterative-closest-point):

  ICP(m, p, max_iter).find_corresponding_opti()   src/GPU/gpu.cc:52-83
  ICP.find_alignment(y)                            src/GPU/gpu.cc:95-151
  compute_Y_w_opti(m, p)                           src/GPU/compute.cu:154-245
  compute_err_w(Y, p, in_place, sr, t)             src/GPU/compute.cu:348-379
  compute_centroid(M)  (mean + substract_col_w)   src/GPU/compute.cu:400-416
  y_p_norm_w(y, p)                                 src/GPU/compute.cu:442-469
  load_matrix / write_matrix                       src/load.cc:3-97

Clouds are numpy float64 arrays of shape (n, 3) here (row = point).  That is the same
memory as the reference's 3 x n column-major Eigen matrix, so no copy is needed at the
C boundary.  There is NO CPU fallback: if libicp_hip.so is missing or no HIP device is
visible, every compute call raises.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ICP_AMD_LIB") or os.path.join(_HERE, "build", "libicp_hip.so")

ICP_OK = 0
ICP_E_ARG = -1
ICP_E_HIP = -2
ICP_E_SIZE_MISMATCH = -3
ICP_E_TOO_FEW_POINTS = -4
ICP_E_NO_MODEL = -5
ICP_E_RCCL = -6
ICP_E_NO_DEVICE = -7
ICP_E_IO = -8
ICP_E_RANGE = -9

NN_CERTIFIED = 0
NN_FP64 = 1
VARIANT_AUTO = 0
VARIANT_VALU = 1
VARIANT_MFMA = 2
VARIANT_MFMA16 = 3
VARIANT_GRID = 4  # exact grid NN for every query
VARIANT_BUNDLE = 5  # f16 pair filter behind the per-(query, 32-point bundle) MFMA bound
RULE_SQUARED = 0    # icp_set_nn_rule: the reference GPU path's squared distance (default)
RULE_CPU_SQRT = 1   # the reference CPU path's sqrt(pow) distance (src/cpu.cc:17-22)
RUN_AUTO = 0        # icp_set_run_mode: one launch for eligible small runs, else the launch loop
RUN_LAUNCHES = 1
RUN_PERSISTENT = 2

# every function include/icp_capi.h declares (checked by tests/test_capi.py)
EXPORTED = [
    "icp_ctx_create", "icp_ctx_create_dist", "icp_rccl_unique_id", "icp_ctx_create_sharded",
    "icp_ctx_destroy",
    "icp_last_error", "icp_strerror", "icp_device_count", "icp_set_model", "icp_set_scene",
    "icp_set_model_device", "icp_set_scene_device", "icp_set_model_device_stream",
    "icp_set_scene_device_stream", "icp_set_progress",
    "icp_get_scene", "icp_set_allow_unequal", "icp_set_nn_variant", "icp_run", "icp_closest_matrix",
    "icp_compute_centroid", "icp_y_p_norm", "icp_err_compute", "icp_find_alignment",
    "icp_horn_solve", "icp_max_element_index", "icp_shard_range", "icp_synthetic_pair",
    "icp_load_matrix", "icp_write_matrix", "icp_free", "icp_get_stats", "icp_reset_stats",
    "icp_ensure_model", "icp_subtract_col", "icp_get_indices", "icp_set_index_digest",
    "icp_get_index_digest", "icp_set_cert_audit", "icp_set_run_mode", "icp_set_nn_rule",
    "icp_get_comm_info", "icp_set_bundle_counters", "icp_get_bundle_counters", "icp_get_model_order",
    "icp_bundle_audit", "icp_sort_pairs",
]


class ICPError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{msg} (code {code})")
        self.code = code


class Result(C.Structure):
    _fields_ = [("iterations", C.c_int), ("converged", C.c_int), ("err", C.c_double),
                ("s", C.c_double), ("R", C.c_double * 9), ("t", C.c_double * 3)]


class Stats(C.Structure):
    _fields_ = [("nn_ms", C.c_double), ("nn_launches", C.c_longlong), ("nn_pairs", C.c_longlong),
                ("ambiguous", C.c_longlong), ("level1_queued", C.c_longlong), ("level1_unrecovered", C.c_longlong), ("iter_ms", C.c_double), ("iterations", C.c_longlong),
                ("grid_fallback", C.c_longlong), ("allreduce_ms", C.c_double),
                ("allreduce_calls", C.c_longlong), ("cert_max_err_ratio", C.c_double),
                ("cert_min_margin", C.c_double), ("cert_audited", C.c_longlong),
                ("persistent_runs", C.c_longlong), ("cpu_rule_ties", C.c_longlong),
                ("cpu_rule_changed", C.c_longlong), ("persistent_fallbacks", C.c_longlong),
                ("last_filter", C.c_int), ("bundle_builds", C.c_longlong),
                ("bundle_builds_in_run", C.c_longlong), ("run_bundle_searches", C.c_longlong),
                ("run_grid_searches", C.c_longlong), ("run_certified", C.c_longlong),
                ("run_walked", C.c_longlong), ("run_path_bits", C.c_ulonglong)]


class BundleAudit(C.Structure):
    _fields_ = [("max_err_ratio", C.c_double), ("min_gap", C.c_double), ("pairs", C.c_longlong),
                ("excluded", C.c_longlong), ("checked", C.c_longlong), ("violations", C.c_longlong)]


# icp_stats.last_filter (ICP_FILTER_*): the search level that decided most queries
FILTER_NAMES = {-1: None, 0: "valu", 1: "mfma", 2: "mfma16", 3: "bundle", 4: "grid", 5: "fp64", 6: "one_launch"}


ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.POINTER(C.c_double), C.c_size_t, C.c_void_p)
PROGRESS_FN = C.CFUNCTYPE(None, C.c_int, C.c_double, C.c_void_p)

_lib = None


def lib() -> C.CDLL:
    """Load libicp_hip.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ICPError(ICP_E_NO_DEVICE, f"{LIB_PATH} not built: run `make -C iterative-closest-point_amd`")
    L = C.CDLL(LIB_PATH)
    dp = C.POINTER(C.c_double)
    vp = C.c_void_p
    sz = C.c_size_t
    L.icp_ctx_create.argtypes = [C.c_int, C.c_int, C.POINTER(vp)]
    L.icp_ctx_create_dist.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_char_p, C.POINTER(vp)]
    L.icp_rccl_unique_id.argtypes = [C.c_char_p]
    L.icp_ctx_create_sharded.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, ALLREDUCE_FN, vp, C.POINTER(vp)]
    L.icp_ctx_destroy.argtypes = [vp]
    L.icp_ctx_destroy.restype = None
    L.icp_last_error.argtypes = [vp]
    L.icp_last_error.restype = C.c_char_p
    L.icp_strerror.argtypes = [C.c_int]
    L.icp_strerror.restype = C.c_char_p
    L.icp_device_count.argtypes = [C.POINTER(C.c_int)]
    L.icp_set_model.argtypes = [vp, dp, sz]
    L.icp_set_model_device.argtypes = [vp, vp, sz]
    L.icp_set_progress.argtypes = [vp, PROGRESS_FN, vp]
    L.icp_set_scene_device.argtypes = [vp, vp, sz, sz]
    if hasattr(L, "icp_set_model_device_stream"):  # (an A/B library of an earlier round may lack them)
        L.icp_set_model_device_stream.argtypes = [vp, vp, sz, vp]
        L.icp_set_scene_device_stream.argtypes = [vp, vp, sz, sz, vp]
    L.icp_set_scene.argtypes = [vp, dp, sz, sz]
    L.icp_get_scene.argtypes = [vp, dp]
    L.icp_set_allow_unequal.argtypes = [vp, C.c_int]
    L.icp_set_nn_variant.argtypes = [vp, C.c_int]
    L.icp_set_run_mode.argtypes = [vp, C.c_int]
    L.icp_set_nn_rule.argtypes = [vp, C.c_int]
    L.icp_run.argtypes = [vp, C.c_int, C.c_double, dp, C.POINTER(Result)]
    L.icp_closest_matrix.argtypes = [vp, dp, sz, dp, C.POINTER(C.c_int32)]
    L.icp_compute_centroid.argtypes = [vp, dp, sz, dp, dp]
    L.icp_y_p_norm.argtypes = [vp, dp, dp, sz, dp, dp]
    L.icp_err_compute.argtypes = [vp, dp, dp, sz, C.c_int, dp, dp, dp]
    L.icp_find_alignment.argtypes = [vp, dp, dp, sz, dp, dp, dp, dp]
    L.icp_horn_solve.argtypes = [dp, dp, dp, C.c_double, C.c_double, dp, dp, dp]
    L.icp_max_element_index.argtypes = [dp]
    L.icp_shard_range.argtypes = [sz, C.c_int, C.c_int, C.POINTER(sz), C.POINTER(sz)]
    L.icp_synthetic_pair.argtypes = [C.c_uint64, sz, C.c_double, dp, dp, dp, dp]
    L.icp_load_matrix.argtypes = [C.c_char_p, C.POINTER(dp), C.POINTER(sz)]
    L.icp_write_matrix.argtypes = [C.c_char_p, dp, sz]
    L.icp_free.argtypes = [vp]
    L.icp_free.restype = None
    L.icp_ensure_model.argtypes = [vp, dp, sz, C.POINTER(C.c_int)]
    L.icp_subtract_col.argtypes = [vp, dp, sz, dp, dp]
    L.icp_get_indices.argtypes = [vp, C.POINTER(C.c_int32)]
    L.icp_get_model_order.argtypes = [vp, C.POINTER(C.c_int32)]
    L.icp_sort_pairs.argtypes = [C.c_int, C.POINTER(C.c_uint32), sz, C.c_int, C.POINTER(C.c_uint32), C.POINTER(C.c_int32)]
    L.icp_set_index_digest.argtypes = [vp, sz]
    L.icp_get_index_digest.argtypes = [vp, C.POINTER(C.c_uint64), sz]
    L.icp_set_cert_audit.argtypes = [vp, C.c_int]
    L.icp_bundle_audit.argtypes = [vp, C.c_int, C.POINTER(BundleAudit)]
    L.icp_get_stats.argtypes = [vp, C.POINTER(Stats)]
    L.icp_reset_stats.argtypes = [vp]
    L.icp_set_bundle_counters.argtypes = [vp, C.c_int]
    L.icp_get_bundle_counters.argtypes = [vp, C.POINTER(C.c_uint64)]
    L.icp_get_comm_info.argtypes = [vp, C.POINTER(C.c_int), C.POINTER(C.c_int), C.c_char_p, C.c_int]
    _lib = L
    return L


def _dp(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _cloud(a) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.float64)
    if a.ndim != 2 or a.shape[1] != 3:
        raise ValueError("clouds are (n, 3) float64 arrays")
    return a


def _vec(a, n) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.float64).reshape(-1)
    if a.size != n:
        raise ValueError(f"expected {n} values")
    return a


# ---------------------------------------------------------------------------------
# host-only helpers (no device needed)
# ---------------------------------------------------------------------------------

def strerror(code: int) -> str:
    return lib().icp_strerror(code).decode()


def device_count() -> int:
    n = C.c_int(0)
    lib().icp_device_count(C.byref(n))
    return n.value


def sort_pairs(keys, bits: int, device: int = 0):
    """The engine's stable LSD radix sort (icp_sort_pairs) -> (order int32, sorted keys uint32)."""
    k = np.ascontiguousarray(keys, dtype=np.uint32)
    order = np.empty(k.size, dtype=np.int32); out = np.empty(k.size, dtype=np.uint32)
    rc = lib().icp_sort_pairs(device, k.ctypes.data_as(C.POINTER(C.c_uint32)), k.size, bits,
                              out.ctypes.data_as(C.POINTER(C.c_uint32)), order.ctypes.data_as(C.POINTER(C.c_int32)))
    if rc != ICP_OK:
        raise ICPError(rc, strerror(rc))
    return order, out


def horn_solve(S, mu_p, mu_y, d_caps: float, sp: float):
    """Host half of find_alignment (gpu.cc:104-146) -> (s, R(3x3), t(3))."""
    S = _vec(S, 9); mu_p = _vec(mu_p, 3); mu_y = _vec(mu_y, 3)
    s = C.c_double(0.0); R = np.zeros(9); t = np.zeros(3)
    rc = lib().icp_horn_solve(_dp(S), _dp(mu_p), _dp(mu_y), d_caps, sp, C.byref(s), _dp(R), _dp(t))
    if rc != ICP_OK:
        raise ICPError(rc, strerror(rc))
    return s.value, R.reshape(3, 3), t


def max_element_index(ev) -> int:
    """gpu.cc:85-93 verbatim (the quirky 'largest' eigenvalue picker)."""
    ev = _vec(ev, 4)
    return lib().icp_max_element_index(_dp(ev))


def shard_range(n_total: int, rank: int, world: int):
    b = C.c_size_t(0); c = C.c_size_t(0)
    rc = lib().icp_shard_range(n_total, rank, world, C.byref(b), C.byref(c))
    if rc != ICP_OK:
        raise ICPError(rc, strerror(rc))
    return b.value, c.value


def synthetic_pair(n: int, seed: int = 42, angle_deg: float = 5.0, axis=(1.0, 2.0, 3.0),
                   t=(0.05, -0.03, 0.02)):
    """SURVEY.md §8d generator: (model, scene) as (n, 3) float64."""
    m = np.empty((n, 3)); p = np.empty((n, 3))
    ax = np.asarray(axis, dtype=np.float64); tt = np.asarray(t, dtype=np.float64)
    rc = lib().icp_synthetic_pair(seed, n, angle_deg, _dp(ax), _dp(tt), _dp(m), _dp(p))
    if rc != ICP_OK:
        raise ICPError(rc, strerror(rc))
    return m, p


def load_matrix(path: str) -> np.ndarray:
    """src/load.cc:3-33 -> (n, 3) float64."""
    ptr = C.POINTER(C.c_double)(); n = C.c_size_t(0)
    rc = lib().icp_load_matrix(path.encode(), C.byref(ptr), C.byref(n))
    if rc != ICP_OK:
        raise ICPError(rc, f"{path}: {strerror(rc)}")
    try:
        out = np.ctypeslib.as_array(ptr, shape=(max(n.value, 1) * 3,))[: n.value * 3].copy()
    finally:
        lib().icp_free(ptr)
    return out.reshape(n.value, 3)


def write_matrix(path: str, xyz) -> None:
    xyz = _cloud(xyz)
    rc = lib().icp_write_matrix(path.encode(), _dp(xyz), xyz.shape[0])
    if rc != ICP_OK:
        raise ICPError(rc, strerror(rc))


def rccl_unique_id() -> bytes:
    buf = C.create_string_buffer(128)
    rc = lib().icp_rccl_unique_id(buf)
    if rc != ICP_OK:
        raise ICPError(rc, strerror(rc))
    return buf.raw


# ---------------------------------------------------------------------------------
# device context
# ---------------------------------------------------------------------------------

class Context:
    """One HIP device context (optionally one rank of an RCCL job)."""

    def __init__(self, device: int = 0, nn_mode: int = NN_CERTIFIED, rank: int = 0,
                 world_size: int = 1, rccl_id: bytes | None = None, host_allreduce=None):
        """host_allreduce(np.ndarray) -> None: in-place sum over ranks (instead of RCCL)."""
        L = lib()
        h = C.c_void_p()
        self._cb = None
        if host_allreduce is not None:
            def _cb(buf, count, _user):
                try:
                    host_allreduce(np.ctypeslib.as_array(buf, shape=(count,)))
                    return 0
                except Exception:  # a failed rendezvous must not unwind through C
                    return 1
            self._cb = ALLREDUCE_FN(_cb)
            rc = L.icp_ctx_create_sharded(device, nn_mode, rank, world_size, self._cb, None, C.byref(h))
        elif world_size > 1 or rccl_id is not None:
            rc = L.icp_ctx_create_dist(device, nn_mode, rank, world_size, rccl_id, C.byref(h))
        else:
            rc = L.icp_ctx_create(device, nn_mode, C.byref(h))
        if rc != ICP_OK:
            raise ICPError(rc, f"context creation failed: {strerror(rc)}")
        self._h = h
        self.rank, self.world_size = rank, world_size

    def _check(self, rc: int):
        if rc != ICP_OK:
            raise ICPError(rc, f"{strerror(rc)}: {lib().icp_last_error(self._h).decode()}")

    def close(self):
        if getattr(self, "_h", None):
            lib().icp_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # resident clouds
    def set_model(self, m):
        m = _cloud(m)
        self._check(lib().icp_set_model(self._h, _dp(m), m.shape[0]))

    def set_model_device(self, ptr: int, nm: int, stream=None):
        """icp_set_model_device: the model's AoS fp64 array already in device memory (a device
        pointer, e.g. a torch tensor's data_ptr()).  stream None: read after all work enqueued so
        far on the device (a device synchronisation); else a HIP stream handle (e.g.
        torch.cuda.current_stream().cuda_stream): read after the work enqueued on that stream
        (icp_set_model_device_stream, no host synchronisation; stream-ordered: keep the array alive
        and unmodified until run() or another synchronising call returns)."""
        if stream is None or not hasattr(lib(), "icp_set_model_device_stream"):
            self._check(lib().icp_set_model_device(self._h, C.c_void_p(ptr), nm))
        else:
            self._check(lib().icp_set_model_device_stream(self._h, C.c_void_p(ptr), nm, C.c_void_p(stream)))

    def set_scene_device(self, ptr: int, np_local: int, np_total: int | None = None, stream=None):
        """icp_set_scene_device: the scene's AoS fp64 array already in device memory (stream: as
        set_model_device)."""
        npt = np_local if np_total is None else np_total
        if stream is None or not hasattr(lib(), "icp_set_scene_device_stream"):
            self._check(lib().icp_set_scene_device(self._h, C.c_void_p(ptr), np_local, npt))
        else:
            self._check(lib().icp_set_scene_device_stream(self._h, C.c_void_p(ptr), np_local, npt,
                                                          C.c_void_p(stream)))
        self._np_local = np_local

    def set_progress(self, fn):
        """icp_set_progress: fn(iteration, err) for each recorded iteration of icp_run, as it ends
        (None switches it off).  The ctypes thunk is kept alive with the context."""
        self._progress = PROGRESS_FN(lambda i, e, _u: fn(i, e)) if fn is not None else None
        self._check(lib().icp_set_progress(self._h, self._progress if fn is not None else PROGRESS_FN(), None))

    def ensure_model(self, m) -> bool:
        """icp_ensure_model: upload unless the resident model has these exact contents."""
        m = _cloud(m)
        up = C.c_int(0)
        self._check(lib().icp_ensure_model(self._h, _dp(m), m.shape[0], C.byref(up)))
        return bool(up.value)

    def set_scene(self, p, np_total: int | None = None):
        p = _cloud(p)
        self._check(lib().icp_set_scene(self._h, _dp(p), p.shape[0], p.shape[0] if np_total is None else np_total))
        self._np_local = p.shape[0]

    def get_scene(self) -> np.ndarray:
        out = np.empty((self._np_local, 3))
        self._check(lib().icp_get_scene(self._h, _dp(out)))
        return out

    def set_nn_variant(self, variant: int):
        self._check(lib().icp_set_nn_variant(self._h, variant))

    def set_nn_rule(self, rule: int):
        """icp_set_nn_rule: RULE_SQUARED (GPU path) / RULE_CPU_SQRT (the reference CPU path)."""
        self._check(lib().icp_set_nn_rule(self._h, rule))

    def set_run_mode(self, mode: int):
        """icp_set_run_mode: RUN_AUTO / RUN_LAUNCHES / RUN_PERSISTENT (bit-identical results)."""
        self._check(lib().icp_set_run_mode(self._h, mode))

    def set_allow_unequal(self, allow: bool):
        self._check(lib().icp_set_allow_unequal(self._h, 1 if allow else 0))

    def run(self, max_iter: int, threshold: float = 1e-5):
        errs = np.zeros(max(max_iter, 1))
        res = Result()
        self._check(lib().icp_run(self._h, max_iter, threshold, _dp(errs), C.byref(res)))
        return res, errs[: res.iterations].copy()

    # per-operation surface
    def closest_matrix(self, p):
        p = _cloud(p)
        y = np.empty_like(p); idx = np.empty(p.shape[0], dtype=np.int32)
        self._check(lib().icp_closest_matrix(self._h, _dp(p), p.shape[0], _dp(y),
                                             idx.ctypes.data_as(C.POINTER(C.c_int32))))
        return y, idx

    def subtract_col(self, xyz, m):
        """substract_col_w (compute.cu:381-416): xyz - m for a caller-given 3-vector m."""
        xyz = _cloud(xyz)
        out = np.empty_like(xyz)
        self._check(lib().icp_subtract_col(self._h, _dp(xyz), xyz.shape[0], _dp(_vec(m, 3)), _dp(out)))
        return out

    def get_indices(self) -> np.ndarray:
        """Correspondences of the last search over the resident scene (np_local int32)."""
        idx = np.empty(self._np_local, dtype=np.int32)
        self._check(lib().icp_get_indices(self._h, idx.ctypes.data_as(C.POINTER(C.c_int32))))
        return idx

    def model_order(self, nm: int) -> np.ndarray:
        """The bundle filter's kd order of the resident model (icp_get_model_order)."""
        kd = np.empty(nm, dtype=np.int32)
        self._check(lib().icp_get_model_order(self._h, kd.ctypes.data_as(C.POINTER(C.c_int32))))
        return kd

    def set_index_digest(self, cap: int):
        self._check(lib().icp_set_index_digest(self._h, cap))
        self._digest_cap = cap

    def set_cert_audit(self, on: bool):
        self._check(lib().icp_set_cert_audit(self._h, 1 if on else 0))

    def bundle_audit(self, groups: int = 64) -> dict:
        """The bundle bound's exclusions checked on `groups` 32-query groups of the resident
        scene (icp_bundle_audit): max MFMA error over its margin, and the excluded bundles'
        geometry (violations must be 0)."""
        out = BundleAudit()
        self._check(lib().icp_bundle_audit(self._h, int(groups), C.byref(out)))
        return {f: getattr(out, f) for f, _ in BundleAudit._fields_}

    def index_digest(self, k: int | None = None) -> np.ndarray:
        """(k, 3) uint64: per icp_run iteration (sum idx, sum (j+1) idx[j], #{idx[j] == j})."""
        k = self._digest_cap if k is None else k
        out = np.zeros((max(k, 1), 3), dtype=np.uint64)
        self._check(lib().icp_get_index_digest(self._h, out.ctypes.data_as(C.POINTER(C.c_uint64)), k))
        return out[:k]

    def compute_centroid(self, xyz, centred: bool = True):
        xyz = _cloud(xyz)
        mu = np.zeros(3); out = np.empty_like(xyz) if centred else None
        self._check(lib().icp_compute_centroid(self._h, _dp(xyz), xyz.shape[0], _dp(mu),
                                               _dp(out) if centred else None))
        return mu, out

    def y_p_norm(self, y, p):
        y = _cloud(y); p = _cloud(p)
        d = C.c_double(0.0); s = C.c_double(0.0)
        self._check(lib().icp_y_p_norm(self._h, _dp(y), _dp(p), y.shape[0], C.byref(d), C.byref(s)))
        return d.value, s.value

    def err_compute(self, y, p, in_place: bool, sR, t):
        y = _cloud(y); p = _cloud(p).copy()
        sR = _vec(sR, 9); t = _vec(t, 3); e = C.c_double(0.0)
        self._check(lib().icp_err_compute(self._h, _dp(y), _dp(p), y.shape[0], 1 if in_place else 0,
                                          _dp(sR), _dp(t), C.byref(e)))
        return e.value, p

    def find_alignment(self, p, y):
        p = _cloud(p); y = _cloud(y)
        s = C.c_double(0.0); R = np.zeros(9); t = np.zeros(3); e = C.c_double(0.0)
        self._check(lib().icp_find_alignment(self._h, _dp(p), _dp(y), p.shape[0], C.byref(s), _dp(R),
                                             _dp(t), C.byref(e)))
        return s.value, R.reshape(3, 3), t, e.value

    def stats(self) -> dict:
        st = Stats()
        self._check(lib().icp_get_stats(self._h, C.byref(st)))
        return {k: getattr(st, k) for k, _ in Stats._fields_}

    def reset_stats(self):
        self._check(lib().icp_reset_stats(self._h))

    def set_bundle_counters(self, on: bool):
        self._check(lib().icp_set_bundle_counters(self._h, 1 if on else 0))

    def bundle_counters(self) -> dict:
        """The bundle filter's executed work since set_bundle_counters(True)."""
        out = (C.c_uint64 * 16)()
        self._check(lib().icp_get_bundle_counters(self._h, out))
        tasks = max(int(out[7]), 1)
        return {"stream_mfma": int(out[8]), "block_triggers": int(out[0]), "group_tests": int(out[1]),
                "pair_tests": int(out[2]), "wave_tasks": int(out[7]),
                "us_per_wave_task": {"prologue": out[3] * 0.01 / tasks, "stream": out[4] * 0.01 / tasks,
                                     "deferred": out[5] * 0.01 / tasks, "epilogue": out[6] * 0.01 / tasks},
                "deferred_us_per_wave_task": {"bound_tests": out[10] * 0.01 / tasks,
                                              "pair_block_waits": out[11] * 0.01 / tasks,
                                              "pair_tests": out[12] * 0.01 / tasks},
                "slowest_task_us_total": out[9] * 0.01}

    def comm_info(self) -> dict:
        """RCCL communicator size / rank (None / this rank without one) and the PCI bus id of
        this context's device: what a multi-GPU run really ran on."""
        cnt, rk = C.c_int(0), C.c_int(0)
        bus = C.create_string_buffer(64)
        self._check(lib().icp_get_comm_info(self._h, C.byref(cnt), C.byref(rk), bus, 64))
        return {"comm_count": cnt.value if cnt.value >= 0 else None, "comm_rank": rk.value,
                "pci_bus_id": bus.value.decode()}


# ---------------------------------------------------------------------------------
# reference-shaped API (src/GPU/gpu.hh)
# ---------------------------------------------------------------------------------

@dataclass
class ICP:
    """GPU::ICP (src/GPU/gpu.hh:41-104): ICP(m, p, max_iter); find_corresponding_opti()."""
    m: np.ndarray
    p: np.ndarray
    max_iter: int
    nn_mode: int = NN_CERTIFIED
    device: int = 0
    threshold: float = 1e-5  # src/GPU/gpu.hh:103
    allow_unequal: bool = False
    new_p: np.ndarray = field(init=False)
    s: float = field(init=False, default=1.0)
    r: np.ndarray = field(init=False)
    t: np.ndarray = field(init=False)
    errors: np.ndarray = field(init=False)

    def __post_init__(self):
        self.m = _cloud(self.m); self.p = _cloud(self.p)
        self.new_p = self.p.copy()
        self.r = np.eye(3); self.t = np.zeros(3)
        self.errors = np.zeros(0)
        self._ctx = Context(self.device, self.nn_mode)
        self._ctx.set_allow_unequal(self.allow_unequal)
        self._ctx.set_model(self.m)
        self._ctx.set_scene(self.p)

    def find_corresponding_opti(self):
        res, errs = self._ctx.run(self.max_iter, self.threshold)
        self.errors = errs
        self.s, self.r, self.t = res.s, np.array(res.R).reshape(3, 3), np.array(res.t)
        self.new_p = self._ctx.get_scene()
        return res

    def find_alignment(self, y):
        s, R, t, e = self._ctx.find_alignment(self.new_p, y)
        self.s, self.r, self.t = s, R, t
        return e

    def compute_y_naive(self):
        """gpu.cc:6-15: one NN search per scene point (compute_distance_w_naive)."""
        Y = np.empty_like(self.new_p)
        for j in range(self.new_p.shape[0]):
            Y[j] = self.m[compute_distance_w_naive(self.m, self.new_p[j], self._ctx)]
        return Y

    def find_corresponding_naive(self):
        """gpu.cc:17-49: the per-point loop; err = (find_alignment + transform residual)/np,
        stop after the iteration whose err < threshold.  Same results as the opti loop."""
        if self.p.shape[0] != self.m.shape[0] and not self.allow_unequal:
            raise ICPError(ICP_E_SIZE_MISMATCH, "Point sets need to have the same number of points.")
        if self.p.shape[0] < 4:
            raise ICPError(ICP_E_TOO_FEW_POINTS, "Need at least 4 point pairs")
        errs = []
        for _ in range(self.max_iter):
            Y = self.compute_y_naive()
            err = self.find_alignment(Y)
            e2, self.new_p = self._ctx.err_compute(Y, self.new_p, True, self.s * self.r, self.t)
            err = (err + e2) / self.p.shape[0]
            errs.append(err)
            if err < self.threshold:
                break
        self.errors = np.array(errs)
        return len(errs)


_default_ctx: Context | None = None


def _ctx_for_model(m) -> Context:
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context()
    _default_ctx.set_model(m)
    return _default_ctx


def compute_distance_w_naive(m, pi, ctx: Context | None = None) -> int:
    """compute.cu:279-308: index of the first nearest model point of one query point."""
    c = ctx if ctx is not None else _ctx_for_model(m)
    _, idx = c.closest_matrix(np.asarray(pi, dtype=np.float64).reshape(1, 3))
    return int(idx[0])


def compute_Y_w_opti(m, p):
    """compute.cu:154-245: Y[j] = m[NN(p_j)] (returns Y, idx)."""
    return _ctx_for_model(m).closest_matrix(p)


def compute_err_w(Y, p, in_place: bool, sr, t):
    """compute.cu:348-379 -> (err, p_after)."""
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context()
    return _default_ctx.err_compute(Y, p, in_place, sr, t)


def compute_centroid(M):
    """rowwise().mean() + substract_col_w (gpu.cc:98-102) on the device -> (mu, M - mu)."""
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context()
    return _default_ctx.compute_centroid(M, centred=True)
