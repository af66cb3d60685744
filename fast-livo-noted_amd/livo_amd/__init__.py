"""livo_amd — Python binding of the MI355X LIO scan-to-map C ABI (include/livo.h).

A thin ctypes layer over fast-livo-noted_amd/lib/liblivo_hip.so used by the
tests, smoke() and bench.py.  It mirrors the reference call surface for this
path:

    KD_TREE::Build / Nearest_Search      -> Context.map_build / Context.knn
    LaserMapping::h_share_model          -> Context.h_share
    IVox (AddPoints / GetClosestPoint)   -> Context.ivox_init / ivox_add_points / ivox_knn
    LaserMapping::map_incremental        -> Context.map_incremental
    IEKF loop of LaserMapping::Run       -> Context.iekf_update(_batch)

There is no CPU fallback: loading fails loudly if the HIP library is missing,
and every compute call raises LivoError when the GPU path fails.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)
LIB_PATH = os.environ.get("LIVO_LIB") or os.path.join(PKG_ROOT, "lib", "liblivo_hip.so")  # LIVO_LIB: A/B builds
HEADER_PATH = os.path.join(os.path.dirname(PKG_ROOT), "include", "livo.h")

DIM_STATE = 18
NUM_MATCH_POINTS = 5
MAX_EVALS = 16

LIVO_OK = 0
ERRORS = {-1: "LIVO_E_INVALID", -2: "LIVO_E_HIP", -3: "LIVO_E_NOMAP", -4: "LIVO_E_NOSCAN", -5: "LIVO_E_OOM",
          -6: "LIVO_E_RANGE", -7: "LIVO_E_CAPACITY", -8: "LIVO_E_BUSY"}
MAX_INFLIGHT = 2  # LIVO_MAX_INFLIGHT
BACKEND_IKDTREE = 0  # -DUSE_ikdtree build (CMakeLists.txt:15)
BACKEND_IVOX = 1     # the reference's default build: faster_lio::IVox


class LivoError(RuntimeError):
    def __init__(self, fn, code):
        self.code = code
        super().__init__(f"{fn} failed: {ERRORS.get(code, code)} ({code})")


class Params(C.Structure):
    _fields_ = [("laser_point_cov", C.c_double), ("R_LI", C.c_double * 9), ("t_LI", C.c_double * 3),
                ("max_residual", C.c_double), ("plane_threshold", C.c_float), ("max_nn_sqdist", C.c_float),
                ("max_iterations", C.c_int32), ("flags", C.c_int32)]


class State(C.Structure):
    _fields_ = [("rot", C.c_double * 9), ("pos", C.c_double * 3), ("vel", C.c_double * 3),
                ("bias_g", C.c_double * 3), ("bias_a", C.c_double * 3), ("gravity", C.c_double * 3),
                ("cov", C.c_double * 324)]


class IterStats(C.Structure):
    _fields_ = [("iterations", C.c_int32), ("knn_passes", C.c_int32), ("converged", C.c_int32),
                ("rematch_num", C.c_int32), ("effct_feat_num", C.c_int64 * MAX_EVALS),
                ("solution", (C.c_double * 18) * MAX_EVALS), ("res_mean", C.c_double * MAX_EVALS)]


class MapInfo(C.Structure):
    _fields_ = [("num_points", C.c_int64), ("depth", C.c_int32), ("ball_chunks", C.c_int32),
                ("num_slots", C.c_int64), ("device_bytes", C.c_int64), ("ball_entries", C.c_int64)]


class PointOut(C.Structure):
    _fields_ = [("normvec", C.c_void_p), ("selected", C.c_void_p), ("nn_idx", C.c_void_p),
                ("nn_sqdist", C.c_void_p), ("world_xyz", C.c_void_p), ("visits", C.c_void_p),
                ("ori_xyz", C.c_void_p), ("corr_normvec", C.c_void_p), ("n_ori", C.c_void_p)]


class Timings(C.Structure):
    _fields_ = [("knn_ms", C.c_double), ("rematch_knn_ms", C.c_double), ("plane_ms", C.c_double),
                ("solve_ms", C.c_double),
                ("knn_launches", C.c_int64), ("knn_visits", C.c_int64), ("knn_queries", C.c_int64),
                ("effct_points", C.c_int64), ("knn_replays", C.c_int64), ("knn_points", C.c_int64),
                ("eval_ms", C.c_double * 16), ("eval_searched", C.c_int32 * 16), ("n_evals", C.c_int32),
                ("reserved_", C.c_int32), ("batch_ms", C.c_double), ("gap_ms", C.c_double)]


# every entry point of include/livo.h, with its ctypes signature
_P = C.c_void_p
IKN = 23  # LIVO_IKFOM_DOF


class IkfomState(C.Structure):
    """livo_ikfom_state: state_ikfom with quaternions (w, x, y, z) and the S2 gravity vector."""
    _fields_ = [("pos", C.c_double * 3), ("rot", C.c_double * 4), ("offset_R", C.c_double * 4),
                ("offset_T", C.c_double * 3), ("vel", C.c_double * 3), ("bg", C.c_double * 3),
                ("ba", C.c_double * 3), ("grav", C.c_double * 3), ("cov", C.c_double * (IKN * IKN))]


class IkfomStats(C.Structure):
    _fields_ = [("iterations", C.c_int32), ("knn_passes", C.c_int32), ("converged", C.c_int32),
                ("t", C.c_int32), ("effct_feat_num", C.c_int64 * 16), ("dx", (C.c_double * IKN) * 16),
                ("res_mean", C.c_double * 16)]


_IK_FIELDS = (("pos", 3), ("rot", 4), ("offset_R", 4), ("offset_T", 3), ("vel", 3), ("bg", 3), ("ba", 3),
              ("grav", 3))


def ikfom_to_c(st: dict) -> IkfomState:
    s = IkfomState()
    for k, n in _IK_FIELDS:
        getattr(s, k)[:] = np.asarray(st[k], np.float64).reshape(n).tolist()
    s.cov[:] = np.asarray(st["cov"], np.float64).reshape(IKN * IKN).tolist()
    return s


def ikfom_from_c(s: IkfomState) -> dict:
    out = {k: np.array(getattr(s, k)[:]) for k, _ in _IK_FIELDS}
    out["cov"] = np.array(s.cov[:]).reshape(IKN, IKN)
    return out


def ikfom_stats_from_c(st: IkfomStats) -> dict:
    ne = st.iterations
    return {"iterations": ne, "knn_passes": st.knn_passes, "converged": st.converged, "t": st.t,
            "effct_feat_num": [st.effct_feat_num[i] for i in range(min(ne, 16))],
            "dx": np.array([list(st.dx[i]) for i in range(min(ne, 16))]),
            "res_mean": [st.res_mean[i] for i in range(min(ne, 16))]}


class IvoxParams(C.Structure):
    _fields_ = [("resolution", C.c_float), ("nearby_type", C.c_int32), ("capacity", C.c_int64)]


class IvoxInfo(C.Structure):
    _fields_ = [("num_points", C.c_int64), ("num_grids", C.c_int64), ("ids_issued", C.c_int64),
                ("max_grid_points", C.c_int64), ("device_bytes", C.c_int64), ("add_passes", C.c_int64)]


class Cam(C.Structure):
    _fields_ = [("fx", C.c_double), ("fy", C.c_double), ("cx", C.c_double), ("cy", C.c_double),
                ("d", C.c_double * 5), ("width", C.c_int32), ("height", C.c_int32)]


class VioParams(C.Structure):
    _fields_ = [("cam", Cam), ("R_ci", C.c_double * 9), ("P_ci", C.c_double * 3), ("img_point_cov", C.c_double),
                ("patch_size", C.c_int32), ("max_iterations", C.c_int32)]


class VioStats(C.Structure):
    _fields_ = [("iterations", C.c_int32 * 3), ("updates", C.c_int32 * 3), ("last_error", C.c_float * 3),
                ("cov_updated", C.c_int32), ("n_meas", C.c_int64), ("out_of_frame", C.c_int64)]


class MapAddStats(C.Structure):
    _fields_ = [("events", C.c_int64), ("added", C.c_int64), ("deleted", C.c_int64), ("ambiguous", C.c_int64),
                ("deferred", C.c_int64), ("map_points", C.c_int64)]


SIGNATURES = {
    "livo_abi_version": (C.c_int, []),
    "livo_error_string": (C.c_char_p, [C.c_int]),
    "livo_params_default": (C.c_int, [C.POINTER(Params)]),
    "livo_ctx_create": (C.c_int, [C.c_int, C.POINTER(Params), C.POINTER(_P)]),
    "livo_ctx_destroy": (C.c_int, [_P]),
    "livo_ctx_set_params": (C.c_int, [_P, C.POINTER(Params)]),
    "livo_ctx_set_profiling": (C.c_int, [_P, C.c_int]),
    "livo_last_timings": (C.c_int, [_P, C.POINTER(Timings)]),
    "livo_map_build": (C.c_int, [_P, _P, C.c_int64, C.c_int64]),
    "livo_map_get_info": (C.c_int, [_P, C.POINTER(MapInfo)]),
    "livo_knn": (C.c_int, [_P, _P, C.c_int64, C.c_int32, _P, _P]),
    "livo_scan_upload": (C.c_int, [_P, _P, C.c_int64, C.c_int64, C.POINTER(C.c_int32)]),
    "livo_scan_upload_async": (C.c_int, [_P, _P, C.c_int64, C.c_int64, C.POINTER(C.c_int32)]),
    "livo_debug_map_rebuilds": (C.c_int, [C.c_void_p, C.POINTER(C.c_int64)]),
    "livo_scan_upload_batch_async": (C.c_int, [_P, _P, _P, C.c_int32, C.c_int64, _P]),
    "livo_host_register": (C.c_int, [_P, _P, C.c_size_t]),
    "livo_host_unregister": (C.c_int, [_P, _P]),
    "livo_scan_release": (C.c_int, [_P, C.c_int32]),
    "livo_scan_neighbors": (C.c_int, [_P, C.c_int32, _P, _P]),
    "livo_h_share": (C.c_int, [_P, C.c_int32, C.POINTER(State), C.c_int, _P, _P, C.POINTER(C.c_int64),
                               C.POINTER(PointOut)]),
    "livo_iekf_update": (C.c_int, [_P, C.c_int32, C.POINTER(State), C.POINTER(State), C.POINTER(IterStats)]),
    "livo_iekf_update_batch": (C.c_int, [_P, C.c_int32, _P, _P, _P, _P]),
    "livo_iekf_update_batch_submit": (C.c_int, [_P, C.c_int32, _P, _P, _P, _P]),
    "livo_iekf_update_batch_wait": (C.c_int, [_P, C.c_int32, _P, _P]),
    "livo_ikfom_update": (C.c_int, [_P, C.c_int32, C.POINTER(IkfomState), C.POINTER(IkfomStats)]),
    "livo_ikfom_update_batch": (C.c_int, [_P, C.c_int32, _P, _P, _P]),
    "livo_ikfom_update_batch_submit": (C.c_int, [_P, C.c_int32, _P, _P, C.POINTER(C.c_int32)]),
    "livo_ikfom_update_batch_wait": (C.c_int, [_P, C.c_int32, _P, _P]),
    "livo_ctx_set_backend": (C.c_int, [_P, C.c_int]),
    "livo_ivox_params_default": (C.c_int, [C.POINTER(IvoxParams)]),
    "livo_ivox_init": (C.c_int, [_P, C.POINTER(IvoxParams)]),
    "livo_ivox_add_points": (C.c_int, [_P, _P, C.c_int64, C.c_int64]),
    "livo_ivox_knn": (C.c_int, [_P, _P, C.c_int64, C.c_int32, C.c_double, _P, _P, _P]),
    "livo_ivox_get_info": (C.c_int, [_P, C.POINTER(IvoxInfo)]),
    "livo_ivox_dump": (C.c_int, [_P, _P, _P, _P, C.c_int64, C.POINTER(C.c_int64)]),
    "livo_map_incremental": (C.c_int, [_P, C.c_int32, C.POINTER(State), C.c_double, C.c_int, _P, _P]),
    "livo_scan_inherit_neighbors": (C.c_int, [_P, C.c_int32, C.c_int32]),
    "livo_scan_preprocess": (C.c_int, [_P, _P, C.c_int64, _P, C.c_int32, _P, _P, C.c_float, C.POINTER(C.c_int32),
                                       _P, _P, C.c_int64, C.POINTER(C.c_int64)]),
    "livo_vio_params_default": (C.c_int, [C.POINTER(VioParams)]),
    "livo_vio_update": (C.c_int, [_P, C.POINTER(VioParams), _P, C.c_int32, C.c_int32, _P, _P, _P, C.c_int64,
                                  C.POINTER(State), C.POINTER(State), _P, C.POINTER(VioStats)]),
    "livo_map_add_points": (C.c_int, [_P, _P, C.c_int64, C.c_int64, C.c_float, C.c_int, C.POINTER(MapAddStats)]),
    "livo_map_delete_boxes": (C.c_int, [_P, _P, C.c_int64, C.POINTER(C.c_int64)]),
    "livo_map_dump": (C.c_int, [_P, _P, _P, C.c_int64, C.POINTER(C.c_int64)]),
    "livo_map_last_add_stats": (C.c_int, [_P, C.POINTER(MapAddStats)]),
    "livo_frame_to_world": (C.c_int, [_P, C.c_int32, C.POINTER(State), _P, C.c_int64, C.POINTER(C.c_int64)]),
    "livo_sync": (C.c_int, [_P]),
}

_lib = None


def load(path: str = LIB_PATH):
    """Load liblivo_hip.so (raises if it was not built: there is no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(path):
            raise ImportError(f"HIP library not built: {path} (run __graft_entry__.build())")
        L = C.CDLL(path)
        # an A/B variant of an older build (LIVO_LIB) may lack entry points added since
        old_ok = os.path.abspath(path) != os.path.abspath(os.path.join(PKG_ROOT, "lib", "liblivo_hip.so"))
        for name, (res, args) in SIGNATURES.items():
            if old_ok and not hasattr(L, name):
                continue
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def page_aligned_copy(a: np.ndarray) -> np.ndarray:
    """A C-contiguous copy of `a` whose data starts on a 4 KiB page (for
    livo_host_register: the copy engine then reads whole pages of it)."""
    a = np.ascontiguousarray(a)
    raw = np.empty(a.nbytes + 4096, np.uint8)
    off = (-raw.ctypes.data) % 4096
    out = raw[off:off + a.nbytes].view(a.dtype).reshape(a.shape)
    out[...] = a
    return out


def _check(fn, rc):
    if rc != LIVO_OK:
        raise LivoError(fn, rc)


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def default_params(**kw) -> Params:
    p = Params()
    _check("livo_params_default", load().livo_params_default(C.byref(p)))
    for k, v in kw.items():
        if k in ("R_LI",):
            p.R_LI[:] = np.asarray(v, np.float64).reshape(9).tolist()
        elif k == "t_LI":
            p.t_LI[:] = np.asarray(v, np.float64).reshape(3).tolist()
        else:
            setattr(p, k, v)
    return p


def state_to_c(st: dict) -> State:
    s = State()
    s.rot[:] = np.asarray(st["rot"], np.float64).reshape(9).tolist()
    for k in ("pos", "vel", "bias_g", "bias_a", "gravity"):
        getattr(s, k)[:] = np.asarray(st[k], np.float64).reshape(3).tolist()
    s.cov[:] = np.asarray(st["cov"], np.float64).reshape(324).tolist()
    return s


def state_from_c(s: State) -> dict:
    return {"rot": np.array(s.rot[:]).reshape(3, 3), "pos": np.array(s.pos[:]), "vel": np.array(s.vel[:]),
            "bias_g": np.array(s.bias_g[:]), "bias_a": np.array(s.bias_a[:]),
            "gravity": np.array(s.gravity[:]), "cov": np.array(s.cov[:]).reshape(18, 18)}


def stats_from_c(st: IterStats) -> dict:
    ne = min(st.iterations, MAX_EVALS)
    return {"iterations": st.iterations, "knn_passes": st.knn_passes, "converged": st.converged,
            "rematch_num": st.rematch_num, "effct_feat_num": [st.effct_feat_num[i] for i in range(ne)],
            "solution": np.array([list(st.solution[i]) for i in range(ne)]).reshape(ne, 18),
            "res_mean": [st.res_mean[i] for i in range(ne)]}


class Context:
    """One livo_ctx: a HIP stream, the device map and resident scans on one GPU."""

    def __init__(self, device: int = 0, params: Params | None = None, **kw):
        L = load()
        self._L = L
        self.params = params if params is not None else default_params(**kw)
        h = C.c_void_p()
        _check("livo_ctx_create", L.livo_ctx_create(device, C.byref(self.params), C.byref(h)))
        self.h = h
        self.scans = {}

    def close(self):
        if getattr(self, "h", None):
            self._L.livo_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def set_params(self, **kw):
        for k, v in kw.items():
            if k == "R_LI":
                self.params.R_LI[:] = np.asarray(v, np.float64).reshape(9).tolist()
            elif k == "t_LI":
                self.params.t_LI[:] = np.asarray(v, np.float64).reshape(3).tolist()
            else:
                setattr(self.params, k, v)
        _check("livo_ctx_set_params", self._L.livo_ctx_set_params(self.h, C.byref(self.params)))

    # ------------------------------------------------------------ map ----
    def map_build(self, xyz: np.ndarray):
        xyz = np.ascontiguousarray(xyz, np.float32)
        assert xyz.ndim == 2 and xyz.shape[1] >= 3
        _check("livo_map_build", self._L.livo_map_build(self.h, _ptr(xyz), xyz.shape[0], xyz.shape[1] * 4))

    def map_rebuilds(self) -> tuple:
        """(grid rebuilds by sorting every id, by merging the added ids, Add_Points batches
        redone with 64-bit box keys, merged rebuilds run inside Add_Points' pass) of the incremental map."""
        out = (C.c_int64 * 4)()
        _check("livo_debug_map_rebuilds", self._L.livo_debug_map_rebuilds(self.h, out))
        return int(out[0]), int(out[1]), int(out[2]), int(out[3])

    def map_info(self) -> dict:
        mi = MapInfo()
        _check("livo_map_get_info", self._L.livo_map_get_info(self.h, C.byref(mi)))
        return {"num_points": mi.num_points, "depth": mi.depth, "num_slots": mi.num_slots,
                "device_bytes": mi.device_bytes, "ball_chunks": mi.ball_chunks, "ball_entries": mi.ball_entries}

    def knn(self, q: np.ndarray, k: int = 5):
        q = np.ascontiguousarray(q, np.float32).reshape(-1, 3)
        n = q.shape[0]
        idx = np.empty((n, k), np.int32)
        d = np.empty((n, k), np.float32)
        _check("livo_knn", self._L.livo_knn(self.h, _ptr(q), n, k, _ptr(idx), _ptr(d)))
        return idx, d

    # ---------------------------------------------------------- scans ----
    def scan_upload(self, xyz: np.ndarray) -> int:
        xyz = np.ascontiguousarray(xyz, np.float32)
        assert xyz.ndim == 2 and xyz.shape[1] >= 3
        sid = C.c_int32()
        _check("livo_scan_upload", self._L.livo_scan_upload(self.h, _ptr(xyz), xyz.shape[0], xyz.shape[1] * 4,
                                                            C.byref(sid)))
        self.scans[sid.value] = xyz.shape[0]
        return sid.value

    def scan_upload_async(self, xyz: np.ndarray) -> int:
        """livo_scan_upload_async: returns once the points are staged; the copy and
        Morton sort run on the context's upload stream (batches wait for them)."""
        xyz = np.ascontiguousarray(xyz, np.float32)
        assert xyz.ndim == 2 and xyz.shape[1] >= 3
        sid = C.c_int32()
        _check("livo_scan_upload_async",
               self._L.livo_scan_upload_async(self.h, _ptr(xyz), xyz.shape[0], xyz.shape[1] * 4, C.byref(sid)))
        self.scans[sid.value] = xyz.shape[0]
        return sid.value

    def scan_upload_batch_async(self, scans) -> list:
        """livo_scan_upload_batch_async: a list of (N_b, w) float32 arrays (one width w
        >= 3 for all) in one pass; returns their scan ids.  Arrays in page-locked
        memory (host_register) with w = 3 are read by the copy engine directly and
        must stay unchanged until a batch using the scans returns."""
        arrs = [np.ascontiguousarray(x, np.float32) for x in scans]
        n = len(arrs)
        w = arrs[0].shape[1] if n else 3
        assert all(a.ndim == 2 and a.shape[1] == w for a in arrs) and w >= 3
        ptrs = (C.c_void_p * max(n, 1))(*[a.ctypes.data for a in arrs])
        ns = (C.c_int64 * max(n, 1))(*[a.shape[0] for a in arrs])
        ids = (C.c_int32 * max(n, 1))()
        _check("livo_scan_upload_batch_async",
               self._L.livo_scan_upload_batch_async(self.h, ptrs, ns, n, w * 4, ids))
        for b in range(n):
            self.scans[ids[b]] = arrs[b].shape[0]
        self._keep = arrs  # (the arrays the device may still read from)
        return [ids[b] for b in range(n)]

    def host_register(self, arr: np.ndarray):
        """Page-lock a C-contiguous array's memory (livo_host_register)."""
        assert arr.flags["C_CONTIGUOUS"] and arr.nbytes > 0
        _check("livo_host_register", self._L.livo_host_register(self.h, arr.ctypes.data, arr.nbytes))

    def host_unregister(self, arr: np.ndarray):
        _check("livo_host_unregister", self._L.livo_host_unregister(self.h, arr.ctypes.data))

    def scan_release(self, sid: int):
        _check("livo_scan_release", self._L.livo_scan_release(self.h, sid))
        self.scans.pop(sid, None)

    def scan_neighbors(self, sid: int):
        """(idx (N, 5) int32, sqdist (N, 5) float32) of the scan's last search."""
        n = self.scans[sid]
        idx = np.empty((n, 5), np.int32)
        d = np.empty((n, 5), np.float32)
        _check("livo_scan_neighbors", self._L.livo_scan_neighbors(self.h, sid, _ptr(idx), _ptr(d)))
        return idx, d

    # -------------------------------------------------------- hot path ----
    def h_share(self, sid: int, state: dict, search_en: bool = True, outputs: bool = True):
        n = self.scans[sid]
        HTH = np.zeros(81)
        HTL = np.zeros(9)
        eff = C.c_int64()
        po = None
        res = {}
        if outputs:
            res = {"normvec": np.zeros((n, 4), np.float32), "sel": np.zeros(n, np.uint8),
                   "nn_idx": np.zeros((n, 5), np.int32), "nn_d": np.zeros((n, 5), np.float32),
                   "world": np.zeros((n, 3), np.float32), "visits": np.zeros(1, np.int64),
                   "ori": np.zeros((n, 3), np.float32), "corr_normvec": np.zeros((n, 4), np.float32),
                   "n_ori": np.zeros(1, np.int64)}
            po = PointOut(_ptr(res["normvec"]), _ptr(res["sel"]), _ptr(res["nn_idx"]), _ptr(res["nn_d"]),
                          _ptr(res["world"]), _ptr(res["visits"]), _ptr(res["ori"]), _ptr(res["corr_normvec"]),
                          _ptr(res["n_ori"]))
        st = state_to_c(state)
        _check("livo_h_share", self._L.livo_h_share(self.h, sid, C.byref(st), int(bool(search_en)), _ptr(HTH),
                                                    _ptr(HTL), C.byref(eff), C.byref(po) if po else None))
        res.update({"HTH": HTH.reshape(9, 9), "HTL": HTL, "effct": eff.value})
        if outputs:
            res["visits"] = int(res["visits"][0])
            k = int(res.pop("n_ori")[0])
            res["ori"] = res["ori"][:k]                    # laserCloudOri
            res["corr_normvec"] = res["corr_normvec"][:k]  # corr_normvect
        return res

    def frame_to_world(self, state: dict, sid: int = -1) -> np.ndarray:
        """RGBpointBodyToWorld of the last preprocessed full-res frame (sid < 0) or a resident
        scan: (n, 5) float32 x, y, z (world), intensity, curvature (livo_frame_to_world)."""
        st = state_to_c(state)
        n = C.c_int64()
        _check("livo_frame_to_world", self._L.livo_frame_to_world(self.h, sid, C.byref(st), None, 0, C.byref(n)))
        out = np.zeros((n.value, 5), np.float32)
        _check("livo_frame_to_world", self._L.livo_frame_to_world(self.h, sid, C.byref(st), _ptr(out), n.value,
                                                                  C.byref(n)))
        return out

    def iekf_update(self, sid: int, state: dict, prior: dict | None = None):
        st = state_to_c(state)
        pr = state_to_c(prior) if prior is not None else None
        stats = IterStats()
        _check("livo_iekf_update", self._L.livo_iekf_update(self.h, sid, C.byref(st),
                                                            C.byref(pr) if pr is not None else None,
                                                            C.byref(stats)))
        return state_from_c(st), stats_from_c(stats)

    def iekf_update_batch(self, sids, states, priors=None, raw: bool = False):
        n = len(sids)
        if raw:
            # hot loop (bench): states / priors are ctypes State arrays (at least
            # n entries each: the library reads and writes n); the id and stats
            # buffers are the context's own, reused while the ids repeat, so the
            # returned stats array is overwritten by the next raw call (copy it
            # to keep it)
            nb = n * C.sizeof(State)
            if C.sizeof(states) < nb or (priors is not None and C.sizeof(priors) < nb):
                raise ValueError(f"iekf_update_batch(raw): states/priors hold fewer than {n} State entries")
            key = tuple(sids)
            cache = getattr(self, "_raw_batch", None)
            if cache is None or cache[0] != key:
                ids = (C.c_int32 * n)(*sids)
                stats = (IterStats * n)()
                cache = self._raw_batch = (key, ids, stats, C.addressof(ids), C.addressof(stats))
            _, ids, stats, p_ids, p_stats = cache
            _check("livo_iekf_update_batch",
                   self._L.livo_iekf_update_batch(self.h, n, p_ids, C.addressof(states),
                                                  C.addressof(priors) if priors is not None else None, p_stats))
            return states, stats
        ids = (C.c_int32 * n)(*sids)
        sts = (State * n)(*[state_to_c(s) for s in states])
        prs = (State * n)(*[state_to_c(s) for s in priors]) if priors is not None else None
        stats = (IterStats * n)()
        _check("livo_iekf_update_batch",
               self._L.livo_iekf_update_batch(self.h, n, C.cast(ids, C.c_void_p), C.cast(sts, C.c_void_p),
                                              C.cast(prs, C.c_void_p) if prs is not None else None,
                                              C.cast(stats, C.c_void_p)))
        return [state_from_c(s) for s in sts], [stats_from_c(s) for s in stats]

    def iekf_update_batch_submit(self, sids, states, priors=None) -> int:
        """Enqueue a batched update and return its ticket (livo_iekf_update_batch_submit).
        states / priors: dicts, or ctypes State arrays of at least len(sids) entries
        (copied at the call); at most MAX_INFLIGHT batches are outstanding."""
        n = len(sids)
        ids = (C.c_int32 * n)(*sids)
        if not isinstance(states, C.Array):
            states = (State * n)(*[state_to_c(s) for s in states])
        if priors is not None and not isinstance(priors, C.Array):
            priors = (State * n)(*[state_to_c(s) for s in priors])
        nb = n * C.sizeof(State)
        if C.sizeof(states) < nb or (priors is not None and C.sizeof(priors) < nb):
            raise ValueError(f"iekf_update_batch_submit: states/priors hold fewer than {n} State entries")
        ticket = C.c_int32(-1)
        _check("livo_iekf_update_batch_submit",
               self._L.livo_iekf_update_batch_submit(self.h, n, C.addressof(ids), C.addressof(states),
                                                     C.addressof(priors) if priors is not None else None,
                                                     C.byref(ticket)))
        return ticket.value

    def iekf_update_batch_wait(self, ticket: int, n: int, out=None, stats=None):
        """Collect a submitted batch of n scans (livo_iekf_update_batch_wait).  With out
        (a ctypes State array of >= n entries) and stats (IterStats array or None) the
        raw arrays are filled and returned; else lists of dicts."""
        raw = out is not None
        if out is None:
            out = (State * max(n, 1))()
            stats = (IterStats * max(n, 1))()
        if C.sizeof(out) < n * C.sizeof(State) or (stats is not None and C.sizeof(stats) < n * C.sizeof(IterStats)):
            raise ValueError(f"iekf_update_batch_wait: output arrays hold fewer than {n} entries")
        _check("livo_iekf_update_batch_wait",
               self._L.livo_iekf_update_batch_wait(self.h, ticket, C.addressof(out),
                                                   C.addressof(stats) if stats is not None else None))
        if raw:
            return out, stats
        return [state_from_c(out[b]) for b in range(n)], [stats_from_c(stats[b]) for b in range(n)]

    # ------------------------------------------------------------ IKFoM ----
    def ikfom_update(self, sid: int, state: dict):
        """IKFoM iterated update (esekfom.hpp:1619-1928) of one resident scan."""
        st = ikfom_to_c(state)
        stats = IkfomStats()
        _check("livo_ikfom_update", self._L.livo_ikfom_update(self.h, sid, C.byref(st), C.byref(stats)))
        return ikfom_from_c(st), ikfom_stats_from_c(stats)

    def ikfom_update_batch(self, sids, states, raw: bool = False):
        n = len(sids)
        ids = (C.c_int32 * n)(*sids)
        sts = states if raw else (IkfomState * n)(*[ikfom_to_c(s) for s in states])
        stats = (IkfomStats * n)()
        _check("livo_ikfom_update_batch",
               self._L.livo_ikfom_update_batch(self.h, n, C.cast(ids, C.c_void_p), C.cast(sts, C.c_void_p),
                                               C.cast(stats, C.c_void_p)))
        if raw:
            return sts, stats
        return [ikfom_from_c(s) for s in sts], [ikfom_stats_from_c(s) for s in stats]

    def ikfom_update_batch_submit(self, sids, states, raw: bool = False) -> int:
        """livo_ikfom_update_batch_submit: enqueue, return the ticket."""
        n = len(sids)
        ids = (C.c_int32 * max(n, 1))(*sids)
        sts = states if raw else (IkfomState * max(n, 1))(*[ikfom_to_c(s) for s in states])
        t = C.c_int32()
        _check("livo_ikfom_update_batch_submit",
               self._L.livo_ikfom_update_batch_submit(self.h, n, C.cast(ids, C.c_void_p), C.cast(sts, C.c_void_p),
                                                      C.byref(t)))
        return t.value

    def ikfom_update_batch_wait(self, ticket: int, n: int, out=None, stats=None):
        """livo_ikfom_update_batch_wait; with out / stats (ctypes arrays) the raw arrays."""
        raw = out is not None
        if out is None:
            out = (IkfomState * max(n, 1))()
            stats = (IkfomStats * max(n, 1))()
        _check("livo_ikfom_update_batch_wait",
               self._L.livo_ikfom_update_batch_wait(self.h, ticket, C.cast(out, C.c_void_p),
                                                    C.cast(stats, C.c_void_p) if stats is not None else None))
        if raw:
            return out, stats
        return [ikfom_from_c(out[b]) for b in range(n)], [ikfom_stats_from_c(stats[b]) for b in range(n)]

    # ----------------------------------------------------------- iVox ----
    def set_backend(self, backend: int):
        _check("livo_ctx_set_backend", self._L.livo_ctx_set_backend(self.h, backend))
        self.backend = backend

    # ------------------------------------------- ikd-Tree incremental map ----
    def map_add_points(self, xyz: np.ndarray, downsample_size: float = 0.5, downsample: bool = True) -> dict:
        """KD_TREE::Add_Points (ikd_Tree.cpp:382-457) on the device map."""
        xyz = np.ascontiguousarray(xyz, np.float32)
        assert xyz.ndim == 2 and xyz.shape[1] >= 3
        st = MapAddStats()
        _check("livo_map_add_points", self._L.livo_map_add_points(self.h, _ptr(xyz), xyz.shape[0], xyz.shape[1] * 4,
                                                                  downsample_size, int(bool(downsample)),
                                                                  C.byref(st)))
        return {k: getattr(st, k) for k, _ in MapAddStats._fields_}

    def map_delete_boxes(self, boxes) -> int:
        """KD_TREE::Delete_Point_Boxes (ikd_Tree.cpp:501-521); boxes (n, 6) = vertex_min, vertex_max."""
        b = np.ascontiguousarray(boxes, np.float32).reshape(-1, 6)
        n = C.c_int64()
        _check("livo_map_delete_boxes", self._L.livo_map_delete_boxes(self.h, _ptr(b), b.shape[0], C.byref(n)))
        return n.value

    def map_dump(self):
        """(xyz (n, 3), ids (n,)) of the map's points in id order."""
        n = C.c_int64()
        _check("livo_map_dump", self._L.livo_map_dump(self.h, None, None, 0, C.byref(n)))
        xyz = np.zeros((n.value, 3), np.float32)
        ids = np.zeros(n.value, np.int32)
        _check("livo_map_dump", self._L.livo_map_dump(self.h, _ptr(xyz), _ptr(ids), n.value, C.byref(n)))
        return xyz, ids

    def map_last_add_stats(self) -> dict:
        st = MapAddStats()
        _check("livo_map_last_add_stats", self._L.livo_map_last_add_stats(self.h, C.byref(st)))
        return {k: getattr(st, k) for k, _ in MapAddStats._fields_}

    def ivox_init(self, resolution: float = 0.2, nearby_type: int = 18, capacity: int = 1_000_000):
        p = IvoxParams(resolution, nearby_type, capacity)
        _check("livo_ivox_init", self._L.livo_ivox_init(self.h, C.byref(p)))

    def ivox_add_points(self, xyz: np.ndarray):
        xyz = np.ascontiguousarray(xyz, np.float32)
        assert xyz.ndim == 2 and xyz.shape[1] >= 3
        _check("livo_ivox_add_points", self._L.livo_ivox_add_points(self.h, _ptr(xyz), xyz.shape[0],
                                                                    xyz.shape[1] * 4))

    def ivox_knn(self, q: np.ndarray, max_num: int = 5, max_range: float = 5.0):
        """GetClosestPoint: idx, sqdist (n, max_num) in the reference's order, cnt (-1: nothing found)."""
        q = np.ascontiguousarray(q, np.float32).reshape(-1, 3)
        n = q.shape[0]
        idx = np.empty((n, max_num), np.int32)
        d = np.empty((n, max_num), np.float32)
        cnt = np.empty(n, np.int32)
        _check("livo_ivox_knn", self._L.livo_ivox_knn(self.h, _ptr(q), n, max_num, max_range, _ptr(idx), _ptr(d),
                                                      _ptr(cnt)))
        return idx, d, cnt

    def ivox_info(self) -> dict:
        i = IvoxInfo()
        _check("livo_ivox_get_info", self._L.livo_ivox_get_info(self.h, C.byref(i)))
        return {k: getattr(i, k) for k, _ in IvoxInfo._fields_}

    def ivox_dump(self):
        """All points (xyz, ids, grid keys), grid by grid, insertion order inside a grid."""
        n = self.ivox_info()["num_points"]
        xyz = np.zeros((n, 3), np.float32)
        ids = np.zeros(n, np.int32)
        keys = np.zeros((n, 3), np.int32)
        got = C.c_int64()
        _check("livo_ivox_dump", self._L.livo_ivox_dump(self.h, _ptr(xyz), _ptr(ids), _ptr(keys), n, C.byref(got)))
        return xyz, ids, keys

    def map_incremental(self, sid: int, state: dict, filter_size_map: float = 0.5, ekf_inited: bool = True):
        """Returns (cat per point: 0 skipped / 1 added / 2 added without downsampling, counts dict).
        With the ikd-Tree backend: Add_Points of every point (cat 1), counts = the add statistics."""
        n = self.scans[sid]
        cat = np.zeros(n, np.uint8)
        counts = np.zeros(2, np.int64)
        s = state_to_c(state)
        _check("livo_map_incremental", self._L.livo_map_incremental(self.h, sid, C.byref(s), filter_size_map,
                                                                    int(bool(ekf_inited)), _ptr(cat),
                                                                    _ptr(counts)))
        if getattr(self, "backend", BACKEND_IKDTREE) == BACKEND_IKDTREE:
            return cat, self.map_last_add_stats()
        return cat, {"added": int(counts[0]), "no_downsample": int(counts[1])}

    def scan_preprocess(self, raw: np.ndarray, poses=None, rot_end=None, pos_end=None, leaf_size: float = 0.5):
        """Raw frame (n, 5: x, y, z, intensity, curvature ms) -> resident scan id, with the de-skewed
        points (n, 5) and the downsampled cloud (k, 5) (livo_scan_preprocess)."""
        raw = np.ascontiguousarray(raw, np.float32).reshape(-1, 5)
        n = raw.shape[0]
        und = np.zeros_like(raw)
        down = np.zeros_like(raw)
        nd = C.c_int64()
        sid = C.c_int32()
        if poses is not None:
            poses = np.ascontiguousarray(poses, np.float64).reshape(-1, 22)
            rot_end = np.ascontiguousarray(rot_end, np.float64).reshape(9)
            pos_end = np.ascontiguousarray(pos_end, np.float64).reshape(3)
        npo = 0 if poses is None else poses.shape[0]
        _check("livo_scan_preprocess", self._L.livo_scan_preprocess(
            self.h, _ptr(raw), n, _ptr(poses), npo, _ptr(rot_end), _ptr(pos_end), leaf_size, C.byref(sid),
            _ptr(und), _ptr(down), n, C.byref(nd)))
        self.scans[sid.value] = int(nd.value)
        return sid.value, und, down[:nd.value].copy()

    # ------------------------------------------------------------ VIO ----
    def vio_update(self, frame: dict, state: dict, prior: dict | None = None, max_iter: int = 4,
                   img_point_cov: float = 10.0):
        """LidarSelector::ComputeJ / UpdateState on a frame dict (livo_amd.synth.make_vio_frame layout):
        image, cam, pos, levels, patches, patch_size, Rci, Pci.  Returns (state, stats, errors)."""
        p = VioParams()
        _check("livo_vio_params_default", self._L.livo_vio_params_default(C.byref(p)))
        cam = frame["cam"]
        p.cam.fx, p.cam.fy, p.cam.cx, p.cam.cy = cam["fx"], cam["fy"], cam["cx"], cam["cy"]
        p.cam.d[:] = list(cam["d"]) + [0.0] * (5 - len(cam["d"]))
        p.cam.width, p.cam.height = cam["width"], cam["height"]
        p.R_ci[:] = np.asarray(frame["Rci"], np.float64).reshape(9).tolist()
        p.P_ci[:] = np.asarray(frame["Pci"], np.float64).reshape(3).tolist()
        p.img_point_cov = img_point_cov
        p.patch_size = frame["patch_size"]
        p.max_iterations = max_iter
        img = np.ascontiguousarray(frame["image"], np.uint8)
        pos = np.ascontiguousarray(frame["pos"], np.float64).reshape(-1, 3)
        lev = np.ascontiguousarray(frame["levels"], np.int32)
        pat = np.ascontiguousarray(frame["patches"], np.float32)
        n = pos.shape[0]
        s = state_to_c(state)
        pr = state_to_c(prior) if prior is not None else None
        err = np.zeros(max(n, 1), np.float32)
        st = VioStats()
        _check("livo_vio_update", self._L.livo_vio_update(
            self.h, C.byref(p), _ptr(img), img.shape[1], img.shape[0], _ptr(pos), _ptr(lev), _ptr(pat), n,
            C.byref(s), C.byref(pr) if pr is not None else None, _ptr(err), C.byref(st)))
        stats = {"iterations": list(st.iterations), "updates": list(st.updates), "last_error": list(st.last_error),
                 "cov_updated": st.cov_updated, "n_meas": st.n_meas, "out_of_frame": st.out_of_frame}
        return state_from_c(s), stats, err[:n]

    def scan_inherit_neighbors(self, dst: int, src: int):
        _check("livo_scan_inherit_neighbors", self._L.livo_scan_inherit_neighbors(self.h, dst, src))

    def set_profiling(self, level):
        """0/False off, 1 first-search timing only, 2/True every stage (livo_ctx_set_profiling)."""
        level = 2 if level is True else int(level)
        _check("livo_ctx_set_profiling", self._L.livo_ctx_set_profiling(self.h, level))

    def last_timings(self) -> dict:
        t = Timings()
        _check("livo_last_timings", self._L.livo_last_timings(self.h, C.byref(t)))
        out = {}
        for f, _ in Timings._fields_:
            v = getattr(t, f)
            out[f] = list(v)[:t.n_evals] if f in ("eval_ms", "eval_searched") else v
        return out

    def sync(self):
        _check("livo_sync", self._L.livo_sync(self.h))
