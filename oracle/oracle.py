"""ctypes wrapper around the CPU restatement (oracle/livo_oracle.cpp).

TEST INFRASTRUCTURE ONLY — imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the checker.  Parity status: "parity unpinned"
(see the header of livo_oracle.cpp and DESIGN.md §Oracle).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "liblivo_oracle.so")

DIM = 18
MAX_EVALS = 16


class OrcState(C.Structure):
    _fields_ = [("rot", C.c_double * 9), ("pos", C.c_double * 3), ("vel", C.c_double * 3),
                ("bias_g", C.c_double * 3), ("bias_a", C.c_double * 3), ("gravity", C.c_double * 3),
                ("cov", C.c_double * 324)]


class OrcIterStats(C.Structure):
    _fields_ = [("iterations", C.c_int32), ("knn_passes", C.c_int32), ("converged", C.c_int32),
                ("rematch_num", C.c_int32), ("effct_feat_num", C.c_int64 * MAX_EVALS),
                ("solution", (C.c_double * 18) * MAX_EVALS), ("res_mean", C.c_double * MAX_EVALS)]


IKN = 23  # state_ikfom degrees of freedom (use-ikfom.hpp:12-21)


class OrcIkfomState(C.Structure):
    """state_ikfom: quaternions (w, x, y, z) for rot / offset_R, S2 gravity as a 3-vector."""
    _fields_ = [("pos", C.c_double * 3), ("rot", C.c_double * 4), ("offset_R", C.c_double * 4),
                ("offset_T", C.c_double * 3), ("vel", C.c_double * 3), ("bg", C.c_double * 3),
                ("ba", C.c_double * 3), ("grav", C.c_double * 3), ("cov", C.c_double * (IKN * IKN))]


class OrcIkfomStats(C.Structure):
    _fields_ = [("iterations", C.c_int32), ("knn_passes", C.c_int32), ("converged", C.c_int32),
                ("t", C.c_int32), ("effct_feat_num", C.c_int64 * MAX_EVALS),
                ("dx", (C.c_double * IKN) * MAX_EVALS), ("res_mean", C.c_double * MAX_EVALS)]


IK_FIELDS = (("pos", 3), ("rot", 4), ("offset_R", 4), ("offset_T", 3), ("vel", 3), ("bg", 3), ("ba", 3),
             ("grav", 3))


def ikfom_to_c(st: dict) -> OrcIkfomState:
    s = OrcIkfomState()
    for k, n in IK_FIELDS:
        getattr(s, k)[:] = np.asarray(st[k], np.float64).reshape(n).tolist()
    s.cov[:] = np.asarray(st["cov"], np.float64).reshape(IKN * IKN).tolist()
    return s


def ikfom_from_c(s) -> dict:
    out = {k: np.array(getattr(s, k)[:]) for k, _ in IK_FIELDS}
    out["cov"] = np.array(s.cov[:]).reshape(IKN, IKN)
    return out


def build(force: bool = False) -> str:
    src = os.path.join(_HERE, "livo_oracle.cpp")
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB_PATH)
        P = C.c_void_p
        fp = np.ctypeslib.ndpointer
        L.orc_tree_build.restype = P
        L.orc_tree_build.argtypes = [P, C.c_int64]
        L.orc_tree_free.argtypes = [P]
        L.orc_tree_size.restype = C.c_int64
        L.orc_tree_size.argtypes = [P]
        L.orc_knn.argtypes = [P, P, C.c_int64, C.c_int, P, P, P, C.c_int]
        L.orc_knn_brute.argtypes = [P, C.c_int64, P, C.c_int64, C.c_int, P, P, C.c_int]
        L.orc_esti_plane.argtypes = [P, C.c_float, P]
        L.orc_to_world.argtypes = [P, C.c_int64, C.c_int, P, P, P, P, P]
        L.orc_h_share.argtypes = [P, P, C.c_int64, P, P, P, P, C.c_int, C.c_double, P, P, P, P, P, P, P, P,
                                  P, P, C.c_int]
        L.orc_iekf_update.argtypes = [P, P, C.c_int64, P, P, C.c_double, C.c_int, C.POINTER(OrcState),
                                      C.POINTER(OrcState), C.POINTER(OrcIterStats), P, C.c_int]
        L.orc_ikfom_update.argtypes = [P, P, C.c_int64, C.c_double, C.c_int, C.POINTER(OrcIkfomState),
                                       C.POINTER(OrcIkfomStats), P, C.c_int]
        L.orc_ikfom_mtk.argtypes = [C.c_int, P, P, P]
        L.orc_ivox_create.restype = P
        L.orc_ivox_create.argtypes = [C.c_float, C.c_int, C.c_int64]
        L.orc_ivox_free.argtypes = [P]
        L.orc_ivox_add_points.argtypes = [P, P, C.c_int64]
        L.orc_ivox_info.argtypes = [P, P]
        L.orc_ivox_knn.argtypes = [P, P, C.c_int64, C.c_int, C.c_double, P, P, P, P, C.c_int]
        L.orc_ivox_dump.restype = C.c_int64
        L.orc_ivox_dump.argtypes = [P, P, P, P, P]
        L.orc_ivox_h_share.argtypes = [P, P, C.c_int64, P, P, P, P, C.c_int, C.c_double, P, P, P, P, P, P, P, P,
                                       P, C.c_int]
        L.orc_ivox_iekf_update.argtypes = [P, P, C.c_int64, P, P, C.c_double, C.c_int, C.POINTER(OrcState),
                                           C.POINTER(OrcState), C.POINTER(OrcIterStats), P, P, P, P, C.c_int]
        L.orc_ivox_map_incremental.argtypes = [P, P, C.c_int64, C.POINTER(OrcState), P, P, P, P, C.c_double,
                                               C.c_int, P, P]
        del fp
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def state_to_c(st: dict) -> OrcState:
    s = OrcState()
    s.rot[:] = np.asarray(st["rot"], np.float64).reshape(9).tolist()
    for k in ("pos", "vel", "bias_g", "bias_a", "gravity"):
        getattr(s, k)[:] = np.asarray(st[k], np.float64).reshape(3).tolist()
    s.cov[:] = np.asarray(st["cov"], np.float64).reshape(324).tolist()
    return s


def state_from_c(s: OrcState) -> dict:
    return {
        "rot": np.array(s.rot[:]).reshape(3, 3),
        "pos": np.array(s.pos[:]), "vel": np.array(s.vel[:]),
        "bias_g": np.array(s.bias_g[:]), "bias_a": np.array(s.bias_a[:]),
        "gravity": np.array(s.gravity[:]), "cov": np.array(s.cov[:]).reshape(18, 18),
    }


class Tree:
    """kd-tree restating ikd-Tree Build (static map, no deletions)."""

    def __init__(self, xyz: np.ndarray):
        self.xyz = np.ascontiguousarray(xyz, np.float32)
        assert self.xyz.ndim == 2 and self.xyz.shape[1] == 3
        self.h = lib().orc_tree_build(_p(self.xyz), self.xyz.shape[0])

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.orc_tree_free(self.h)
            self.h = None

    def knn(self, q: np.ndarray, k: int = 5, threads: int = 1):
        q = np.ascontiguousarray(q, np.float32)
        n = q.shape[0]
        idx = np.empty((n, k), np.int32)
        d = np.empty((n, k), np.float32)
        vis = np.empty(n, np.int64)
        rc = lib().orc_knn(self.h, _p(q), n, k, _p(idx), _p(d), _p(vis), threads)
        assert rc == 0
        return idx, d, vis

    def h_share(self, body, rot, pos, R_LI, t_LI, search_en, cache=None, lpc=0.001, threads=1):
        body = np.ascontiguousarray(body, np.float32)
        n = body.shape[0]
        if cache is None:
            cache = {"xyz": np.zeros((n, 15), np.float32), "cnt": np.zeros(n, np.int32),
                     "idx": np.full((n, 5), -1, np.int32), "d": np.zeros((n, 5), np.float32)}
        HTH = np.zeros(81)
        HTL = np.zeros(9)
        eff = np.zeros(1, np.int64)
        vis = np.zeros(1, np.int64)
        nv = np.zeros((n, 4), np.float32)
        sel = np.zeros(n, np.uint8)
        rot = np.ascontiguousarray(rot, np.float64)
        pos = np.ascontiguousarray(pos, np.float64)
        R_LI = np.ascontiguousarray(R_LI, np.float64)
        t_LI = np.ascontiguousarray(t_LI, np.float64)
        lib().orc_h_share(self.h, _p(body), n, _p(rot), _p(pos), _p(R_LI), _p(t_LI), int(bool(search_en)),
                          lpc, _p(cache["xyz"]), _p(cache["cnt"]), _p(cache["idx"]), _p(cache["d"]),
                          _p(HTH), _p(HTL), _p(eff), _p(nv), _p(sel), _p(vis), threads)
        return {"HTH": HTH.reshape(9, 9), "HTL": HTL, "effct": int(eff[0]), "normvec": nv, "sel": sel,
                "visits": int(vis[0]), "cache": cache}

    def iekf_update(self, body, state: dict, prior: dict | None = None, R_LI=None, t_LI=None,
                    max_iter: int = 4, lpc: float = 0.001, threads: int = 1):
        from_state = state_to_c(state)
        pr = state_to_c(prior if prior is not None else state)
        st = OrcIterStats()
        vt = np.zeros(1, np.int64)
        body = np.ascontiguousarray(body, np.float32)
        R_LI = np.ascontiguousarray(np.eye(3) if R_LI is None else R_LI, np.float64)
        t_LI = np.ascontiguousarray(np.zeros(3) if t_LI is None else t_LI, np.float64)
        rc = lib().orc_iekf_update(self.h, _p(body), body.shape[0], _p(R_LI), _p(t_LI), lpc, max_iter,
                                   C.byref(from_state), C.byref(pr), C.byref(st), _p(vt), threads)
        assert rc == 0
        ne = st.iterations
        stats = {
            "iterations": ne, "knn_passes": st.knn_passes, "converged": st.converged,
            "rematch_num": st.rematch_num,
            "effct_feat_num": [st.effct_feat_num[i] for i in range(ne)],
            "solution": np.array([list(st.solution[i]) for i in range(ne)]),
            "res_mean": [st.res_mean[i] for i in range(ne)],
            "visits": int(vt[0]),
        }
        return state_from_c(from_state), stats


def _ikfom_update(self, body, state: dict, max_iter: int = 4, lpc: float = 0.001, threads: int = 1):
    """IKFoM scan update (esekfom.hpp:1619-1928 with origin_laserMapping.cpp:916-1048)."""
    cs = ikfom_to_c(state)
    st = OrcIkfomStats()
    vt = np.zeros(1, np.int64)
    body = np.ascontiguousarray(body, np.float32)
    rc = lib().orc_ikfom_update(self.h, _p(body), body.shape[0], lpc, max_iter, C.byref(cs), C.byref(st), _p(vt),
                                threads)
    assert rc == 0
    ne = st.iterations
    stats = {"iterations": ne, "knn_passes": st.knn_passes, "converged": st.converged, "t": st.t,
             "effct_feat_num": [st.effct_feat_num[i] for i in range(ne)],
             "dx": np.array([list(st.dx[i]) for i in range(ne)]),
             "res_mean": [st.res_mean[i] for i in range(ne)], "visits": int(vt[0])}
    return ikfom_from_c(cs), stats


Tree.ikfom_update = _ikfom_update


def mtk(op: int, a, b):
    """MTK pieces: 0 S2 boxplus (vec3, delta2), 1 S2 boxminus (a3, b3), 2 A_matrix (v3),
    3 state boxplus/boxminus round trip (ikfom state dict, dx23)."""
    if op == 3:
        sa = ikfom_to_c(a)
        a_buf = np.frombuffer(bytes(sa), np.float64).copy()
        out = np.zeros(IKN)
    else:
        a_buf = np.ascontiguousarray(a, np.float64)
        out = np.zeros({0: 3, 1: 2, 2: 9}[op])
    b_buf = np.ascontiguousarray(b, np.float64)
    assert lib().orc_ikfom_mtk(op, _p(a_buf), _p(b_buf), _p(out)) == 0
    return out


def to_world(pts, state: dict, R_LI=None, t_LI=None) -> np.ndarray:
    """RGBpointBodyToWorld of (n, 3) or (n, 5) points -> (n, 5) float32 (orc_to_world)."""
    pts = np.ascontiguousarray(pts, np.float32)
    n, stride = pts.shape
    out = np.zeros((n, 5), np.float32)
    rot = np.ascontiguousarray(state["rot"], np.float64)
    pos = np.ascontiguousarray(state["pos"], np.float64)
    R_LI = np.ascontiguousarray(np.eye(3) if R_LI is None else R_LI, np.float64)
    t_LI = np.ascontiguousarray(np.zeros(3) if t_LI is None else t_LI, np.float64)
    assert lib().orc_to_world(_p(pts), n, stride, _p(rot), _p(pos), _p(R_LI), _p(t_LI), _p(out)) == 0
    return out


def knn_brute(xyz, q, k=5, threads=8):
    xyz = np.ascontiguousarray(xyz, np.float32)
    q = np.ascontiguousarray(q, np.float32)
    n = q.shape[0]
    idx = np.empty((n, k), np.int32)
    d = np.empty((n, k), np.float32)
    rc = lib().orc_knn_brute(_p(xyz), xyz.shape[0], _p(q), n, k, _p(idx), _p(d), threads)
    assert rc == 0
    return idx, d


def esti_plane(pts5x3, threshold=0.1):
    p = np.ascontiguousarray(pts5x3, np.float32).reshape(15)
    out = np.zeros(4, np.float32)
    ok = lib().orc_esti_plane(_p(p), C.c_float(threshold), _p(out))
    return bool(ok), out


def new_cache(n: int) -> dict:
    """An empty neighbour cache (Nearest_Points, laser_mapping.h:165) for n points."""
    return {"xyz": np.zeros((n, 15), np.float32), "cnt": np.zeros(n, np.int32),
            "idx": np.full((n, 5), -1, np.int32), "d": np.zeros((n, 5), np.float32)}


def resize_cache(cache: dict, n: int) -> dict:
    """Nearest_Points.resize(n) (laser_mapping.cpp:165): entries below the old size are kept."""
    out = new_cache(n)
    m = min(n, cache["cnt"].shape[0])
    for k in out:
        out[k][:m] = cache[k][:m]
    return out


def _stats(st) -> dict:
    ne = st.iterations
    return {"iterations": ne, "knn_passes": st.knn_passes, "converged": st.converged,
            "rematch_num": st.rematch_num, "effct_feat_num": [st.effct_feat_num[i] for i in range(ne)],
            "solution": np.array([list(st.solution[i]) for i in range(ne)]),
            "res_mean": [st.res_mean[i] for i in range(ne)]}


class Ivox:
    """faster_lio::IVox<3, DEFAULT, PointType> (ivox3d.h, ivox3d_node.hpp) restated with std containers."""

    def __init__(self, resolution: float = 0.2, nearby_type: int = 18, capacity: int = 1_000_000):
        self.h = lib().orc_ivox_create(C.c_float(resolution), nearby_type, capacity)
        if not self.h:
            raise ValueError("bad iVox options")

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.orc_ivox_free(self.h)
            self.h = None

    def add_points(self, xyz):
        xyz = np.ascontiguousarray(xyz, np.float32).reshape(-1, 3)
        lib().orc_ivox_add_points(self.h, _p(xyz), xyz.shape[0])

    def info(self) -> dict:
        c = np.zeros(3, np.int64)
        lib().orc_ivox_info(self.h, _p(c))
        return {"num_points": int(c[0]), "num_grids": int(c[1]), "ids_issued": int(c[2])}

    def knn(self, q, max_num: int = 5, max_range: float = 5.0, threads: int = 8):
        """idx, sqdist, xyz (n x max_num) and cnt (-1: nothing found, output untouched = pad)."""
        q = np.ascontiguousarray(q, np.float32).reshape(-1, 3)
        n = q.shape[0]
        idx = np.full((n, max_num), -1, np.int32)
        d = np.full((n, max_num), np.inf, np.float32)
        xyz = np.zeros((n, max_num, 3), np.float32)
        cnt = np.zeros(n, np.int32)
        assert lib().orc_ivox_knn(self.h, _p(q), n, max_num, max_range, _p(idx), _p(d), _p(xyz), _p(cnt),
                                  threads) == 0
        return idx, d, xyz, cnt

    def dump(self):
        """Points grid by grid in LRU order (most recent first): xyz, id, grid ordinal; grid keys."""
        n = lib().orc_ivox_dump(self.h, None, None, None, None)
        g = self.info()["num_grids"]
        xyz = np.zeros((n, 3), np.float32)
        ids = np.zeros(n, np.int32)
        keys = np.zeros((g, 3), np.int32)
        gof = np.zeros(n, np.int32)
        lib().orc_ivox_dump(self.h, _p(xyz), _p(ids), _p(keys), _p(gof))
        return xyz, ids, gof, keys

    def h_share(self, body, rot, pos, R_LI, t_LI, search_en, cache, lpc=0.001, threads=8):
        body = np.ascontiguousarray(body, np.float32)
        n = body.shape[0]
        HTH = np.zeros(81)
        HTL = np.zeros(9)
        eff = np.zeros(1, np.int64)
        nv = np.zeros((n, 4), np.float32)
        sel = np.zeros(n, np.uint8)
        args = [np.ascontiguousarray(a, np.float64) for a in (rot, pos, R_LI, t_LI)]
        lib().orc_ivox_h_share(self.h, _p(body), n, *[_p(a) for a in args], int(bool(search_en)), lpc,
                               _p(cache["xyz"]), _p(cache["cnt"]), _p(cache["idx"]), _p(cache["d"]), _p(HTH),
                               _p(HTL), _p(eff), _p(nv), _p(sel), threads)
        return {"HTH": HTH.reshape(9, 9), "HTL": HTL, "effct": int(eff[0]), "normvec": nv, "sel": sel,
                "cache": cache}

    def iekf_update(self, body, state: dict, cache: dict, prior: dict | None = None, R_LI=None, t_LI=None,
                    max_iter: int = 4, lpc: float = 0.001, threads: int = 8):
        cs = state_to_c(state)
        pr = state_to_c(prior if prior is not None else state)
        st = OrcIterStats()
        body = np.ascontiguousarray(body, np.float32)
        R_LI = np.ascontiguousarray(np.eye(3) if R_LI is None else R_LI, np.float64)
        t_LI = np.ascontiguousarray(np.zeros(3) if t_LI is None else t_LI, np.float64)
        rc = lib().orc_ivox_iekf_update(self.h, _p(body), body.shape[0], _p(R_LI), _p(t_LI), lpc, max_iter,
                                        C.byref(cs), C.byref(pr), C.byref(st), _p(cache["xyz"]), _p(cache["cnt"]),
                                        _p(cache["idx"]), _p(cache["d"]), threads)
        assert rc == 0
        return state_from_c(cs), _stats(st)

    def map_incremental(self, body, state: dict, cache: dict, R_LI=None, t_LI=None,
                        filter_size_map: float = 0.5, ekf_inited: bool = True):
        """Returns the per-point category (0 skipped, 1 added, 2 added without downsampling) and counts."""
        body = np.ascontiguousarray(body, np.float32)
        n = body.shape[0]
        cs = state_to_c(state)
        R_LI = np.ascontiguousarray(np.eye(3) if R_LI is None else R_LI, np.float64)
        t_LI = np.ascontiguousarray(np.zeros(3) if t_LI is None else t_LI, np.float64)
        cat = np.zeros(n, np.uint8)
        counts = np.zeros(2, np.int64)
        lib().orc_ivox_map_incremental(self.h, _p(body), n, C.byref(cs), _p(R_LI), _p(t_LI), _p(cache["xyz"]),
                                       _p(cache["cnt"]), filter_size_map, int(bool(ekf_inited)), _p(cat),
                                       _p(counts))
        return cat, {"added": int(counts[0]), "no_downsample": int(counts[1])}


def _front_lib():
    L = lib()
    if not getattr(L, "_front", False):
        L.orc_undistort.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                    C.c_void_p]
        L.orc_voxel_grid.restype = C.c_int64
        L.orc_voxel_grid.argtypes = [C.c_void_p, C.c_int64, C.c_float, C.c_void_p]
        L._front = True
    return L


def undistort(raw, poses, rot_end, pos_end, R_LI=None, t_LI=None):
    """UndistortPcl's backward propagation (IMU_Processing.cpp:340-378).
    raw: (n, 5) float32 x, y, z, intensity, curvature(ms); poses: (m, 22) float64 Pose6D rows
    (offset_time, acc3, gyr3, vel3, pos3, rot9).  Returns the compensated copy."""
    out = np.ascontiguousarray(raw, np.float32).copy()
    poses = np.ascontiguousarray(poses, np.float64).reshape(-1, 22)
    R_LI = np.ascontiguousarray(np.eye(3) if R_LI is None else R_LI, np.float64)
    t_LI = np.ascontiguousarray(np.zeros(3) if t_LI is None else t_LI, np.float64)
    _front_lib().orc_undistort(_p(out), out.shape[0], _p(poses), poses.shape[0],
                               _p(np.ascontiguousarray(rot_end, np.float64)),
                               _p(np.ascontiguousarray(pos_end, np.float64)), _p(R_LI), _p(t_LI))
    return out


def voxel_grid(raw, leaf):
    """PCL VoxelGrid (downsample_all_data_) of (n, 5) raw points -> (k, 5) centroids, ascending leaf index."""
    raw = np.ascontiguousarray(raw, np.float32)
    out = np.zeros_like(raw)
    k = _front_lib().orc_voxel_grid(_p(raw), raw.shape[0], C.c_float(leaf), _p(out))
    return out[:k].copy()


class OrcCam(C.Structure):
    _fields_ = [("fx", C.c_double), ("fy", C.c_double), ("cx", C.c_double), ("cy", C.c_double),
                ("d", C.c_double * 5), ("width", C.c_int32), ("height", C.c_int32)]


class OrcVioStats(C.Structure):
    _fields_ = [("iterations", C.c_int32 * 3), ("updates", C.c_int32 * 3), ("last_error", C.c_float * 3),
                ("cov_updated", C.c_int32), ("n_meas", C.c_int64), ("out_of_frame", C.c_int64)]


def cam_to_c(cam: dict) -> OrcCam:
    c = OrcCam()
    c.fx, c.fy, c.cx, c.cy = cam["fx"], cam["fy"], cam["cx"], cam["cy"]
    c.d[:] = list(cam["d"]) + [0.0] * (5 - len(cam["d"]))
    c.width, c.height = cam["width"], cam["height"]
    return c


def vio_stats_from(st) -> dict:
    return {"iterations": list(st.iterations), "updates": list(st.updates), "last_error": list(st.last_error),
            "cov_updated": st.cov_updated, "n_meas": st.n_meas, "out_of_frame": st.out_of_frame}


def vio_update(frame: dict, state: dict, prior: dict | None = None, max_iter: int = 4, img_point_cov: float = 10.0):
    """ComputeJ + UpdateState (lidar_selection.cpp:748-978) on a frame dict from synth.make_vio_frame."""
    L = lib()
    if not getattr(L, "_vio", False):
        L.orc_vio_update.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(OrcCam), C.c_void_p, C.c_void_p,
                                     C.c_void_p, C.c_int64, C.c_int, C.c_void_p, C.c_void_p, C.c_double, C.c_int,
                                     C.POINTER(OrcState), C.POINTER(OrcState), C.c_void_p, C.POINTER(OrcVioStats)]
        L._vio = True
    img = np.ascontiguousarray(frame["image"], np.uint8)
    pos = np.ascontiguousarray(frame["pos"], np.float64)
    lev = np.ascontiguousarray(frame["levels"], np.int32)
    pat = np.ascontiguousarray(frame["patches"], np.float32)
    n = pos.shape[0]
    cs = state_to_c(state)
    pr = state_to_c(prior if prior is not None else state)
    err = np.zeros(n, np.float32)
    st = OrcVioStats()
    cam = cam_to_c(frame["cam"])
    L.orc_vio_update(_p(img), img.shape[1], img.shape[0], C.byref(cam), _p(pos), _p(lev), _p(pat), n,
                     frame["patch_size"], _p(np.ascontiguousarray(frame["Rci"], np.float64)),
                     _p(np.ascontiguousarray(frame["Pci"], np.float64)), img_point_cov, max_iter, C.byref(cs),
                     C.byref(pr), _p(err), C.byref(st))
    return state_from_c(cs), vio_stats_from(st), err


def _dyn_lib():
    L = lib()
    if not getattr(L, "_dyn", False):
        P = C.c_void_p
        L.orc_dyn_create.restype = P
        L.orc_dyn_create.argtypes = [P, C.c_int64]
        L.orc_dyn_free.argtypes = [P]
        L.orc_dyn_add_points.argtypes = [P, P, C.c_int64, C.c_float, C.c_int, P]
        L.orc_dyn_delete_boxes.restype = C.c_int64
        L.orc_dyn_delete_boxes.argtypes = [P, P, C.c_int64]
        L.orc_dyn_dump.restype = C.c_int64
        L.orc_dyn_dump.argtypes = [P, P, P]
        L.orc_dyn_knn.argtypes = [P, P, C.c_int64, C.c_int, P, P, C.c_int]
        L.orc_dyn_iekf_update.argtypes = [P, P, C.c_int64, P, P, C.c_double, C.c_int, C.POINTER(OrcState),
                                          C.POINTER(OrcState), C.POINTER(OrcIterStats), C.c_int]
        L.orc_dyn_map_incremental.argtypes = [P, P, C.c_int64, C.POINTER(OrcState), P, P, C.c_double, P]
        L._dyn = True
    return L


def _add_stats(st) -> dict:
    return {"events": int(st[0]), "added": int(st[1]), "deleted": int(st[2]), "ambiguous": int(st[3])}


class DynMap:
    """The ikd-Tree map under KD_TREE::Add_Points / Delete_Point_Boxes (ikd_Tree.cpp:382-521) as a
    point set with ids (initial map = its indices, kept points of a call = the next ids in input order)."""

    def __init__(self, xyz: np.ndarray):
        xyz = np.ascontiguousarray(xyz, np.float32).reshape(-1, 3)
        self.h = _dyn_lib().orc_dyn_create(_p(xyz), xyz.shape[0])

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.orc_dyn_free(self.h)
            self.h = None

    def add_points(self, xyz, downsample_size: float = 0.5, downsample: bool = True) -> dict:
        xyz = np.ascontiguousarray(xyz, np.float32).reshape(-1, 3)
        st = np.zeros(4, np.int64)
        assert _dyn_lib().orc_dyn_add_points(self.h, _p(xyz), xyz.shape[0], C.c_float(downsample_size),
                                             int(bool(downsample)), _p(st)) == 0
        return _add_stats(st)

    def delete_boxes(self, boxes) -> int:
        """boxes (n, 6): vertex_min xyz, vertex_max xyz (BoxPointType)."""
        b = np.ascontiguousarray(boxes, np.float32).reshape(-1, 6)
        return int(_dyn_lib().orc_dyn_delete_boxes(self.h, _p(b), b.shape[0]))

    def dump(self):
        """(xyz (n, 3), ids (n,)) of the alive points in id order."""
        n = _dyn_lib().orc_dyn_dump(self.h, None, None)
        xyz = np.zeros((n, 3), np.float32)
        ids = np.zeros(n, np.int32)
        _dyn_lib().orc_dyn_dump(self.h, _p(xyz), _p(ids))
        return xyz, ids

    def knn(self, q, k: int = 5, threads: int = 8):
        q = np.ascontiguousarray(q, np.float32).reshape(-1, 3)
        n = q.shape[0]
        idx = np.empty((n, k), np.int32)
        d = np.empty((n, k), np.float32)
        assert _dyn_lib().orc_dyn_knn(self.h, _p(q), n, k, _p(idx), _p(d), threads) == 0
        return idx, d

    def iekf_update(self, body, state: dict, prior: dict | None = None, R_LI=None, t_LI=None,
                    max_iter: int = 4, lpc: float = 0.001, threads: int = 8):
        cs = state_to_c(state)
        pr = state_to_c(prior if prior is not None else state)
        st = OrcIterStats()
        body = np.ascontiguousarray(body, np.float32)
        R_LI = np.ascontiguousarray(np.eye(3) if R_LI is None else R_LI, np.float64)
        t_LI = np.ascontiguousarray(np.zeros(3) if t_LI is None else t_LI, np.float64)
        assert _dyn_lib().orc_dyn_iekf_update(self.h, _p(body), body.shape[0], _p(R_LI), _p(t_LI), lpc, max_iter,
                                              C.byref(cs), C.byref(pr), C.byref(st), threads) == 0
        return state_from_c(cs), _stats(st)

    def map_incremental(self, body, state: dict, R_LI=None, t_LI=None, filter_size_map: float = 0.5) -> dict:
        """map_incremental with USE_ikdtree (laser_mapping.cpp:383-384)."""
        body = np.ascontiguousarray(body, np.float32)
        cs = state_to_c(state)
        R_LI = np.ascontiguousarray(np.eye(3) if R_LI is None else R_LI, np.float64)
        t_LI = np.ascontiguousarray(np.zeros(3) if t_LI is None else t_LI, np.float64)
        st = np.zeros(4, np.int64)
        assert _dyn_lib().orc_dyn_map_incremental(self.h, _p(body), body.shape[0], C.byref(cs), _p(R_LI), _p(t_LI),
                                                  filter_size_map, _p(st)) == 0
        return _add_stats(st)
