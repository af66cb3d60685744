"""Deterministic synthetic inputs for the LIO scan-to-map path.

The reference ships no bags, fixtures or golden vectors, so every
workload here is generated from fixed seeds:

* scene   — planar room (ground z=-1.6, ceiling z=2.4, four walls of a 60x40 m
            box) plus 20 axis-aligned boxes, seed 0x5EED0001.  The world
            origin is the sensor's start position, as in the reference (the
            first scan defines the map frame), and no surface plane passes
            within 0.5 m of it: esti_plane's A x = -1 formulation
            (common_lib.h:670-702) cannot represent a plane through the origin;
* map     — points sampled area-weighted on every surface with N(0, 0.01 m)
            noise along the surface normal, exact duplicates removed,
            seed 0x5EED0002;
* scan    — a Livox-Avia-shaped rosette (70.4 x 77.2 deg FoV, 6 emitter
            lines, `config/avia_resize.yaml:25`) ray-cast into the scene with
            N(0, 0.02 m) range noise, kept when x^2+y^2 is in [blind, 900]
            (`preprocess.cpp:322`), seed 0x5EED0003 + scan_id;
* state   — true IMU pose perturbed by a rotation in a 1 deg ball and a
            translation in a 0.1 m ball, seed 0x5EED0004 + scan_id;
            P = INIT_COV * I18 (`common_lib.h:36,527`).

Body frame = LiDAR frame; extrinsic R_LI = I, t_LI = [0.04165, 0.02326,
-0.0284] (`config/avia_resize.yaml:31-34`).  Everything is numpy; nothing here
runs on the GPU.
"""
from __future__ import annotations

import dataclasses
import math
import os

import numpy as np

SEED_SCENE = 0x5EED0001
SEED_MAP = 0x5EED0002
SEED_SCAN = 0x5EED0003
SEED_STATE = 0x5EED0004

ROOM_MIN = np.array([-30.0, -20.0, -1.6])
ROOM_MAX = np.array([30.0, 20.0, 2.4])
T_LI = np.array([0.04165, 0.02326, -0.0284])
R_LI = np.eye(3)
INIT_COV = 0.001
DIM_STATE = 18


@dataclasses.dataclass
class Scene:
    boxes_min: np.ndarray  # (B, 3)
    boxes_max: np.ndarray  # (B, 3)


def make_scene(n_boxes: int = 20, seed: int = SEED_SCENE) -> Scene:
    rng = np.random.default_rng(seed)
    mins, maxs = [], []
    while len(mins) < n_boxes:
        c = rng.uniform([-26.0, -16.0], [26.0, 16.0])
        sx, sy = rng.uniform(0.6, 4.0, size=2)
        top = rng.choice([rng.uniform(-1.1, -0.5), rng.uniform(0.5, 2.0)])
        lo = np.array([c[0] - sx / 2, c[1] - sy / 2])
        hi = np.array([c[0] + sx / 2, c[1] + sy / 2])
        # keep the sensor region clear and every face plane >= 1 m from the origin
        if np.any((lo < 1.0) & (hi > -1.0)) or np.any(np.abs(np.concatenate([lo, hi])) < 1.0):
            continue
        if abs(c[0]) < 5.0 and abs(c[1]) < 5.0:
            continue
        mins.append([lo[0], lo[1], ROOM_MIN[2]])
        maxs.append([hi[0], hi[1], top])
    return Scene(np.array(mins), np.array(maxs))


def _faces(scene: Scene):
    """(origin, u, v, normal) for every sampled rectangle."""
    faces = []
    lo, hi = ROOM_MIN, ROOM_MAX
    ext = hi - lo
    e = np.eye(3)
    # room: floor, ceiling, 4 walls
    faces.append((lo.copy(), e[0] * ext[0], e[1] * ext[1], e[2]))
    faces.append((np.array([lo[0], lo[1], hi[2]]), e[0] * ext[0], e[1] * ext[1], e[2]))
    faces.append((lo.copy(), e[1] * ext[1], e[2] * ext[2], e[0]))
    faces.append((np.array([hi[0], lo[1], lo[2]]), e[1] * ext[1], e[2] * ext[2], e[0]))
    faces.append((lo.copy(), e[0] * ext[0], e[2] * ext[2], e[1]))
    faces.append((np.array([lo[0], hi[1], lo[2]]), e[0] * ext[0], e[2] * ext[2], e[1]))
    for bmin, bmax in zip(scene.boxes_min, scene.boxes_max):
        d = bmax - bmin
        faces.append((np.array([bmin[0], bmin[1], bmax[2]]), e[0] * d[0], e[1] * d[1], e[2]))
        faces.append((bmin.copy(), e[1] * d[1], e[2] * d[2], e[0]))
        faces.append((np.array([bmax[0], bmin[1], bmin[2]]), e[1] * d[1], e[2] * d[2], e[0]))
        faces.append((bmin.copy(), e[0] * d[0], e[2] * d[2], e[1]))
        faces.append((np.array([bmin[0], bmax[1], bmin[2]]), e[0] * d[0], e[2] * d[2], e[1]))
    return faces


def make_map(n_points: int, scene: Scene | None = None, seed: int = SEED_MAP,
             noise: float = 0.01) -> np.ndarray:
    """(M, 3) float32 map points, area-weighted on every scene surface."""
    scene = scene or make_scene()
    faces = _faces(scene)
    areas = np.array([np.linalg.norm(np.cross(u, v)) for _, u, v, _ in faces])
    rng = np.random.default_rng(seed)
    out = np.empty((0, 3), np.float32)
    need = n_points
    while need > 0:
        m = int(need * 1.02) + 16
        fidx = rng.choice(len(faces), size=m, p=areas / areas.sum())
        a = rng.random(m)
        b = rng.random(m)
        nz = rng.normal(0.0, noise, size=m)
        O = np.stack([faces[i][0] for i in range(len(faces))])
        U = np.stack([faces[i][1] for i in range(len(faces))])
        V = np.stack([faces[i][2] for i in range(len(faces))])
        Nn = np.stack([faces[i][3] for i in range(len(faces))])
        pts = O[fidx] + a[:, None] * U[fidx] + b[:, None] * V[fidx] + nz[:, None] * Nn[fidx]
        out = np.concatenate([out, pts.astype(np.float32)])
        # remove exact duplicates, keep first occurrence order
        _, first = np.unique(out, axis=0, return_index=True)
        out = out[np.sort(first)]
        need = n_points - len(out)
    return np.ascontiguousarray(out[:n_points])


def so3_exp(w: np.ndarray) -> np.ndarray:
    th = float(np.linalg.norm(w))
    if th < 1e-12:
        return np.eye(3)
    k = w / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + math.sin(th) * K + (1 - math.cos(th)) * K @ K


def _ball(rng, radius):
    v = rng.normal(size=3)
    v /= np.linalg.norm(v)
    return v * radius * rng.random() ** (1.0 / 3.0)


def true_pose(scan_id: int):
    rng = np.random.default_rng(SEED_SCAN + scan_id)
    yaw = rng.uniform(0, 2 * math.pi)
    roll, pitch = rng.uniform(-math.radians(5), math.radians(5), size=2)
    R = so3_exp(np.array([0, 0, yaw])) @ so3_exp(np.array([0, pitch, 0])) @ so3_exp(np.array([roll, 0, 0]))
    p = np.array([rng.uniform(-0.4, 0.4), rng.uniform(-0.4, 0.4), rng.uniform(-0.2, 0.2)])
    return R, p, rng


def _rosette_dirs(n, rng):
    """Livox-Avia-like non-repetitive rosette directions in the LiDAR frame (+x forward)."""
    half_h, half_v = math.radians(70.4) / 2, math.radians(77.2) / 2
    line = np.arange(n) % 6
    t = np.sort(rng.uniform(0, 0.1, size=n))  # 100 ms frame
    w1, w2 = 2 * math.pi * 1300.0, 2 * math.pi * 1873.0  # incommensurate rates
    phase = line * (math.pi / 3.0) + rng.normal(0, 0.002, size=n)
    rho = np.abs(np.sin(w2 * t + line * 0.37))
    phi = w1 * t + phase
    az = half_h * rho * np.cos(phi)
    el = half_v * rho * np.sin(phi)
    d = np.stack([np.cos(el) * np.cos(az), np.cos(el) * np.sin(az), np.sin(el)], axis=1)
    return d, t


def _raycast(o, d, scene: Scene):
    """Range along unit rays d from origin o to the first surface (room is a closed box)."""
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = 1.0 / d
        t1 = (ROOM_MIN - o) * inv
        t2 = (ROOM_MAX - o) * inv
        tmax = np.where(inv > 0, t2, t1)
        t = np.nanmin(np.where(np.isfinite(tmax), tmax, np.inf), axis=1)
        for bmin, bmax in zip(scene.boxes_min, scene.boxes_max):
            a = (bmin - o) * inv
            b = (bmax - o) * inv
            tn = np.nanmax(np.where(np.isfinite(np.minimum(a, b)), np.minimum(a, b), -np.inf), axis=1)
            tf = np.nanmin(np.where(np.isfinite(np.maximum(a, b)), np.maximum(a, b), np.inf), axis=1)
            hit = (tn <= tf) & (tn > 1e-6)
            t = np.where(hit & (tn < t), tn, t)
    return t


def make_scan(n_points: int, scan_id: int = 0, scene: Scene | None = None,
              range_noise: float = 0.02, blind: float = 0.8):
    """(N, 3) float32 body-frame (= LiDAR-frame) points + ground-truth IMU pose."""
    scene = scene or make_scene()
    R, p, rng = true_pose(scan_id)
    R_wl = R @ R_LI
    o_l = R @ T_LI + p
    pts = np.empty((0, 3))
    while len(pts) < n_points:
        m = int((n_points - len(pts)) * 1.3) + 64
        d_l, _ = _rosette_dirs(m, rng)
        d_w = d_l @ R_wl.T
        r = _raycast(o_l, d_w, scene) + rng.normal(0, range_noise, size=m)
        q = r[:, None] * d_l
        rr = q[:, 0] ** 2 + q[:, 1] ** 2
        keep = np.isfinite(r) & (rr >= blind) & (rr <= 900.0)
        pts = np.concatenate([pts, q[keep]])
    return np.ascontiguousarray(pts[:n_points].astype(np.float32)), R, p


def make_state(scan_id: int = 0, rot_deg: float = 1.0, trans_m: float = 0.1):
    """Initial IEKF state (dict of float64 arrays) = truth perturbed, P = 0.001 I."""
    R, p, _ = true_pose(scan_id)
    rng = np.random.default_rng(SEED_STATE + scan_id)
    dth = _ball(rng, math.radians(rot_deg))
    dp = _ball(rng, trans_m)
    return {
        "rot": R @ so3_exp(dth),
        "pos": p + dp,
        "vel": np.zeros(3),
        "bias_g": np.zeros(3),
        "bias_a": np.zeros(3),
        "gravity": np.array([0.0, 0.0, -9.81]),
        "cov": np.eye(DIM_STATE) * INIT_COV,
    }


IKN = 23                   # state_ikfom DOF (use-ikfom.hpp:12-21)
S2_LEN = 98090.0 / 10000.0  # MTK::S2<double, 98090, 10000, 1> length (use-ikfom.hpp:9)


def rot_to_quat(R: np.ndarray) -> np.ndarray:
    """Unit quaternion (w, x, y, z), w >= 0, of a rotation matrix (Shepperd's method)."""
    R = np.asarray(R, np.float64)
    t = np.trace(R)
    if t > 0:
        s = math.sqrt(t + 1.0) * 2
        q = [0.25 * s, (R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s]
    else:
        i = int(np.argmax(np.diag(R)))
        j, k = (i + 1) % 3, (i + 2) % 3
        s = math.sqrt(1.0 + R[i, i] - R[j, j] - R[k, k]) * 2
        q = [0.0] * 4
        q[0] = (R[k, j] - R[j, k]) / s
        q[1 + i] = 0.25 * s
        q[1 + j] = (R[j, i] + R[i, j]) / s
        q[1 + k] = (R[k, i] + R[i, k]) / s
    q = np.array(q)
    q /= np.linalg.norm(q)
    return q if q[0] >= 0 else -q


def quat_to_rot(q) -> np.ndarray:
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def ikfom_cov() -> np.ndarray:
    """Initial P of the IKFoM state (FAST-LIO style diagonal: pose 1e-3, extrinsic 1e-5,
    vel 1e-3, bg 1e-4, ba 1e-3, gravity 1e-5)."""
    d = np.full(IKN, 1e-3)
    d[6:12] = 1e-5
    d[15:18] = 1e-4
    d[21:23] = 1e-5
    return np.diag(d)


def make_ikfom_state(scan_id: int = 0, rot_deg: float = 1.0, trans_m: float = 0.1) -> dict:
    """state_ikfom of the same perturbed pose as make_state (identity extrinsic rotation,
    offset_T = T_LI, gravity on the S2 of length 9.809)."""
    st = make_state(scan_id, rot_deg, trans_m)
    return {"pos": st["pos"], "rot": rot_to_quat(st["rot"]), "offset_R": np.array([1.0, 0.0, 0.0, 0.0]),
            "offset_T": T_LI.copy(), "vel": np.zeros(3), "bg": np.zeros(3), "ba": np.zeros(3),
            "grav": np.array([0.0, 0.0, -S2_LEN]), "cov": ikfom_cov()}


_CACHE_DIR = os.environ.get("LIVO_SYNTH_CACHE", "/tmp/livo_synth_cache")


def cached_map(n_points: int) -> np.ndarray:
    """make_map with an on-disk cache (maps of 1M-10M points take seconds to generate)."""
    os.makedirs(_CACHE_DIR, exist_ok=True)
    path = os.path.join(_CACHE_DIR, f"map_{n_points}_{SEED_MAP:x}.npy")
    if os.path.exists(path):
        try:
            return np.load(path)
        except Exception:
            pass
    m = make_map(n_points)
    tmp = path + f".{os.getpid()}.tmp.npy"
    np.save(tmp, m)
    os.replace(tmp, path)
    return m


def make_raw_scan(n_points: int, scan_id: int = 0, n_imu: int = 21, scene: Scene | None = None,
                  still: bool = False):
    """A raw (not yet de-skewed) scan and the IMU poses of its frame.

    Points (n, 5) float32: x, y, z, intensity, curvature = offset time in ms
    (preprocess.cpp:346), sorted by time as the Livox handler delivers them.
    poses (n_imu, 22) float64: Pose6D rows (offset_time s, acc, gyr, vel, pos,
    rot), offset 0 first, one per 5 ms, a smooth synthetic motion.  Returns
    (raw, poses, rot_end, pos_end).  still: the sensor does not move during
    the frame (every pose is the scan's ground-truth pose), so the de-skew
    leaves the points where make_scan put them.
    """
    body, R, p = make_scan(n_points, scan_id, scene)
    rng = np.random.default_rng(SEED_SCAN + 7919 * (scan_id + 1))
    t_ms = np.sort(rng.uniform(0.0, 100.0, size=n_points)).astype(np.float32)
    inten = rng.uniform(0, 255, size=n_points).astype(np.float32)
    raw = np.concatenate([body, inten[:, None], t_ms[:, None]], axis=1).astype(np.float32)
    w = rng.normal(0, 0.3, size=3)          # rad/s
    v = rng.normal(0, 1.0, size=3)          # m/s
    acc = rng.normal(0, 0.2, size=3)
    if still:
        w, v, acc = np.zeros(3), np.zeros(3), np.zeros(3)
    poses = np.zeros((n_imu, 22))
    for k in range(n_imu):
        t = 0.005 * k
        poses[k, 0] = t
        poses[k, 1:4] = acc
        poses[k, 4:7] = w + rng.normal(0, 0.01, size=3)
        poses[k, 7:10] = v + acc * t
        poses[k, 10:13] = p + v * t + 0.5 * acc * t * t
        poses[k, 13:22] = (R @ so3_exp(w * t)).reshape(9)
    t_end = 0.1
    rot_end = R @ so3_exp(w * t_end)
    pos_end = p + v * t_end + 0.5 * acc * t_end * t_end
    return np.ascontiguousarray(raw), poses, rot_end, pos_end


# BASELINE configs[4]: a 200k-point scan at filter_size_surf = 0.05, i.e. the
# output of downSizeFilterSurf (laser_mapping.cpp:129-130,1111) on a raw frame
# dense enough to leave about 200k points (the rosette's centre is denser than
# a 5 cm voxel, so the frame has more raw points than that).
CONFIG5_RAW_POINTS = 720_000
CONFIG5_LEAF = 0.05


def make_config5_frame(scan_id: int):
    """Raw still frame of config 5 (make_raw_scan(CONFIG5_RAW_POINTS, still=True));
    livo_scan_preprocess(leaf_size=CONFIG5_LEAF) turns it into the ~200k-point scan."""
    return make_raw_scan(CONFIG5_RAW_POINTS, scan_id, still=True)


# ---------------------------------------------------------------- VIO ----
# camera_pinhole_resize.yaml (640x512 pinhole, radial-tangential d0..d3)
PINHOLE = {"width": 640, "height": 512, "fx": 431.795259219, "fy": 431.550090267, "cx": 310.833037316,
           "cy": 266.985989326, "d": [-0.0944205499243979, 0.0946727677776504, -0.00807970960613932,
                                      8.07461209775283e-05, 0.0]}
# IMU (x forward, z up) -> camera (z forward, y down)
R_CI = np.array([[0.0, -1.0, 0.0], [0.0, 0.0, -1.0], [1.0, 0.0, 0.0]])
P_CI = np.array([0.02, -0.05, 0.03])


def _texture(w: int, h: int, rng) -> np.ndarray:
    """A smooth, textured 8-bit image (sums of oriented sinusoids and blobs)."""
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    img = np.full((h, w), 128.0)
    for _ in range(24):
        k = rng.uniform(0.02, 0.12)
        th = rng.uniform(0, np.pi)
        ph = rng.uniform(0, 2 * np.pi)
        img += rng.uniform(6, 14) * np.sin(k * (np.cos(th) * xx + np.sin(th) * yy) + ph)
    for _ in range(60):
        cx, cy, r = rng.uniform(0, w), rng.uniform(0, h), rng.uniform(4, 25)
        img += rng.uniform(-40, 40) * np.exp(-((xx - cx) ** 2 + (yy - cy) ** 2) / (2 * r * r))
    return np.clip(img, 0, 255).astype(np.uint8)


def _world2cam(cam, pc):
    u, v = pc[..., 0] / pc[..., 2], pc[..., 1] / pc[..., 2]
    d = cam["d"]
    r2 = u * u + v * v
    cd = 1 + d[0] * r2 + d[1] * r2 * r2 + d[4] * r2 * r2 * r2
    xd = u * cd + d[2] * 2 * u * v + d[3] * (r2 + 2 * u * u)
    yd = v * cd + d[2] * (r2 + 2 * v * v) + d[3] * 2 * u * v
    return np.stack([xd * cam["fx"] + cam["cx"], yd * cam["fy"] + cam["cy"]], axis=-1)


def _patch(img, px, level, ps=4):
    """The reference patch of one point at one level: the same bilinear sample
    the update uses (lidar_selection.cpp:818-842), at the true projection."""
    scale = 1 << level
    h, w = img.shape
    ui = int(np.floor(np.float32(px[0] / scale)) * scale)
    vi = int(np.floor(np.float32(px[1] / scale)) * scale)
    su = np.float32((np.float32(px[0]) - ui) / scale)
    sv = np.float32((np.float32(px[1]) - vi) / scale)
    wtl, wtr = np.float32((1 - su) * (1 - sv)), np.float32(su * (1 - sv))
    wbl, wbr = np.float32((1 - su) * sv), np.float32(su * sv)
    out = np.zeros(ps * ps, np.float32)
    half = ps // 2
    for x in range(ps):
        for y in range(ps):
            r = vi + x * scale - half * scale
            c = ui - half * scale + y * scale
            out[x * ps + y] = wtl * img[r, c] + wtr * img[r, c + scale] + wbl * img[r + scale, c] + \
                wbr * img[r + scale, c + scale]
    return out


def make_vio_frame(n_points: int, frame_id: int = 0, patch_size: int = 4, rot_deg: float = 0.3,
                   trans_m: float = 0.02):
    """A synthetic VIO frame for the photometric update:
    a textured 640x512 image, n visual points (world positions) seen in it,
    their reference patches at levels 0..2 (sampled at the true pose), search
    levels 0..2, and an initial state = truth perturbed.  Returns (frame, state0, truth)."""
    rng = np.random.default_rng(SEED_SCAN + 104729 * (frame_id + 1))
    cam = dict(PINHOLE)
    img = _texture(cam["width"], cam["height"], rng)
    R, p, _ = true_pose(frame_id)
    margin = 80
    px = np.stack([rng.uniform(margin, cam["width"] - margin, n_points),
                   rng.uniform(margin, cam["height"] - margin, n_points)], axis=1)
    depth = rng.uniform(2.0, 12.0, n_points)
    # back-project (distortion ignored: the point is then wherever world2cam puts it)
    xc = np.stack([(px[:, 0] - cam["cx"]) / cam["fx"], (px[:, 1] - cam["cy"]) / cam["fy"], np.ones(n_points)], 1)
    pcam = xc * depth[:, None]
    pos = ((pcam - P_CI) @ R_CI) @ R.T + p     # p_w = R (R_ci^T (p_c - P_ci)) + p
    pc_true = ((pos - p) @ R) @ R_CI.T + P_CI
    pix = _world2cam(cam, pc_true)
    ok = (pix[:, 0] > 64) & (pix[:, 0] < cam["width"] - 64) & (pix[:, 1] > 64) & (pix[:, 1] < cam["height"] - 64)
    pos, pix = pos[ok], pix[ok]
    levels = rng.integers(0, 3, size=len(pos)).astype(np.int32)
    pst = patch_size * patch_size
    patches = np.zeros((len(pos), 3 * pst), np.float32)
    for i in range(len(pos)):
        for lv in range(3):
            patches[i, lv * pst:(lv + 1) * pst] = _patch(img, pix[i], lv + levels[i], patch_size)
    frame = {"image": img, "cam": cam, "pos": pos, "levels": levels, "patches": patches, "patch_size": patch_size,
             "Rci": R_CI, "Pci": P_CI}
    st = make_state(frame_id, rot_deg=rot_deg, trans_m=trans_m)
    truth = dict(st)
    truth["rot"], truth["pos"] = R, p
    return frame, st, truth


def boundary_points(rng, ds: float, n: int, span: int = 40) -> np.ndarray:
    """(n, 3) float32 points within a few ulps of ikd-Tree downsample box faces j * ds
    (ikd_Tree.cpp:392-397), where float rounding makes neighbouring boxes overlap or
    leave gaps; about half the coordinates are on a face, the rest inside a box."""
    f32 = np.float32
    j = rng.integers(-span, span, size=(n, 3)).astype(f32)
    face = (j * f32(ds)).astype(f32)
    steps = rng.integers(-3, 4, size=(n, 3))
    for k in range(3):
        up = steps > k
        dn = steps < -k
        face = np.where(up, np.nextafter(face, f32(np.inf)), face)
        face = np.where(dn, np.nextafter(face, f32(-np.inf)), face)
    inner = (j * f32(ds) + rng.uniform(0, ds, size=(n, 3))).astype(f32)
    return np.where(rng.random((n, 3)) < 0.5, face, inner).astype(f32)


def centre_tie_points(ds: float, boxes: int = 8) -> tuple[np.ndarray, np.ndarray]:
    """Map points in pairs at exactly the same distance from their box centre (different
    coordinates) and one farther query point per box: Add_Points then keeps a stored point
    picked by Search_by_range's order (ikd_Tree.cpp:405-411)."""
    f32 = np.float32
    pairs, far = [], []
    for b in range(boxes):
        lo = (np.floor(np.array([b * 1.7 + 0.2, 0.3 * b, -0.4 * b], f32) / f32(ds)) * f32(ds)).astype(f32)
        hi = (lo + f32(ds)).astype(f32)
        mid = (lo.astype(np.float64) + (hi - lo).astype(np.float64) / 2.0).astype(f32)
        e = f32(ds / 8.0)
        pairs += [mid + np.array([e, 0, 0], f32), mid - np.array([e, 0, 0], f32)]
        far.append((lo + f32(ds) * f32(0.01)).astype(f32))
    return np.array(pairs, f32), np.array(far, f32)
