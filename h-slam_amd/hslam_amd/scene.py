"""Deterministic synthetic scenes for the photometric-BA hot path.

The reference reads real datasets through OpenCV (Include/DatasetLoader.h); that
layer is out of scope, so benches and parity tests run on scenes rendered here:

* camera 640x480, TumMono useK intrinsics fx=256.0 fy=254.4 cx=319.5 cy=239.5
  (Src/GeometricUndistorter.cpp:111-122), pyramid levels by Include/CalibData.h:107-115;
* three textured planes at Z = 2, 3, 5 m, texture = 24 random-phase sinusoids
  (6-48 px wavelength on the image plane) + blurred uniform noise, intensity 20..235;
* images rendered by exact ray/plane intersection (photo-consistent up to occlusion);
* direct pyramids + central-difference gradients exactly as Frame::CreateDirPyrs
  (Src/Frame.cpp:104-166) in float32 (rows 0 and h-1, which the reference leaves
  uninitialised, get gradient 0);
* points: best |grad|^2 pixel per cell, colour / weight sampled as the ImmaturePoint
  constructor (Src/ImmaturePoint.cpp:7-32), idepth = 1/Z (1 + N(0, 0.01));
* one residual per (host, other KF) whose centre projects inside the image.

Everything is seeded (default 20261015) and float32 where the reference is float.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

PATTERN = np.array([[0, -2], [-1, -1], [1, -1], [-2, 0], [0, 0], [2, 0], [-1, 1], [0, 2]], dtype=np.int32)
SEED = 20261015


def pyramid_levels(w: int, h: int, max_levels: int = 6) -> int:
    """CalibData constructor rule (Include/CalibData.h:107-115)."""
    lv = 1
    while w % 2 == 0 and h % 2 == 0 and w * h > 5000 and lv < max_levels:
        w //= 2
        h //= 2
        lv += 1
    return lv


# ----------------------------------------------------------------- rotations / SE3 (fp64)
def rodrigues(w):
    w = np.asarray(w, dtype=np.float64)
    th = np.linalg.norm(w)
    if th < 1e-15:
        return np.eye(3)
    k = w / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + math.sin(th) * K + (1 - math.cos(th)) * (K @ K)


def rot_to_quat(R):
    """Unit quaternion (x, y, z, w) of a rotation matrix (w >= 0)."""
    tr = R[0, 0] + R[1, 1] + R[2, 2]
    if tr > 0:
        s = math.sqrt(tr + 1.0) * 2
        w = 0.25 * s
        x = (R[2, 1] - R[1, 2]) / s
        y = (R[0, 2] - R[2, 0]) / s
        z = (R[1, 0] - R[0, 1]) / s
    elif R[0, 0] > R[1, 1] and R[0, 0] > R[2, 2]:
        s = math.sqrt(1.0 + R[0, 0] - R[1, 1] - R[2, 2]) * 2
        w = (R[2, 1] - R[1, 2]) / s
        x = 0.25 * s
        y = (R[0, 1] + R[1, 0]) / s
        z = (R[0, 2] + R[2, 0]) / s
    elif R[1, 1] > R[2, 2]:
        s = math.sqrt(1.0 + R[1, 1] - R[0, 0] - R[2, 2]) * 2
        w = (R[0, 2] - R[2, 0]) / s
        x = (R[0, 1] + R[1, 0]) / s
        y = 0.25 * s
        z = (R[1, 2] + R[2, 1]) / s
    else:
        s = math.sqrt(1.0 + R[2, 2] - R[0, 0] - R[1, 1]) * 2
        w = (R[1, 0] - R[0, 1]) / s
        x = (R[0, 2] + R[2, 0]) / s
        y = (R[1, 2] + R[2, 1]) / s
        z = 0.25 * s
    q = np.array([x, y, z, w])
    q /= np.linalg.norm(q)
    if q[3] < 0:
        q = -q
    return q


def quat_to_rot(q):
    x, y, z, w = q
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
        [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
        [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)],
    ])


def se3_data(R, t):
    """Sophus SE3d::data() layout: qx qy qz qw tx ty tz."""
    q = rot_to_quat(R)
    return np.concatenate([q, np.asarray(t, dtype=np.float64)])


def se3_from_data(d):
    return quat_to_rot(np.asarray(d[:4]) / np.linalg.norm(d[:4])), np.asarray(d[4:7], dtype=np.float64)


# ----------------------------------------------------------------- texture / rendering
@dataclass
class Plane:
    z: float
    xmin: float = -1e9
    xmax: float = 1e9
    ymin: float = -1e9
    ymax: float = 1e9
    dirs: np.ndarray = field(default=None)
    freqs: np.ndarray = field(default=None)
    phases: np.ndarray = field(default=None)
    amps: np.ndarray = field(default=None)
    noise: np.ndarray = field(default=None)
    noise_step: float = 0.0
    lo: float = 0.0
    hi: float = 1.0


def _blur1(a):
    """Separable Gaussian blur, sigma = 1 sample."""
    k = np.exp(-0.5 * np.arange(-3, 4) ** 2)
    k /= k.sum()
    a = np.apply_along_axis(lambda r: np.convolve(r, k, mode="same"), 0, a)
    a = np.apply_along_axis(lambda r: np.convolve(r, k, mode="same"), 1, a)
    return a


def make_plane(rng, z, f, **kw):
    p = Plane(z=z, **kw)
    n = 24
    ang = rng.uniform(0, 2 * np.pi, n)
    lam_px = rng.uniform(6.0, 48.0, n)
    lam_world = lam_px * z / f
    p.dirs = np.stack([np.cos(ang), np.sin(ang)], 1)
    p.freqs = 2 * np.pi / lam_world
    p.phases = rng.uniform(0, 2 * np.pi, n)
    p.amps = rng.uniform(0.5, 1.0, n)
    # blurred uniform noise on a grid of 1 px (at this depth) spacing, 2048 x 2048 samples
    p.noise_step = z / f
    p.noise = _blur1(rng.uniform(-1, 1, (512, 512)))
    p.noise *= 1.0 / (np.abs(p.noise).max() + 1e-12)
    # normalise the sinusoid sum to [lo, hi] via the amplitude bound
    p.lo, p.hi = -p.amps.sum(), p.amps.sum()
    return p


def plane_texture(p: Plane, X, Y):
    s = np.zeros_like(X)
    for k in range(len(p.freqs)):
        s += p.amps[k] * np.sin(p.freqs[k] * (p.dirs[k, 0] * X + p.dirs[k, 1] * Y) + p.phases[k])
    s = (s - p.lo) / (p.hi - p.lo)  # 0..1, concentrated around 0.5
    s = 0.5 + 2.2 * (s - 0.5)
    gx = X / p.noise_step
    gy = Y / p.noise_step
    n = p.noise.shape[0]
    ix = np.floor(gx).astype(np.int64)
    iy = np.floor(gy).astype(np.int64)
    fx = gx - ix
    fy = gy - iy
    ix0, iy0 = ix % n, iy % n
    ix1, iy1 = (ix + 1) % n, (iy + 1) % n
    nz = (p.noise[iy0, ix0] * (1 - fx) * (1 - fy) + p.noise[iy0, ix1] * fx * (1 - fy)
          + p.noise[iy1, ix0] * (1 - fx) * fy + p.noise[iy1, ix1] * fx * fy)
    val = s + 0.08 * nz
    return np.clip(20.0 + 215.0 * val, 20.0, 235.0)


def render(planes, K, R_c2w, C, w, h, a=0.0, b=0.0):
    """Exact ray/plane intersection at pixel centres; returns float32 image and depth."""
    xs, ys = np.meshgrid(np.arange(w, dtype=np.float64), np.arange(h, dtype=np.float64))
    Ki = np.linalg.inv(K)
    d = np.stack([xs, ys, np.ones_like(xs)], -1) @ Ki.T
    dw = d @ R_c2w.T
    best = np.full((h, w), np.inf)
    img = np.zeros((h, w))
    for p in planes:
        s = (p.z - C[2]) / dw[..., 2]
        X = C[0] + s * dw[..., 0]
        Y = C[1] + s * dw[..., 1]
        ok = (s > 0) & (X >= p.xmin) & (X <= p.xmax) & (Y >= p.ymin) & (Y <= p.ymax) & (s < best)
        if not ok.any():
            continue
        tex = plane_texture(p, X[ok], Y[ok])
        img[ok] = tex
        best[ok] = s[ok]
    # camera-frame depth Z = s * d_z (d_z = 1 for the normalised ray)
    depth = best * d[..., 2]
    img = math.exp(a) * img + b
    return img.astype(np.float32), depth


def make_dir_pyramid(img0: np.ndarray, levels: int):
    """Frame::CreateDirPyrs (Src/Frame.cpp:104-166): list of (h_l, w_l, 3) float32 [I, dx, dy]."""
    pyr = []
    I = img0.astype(np.float32)
    for lvl in range(levels):
        if lvl > 0:
            prev = pyr[-1][..., 0]
            h, w = prev.shape[0] // 2, prev.shape[1] // 2
            a = prev[0:2 * h:2, 0:2 * w:2]
            bb = prev[0:2 * h:2, 1:2 * w:2]
            c = prev[1:2 * h:2, 0:2 * w:2]
            d = prev[1:2 * h:2, 1:2 * w:2]
            I = np.float32(0.25) * (((a + bb) + c) + d)
        h, w = I.shape
        out = np.zeros((h, w, 3), dtype=np.float32)
        out[..., 0] = I
        flat = I.reshape(-1)
        idx = np.arange(w, w * (h - 1))
        dx = np.float32(0.5) * (flat[idx + 1] - flat[idx - 1])
        dy = np.float32(0.5) * (flat[idx + w] - flat[idx - w])
        dx[~np.isfinite(dx)] = 0
        dy[~np.isfinite(dy)] = 0
        o = out.reshape(-1, 3)
        o[idx, 1] = dx
        o[idx, 2] = dy
        pyr.append(out)
    return pyr


# ----------------------------------------------------------------- BA window
@dataclass
class BAScene:
    width: int
    height: int
    K: np.ndarray                 # level-0 intrinsics (fp64)
    n_levels: int
    frames_pose: np.ndarray       # [nF, 7] true worldToCam (SE3 data)
    frames_eval: np.ndarray       # [nF, 7] evalPT given to the BA (perturbed)
    frames_state: np.ndarray      # [nF, 10]
    frames_state_zero: np.ndarray
    frames_exposure: np.ndarray   # [nF] float32
    frames_energyTH: np.ndarray   # [nF] float32
    frames_id: np.ndarray         # [nF] int32
    pyramids: list                # per frame: list of (h_l, w_l, 3) float32
    pt_host: np.ndarray           # [n] int32 (sorted)
    pt_u: np.ndarray              # [n] float32
    pt_v: np.ndarray
    pt_idepth: np.ndarray
    pt_idepth_zero: np.ndarray
    pt_color: np.ndarray          # [n, 8] float32
    pt_weights: np.ndarray        # [n, 8] float32
    pt_idepth_true: np.ndarray
    res_point: np.ndarray         # [m] int32 (grouped by point)
    res_target: np.ndarray        # [m] int32
    planes: list = field(default=None, repr=False)

    @property
    def n_frames(self):
        return len(self.frames_id)

    @property
    def n_points(self):
        return len(self.pt_u)

    @property
    def n_res(self):
        return len(self.res_point)

    def shard(self, rank: int, nranks: int) -> "BAScene":
        """Point shard for multi-GPU: points p with p % nranks == rank (stays sorted by host),
        with their residuals (all residuals of a point live on one rank)."""
        import copy
        sel = np.nonzero(np.arange(self.n_points) % nranks == rank)[0]
        remap = -np.ones(self.n_points, np.int64)
        remap[sel] = np.arange(len(sel))
        rsel = remap[self.res_point] >= 0
        out = copy.copy(self)
        for name in ("pt_host", "pt_u", "pt_v", "pt_idepth", "pt_idepth_zero", "pt_color", "pt_weights",
                     "pt_idepth_true", "pt_has_prior"):
            if getattr(self, name, None) is not None:
                setattr(out, name, np.ascontiguousarray(getattr(self, name)[sel]))
        out.res_point = remap[self.res_point[rsel]].astype(np.int32)
        out.res_target = np.ascontiguousarray(self.res_target[rsel])
        return out

    def images_level0(self):
        return [np.ascontiguousarray(p[0]) for p in self.pyramids]


def _select_points(img_pyr0, n_pts, border, rng):
    h, w = img_pyr0.shape[:2]
    g2 = img_pyr0[..., 1].astype(np.float64) ** 2 + img_pyr0[..., 2].astype(np.float64) ** 2
    area = (w - 2 * border) * (h - 2 * border)
    cell = max(1, int(math.floor(math.sqrt(area / float(n_pts)))))
    cands = []
    for y0 in range(border, h - border - cell + 1, cell):
        for x0 in range(border, w - border - cell + 1, cell):
            blk = g2[y0:y0 + cell, x0:x0 + cell]
            k = int(np.argmax(blk))
            cands.append((y0 + k // cell, x0 + k % cell))
    while len(cands) < n_pts:  # degenerate: fall back to random pixels
        cands.append((int(rng.integers(border, h - border)), int(rng.integers(border, w - border))))
    cands = np.array(cands)
    sel = np.round(np.arange(n_pts) * (len(cands) / float(n_pts))).astype(np.int64)
    sel = np.minimum(sel, len(cands) - 1)
    return cands[sel]


def make_ba_scene(n_points: int = 2000, n_frames: int = 8, width: int = 640, height: int = 480,
                  K=None, seed: int = SEED, pose_noise=(0.004, 0.002), idepth_noise: float = 0.01,
                  baseline: float = 0.06, max_rot_deg: float = 1.0, kitti: bool = False) -> BAScene:
    """C3/C4 window: n_frames KFs x n_points (n_points / n_frames per host)."""
    rng = np.random.default_rng(seed)
    if K is None:
        if kitti:
            K = np.array([[718.856, 0, 615.5], [0, 718.856, 183.5], [0, 0, 1.0]])
        else:
            K = np.array([[256.0, 0, 319.5], [0, 254.4, 239.5], [0, 0, 1.0]])
    K = np.asarray(K, dtype=np.float64)
    f = K[0, 0]
    planes = [make_plane(rng, 5.0, f), make_plane(rng, 3.0, f, xmax=-0.25), make_plane(rng, 2.0, f, xmin=0.55, ymax=0.15)]
    levels = pyramid_levels(width, height)
    poses, evals, pyrs = [], [], []
    for i in range(n_frames):
        ax = rng.normal(size=3)
        ax /= np.linalg.norm(ax)
        ang = math.radians(rng.uniform(0, max_rot_deg))
        R_c2w = rodrigues(ax * ang)
        C = np.array([baseline * i, 0.0, 0.0])
        img, _ = render(planes, K, R_c2w, C, width, height)
        pyrs.append(make_dir_pyramid(img, levels))
        R_w2c = R_c2w.T
        t_w2c = -R_w2c @ C
        poses.append(se3_data(R_w2c, t_w2c))
        if i == 0:
            evals.append(se3_data(R_w2c, t_w2c))
        else:
            dR = rodrigues(rng.normal(size=3) * pose_noise[1])
            dt = rng.normal(size=3) * pose_noise[0]
            evals.append(se3_data(dR @ R_w2c, dR @ t_w2c + dt))
    poses = np.array(poses)
    evals = np.array(evals)

    per = [n_points // n_frames + (1 if i < n_points % n_frames else 0) for i in range(n_frames)]
    hosts, us, vs, ids, idt, cols, wts = [], [], [], [], [], [], []
    for hst in range(n_frames):
        if per[hst] == 0:
            continue
        pix = _select_points(pyrs[hst][0], per[hst], 4, rng)
        R_w2c, t_w2c = se3_from_data(poses[hst])
        R_c2w = R_w2c.T
        C = -R_c2w @ t_w2c
        _, depth = render_depth_at(planes, K, R_c2w, C, pix)
        lvl0 = pyrs[hst][0]
        py = pix[:, 0:1] + PATTERN[None, :, 1]
        px = pix[:, 1:2] + PATTERN[None, :, 0]
        smp = lvl0[py, px]                       # [n, 8, 3], exact pixels (BiLin at integer coords)
        gx, gy = smp[..., 1], smp[..., 2]
        c2500 = np.float32(2500.0)
        wgt = np.sqrt(c2500 / (c2500 + (gx * gx + gy * gy))).astype(np.float32)
        it = 1.0 / depth
        hosts.append(np.full(len(pix), hst, np.int32))
        us.append(pix[:, 1].astype(np.float32))
        vs.append(pix[:, 0].astype(np.float32))
        idt.append(it)
        ids.append((it * (1.0 + idepth_noise * rng.normal(size=len(pix)))).astype(np.float32))
        cols.append(smp[..., 0].astype(np.float32))
        wts.append(wgt)
    pt_host = np.concatenate(hosts)
    pt_u = np.concatenate(us)
    pt_v = np.concatenate(vs)
    pt_id = np.concatenate(ids)

    # residuals: centre projection of the noisy point into every other KF with the evalPT poses
    Ki = np.linalg.inv(K)
    hom = np.stack([pt_u, pt_v, np.ones_like(pt_u)], 1).astype(np.float64) @ Ki.T
    ok_all = np.zeros((len(pt_host), n_frames), bool)
    for hst in range(n_frames):
        sel = np.nonzero(pt_host == hst)[0]
        Rh, th = se3_from_data(evals[hst])
        for t in range(n_frames):
            if t == hst or len(sel) == 0:
                continue
            Rt, tt = se3_from_data(evals[t])
            R = Rt @ Rh.T
            tr = tt - R @ th
            q = hom[sel] @ R.T + tr[None, :] * pt_id[sel, None].astype(np.float64)
            with np.errstate(divide="ignore", invalid="ignore"):
                ku = K[0, 0] * q[:, 0] / q[:, 2] + K[0, 2]
                kv = K[1, 1] * q[:, 1] / q[:, 2] + K[1, 2]
            ok_all[sel, t] = (q[:, 2] > 0) & (ku > 5.0) & (ku < width - 6) & (kv > 5.0) & (kv < height - 6)
    rp, rt = np.nonzero(ok_all)   # row-major: grouped by point, targets ascending
    rp = rp.astype(np.int32)
    rt = rt.astype(np.int32)
    return BAScene(
        width=width, height=height, K=K, n_levels=levels,
        frames_pose=poses, frames_eval=evals,
        frames_state=np.zeros((n_frames, 10)), frames_state_zero=np.zeros((n_frames, 10)),
        frames_exposure=np.ones(n_frames, np.float32),
        frames_energyTH=np.full(n_frames, 8 * 8 * 8, np.float32),
        frames_id=np.arange(n_frames, dtype=np.int32),
        pyramids=pyrs,
        pt_host=pt_host, pt_u=pt_u, pt_v=pt_v, pt_idepth=pt_id, pt_idepth_zero=pt_id.copy(),
        pt_color=np.ascontiguousarray(np.concatenate(cols)), pt_weights=np.ascontiguousarray(np.concatenate(wts)),
        pt_idepth_true=np.concatenate(idt),
        res_point=rp, res_target=rt, planes=planes)


KITTI_W, KITTI_H = 1232, 368   # Extras/Calib/Kitti00to02.yaml output size


def make_ba_scene_kitti(n_points: int = 2000, n_frames: int = 8, seed: int = SEED) -> BAScene:
    """C5's BA half (BASELINE.json configs[4]): the C4 window at KITTI 1232x368, 5 pyramid levels, fx = fy =
    718.856.  The pose / depth perturbations are the C4 ones scaled by the focal-length ratio (256 / 718.9), so
    the initial pixel errors, and with them the IN / OUT mix of the first linearization, match C4's."""
    return make_ba_scene(n_points=n_points, n_frames=n_frames, width=KITTI_W, height=KITTI_H, seed=seed,
                         kitti=True, pose_noise=(0.0015, 0.0007), idepth_noise=0.004)


def render_depth_at(planes, K, R_c2w, C, pix):
    """Depth (camera Z) of the visible surface at integer pixels (y, x)."""
    ys = pix[:, 0].astype(np.float64)
    xs = pix[:, 1].astype(np.float64)
    Ki = np.linalg.inv(K)
    d = np.stack([xs, ys, np.ones_like(xs)], -1) @ Ki.T
    dw = d @ R_c2w.T
    best = np.full(len(xs), np.inf)
    for p in planes:
        s = (p.z - C[2]) / dw[:, 2]
        X = C[0] + s * dw[:, 0]
        Y = C[1] + s * dw[:, 1]
        ok = (s > 0) & (X >= p.xmin) & (X <= p.xmax) & (Y >= p.ymin) & (Y <= p.ymax) & (s < best)
        best[ok] = s[ok]
    return None, best * d[:, 2]


# ----------------------------------------------------------------- tracking pair (C2 / C5)
@dataclass
class TrackScene:
    width: int
    height: int
    K: np.ndarray                 # level-0 intrinsics (fp64)
    n_levels: int
    ref_pyr: list                 # lastRef DirPyr: per level (h_l, w_l, 3) float32
    new_pyr: list                 # the frame being tracked
    ref_exposure: float
    new_exposure: float
    ref_aff: np.ndarray           # lastRef aff_g2l (a, b)
    pt_u: np.ndarray              # [n] float32 centerProjectedTo u in lastRef
    pt_v: np.ndarray
    pt_idepth: np.ndarray         # [n] float32 centerProjectedTo idepth
    pt_hdi: np.ndarray            # [n] float32 point HdiF
    T_true: np.ndarray            # [7] true refToNew (SE3 data)
    aff_true: np.ndarray          # [2] true aff_g2l of the new frame
    planes: list = field(default=None, repr=False)

    @property
    def K4(self):
        return np.array([self.K[0, 0], self.K[1, 1], self.K[0, 2], self.K[1, 2]], np.float32)


def make_track_scene(n_points: int = 2000, width: int = 640, height: int = 480, K=None, seed: int = SEED,
                     trans: float = 0.02, rot_deg: float = 0.5, a: float = 0.05, b: float = 3.0,
                     idepth_noise: float = 0.01, dup_frac: float = 0.05, kitti: bool = False,
                     n_levels: int | None = None) -> TrackScene:
    """lastRef + a new frame moved by (rot_deg about a random axis, trans m in a random direction) and
    re-lit by I_new = e^a I + b.  The reference points are the centre projections of window points into
    lastRef (sub-pixel positions, idepth with 1% noise, HdiF in [5e-4, 2e-3]); dup_frac of them are
    near-duplicates that round to the same pixel, exercising the scatter-add order of makeCoarseDepthL0."""
    rng = np.random.default_rng(seed + 7)
    if K is None:
        K = (np.array([[718.856, 0, 615.5], [0, 718.856, 183.5], [0, 0, 1.0]]) if kitti
             else np.array([[256.0, 0, 319.5], [0, 254.4, 239.5], [0, 0, 1.0]]))
    K = np.asarray(K, dtype=np.float64)
    f = K[0, 0]
    planes = [make_plane(rng, 5.0, f), make_plane(rng, 3.0, f, xmax=-0.25), make_plane(rng, 2.0, f, xmin=0.55, ymax=0.15)]
    levels = n_levels or min(pyramid_levels(width, height), 5)
    R_ref_c2w = rodrigues(np.array([0.0, 0.01, 0.0]))
    C_ref = np.array([0.3, 0.0, 0.0])
    img_ref, _ = render(planes, K, R_ref_c2w, C_ref, width, height)
    ax = rng.normal(size=3)
    ax /= np.linalg.norm(ax)
    dR = rodrigues(ax * math.radians(rot_deg))
    dt = rng.normal(size=3)
    dt *= trans / np.linalg.norm(dt)
    # refToNew = (dR, dt): X_new = dR X_ref + dt
    R_new_w2c = dR @ R_ref_c2w.T
    t_new_w2c = dR @ (-R_ref_c2w.T @ C_ref) + dt
    R_new_c2w = R_new_w2c.T
    C_new = -R_new_c2w @ t_new_w2c
    img_new, _ = render(planes, K, R_new_c2w, C_new, width, height, a=a, b=b)
    ref_pyr = make_dir_pyramid(img_ref, levels)
    new_pyr = make_dir_pyramid(img_new, levels)
    n_dup = int(round(n_points * dup_frac))
    n_base = n_points - n_dup
    pix = _select_points(ref_pyr[0], n_base, 6, rng)
    u = pix[:, 1] + rng.uniform(-0.45, 0.45, n_base)
    v = pix[:, 0] + rng.uniform(-0.45, 0.45, n_base)
    _, depth = render_depth_at(planes, K, R_ref_c2w, C_ref, pix)
    idp = (1.0 / depth) * (1.0 + idepth_noise * rng.normal(size=n_base))
    if n_dup:
        src = rng.integers(0, n_base, n_dup)
        du = np.round(u[src]) + rng.uniform(-0.45, 0.45, n_dup)
        dv = np.round(v[src]) + rng.uniform(-0.45, 0.45, n_dup)
        u = np.concatenate([u, du])
        v = np.concatenate([v, dv])
        idp = np.concatenate([idp, idp[src] * (1.0 + idepth_noise * rng.normal(size=n_dup))])
        perm = rng.permutation(n_points)
        u, v, idp = u[perm], v[perm], idp[perm]
    hdi = rng.uniform(5e-4, 2e-3, n_points)
    return TrackScene(width=width, height=height, K=K, n_levels=levels, ref_pyr=ref_pyr, new_pyr=new_pyr,
                      ref_exposure=1.0, new_exposure=1.0, ref_aff=np.zeros(2),
                      pt_u=u.astype(np.float32), pt_v=v.astype(np.float32), pt_idepth=idp.astype(np.float32),
                      pt_hdi=hdi.astype(np.float32), T_true=se3_data(dR, dt), aff_true=np.array([a, b]),
                      planes=planes)


# ----------------------------------------------------------------- immature-point tracing (C5)
@dataclass
class TraceScene:
    width: int
    height: int
    K: np.ndarray                 # level-0 intrinsics (fp64)
    host_imgs: list               # per host KF: DirPyr[0] (h, w, 3) float32
    new_img: np.ndarray           # the new frame's DirPyr[0]
    KRKi: np.ndarray              # [nH, 9] float32 (traceNewCoarse, Src/Mapping.cpp:505-507)
    Kt: np.ndarray                # [nH, 3] float32
    aff: np.ndarray               # [nH, 2] float32 (AffLight::fromToVecExposure host -> new)
    pt_host: np.ndarray           # [n] int32
    pt_u: np.ndarray              # [n] float32
    pt_v: np.ndarray
    pt_idepth_true: np.ndarray    # [n] float64 (ground truth, for interval variants)
    planes: list = field(default=None, repr=False)

    @property
    def n_points(self):
        return len(self.pt_u)

    @property
    def n_hosts(self):
        return len(self.host_imgs)

    def finite_intervals(self, seed: int = 3):
        """A second-trace state: [idepth_min, idepth_max] around the true idepth with widths from 0.2% to 60%
        (mixes SKIPPED, BADCONDITION and GOOD), some intervals offset so the truth lies outside."""
        rng = np.random.default_rng(seed)
        n = self.n_points
        w = np.exp(rng.uniform(np.log(0.002), np.log(0.6), n))
        c = self.pt_idepth_true * (1.0 + rng.normal(0, 0.05, n))
        lo = np.maximum(c * (1.0 - w), 0.0)
        hi = c * (1.0 + w)
        return lo.astype(np.float32), hi.astype(np.float32)


def make_trace_scene(n_points: int = 20000, n_hosts: int = 8, width: int = 1232, height: int = 368, K=None,
                     seed: int = SEED, spacing: float = 0.02, new_offset=(0.02, 0.03, 0.01), a: float = 0.05,
                     b: float = 3.0, max_rot_deg: float = 0.5, subpixel_frac: float = 0.3) -> TraceScene:
    """n_hosts keyframes spaced `spacing` m along x and one new frame `new_offset` past the last one, relit by
    I_new = e^a I + b.  n_points immature points (n_points / n_hosts per host) at the top-gradient pixel per
    cell (a fraction at sub-pixel positions).  Default = C5 (KITTI 1232x368, 20k points, 8 hosts)."""
    rng = np.random.default_rng(seed + 13)
    if K is None:
        K = (np.array([[718.856, 0, 615.5], [0, 718.856, 183.5], [0, 0, 1.0]]) if width >= 1000
             else np.array([[256.0, 0, 319.5], [0, 254.4, 239.5], [0, 0, 1.0]]))
    K = np.asarray(K, dtype=np.float64)
    f = K[0, 0]
    planes = [make_plane(rng, 5.0, f), make_plane(rng, 3.0, f, xmax=-0.25), make_plane(rng, 2.0, f, xmin=0.55, ymax=0.15)]
    poses = []
    imgs = []
    for i in range(n_hosts + 1):
        ax = rng.normal(size=3)
        ax /= np.linalg.norm(ax)
        R_c2w = rodrigues(ax * math.radians(rng.uniform(0, max_rot_deg)))
        C = (np.array([spacing * i, 0.0, 0.0]) if i < n_hosts
             else np.array([spacing * (n_hosts - 1), 0.0, 0.0]) + np.asarray(new_offset, np.float64))
        img, _ = render(planes, K, R_c2w, C, width, height, *((a, b) if i == n_hosts else (0.0, 0.0)))
        imgs.append(make_dir_pyramid(img, 1)[0])
        poses.append((R_c2w, C))
    Rn_c2w, Cn = poses[-1]
    Rn_w2c = Rn_c2w.T
    KRKi, Kt, aff = [], [], []
    Ki = np.linalg.inv(K)
    for i in range(n_hosts):
        Rh_c2w, Ch = poses[i]
        R = Rn_w2c @ Rh_c2w                  # hostToNew = worldToNew * hostToWorld
        t = Rn_w2c @ (Ch - Cn)
        KRKi.append((K @ R @ Ki).astype(np.float32).reshape(9))
        Kt.append((K @ t).astype(np.float32))
        aff.append(np.array([math.exp(a), b], np.float32))
    per = [n_points // n_hosts + (1 if i < n_points % n_hosts else 0) for i in range(n_hosts)]
    hosts, us, vs, idt = [], [], [], []
    for h in range(n_hosts):
        if per[h] == 0:
            continue
        pix = _select_points(imgs[h], per[h], 8, rng)
        Rh_c2w, Ch = poses[h]
        _, depth = render_depth_at(planes, K, Rh_c2w, Ch, pix)
        u = pix[:, 1].astype(np.float64)
        v = pix[:, 0].astype(np.float64)
        sub = rng.uniform(size=len(u)) < subpixel_frac
        u[sub] += rng.uniform(-0.45, 0.45, sub.sum())
        v[sub] += rng.uniform(-0.45, 0.45, sub.sum())
        hosts.append(np.full(len(u), h, np.int32))
        us.append(u.astype(np.float32))
        vs.append(v.astype(np.float32))
        idt.append(1.0 / depth)
    return TraceScene(width=width, height=height, K=K, host_imgs=imgs[:n_hosts], new_img=imgs[-1],
                      KRKi=np.array(KRKi), Kt=np.array(Kt), aff=np.array(aff), pt_host=np.concatenate(hosts),
                      pt_u=np.concatenate(us), pt_v=np.concatenate(vs), pt_idepth_true=np.concatenate(idt),
                      planes=planes)


# ----------------------------------------------------------------- point activation
@dataclass
class ActivationScene:
    width: int
    height: int
    K: np.ndarray                 # level-0 intrinsics (fp64)
    imgs: list                    # per window KF: DirPyr[0] (h, w, 3) float32
    slots: np.ndarray             # [nF] tracer image slot of each KF
    flagged: np.ndarray           # [nF] FlaggedForMarginalization
    KRKi1: np.ndarray             # [nF, 9] float32 CoarseDistanceMap K[1] R(f -> newest) Ki[0]
    Kt1: np.ndarray               # [nF, 3] float32
    RTll: np.ndarray              # [nF*nF, 9] float32 targetPrecalc PRE_RTll (host-major)
    tTll: np.ndarray              # [nF*nF, 3]
    aff: np.ndarray               # [nF*nF, 2] PRE_aff_mode
    act_frame: np.ndarray         # active MapPoints: window frame, u, v, idepth
    act_u: np.ndarray
    act_v: np.ndarray
    act_idepth: np.ndarray
    imm_frame: np.ndarray         # immature points: host window frame, u, v and their trace state
    imm_u: np.ndarray
    imm_v: np.ndarray
    imm_idepth_min: np.ndarray
    imm_idepth_max: np.ndarray
    imm_quality: np.ndarray
    imm_status: np.ndarray
    imm_interval: np.ndarray
    imm_type: np.ndarray
    order: np.ndarray             # the reference's loop order over the stored points
    ef_nPoints: int
    currentMinActDist: float

    @property
    def n_frames(self):
        return len(self.imgs)

    @property
    def K4(self):
        return np.array([self.K[0, 0], self.K[1, 1], self.K[0, 2], self.K[1, 2]], np.float32)


def make_activation_scene(n_active: int = 1500, n_immature: int = 3000, n_frames: int = 8, width: int = 640,
                          height: int = 480, seed: int = SEED, kitti: bool = False,
                          currentMinActDist: float = 2.0) -> ActivationScene:
    """A window (make_ba_scene's keyframes, evalPT as PRE_worldToCam) with n_active MapPoints and n_immature traced
    immature points on all keyframes: intervals around the true idepth (1% .. 50% wide, some NaN / negative),
    every lastTraceStatus, quality 0..20, lastTracePixelInterval 0..12, my_type 1/2/4.  Points are stored
    interleaved across hosts; `order` is the reference's per-host loop order.  Slots are 2f+1 and keyframe 0 is
    flagged for marginalization."""
    bs = make_ba_scene(n_points=n_active, n_frames=n_frames, width=width, height=height, seed=seed, kitti=kitti,
                       pose_noise=(0.001, 0.0005))
    rng = np.random.default_rng(seed + 29)
    K = bs.K
    nF = n_frames
    Rs, ts = zip(*[se3_from_data(e) for e in bs.frames_eval])
    aff_g2l = np.where(rng.random((nF, 1)) < 0.5, 0.0, rng.uniform([-0.02, -2.0], [0.02, 2.0], (nF, 2)))
    # CoarseDistanceMap::makeK (Src/CoarseTracker.cpp:870-899): level-1 K in float, Ki[0] = K[0].inverse()
    fx0, fy0, cx0, cy0 = (np.float32(x) for x in (K[0, 0], K[1, 1], K[0, 2], K[1, 2]))
    K1 = np.array([[np.float32(fx0 * 0.5), 0, np.float32((float(cx0) + 0.5) / 2 - 0.5)],
                   [0, np.float32(fy0 * 0.5), np.float32((float(cy0) + 0.5) / 2 - 0.5)], [0, 0, 1]], np.float32)
    K0 = np.array([[fx0, 0, cx0], [0, fy0, cy0], [0, 0, 1]], np.float64)
    Ki0 = np.linalg.inv(K0).astype(np.float32)
    new = nF - 1
    KRKi1, Kt1 = [], []
    for f in range(nF):
        R = Rs[new] @ Rs[f].T
        t = ts[new] - R @ ts[f]
        KRKi1.append((K1 @ R.astype(np.float32) @ Ki0).reshape(9))
        Kt1.append(K1 @ t.astype(np.float32))
    RT, tT, af = [], [], []
    for h in range(nF):
        for t_ in range(nF):
            R = Rs[t_] @ Rs[h].T
            RT.append(R.astype(np.float32).reshape(9))
            tT.append((ts[t_] - R @ ts[h]).astype(np.float32))
            a = math.exp(aff_g2l[t_, 0] - aff_g2l[h, 0])
            af.append(np.array([a, aff_g2l[t_, 1] - a * aff_g2l[h, 1]], np.float32))
    # immature points: top-gradient pixels of every host (not the MapPoints' cells), sub-pixel offsets
    per = [n_immature // nF + (1 if i < n_immature % nF else 0) for i in range(nF)]
    fr, us, vs, tru = [], [], [], []
    for f in range(nF):
        if per[f] == 0:
            continue
        pix = _select_points(bs.pyramids[f][0], per[f], 8, rng)
        R_w2c, t_w2c = se3_from_data(bs.frames_pose[f])
        R_c2w = R_w2c.T
        _, depth = render_depth_at(bs.planes, K, R_c2w, -R_c2w @ t_w2c, pix)
        fr.append(np.full(len(pix), f, np.int32))
        us.append(pix[:, 1] + rng.uniform(-0.4, 0.4, len(pix)))
        vs.append(pix[:, 0] + rng.uniform(-0.4, 0.4, len(pix)))
        tru.append(1.0 / depth)
    fr, us, vs, tru = (np.concatenate(x) for x in (fr, us, vs, tru))
    n = len(fr)
    c = tru * (1.0 + rng.normal(0, 0.02, n))
    w = np.exp(rng.uniform(np.log(0.01), np.log(0.5), n))
    lo, hi = c * (1.0 - w), c * (1.0 + w)
    hi[rng.random(n) < 0.05] = np.nan
    neg = rng.random(n) < 0.02
    lo[neg] = -hi[neg] - 0.01
    status = rng.choice(6, n, p=[0.45, 0.1, 0.1, 0.1, 0.1, 0.15]).astype(np.uint8)  # IPS_* order: G,OOB,OUT,SK,BC,UN
    perm = rng.permutation(n)
    fr, us, vs, lo, hi, status = fr[perm], us[perm], vs[perm], lo[perm], hi[perm], status[perm]
    order = np.argsort(fr, kind="stable").astype(np.int32)
    return ActivationScene(
        width=width, height=height, K=K, imgs=bs.images_level0(), slots=(2 * np.arange(nF) + 1).astype(np.int32),
        flagged=(np.arange(nF) == 0).astype(np.int32), KRKi1=np.array(KRKi1, np.float32),
        Kt1=np.array(Kt1, np.float32), RTll=np.array(RT, np.float32), tTll=np.array(tT, np.float32),
        aff=np.array(af, np.float32), act_frame=bs.pt_host.astype(np.int32), act_u=bs.pt_u, act_v=bs.pt_v,
        act_idepth=bs.pt_idepth, imm_frame=fr, imm_u=us.astype(np.float32), imm_v=vs.astype(np.float32),
        imm_idepth_min=lo.astype(np.float32), imm_idepth_max=hi.astype(np.float32),
        imm_quality=rng.uniform(0, 20, n).astype(np.float32), imm_status=status,
        imm_interval=rng.uniform(0, 12, n).astype(np.float32),
        imm_type=rng.choice([1.0, 2.0, 4.0], n, p=[0.6, 0.25, 0.15]).astype(np.float32), order=order,
        ef_nPoints=n_active, currentMinActDist=currentMinActDist)


def make_select_frames(n_frames: int = 3, width: int = 640, height: int = 480, seed: int = SEED,
                       quantize: bool = False, flat_frac: float = 0.0, contrast_ramp: bool = False):
    """Raw level-0 frames for PixelSelector::makeMaps (Src/PixelSelector.cpp:118-262): the textured planes seen from
    a camera drifting along x.  quantize=True rounds to 8-bit values, as a camera image, so gradients are multiples
    of 0.5 and axis-aligned / diagonal ones score exactly 0 against some directions (the ambiguous-slot path of the
    device select).  flat_frac blanks that fraction of the image rows (textureless regions); contrast_ramp scales the
    texture contrast from 3% at the left edge to 100% at the right, so cells span the regimes where select takes a
    level-0, a level-1 (2pot) or a level-2 (4pot) pixel."""
    rng = np.random.default_rng(seed + 29)
    K = (np.array([[718.856, 0, 615.5], [0, 718.856, 183.5], [0, 0, 1.0]]) if width >= 1000
         else np.array([[0.4 * width, 0, width / 2 - 0.5], [0, 0.53 * height, height / 2 - 0.5], [0, 0, 1.0]]))
    f = K[0, 0]
    planes = [make_plane(rng, 5.0, f), make_plane(rng, 3.0, f, xmax=-0.25), make_plane(rng, 2.0, f, xmin=0.55, ymax=0.15)]
    out = []
    for i in range(n_frames):
        ax = rng.normal(size=3)
        ax /= np.linalg.norm(ax)
        R_c2w = rodrigues(ax * math.radians(rng.uniform(0, 1.0)))
        img, _ = render(planes, K, R_c2w, np.array([0.05 * i, 0.0, 0.0]), width, height)
        if contrast_ramp:
            img = (128.0 + (img - 128.0) * np.linspace(0.03, 1.0, width)[None, :] ** 2).astype(np.float32)
        if flat_frac > 0:
            img[: int(flat_frac * height)] = 128.0
        if quantize:
            img = np.round(img).astype(np.float32)
        out.append(img)
    return out


# ----------------------------------------------------------------- initializer refinement (DirectRefinement)
@dataclass
class RefineScene:
    width: int
    height: int
    K: np.ndarray
    img1: np.ndarray      # FirstFrame DirPyr[0], H*W*3
    img2: np.ndarray      # SecondFrame DirPyr[0]
    expo1: float
    expo2: float
    u: np.ndarray         # mvKeys[i].pt (sub-pixel)
    v: np.ndarray
    tri: np.ndarray       # Triangulated[i]
    z: np.ndarray         # Pts3D[i].z (noisy where triangulated, 1 elsewhere)
    T_true: np.ndarray    # refToNew (first -> second), SE3 data
    T_init: np.ndarray    # the initializer's pose handed to DirectRefinement

    @property
    def n_points(self):
        return len(self.u)

    @property
    def K4(self):
        return np.array([self.K[0, 0], self.K[1, 1], self.K[0, 2], self.K[1, 2]], np.float64)


def make_refine_scene(n_points: int = 2000, width: int = 640, height: int = 480, K=None, seed: int = SEED,
                      trans: float = 0.15, rot_deg: float = 2.0, tri_frac: float = 0.85, z_noise: float = 0.03,
                      pose_rot_deg: float = 0.3, pose_trans_frac: float = 0.1, exposures=(1.0, 1.0)) -> RefineScene:
    """Two frames of the textured-plane world with a wide baseline (the monocular initializer's pair), ORB-like
    sub-pixel keypoints in the first frame, Triangulated for tri_frac of them with Pts3D.z carrying z_noise
    relative noise, and an initial refToNew perturbed from the truth (pose_rot_deg, pose_trans_frac of |t|)."""
    ts = make_track_scene(n_points=n_points, width=width, height=height, K=K, seed=seed, trans=trans,
                          rot_deg=rot_deg, a=0.0, b=0.0, idepth_noise=0.0, dup_frac=0.0, n_levels=1)
    rng = np.random.default_rng(seed + 11)
    n = len(ts.pt_u)
    tri = (rng.random(n) < tri_frac).astype(np.uint8)
    z = (1.0 / ts.pt_idepth.astype(np.float64)) * (1.0 + z_noise * rng.normal(size=n))
    z = np.where(tri == 1, z, 1.0).astype(np.float32)
    R_true, t_true = quat_to_rot(ts.T_true[:4]), ts.T_true[4:]
    ax = rng.normal(size=3)
    ax /= np.linalg.norm(ax)
    dR = rodrigues(ax * math.radians(pose_rot_deg))
    dt = rng.normal(size=3)
    dt *= pose_trans_frac * np.linalg.norm(t_true) / np.linalg.norm(dt)
    T_init = se3_data(dR @ R_true, t_true + dt)
    return RefineScene(width=width, height=height, K=ts.K, img1=ts.ref_pyr[0], img2=ts.new_pyr[0],
                       expo1=float(exposures[0]), expo2=float(exposures[1]), u=ts.pt_u, v=ts.pt_v, tri=tri, z=z,
                       T_true=ts.T_true, T_init=T_init)
