"""The keyframe path of the BA through the incremental C-ABI: System::AddKeyframe's BA part (Src/Mapping.cpp:12-140).

A synthetic keyframe *sequence* (``make_ba_sequence``: the C4 / C5 scenes' planes, a camera translating along x) and a
driver (``KeyframeBA``) that runs, per keyframe, what AddKeyframe does around the BA:

    insertFrame + setPrecalcValues                     hs_ba_insert_frame (image from the device or a raw upload)
    new residuals of the old points into the new KF    hs_ba_add_residuals_to_newest
    activatePointsMT's new points and residuals        hs_ba_insert_points / hs_ba_insert_residuals
    makeIDX + optimize(6) + the tail                   hs_ba_optimize / hs_ba_fix_linearization
    linearizeAll(true)'s toRemove, removeOutliers      hs_ba_drop_inactive_residuals / _remove_points_without_residuals
    setCoarseTrackingRef (optional tracker)            hs_tracker_set_ref_ba (device hand-off)
    flagPointsForRemoval + marginalizePointsF          (decisions here, System code) + hs_ba_marginalize_points /
                                                       hs_ba_remove_points
    marginalizeFrame                                   hs_ba_remove_frame(marginalize=1)

The System-level decisions (which frame to marginalize, flagPointsForRemoval's per-point tests, the lastResiduals
bookkeeping) are the caller's code in the reference too; they run here in numpy and are not part of the timed library
work.  Frame policy: the window holds ``window`` keyframes during optimize and the oldest is marginalized afterwards
(flagFramesForMarginalization's steady state; its distance score and point-count rules are not modelled).
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass

import numpy as np

from .ba import BAWindow, make_frame
from .scene import (PATTERN, SEED, _select_points, make_dir_pyramid, make_plane, pyramid_levels, render,
                    render_depth_at, rodrigues, se3_data, se3_from_data)

RES_IN, RES_OOB, RES_OUT = 0, 1, 2
MIN_GOOD_ACTIVE_RES_FOR_MARG = 3   # setting_minGoodActiveResForMarg (Src/Settings.cpp:96)
MIN_GOOD_RES_FOR_MARG = 4          # setting_minGoodResForMarg (:97)
MIN_IDEPTH_H_MARG = 50.0           # setting_minIdepthH_marg (:119)


@dataclass
class BASequence:
    width: int
    height: int
    K: np.ndarray
    n_levels: int
    poses: np.ndarray        # [N, 7] true worldToCam
    evals: np.ndarray        # [N, 7] the poses the BA starts from (noisy, frame 0 exact)
    raw: list                # [N] (h, w) float32 level-0 images (ImageData::fImgL)
    pyr0: list               # [N] (h, w, 3) float32 DirPyr[0]
    cand: list               # [N] dict(u, v, idepth, idepth_true, color [n, 8], weights [n, 8]): points hosted there

    @property
    def n_frames(self):
        return len(self.raw)


def make_ba_sequence(n_kf: int = 12, points_per_kf: int = 250, width: int = 640, height: int = 480, K=None,
                     seed: int = SEED, baseline: float = 0.06, max_rot_deg: float = 1.0, pose_noise=(0.004, 0.002),
                     idepth_noise: float = 0.01, kitti: bool = False) -> BASequence:
    """n_kf keyframes of the C4 scene (C5's at KITTI size with kitti=True): camera i at x = baseline * i."""
    rng = np.random.default_rng(seed)
    if K is None:
        K = (np.array([[718.856, 0, 615.5], [0, 718.856, 183.5], [0, 0, 1.0]]) if kitti else
             np.array([[256.0, 0, 319.5], [0, 254.4, 239.5], [0, 0, 1.0]]))
    K = np.asarray(K, np.float64)
    f = K[0, 0]
    if kitti:  # the C4 perturbations in pixels (scene.make_ba_scene_kitti)
        s = 256.0 / f
        pose_noise = (pose_noise[0] * s, pose_noise[1] * s)
        idepth_noise *= s
    planes = [make_plane(rng, 5.0, f), make_plane(rng, 3.0, f, xmax=-0.25 + baseline * n_kf),
              make_plane(rng, 2.0, f, xmin=0.55, ymax=0.15)]
    levels = pyramid_levels(width, height)
    poses, evals, raws, pyrs, cands = [], [], [], [], []
    for i in range(n_kf):
        ax = rng.normal(size=3)
        ax /= np.linalg.norm(ax)
        R_c2w = rodrigues(ax * math.radians(rng.uniform(0, max_rot_deg)))
        C = np.array([baseline * i, 0.0, 0.0])
        img, _ = render(planes, K, R_c2w, C, width, height)
        pyr = make_dir_pyramid(img, 1)
        R_w2c = R_c2w.T
        t_w2c = -R_w2c @ C
        poses.append(se3_data(R_w2c, t_w2c))
        if i == 0:
            evals.append(se3_data(R_w2c, t_w2c))
        else:
            dR = rodrigues(rng.normal(size=3) * pose_noise[1])
            dt = rng.normal(size=3) * pose_noise[0]
            evals.append(se3_data(dR @ R_w2c, dR @ t_w2c + dt))
        raws.append(img)
        pyrs.append(pyr[0])
        pix = _select_points(pyr[0], points_per_kf, 4, rng)
        _, depth = render_depth_at(planes, K, R_c2w, C, pix)
        smp = pyr[0][pix[:, 0:1] + PATTERN[None, :, 1], pix[:, 1:2] + PATTERN[None, :, 0]]
        gx, gy = smp[..., 1], smp[..., 2]
        c2500 = np.float32(2500.0)
        wgt = np.sqrt(c2500 / (c2500 + (gx * gx + gy * gy))).astype(np.float32)
        it = 1.0 / depth
        cands.append(dict(u=pix[:, 1].astype(np.float32), v=pix[:, 0].astype(np.float32),
                          idepth=(it * (1.0 + idepth_noise * rng.normal(size=len(pix)))).astype(np.float32),
                          idepth_true=it, color=np.ascontiguousarray(smp[..., 0], np.float32),
                          weights=np.ascontiguousarray(wgt)))
    return BASequence(width=width, height=height, K=K, n_levels=levels, poses=np.array(poses), evals=np.array(evals),
                      raw=raws, pyr0=pyrs, cand=cands)


def in_bounds_targets(seq: BASequence, host: int, targets, u, v, idepth):
    """[n, len(targets)] bool: the point's centre projects inside the image of each target (evalPT poses), the
    residual set the activation's optimizeImmaturePoint keeps IN on a photo-consistent scene."""
    K = seq.K
    hom = np.stack([u, v, np.ones_like(u)], 1).astype(np.float64) @ np.linalg.inv(K).T
    Rh, th = se3_from_data(seq.evals[host])
    out = np.zeros((len(u), len(targets)), bool)
    for j, t in enumerate(targets):
        if t == host:
            continue
        Rt, tt = se3_from_data(seq.evals[t])
        R = Rt @ Rh.T
        tr = tt - R @ th
        q = hom @ R.T + tr[None, :] * idepth[:, None].astype(np.float64)
        with np.errstate(divide="ignore", invalid="ignore"):
            ku = K[0, 0] * q[:, 0] / q[:, 2] + K[0, 2]
            kv = K[1, 1] * q[:, 1] / q[:, 2] + K[1, 2]
        out[:, j] = (q[:, 2] > 0) & (ku > 5.0) & (ku < seq.width - 6) & (kv > 5.0) & (kv < seq.height - 6)
    return out


class _Timer:
    """Wall time spent inside library calls, per phase (the driver's own numpy bookkeeping excluded)."""

    def __init__(self):
        self.t = {}
        self.calls = {}  # per library call (phase/function name)

    def run(self, phase, fn, *a, **k):
        t0 = time.perf_counter()
        r = fn(*a, **k)
        dt = time.perf_counter() - t0
        self.t[phase] = self.t.get(phase, 0.0) + dt
        name = f"{phase}/{getattr(fn, '__name__', 'call')}"
        self.calls[name] = self.calls.get(name, 0.0) + dt
        return r


class KeyframeBA:
    """System::AddKeyframe's BA part over a BASequence, through the incremental C-ABI (module docstring)."""

    def __init__(self, seq: BASequence, device: int = 0, window: int = 8, capacity: int = 0, params=None,
                 tracker=None, image_path: str = "raw", iters: int = 6, allow_break: bool = False):
        self.seq = seq
        self.window = window
        self.iters = iters
        # System::optimize's canbreak (Src/FullSystemOptimize.cpp:493), tested on the device; off by default so that
        # a parity run's iteration count cannot flip on a borderline step norm
        self.allow_break = allow_break
        self.tracker = tracker
        self.image_path = image_path
        ppk = len(seq.cand[0]["u"])
        cap = capacity or ppk * (window + 2) + 64
        self.ba = BAWindow(camera=(seq.width, seq.height, seq.n_levels, seq.K), capacity=cap, device=device,
                           params=params)
        self.frames = []                 # window frames as sequence indices (frameHessians order)
        self.cand_of = {}                # handle -> (host sequence index, candidate index)
        self.last_state = {}             # handle -> [lastResiduals[0].second, [1].second] (System bookkeeping)
        self.history = []

    # ---------------------------------------------------------------- helpers
    def _frame(self, k):
        s = self.seq
        return make_frame(s.evals[k], exposure=1.0, energyTH=8 * 8 * 8, fid=k)

    def _insert_frame(self, k, timer):
        ba = self.ba
        if self.image_path == "host":
            timer.run("setup", ba.insertFrame, self._frame(k), image=self.seq.pyr0[k])
        elif self.image_path in ("device", "device_ptr") and self.tracker is not None:
            # the frame was tracked before it became a keyframe: its pyramid is already on the device (tracking
            # work, reported apart from the BA's)
            timer.run("track_frame", self.tracker.set_frame_raw, self.seq.raw[k])
            if self.image_path == "device_ptr":  # through the texels' address (hs_ba_set_frame_image_device)
                timer.run("setup", ba.insertFrame, self._frame(k), device_texels=self.tracker.frame_texels(0))
            else:
                timer.run("setup", ba.insertFrame, self._frame(k), tracker=self.tracker)
        else:
            timer.run("setup", ba.insertFrame, self._frame(k), raw=self.seq.raw[k])
        self.frames.append(k)

    def _activate(self, host_k, timer, cand_idx=None):
        """activatePointsMT's result for the points hosted by sequence frame host_k: insertPoint + insertResidual
        into every other window frame the centre projects into."""
        c = self.seq.cand[host_k]
        idx = np.arange(len(c["u"])) if cand_idx is None else np.asarray(cand_idx)
        h = self.frames.index(host_k)
        ok = in_bounds_targets(self.seq, host_k, self.frames, c["u"][idx], c["v"][idx], c["idepth"][idx])
        keep = ok.sum(1) > 0
        idx, ok = idx[keep], ok[keep]
        handles = timer.run("setup", self.ba.insertPoints, np.full(len(idx), h, np.int32), c["u"][idx], c["v"][idx],
                            c["idepth"][idx], c["idepth"][idx], c["color"][idx], c["weights"][idx])
        pi, ti = np.nonzero(ok)
        timer.run("setup", self.ba.insertResiduals, handles[pi], ti.astype(np.int32))
        newest, second = len(self.frames) - 1, len(self.frames) - 2
        for j, hd in enumerate(handles):
            self.cand_of[int(hd)] = (host_k, int(idx[j]))
            self.last_state[int(hd)] = [RES_IN if ok[j, newest] else RES_OOB,
                                        RES_IN if second >= 0 and ok[j, second] else RES_OOB]
        return handles

    # ---------------------------------------------------------------- the sequence
    def bootstrap(self, n_frames=None):
        """The first window: keyframes 0 .. n-1 with the points of frames 0 .. n-2 (the newest KF's points activate
        with the next keyframe, as in the steady state)."""
        n = n_frames or self.window - 1
        timer = _Timer()
        for k in range(n):
            self._insert_frame(k, timer)
        for k in range(n - 1):
            self._activate(k, timer)
        self.ba.makeIDX()

    def add_keyframe(self, k, marginalize=True, check=None):
        """AddKeyframe(k)'s BA part.  check(driver, phase) is called at 'optimize' (before it), 'tail' (after the
        tail, before its drops), and with marginalization at 'marginalize' (before marginalizePointsF of
        self.marg_points), 'points_marginalized' (after it) and 'frame_marginalized' (after marginalizeFrame of
        self.marg_frame): parity tests rebuild the window there.  Returns dict of per-phase seconds."""
        ba, timer = self.ba, _Timer()
        wall0 = time.perf_counter()
        # insertFrame, new residuals of the old points, activation of the previous newest KF's points
        self._insert_frame(k, timer)
        timer.run("setup", ba.addResidualsToNewest)
        for hd, st in self.last_state.items():
            st[1], st[0] = st[0], RES_IN
        self._activate(self.frames[-2], timer)
        timer.run("setup", ba.makeIDX)
        timer.run("setup", ba.synchronize)
        if check:
            check(self, "optimize")
        # optimize + tail
        n_it, energies = timer.run("optimize", ba.optimize, self.iters, self.allow_break)
        # the per-point maxRelBaseline / numGoodResiduals stay on the device (read with point_state when needed)
        tail = self.last_tail = timer.run("tail", ba.fixLinearization, None, None, False)
        if check:
            check(self, "tail")
        # lastResiduals[.].second from the tail's states (System::linearizeAll(true), Src/FullSystemOptimize.cpp:128)
        st = ba.structure()
        res = ba.residuals()
        handles = st["handles"]
        newest, second = len(self.frames) - 1, len(self.frames) - 2
        for r in np.nonzero((st["res_target"] == newest) | (st["res_target"] == second))[0]:
            hd = int(handles[st["res_point"][r]])
            self.last_state[hd][0 if st["res_target"][r] == newest else 1] = int(res["state"][r])
        hdif = tail["HdiF"]
        # toRemove, removeOutliers, the tracker's new reference
        timer.run("post", ba.dropInactiveResiduals)
        gone = timer.run("post", ba.removeOutliers)
        for hd in gone:
            self.cand_of.pop(int(hd), None)
            self.last_state.pop(int(hd), None)
        if self.tracker is not None:
            timer.run("post", self.tracker.set_ref_ba, ba, self.image_path in ("device", "device_ptr"))
        # flagPointsForRemoval (Src/Mapping.cpp:248-328), the frame to marginalize: the oldest once the window is full
        info = dict(energies=energies, iters=n_it, n_points=ba.n_points, n_res=ba.n_res, dropped_points=len(gone))
        if marginalize and len(self.frames) >= self.window:
            marg_f = 0
            st = ba.structure()
            ps = ba.point_state()
            res = ba.residuals()
            hd_all, host, nres = st["handles"], st["pt_host"], st["nres"]
            # the tail's per-point values in the tail's layout -> by handle (removeOutliers only removed points)
            vis_marg = np.zeros(len(hd_all), np.int32)
            sel = (st["res_target"] == marg_f) & (res["state"] == RES_IN)
            np.add.at(vis_marg, st["res_point"][sel], 1)
            last0 = np.array([self.last_state[int(h)][0] for h in hd_all])
            last1 = np.array([self.last_state[int(h)][1] for h in hd_all])
            ng = ps["numGoodResiduals"]
            oob = ((nres >= MIN_GOOD_ACTIVE_RES_FOR_MARG) & (ng > MIN_GOOD_RES_FOR_MARG + 10) &
                   (nres - vis_marg < MIN_GOOD_ACTIVE_RES_FOR_MARG))
            oob |= last0 == RES_OOB
            oob |= (nres >= 2) & (last0 == RES_OUT) & (last1 == RES_OUT)
            flag = oob | (host == marg_f)
            drop_now = (ps["idepth"] < 0) | (nres == 0)
            inl = (nres >= MIN_GOOD_ACTIVE_RES_FOR_MARG) & (ng >= MIN_GOOD_RES_FOR_MARG)
            hdif_now = self._hdif_by_handle(hd_all, tail_handles=handles, hdif=hdif)
            with np.errstate(divide="ignore"):
                idepth_h = np.where(hdif_now > 0, 1.0 / hdif_now, 0.0)
            marg = flag & ~drop_now & inl & (idepth_h > MIN_IDEPTH_H_MARG)
            drop = drop_now | (flag & ~marg)
            mpos = np.nonzero(marg)[0].astype(np.int32)
            self.marg_points, self.marg_frame = mpos, marg_f
            if check:
                check(self, "marginalize")  # before marginalizePointsF: the window as the tail and drops left it
            if len(mpos):
                timer.run("post", ba.marginalizePointsF, mpos, False)
            if check:
                check(self, "points_marginalized")
            rm = hd_all[marg | drop]
            timer.run("post", ba.removePoints, rm)
            for hd in rm:
                self.cand_of.pop(int(hd), None)
                self.last_state.pop(int(hd), None)
            timer.run("post", ba.removeFrame, marg_f, True)
            self.frames.pop(marg_f)
            if check:
                check(self, "frame_marginalized")
            info.update(marginalized_points=int(marg.sum()), dropped=int(drop.sum()))
        timer.run("post", ba.synchronize)
        info["wall_s"] = time.perf_counter() - wall0
        info["phase_s"] = dict(timer.t)
        info["call_s"] = dict(timer.calls)
        info["lib_s"] = sum(v for p, v in timer.t.items() if p != "track_frame")
        self.history.append(info)
        return info

    @staticmethod
    def _hdif_by_handle(hd_now, tail_handles, hdif):
        pos = {int(h): i for i, h in enumerate(tail_handles)}
        return np.array([hdif[pos[int(h)]] for h in hd_now], np.float64)
