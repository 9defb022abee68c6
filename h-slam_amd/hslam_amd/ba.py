"""Host-side mirror of the reference's BA call surface over the C-ABI (include/hs_ba.h).

``EnergyFunctional`` / ``System`` method names follow the reference
(Include/EnergyFunctional.h:37-120, Include/System.h:74-98) so a parity test
reads like the reference's own control flow:

    ba = BAWindow(scene)                # insertFrame/insertPoint/insertResidual + makeIDX + setAdjointsF
    E = ba.linearizeAll(reset=True)     # System::linearizeAll(false) + applyRes (+ fused accumulation)
    x = ba.solveSystem(iteration)       # System::solveSystem -> EnergyFunctional::solveSystemF
    ba.doStepFromBackup()               # System::backupState + doStepFromBackup
    ba.optimize(6)                      # System::optimize GN loop
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import (check, default_params, hs_camera, hs_frame, hs_points, hs_residuals, load, ptr)


SOLVER_FIX_LAMBDA = 1e-5  # Src/EnergyFunctional.cpp:707-708


def pack_system_vector(HA, bA, HSC, bSC, energy=0.0, sum_idepth=0.0, n_points=0.0):
    """The vector the ranks of a point-sharded window all-reduce every GN iteration (hs_ba.cpp launch_reduce,
    hs_k_stitch): the upper triangle of HA diag(1+lambda) - HSC / (1+lambda) in the n x n layout
    (solveSystemF's combination, Src/EnergyFunctional.cpp:705-763), bA - bSC, then energy, sum |idepth|, #points.
    Sums over the ranks of the shards' vectors give the full window's."""
    n = HA.shape[0]
    sc = 1.0 / (1 + SOLVER_FIX_LAMBDA)
    H = np.triu(HA - HSC * sc)
    H[np.diag_indices(n)] = np.diag(HA) * (1 + SOLVER_FIX_LAMBDA) - np.diag(HSC) * sc
    return np.concatenate([H.ravel(), bA - bSC, [energy, sum_idepth, n_points]])


def unpack_system_vector(v, n):
    """(H upper triangle mirrored, b, energy) of a packed system vector."""
    H = v[:n * n].reshape(n, n)
    H = np.triu(H) + np.triu(H, 1).T
    return H, v[n * n:n * n + n], v[n * n + n]


def _camera(width, height, n_levels, K):
    return hs_camera(int(width), int(height), int(n_levels), 0, float(K[0, 0]), float(K[1, 1]), float(K[0, 2]),
                     float(K[1, 2]))


def make_frame(evalPT, state=None, state_zero=None, exposure=1.0, energyTH=8 * 8 * 8, fid=1):
    """hs_frame of a keyframe (FrameOptimizationData: evalPT as SE3 data, state / state_zero, ab_exposure,
    frameEnergyTH, id; id 0 takes the strong first-frame prior)."""
    f = hs_frame()
    f.worldToCam_evalPT[:] = list(map(float, evalPT))
    f.state[:] = list(map(float, np.zeros(10) if state is None else state))
    f.state_zero[:] = list(map(float, np.zeros(10) if state_zero is None else state_zero))
    f.ab_exposure = float(exposure)
    f.frameEnergyTH = float(energyTH)
    f.id = int(fid)
    return f


class BAWindow:
    def __init__(self, scene=None, device: int = 0, params=None, point_slice=None, comm=None, camera=None,
                 capacity: int = 0):
        """scene: hslam_amd.scene.BAScene (or any object with the same fields): the whole window at once
        (hs_ba_set_window).  Without a scene, an empty incremental window of `capacity` points for `camera`
        (width, height, n_levels, K) is reserved (hs_ba_reserve) and built with the keyframe calls below.
        point_slice: optional (begin, end) to load only a contiguous shard of the points.
        comm: optional (unique_id_bytes, rank, nranks) -> RCCL communicator (before the window is set)."""
        self.lib = load()
        self.params = params if params is not None else default_params()
        h = C.c_void_p()
        check(self.lib.hs_create(C.byref(h), C.byref(self.params), device))
        self.h = h
        if comm is not None:
            self.comm_init(*comm)
        if scene is not None:
            self.nF = scene.n_frames
            self.dim = 4 + 8 * self.nF
            self._set_window(scene, point_slice)
        else:
            w, hh, nl, K = camera
            self._cam = _camera(w, hh, nl, np.asarray(K, np.float64))
            check(self.lib.hs_ba_reserve(self.h, C.byref(self._cam), int(capacity)))
            self.nF, self.dim, self.n_points, self.n_res = 0, 4, 0, 0

    def _set_window(self, s, point_slice):
        nF = s.n_frames
        cam = hs_camera(s.width, s.height, s.n_levels, 0, float(s.K[0, 0]), float(s.K[1, 1]), float(s.K[0, 2]),
                        float(s.K[1, 2]))
        fr = (hs_frame * nF)()
        for i in range(nF):
            fr[i].worldToCam_evalPT[:] = list(map(float, s.frames_eval[i]))
            fr[i].state[:] = list(map(float, s.frames_state[i]))
            fr[i].state_zero[:] = list(map(float, s.frames_state_zero[i]))
            fr[i].ab_exposure = float(s.frames_exposure[i])
            fr[i].frameEnergyTH = float(s.frames_energyTH[i])
            fr[i].id = int(s.frames_id[i])
        imgs = [np.ascontiguousarray(s.pyramids[i][0], dtype=np.float32) for i in range(nF)]
        img_ptrs = (C.c_void_p * nF)(*[im.ctypes.data for im in imgs])
        if point_slice is None:
            p0, p1 = 0, s.n_points
        else:
            p0, p1 = point_slice
        sel_r = (s.res_point >= p0) & (s.res_point < p1)
        host = np.ascontiguousarray(s.pt_host[p0:p1], np.int32)
        arrs = [np.ascontiguousarray(a[p0:p1], np.float32) for a in (s.pt_u, s.pt_v, s.pt_idepth, s.pt_idepth_zero)]
        col = np.ascontiguousarray(s.pt_color[p0:p1], np.float32)
        wgt = np.ascontiguousarray(s.pt_weights[p0:p1], np.float32)
        # optional per-point depth priors (PointHessian::hasDepthPrior): scene.pt_has_prior (uint8), else none
        hp = getattr(s, "pt_has_prior", None)
        hp = None if hp is None else np.ascontiguousarray(hp[p0:p1], np.uint8)
        self._keep_prior = hp
        pts = hs_points(p1 - p0, ptr(host), *[ptr(a) for a in arrs], ptr(col), ptr(wgt), None if hp is None else ptr(hp))
        rp = np.ascontiguousarray(s.res_point[sel_r] - p0, np.int32)
        rt = np.ascontiguousarray(s.res_target[sel_r], np.int32)
        rs = hs_residuals(len(rp), ptr(rp), ptr(rt), None)
        self.n_points = p1 - p0
        self.n_res = len(rp)
        check(self.lib.hs_ba_set_window(self.h, C.byref(cam), nF, C.cast(fr, C.c_void_p), C.cast(img_ptrs, C.c_void_p),
                                        C.byref(pts), C.byref(rs)))

    # --------------------------------------------------------------- incremental window (keyframe path)
    def _sync(self):
        """EnergyFunctional::makeIDX: commit pending edits; refresh the window sizes."""
        nF, nP, nR = C.c_int(), C.c_int(), C.c_int()
        check(self.lib.hs_ba_make_idx(self.h, C.byref(nF), C.byref(nP), C.byref(nR)))
        self.nF, self.n_points, self.n_res = nF.value, nP.value, nR.value
        self.dim = 4 + 8 * self.nF

    makeIDX = _sync

    def insertFrame(self, frame, image=None, raw=None, device_texels=None, tracker=None):
        """EnergyFunctional::insertFrame (+ the frame's level-0 image: (h, w, 3) (I, dx, dy) host array, or a raw
        (h, w) image whose level 0 is built on the device, or a device pointer of float4 texels, or the frame last
        set on a hslam_amd.track.CoarseTracker, handed over on the device)."""
        img = None if image is None else np.ascontiguousarray(image, np.float32)
        check(self.lib.hs_ba_insert_frame(self.h, C.byref(frame), ptr(img)))
        idx = self._n_frames_mirror = getattr(self, "_n_frames_mirror", self.nF) + 1
        if raw is not None:
            check(self.lib.hs_ba_set_frame_image_raw(self.h, idx - 1, ptr(np.ascontiguousarray(raw, np.float32))))
        if device_texels is not None:
            check(self.lib.hs_ba_set_frame_image_device(self.h, idx - 1, C.c_void_p(device_texels)))
        if tracker is not None:
            tracker.frame_to_ba(self, idx - 1)
        return idx - 1

    def insertPoints(self, host, u, v, idepth, idepth_zero=None, color=None, weights=None, has_prior=None,
                     max_rel_baseline=None, num_good=None):
        """EnergyFunctional::insertPoint for n points (host: window frame index).  Returns their handles."""
        host = np.ascontiguousarray(host, np.int32)
        n = len(host)
        f = [np.ascontiguousarray(a, np.float32) for a in (u, v, idepth, idepth if idepth_zero is None else idepth_zero)]
        col = np.ascontiguousarray(color, np.float32).reshape(n, 8)
        wgt = np.ascontiguousarray(weights, np.float32).reshape(n, 8)
        hp = None if has_prior is None else np.ascontiguousarray(has_prior, np.uint8)
        pts = hs_points(n, ptr(host), *[ptr(a) for a in f], ptr(col), ptr(wgt), None if hp is None else ptr(hp))
        rb = None if max_rel_baseline is None else np.ascontiguousarray(max_rel_baseline, np.float32)
        ng = None if num_good is None else np.ascontiguousarray(num_good, np.int32)
        out = np.zeros(n, np.int32)
        check(self.lib.hs_ba_insert_points(self.h, C.byref(pts), ptr(rb), ptr(ng), ptr(out)))
        return out

    def insertResiduals(self, handles, targets, states=None):
        """EnergyFunctional::insertResidual (appended to each point's residual list)."""
        hd = np.ascontiguousarray(handles, np.int32)
        tg = np.ascontiguousarray(targets, np.int32)
        st = None if states is None else np.ascontiguousarray(states, np.uint8)
        check(self.lib.hs_ba_insert_residuals(self.h, len(hd), ptr(hd), ptr(tg), ptr(st)))

    def addResidualsToNewest(self):
        """AddKeyframe's loop: every point not hosted by the newest frame gets a residual into it (state IN)."""
        n = C.c_int()
        check(self.lib.hs_ba_add_residuals_to_newest(self.h, C.byref(n)))
        return n.value

    def dropResiduals(self, handles, targets):
        hd = np.ascontiguousarray(handles, np.int32)
        tg = np.ascontiguousarray(targets, np.int32)
        check(self.lib.hs_ba_drop_residuals(self.h, len(hd), ptr(hd), ptr(tg)))

    def dropInactiveResiduals(self):
        """linearizeAll(true)'s toRemove loop after fixLinearization."""
        n = C.c_int()
        check(self.lib.hs_ba_drop_inactive_residuals(self.h, C.byref(n)))
        return n.value

    def removePoints(self, handles):
        hd = np.ascontiguousarray(handles, np.int32)
        check(self.lib.hs_ba_remove_points(self.h, len(hd), ptr(hd)))

    def removeOutliers(self):
        """System::removeOutliers: every point without residuals; returns the removed handles."""
        out = np.zeros(max(self.n_points + 1, 1) * 2 + 4096, np.int32)
        n = C.c_int()
        check(self.lib.hs_ba_remove_points_without_residuals(self.h, ptr(out), C.byref(n)))
        return out[: n.value].copy()

    def removeFrame(self, frame, marginalize=True):
        """System::marginalizeFrame (marginalize=True) of window frame `frame` (it must host no point)."""
        check(self.lib.hs_ba_remove_frame(self.h, int(frame), int(marginalize)))
        self._n_frames_mirror = getattr(self, "_n_frames_mirror", self.nF) - 1

    def structure(self):
        """The committed window: dict(handles, pt_host, nres, res_target (activeResiduals order))."""
        self._sync()
        o = dict(handles=np.zeros(self.n_points, np.int32), pt_host=np.zeros(self.n_points, np.int32),
                 nres=np.zeros(self.n_points, np.int32), res_target=np.zeros(self.n_res, np.int32))
        check(self.lib.hs_ba_get_structure(self.h, *[ptr(o[k]) for k in ("handles", "pt_host", "nres", "res_target")]))
        o["res_point"] = np.repeat(np.arange(self.n_points, dtype=np.int32), o["nres"])
        return o

    def frame_eval(self):
        """dict(evalPT [nF][7], state_zero [nF][10]): each frame's linearization point."""
        self._sync()
        ev, sz = np.zeros((self.nF, 7)), np.zeros((self.nF, 10))
        check(self.lib.hs_ba_get_frame_eval(self.h, ptr(ev), ptr(sz)))
        return dict(evalPT=ev, state_zero=sz)

    def marginal_prior(self):
        self._sync()
        HM, bM = np.zeros((self.dim, self.dim)), np.zeros(self.dim)
        check(self.lib.hs_ba_get_marginal_prior(self.h, ptr(HM), ptr(bM)))
        return HM, bM

    def point_state(self):
        """dict(idepth, idepth_zero, maxRelBaseline, numGoodResiduals, HdiF (the last solve's)) in window order."""
        self._sync()
        n = self.n_points
        o = dict(idepth=np.zeros(n, np.float32), idepth_zero=np.zeros(n, np.float32),
                 maxRelBaseline=np.zeros(n, np.float32), numGoodResiduals=np.zeros(n, np.int32),
                 HdiF=np.zeros(n, np.float32))
        check(self.lib.hs_ba_get_point_state(self.h, *[ptr(o[k]) for k in ("idepth", "idepth_zero", "maxRelBaseline",
                                                                             "numGoodResiduals", "HdiF")]))
        return o

    def synchronize(self):
        check(self.lib.hs_ba_synchronize(self.h))

    def system_vector(self, raw=False):
        """The packed system vector of the last linearization as the solve consumes it (test hook): n*n | n | energy,
        sum |idepth|, #points.  raw: as the stitch wrote it, the diagonal blocks' host-f Schur terms [nF][64] unfolded
        at the end (what a multi-rank exchange all-gathers)."""
        n = self.dim
        out = np.zeros(n * n + n + 3 + (64 * self.nF if raw else 0))
        self.lib.hs_debug_get_sysvec.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
        check(self.lib.hs_debug_get_sysvec(self.h, ptr(out), int(raw)))
        return out

    def candidates(self):
        """This rank's newest-frame candidates of the last linearization (NaN = none; test hook)."""
        st = C.c_int()
        self.lib.hs_debug_get_candidates.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        check(self.lib.hs_debug_get_candidates(self.h, None, C.byref(st)))
        out = np.zeros(st.value, np.float32)
        check(self.lib.hs_debug_get_candidates(self.h, ptr(out), C.byref(st)))
        return out

    def debug_state(self) -> bytes:
        buf = C.create_string_buffer(self.lib.hs_debug_state_size())
        check(self.lib.hs_debug_get_state(self.h, buf))
        return buf.raw

    def debug_nullspace_error(self) -> float:
        """max |device nullspaces - setStateZero(evalPT)| over the window's frames (0: no stale device copy)."""
        e = C.c_double(0)
        check(self.lib.hs_debug_nullspace_error(self.h, C.byref(e)))
        return e.value

    def debug_set_state(self, blob: bytes):
        buf = C.create_string_buffer(blob, len(blob))
        check(self.lib.hs_debug_set_state(self.h, buf))

    def close(self):
        if getattr(self, "h", None):
            self.lib.hs_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    @staticmethod
    def rank_group(shards, device: int = 0, params=None):
        """Test hook: the shards as the ranks of one in-process group on `device` (hs_ba_debug_group): the
        library's multi-rank path (one exchange of system vectors + candidates per linearization, rank-order sums,
        the select beside the solve) with device copies in place of the RCCL all-gather.  Returns RankGroup."""
        ws = []
        for _ in shards:
            w = BAWindow.__new__(BAWindow)
            w.lib = load()
            w.params = params if params is not None else default_params()
            h = C.c_void_p()
            check(w.lib.hs_create(C.byref(h), C.byref(w.params), device))
            w.h = h
            ws.append(w)
        stride = max(s.n_points for s in shards)
        arr = (C.c_void_p * len(ws))(*[w.h.value for w in ws])
        check(ws[0].lib.hs_ba_debug_group(C.cast(arr, C.c_void_p), len(ws), int(stride)))
        for w, s in zip(ws, shards):
            w.nF = s.n_frames
            w.dim = 4 + 8 * w.nF
            w._set_window(s, None)
        return RankGroup(ws)

    # --------------------------------------------------------------- reference call surface
    def linearizeAll(self, reset=False):
        e = C.c_double()
        check(self.lib.hs_ba_linearize(self.h, int(reset), C.byref(e)))
        return e.value

    def set_marginal_prior(self, HM, bM):
        """EnergyFunctional::HM / bM (Include/EnergyFunctional.h:62-63), dim x dim and dim."""
        check(self.lib.hs_ba_set_marginal_prior(self.h, ptr(np.ascontiguousarray(HM, np.float64)),
                                                ptr(np.ascontiguousarray(bM, np.float64))))

    def marginalizePointsF(self, points, return_prior=True):
        """flagPointsForRemoval (per-point part) + EnergyFunctional::marginalizePointsF for window points
        `points` (Src/Mapping.cpp:280-293, Src/EnergyFunctional.cpp:545-609).  Returns the updated (HM, bM)
        (return_prior=False: nothing is read back and the call does not wait for the device); the window's
        linearization is consumed (drop the points and relinearize)."""
        self._sync()
        p = np.ascontiguousarray(points, np.int32)
        HM, bM = (np.zeros((self.dim, self.dim)), np.zeros(self.dim)) if return_prior else (None, None)
        check(self.lib.hs_ba_marginalize_points(self.h, len(p), ptr(p), ptr(HM), ptr(bM)))
        return HM, bM

    def marginalizeFrame(self, frame):
        """EnergyFunctional::marginalizeFrame (Src/EnergyFunctional.cpp:456-543) on this window's HM / bM:
        returns the (dim-8) prior of the window without `frame`."""
        self._sync()
        n = self.dim - 8
        HM, bM = np.zeros((n, n)), np.zeros(n)
        check(self.lib.hs_ba_marginalize_frame(self.h, int(frame), ptr(HM), ptr(bM)))
        return HM, bM

    def solveSystem(self, iteration):
        x = np.zeros(self.dim)
        check(self.lib.hs_ba_solve_system(self.h, iteration, ptr(x)))
        return x

    def doStepFromBackup(self):
        cb = C.c_int()
        check(self.lib.hs_ba_do_step(self.h, C.byref(cb)))
        return bool(cb.value)

    def optimize(self, iters=6, allow_break=False):
        self._sync()
        # System::optimize's overrides for tiny windows (Src/FullSystemOptimize.cpp:366-367), applied here so the
        # energy buffer (max_iters + 1 entries, include/hs_ba.h) holds the whole trajectory
        if self.nF < 3:
            iters = 20
        if self.nF < 4:
            iters = 15
        e = np.zeros(iters + 1)
        n = C.c_int()
        check(self.lib.hs_ba_optimize(self.h, iters, int(allow_break), ptr(e), C.byref(n)))
        return n.value, e[: n.value + 1]

    def iterate(self, first_iteration, n_iters):
        e = np.zeros(n_iters)
        check(self.lib.hs_ba_iterate(self.h, first_iteration, n_iters, ptr(e)))
        return e

    def fixLinearization(self, max_rel_baseline=None, num_good=None, point_state=True):
        """System::optimize's tail (Src/FullSystemOptimize.cpp:498-516): newest frame setEvalPT, setAdjointsF,
        setPrecalcValues, linearizeAll(true).  Returns dict(energy, drop[n_res], maxRelBaseline[n_points],
        numGoodResiduals[n_points], HdiF[n_points]) (HdiF of the last solve's Schur prelude).  Without arrays the
        context's own per-point values are used and returned (point_state=False: not read back, None)."""
        self._sync()
        if max_rel_baseline is None and num_good is None:
            drop = np.zeros(self.n_res, np.uint8)
            hdi = np.zeros(self.n_points, np.float32)
            e = C.c_double()
            check(self.lib.hs_ba_fix_linearization(self.h, C.byref(e), ptr(drop), None, None, ptr(hdi)))
            ps = self.point_state() if point_state else {"maxRelBaseline": None, "numGoodResiduals": None}
            return dict(energy=e.value, drop=drop, maxRelBaseline=ps["maxRelBaseline"],
                        numGoodResiduals=ps["numGoodResiduals"], HdiF=hdi)
        rb = np.zeros(self.n_points, np.float32) if max_rel_baseline is None else \
            np.array(max_rel_baseline, np.float32)
        ng = np.zeros(self.n_points, np.int32) if num_good is None else np.array(num_good, np.int32)
        drop = np.zeros(self.n_res, np.uint8)
        hdi = np.zeros(self.n_points, np.float32)
        e = C.c_double()
        check(self.lib.hs_ba_fix_linearization(self.h, C.byref(e), ptr(drop), ptr(rb), ptr(ng), ptr(hdi)))
        return dict(energy=e.value, drop=drop, maxRelBaseline=rb, numGoodResiduals=ng, HdiF=hdi)

    def calcEnergies(self):
        """EnergyFunctional::calcLEnergyF_MT / calcMEnergyF (dormant under setting_forceAceptStep): (L, M)."""
        el, em = C.c_double(), C.c_double()
        check(self.lib.hs_ba_calc_energies(self.h, C.byref(el), C.byref(em)))
        return el.value, em.value

    # --------------------------------------------------------------- read-back
    def system(self, which):
        self._sync()
        H = np.zeros((self.dim, self.dim))
        b = np.zeros(self.dim)
        check(self.lib.hs_ba_get_system(self.h, which, ptr(H), ptr(b)))
        return H, b

    def residuals(self):
        self._sync()
        m = self.n_res
        out = dict(state=np.zeros(m, np.uint8), active=np.zeros(m, np.uint8), energy=np.zeros(m, np.float32),
                   energy_wo=np.zeros(m, np.float32), JpJdF=np.zeros((m, 8), np.float32),
                   center=np.zeros((m, 3), np.float32))
        check(self.lib.hs_ba_get_residuals(self.h, *[ptr(out[k]) for k in ("state", "active", "energy", "energy_wo",
                                                                           "JpJdF", "center")]))
        return out

    def points(self):
        self._sync()
        n = self.n_points
        out = {k: np.zeros(n, np.float32) for k in ("idepth", "step", "HdiF", "bdSumF")}
        check(self.lib.hs_ba_get_points(self.h, *[ptr(out[k]) for k in ("idepth", "step", "HdiF", "bdSumF")]))
        return out

    def frames(self):
        self._sync()
        st = np.zeros((self.nF, 10))
        th = np.zeros(self.nF, np.float32)
        pose = np.zeros((self.nF, 7))
        cal = np.zeros(4)
        check(self.lib.hs_ba_get_frames(self.h, ptr(st), ptr(th), ptr(pose), ptr(cal)))
        return dict(state=st, energyTH=th, pose=pose, calib=cal)

    def timings(self):
        t = np.zeros(6)
        check(self.lib.hs_ba_get_timings(self.h, ptr(t)))
        return dict(linearize_ms=t[0], acc_stitch_ms=t[1], solve_ms=t[2], timed_iters=int(t[3]), wall_ms=t[4],
                    iters=int(t[5]))

    def set_event_timing(self, mode: int):
        """HIP event pairs in later GN loops: 0 none, 1 the linearize kernel, 2 every phase (measurement only)."""
        check(self.lib.hs_ba_set_event_timing(self.h, int(mode)))

    def partition(self):
        """The linearize partitioning: dict(kernel='hs_k_lin' | 'hs_k_lin8', blocks, waves, exact)."""
        o = np.zeros(4, np.int32)
        check(self.lib.hs_ba_get_partition(self.h, ptr(o)))
        return dict(kernel="hs_k_lin8" if o[0] else "hs_k_lin", blocks=int(o[1]), waves=int(o[2]), exact=bool(o[3]))

    def time_linearize(self, reps: int) -> float:
        """Average ms of `reps` back-to-back linearize launches (one HIP event pair)."""
        t = np.zeros(1)
        check(self.lib.hs_ba_time_linearize(self.h, int(reps), ptr(t)))
        return float(t[0])

    # --------------------------------------------------------------- multi-GPU
    @staticmethod
    def comm_unique_id() -> bytes:
        buf = C.create_string_buffer(128)
        check(load().hs_comm_get_unique_id(buf))
        return buf.raw

    def comm_init(self, uid: bytes, rank: int, nranks: int):
        buf = C.create_string_buffer(uid, 128)
        check(self.lib.hs_comm_init(self.h, buf, rank, nranks))

    def comm_size(self):
        """(ranks the communicator holds, this context's rank) — from RCCL itself (ncclCommCount); (1, 0) without one."""
        n, r = C.c_int(), C.c_int()
        check(self.lib.hs_comm_size(self.h, C.byref(n), C.byref(r)))
        return n.value, r.value


class RankGroup:
    """The members of BAWindow.rank_group, driven together (hs_ba_group_linearize / hs_ba_group_iterate)."""

    def __init__(self, members):
        self.members = members
        self._arr = (C.c_void_p * len(members))(*[w.h.value for w in members])

    def linearizeAll(self, reset=False):
        e = C.c_double()
        check(self.members[0].lib.hs_ba_group_linearize(C.cast(self._arr, C.c_void_p), len(self.members), int(reset),
                                                        C.byref(e)))
        return e.value

    def iterate(self, first_iteration, n_iters):
        e = np.zeros(n_iters)
        check(self.members[0].lib.hs_ba_group_iterate(C.cast(self._arr, C.c_void_p), len(self.members),
                                                      first_iteration, n_iters, ptr(e)))
        return e

    def close(self):
        for w in self.members:
            w.close()
