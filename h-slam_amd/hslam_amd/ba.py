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


class BAWindow:
    def __init__(self, scene, device: int = 0, params=None, point_slice=None, comm=None):
        """scene: hslam_amd.scene.BAScene (or any object with the same fields).
        point_slice: optional (begin, end) to load only a contiguous shard of the points.
        comm: optional (unique_id_bytes, rank, nranks) -> RCCL communicator (before the window is set)."""
        self.lib = load()
        self.params = params if params is not None else default_params()
        h = C.c_void_p()
        check(self.lib.hs_create(C.byref(h), C.byref(self.params), device))
        self.h = h
        if comm is not None:
            self.comm_init(*comm)
        self.nF = scene.n_frames
        self.dim = 4 + 8 * self.nF
        self._set_window(scene, point_slice)

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

    def close(self):
        if getattr(self, "h", None):
            self.lib.hs_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    # --------------------------------------------------------------- reference call surface
    def linearizeAll(self, reset=False):
        e = C.c_double()
        check(self.lib.hs_ba_linearize(self.h, int(reset), C.byref(e)))
        return e.value

    def set_marginal_prior(self, HM, bM):
        """EnergyFunctional::HM / bM (Include/EnergyFunctional.h:62-63), dim x dim and dim."""
        check(self.lib.hs_ba_set_marginal_prior(self.h, ptr(np.ascontiguousarray(HM, np.float64)),
                                                ptr(np.ascontiguousarray(bM, np.float64))))

    def marginalizePointsF(self, points):
        """flagPointsForRemoval (per-point part) + EnergyFunctional::marginalizePointsF for window points
        `points` (Src/Mapping.cpp:280-293, Src/EnergyFunctional.cpp:545-609).  Returns the updated (HM, bM);
        the window's linearization is consumed (drop the points and relinearize)."""
        p = np.ascontiguousarray(points, np.int32)
        HM, bM = np.zeros((self.dim, self.dim)), np.zeros(self.dim)
        check(self.lib.hs_ba_marginalize_points(self.h, len(p), ptr(p), ptr(HM), ptr(bM)))
        return HM, bM

    def marginalizeFrame(self, frame):
        """EnergyFunctional::marginalizeFrame (Src/EnergyFunctional.cpp:456-543) on this window's HM / bM:
        returns the (dim-8) prior of the window without `frame`."""
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

    def fixLinearization(self, max_rel_baseline=None, num_good=None):
        """System::optimize's tail (Src/FullSystemOptimize.cpp:498-516): newest frame setEvalPT, setAdjointsF,
        setPrecalcValues, linearizeAll(true).  Returns dict(energy, drop[n_res], maxRelBaseline[n_points],
        numGoodResiduals[n_points], HdiF[n_points]) (HdiF of the last solve's Schur prelude)."""
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
        H = np.zeros((self.dim, self.dim))
        b = np.zeros(self.dim)
        check(self.lib.hs_ba_get_system(self.h, which, ptr(H), ptr(b)))
        return H, b

    def residuals(self):
        m = self.n_res
        out = dict(state=np.zeros(m, np.uint8), active=np.zeros(m, np.uint8), energy=np.zeros(m, np.float32),
                   energy_wo=np.zeros(m, np.float32), JpJdF=np.zeros((m, 8), np.float32),
                   center=np.zeros((m, 3), np.float32))
        check(self.lib.hs_ba_get_residuals(self.h, *[ptr(out[k]) for k in ("state", "active", "energy", "energy_wo",
                                                                           "JpJdF", "center")]))
        return out

    def points(self):
        n = self.n_points
        out = {k: np.zeros(n, np.float32) for k in ("idepth", "step", "HdiF", "bdSumF")}
        check(self.lib.hs_ba_get_points(self.h, *[ptr(out[k]) for k in ("idepth", "step", "HdiF", "bdSumF")]))
        return out

    def frames(self):
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
