"""Host-side mirror of the reference's CoarseTracker call surface over the C-ABI (include/hs_track.h).

Method names follow Include/CoarseTracker.h:21-29 and Src/System.cpp:333-524 so a parity test reads
like the reference's own control flow:

    ct = CoarseTracker(w, h, K4, n_levels)         # CoarseTracker(w, h) + makeK
    ct.setCoarseTrackingRef(ref_pyr, ...)          # setCoarseTrackingRef -> makeCoarseDepthL0
    ct.setNewFrame(new_pyr, ab_exposure)           # fh->DirPyr
    ok, T, aff = ct.trackNewestCoarse(T, aff, lvl, minResForAbort)
    out = trackNewCoarse(ct, tries, aff_last_2_l, lastCoarseRMSE)   # System::trackNewCoarse try loop

All compute runs in libhslam_amd.so on the GPU; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import check, default_params, load, ptr
from .se3 import SE3


def _pyr_ptrs(pyr):
    arrs = [np.ascontiguousarray(p, dtype=np.float32) for p in pyr]
    return arrs, (C.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])


class CoarseTracker:
    def __init__(self, width: int, height: int, K4, n_levels: int, params=None, device: int = 0):
        self.lib = load()
        self.params = params if params is not None else default_params()
        self.width, self.height, self.n_levels = width, height, n_levels
        self.wl = [width >> l for l in range(n_levels)]
        self.hl = [height >> l for l in range(n_levels)]
        k4 = np.ascontiguousarray(K4, dtype=np.float32)
        h = C.c_void_p()
        check(self.lib.hs_tracker_create(C.byref(h), C.byref(self.params), device, width, height, n_levels, ptr(k4)))
        self.h = h
        self.lastResiduals = np.full(5, np.nan)
        self.lastFlowIndicators = np.full(3, 1000.0)

    def close(self):
        if getattr(self, "h", None):
            self.lib.hs_tracker_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    # Src/CoarseTracker.cpp:492-504
    def setCoarseTrackingRef(self, ref_pyr, ab_exposure, aff_g2l, u, v, idepth, hdi):
        arrs, pp = _pyr_ptrs(ref_pyr)
        aff = np.ascontiguousarray(aff_g2l, dtype=np.float64)
        cols = [np.ascontiguousarray(a, dtype=np.float32) for a in (u, v, idepth, hdi)]
        check(self.lib.hs_tracker_set_ref(self.h, C.cast(pp, C.c_void_p), float(ab_exposure), ptr(aff),
                                          len(cols[0]), *[ptr(c) for c in cols]))

    def setNewFrame(self, new_pyr, ab_exposure):
        arrs, pp = _pyr_ptrs(new_pyr)
        check(self.lib.hs_tracker_set_frame(self.h, C.cast(pp, C.c_void_p), float(ab_exposure)))

    def setNewFrameRaw(self, img, ab_exposure):
        """The frame to track as its raw level-0 image: Frame::CreateDirPyrs runs on the device."""
        a = np.ascontiguousarray(img, dtype=np.float32)
        assert a.shape == (self.height, self.width)
        check(self.lib.hs_tracker_set_frame_raw(self.h, ptr(a), float(ab_exposure)))

    def setCoarseTrackingRefBA(self, ba, promote: bool, ab_exposure=1.0, aff_g2l=(0.0, 0.0)):
        """setCoarseTrackingRef from a BA context (hslam_amd.ba.BAWindow) on the device: the points with an IN
        residual into its newest frame, no host round trip.  promote: the frame last set here becomes the reference
        pyramid (else it is rebuilt from the BA's newest frame image)."""
        aff = np.ascontiguousarray(aff_g2l, dtype=np.float64)
        check(self.lib.hs_tracker_set_ref_ba(self.h, ba.h, int(promote), float(ab_exposure), ptr(aff)))

    set_ref_ba = setCoarseTrackingRefBA

    def frame_texels(self, lvl: int = 0) -> int:
        """Device address of level lvl of the frame last set (float4 texels): hs_ba_set_frame_image_device."""
        p = C.c_void_p()
        check(self.lib.hs_tracker_frame_texels(self.h, int(lvl), C.byref(p)))
        return p.value

    def frame_to_ba(self, ba, frame: int):
        """The frame last set becomes window frame `frame`'s image in ba (hslam_amd.ba.BAWindow), device to
        device, ordered on the device both ways (hs_tracker_frame_to_ba)."""
        check(self.lib.hs_tracker_frame_to_ba(self.h, ba.h, int(frame)))

    def set_frame_raw(self, img, ab_exposure=1.0):
        self.setNewFrameRaw(img, ab_exposure)

    def set_scene(self, s):
        """Reference + new frame of a hslam_amd.scene.TrackScene."""
        self.setCoarseTrackingRef(s.ref_pyr, s.ref_exposure, s.ref_aff, s.pt_u, s.pt_v, s.pt_idepth, s.pt_hdi)
        self.setNewFrame(s.new_pyr, s.new_exposure)

    def pc(self, lvl: int):
        """pc_u / pc_v / pc_idepth / pc_color of one level (Include/CoarseTracker.h:73-77)."""
        cap = self.wl[lvl] * self.hl[lvl]
        out = {k: np.zeros(cap, np.float32) for k in ("u", "v", "idepth", "color")}
        n = C.c_int()
        check(self.lib.hs_tracker_get_ref(self.h, lvl, C.byref(n), *[ptr(out[k]) for k in ("u", "v", "idepth",
                                                                                           "color")]))
        return {k: a[: n.value] for k, a in out.items()}

    # Src/CoarseTracker.cpp:329-485 (+ calcGSSSE 267-324 on its warped buffer)
    def calcRes(self, lvl, T7, aff, cutoffTH):
        T = np.ascontiguousarray(T7, dtype=np.float64)
        a = np.ascontiguousarray(aff, dtype=np.float64)
        res6, H, b = np.zeros(6), np.zeros(64), np.zeros(8)
        nw = C.c_int()
        check(self.lib.hs_tracker_calc_res(self.h, lvl, ptr(T), ptr(a), float(cutoffTH), ptr(res6), ptr(H), ptr(b),
                                           C.byref(nw)))
        return res6, H.reshape(8, 8), b, nw.value

    # Src/CoarseTracker.cpp:506-683
    def trackNewestCoarse(self, T7, aff, coarsestLvl, minResForAbort):
        # one staging block per tracker (T 7 | aff 2 | minRes 5 | lastResiduals 5 | flow 3 | ok), its addresses taken
        # once: the per-call cost is the copies, not ctypes pointer objects
        if getattr(self, "_stage", None) is None:
            self._stage = np.zeros(23)
            base = self._stage.ctypes.data
            self._stage_ptrs = tuple(base + 8 * o for o in (0, 7, 9, 14, 19, 22))
        st = self._stage
        st[0:7] = T7
        st[7:9] = aff
        st[9:14] = minResForAbort
        st[22] = 0.0
        pT, pa, pmr, plr, pfl, pok = self._stage_ptrs
        check(self.lib.hs_tracker_track(self.h, pT, pa, coarsestLvl, pmr, plr, pfl, pok))
        self.lastResiduals, self.lastFlowIndicators = st[14:19].copy(), st[19:22].copy()
        return bool(st[22:23].view(np.int32)[0]), st[0:7].copy(), st[7:9].copy()

    def track_tries(self, tries, aff_last_2_l, lastCoarseRMSE, reTrackThreshold=None):
        tr = np.ascontiguousarray(np.asarray(tries, dtype=np.float64).reshape(-1, 7))
        al = np.ascontiguousarray(aff_last_2_l, dtype=np.float64)
        lc = np.ascontiguousarray(lastCoarseRMSE, dtype=np.float64)
        th = 1.5 if reTrackThreshold is None else reTrackThreshold  # setting_reTrackThreshold (Src/Settings.cpp)
        T, a, ach, fl = np.zeros(7), np.zeros(2), np.zeros(5), np.zeros(3)
        good, n = C.c_int(), C.c_int()
        check(self.lib.hs_tracker_track_tries(self.h, len(tr), ptr(tr), ptr(al), ptr(lc), float(th), ptr(T), ptr(a),
                                              ptr(ach), ptr(fl), C.byref(good), C.byref(n)))
        return dict(T=T, aff=a, achievedRes=ach, flowVecs=fl, haveOneGood=bool(good.value), tryIterations=n.value)

    def lm_log(self, try_idx: int = 0, cap: int = 256):
        """Per-iteration LM test operands (level, resNew/N, resOld/N, |inc|) of one hypothesis of the last call."""
        lvl, nr, orr, inc = np.zeros(cap, np.int32), np.zeros(cap), np.zeros(cap), np.zeros(cap)
        n = C.c_int()
        check(self.lib.hs_tracker_get_lm_log(self.h, try_idx, cap, C.byref(n), ptr(lvl), ptr(nr), ptr(orr),
                                             ptr(inc)))
        m = min(n.value, cap)
        return lvl[:m], nr[:m], orr[:m], inc[:m]

    def launch_info(self):
        """(G workgroups per hypothesis of the last launch, launches rerun with G = 1 after a meeting timeout)."""
        g, f = C.c_int(), C.c_int()
        check(self.lib.hs_tracker_launch_info(self.h, C.byref(g), C.byref(f)))
        return g.value, f.value

    def last_stats(self, try_idx: int = 0):
        """(device ms, passes, point-passes) of one hypothesis of the last call."""
        ms, ps, pp = C.c_double(), C.c_int(), C.c_longlong()
        check(self.lib.hs_tracker_last_stats(self.h, try_idx, C.byref(ms), C.byref(ps), C.byref(pp)))
        return ms.value, ps.value, pp.value

    def set_event_timing(self, on: bool = True):
        """hs_tracker_set_event_timing: the per-call event pair (off by default) that last_ms / last_stats report."""
        check(self.lib.hs_tracker_set_event_timing(self.h, int(bool(on))))

    def last_ms(self):
        ms = C.c_double()
        check(self.lib.hs_tracker_last_ms(self.h, C.byref(ms)))
        return ms.value


def motion_hypotheses(lastF_c2w: SE3, slast_c2w: SE3, sprelast_c2w: SE3, poses_valid: bool = True):
    """lastF_2_fh_tries of System::trackNewCoarse (Src/System.cpp:346-411): 5 motion models then the 26
    rotation jitters with rotDelta = 0.02 (the float loop runs once).  Returns [n, 7] SE3 data."""
    if not poses_valid:
        return np.array([SE3().data()])
    slast_2_sprelast = sprelast_c2w.inverse() * slast_c2w
    lastF_2_slast = slast_c2w.inverse() * lastF_c2w
    fh_2_slast = slast_2_sprelast
    inv = fh_2_slast.inverse()
    tries = [inv * lastF_2_slast, inv * inv * lastF_2_slast, SE3.exp(fh_2_slast.log() * 0.5).inverse() * lastF_2_slast,
             lastF_2_slast, SE3()]
    d = np.float32(0.02)
    d = float(d)  # float rotDelta promoted to double in the Quaterniond constructor
    jit = [(d, 0, 0), (0, d, 0), (0, 0, d), (-d, 0, 0), (0, -d, 0), (0, 0, -d),
           (d, d, 0), (0, d, d), (d, 0, d), (-d, d, 0), (0, -d, d), (-d, 0, d),
           (d, -d, 0), (0, d, -d), (d, 0, -d), (-d, -d, 0), (0, -d, -d), (-d, 0, -d),
           (-d, -d, -d), (-d, -d, d), (-d, d, -d), (-d, d, d), (d, -d, -d), (d, -d, d), (d, d, -d), (d, d, d)]
    base = inv * lastF_2_slast
    for x, y, z in jit:
        tries.append(base * SE3.from_quat_wxyz(1.0, x, y, z))
    return np.array([t.data() for t in tries])


def trackNewCoarse(tracker: CoarseTracker, tries, aff_last_2_l, lastCoarseRMSE, reTrackThreshold=None):
    """System::trackNewCoarse's try loop (Src/System.cpp:413-499) on the device tracker: returns the dict of
    CoarseTracker.track_tries plus camToTrackingRef = lastF_2_fh.inverse()."""
    out = tracker.track_tries(tries, aff_last_2_l, lastCoarseRMSE, reTrackThreshold)
    out["camToTrackingRef"] = SE3.from_data(out["T"]).inverse().data()
    return out
