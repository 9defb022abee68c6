"""Host-side mirror of the reference's immature-point tracing over the C-ABI (include/hs_trace.h).

Names follow the reference (Include/ImmaturePoint.h:34-71, Src/Mapping.cpp:494-538):

    tr = ImmatureTracer(W, H, capacity)
    tr.set_host_image(slot, DirPyr0)        # a host keyframe
    tr.add_points(host, u, v)               # new ImmaturePoint(u, v, host, ...) for each point
    tr.set_frame(new_DirPyr0)
    counts = tr.traceNewCoarse(KRKi, Kt, aff)   # traceOn of every point, per-host (KRKi, Kt, aff)
    pts = tr.points()                       # lastTraceStatus, idepth_min/max, quality, lastTraceUV, ...
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import check, default_params, load, ptr

FIELDS = ("status", "idepth_min", "idepth_max", "quality", "uv", "interval", "energyTH", "color", "weights", "gradH")
IPS = ("GOOD", "OOB", "OUTLIER", "SKIPPED", "BADCONDITION", "UNINITIALIZED")


ACT = ("KEEP", "DELETED", "ACTIVATED")
# hs_act_frame / hs_act_pair (include/hs_trace.h) as numpy records
ACT_FRAME_DT = np.dtype([("slot", np.int32), ("flagged_for_marg", np.int32), ("KRKi", np.float32, 9),
                         ("Kt", np.float32, 3)])
ACT_PAIR_DT = np.dtype([("RTll", np.float32, 9), ("tTll", np.float32, 3), ("aff", np.float32, 2)])


def act_frames_array(slot, flagged, KRKi, Kt):
    """[nF] hs_act_frame records: tracer slot, FlaggedForMarginalization, level-1 KRKi / Kt to the newest KF."""
    out = np.zeros(len(slot), ACT_FRAME_DT)
    out["slot"] = slot
    out["flagged_for_marg"] = flagged
    out["KRKi"] = np.asarray(KRKi, np.float32).reshape(-1, 9)
    out["Kt"] = np.asarray(Kt, np.float32).reshape(-1, 3)
    return out


def act_pairs_array(RTll, tTll, aff):
    """[nF*nF] hs_act_pair records (FrameFramePrecalc PRE_RTll / PRE_tTll / PRE_aff_mode, host-major)."""
    out = np.zeros(len(RTll), ACT_PAIR_DT)
    out["RTll"] = np.asarray(RTll, np.float32).reshape(-1, 9)
    out["tTll"] = np.asarray(tTll, np.float32).reshape(-1, 3)
    out["aff"] = np.asarray(aff, np.float32).reshape(-1, 2)
    return out


def hosts_array(KRKi, Kt, aff):
    """[nH] hs_trace_host records (KRKi[9], Kt[3], aff[2], float32) as a contiguous [nH, 14] float32 array."""
    return np.ascontiguousarray(np.concatenate([np.asarray(KRKi, np.float32).reshape(-1, 9),
                                                np.asarray(Kt, np.float32).reshape(-1, 3),
                                                np.asarray(aff, np.float32).reshape(-1, 2)], 1))


class ImmatureTracer:
    def __init__(self, width: int, height: int, capacity: int, device: int = 0, params=None):
        self.lib = load()
        self.params = params if params is not None else default_params()
        h = C.c_void_p()
        check(self.lib.hs_tracer_create(C.byref(h), C.byref(self.params), device, width, height, capacity))
        self.h = h
        self.W, self.H = width, height
        self.n = 0

    def close(self):
        if getattr(self, "h", None):
            self.lib.hs_tracer_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def set_host_image(self, slot: int, img):
        a = np.ascontiguousarray(img, np.float32)
        assert a.shape == (self.H, self.W, 3)
        check(self.lib.hs_tracer_set_host_image(self.h, slot, ptr(a)))

    def add_points(self, host, u, v):
        h = np.ascontiguousarray(host, np.int32)
        uu = np.ascontiguousarray(u, np.float32)
        vv = np.ascontiguousarray(v, np.float32)
        check(self.lib.hs_tracer_add_points(self.h, len(h), ptr(h), ptr(uu), ptr(vv)))
        self.n += len(h)

    def set_state(self, idepth_min=None, idepth_max=None, quality=None, status=None, interval=None):
        arr = [None if a is None else np.ascontiguousarray(a, dt)
               for a, dt in ((idepth_min, np.float32), (idepth_max, np.float32), (quality, np.float32),
                             (status, np.uint8), (interval, np.float32))]
        check(self.lib.hs_tracer_set_state(self.h, *[ptr(a) for a in arr]))

    def set_frame(self, img):
        a = np.ascontiguousarray(img, np.float32)
        assert a.shape == (self.H, self.W, 3)
        check(self.lib.hs_tracer_set_frame(self.h, ptr(a)))

    def set_frame_raw(self, img):
        """The frame to trace on as its raw level-0 image: DirPyr[0] is built on the device."""
        a = np.ascontiguousarray(img, np.float32)
        assert a.shape == (self.H, self.W)
        check(self.lib.hs_tracer_set_frame_raw(self.h, ptr(a)))

    def traceNewCoarse(self, KRKi, Kt, aff, counts=True):
        hosts = hosts_array(KRKi, Kt, aff)
        c = np.zeros(6, np.int32)
        check(self.lib.hs_tracer_trace(self.h, len(hosts), ptr(hosts), ptr(c) if counts else None))
        return c if counts else None

    def set_scene(self, s):
        for i, img in enumerate(s.host_imgs):
            self.set_host_image(i, img)
        self.add_points(s.pt_host, s.pt_u, s.pt_v)
        self.set_frame(s.new_img)

    def points(self):
        n = self.n
        out = dict(status=np.zeros(n, np.uint8), idepth_min=np.zeros(n, np.float32),
                   idepth_max=np.zeros(n, np.float32), quality=np.zeros(n, np.float32), uv=np.zeros((n, 2), np.float32),
                   interval=np.zeros(n, np.float32), energyTH=np.zeros(n, np.float32),
                   color=np.zeros((n, 8), np.float32), weights=np.zeros((n, 8), np.float32),
                   gradH=np.zeros((n, 4), np.float32))
        m = C.c_int()
        check(self.lib.hs_tracer_get_points(self.h, C.byref(m), *[ptr(out[k]) for k in FIELDS]))
        return out

    def set_types(self, my_type):
        """ImmaturePoint::my_type of every stored point (PixelSelector's 1 / 2 / 4)."""
        a = np.ascontiguousarray(my_type, np.float32)
        assert len(a) == self.n
        check(self.lib.hs_tracer_set_types(self.h, ptr(a)))

    # Src/Mapping.cpp:330-480 (System::activatePointsMT)
    def activatePointsMT(self, K4, frames, pairs, act_frame, act_u, act_v, act_idepth, ef_nPoints,
                         currentMinActDist, order=None):
        """One activation over the stored points.  frames / pairs: act_frames_array / act_pairs_array records.
        Returns dict(action, idepth, res_in, activated, currentMinActDist)."""
        k4 = np.ascontiguousarray(K4, np.float32)
        fr = np.ascontiguousarray(frames, ACT_FRAME_DT)
        pr = np.ascontiguousarray(pairs, ACT_PAIR_DT)
        af = np.ascontiguousarray(act_frame, np.int32)
        au, av, ai = (np.ascontiguousarray(x, np.float32) for x in (act_u, act_v, act_idepth))
        od = None if order is None else np.ascontiguousarray(order, np.int32)
        n = self.n
        action, idepth, res_in = np.zeros(n, np.uint8), np.zeros(n, np.float32), np.zeros(n, np.uint8)
        activated = np.zeros(max(n, 1), np.int32)
        cmad = C.c_float(currentMinActDist)
        na = C.c_int()
        check(self.lib.hs_tracer_activate(self.h, ptr(k4), len(fr), ptr(fr), ptr(pr), len(af), ptr(af), ptr(au),
                                          ptr(av), ptr(ai), int(ef_nPoints), C.byref(cmad),
                                          0 if od is None else len(od), ptr(od), ptr(action), ptr(idepth),
                                          ptr(res_in), ptr(activated), C.byref(na)))
        return dict(action=action, idepth=idepth, res_in=res_in, activated=activated[: na.value],
                    currentMinActDist=cmad.value)

    def distance_map(self):
        """CoarseDistanceMap::fwdWarpedIDDistFinal after the last activation, (H/2, W/2) float32."""
        out = np.zeros((self.H >> 1) * (self.W >> 1), np.float32)
        check(self.lib.hs_tracer_get_distance_map(self.h, ptr(out)))
        return out.reshape(self.H >> 1, self.W >> 1)

    def compact(self, keep):
        """Drop the points with keep == 0 (survivors keep their order)."""
        k = np.ascontiguousarray(keep, np.uint8)
        assert len(k) == self.n
        check(self.lib.hs_tracer_compact(self.h, ptr(k)))
        self.n = int(k.astype(bool).sum())

    def reinit(self):
        """ImmaturePoint ctor again on every stored point (a fresh first-trace state), on the device."""
        check(self.lib.hs_tracer_reinit(self.h))

    def last_stats(self):
        """(device ms of the last traceOn kernel, discrete-search steps it evaluated)"""
        ms, st = C.c_double(), C.c_longlong()
        check(self.lib.hs_tracer_last_stats(self.h, C.byref(ms), C.byref(st)))
        return ms.value, st.value
