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

    def set_state(self, idepth_min=None, idepth_max=None, quality=None, status=None):
        arr = [None if a is None else np.ascontiguousarray(a, dt)
               for a, dt in ((idepth_min, np.float32), (idepth_max, np.float32), (quality, np.float32),
                             (status, np.uint8))]
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

    def reinit(self):
        """ImmaturePoint ctor again on every stored point (a fresh first-trace state), on the device."""
        check(self.lib.hs_tracer_reinit(self.h))

    def last_stats(self):
        """(device ms of the last traceOn kernel, discrete-search steps it evaluated)"""
        ms, st = C.c_double(), C.c_longlong()
        check(self.lib.hs_tracer_last_stats(self.h, C.byref(ms), C.byref(st)))
        return ms.value, st.value
