"""Host-side mirror of the initializer's DirectRefinement over the C-ABI (include/hs_refine.h).

Names follow Include/Initializer.h:108-157 / Src/Initializer.cpp:1330-2270:

    dr = DirectRefinement(scene)          # ctor: calib, frames, Pnt set-up from mvKeys / Pts3D / Triangulated
    pose, videpth, good = dr.Refine(pose) # Refine + the ctor's _Pose / _videpth write-back
    H, b, Hsc, bsc, res = dr.calcResAndGS(T, aff)   # resetPoints + one calcResAndGS (parity seam)

The LM loop runs on the GPU in one workgroup (hs_k_refine); there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import check, load, ptr


class DirectRefinement:
    def __init__(self, scene, device: int = 0):
        self.lib = load()
        s = scene
        h = C.c_void_p()
        check(self.lib.hs_refiner_create(C.byref(h), device, s.width, s.height,
                                         ptr(np.ascontiguousarray(s.K4, np.float64))))
        self.h = h
        self.n = s.n_points
        check(self.lib.hs_refiner_set_frames(self.h, ptr(np.ascontiguousarray(s.img1, np.float32)),
                                             ptr(np.ascontiguousarray(s.img2, np.float32)),
                                             float(s.expo1), float(s.expo2)))
        self.set_points(s.u, s.v, s.tri, s.z)

    def set_points(self, u, v, tri, z):
        cols = [np.ascontiguousarray(u, np.float32), np.ascontiguousarray(v, np.float32),
                np.ascontiguousarray(tri, np.uint8), np.ascontiguousarray(z, np.float32)]
        self.n = len(cols[0])
        check(self.lib.hs_refiner_set_points(self.h, self.n, *[ptr(c) for c in cols]))

    def close(self):
        if getattr(self, "h", None):
            self.lib.hs_refiner_destroy(self.h)
            self.h = None

    __del__ = close

    def Refine(self, pose7, videpth=None):
        """Returns (refined pose, videpth with the good + triangulated points updated, isGood, iterations, snapped)."""
        T = np.array(pose7, np.float64)
        vid = np.zeros(self.n, np.float32) if videpth is None else np.array(videpth, np.float32)
        good = np.zeros(self.n, np.uint8)
        it, sn = C.c_int(), C.c_int()
        check(self.lib.hs_refiner_refine(self.h, ptr(T), ptr(vid), ptr(good), C.byref(it), C.byref(sn)))
        return T, vid, good, it.value, bool(sn.value)

    def calcResAndGS(self, T7, aff=(0.0, 0.0)):
        H, Hs = np.zeros(64, np.float32), np.zeros(64, np.float32)
        b, bs, res = np.zeros(8, np.float32), np.zeros(8, np.float32), np.zeros(3, np.float32)
        check(self.lib.hs_refiner_calc_res(self.h, ptr(np.ascontiguousarray(T7, np.float64)),
                                           ptr(np.ascontiguousarray(aff, np.float64)),
                                           ptr(H), ptr(b), ptr(Hs), ptr(bs), ptr(res)))
        return H.reshape(8, 8), b, Hs.reshape(8, 8), bs, res

    def log(self):
        out = np.zeros((1001, 8), np.float32)
        n = self.lib.hs_refiner_get_log(self.h, 1001, ptr(out))
        if n < 0:
            check(n)
        return out[:n]

    def points(self):
        f7 = np.zeros((self.n, 7), np.float32)
        g2 = np.zeros((self.n, 2), np.uint8)
        jb = np.zeros((self.n, 10), np.float32)
        check(self.lib.hs_refiner_get_points(self.h, ptr(f7), ptr(g2), ptr(jb)))
        return dict(idepth=f7[:, 0], idepth_new=f7[:, 1], iR=f7[:, 2], energy_new0=f7[:, 3], energy_new1=f7[:, 4],
                    maxstep=f7[:, 5], lastHessian_new=f7[:, 6], isGood=g2[:, 0], isGood_new=g2[:, 1], jb_new=jb)

    def last_ms(self) -> float:
        t = np.zeros(1)
        check(self.lib.hs_refiner_last_ms(self.h, ptr(t)))
        return float(t[0])
