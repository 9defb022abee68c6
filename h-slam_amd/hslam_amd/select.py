"""PixelSelector (Src/PixelSelector.cpp:14-418) on the device through include/hs_select.h.

The mirror keeps the reference's interface: ``PixelSelector(width, height)`` (the constructor's randomPattern and
currentPotential = 3), ``makeMaps(DirPyr, id, GradPyr, density, recursionsLeft=1, thFactor=1)`` returning the
selection map (0 / 1 / 2 / 4 per pixel, FeatureDetector's ``selectionMap``) and numHaveSub, and
``currentPotential`` as a read/write attribute.  ``makeMapsRaw`` takes the undistorted level-0 image instead and
builds the pyramid on the device (Frame::CreateDirPyrs, include/hs_pyr.h).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import check, default_params, load, ptr


class PixelSelector:
    def __init__(self, width: int, height: int, params=None, device: int = 0):
        self.lib = load()
        self.W, self.H = int(width), int(height)
        self.params = params if params is not None else default_params()
        self.h = C.c_void_p()
        check(self.lib.hs_selector_create(C.byref(self.h), C.byref(self.params), device, self.W, self.H))

    def __del__(self):
        if getattr(self, "h", None) and self.h.value:
            self.lib.hs_selector_destroy(self.h)
            self.h = C.c_void_p()

    def makeMaps(self, DirPyr, id: int, GradPyr, density: float, recursionsLeft: int = 1, thFactor: float = 1.0):
        """DirPyr: level 0 (H, W, 3) or the list of levels; GradPyr: absSquaredGrad levels (0..2 are read)."""
        d0 = DirPyr[0] if isinstance(DirPyr, (list, tuple)) else DirPyr
        d0 = np.ascontiguousarray(d0, np.float32)
        if d0.shape != (self.H, self.W, 3):
            raise ValueError(f"DirPyr[0] must be ({self.H}, {self.W}, 3), got {d0.shape}")
        g = [np.ascontiguousarray(x, np.float32) for x in GradPyr[:3]]
        for l, x in enumerate(g):
            if x.shape != (self.H >> l, self.W >> l):
                raise ValueError(f"GradPyr[{l}] must be ({self.H >> l}, {self.W >> l}), got {x.shape}")
        out = np.empty((self.H, self.W), np.float32)
        n = C.c_int()
        check(self.lib.hs_selector_make_maps(self.h, int(id), ptr(d0), ptr(g[0]), ptr(g[1]), ptr(g[2]),
                                             float(density), int(recursionsLeft), float(thFactor), ptr(out),
                                             C.byref(n)))
        return out, n.value

    def makeMapsRaw(self, img, id: int, density: float, recursionsLeft: int = 1, thFactor: float = 1.0,
                    want_map: bool = True):
        img = np.ascontiguousarray(img, np.float32)
        if img.shape != (self.H, self.W):
            raise ValueError(f"image must be ({self.H}, {self.W}), got {img.shape}")
        out = np.empty((self.H, self.W), np.float32) if want_map else None
        n = C.c_int()
        check(self.lib.hs_selector_make_maps_raw(self.h, int(id), ptr(img), float(density), int(recursionsLeft),
                                                 float(thFactor), ptr(out) if want_map else None, C.byref(n)))
        return out, n.value

    @property
    def currentPotential(self) -> int:
        p = C.c_int()
        check(self.lib.hs_selector_get_potential(self.h, C.byref(p)))
        return p.value

    @currentPotential.setter
    def currentPotential(self, p: int):
        check(self.lib.hs_selector_set_potential(self.h, int(p)))

    def last_stats(self):
        """(device ms of the last makeMaps incl. its host decisions, select passes run)."""
        ms, passes = C.c_double(), C.c_int()
        check(self.lib.hs_selector_last_stats(self.h, C.byref(ms), C.byref(passes)))
        return ms.value, passes.value
