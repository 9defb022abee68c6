"""Frame::CreateDirPyrs (Src/Frame.cpp:104-181) on the device through include/hs_pyr.h."""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import check, load, ptr


def dir_pyramid(img, n_levels: int, device: int = 0):
    """([(h_l, w_l, 3) float32 DirPyr levels], [(h_l, w_l) absSquaredGrad]) of a H x W fp32 image."""
    img = np.ascontiguousarray(img, np.float32)
    H, W = img.shape
    sizes = [(H >> l, W >> l) for l in range(n_levels)]
    out = np.zeros(sum(h * w * 3 for h, w in sizes), np.float32)
    ag = np.zeros(sum(h * w for h, w in sizes), np.float32)
    check(load().hs_dir_pyramid(device, W, H, n_levels, ptr(img), ptr(out), ptr(ag)))
    pyr, grads, o3, o1 = [], [], 0, 0
    for h, w in sizes:
        pyr.append(out[o3:o3 + h * w * 3].reshape(h, w, 3))
        grads.append(ag[o1:o1 + h * w].reshape(h, w))
        o3 += h * w * 3
        o1 += h * w
    return pyr, grads
