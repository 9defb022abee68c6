"""setNewFrameEnergyTH's select (Src/FullSystemOptimize.cpp:60-101) on the device: hs_k_reduce's pass-1 histogram
blocks + the select block of the stitch launch (through the test hook hs_debug_threshold), against nth_element
restated in numpy fp32.  Bit-exact, including the fallback when more than TH_CAP candidates share the first
12-bit bin, ties, and windows without a newest-frame residual."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

THN, FAC, CW, OW = 0.7, 2.0, 0.5, 1.0


def ref_threshold(c):
    f32 = np.float32
    v = c[c >= 0]  # r->state_NewEnergyWithOutlier >= 0 (NaN fails)
    if v.size == 0:
        return f32(12 * 12 * 8)
    k = int(f32(THN) * f32(v.size))
    nth = np.sqrt(np.partition(v, k)[k], dtype=f32)
    th = f32(nth * f32(FAC))
    th = f32(f32(26.0) * f32(CW) + th * f32(1 - f32(CW)))
    th = f32(th * th)
    return f32(th * f32(f32(OW) * f32(OW)))


def device_threshold(c):
    from hslam_amd._lib import check, load
    lib = load()
    fn = lib.hs_debug_threshold
    fn.argtypes = [C.c_void_p, C.c_int, C.c_float, C.c_float, C.c_float, C.c_float, C.c_void_p]
    fn.restype = C.c_int
    c = np.ascontiguousarray(c, np.float32)
    out = np.zeros(1, np.float32)
    check(fn(c.ctypes.data, c.size, THN, FAC, CW, OW, out.ctypes.data))
    return out[0]


def _cases():
    rng = np.random.default_rng(11)
    yield "exp2k", rng.exponential(300.0, 2000).astype(np.float32)
    yield "spread200k", (rng.lognormal(5.0, 2.0, 200_000)).astype(np.float32)
    yield "equal200k", np.full(200_000, 417.25, np.float32)  # every candidate in one bin: the re-scan path
    narrow = (1000.0 + rng.integers(0, 64, 60_000) * np.float32(1.0 / 1024)).astype(np.float32)
    yield "ties60k", narrow
    mixed = rng.exponential(50.0, 30_000).astype(np.float32)
    mixed[::3] = -1.0
    mixed[1::7] = np.nan
    mixed[2::11] = 0.0
    yield "mixed30k", mixed
    yield "none", np.full(500, -1.0, np.float32)
    yield "one", np.array([-1.0, 5.0, -1.0], np.float32)


@pytest.mark.parametrize("name,c", list(_cases()), ids=[n for n, _ in _cases()])
def test_threshold_select_matches_nth_element(name, c):
    assert device_threshold(c) == ref_threshold(c)
