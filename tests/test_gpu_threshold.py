"""setNewFrameEnergyTH's select (Src/FullSystemOptimize.cpp:60-101) on the device: hs_k_reduce's pass-1 histogram
blocks + the select block of the stitch launch (through the test hook hs_debug_threshold), against nth_element
restated in numpy fp32.  Bit-exact, including the fallback when more than TH_CAP candidates share the first
12-bit bin, ties, and windows without a newest-frame residual.  multi: the large-window path (pass 2 over up to 64
blocks with a global survivor list, pass 3 on it), including every block overflowing its LDS survivor buffer."""
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


def device_threshold(c, multi=0, thn=THN, fac=FAC, cw=CW, ow=OW):
    from hslam_amd._lib import check, load
    lib = load()
    fn = lib.hs_debug_threshold
    fn.argtypes = [C.c_void_p, C.c_int, C.c_float, C.c_float, C.c_float, C.c_float, C.c_int, C.c_void_p]
    fn.restype = C.c_int
    c = np.ascontiguousarray(c, np.float32)
    out = np.zeros(1, np.float32)
    check(fn(c.ctypes.data, c.size, thn, fac, cw, ow, int(multi), out.ctypes.data))
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


def _multi_cases():
    rng = np.random.default_rng(12)
    yield "spread200k", (rng.lognormal(5.0, 2.0, 200_000)).astype(np.float32), 0
    yield "spread200k_np2_3", (rng.lognormal(5.0, 2.0, 200_000)).astype(np.float32), 3
    # every pass-2 block keeps more than TH_CAP (24576) survivors: > 64 * TH_CAP equal candidates
    yield "equal1.7M", np.full(1_700_000, 417.25, np.float32), 0
    narrow = (1000.0 + rng.integers(0, 64, 400_000) * np.float32(1.0 / 1024)).astype(np.float32)
    yield "ties400k", narrow, 0
    mixed = rng.exponential(50.0, 120_000).astype(np.float32)
    mixed[::3] = -1.0
    mixed[1::7] = np.nan
    yield "mixed120k_np2_7", mixed, 7


@pytest.mark.parametrize("name,c,np2", list(_multi_cases()), ids=[n for n, _, _ in _multi_cases()])
def test_multi_block_threshold_matches_nth_element(name, c, np2):
    assert device_threshold(c, multi=np2 if np2 > 1 else 1) == ref_threshold(c)


@pytest.mark.parametrize("name,c", list(_cases()), ids=[n for n, _ in _cases()])
def test_rank_select_block_matches_nth_element(name, c):
    """The multi-rank path's one-block select (block 1 of the solve / hs_k_combine launch, 512 threads, pass 1
    counted in LDS, SOLVE_TH_CAP survivors in the solve's LDS; more: the pass-3 re-scan)."""
    assert device_threshold(c, multi=-1) == ref_threshold(c)
