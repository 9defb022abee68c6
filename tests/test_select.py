"""PixelSelector::makeHists / makeMaps / select (Src/PixelSelector.cpp:14-418): the oracle restatement
(oracle/sel_oracle.cpp) pinned against a second, pure-Python loop restatement on small images and the C
library's generator; the device path (include/hs_select.h) bit-exact against the oracle.  Bar: bit-exact — the
selection is integer / categorical work (float comparisons in the reference's operation order)."""
import ctypes

import numpy as np
import pytest

DIRS = [(0, 1.0000), (0.3827, 0.9239), (0.1951, 0.9808), (0.9239, 0.3827), (0.7071, 0.7071), (0.3827, -0.9239),
        (0.8315, 0.5556), (0.8315, -0.5556), (0.5556, -0.8315), (0.9808, 0.1951), (0.9239, -0.3827),
        (0.7071, -0.7071), (0.5556, 0.8315), (0.9808, -0.1951), (1.0000, 0.0000), (0.1951, -0.9808)]
F = np.float32


class LoopSelector:
    """Pure-Python loops after Src/PixelSelector.cpp (small images only); fp32 via numpy scalars."""

    def __init__(self, W, H, pattern):
        self.W, self.H, self.pat = W, H, pattern
        self.pot, self.histFrame = 3, -1
        w32, h32 = W // 32, H // 32
        self.ths = np.zeros(max(w32 * h32 + 100, w32 * (h32 + 1) + 1), F)
        self.thsS = np.zeros_like(self.ths)

    def hists(self, g0, id):  # :57-117
        self.histFrame = id
        W, H = self.W, self.H
        w32, h32 = W // 32, H // 32
        for y in range(h32):
            for x in range(w32):
                hist = [0] * 50
                for j in range(32):
                    for i in range(32):
                        it, jt = i + 32 * x, j + 32 * y
                        if it > W - 2 or jt > H - 2 or it < 1 or jt < 1:
                            continue
                        g = min(int(np.sqrt(F(g0[jt, it]))), 48)
                        hist[g + 1] += 1
                        hist[0] += 1
                th = int(F(hist[0]) * F(0.5) + F(0.5))
                q = 90
                for i in range(90):
                    th -= hist[i + 1] if i + 1 < 50 else 0
                    if th < 0:
                        q = i
                        break
                self.ths[x + y * w32] = F(q) + F(7)
        for y in range(h32):
            for x in range(w32):
                s, n = F(0), F(0)
                t = self.ths
                nb = []
                if x > 0:
                    if y > 0: nb.append(t[x - 1 + (y - 1) * w32])
                    if y < h32 - 1: nb.append(t[x - 1 + (y + 1) * w32])
                    nb.append(t[x - 1 + y * w32])
                if x < w32 - 1:
                    if y > 0: nb.append(t[x + 1 + (y - 1) * w32])
                    if y < h32 - 1: nb.append(t[x + 1 + (y + 1) * w32])
                    nb.append(t[x + 1 + y * w32])
                if y > 0: nb.append(t[x + (y - 1) * w32])
                if y < h32 - 1: nb.append(t[x + (y + 1) * w32])
                nb.append(t[x + y * w32])
                for v in nb:
                    s = F(s + v)
                    n = F(n + 1)
                self.thsS[x + y * w32] = F(F(s / n) * F(s / n))

    def select(self, d0, g, pot, thF):  # :265-415
        W, H = self.W, self.H
        w1, w2 = W >> 1, W >> 2
        out = np.zeros((H, W), F)
        dw1 = F(0.75)
        dw2 = F(dw1 * dw1)
        n2 = n3 = n4 = 0
        gx, gy = d0[..., 1].ravel(), d0[..., 2].ravel()
        g0, g1, g2 = g[0].ravel(), g[1].ravel(), g[2].ravel()

        def dot(idx, d):
            return abs(F(F(gx[idx] * F(d[0])) + F(gy[idx] * F(d[1]))))

        for y4 in range(0, H, 4 * pot):
            for x4 in range(0, W, 4 * pot):
                my3, mx3 = min(4 * pot, H - y4), min(4 * pot, W - x4)
                b4, v4 = -1, F(0)
                dir4 = DIRS[self.pat[n2] & 0xF]
                for y3 in range(0, my3, 2 * pot):
                    for x3 in range(0, mx3, 2 * pot):
                        x34, y34 = x3 + x4, y3 + y4
                        my2, mx2 = min(2 * pot, H - y34), min(2 * pot, W - x34)
                        b3, v3 = -1, F(0)
                        dir3 = DIRS[self.pat[n2] & 0xF]
                        for y2 in range(0, my2, pot):
                            for x2 in range(0, mx2, pot):
                                x234, y234 = x2 + x34, y2 + y34
                                my1, mx1 = min(pot, H - y234), min(pot, W - x234)
                                b2, v2 = -1, F(0)
                                dir2 = DIRS[self.pat[n2] & 0xF]
                                for y1 in range(my1):
                                    for x1 in range(mx1):
                                        xf, yf = x1 + x234, y1 + y234
                                        idx = xf + W * yf
                                        if xf < 4 or xf >= W - 5 or yf < 4 or yf > H - 4:
                                            continue
                                        t0 = self.thsS[(xf >> 5) + (yf >> 5) * (W // 32)]
                                        t1 = F(t0 * dw1)
                                        t2 = F(t1 * dw2)
                                        if g0[idx] > F(t0 * F(thF)):
                                            dn = dot(idx, dir2)
                                            if dn > v2:
                                                v2, b2, b3, b4 = dn, idx, -2, -2
                                        if b3 == -2:
                                            continue
                                        ag1 = g1[int(F(F(xf) * F(0.5)) + F(0.25)) + int(F(F(yf) * F(0.5)) + F(0.25)) * w1]
                                        if ag1 > F(t1 * F(thF)):
                                            dn = dot(idx, dir3)
                                            if dn > v3:
                                                v3, b3, b4 = dn, idx, -2
                                        if b4 == -2:
                                            continue
                                        ag2 = g2[int(xf * 0.25 + 0.125) + int(yf * 0.25 + 0.125) * w2]
                                        if ag2 > F(t2 * F(thF)):
                                            dn = dot(idx, dir4)
                                            if dn > v4:
                                                v4, b4 = dn, idx
                                if b2 > 0:
                                    out.flat[b2] = 1
                                    v3 = F(1e10)
                                    n2 += 1
                        if b3 > 0:
                            out.flat[b3] = 2
                            v4 = F(1e10)
                            n3 += 1
                if b4 > 0:
                    out.flat[b4] = 4
                    n4 += 1
        return out, (n2, n3, n4)

    def makeMaps(self, d0, g, id, density, rec=1, thF=1.0):  # :118-262
        if id != self.histFrame:
            self.hists(g[0], id)
        out, n = self.select(d0, g, self.pot, thF)
        numHave = F(sum(n))
        quotia = F(F(density) / numHave)
        K = F(numHave * F((self.pot + 1) * (self.pot + 1)))
        ideal = max(int(F(np.sqrt(F(K / F(density)))) - F(1)), 1)
        if rec > 0 and quotia > 1.25 and self.pot > 1:
            self.pot = min(ideal, self.pot - 1)
            return self.makeMaps(d0, g, id, density, rec - 1, thF)
        if rec > 0 and quotia < 0.25:
            self.pot = max(ideal, self.pot + 1)
            return self.makeMaps(d0, g, id, density, rec - 1, thF)
        sub = int(numHave)
        if quotia < 0.95:
            charTH = int(F(255) * quotia)
            rn = 0
            flat = out.ravel()
            for i in range(flat.size):
                if flat[i] != 0:
                    if self.pat[rn] > charTH:
                        flat[i] = 0
                        sub -= 1
                    rn += 1
        self.pot = ideal
        return out, sub


def pyr3(img):
    from oracle_ffi import dir_pyramid
    p, g = dir_pyramid(img, 3)
    return p[0], g


@pytest.fixture(scope="module")
def frames():
    from hslam_amd.scene import make_select_frames
    return {
        "vga": make_select_frames(3, contrast_ramp=True),
        "vga_q": make_select_frames(3, contrast_ramp=True, quantize=True, seed=11),
        "kitti": make_select_frames(2, width=1232, height=368, contrast_ramp=True, flat_frac=0.2),
        "plain": make_select_frames(2, seed=5),
    }


# ------------------------------------------------------------------------------------------ oracle (CPU)

def test_random_pattern_is_the_c_library_generator():
    from oracle_ffi import PixelSelector
    s = PixelSelector(64, 48)
    libc = ctypes.CDLL("libc.so.6")
    libc.srand(3141592)
    ref = np.array([libc.rand() & 0xFF for _ in range(64 * 48)], np.uint8)
    assert np.array_equal(s.randomPattern(), ref)


@pytest.mark.parametrize("quant", [False, True])
def test_oracle_matches_python_loops(quant):
    """Two independent restatements of the reference agree map for map across a frame sequence (potential and
    histogram caching carried over), densities that trigger both re-selection branches and the sub-sampling."""
    from hslam_amd.scene import make_select_frames
    from oracle_ffi import PixelSelector
    W, H = 160, 96
    imgs = make_select_frames(3, width=W, height=H, contrast_ramp=True, quantize=quant, seed=3)
    o = PixelSelector(W, H)
    py = LoopSelector(W, H, o.randomPattern())
    for i, (img, dens) in enumerate(zip(imgs + imgs[:1], (300, 60, 900, 150))):
        d0, g = pyr3(img)
        mo, no = o.makeMaps(i, d0, g, dens)
        mp, npy = py.makeMaps(d0, g, i, dens)
        assert no == npy and np.array_equal(mo, mp), i
        assert o.currentPotential == py.pot, i
    ths, thsS = o.ths()
    assert np.array_equal(thsS.ravel(), py.thsS[:thsS.size])


def test_oracle_thfactor_and_no_recursion():
    from hslam_amd.scene import make_select_frames
    from oracle_ffi import PixelSelector
    W, H = 128, 96
    img = make_select_frames(1, width=W, height=H, contrast_ramp=True, seed=4)[0]
    d0, g = pyr3(img)
    for thF, rec in ((2.0, 0), (0.5, 1), (1.0, 2)):
        o = PixelSelector(W, H)
        py = LoopSelector(W, H, o.randomPattern())
        mo, no = o.makeMaps(0, d0, g, 200, rec, thF)
        mp, npy = py.makeMaps(d0, g, 0, 200, rec, thF)
        assert no == npy and np.array_equal(mo, mp), (thF, rec)


def test_oracle_selection_invariants(frames):
    """Map values are 0/1/2/4; at most one level-0 pixel per pot-block; nothing inside the 4-px border."""
    from oracle_ffi import PixelSelector
    img = frames["vga"][0]
    d0, g = pyr3(img)
    o = PixelSelector(640, 480)
    o.currentPotential = 4
    m, n = o.makeMaps(0, d0, g, 1e9, 0)  # recursionsLeft 0, quotia >= 0.95: no sub-sampling, pot stays 4 here
    assert set(np.unique(m)) <= {0.0, 1.0, 2.0, 4.0}
    assert n == int((m != 0).sum())
    assert not m[:4].any() and not m[:, :4].any() and not m[:, 640 - 5:].any() and not m[480 - 3:].any()
    ones = (m == 1).reshape(480 // 4, 4, 640 // 4, 4).sum((1, 3))
    assert ones.max() <= 1


def test_oracle_kitti_partial_cells(frames):
    """1232 x 368: the last partial 32-cell column / row reads the zeroed slack of the threshold table."""
    from oracle_ffi import PixelSelector
    img = frames["kitti"][0]
    d0, g = pyr3(img)
    o = PixelSelector(1232, 368)
    m, n = o.makeMaps(0, d0, g, 2000)
    assert 1500 < n < 2600
    # rows >= 352 sit in the slack (threshold 0): their pixels pass on any non-zero gradient
    assert (m[352:] != 0).sum() > 0


# ------------------------------------------------------------------------------------------ device

def _pair(W, H, params=None):
    from hslam_amd.select import PixelSelector as Dev
    from oracle_ffi import PixelSelector as Ora
    return Dev(W, H, params=params), Ora(W, H, params=params)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["vga", "vga_q", "kitti", "plain"])
def test_device_make_maps_bit_exact(frames, name):
    imgs = frames[name]
    H, W = imgs[0].shape
    dev, ora = _pair(W, H)
    seq = [(0, 2000), (1, 2000), (1, 700), (2 % len(imgs), 6000), (0, 2000), (1, 150)]
    for fid, dens in seq:
        d0, g = pyr3(imgs[fid])
        md, nd = dev.makeMaps(d0, fid, g, dens)
        mo, no = ora.makeMaps(fid, d0, g, dens)
        assert nd == no, (name, fid, dens, nd, no)
        assert np.array_equal(md, mo), (name, fid, dens, int((md != mo).sum()))
        assert dev.currentPotential == ora.currentPotential


@pytest.mark.gpu
def test_device_potentials_thfactor_dirdist(frames):
    from hslam_amd._lib import default_params
    img = frames["vga_q"][0]
    d0, g = pyr3(img)
    for dirdist in (1, 0):
        p = default_params()
        p.selectDirectionDistribution = dirdist
        dev, ora = _pair(640, 480, params=p)
        for pot in (1, 2, 3, 7, 16, 40):
            for thF, rec in ((1.0, 0), (2.0, 0), (0.5, 1)):
                dev.currentPotential = pot
                ora.currentPotential = pot
                md, nd = dev.makeMaps(d0, 0, g, 1500, rec, thF)
                mo, no = ora.makeMaps(0, d0, g, 1500, rec, thF)
                assert nd == no and np.array_equal(md, mo), (dirdist, pot, thF, rec)
                assert dev.currentPotential == ora.currentPotential


@pytest.mark.gpu
def test_device_raw_frame_matches_host_pyramid(frames):
    imgs = frames["kitti"]
    a, _ = _pair(1232, 368)
    from hslam_amd.select import PixelSelector as Dev
    b = Dev(1232, 368)
    for fid, img in enumerate(imgs):
        d0, g = pyr3(img)
        ma, na = a.makeMaps(d0, fid, g, 2000)
        mb, nb = b.makeMapsRaw(img, fid, 2000)
        assert na == nb and np.array_equal(ma, mb), fid
    ms, passes = b.last_stats()
    assert ms > 0 and passes in (1, 2)


@pytest.mark.gpu
def test_device_rejects_bad_arguments():
    from hslam_amd._lib import HsError
    from hslam_amd.select import PixelSelector as Dev
    d = Dev(64, 64)
    with pytest.raises(HsError):
        d.makeMapsRaw(np.zeros((64, 64), np.float32), 0, -1.0)
    with pytest.raises(HsError):
        d.currentPotential = 0
    with pytest.raises(ValueError):
        d.makeMapsRaw(np.zeros((32, 64), np.float32), 0, 100.0)
