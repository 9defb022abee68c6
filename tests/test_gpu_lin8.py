"""GPU parity of hs_k_lin8, the production linearize + accumulate kernel with lane = (point, target slot)
(h-slam_amd/csrc/hs_lin8_kernels.hip), forced on with HS_LIN8=1 at every window size.

Bars:
* per-residual outputs (state, active, energy, energy-with-outlier, JpJdF, centre projection) and the per-point
  Schur prelude (HdiF, bdSumF, the fused point step, idepth): bit-exact against the oracle and against hs_k_lin
  (HS_LIN8=0) -- the per-residual arithmetic is the reference's, in its order;
* stitched H / b: the production bar of tests/test_gpu_ba.py (H_TOL, the fp32 accumulation order differs);
* the GN trajectory: as close to the single-thread oracle as the oracle's own 8-thread pool (x 10), like
  test_split_accumulation_matches_threaded_reference;
* two runs: bit-identical (fixed-order block partials, no order-dependent atomics).
"""
import os

import numpy as np
import pytest

from test_gpu_ba import _close_b, _close_H

pytestmark = pytest.mark.gpu


def _window(scene, lin8):
    from hslam_amd.ba import BAWindow
    os.environ["HS_LIN8"] = "1" if lin8 else "0"
    try:
        return BAWindow(scene)
    finally:
        os.environ.pop("HS_LIN8", None)


@pytest.mark.parametrize("scene_name", ["scene_small", "scene2k", "scene_kitti2k", "scene_kitti20k"])
def test_lin8_linearize_bit_exact(scene_name, request):
    from oracle_ffi import OracleBA
    scene = request.getfixturevalue(scene_name)
    g = _window(scene, True)
    o = OracleBA(scene)
    eg = g.linearizeAll(reset=True)
    eo = o.linearize_all(reset=True)
    o.apply_res()
    rg, ro = g.residuals(), o.residuals()
    assert np.array_equal(rg["state"], ro["state"])
    active_o = ro["state"] == 0
    assert np.array_equal(rg["active"].astype(bool), active_o)
    assert np.array_equal(rg["energy"], ro["energy"].astype(np.float32))
    assert np.array_equal(rg["energy_wo"], ro["energy_wo"].astype(np.float32))
    assert np.array_equal(rg["JpJdF"][active_o], ro["JpJdF"][active_o])
    assert np.array_equal(rg["center"][active_o], ro["center"][active_o])
    assert abs(eg - eo) <= 1e-9 * abs(eo)
    assert np.array_equal(g.frames()["energyTH"], o.frames()["energyTH"])
    for which in (0, 1, 2):
        Ho, bo = o.accumulate(which)
        Hg, bg = g.system(which)
        okH, rH = _close_H(Hg, Ho)
        okb, rb = _close_b(bg, bo, Ho)
        assert okH, f"which={which} H worst ratio {rH}"
        assert okb, f"which={which} b worst ratio {rb}"
    g.close()


@pytest.mark.parametrize("scene_name", ["scene2k", "scene_kitti20k"])
def test_lin8_matches_lin(scene_name, request):
    """hs_k_lin8 against hs_k_lin on the same window through two fused GN iterations: the per-residual and
    per-point outputs bit-identical after the first linearization (same inputs), the systems at the H bar."""
    scene = request.getfixturevalue(scene_name)
    g8, g1 = _window(scene, True), _window(scene, False)
    for g in (g8, g1):
        g.linearizeAll(reset=True)
    r8, r1 = g8.residuals(), g1.residuals()
    for k in r8:
        assert np.array_equal(r8[k], r1[k]), k
    p8, p1 = g8.points(), g1.points()
    for k in ("HdiF", "bdSumF", "idepth"):
        assert np.array_equal(p8[k], p1[k]), k
    for which in (0, 1, 2):
        H8, b8 = g8.system(which)
        H1, b1 = g1.system(which)
        assert _close_H(H8, H1)[0] and _close_b(b8, b1, H1)[0], which
    # fused GN iterations (hs_k_lin8's in-kernel resubstitution + point step): the two kernels' systems differ in
    # fp32 accumulation order only, so the energies stay together at the GN-step level
    e8 = g8.iterate(0, 3)
    e1 = g1.iterate(0, 3)
    assert np.all(np.abs(e8 - e1) <= 1e-3 * np.abs(e1)), (e8, e1)
    g8.close()
    g1.close()


@pytest.mark.parametrize("scene_name", ["scene2k", "scene_kitti2k"])
def test_lin8_trajectory(scene_name, request):
    from oracle_ffi import OracleBA
    scene = request.getfixturevalue(scene_name)
    g = _window(scene, True)
    o1 = OracleBA(scene)
    o8 = OracleBA(scene, nthreads=8)
    _, eg = g.optimize(6)
    _, e1 = o1.optimize(6)
    _, e8 = o8.optimize(6)
    dev_pool = np.abs(e8 - e1) / np.abs(e1)
    dev_gpu = np.abs(eg - e1) / np.abs(e1)
    assert dev_gpu[0] <= 1e-9
    assert np.all(dev_gpu <= np.maximum(10 * dev_pool, 1e-3))
    assert eg[-1] < 0.5 * eg[0]
    g.close()


def test_lin8_grid_fills_every_cu(scene_kitti20k):
    """At 20k points a wave takes more than one point group, so the partition gives every host floor(256 nh / nP)
    blocks instead of ceil(nh / (64 ppw)): one block per CU of the 256, a host's blocks covering equal shares of its
    (row-major) points (hs_ba.cpp make_partition; DESIGN.md §4, hs_k_lin8 round 6).  Against the old count
    (HS_LIN8_NOFILL=1): the per-residual and per-point outputs bit-identical (the blocks only regroup the points), the
    systems at the H bar (the fp32 block partials group differently)."""
    g = _window(scene_kitti20k, True)
    os.environ["HS_LIN8_NOFILL"] = "1"
    try:
        g0 = _window(scene_kitti20k, True)
    finally:
        os.environ.pop("HS_LIN8_NOFILL", None)
    nF = len(scene_kitti20k.frames_id)
    pf, p0 = g.partition(), g0.partition()
    assert pf["kernel"] == p0["kernel"] == "hs_k_lin8"
    assert 256 <= pf["blocks"] <= 256 + nF and p0["blocks"] < pf["blocks"], (pf, p0)
    for w in (g, g0):
        w.linearizeAll(reset=True)
    rf, r0 = g.residuals(), g0.residuals()
    for k in rf:
        assert np.array_equal(rf[k], r0[k]), k
    for k in ("HdiF", "bdSumF", "idepth"):
        assert np.array_equal(g.points()[k], g0.points()[k]), k
    for which in (0, 1, 2):
        Hf, bf = g.system(which)
        H0, b0 = g0.system(which)
        assert _close_H(Hf, H0)[0] and _close_b(bf, b0, H0)[0], which
    g.close()
    g0.close()


def test_lin8_filled_grid_five_frames():
    """The filled partition on a 5-frame window of 20k points with unequal hosts (floor(256 nh / nP) blocks per host,
    Σ within 256 + nF): hs_k_lin8 against hs_k_lin -- per-residual and per-point outputs bit-identical, the systems
    at the H bar, two fused GN iterations together."""
    from hslam_amd.scene import make_ba_scene
    scene = make_ba_scene(n_points=20003, n_frames=5, seed=11)
    g8, g1 = _window(scene, True), _window(scene, False)
    p8 = g8.partition()
    assert p8["kernel"] == "hs_k_lin8" and 250 <= p8["blocks"] <= 256 + 5, p8
    for g in (g8, g1):
        g.linearizeAll(reset=True)
    r8, r1 = g8.residuals(), g1.residuals()
    for k in r8:
        assert np.array_equal(r8[k], r1[k]), k
    for k in ("HdiF", "bdSumF", "idepth"):
        assert np.array_equal(g8.points()[k], g1.points()[k]), k
    for which in (0, 1, 2):
        H8, b8 = g8.system(which)
        H1, b1 = g1.system(which)
        assert _close_H(H8, H1)[0] and _close_b(b8, b1, H1)[0], which
    e8 = g8.iterate(0, 2)
    e1 = g1.iterate(0, 2)
    assert np.all(np.abs(e8 - e1) <= 1e-3 * np.abs(e1)), (e8, e1)
    g8.close()
    g1.close()


def test_lin8_runs_are_bit_reproducible(scene_kitti20k):
    outs = []
    for _ in range(2):
        g = _window(scene_kitti20k, True)
        g.linearizeAll(reset=True)
        H0, b0 = g.system(0)
        H2, b2 = g.system(2)
        e = g.iterate(0, 3)
        outs.append((H0, b0, H2, b2, e, g.frames()["state"], g.points()["idepth"]))
        g.close()
    for a, b in zip(*outs):
        assert np.array_equal(a, b)


def test_multi_block_select_matches_in_stitch_select(scene2k):
    """setNewFrameEnergyTH's select as a multi-block pass 2 in the stitch launch + a one-block pass 3 (HS_TH_MULTI=1,
    the default from 60k points) against the stitch's single select block (HS_TH_MULTI=0): the same counts, so the
    fused GN loop's energies, thresholds, frame states and depths are bit-identical."""
    from hslam_amd.ba import BAWindow
    outs = []
    for mode in ("1", "0"):
        os.environ["HS_TH_MULTI"] = mode
        try:
            g = BAWindow(scene2k)
        finally:
            os.environ.pop("HS_TH_MULTI", None)
        g.linearizeAll(reset=True)
        e = g.iterate(0, 5)
        f = g.frames()
        outs.append((e, f["energyTH"], f["state"], g.points()["idepth"]))
        g.close()
    for a, b in zip(*outs):
        assert np.array_equal(a, b)


def test_lin8_counted_histogram_matches_reduce_blocks(scene_kitti20k):
    """The multi-block select's pass-1 histogram counted inside hs_k_lin8 as the candidates are written (the default
    for large single-rank windows) against hs_k_reduce's histogram blocks (HS_LIN8_HIST=0) and against the one-block
    select (HS_TH_MULTI=0): integer counts, so the fused GN loop's energies, thresholds, frame states and depths are
    bit-identical (HS_TH_MULTI=1 / HS_LIN8=1 force the large-window path on the 20k window)."""
    from hslam_amd.ba import BAWindow
    outs = []
    for multi, lin_hist in (("1", "1"), ("1", "0"), ("0", "1")):
        os.environ.update(HS_TH_MULTI=multi, HS_LIN8="1", HS_LIN8_HIST=lin_hist)
        try:
            g = BAWindow(scene_kitti20k)
            g.linearizeAll(reset=True)
            e = g.iterate(0, 5)
            f = g.frames()
            outs.append((e, f["energyTH"], f["state"], g.points()["idepth"]))
            g.close()
        finally:
            for k in ("HS_TH_MULTI", "HS_LIN8", "HS_LIN8_HIST"):
                os.environ.pop(k, None)
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            assert np.array_equal(a, b)


def _fastmath(a, b):
    import ctypes as C
    from hslam_amd import _lib
    lib = _lib.load()
    fn = lib.hs_debug_fastmath
    fn.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
    fn.restype = C.c_int
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    out = np.zeros((len(a), 4), np.float32)
    assert fn(len(a), a.ctypes.data, b.ctypes.data, out.ctypes.data) == 0
    return out


def test_fast_div_sqrt_match_ieee():
    """hs_k_lin8's range-step-free quotient / square root (div_nr, sqrt_nr) against the device's IEEE a / b and
    sqrtf, bitwise, over the ranges the pixel loop admits (log-uniform magnitudes, random signs, plus the range ends
    and exact cases); the IEEE forms against numpy's correctly rounded float32 results."""
    rng = np.random.default_rng(3)
    n = 1 << 21
    lb = rng.uniform(-60, 60, n)
    lq = rng.uniform(-90, 90, n)
    lq = np.clip(lq, -60 - lb, 127.9 - lb)  # |a| = |q| |b| in [2^-60, 2^127.9] (finite)
    sgn = lambda: rng.choice([-1.0, 1.0], n)  # noqa: E731
    b = (sgn() * np.exp2(lb)).astype(np.float32)
    a = (sgn() * np.exp2(lq) * b.astype(np.float64)).astype(np.float32)
    ends = np.array([2.0 ** -60, 2.0 ** 60, 1.0, 3.0, 0.1, 2500.0, 9.0, 2.0 ** 59.5], np.float32)
    ea, eb = np.meshgrid(ends, ends)
    a = np.concatenate([a, ea.ravel(), -ea.ravel(), np.zeros(4, np.float32)])
    b = np.concatenate([b, eb.ravel(), eb.ravel(), np.array([1, -1, 2.0 ** -60, 2.0 ** 60], np.float32)])
    out = _fastmath(a, b)
    bad = out[:, 0].view(np.uint32) != out[:, 1].view(np.uint32)
    assert not bad.any(), (a[bad][:5], b[bad][:5], out[bad][:5])
    assert np.array_equal(out[:, 1], a / b)
    ls = rng.uniform(-96, 127.9, n)
    x = np.concatenate([np.exp2(ls), [0.0, 1.0, 2.0 ** -96, 4.0, 2.0, 0.25]]).astype(np.float32)
    out = _fastmath(x, np.ones_like(x))
    assert np.array_equal(out[:, 2].view(np.uint32), out[:, 3].view(np.uint32))
    assert np.array_equal(out[:, 3], np.sqrt(x))


def test_lin8_out_of_range_group_falls_back(scene2k):
    """Texels whose gradients put the pixel loop's operands outside div_nr / sqrt_nr's exact ranges (|grad|^2 above
    2^60, infinite gradients): the affected point groups are redone with IEEE a / b and sqrtf, so the per-residual
    outputs stay bit-identical to hs_k_lin's and the oracle's."""
    import copy

    from oracle_ffi import OracleBA
    scene = copy.deepcopy(scene2k)
    for f, val in ((1, 3e18), (2, np.inf), (3, 1e30)):
        img = scene.pyramids[f][0]
        h, w = img.shape[:2]
        img[h // 4: h // 2, w // 4: w // 2, 1:3] = val
    g8, g1 = _window(scene, True), _window(scene, False)
    o = OracleBA(scene)
    g8.linearizeAll(reset=True)
    g1.linearizeAll(reset=True)
    o.linearize_all(reset=True)
    o.apply_res()
    r8, r1, ro = g8.residuals(), g1.residuals(), o.residuals()
    for k in r8:
        assert np.array_equal(r8[k], r1[k], equal_nan=True), k
    assert np.array_equal(r8["state"], ro["state"])
    assert np.array_equal(r8["energy"], ro["energy"].astype(np.float32), equal_nan=True)
    g8.close()
    g1.close()
