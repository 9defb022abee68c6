"""GPU parity of the CoarseTracker path (HIP kernels through include/hs_track.h) against the CPU oracle.

Bars:
* makeCoarseDepthL0 pc_u / pc_v / pc_idepth / pc_color and pc_n per level: bit-exact;
* calcRes categorical counts (numTermsInE, saturated, buf_warped_n): exact;
  energy E (fp32 sum in a different order): rel <= 2e-5; flow indicators rel <= 1e-4;
  calcGSSSE H / b: |d| <= 1e-4 (|ref| + 1e-3 max|diag H|);
* trackNewestCoarse / the try loop: the per-iteration LM logs (accept-test ratios, step norms) agree up to the
  first decision that is a near-tie in the oracle itself (fp32 sums in another order can flip a tie), at bars tied
  to the oracle's OWN summation-order spread: the oracle run again with every calcRes / calcGSSSE sum formed in
  reversed point order (hso_trk_set_sum_order) moves the ratios / step norms / final pose by s; the GPU (whose
  sums are wave trees and, with HS_TRK_G > 1, workgroup partials) may deviate by max(floor, 10 s) -- floors 1e-4
  (ratios), 1e-3 (step norms), 1e-5 (pose).  If no tie occurs the final pose agrees to that bar and
  lastResiduals to 1e-4 rel, otherwise to the LM's own stopping tolerance (pose 2e-3, lastResiduals 1e-2 rel).
  ok / haveOneGood / tryIterations: equal.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def vga():
    from hslam_amd.scene import make_track_scene
    return make_track_scene(n_points=2000, n_levels=5)


@pytest.fixture(scope="module")
def pair(vga):
    from hslam_amd.track import CoarseTracker
    from oracle_ffi import OracleTracker
    g = CoarseTracker(vga.width, vga.height, vga.K4, vga.n_levels)
    g.set_scene(vga)
    o = OracleTracker(vga.width, vga.height, vga.K4, vga.n_levels)
    o.set_scene(vga)
    return g, o


def _pose_err(a, b):
    from hslam_amd.se3 import SE3
    return float(np.linalg.norm((SE3.from_data(a) * SE3.from_data(b).inverse()).log()))


def test_coarse_depth_bit_exact(vga, pair):
    g, o = pair
    for l in range(vga.n_levels):
        pg, po = g.pc(l), o.pc(l)
        assert len(pg["u"]) == len(po["u"]) > 0
        for k in ("u", "v", "idepth", "color"):
            assert np.array_equal(pg[k], po[k]), (l, k)


@pytest.mark.parametrize("kitti", [False, True])
def test_coarse_depth_dups_and_kitti(kitti):
    from hslam_amd.scene import make_track_scene
    from hslam_amd.track import CoarseTracker
    from oracle_ffi import OracleTracker
    s = (make_track_scene(n_points=3000, width=1232, height=368, kitti=True, n_levels=5, dup_frac=0.2) if kitti
         else make_track_scene(n_points=1500, dup_frac=0.4, seed=11))
    g = CoarseTracker(s.width, s.height, s.K4, s.n_levels)
    g.set_scene(s)
    o = OracleTracker(s.width, s.height, s.K4, s.n_levels)
    o.set_scene(s)
    for l in range(s.n_levels):
        pg, po = g.pc(l), o.pc(l)
        for k in ("u", "v", "idepth", "color"):
            assert np.array_equal(pg[k], po[k]), (l, k)


def _close_H(Hg, Ho, tol=1e-4):
    scale = np.abs(np.diag(Ho)).max()
    return bool(np.all(np.abs(Hg - Ho) <= tol * (np.abs(Ho) + 1e-3 * scale)))


@pytest.mark.parametrize("which", ["identity", "truth", "perturbed"])
def test_calc_res_parity(vga, pair, which):
    from hslam_amd.se3 import SE3
    g, o = pair
    T = {"identity": SE3().data(), "truth": vga.T_true,
         "perturbed": (SE3.exp([0.004, -0.003, 0.002, 0.002, 0.001, -0.002]) * SE3.from_data(vga.T_true)).data()}[which]
    aff = [0.0, 0.0] if which == "identity" else list(vga.aff_true)
    for lvl in range(vga.n_levels):
        for cut in (g.params.coarseCutoffTH, 2 * g.params.coarseCutoffTH):
            rg, Hg, bg, ng = g.calcRes(lvl, T, aff, cut)
            ro, Ho, bo, no = o.calc_res(lvl, T, aff, cut)
            assert ng == no and rg[1] == ro[1], (lvl, cut)
            assert round(rg[5] * rg[1]) == round(ro[5] * ro[1])
            assert abs(rg[0] - ro[0]) <= 2e-5 * abs(ro[0]) + 1e-3
            for k in (2, 4):
                assert abs(rg[k] - ro[k]) <= 1e-4 * abs(ro[k]) + 1e-6
            assert _close_H(Hg, Ho), (lvl, np.abs(Hg - Ho).max())
            sb = np.abs(bo).max() + 1e-30
            assert np.all(np.abs(bg - bo) <= 1e-4 * (np.abs(bo) + 1e-3 * sb))


def _order_spread(o, T0, aff, coarsest, minRes):
    """The oracle's own summation-order spread on this LM run: (ratio, step norm, pose) relative deviations of the
    reversed-order run from the reference-order run, over their common prefix (until a level or decision differs).
    Leaves the oracle in the reference order with the reference-order run as its last run."""
    o.set_sum_order(1)
    r1 = o.track(T0, aff, coarsest, minRes)
    l1 = o.lm_log()
    o.set_sum_order(0)
    r0 = o.track(T0, aff, coarsest, minRes)
    l0 = o.lm_log()
    sr, si = 0.0, 0.0
    tie = len(l0[0]) != len(l1[0])
    for k in range(min(len(l0[0]), len(l1[0]))):
        if l0[0][k] != l1[0][k] or (l0[1][k] < l0[2][k]) != (l1[1][k] < l1[2][k]) or \
                (l0[3][k] > 1e-3) != (l1[3][k] > 1e-3) or l0[3][k] > 1.0:
            tie = True
            break
        sr = max(sr, abs(l1[1][k] - l0[1][k]) / abs(l0[1][k]), abs(l1[2][k] - l0[2][k]) / abs(l0[2][k]))
        si = max(si, abs(l1[3][k] - l0[3][k]) / max(l0[3][k], 1e-12))
    sp = 0.0 if tie else _pose_err(r1["T"], r0["T"])
    return sr, si, sp


def _lm_divergence(lg, lo, spread=(0.0, 0.0, 0.0)):
    """Walk the two LM logs (level, resNew/N, resOld/N, |inc|) in lockstep.  Until the trajectories part, every
    operand agrees to fp32-summation-order precision; they may only part at a decision that is a near-tie in
    the oracle itself (accept: resNew/N vs resOld/N, break: |inc| vs 1e-3) or at a step from a near-singular
    system (|inc| > 1).  Returns the index of that decision, or None when the logs are identical in length and
    decisions."""
    lvg, ng, og, ig = lg
    lvo, no, oo, io = lo
    # tied to the oracle's own spread, with ceilings so a run with a large spread cannot quietly loosen the check
    tr, ti = min(max(1e-4, 10 * spread[0]), 1e-3), min(max(1e-3, 10 * spread[1]), 3e-2)
    print(f"LM bars: ratios {tr:.2e}, step norms {ti:.2e} (oracle order spread {spread[0]:.2e}, {spread[1]:.2e})")
    for k in range(min(len(lvg), len(lvo))):
        assert lvg[k] == lvo[k], k
        assert abs(ng[k] - no[k]) <= tr * abs(no[k]), (k, ng[k], no[k], tr)
        assert abs(og[k] - oo[k]) <= tr * abs(oo[k]), (k, og[k], oo[k], tr)
        if io[k] > 1.0:   # a step of > 1 (scaled units) comes from a near-singular H: fp order decides the rest
            return k
        assert abs(ig[k] - io[k]) <= ti * io[k] + 1e-7, (k, ig[k], io[k], ti)
        if (ng[k] < og[k]) != (no[k] < oo[k]):
            assert abs(no[k] - oo[k]) <= 2 * tr * oo[k], ("accept flip without a tie", k)
            return k
        if (ig[k] > 1e-3) != (io[k] > 1e-3):
            assert abs(io[k] - 1e-3) <= 1e-6, ("break flip without a tie", k)
            return k
    assert len(lvg) == len(lvo)
    return None


@pytest.mark.parametrize("start", ["identity", "near"])
def test_track_parity(vga, pair, start):
    from hslam_amd.se3 import SE3
    g, o = pair
    g.set_event_timing(True)  # last_ms below (off by default: the done-word path)
    T0 = SE3().data() if start == "identity" else (SE3.exp([0.002, 0, -0.001, 0, 0.001, 0]) *
                                                   SE3.from_data(vga.T_true)).data()
    minRes = np.full(5, np.nan)
    okg, Tg, ag = g.trackNewestCoarse(T0, [0.0, 0.0], vga.n_levels - 1, minRes)
    spread = _order_spread(o, T0, [0.0, 0.0], vga.n_levels - 1, minRes)
    ro = o.track(T0, [0.0, 0.0], vga.n_levels - 1, minRes)
    assert okg == ro["ok"] and okg
    k = _lm_divergence(g.lm_log(0), o.lm_log(), spread)
    tol_T, tol_a, tol_b = (min(max(1e-5, 10 * spread[2]), 1e-4), 1e-5, 1e-3) if k is None else (2e-3, 1e-2, 0.5)
    print(f"pose bar {tol_T:.2e} (oracle order spread {spread[2]:.2e}), first near-tie {k}")
    assert _pose_err(Tg, ro["T"]) < tol_T, k
    assert abs(ag[0] - ro["aff"][0]) < tol_a and abs(ag[1] - ro["aff"][1]) < tol_b, k
    lr = g.lastResiduals
    fin = np.isfinite(ro["lastResiduals"])
    assert np.array_equal(np.isfinite(lr), fin)
    assert np.allclose(lr[fin], ro["lastResiduals"][fin], rtol=1e-4 if k is None else 1e-2)
    assert _pose_err(Tg, vga.T_true) < 3e-3
    assert g.last_ms() > 0


def test_track_abort_parity(vga, pair):
    from hslam_amd.se3 import SE3
    g, o = pair
    T0 = SE3().data()
    minRes = np.full(5, 1e-3)
    okg, Tg, ag = g.trackNewestCoarse(T0, [0.0, 0.0], vga.n_levels - 1, minRes)
    ro = o.track(T0, [0.0, 0.0], vga.n_levels - 1, minRes)
    assert not okg and not ro["ok"]
    assert np.array_equal(Tg, T0) and np.array_equal(Tg, ro["T"])
    assert np.array_equal(np.isfinite(g.lastResiduals), np.isfinite(ro["lastResiduals"]))


def test_track_tries_parity(vga, pair):
    from hslam_amd.se3 import SE3
    from hslam_amd.track import motion_hypotheses, trackNewCoarse
    g, o = pair
    # hypotheses around a last-frame motion that is half the true one
    half = SE3.exp(SE3.from_data(vga.T_true).log() * 0.5)
    lastF = SE3()
    slast = half.inverse()
    sprelast = (half * half).inverse()
    tries = motion_hypotheses(lastF, slast, sprelast)
    tries = np.concatenate([SE3.exp([0, 0, 0, 0.3, -0.25, 0.2]).data()[None], tries])  # a hopeless first try
    for rmse in (np.full(5, 100.0), np.full(5, 1e-6)):
        og = trackNewCoarse(g, tries, [0.0, 0.0], rmse)
        oo = o.track_tries(tries, [0.0, 0.0], rmse)
        assert og["haveOneGood"] == oo["haveOneGood"]
        assert og["tryIterations"] == oo["tryIterations"]
        assert _pose_err(og["T"], oo["T"]) < 2e-3
        fin = np.isfinite(oo["achievedRes"])
        assert np.array_equal(np.isfinite(og["achievedRes"]), fin)
        assert np.allclose(og["achievedRes"][fin], oo["achievedRes"][fin], rtol=1e-2)
    # every hypothesis' own LM run agrees with the oracle's run of that hypothesis up to a near-tie
    for i in (0, 1, 5, 17, len(tries) - 1):
        spread = _order_spread(o, tries[i], [0.0, 0.0], vga.n_levels - 1, np.full(5, np.nan))
        _lm_divergence(g.lm_log(i), o.lm_log(), spread)


def test_errors_are_loud(vga):
    from hslam_amd._lib import HsError
    from hslam_amd.se3 import SE3
    from hslam_amd.track import CoarseTracker
    g = CoarseTracker(vga.width, vga.height, vga.K4, vga.n_levels)
    with pytest.raises(HsError):
        g.calcRes(0, SE3().data(), [0, 0], 20.0)        # no reference / frame yet
    g.set_scene(vga)
    with pytest.raises(HsError):
        g.trackNewestCoarse(SE3().data(), [0, 0], 5, np.full(5, np.nan))   # coarsest must be < 5
    with pytest.raises(HsError):
        CoarseTracker(vga.width, vga.height, vga.K4, 7)


@pytest.fixture(scope="module")
def vga4():
    """640x480 with the reference's own level rule (Include/CalibData.h:110-115 gives 4 levels here)."""
    from hslam_amd.scene import make_track_scene
    return make_track_scene(n_points=2000, n_levels=4)


@pytest.mark.parametrize("start", ["identity", "near"])
def test_track_parity_4_levels(vga4, start):
    """trackNewestCoarse on the 4-level pyramid: the LM log agrees with the oracle's up to a near-tie, then the
    final pose / affine / lastResiduals at the bars of the module docstring."""
    from hslam_amd.se3 import SE3
    from hslam_amd.track import CoarseTracker
    from oracle_ffi import OracleTracker
    g = CoarseTracker(vga4.width, vga4.height, vga4.K4, vga4.n_levels)
    g.set_event_timing(True)  # last_stats' device time below
    g.set_scene(vga4)
    o = OracleTracker(vga4.width, vga4.height, vga4.K4, vga4.n_levels)
    o.set_scene(vga4)
    T0 = SE3().data() if start == "identity" else (SE3.exp([0.002, 0, -0.001, 0, 0.001, 0]) *
                                                   SE3.from_data(vga4.T_true)).data()
    minRes = np.full(5, np.nan)
    okg, Tg, ag = g.trackNewestCoarse(T0, [0.0, 0.0], vga4.n_levels - 1, minRes)
    spread = _order_spread(o, T0, [0.0, 0.0], vga4.n_levels - 1, minRes)
    ro = o.track(T0, [0.0, 0.0], vga4.n_levels - 1, minRes)
    assert okg == ro["ok"] and okg
    k = _lm_divergence(g.lm_log(0), o.lm_log(), spread)
    tol_T, tol_a, tol_b = (min(max(1e-5, 10 * spread[2]), 1e-4), 1e-5, 1e-3) if k is None else (2e-3, 1e-2, 0.5)
    print(f"pose bar {tol_T:.2e} (oracle order spread {spread[2]:.2e}), first near-tie {k}")
    assert _pose_err(Tg, ro["T"]) < tol_T, k
    assert abs(ag[0] - ro["aff"][0]) < tol_a and abs(ag[1] - ro["aff"][1]) < tol_b, k
    lr = g.lastResiduals
    fin = np.isfinite(ro["lastResiduals"])
    assert np.array_equal(np.isfinite(lr), fin)
    assert np.allclose(lr[fin], ro["lastResiduals"][fin], rtol=1e-4 if k is None else 1e-2)
    # the roofline's work counters: one pass per LM iteration plus >= one calcRes per level
    ms, passes, point_passes = g.last_stats(0)
    lv = g.lm_log(0)[0]
    assert passes >= len(lv) + vga4.n_levels
    pcn = [len(g.pc(l)["u"]) for l in range(vga4.n_levels)]
    assert sum(pcn[l] * int((lv == l).sum()) for l in range(vga4.n_levels)) + sum(pcn) <= point_passes
    assert ms > 0
    g.close()


@pytest.mark.parametrize("noevt", ["0", "1"])
def test_member_meeting_timeout_falls_back_to_one_workgroup(vga, monkeypatch, noevt):
    """The G member workgroups of a hypothesis meet once per pass and must be co-resident.  With the meeting's poll
    bound forced to one poll (HS_TRK_SPIN=1) and G past the co-residency cap (HS_TRK_G_UNCHECKED=16), meetings time
    out; the launch is then rerun with G = 1 and the track is the one-workgroup track, bit for bit.  noevt = 1: the
    host takes the results from the leads' done words instead of the stream's end (HS_TRK_NOEVT; the default)."""
    from hslam_amd.se3 import SE3
    monkeypatch.setenv("HS_TRK_NOEVT", noevt)
    from hslam_amd.track import CoarseTracker
    T0 = SE3().data()
    minRes = np.full(5, np.nan)
    g1 = CoarseTracker(vga.width, vga.height, vga.K4, vga.n_levels)
    g1.set_scene(vga)
    monkeypatch.setenv("HS_TRK_G", "1")
    ok1, T1, a1 = g1.trackNewestCoarse(T0, [0.0, 0.0], vga.n_levels - 1, minRes)
    assert g1.launch_info() == (1, 0)
    monkeypatch.delenv("HS_TRK_G")
    g2 = CoarseTracker(vga.width, vga.height, vga.K4, vga.n_levels)
    g2.set_scene(vga)
    monkeypatch.setenv("HS_TRK_SPIN", "1")
    monkeypatch.setenv("HS_TRK_G_UNCHECKED", "16")
    ok2, T2, a2 = g2.trackNewestCoarse(T0, [0.0, 0.0], vga.n_levels - 1, minRes)
    G, fallbacks = g2.launch_info()
    assert fallbacks >= 1 and G == 1
    assert ok1 == ok2 and np.array_equal(T1, T2) and np.array_equal(a1, a2)
    assert np.array_equal(g1.lastResiduals, g2.lastResiduals, equal_nan=True)
    monkeypatch.delenv("HS_TRK_SPIN")
    monkeypatch.delenv("HS_TRK_G_UNCHECKED")
    ok3, T3, a3 = g2.trackNewestCoarse(T0, [0.0, 0.0], vga.n_levels - 1, minRes)  # co-resident again: G > 1
    assert g2.launch_info()[0] > 1 and g2.launch_info()[1] == fallbacks and ok3
    g1.close()
    g2.close()


def test_done_word_results_match_synchronized(vga):
    """HS_TRK_NOEVT=1 (no event pair, the library default): the host reads each hypothesis' record once its lead's done word (a system-scope
    release after the record) shows the launch, without waiting for the launch's end.  Tracks and try sequences
    bit-identical to the synchronized path, over repeated calls (the done words carry a per-launch sequence number)."""
    from hslam_amd.se3 import SE3
    from hslam_amd.track import CoarseTracker
    T0 = SE3().data()
    minRes = np.full(5, np.nan)
    outs = {}
    for mode in ("0", "1"):
        os.environ["HS_TRK_NOEVT"] = mode
        try:
            g = CoarseTracker(vga.width, vga.height, vga.K4, vga.n_levels)
            g.set_scene(vga)
            runs = []
            for _ in range(3):
                ok, T, a = g.trackNewestCoarse(T0, [0.0, 0.0], vga.n_levels - 1, minRes)
                runs.append((ok, T, a, g.lastResiduals.copy()))
            tr = g.track_tries([T0, T0], [0.0, 0.0], np.full(5, np.nan))
            runs.append(tr)
            g.close()
        finally:
            os.environ.pop("HS_TRK_NOEVT", None)
        outs[mode] = runs
    for r0, r1 in zip(outs["0"][:3], outs["1"][:3]):
        assert r0[0] == r1[0] and np.array_equal(r0[1], r1[1]) and np.array_equal(r0[2], r1[2])
        assert np.array_equal(r0[3], r1[3], equal_nan=True)
    t0, t1 = outs["0"][3], outs["1"][3]
    assert np.array_equal(t0["T"], t1["T"]) and t0["tryIterations"] == t1["tryIterations"]
