"""CPU tests of the CoarseTracker oracle (oracle/track_oracle.cpp) and the tracker host logic.

* makeCoarseDepthL0 is checked bit-exact against an independent numpy restatement of
  Src/CoarseTracker.cpp:105-263 (scatter in point order, 2x2 sums, dilation, normalise + raster compaction);
* calcRes / calcGSSSE: structural properties (H symmetric PSD, energy minimal near the true motion);
* trackNewestCoarse converges to the rendered motion; the try loop's take-over / fallback rules;
* the host SE3 (hslam_amd/se3.py) used for System::trackNewCoarse's hypotheses agrees with the oracle's.
"""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def tscene():
    from hslam_amd.scene import make_track_scene
    return make_track_scene(n_points=600, width=320, height=240, K=np.array([[128.0, 0, 159.5], [0, 127.2, 119.5],
                                                                            [0, 0, 1.0]]), n_levels=4)


@pytest.fixture(scope="module")
def otrk(tscene):
    from oracle_ffi import OracleTracker
    t = OracleTracker(tscene.width, tscene.height, tscene.K4, tscene.n_levels)
    t.set_scene(tscene)
    return t


def np_make_coarse_depth(s):
    """Independent numpy restatement of makeCoarseDepthL0 (Src/CoarseTracker.cpp:105-263), float32 op order."""
    f32 = np.float32
    L = s.n_levels
    w = [s.width >> l for l in range(L)]
    h = [s.height >> l for l in range(L)]
    idp = [np.zeros(w[l] * h[l], f32) for l in range(L)]
    ws = [np.zeros(w[l] * h[l], f32) for l in range(L)]
    u = (s.pt_u + f32(0.5)).astype(np.int64)
    v = (s.pt_v + f32(0.5)).astype(np.int64)
    wt = np.sqrt((1e-3 / (s.pt_hdi.astype(np.float64) + 1e-12)).astype(f32))
    idx = u + w[0] * v
    np.add.at(idp[0], idx, s.pt_idepth * wt)   # unbuffered: sequential in point order
    np.add.at(ws[0], idx, wt)
    for l in range(1, L):
        a = idp[l - 1].reshape(h[l - 1], w[l - 1])
        b = ws[l - 1].reshape(h[l - 1], w[l - 1])
        for src, dst in ((a, idp), (b, ws)):
            q = src[: 2 * h[l], : 2 * w[l]]
            dst[l] = (((q[0::2, 0::2] + q[0::2, 1::2]) + q[1::2, 0::2]) + q[1::2, 1::2]).reshape(-1).astype(f32)
    for l in range(L):
        wl = w[l]
        bak = ws[l].copy()
        i = np.arange(wl, w[l] * h[l] - wl)
        nb = [1 + wl, -1 - wl, wl - 1, -wl + 1] if l < 2 else [1, -1, wl, -wl]
        todo = bak[i] <= 0
        sm = np.zeros(len(i), f32)
        num = np.zeros(len(i), f32)
        numn = np.zeros(len(i), f32)
        for d in nb:
            j = np.clip(i + d, 0, len(bak) - 1)
            c = (bak[j] > 0) & (i + d >= 0) & (i + d < len(bak))   # out-of-range neighbours: empty
            sm = np.where(c, sm + idp[l][j], sm).astype(f32)
            num = np.where(c, num + bak[j], num).astype(f32)
            numn = np.where(c, numn + f32(1), numn).astype(f32)
        upd = todo & (numn > 0)
        with np.errstate(invalid="ignore", divide="ignore"):
            idp[l][i[upd]] = (sm / numn)[upd]
            ws[l][i[upd]] = (num / numn)[upd]
    out = []
    for l in range(L):
        wl, hl = w[l], h[l]
        ys, xs = np.meshgrid(np.arange(2, hl - 2), np.arange(2, wl - 2), indexing="ij")
        ii = (xs + ys * wl).reshape(-1)
        sel = ii[ws[l][ii] > 0]
        with np.errstate(invalid="ignore", divide="ignore"):
            nid = (idp[l][sel] / ws[l][sel]).astype(f32)
        col = s.ref_pyr[l].reshape(-1, 3)[sel, 0]
        keep = np.isfinite(col) & (nid > 0)
        out.append(dict(u=(sel % wl)[keep].astype(f32), v=(sel // wl)[keep].astype(f32), idepth=nid[keep],
                        color=col[keep]))
    return out


def test_make_coarse_depth_bit_exact_vs_numpy(tscene, otrk):
    ref = np_make_coarse_depth(tscene)
    for l in range(tscene.n_levels):
        pc = otrk.pc(l)
        assert len(pc["u"]) > 0
        for k in ("u", "v", "idepth", "color"):
            assert np.array_equal(pc[k], ref[l][k]), (l, k)


def test_make_coarse_depth_raster_order(tscene, otrk):
    for l in range(tscene.n_levels):
        pc = otrk.pc(l)
        wl = tscene.width >> l
        lin = pc["v"].astype(np.int64) * wl + pc["u"].astype(np.int64)
        assert np.all(np.diff(lin) > 0)
        assert np.all(pc["idepth"] > 0)


def test_duplicates_scatter_accumulate(tscene):
    from hslam_amd.scene import make_track_scene
    s = make_track_scene(n_points=300, width=160, height=120, dup_frac=0.3, n_levels=3,
                         K=np.array([[64.0, 0, 79.5], [0, 63.6, 59.5], [0, 0, 1.0]]))
    pix = (s.pt_u + np.float32(0.5)).astype(int) + 160 * (s.pt_v + np.float32(0.5)).astype(int)
    assert len(np.unique(pix)) < len(pix)  # the case exercises shared pixels
    from oracle_ffi import OracleTracker
    t = OracleTracker(s.width, s.height, s.K4, s.n_levels)
    t.set_scene(s)
    ref = np_make_coarse_depth(s)
    for l in range(s.n_levels):
        pc = t.pc(l)
        for k in ("u", "v", "idepth", "color"):
            assert np.array_equal(pc[k], ref[l][k]), (l, k)


def test_calc_res_structure(tscene, otrk):
    from hslam_amd.se3 import SE3
    cut = otrk.params.coarseCutoffTH
    for lvl in range(tscene.n_levels):
        res_t, H, b, nw = otrk.calc_res(lvl, tscene.T_true, tscene.aff_true, cut)
        n_sat = round(res_t[5] * res_t[1])   # saturated residuals count in E but are not warped
        assert nw % 4 == 0 and res_t[1] - n_sat <= nw <= res_t[1] - n_sat + 3
        assert np.allclose(H, H.T, rtol=1e-12, atol=0)
        ev = np.linalg.eigvalsh(H)
        assert ev.min() > -1e-6 * ev.max()
        res_0, *_ = otrk.calc_res(lvl, SE3().data(), [0.0, 0.0], cut)
        assert res_t[0] / res_t[1] < res_0[0] / res_0[1]
    # flow indicators vanish at identity
    r, *_ = otrk.calc_res(0, SE3().data(), [0.0, 0.0], cut)
    assert abs(r[2]) < 1e-6 and abs(r[4]) < 1e-6


def test_track_converges(tscene, otrk):
    from hslam_amd.se3 import SE3
    out = otrk.track(SE3().data(), [0.0, 0.0], tscene.n_levels - 1, np.full(5, np.nan))
    assert out["ok"]
    err = (SE3.from_data(out["T"]) * SE3.from_data(tscene.T_true).inverse()).log()
    assert np.linalg.norm(err[3:]) < 2e-3 and np.linalg.norm(err[:3]) < 3e-3
    assert np.all(np.isfinite(out["lastResiduals"][: tscene.n_levels]))
    assert np.all(np.isnan(out["lastResiduals"][tscene.n_levels:]))


def test_sum_order_spread_is_rounding_level(tscene, otrk):
    """The order-spread hook the GPU LM bars are tied to (tests/test_gpu_track.py): with every calcRes /
    calcGSSSE sum formed in reversed point order the per-point decisions are unchanged, the calcRes energy and the
    normal equations move at fp32 summation-order level only, and the LM run still converges to the same pose."""
    from hslam_amd.se3 import SE3
    T = SE3.exp([0.004, -0.003, 0.002, 0.002, 0.001, -0.002]) * SE3.from_data(tscene.T_true)
    r0 = otrk.calc_res(0, T.data(), [0.0, 0.0], 20.0)
    otrk.set_sum_order(1)
    try:
        r1 = otrk.calc_res(0, T.data(), [0.0, 0.0], 20.0)
        out1 = otrk.track(SE3().data(), [0.0, 0.0], tscene.n_levels - 1, np.full(5, np.nan))
    finally:
        otrk.set_sum_order(0)
    out0 = otrk.track(SE3().data(), [0.0, 0.0], tscene.n_levels - 1, np.full(5, np.nan))
    assert r1[3] == r0[3] and r1[0][1] == r0[0][1]            # warped count, numTermsInE
    assert r1[0][0] != r0[0][0] or not np.array_equal(r1[1], r0[1])  # another order: other roundings
    assert abs(r1[0][0] - r0[0][0]) <= 1e-5 * abs(r0[0][0])
    assert np.allclose(r1[1], r0[1], rtol=1e-4, atol=1e-6 * np.abs(r0[1]).max())
    err = (SE3.from_data(out1["T"]) * SE3.from_data(out0["T"]).inverse()).log()
    assert out1["ok"] and np.linalg.norm(err) < 1e-4


def test_track_abort_keeps_inputs(tscene, otrk):
    from hslam_amd.se3 import SE3
    T0 = SE3().data()
    out = otrk.track(T0, [0.0, 0.0], tscene.n_levels - 1, np.full(5, 1e-3))  # impossible bound: aborts at coarsest
    assert not out["ok"]
    assert np.array_equal(out["T"], T0) and np.array_equal(out["aff"], [0.0, 0.0])
    lr = out["lastResiduals"]
    assert np.isfinite(lr[tscene.n_levels - 1]) and np.all(np.isnan(lr[: tscene.n_levels - 1]))


def test_track_tries_takeover_and_break(tscene, otrk):
    from hslam_amd.se3 import SE3
    bad = SE3.exp([0.0, 0.0, 0.0, 0.25, -0.2, 0.3]).data()   # far off: fails / worse
    good = SE3().data()
    tries = np.stack([bad, good, good, good])
    out = otrk.track_tries(tries, [0.0, 0.0], np.full(5, 100.0))
    assert out["haveOneGood"]
    # with lastCoarseRMSE large the loop breaks right after the first good try
    assert out["tryIterations"] <= 2
    err = (SE3.from_data(out["T"]) * SE3.from_data(tscene.T_true).inverse()).log()
    assert np.linalg.norm(err) < 5e-3
    # lastCoarseRMSE tiny: all tries run
    out2 = otrk.track_tries(tries, [0.0, 0.0], np.full(5, 1e-6))
    assert out2["tryIterations"] == 4 and out2["haveOneGood"]


def test_track_tries_none_good_fallback(tscene):
    from hslam_amd.se3 import SE3
    from oracle_ffi import OracleTracker
    t = OracleTracker(tscene.width, tscene.height, tscene.K4, tscene.n_levels)
    t.set_scene(tscene)
    assert t.params.affineOptModeA != 0   # default 1e12: |a| > 1.2 fails the sanity check (CoarseTracker.cpp:667)
    # a 30x exposure ratio drives a to about -log(30) on every try: no try is good
    t.set_frame(tscene.new_pyr, 30.0)
    tries = np.stack([SE3().data(), SE3.exp([0.01, 0, 0, 0, 0, 0]).data()])
    out = t.track_tries(tries, [0.0, 0.0], np.full(5, 1.0))
    assert not out["haveOneGood"] and out["tryIterations"] == 2
    assert np.array_equal(out["T"], tries[0]) and np.array_equal(out["flowVecs"], [0, 0, 0])
    assert np.array_equal(out["aff"], [0.0, 0.0])
    assert np.all(np.isnan(out["achievedRes"]))


def test_host_se3_matches_oracle():
    import oracle_ffi as O
    from hslam_amd.se3 import SE3
    rng = np.random.default_rng(3)
    for _ in range(20):
        a = rng.normal(size=6) * np.array([0.3, 0.3, 0.3, 0.5, 0.5, 0.5])
        b = rng.normal(size=6) * 0.2
        A, B = SE3.exp(a), SE3.exp(b)
        assert np.allclose(A.data(), O.se3_exp(a), atol=1e-14)
        assert np.allclose(A.log(), O.se3_log(A.data()), atol=1e-12)
        assert np.allclose((A * B).data(), O.se3_mul(A.data(), B.data()), atol=1e-14)
        assert np.allclose(A.inverse().data(), O.se3_inverse(A.data()), atol=1e-14)


def test_motion_hypotheses():
    from hslam_amd.se3 import SE3
    from hslam_amd.track import motion_hypotheses
    lastF = SE3.exp([0.1, 0, 0, 0, 0.01, 0])
    slast = SE3.exp([0.15, 0, 0.01, 0, 0.012, 0])
    sprelast = SE3.exp([0.2, 0.0, 0.02, 0, 0.014, 0])
    tr = motion_hypotheses(lastF, slast, sprelast)
    assert tr.shape == (31, 7)
    assert np.allclose(tr[4], SE3().data())
    lastF_2_slast = slast.inverse() * lastF
    assert np.allclose(tr[3], lastF_2_slast.data())
    const = (sprelast.inverse() * slast).inverse() * lastF_2_slast
    assert np.allclose(tr[0], const.data())
    # jitters: rotation about +x by 2*atan(0.02) composed on the right of the constant-motion guess
    j = SE3.from_data(const.inverse().data()) * SE3.from_data(tr[5])
    assert np.allclose(j.log()[3:], [2 * np.arctan(np.float32(0.02)), 0, 0], atol=1e-12)
    assert np.allclose(j.log()[:3], 0, atol=1e-12)
    assert motion_hypotheses(lastF, slast, sprelast, poses_valid=False).shape == (1, 7)
