"""Frame::CreateDirPyrs (Src/Frame.cpp:104-181): the oracle restatement, the device kernels and the contexts' raw
frame entries.  Bar: bit-exact (the pyramid is elementwise fp32 arithmetic in the reference's operation order)."""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def raw():
    from hslam_amd.scene import make_track_scene
    s = make_track_scene(n_points=400, width=320, height=240, n_levels=4,
                         K=np.array([[128.0, 0, 159.5], [0, 127.2, 119.5], [0, 0, 1.0]]))
    return s


def test_oracle_matches_scene_pyramid(raw):
    """The oracle restatement against the numpy generator the scenes use (hslam_amd.scene.make_dir_pyramid)."""
    from hslam_amd.scene import make_dir_pyramid
    from oracle_ffi import dir_pyramid
    img = raw.new_pyr[0][..., 0]
    po, go = dir_pyramid(img, 4)
    pn = make_dir_pyramid(img, 4)
    for l in range(4):
        assert np.array_equal(po[l], pn[l]), l
        g = po[l][..., 1] ** 2 + po[l][..., 2] ** 2
        assert np.array_equal(go[l], g.astype(np.float32)), l


def test_oracle_nonfinite_gradients_are_zero():
    from oracle_ffi import dir_pyramid
    img = np.full((16, 24), 7.0, np.float32)
    img[5, 6] = np.inf
    p, _ = dir_pyramid(img, 2)
    assert np.all(np.isfinite(p[0][..., 1:])) and np.isinf(p[0][5, 6, 0])


@pytest.mark.gpu
def test_device_pyramid_bit_exact(raw):
    from hslam_amd.pyr import dir_pyramid as dev
    from oracle_ffi import dir_pyramid
    for img in (raw.new_pyr[0][..., 0], raw.ref_pyr[0][..., 0]):
        pg, gg = dev(img, 4)
        po, go = dir_pyramid(img, 4)
        for l in range(4):
            assert np.array_equal(pg[l], po[l]), l
            assert np.array_equal(gg[l], go[l]), l


@pytest.mark.gpu
def test_tracker_raw_frame_matches_host_pyramid(raw):
    from hslam_amd.track import CoarseTracker
    a = CoarseTracker(raw.width, raw.height, raw.K4, raw.n_levels)
    a.set_scene(raw)
    b = CoarseTracker(raw.width, raw.height, raw.K4, raw.n_levels)
    b.setCoarseTrackingRef(raw.ref_pyr, raw.ref_exposure, raw.ref_aff, raw.pt_u, raw.pt_v, raw.pt_idepth, raw.pt_hdi)
    b.setNewFrameRaw(raw.new_pyr[0][..., 0], raw.new_exposure)
    for lvl in range(raw.n_levels):
        ra, _, _, na = a.calcRes(lvl, raw.T_true, raw.aff_true, 20.0)
        rb, _, _, nb = b.calcRes(lvl, raw.T_true, raw.aff_true, 20.0)
        assert na == nb and np.array_equal(ra, rb), lvl


@pytest.mark.gpu
def test_tracer_raw_frame_matches_host_image():
    from hslam_amd.scene import make_trace_scene
    from hslam_amd.trace import ImmatureTracer
    s = make_trace_scene(n_points=500, n_hosts=4, width=320, height=240, seed=9)
    a = ImmatureTracer(s.width, s.height, s.n_points)
    a.set_scene(s)
    b = ImmatureTracer(s.width, s.height, s.n_points)
    for i, im in enumerate(s.host_imgs):
        b.set_host_image(i, im)
    b.add_points(s.pt_host, s.pt_u, s.pt_v)
    b.set_frame_raw(s.new_img[..., 0])
    assert np.array_equal(a.traceNewCoarse(s.KRKi, s.Kt, s.aff), b.traceNewCoarse(s.KRKi, s.Kt, s.aff))
    pa, pb = a.points(), b.points()
    for k in pa:
        assert np.array_equal(pa[k], pb[k], equal_nan=True), k
