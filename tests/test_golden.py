"""Golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py from the CPU restatement).

The reference ships no vectors for this path, so the fixtures are oracle outputs on seeded
synthetic scenes: 'parity unpinned' against the reference itself.  CPU tests: the scene generator still
produces the fixture's inputs (SHA-256 digest) and the oracle reproduces every stored output bit for bit.
GPU tests: the HIP path matches the stored outputs at the parity bars of tests/test_gpu_*.py.
"""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_golden as mg  # noqa: E402


def _load(name):
    return np.load(os.path.join(HERE, "golden", name))


def _eq(a, b):
    return np.array_equal(np.asarray(a), np.asarray(b), equal_nan=True)


@pytest.fixture(scope="module")
def scenes():
    return dict(pair=mg.scene_ba_pair64(), w8=mg.scene_ba_8x200(), track=mg.scene_track160(), trace=mg.scene_trace100(),
                refine=mg.scene_refine300())


# ------------------------------------------------------------------------------------------------ CPU
def test_fixture_inputs_unchanged(scenes):
    assert str(_load("ba_pair64.npz")["digest"]) == mg.ba_scene_digest(scenes["pair"])
    assert str(_load("ba_8x200.npz")["digest"]) == mg.ba_scene_digest(scenes["w8"])
    assert str(_load("track_160.npz")["digest"]) == mg.track_scene_digest(scenes["track"])
    assert str(_load("trace_100.npz")["digest"]) == mg.trace_scene_digest(scenes["trace"])
    assert str(_load("refine_300.npz")["digest"]) == mg.refine_scene_digest(scenes["refine"])


def test_oracle_reproduces_refine_fixture(scenes):
    g = _load("refine_300.npz")
    out = mg.refine_outputs(scenes["refine"])
    for k, v in out.items():
        assert _eq(v, g[k]), k


@pytest.mark.parametrize("name,key", [("ba_pair64.npz", "pair"), ("ba_8x200.npz", "w8")])
def test_oracle_reproduces_ba_fixture(name, key, scenes):
    from oracle_ffi import OracleBA
    g = _load(name)
    out = mg.ba_outputs(OracleBA(scenes[key]))
    for k, v in out.items():
        assert _eq(v, g[k]), (name, k)
    if "E_iters" in g:
        o = OracleBA(scenes[key])
        o.linearize_all(reset=True)
        o.apply_res()
        assert _eq(o.iterate(0, len(g["E_iters"])), g["E_iters"])


def test_oracle_reproduces_track_fixture(scenes):
    from oracle_ffi import OracleTracker
    s, g = scenes["track"], _load("track_160.npz")
    o = OracleTracker(s.width, s.height, s.K4, s.n_levels)
    o.set_scene(s)
    for l in range(s.n_levels):
        for k, v in o.pc(l).items():
            assert _eq(v, g[f"pc{l}_{k}"]), (l, k)
    res6, H, b, nw = o.calc_res(0, s.T_true, s.aff_true, 20.0)
    assert _eq(res6, g["calc_res6"]) and _eq(H, g["calc_H"]) and _eq(b, g["calc_b"]) and nw == g["calc_nwarped"]
    t = o.track(np.array([0, 0, 0, 1.0, 0, 0, 0]), [0.0, 0.0], s.n_levels - 1, np.full(5, np.nan))
    assert t["ok"] == bool(g["track_ok"]) and _eq(t["T"], g["track_T"]) and _eq(t["lastResiduals"], g["track_lastResiduals"])


def test_oracle_reproduces_trace_fixture(scenes):
    from oracle_ffi import OracleTracer
    s, g = scenes["trace"], _load("trace_100.npz")
    o = OracleTracer(s.width, s.height)
    o.set_scene(s)
    for k, v in o.points().items():
        assert _eq(v, g["ctor_" + k]), k
    for rnd in (1, 2):
        assert _eq(o.trace(s.new_img, s.KRKi, s.Kt, s.aff), g[f"counts{rnd}"])
        p = o.points()
        for k in ("status", "idepth_min", "idepth_max", "quality", "uv", "interval"):
            assert _eq(p[k], g[f"trace{rnd}_{k}"]), (rnd, k)


# ------------------------------------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("name,key", [("ba_pair64.npz", "pair"), ("ba_8x200.npz", "w8")])
def test_gpu_matches_ba_fixture(name, key, scenes):
    import os as _os
    from hslam_amd.ba import BAWindow
    from test_gpu_ba import _close_H, _close_b
    g = _load(name)
    _os.environ["HS_ACC_EXACT"] = "1"
    try:
        w = BAWindow(scenes[key])
    finally:
        _os.environ.pop("HS_ACC_EXACT", None)
    E0 = w.linearizeAll(reset=True)
    r = w.residuals()
    act = g["res_state"] == 0
    assert _eq(r["state"], g["res_state"]) and _eq(r["energy"], g["res_energy"])
    assert _eq(r["energy_wo"], g["res_energy_wo"])
    assert _eq(r["JpJdF"][act], g["res_JpJdF"][act]) and _eq(r["center"][act], g["res_center"][act])
    assert abs(E0 - float(g["E0"])) <= 1e-9 * abs(float(g["E0"]))
    assert _eq(w.frames()["energyTH"], g["energyTH"])
    for which, nm in ((0, "A"), (1, "L"), (2, "SC")):
        H, b = w.system(which)
        assert _close_H(H, g["H" + nm])[0] and _close_b(b, g["b" + nm], g["H" + nm])[0], nm
    x = w.solveSystem(0)
    assert np.linalg.norm(x - g["x0"]) <= 1e-3 * np.linalg.norm(g["x0"])
    if "E_iters" in g:
        w2 = BAWindow(scenes[key])
        w2.linearizeAll(reset=True)
        E = w2.iterate(0, len(g["E_iters"]))
        np.testing.assert_allclose(E, g["E_iters"], rtol=1e-3)


@pytest.mark.gpu
def test_gpu_matches_track_fixture(scenes):
    from hslam_amd.track import CoarseTracker
    s, g = scenes["track"], _load("track_160.npz")
    ct = CoarseTracker(s.width, s.height, s.K4, s.n_levels)
    ct.set_scene(s)
    for l in range(s.n_levels):
        for k, v in ct.pc(l).items():
            assert _eq(v, g[f"pc{l}_{k}"]), (l, k)
    res6, H, b, nw = ct.calcRes(0, s.T_true, s.aff_true, 20.0)
    r = g["calc_res6"]
    assert nw == int(g["calc_nwarped"]) and res6[1] == r[1] and abs(res6[0] - r[0]) <= 2e-5 * abs(r[0])
    ok, T, a = ct.trackNewestCoarse(np.array([0, 0, 0, 1.0, 0, 0, 0]), [0.0, 0.0], s.n_levels - 1, np.full(5, np.nan))
    assert ok == bool(g["track_ok"])
    np.testing.assert_allclose(T, g["track_T"], atol=2e-3)
    np.testing.assert_allclose(ct.lastResiduals, g["track_lastResiduals"], rtol=1e-2)


@pytest.mark.gpu
def test_gpu_matches_trace_fixture(scenes):
    from hslam_amd.trace import ImmatureTracer
    s, g = scenes["trace"], _load("trace_100.npz")
    t = ImmatureTracer(s.width, s.height, s.n_points)
    t.set_scene(s)
    for k, v in t.points().items():
        assert _eq(v, g["ctor_" + k]), k
    for rnd in (1, 2):
        assert _eq(t.traceNewCoarse(s.KRKi, s.Kt, s.aff), g[f"counts{rnd}"])
        p = t.points()
        for k in ("status", "idepth_min", "idepth_max", "quality", "uv", "interval"):
            assert _eq(p[k], g[f"trace{rnd}_{k}"]), (rnd, k)


@pytest.mark.gpu
def test_gpu_matches_refine_fixture(scenes):
    """per-point outputs of calcResAndGS bit-exact; H / res and the Refine trajectory at the bars of
    tests/test_gpu_refine.py"""
    from hslam_amd.refine import DirectRefinement
    s, g = scenes["refine"], _load("refine_300.npz")
    d = DirectRefinement(s)
    H, b, Hsc, bsc, res = d.calcResAndGS(s.T_init)
    p = d.points()
    good = g["calc_isGood_new"] == 1
    assert _eq(p["isGood_new"], g["calc_isGood_new"])
    for k in ("energy_new0", "energy_new1", "maxstep"):
        assert _eq(p[k], g["calc_" + k]), k
    assert _eq(p["jb_new"][good], g["calc_jb_new"][good])
    scale = 1e-4 * np.abs(np.diag(g["calc_H"])).max()
    assert np.all(np.abs(H - g["calc_H"]) <= 1e-4 * np.abs(g["calc_H"]) + scale)
    assert abs(res[0] - g["calc_res"][0]) <= 1e-5 * abs(g["calc_res"][0]) and res[1] == g["calc_res"][1]
    d.set_points(s.u, s.v, s.tri, s.z)
    T, vid, gd, it, sn = d.Refine(s.T_init)
    from hslam_amd.se3 import SE3
    err = float(np.linalg.norm((SE3.from_data(T) * SE3.from_data(g["refine_T"]).inverse()).log()))
    assert err <= 2e-3
    L = d.log()
    n = min(len(L), len(g["refine_log"]), 3)
    np.testing.assert_allclose(L[:n, [0, 1]], g["refine_log"][:n, [0, 1]], rtol=1e-4)
    d.close()
