"""The product SE3 (h-slam_amd/csrc/hs_se3.h, and the solve's doStep forms se3_exp_step / se3_mul_step) evaluated on the
device, pinned by the reference-held Sophus vectors: the element / tangent sets of
Thirdparty/Sophus/sophus/test_se3.cpp:41-90 (tests/test_oracle_se3.py holds them as data) and the properties of
Thirdparty/Sophus/sophus/tests.hpp:43-200 (exp/log round trip, adjoint, exp vs the matrix exponential, group
action), plus agreement with the oracle's SE3 and with the same header compiled for the host (the host algebra of
setAdjointsF / setPrecalcValues) at <= 1e-12.  This is the one place where reference-held data pins the product path
itself."""
import ctypes as C

import numpy as np
import pytest
from scipy.linalg import expm

import oracle_ffi as of
from test_oracle_se3 import EPS, TANGENTS, group_elements, hat, vee

pytestmark = pytest.mark.gpu

OP = dict(exp=0, exp_step=1, log=2, adj=3, mul=4, inverse=5, mul_step=6, rot=7)


def run(op, rows, device=True):
    from hslam_amd._lib import check, load
    lib = load()
    fn = lib.hs_debug_se3
    fn.argtypes = [C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
    fn.restype = C.c_int
    x = np.zeros((len(rows), 14))
    for i, r in enumerate(rows):
        r = np.concatenate([np.asarray(a, float).ravel() for a in (r if isinstance(r, tuple) else (r,))])
        x[i, : len(r)] = r
    out = np.zeros((len(rows), 36))
    check(fn(int(device), OP[op], len(rows), x.ctypes.data, out.ctypes.data))
    return out


def matrix(d):
    d = np.asarray(d, float)
    T = np.eye(4)
    T[:3, :3] = of.se3_matrix(d[:7])
    T[:3, 3] = d[4:7]
    return T


def step_tangents():
    """GN-step sized tangents for the solve's series exp (theta^2 < 1e-2) and a few past its switch."""
    rng = np.random.default_rng(4)
    ts = [rng.normal(size=6) * s for s in (1e-9, 1e-6, 1e-4, 1e-3, 1e-2, 3e-2, 5e-2)]
    ts += [np.array([0.01, -0.02, 0.03, 0.0577, 0.0577, 0.0577]),  # theta^2 just below 1e-2
           np.array([0.01, -0.02, 0.03, 0.058, 0.058, 0.058])]     # just above: the reference formulas
    return ts + list(TANGENTS)


def test_device_exp_matches_oracle_and_expm():
    xs = list(TANGENTS) + step_tangents()
    dev = run("exp", xs)
    for x, d in zip(xs, dev):
        o = of.se3_exp(x)
        assert np.abs(d[:7] - o).max() <= 1e-12 * max(1.0, np.abs(o).max()), x
        E = expm(hat(x))
        assert np.linalg.norm(matrix(d) - E) <= 10 * EPS * max(1.0, np.linalg.norm(E))  # tests.hpp expMapTest


def test_series_step_exp_matches_sophus_exp():
    xs = step_tangents()
    ser = run("exp_step", xs)
    ref = run("exp", xs)
    for x, s, r in zip(xs, ser, ref):
        # the quaternion's sign is fixed by real > 0 in both; rounding-level differences only
        assert np.abs(s[:7] - r[:7]).max() <= 1e-12 * max(1.0, np.abs(r[:7]).max()), x
        assert np.abs(s[:7] - of.se3_exp(x)).max() <= 1e-12 * max(1.0, np.abs(r[:7]).max()), x


@pytest.mark.parametrize("i", range(9))
def test_device_log_adj_inverse(i):
    g = group_elements()[i]
    lg = run("log", [g])[0][:6]
    # tests.hpp expLogTest on the device results
    back = run("exp", [lg])[0][:7]
    assert np.linalg.norm(matrix(g) - matrix(back)) <= 10 * EPS
    assert np.abs(lg - of.se3_log(g)).max() <= 1e-12 * max(1.0, np.abs(lg).max())
    Ad = run("adj", [g])[0].reshape(6, 6)
    assert np.abs(Ad - of.se3_adj(g).reshape(6, 6)).max() <= 1e-12 * max(1.0, np.abs(Ad).max())
    inv = run("inverse", [g])[0][:7]
    assert np.abs(inv - of.se3_inverse(g)).max() <= 1e-12 * max(1.0, np.abs(inv).max())
    T, Ti = matrix(g), matrix(inv)
    for x in TANGENTS:  # tests.hpp adjointTest
        assert np.linalg.norm(Ad @ x - vee(T @ hat(x) @ Ti)) <= 20 * EPS * max(1.0, np.linalg.norm(Ad @ x))


@pytest.mark.parametrize("i", range(9))
def test_device_products(i):
    gs = group_elements()
    g = gs[i]
    pairs = [(g, h) for h in gs]
    prod = run("mul", pairs)
    step = run("mul_step", pairs)
    for (a, b), p, s in zip(pairs, prod, step):
        o = of.se3_mul(a, b)
        scale = max(1.0, np.abs(o).max())
        assert np.abs(p[:7] - o).max() <= 1e-12 * scale
        assert np.abs(s[:7] - o).max() <= 1e-12 * scale
        assert np.linalg.norm(matrix(p) - matrix(a) @ matrix(b)) <= 1e-8 * max(1.0, np.linalg.norm(matrix(p)))


def test_device_matches_host_build():
    """hs_se3.h compiled for the device and for the host (the host algebra of the window set-up) agree to a few ulps."""
    gs = group_elements()
    for op, rows in (("exp", list(TANGENTS) + step_tangents()), ("log", gs), ("adj", gs), ("inverse", gs),
                     ("mul", [(a, b) for a in gs for b in gs]), ("rot", gs)):
        d = run(op, rows, device=True)
        h = run(op, rows, device=False)
        assert np.abs(d - h).max() <= 1e-14 * max(1.0, np.abs(h).max()), op
