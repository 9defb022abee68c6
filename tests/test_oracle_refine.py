"""CPU tests of the DirectRefinement oracle (oracle/refine_oracle.cpp).

The C restatement is pinned against an independent pure-Python / numpy-float32 loop restatement of
calcResAndGS's per-point arithmetic (Src/Initializer.cpp:1970-2073) on a handful of points (bit-exact: every
float32 operation in the reference's order), and by property tests of Refine: the pose moves toward the
truth, accepted steps lower the total energy, the reference's quirks (E.num = 2 npts, EAlpha never updated,
the alpha regularizer snapping off for |t| > sqrt(alphaK / alphaW)) hold.
"""
import math

import numpy as np
import pytest

f32 = np.float32
PATTERN = [(0, -2), (-1, -1), (1, -1), (-2, 0), (0, 0), (2, 0), (-1, 1), (0, 2)]


def _pose_err(a, b):
    from hslam_amd.se3 import SE3
    return float(np.linalg.norm((SE3.from_data(a) * SE3.from_data(b).inverse()).log()))


@pytest.fixture(scope="module")
def scene():
    from hslam_amd.scene import make_refine_scene
    return make_refine_scene(600, seed=21)


def _interp(img, x, y, ch):
    ix, iy = int(x), int(y)
    dx, dy = f32(x - f32(ix)), f32(y - f32(iy))
    dxdy = f32(dx * dy)
    p = lambda xx, yy: f32(img[yy, xx, ch])  # noqa: E731
    w11, w01, w10 = dxdy, f32(dy - dxdy), f32(dx - dxdy)
    w00 = f32(f32(f32(f32(1) - dx) - dy) + dxdy)
    return f32(f32(f32(f32(w11 * p(ix + 1, iy + 1)) + f32(w01 * p(ix, iy + 1))) + f32(w10 * p(ix + 1, iy))) +
               f32(w00 * p(ix, iy)))


def _py_point(s, i, RKi, t, fx, fy, cx, cy, idn, tri):
    """calcResAndGS for point i, float32 scalars in the reference's operation order (no fused multiply-add)."""
    img1 = s.img1.reshape(s.height, s.width, 3)
    img2 = s.img2.reshape(s.height, s.width, 3)
    energy = f32(0)
    jb = [f32(0)] * 10
    ms = f32(1e10)
    for dx, dy in PATTERN:
        x, y = f32(f32(s.u[i]) + f32(dx)), f32(f32(s.v[i]) + f32(dy))
        pt = [f32(f32(f32(f32(RKi[q, 0] * x) + f32(RKi[q, 1] * y)) + f32(RKi[q, 2] * f32(1))) + f32(t[q] * idn))
              for q in range(3)]
        u, v = f32(pt[0] / pt[2]), f32(pt[1] / pt[2])
        Ku, Kv = f32(f32(fx * u) + cx), f32(f32(fy * v) + cy)
        nid = f32(idn / pt[2])
        if not (Ku > 1 and Kv > 1 and Ku < s.width - 2 and Kv < s.height - 2 and nid > 0):
            return None
        h = [_interp(img2, Ku, Kv, c) for c in range(3)]
        rlR = _interp(img1, x, y, 0)
        res = f32(f32(h[0] - f32(f32(1) * rlR)) - f32(0))
        hw = f32(1) if abs(res) < f32(9) else f32(f32(9) / abs(res))
        if not tri:
            hw = f32(float(hw) * 0.1)
        energy = f32(energy + f32(f32(f32(hw * res) * res) * f32(f32(2) - hw)))
        dxdd = f32(f32(t[0] - f32(t[2] * u)) / pt[2])
        dydd = f32(f32(t[1] - f32(t[2] * v)) / pt[2])
        if hw < 1:
            hw = f32(math.sqrt(hw))
        dxI, dyI = f32(f32(hw * h[1]) * fx), f32(f32(hw * h[2]) * fy)
        dp = [f32(nid * dxI), f32(nid * dyI), f32(f32(-nid) * f32(f32(u * dxI) + f32(v * dyI))),
              f32(f32(f32(f32(-u) * v) * dxI) - f32(f32(f32(1) + f32(v * v)) * dyI)),
              f32(f32(f32(f32(1) + f32(u * u)) * dxI) + f32(f32(u * v) * dyI)),
              f32(f32(f32(-v) * dxI) + f32(u * dyI)),
              f32(f32(f32(-hw) * f32(1)) * rlR), f32(f32(-hw) * f32(1))]
        dd = f32(f32(dxI * dxdd) + f32(dyI * dydd))
        r = f32(hw * res)
        nx, ny = f32(dxdd * fx), f32(dydd * fy)
        m = f32(f32(1) / f32(math.sqrt(f32(f32(nx * nx) + f32(ny * ny)))))
        ms = min(ms, m)
        for k in range(8):
            jb[k] = f32(jb[k] + f32(dp[k] * dd))
        jb[8] = f32(jb[8] + f32(r * dd))
        jb[9] = f32(jb[9] + f32(dd * dd))
    return energy, ms, jb


def _rki(T7, K4):
    """(refToNew.rotationMatrix() * pyrKi[0]).cast<float>() with Eigen's quaternion -> matrix and 3x3 cofactor
    inverse formulas in double"""
    q = np.asarray(T7[:4], np.float64)
    q = q / math.sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3])
    x, y, z, w = q
    tx, ty, tz = 2 * x, 2 * y, 2 * z
    twx, twy, twz, txx, txy, txz = tx * w, ty * w, tz * w, tx * x, ty * x, tz * x
    tyy, tyz, tzz = ty * y, tz * y, tz * z
    R = np.array([[1 - (tyy + tzz), txy - twz, txz + twy], [txy + twz, 1 - (txx + tzz), tyz - twx],
                  [txz - twy, tyz + twx, 1 - (txx + tyy)]])
    m = np.array([[K4[0], 0, K4[2]], [0, K4[1], K4[3]], [0, 0, 1.0]])
    cof = lambda i, j: (m[(i + 1) % 3, (j + 1) % 3] * m[(i + 2) % 3, (j + 2) % 3] -  # noqa: E731
                        m[(i + 1) % 3, (j + 2) % 3] * m[(i + 2) % 3, (j + 1) % 3])
    invdet = 1.0 / (cof(0, 0) * m[0, 0] + cof(1, 0) * m[1, 0] + cof(2, 0) * m[2, 0])
    Ki = np.array([[cof(j, i) * invdet for j in range(3)] for i in range(3)])
    RK = np.array([[R[r, 0] * Ki[0, c] + R[r, 1] * Ki[1, c] + R[r, 2] * Ki[2, c] for c in range(3)] for r in range(3)])
    return RK.astype(np.float32)


def test_oracle_pinned_by_python_restatement(scene):
    from oracle_ffi import OracleRefiner
    s = scene
    o = OracleRefiner(s)
    o.calc_res(s.T_init)
    p = o.points()
    RKi = _rki(s.T_init, s.K4)
    t = np.asarray(s.T_init[4:], np.float64).astype(np.float32)
    fx, fy, cx, cy = (f32(x) for x in s.K4)
    checked = 0
    for i in range(0, s.n_points, 23):
        idn = f32(p["idepth_new"][i])
        out = _py_point(s, i, RKi, t, fx, fy, cx, cy, idn, bool(s.tri[i]))
        if out is None:
            assert p["isGood_new"][i] == 0
            continue
        energy, ms, jb = out
        if energy > f32(8 * 144 * 20):
            assert p["isGood_new"][i] == 0
            continue
        assert p["isGood_new"][i] == 1
        assert p["energy_new0"][i] == energy
        assert p["maxstep"][i] == ms
        assert p["lastHessian_new"][i] == jb[9]
        assert np.array_equal(p["jb_new"][i][:8], np.array(jb[:8], np.float32))
        checked += 1
    assert checked >= 15


def test_oracle_refine_properties(scene):
    from oracle_ffi import OracleRefiner
    s = scene
    o = OracleRefiner(s)
    T, it, snapped = o.refine(s.T_init)
    L = o.log()
    assert len(L) == it and it >= 3
    assert snapped  # |t| = 0.15 >> sqrt(alphaK / alphaW) = 0.0167
    assert _pose_err(T, s.T_true) < 0.5 * _pose_err(s.T_init, s.T_true)
    acc = L[L[:, 2] == 1]
    assert np.all(acc[:, 1] < acc[:, 0])  # accepted steps lower eTotal
    assert np.all(L[:, 6] == np.float32(2.5 * 2.5) * np.float32(s.n_points))  # alphaEnergy capped


def test_oracle_calc_res_quirks(scene):
    from oracle_ffi import OracleRefiner
    s = scene
    o = OracleRefiner(s)
    H, b, Hsc, bsc, res = o.calc_res(s.T_init)
    assert res[2] == 2 * s.n_points  # E.num counts both energy loops
    assert np.allclose(H, H.T) and np.allclose(Hsc, Hsc.T)
    assert np.all(np.linalg.eigvalsh(H.astype(np.float64)) > -1e-3 * np.abs(H).max())
    # small baseline: alphaEnergy = alphaW |t|^2 npts (EAlpha never updated), alphaOpt = alphaW adds npts*alphaW
    T = np.array(s.T_init)
    T[4:] = T[4:] / np.linalg.norm(T[4:]) * 0.01
    H2, b2, _, _, res2 = o.calc_res(T)
    assert res2[1] == np.float32(np.float32(150 * 150) * (0.01 ** 2 * s.n_points))
