"""Pin the oracle's fp64 SE3 (restated Sophus 0.9a) with the vendored Sophus test sets.

Element / tangent / point sets copied as data from Thirdparty/Sophus/sophus/test_se3.cpp:41-90;
properties from Thirdparty/Sophus/sophus/tests.hpp:43-200 (adjoint, exp/log round trip,
exp vs matrix exponential, group action), SMALL_EPS = 1e-10 for double.
"""
import math

import numpy as np
import pytest
from scipy.linalg import expm

import oracle_ffi as of

EPS = 1e-10


def _se3(w, t):
    d = of.se3_exp(np.array([0.0, 0.0, 0.0, *w]))
    d[4:7] = t
    return d


def group_elements():
    g = [_se3((0.2, 0.5, 0.0), (0, 0, 0)), _se3((0.2, 0.5, -1.0), (10, 0, 0)), _se3((0., 0., 0.), (0, 100, 5)),
         _se3((0., 0., 0.00001), (0, 0, 0)), _se3((0., 0., 0.00001), (0, -0.00000001, 0.0000000001)),
         _se3((0., 0., 0.00001), (0.01, 0, 0)), _se3((math.pi, 0, 0), (4, -5, 0))]
    a = of.se3_mul(of.se3_mul(_se3((0.2, 0.5, 0.0), (0, 0, 0)), _se3((math.pi, 0, 0), (0, 0, 0))),
                   _se3((-0.2, -0.5, -0.0), (0, 0, 0)))
    b = of.se3_mul(of.se3_mul(_se3((0.3, 0.5, 0.1), (2, 0, -7)), _se3((math.pi, 0, 0), (0, 0, 0))),
                   _se3((-0.3, -0.5, -0.1), (0, 6, 0)))
    return g + [a, b]


TANGENTS = [np.array(v, float) for v in ([0, 0, 0, 0, 0, 0], [1, 0, 0, 0, 0, 0], [0, 1, 0, 1, 0, 0],
                                          [0, -5, 10, 0, 0, 0], [-1, 1, 0, 0, 0, 1], [20, -1, 0, -1, 1, 0],
                                          [30, 5, -1, 20, -1, 0])]


def matrix(d):
    T = np.eye(4)
    T[:3, :3] = of.se3_matrix(d)
    T[:3, 3] = d[4:7]
    return T


def hat(x):
    w = x[3:]
    T = np.zeros((4, 4))
    T[:3, :3] = [[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]]
    T[:3, 3] = x[:3]
    return T


def vee(T):
    return np.array([T[0, 3], T[1, 3], T[2, 3], T[2, 1], T[0, 2], T[1, 0]])


@pytest.mark.parametrize("i", range(9))
def test_exp_log_roundtrip(i):
    g = group_elements()[i]
    T1 = matrix(g)
    T2 = matrix(of.se3_exp(of.se3_log(g)))
    assert np.linalg.norm(T1 - T2) <= EPS * 10  # tests.hpp expLogTest (SMALL_EPS; 10x slack for the pi case)


@pytest.mark.parametrize("i", range(9))
def test_adjoint(i):
    g = group_elements()[i]
    T = matrix(g)
    Ad = of.se3_adj(g)
    Tinv = matrix(of.se3_inverse(g))
    for x in TANGENTS:
        ad1 = Ad @ x
        ad2 = vee(T @ hat(x) @ Tinv)
        assert np.linalg.norm(ad1 - ad2) <= 20 * EPS * max(1.0, np.linalg.norm(ad2))


@pytest.mark.parametrize("j", range(7))
def test_exp_map(j):
    x = TANGENTS[j]
    assert np.linalg.norm(matrix(of.se3_exp(x)) - expm(hat(x))) <= 10 * EPS * max(1.0, np.linalg.norm(expm(hat(x))))


@pytest.mark.parametrize("i", range(9))
def test_group_action_and_mul(i):
    gs = group_elements()
    g = gs[i]
    p = np.array([1.0, 2.0, 4.0])
    T = matrix(g)
    res2 = T[:3, :3] @ p + T[:3, 3]
    inv = of.se3_inverse(g)
    assert np.linalg.norm(matrix(of.se3_mul(g, inv)) - np.eye(4)) <= 100 * EPS * max(1.0, np.linalg.norm(T))
    for h in gs:
        assert np.linalg.norm(matrix(of.se3_mul(g, h)) - T @ matrix(h)) <= 1e-8 * max(1.0, np.linalg.norm(T @ matrix(h)))
    assert np.all(np.isfinite(res2))
