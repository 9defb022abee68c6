"""Minimal fp64 SE3 on Sophus' data layout (qx qy qz qw tx ty tz) for the host-side caller logic
(System::trackNewCoarse's motion hypotheses, Src/System.cpp:346-405).  Sophus v0.9a semantics:
exp/log with the left Jacobian V, quaternions normalised on construction."""
from __future__ import annotations

import math

import numpy as np


def _hat(w):
    return np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]], dtype=np.float64)


def quat_to_rot(q):
    x, y, z, w = q
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
        [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
        [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def _quat_mul(a, b):
    ax, ay, az, aw = a
    bx, by, bz, bw = b
    return np.array([aw * bx + ax * bw + ay * bz - az * by,
                     aw * by - ax * bz + ay * bw + az * bx,
                     aw * bz + ax * by - ay * bx + az * bw,
                     aw * bw - ax * bx - ay * by - az * bz])


def _rotate(q, p):
    return quat_to_rot(q) @ p


class SE3:
    __slots__ = ("q", "t")

    def __init__(self, q=(0.0, 0.0, 0.0, 1.0), t=(0.0, 0.0, 0.0)):
        q = np.asarray(q, dtype=np.float64)
        self.q = q / np.linalg.norm(q)
        self.t = np.asarray(t, dtype=np.float64).copy()

    @staticmethod
    def from_quat_wxyz(w, x, y, z, t=(0.0, 0.0, 0.0)):
        """Sophus::Quaterniond(w, x, y, z) (Eigen's constructor order), normalised by SE3()."""
        return SE3((x, y, z, w), t)

    @staticmethod
    def from_data(d):
        d = np.asarray(d, dtype=np.float64)
        return SE3(d[:4], d[4:7])

    def data(self):
        return np.concatenate([self.q, self.t])

    def __mul__(self, o: "SE3") -> "SE3":
        return SE3(_quat_mul(self.q, o.q), self.t + _rotate(self.q, o.t))

    def inverse(self) -> "SE3":
        qi = np.array([-self.q[0], -self.q[1], -self.q[2], self.q[3]])
        return SE3(qi, -_rotate(qi, self.t))

    def matrix(self):
        M = np.eye(4)
        M[:3, :3] = quat_to_rot(self.q)
        M[:3, 3] = self.t
        return M

    @staticmethod
    def exp(xi) -> "SE3":
        """xi = (translation upsilon, rotation omega) as Sophus::SE3::exp."""
        xi = np.asarray(xi, dtype=np.float64)
        ups, om = xi[:3], xi[3:6]
        th = float(np.linalg.norm(om))
        half = 0.5 * th
        if th < 1e-10:
            th2 = th * th
            imag = 0.5 - th2 / 48.0 + th2 * th2 / 3840.0
            real = 1.0 - th2 / 8.0 + th2 * th2 / 384.0
        else:
            imag = math.sin(half) / th
            real = math.cos(half)
        q = np.array([imag * om[0], imag * om[1], imag * om[2], real])
        Om = _hat(om)
        if th < 1e-10:
            V = np.eye(3) + 0.5 * Om + Om @ Om / 6.0
        else:
            V = np.eye(3) + (1 - math.cos(th)) / (th * th) * Om + (th - math.sin(th)) / th ** 3 * (Om @ Om)
        return SE3(q, V @ ups)

    def log(self):
        x, y, z, w = self.q
        n = math.sqrt(x * x + y * y + z * z)
        if n < 1e-10:
            two_atan = 2.0 / w - 2.0 * n * n / (w ** 3)
        elif abs(w) < 1e-10:
            two_atan = math.pi / n if w > 0 else -math.pi / n
        else:
            two_atan = 2.0 * math.atan(n / w) / n
        om = two_atan * np.array([x, y, z])
        th = float(np.linalg.norm(om))
        Om = _hat(om)
        if abs(th) < 1e-10:
            Vi = np.eye(3) - 0.5 * Om + Om @ Om / 12.0
        else:
            half = 0.5 * th
            Vi = np.eye(3) - 0.5 * Om + (1 - half * math.cos(half) / math.sin(half)) / (th * th) * (Om @ Om)
        return np.concatenate([Vi @ self.t, om])
