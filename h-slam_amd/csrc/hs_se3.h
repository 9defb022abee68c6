// hs_se3.h — fp64 SE(3) of the host/device algebra, restating the vendored Sophus 0.9a
// the reference uses (usable from host code and from the on-device solve kernel):
//   exp           Thirdparty/Sophus/sophus/se3.hpp:407-427, so3.hpp:343-369
//   log           se3.hpp:560-588, so3.hpp:491-531
//   operator*     so3.hpp:229-269 (quaternion product + normalize), se3 fastMultiply
//   inverse       se3.hpp:164-168, so3.hpp:173-175
//   Adj           se3.hpp:128-137
//   rotation      Eigen Quaternion::toRotationMatrix
// Checked against the Sophus test_se3.cpp element/tangent sets in tests/.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>

#ifndef HS_HD
#define HS_HD __host__ __device__
#endif

namespace hs {

static constexpr double kSophusEps = 1e-10;  // SophusConstants<double>::epsilon()

struct Quat {
  double x, y, z, w;
};

HS_HD inline Quat qmul(const Quat& a, const Quat& b) {
  Quat r;
  r.w = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
  r.x = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
  r.y = a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z;
  r.z = a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x;
  return r;
}
HS_HD inline Quat qnormalize(Quat q) {
  double n = sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
  q.x /= n;
  q.y /= n;
  q.z /= n;
  q.w /= n;
  return q;
}
// Eigen _transformVector
HS_HD inline void qrot(const Quat& q, const double v[3], double out[3]) {
  double uv[3] = {q.y * v[2] - q.z * v[1], q.z * v[0] - q.x * v[2], q.x * v[1] - q.y * v[0]};
  uv[0] += uv[0];
  uv[1] += uv[1];
  uv[2] += uv[2];
  double c[3] = {q.y * uv[2] - q.z * uv[1], q.z * uv[0] - q.x * uv[2], q.x * uv[1] - q.y * uv[0]};
  out[0] = v[0] + q.w * uv[0] + c[0];
  out[1] = v[1] + q.w * uv[1] + c[1];
  out[2] = v[2] + q.w * uv[2] + c[2];
}

struct SE3 {
  Quat q{0, 0, 0, 1};
  double t[3]{0, 0, 0};

  HS_HD static SE3 fromData(const double d[7]) {
    SE3 s;
    s.q = qnormalize(Quat{d[0], d[1], d[2], d[3]});
    s.t[0] = d[4];
    s.t[1] = d[5];
    s.t[2] = d[6];
    return s;
  }
  HS_HD void toData(double d[7]) const {
    d[0] = q.x; d[1] = q.y; d[2] = q.z; d[3] = q.w; d[4] = t[0]; d[5] = t[1]; d[6] = t[2];
  }
  HS_HD void rotationMatrix(double R[9]) const {
    const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
    const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
    R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
  }
  HS_HD SE3 operator*(const SE3& o) const {
    SE3 r;
    double rt[3];
    qrot(q, o.t, rt);
    r.t[0] = t[0] + rt[0];
    r.t[1] = t[1] + rt[1];
    r.t[2] = t[2] + rt[2];
    r.q = qnormalize(qmul(q, o.q));
    return r;
  }
  HS_HD SE3 inverse() const {
    SE3 r;
    r.q = Quat{-q.x, -q.y, -q.z, q.w};
    double mt[3] = {-t[0], -t[1], -t[2]};
    qrot(r.q, mt, r.t);
    return r;
  }
  // Adj = [R, hat(t)R; 0, R] (row-major 6x6)
  HS_HD void Adj(double A[36]) const {
    double R[9];
    rotationMatrix(R);
    for (int i = 0; i < 36; i++) A[i] = 0;
    double H[9] = {0, -t[2], t[1], t[2], 0, -t[0], -t[1], t[0], 0};
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) {
        A[r * 6 + c] = R[r * 3 + c];
        A[(r + 3) * 6 + c + 3] = R[r * 3 + c];
        double s = 0;
        for (int k = 0; k < 3; k++) s += H[r * 3 + k] * R[k * 3 + c];
        A[r * 6 + c + 3] = s;
      }
  }
  HS_HD static void hat3(const double w[3], double O[9]) {
    O[0] = 0; O[1] = -w[2]; O[2] = w[1];
    O[3] = w[2]; O[4] = 0; O[5] = -w[0];
    O[6] = -w[1]; O[7] = w[0]; O[8] = 0;
  }
  HS_HD static void mm3(const double A[9], const double B[9], double C[9]) {
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++)
        C[r * 3 + c] = A[r * 3 + 0] * B[0 * 3 + c] + A[r * 3 + 1] * B[1 * 3 + c] + A[r * 3 + 2] * B[2 * 3 + c];
  }
  HS_HD static Quat so3expq(const double w[3], double* theta) {
    const double theta_sq = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    *theta = sqrt(theta_sq);
    const double half_theta = 0.5 * (*theta);
    double imag, real;
    if (*theta < kSophusEps) {
      const double theta_po4 = theta_sq * theta_sq;
      imag = 0.5 - (1.0 / 48.0) * theta_sq + (1.0 / 3840.0) * theta_po4;
      real = 1 - 0.5 * theta_sq + (1.0 / 384.0) * theta_po4;
    } else {
      imag = sin(half_theta) / (*theta);
      real = cos(half_theta);
    }
    return qnormalize(Quat{imag * w[0], imag * w[1], imag * w[2], real});
  }
  // tangent = (upsilon[3] translation, omega[3] rotation)
  HS_HD static SE3 exp(const double a[6]) {
    const double* w = a + 3;
    double theta;
    SE3 r;
    r.q = so3expq(w, &theta);
    double V[9];
    if (theta < kSophusEps) {
      r.rotationMatrix(V);
    } else {
      double O[9], O2[9];
      hat3(w, O);
      mm3(O, O, O2);
      const double theta_sq = theta * theta;
      const double c1 = (1.0 - cos(theta)) / theta_sq;
      const double c2 = (theta - sin(theta)) / (theta_sq * theta);
      for (int i = 0; i < 9; i++) V[i] = ((i % 4 == 0) ? 1.0 : 0.0) + c1 * O[i] + c2 * O2[i];
    }
    for (int i = 0; i < 3; i++) r.t[i] = V[i * 3 + 0] * a[0] + V[i * 3 + 1] * a[1] + V[i * 3 + 2] * a[2];
    return r;
  }
  HS_HD static void so3log(const Quat& q, double w[3], double* theta) {
    const double squared_n = q.x * q.x + q.y * q.y + q.z * q.z;
    const double n = sqrt(squared_n);
    const double qw = q.w;
    double f;
    if (n < kSophusEps) {
      const double squared_w = qw * qw;
      f = 2.0 / qw - 2.0 * squared_n / (qw * squared_w);
    } else {
      if (fabs(qw) < kSophusEps) f = (qw > 0 ? M_PI : -M_PI) / n;
      else f = 2.0 * atan(n / qw) / n;
    }
    *theta = f * n;
    w[0] = f * q.x;
    w[1] = f * q.y;
    w[2] = f * q.z;
  }
  HS_HD void log(double out[6]) const {
    double theta;
    double* w = out + 3;
    so3log(q, w, &theta);
    double O[9], O2[9], Vi[9];
    hat3(w, O);
    mm3(O, O, O2);
    double c;
    if (fabs(theta) < kSophusEps) c = 1. / 12.;
    else c = (1.0 - theta / (2.0 * tan(theta / 2.0))) / (theta * theta);
    for (int i = 0; i < 9; i++) Vi[i] = ((i % 4 == 0) ? 1.0 : 0.0) - 0.5 * O[i] + c * O2[i];
    for (int i = 0; i < 3; i++) out[i] = Vi[i * 3 + 0] * t[0] + Vi[i * 3 + 1] * t[1] + Vi[i * 3 + 2] * t[2];
  }
};

}  // namespace hs
