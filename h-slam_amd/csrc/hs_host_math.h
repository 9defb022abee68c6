// hs_host_math.h — fp64 host algebra of the BA path (the parts the reference
// runs with Eigen/Sophus on the host, not the hot path):
//   FrameOptimizationData setState/setStateZero/getPrior   Include/Frame.h:151-258
//   CalibData setValue/setValueScaled                      Include/CalibData.h:60-91
//   FrameFramePrecalc::set                                  Src/OptimizationClasses.cpp:13-39
//   EnergyFunctional::setAdjointsF                          Src/EnergyFunctional.cpp:22-82
//   System::getNullspaces + EnergyFunctional::orthogonalize Src/FullSystemOptimize.cpp:616-670,
//                                                           Src/EnergyFunctional.cpp:648-702
//   Eigen::LDLT solve used by solveSystemF                  Src/EnergyFunctional.cpp:799-801
#pragma once
#include <algorithm>
#include <cmath>
#include <limits>
#include <vector>

#include "../../include/hs_types.h"
#include "hs_layout.h"
#include "hs_se3.h"

#ifndef HS_HD
#define HS_HD __host__ __device__
#endif

namespace hs {

constexpr float SCALE_XI_ROT = 1.0f, SCALE_XI_TRANS = 0.5f, SCALE_F = 50.0f, SCALE_C = 50.0f;
constexpr float SCALE_A = 10.0f, SCALE_B = 1000.0f;
constexpr float SCALE_XI_ROT_INVERSE = 1.0f / SCALE_XI_ROT, SCALE_XI_TRANS_INVERSE = 1.0f / SCALE_XI_TRANS;
constexpr float SCALE_F_INVERSE = 1.0f / SCALE_F, SCALE_C_INVERSE = 1.0f / SCALE_C;

HS_HD inline void mm3f(const float A[9], const float B[9], float C[9]) {
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++)
      C[r * 3 + c] = A[r * 3 + 0] * B[0 * 3 + c] + A[r * 3 + 1] * B[1 * 3 + c] + A[r * 3 + 2] * B[2 * 3 + c];
}
HS_HD inline void mv3f(const float A[9], const float v[3], float o[3]) {
  for (int r = 0; r < 3; r++) o[r] = A[r * 3 + 0] * v[0] + A[r * 3 + 1] * v[1] + A[r * 3 + 2] * v[2];
}
// Eigen compute_inverse_size3 in float
HS_HD inline void inv3f(const float m[9], float r[9]) {
  auto M = [&](int i, int j) { return m[i * 3 + j]; };
  auto cof = [&](int i, int j) {
    int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
    return M(i1, j1) * M(i2, j2) - M(i1, j2) * M(i2, j1);
  };
  float c00 = cof(0, 0), c10 = cof(1, 0), c20 = cof(2, 0);
  float det = c00 * M(0, 0) + c10 * M(1, 0) + c20 * M(2, 0);
  float invdet = 1.0f / det;
  r[0] = c00 * invdet; r[1] = c10 * invdet; r[2] = c20 * invdet;
  r[3] = cof(0, 1) * invdet; r[4] = cof(1, 1) * invdet; r[5] = cof(2, 1) * invdet;
  r[6] = cof(0, 2) * invdet; r[7] = cof(1, 2) * invdet; r[8] = cof(2, 2) * invdet;
}
HS_HD inline void fromToVecExposure(float eF, float eT, double g2Fa, double g2Fb, double g2Ta, double g2Tb,
                              double out[2]) {
  if (eF == 0 || eT == 0) eT = eF = 1;
  double a = exp(g2Ta - g2Fa) * eT / eF;
  out[0] = a;
  out[1] = g2Tb - a * g2Fb;
}

struct CalibH {
  int W = 0, H = 0;
  double value[4], value_zero[4], value_minus_value_zero[4], value_scaled[4], value_backup[4], step[4];
  float value_scaledf[4], value_scaledi[4];
  HS_HD void setValueScaled(const double vs[4]) {
    for (int i = 0; i < 4; i++) value_scaled[i] = vs[i];
    for (int i = 0; i < 4; i++) value_scaledf[i] = (float)value_scaled[i];
    value[0] = SCALE_F_INVERSE * vs[0];
    value[1] = SCALE_F_INVERSE * vs[1];
    value[2] = SCALE_C_INVERSE * vs[2];
    value[3] = SCALE_C_INVERSE * vs[3];
    for (int i = 0; i < 4; i++) value_minus_value_zero[i] = value[i] - value_zero[i];
    scaledi();
  }
  HS_HD void setValue(const double v[4]) {
    for (int i = 0; i < 4; i++) value[i] = v[i];
    value_scaled[0] = SCALE_F * v[0];
    value_scaled[1] = SCALE_F * v[1];
    value_scaled[2] = SCALE_C * v[2];
    value_scaled[3] = SCALE_C * v[3];
    for (int i = 0; i < 4; i++) value_scaledf[i] = (float)value_scaled[i];
    scaledi();
    for (int i = 0; i < 4; i++) value_minus_value_zero[i] = value[i] - value_zero[i];
  }
  HS_HD void scaledi() {
    value_scaledi[0] = 1.0f / value_scaledf[0];
    value_scaledi[1] = 1.0f / value_scaledf[1];
    value_scaledi[2] = -value_scaledf[2] / value_scaledf[0];
    value_scaledi[3] = -value_scaledf[3] / value_scaledf[1];
  }
  HS_HD HsCalib device() const {
    HsCalib c;
    c.fxl = value_scaledf[0]; c.fyl = value_scaledf[1]; c.cxl = value_scaledf[2]; c.cyl = value_scaledf[3];
    c.fxli = value_scaledi[0]; c.fyli = value_scaledi[1];
    c.W = W; c.H = H;
    return c;
  }
};

struct FrameH {
  int id = 0, idx = 0;
  float ab_exposure = 1, frameEnergyTH = 8 * 8 * 8;
  SE3 evalPT, PRE_worldToCam, PRE_camToWorld;
  double state[10] = {0}, state_zero[10] = {0}, state_scaled[10] = {0}, step[10] = {0}, state_backup[10] = {0};
  double nullspaces_pose[6][6], nullspaces_scale[6];
  double prior[8] = {0}, delta_prior[8] = {0}, delta[8] = {0};

  HS_HD double aff_a() const { return state_scaled[6]; }
  HS_HD double aff_b() const { return state_scaled[7]; }
  HS_HD double aff0_a() const { return state_zero[6] * SCALE_A; }
  HS_HD double aff0_b() const { return state_zero[7] * SCALE_B; }

  HS_HD void setState(const double s[10]) {
    for (int i = 0; i < 10; i++) state[i] = s[i];
    for (int i = 0; i < 3; i++) state_scaled[i] = SCALE_XI_TRANS * s[i];
    for (int i = 3; i < 6; i++) state_scaled[i] = SCALE_XI_ROT * s[i];
    state_scaled[6] = SCALE_A * s[6];
    state_scaled[7] = SCALE_B * s[7];
    state_scaled[8] = SCALE_A * s[8];
    state_scaled[9] = SCALE_B * s[9];
    PRE_worldToCam = SE3::exp(state_scaled) * evalPT;
    PRE_camToWorld = PRE_worldToCam.inverse();
  }
  HS_HD void setStateZero(const double sz[10]) {
    for (int i = 0; i < 10; i++) state_zero[i] = sz[i];
    for (int i = 0; i < 6; i++) {
      double ep[6] = {0, 0, 0, 0, 0, 0}, em[6] = {0, 0, 0, 0, 0, 0};
      ep[i] = 1e-3;
      em[i] = -1e-3;
      SE3 P = (evalPT * SE3::exp(ep)) * evalPT.inverse();
      SE3 M = (evalPT * SE3::exp(em)) * evalPT.inverse();
      double lp[6], lm[6];
      P.log(lp);
      M.log(lm);
      for (int k = 0; k < 6; k++) nullspaces_pose[i][k] = (lp[k] - lm[k]) / (2e-3);
    }
    SE3 P = evalPT;
    for (int k = 0; k < 3; k++) P.t[k] *= 1.00001;
    P = P * evalPT.inverse();
    SE3 M = evalPT;
    for (int k = 0; k < 3; k++) M.t[k] /= 1.00001;
    M = M * evalPT.inverse();
    double lp[6], lm[6];
    P.log(lp);
    M.log(lm);
    for (int k = 0; k < 6; k++) nullspaces_scale[k] = (lp[k] - lm[k]) / (2e-3);
  }
  HS_HD void takeData(const hs_params& P) {
    double p[10] = {0};
    if (id == 0) {
      for (int i = 0; i < 3; i++) p[i] = P.initialTransPrior;
      for (int i = 3; i < 6; i++) p[i] = P.initialRotPrior;
      p[6] = P.initialAffAPrior;
      p[7] = P.initialAffBPrior;
    } else {
      p[6] = P.affineOptModeA < 0 ? P.initialAffAPrior : P.affineOptModeA;
      p[7] = P.affineOptModeB < 0 ? P.initialAffBPrior : P.affineOptModeB;
    }
    for (int i = 0; i < 8; i++) {
      prior[i] = p[i];
      delta[i] = state[i] - state_zero[i];
      delta_prior[i] = state[i] - 0.0;
    }
  }
};

// FrameFramePrecalc::set -> device record
HS_HD inline HsPrecalc make_precalc(const FrameH& H, const FrameH& T, const CalibH& cal) {
  HsPrecalc pc;
  SE3 l2l0 = T.evalPT * H.evalPT.inverse();
  double R0[9];
  l2l0.rotationMatrix(R0);
  for (int i = 0; i < 9; i++) pc.R0[i] = (float)R0[i];
  for (int i = 0; i < 3; i++) pc.t0[i] = (float)l2l0.t[i];
  SE3 l2l = T.PRE_worldToCam * H.PRE_camToWorld;
  double R[9];
  l2l.rotationMatrix(R);
  float RT[9], tT[3];
  for (int i = 0; i < 9; i++) RT[i] = (float)R[i];
  for (int i = 0; i < 3; i++) tT[i] = (float)l2l.t[i];
  float K[9] = {cal.value_scaledf[0], 0, cal.value_scaledf[2], 0, cal.value_scaledf[1], cal.value_scaledf[3], 0, 0, 1};
  float Ki[9], KR[9];
  inv3f(K, Ki);
  mm3f(K, RT, KR);
  mm3f(KR, Ki, pc.KRKi);
  mv3f(K, tT, pc.Kt);
  double aff[2];
  fromToVecExposure(H.ab_exposure, T.ab_exposure, H.aff_a(), H.aff_b(), T.aff_a(), T.aff_b(), aff);
  pc.aff[0] = (float)aff[0];
  pc.aff[1] = (float)aff[1];
  pc.b0 = (float)H.aff0_b();
  pc.pad = 0;
  return pc;
}

// setAdjointsF for one (h, t): AH, AT (row-major 8x8, fp64) + float copies
HS_HD inline void make_adjoints(const FrameH& H, const FrameH& T, double AH[64], double AT[64]) {
  SE3 h2t = T.evalPT * H.evalPT.inverse();
  for (int i = 0; i < 64; i++) AH[i] = AT[i] = (i % 9 == 0) ? 1.0 : 0.0;
  double Ad[36];
  h2t.Adj(Ad);
  for (int r = 0; r < 6; r++)
    for (int c = 0; c < 6; c++) {
      AH[r * 8 + c] = -Ad[c * 6 + r];
      AT[r * 8 + c] = (r == c) ? 1.0 : 0.0;
    }
  double affd[2];
  fromToVecExposure(H.ab_exposure, T.ab_exposure, H.aff0_a(), H.aff0_b(), T.aff0_a(), T.aff0_b(), affd);
  float aff0 = (float)affd[0];
  AT[6 * 8 + 6] = -aff0;
  AH[6 * 8 + 6] = aff0;
  AT[7 * 8 + 7] = -1;
  AH[7 * 8 + 7] = aff0;
  for (int r = 0; r < 8; r++) {
    double s = r < 3 ? SCALE_XI_TRANS : (r < 6 ? SCALE_XI_ROT : (r == 6 ? SCALE_A : SCALE_B));
    for (int c = 0; c < 8; c++) { AH[r * 8 + c] *= s; AT[r * 8 + c] *= s; }
  }
}

// Eigen::LDLT (diagonal pivoting) solve of the dense symmetric system
inline void ldlt_solve(std::vector<double> A, int n, const std::vector<double>& b, std::vector<double>& x) {
  std::vector<int> transp(n);
  std::vector<double> temp(n);
  auto at = [&](int i, int j) -> double& { return A[i * n + j]; };
  for (int k = 0; k < n; k++) {
    int idx = k;
    double best = std::fabs(at(k, k));
    for (int i = k + 1; i < n; i++)
      if (std::fabs(at(i, i)) > best) { best = std::fabs(at(i, i)); idx = i; }
    transp[k] = idx;
    if (k != idx) {
      for (int j = 0; j < n; j++) std::swap(at(k, j), at(idx, j));
      for (int i = 0; i < n; i++) std::swap(at(i, k), at(i, idx));
    }
    if (k > 0) {
      for (int j = 0; j < k; j++) temp[j] = at(j, j) * at(k, j);
      double s = 0;
      for (int j = 0; j < k; j++) s += at(k, j) * temp[j];
      at(k, k) -= s;
      for (int i = k + 1; i < n; i++) {
        double t = 0;
        for (int j = 0; j < k; j++) t += at(i, j) * temp[j];
        at(i, k) -= t;
      }
    }
    const double akk = at(k, k);
    const bool valid = std::fabs(akk) > std::numeric_limits<double>::min();
    if (valid)
      for (int i = k + 1; i < n; i++) at(i, k) /= akk;
    for (int i = k + 1; i < n; i++) at(k, i) = at(i, k);
  }
  x = b;
  for (int k = 0; k < n; k++)
    if (transp[k] != k) std::swap(x[k], x[transp[k]]);
  for (int i = 0; i < n; i++)
    for (int j = 0; j < i; j++) x[i] -= at(i, j) * x[j];
  for (int i = 0; i < n; i++) x[i] = std::fabs(at(i, i)) > std::numeric_limits<double>::min() ? x[i] / at(i, i) : 0.0;
  for (int i = n - 1; i >= 0; i--)
    for (int j = i + 1; j < n; j++) x[i] -= at(j, i) * x[j];
  for (int k = n - 1; k >= 0; k--)
    if (transp[k] != k) std::swap(x[k], x[transp[k]]);
}

// symmetric projector N (N^T N)^+ N^T with the reference's singular-value cut (one-sided Jacobi SVD)
// P = (N Npi^T + Npi N^T) / 2 (EnergyFunctional::orthogonalize); factors (nullable) = [N | Npi], each [n][m]
inline void nullspace_projector(const std::vector<std::vector<double>>& ns, int n, double cut, std::vector<double>& P,
                               std::vector<double>* factors = nullptr) {
  const int m = (int)ns.size();
  std::vector<double> U(n * m), V(m * m, 0.0);
  for (int j = 0; j < m; j++) {
    double nn = 0;
    for (int i = 0; i < n; i++) nn += ns[j][i] * ns[j][i];
    nn = std::sqrt(nn);
    for (int i = 0; i < n; i++) U[i * m + j] = ns[j][i] / nn;
    V[j * m + j] = 1;
  }
  std::vector<double> N = U;
  for (int sweep = 0; sweep < 60; sweep++) {
    double off = 0;
    for (int p = 0; p < m; p++)
      for (int q = p + 1; q < m; q++) {
        double a = 0, b = 0, c = 0;
        for (int i = 0; i < n; i++) {
          a += U[i * m + p] * U[i * m + p];
          b += U[i * m + q] * U[i * m + q];
          c += U[i * m + p] * U[i * m + q];
        }
        if (std::fabs(c) <= 1e-300) continue;
        off = std::max(off, std::fabs(c) / std::sqrt(a * b));
        double zeta = (b - a) / (2 * c);
        double t = (zeta >= 0 ? 1.0 : -1.0) / (std::fabs(zeta) + std::sqrt(1 + zeta * zeta));
        double cs = 1 / std::sqrt(1 + t * t), sn = cs * t;
        for (int i = 0; i < n; i++) {
          double up = U[i * m + p], uq = U[i * m + q];
          U[i * m + p] = cs * up - sn * uq;
          U[i * m + q] = sn * up + cs * uq;
        }
        for (int i = 0; i < m; i++) {
          double vp = V[i * m + p], vq = V[i * m + q];
          V[i * m + p] = cs * vp - sn * vq;
          V[i * m + q] = sn * vp + cs * vq;
        }
      }
    if (off < 1e-15) break;
  }
  std::vector<double> S(m);
  double maxSv = 0;
  for (int j = 0; j < m; j++) {
    double s = 0;
    for (int i = 0; i < n; i++) s += U[i * m + j] * U[i * m + j];
    S[j] = std::sqrt(s);
    maxSv = std::max(maxSv, S[j]);
  }
  std::vector<double> Npi(n * m, 0.0);
  for (int k = 0; k < m; k++) {
    if (!(S[k] > cut * maxSv)) continue;
    double inv2 = 1.0 / (S[k] * S[k]);
    for (int i = 0; i < n; i++) {
      double uk = U[i * m + k] * inv2;
      for (int j = 0; j < m; j++) Npi[i * m + j] += uk * V[j * m + k];
    }
  }
  std::vector<double> NNpiT(n * n);
  for (int i = 0; i < n; i++)
    for (int j = 0; j < n; j++) {
      double s = 0;
      for (int k = 0; k < m; k++) s += N[i * m + k] * Npi[j * m + k];
      NNpiT[i * n + j] = s;
    }
  P.assign(n * n, 0.0);
  for (int i = 0; i < n; i++)
    for (int j = 0; j < n; j++) P[i * n + j] = 0.5 * (NNpiT[i * n + j] + NNpiT[j * n + i]);
  if (factors) {
    factors->assign(N.begin(), N.end());
    factors->insert(factors->end(), Npi.begin(), Npi.end());
  }
}

}  // namespace hs
