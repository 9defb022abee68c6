/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  See oracle_common.h for the parity status
 * ("parity unpinned": the reference cannot be built here, no golden vectors).
 *
 * CPU restatement of the reference's windowed photometric BA hot path, one
 * function per reference function, in the reference's operation order:
 *   FrameFramePrecalc::set                 Src/OptimizationClasses.cpp:13-39
 *   PointFrameResidual::linearize          Src/OptimizationClasses.cpp:43-233
 *   PointFrameResidual::applyRes/takeData  Src/OptimizationClasses.cpp:235-256, Include/OptimizationClasses.h:195-201
 *   fixLinearizationF                      Src/OptimizationClasses.cpp:258-284
 *   AccumulatedTopHessianSSE::addPoint     Src/AccumulatedTopHessian.cpp:21-141
 *   AccumulatedTopHessianSSE::stitchDoubleInternal/MT  Src/AccumulatedTopHessian.cpp:218-280, Include/AccumulatedTopHessian.h:69-117
 *   AccumulatedSCHessianSSE::addPoint      Src/AccumulatedSCHessian.cpp:10-53
 *   AccumulatedSCHessianSSE::stitchDoubleInternal/MT   Src/AccumulatedSCHessian.cpp:54-133, Include/AccumulatedSCHessian.h:70-111
 *   EnergyFunctional::setAdjointsF/setDeltaF           Src/EnergyFunctional.cpp:22-82,128-152
 *   EnergyFunctional::accumulate{A,L,SC}F_MT           Src/EnergyFunctional.cpp:155-220
 *   EnergyFunctional::resubstituteF_MT/FPt             Src/EnergyFunctional.cpp:222-274
 *   EnergyFunctional::orthogonalize/solveSystemF       Src/EnergyFunctional.cpp:648-817
 *   System::linearizeAll(_Reductor), setNewFrameEnergyTH, applyRes_Reductor  Src/FullSystemOptimize.cpp:19-165
 *   System::doStepFromBackup/backupState   Src/FullSystemOptimize.cpp:171-314
 *   System::optimize / solveSystem / getNullspaces     Src/FullSystemOptimize.cpp:362-561,616-670
 *   FrameOptimizationData setState/setStateZero/getPrior/takeData  Include/Frame.h:151-275
 *   CalibData::setValue/setValueScaled     Include/CalibData.h:60-91
 * Eigen's LDLT (diagonal pivoting) and a one-sided Jacobi SVD stand in for
 * the Eigen calls (version unpinned).
 */
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <memory>
#include <vector>

#include "ldlt.h"
#include "accum.h"
#include "ba_oracle.h"
#include "oracle_common.h"
#include "pool.h"
#include "se3.h"

namespace hso {

struct Calib {
  int W = 0, H = 0;
  double value[4], value_zero[4], value_minus_value_zero[4], value_scaled[4], value_backup[4], step[4];
  float value_scaledf[4], value_scaledi[4];
  float fxl() const { return value_scaledf[0]; }
  float fyl() const { return value_scaledf[1]; }
  float cxl() const { return value_scaledf[2]; }
  float cyl() const { return value_scaledf[3]; }
  float fxli() const { return value_scaledi[0]; }
  float fyli() const { return value_scaledi[1]; }
  void setValueScaled(const double vs[4]) {
    for (int i = 0; i < 4; i++) value_scaled[i] = vs[i];
    for (int i = 0; i < 4; i++) value_scaledf[i] = (float)value_scaled[i];
    value[0] = SCALE_F_INVERSE * vs[0];
    value[1] = SCALE_F_INVERSE * vs[1];
    value[2] = SCALE_C_INVERSE * vs[2];
    value[3] = SCALE_C_INVERSE * vs[3];
    for (int i = 0; i < 4; i++) value_minus_value_zero[i] = value[i] - value_zero[i];
    value_scaledi[0] = 1.0f / value_scaledf[0];
    value_scaledi[1] = 1.0f / value_scaledf[1];
    value_scaledi[2] = -value_scaledf[2] / value_scaledf[0];
    value_scaledi[3] = -value_scaledf[3] / value_scaledf[1];
  }
  void setValue(const double v[4]) {
    for (int i = 0; i < 4; i++) value[i] = v[i];
    value_scaled[0] = SCALE_F * v[0];
    value_scaled[1] = SCALE_F * v[1];
    value_scaled[2] = SCALE_C * v[2];
    value_scaled[3] = SCALE_C * v[3];
    for (int i = 0; i < 4; i++) value_scaledf[i] = (float)value_scaled[i];
    value_scaledi[0] = 1.0f / value_scaledf[0];
    value_scaledi[1] = 1.0f / value_scaledf[1];
    value_scaledi[2] = -value_scaledf[2] / value_scaledf[0];
    value_scaledi[3] = -value_scaledf[3] / value_scaledf[1];
    for (int i = 0; i < 4; i++) value_minus_value_zero[i] = value[i] - value_zero[i];
  }
};

struct FrameO {
  int id = 0, idx = 0;
  float ab_exposure = 1, frameEnergyTH = 8 * 8 * 8;
  SE3 evalPT, PRE_worldToCam, PRE_camToWorld;
  double state[10] = {0}, state_zero[10] = {0}, state_scaled[10] = {0}, step[10] = {0}, state_backup[10] = {0};
  double nullspaces_pose[6][6];  // [col][row]
  double nullspaces_scale[6];
  double nullspaces_affine[2][4];
  double prior[8] = {0}, delta_prior[8] = {0}, delta[8] = {0};
  const float* img = nullptr;  // level-0 (I,dx,dy) AoS
  std::vector<int> points;     // hosted points (pointHessians)

  double aff_a() const { return state_scaled[6]; }
  double aff_b() const { return state_scaled[7]; }
  double aff0_a() const { return state_zero[6] * SCALE_A; }
  double aff0_b() const { return state_zero[7] * SCALE_B; }

  void setState(const double s[10]) {
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
  void setStateZero(const double sz[10]) {
    for (int i = 0; i < 10; i++) state_zero[i] = sz[i];
    for (int i = 0; i < 6; i++) {
      double eps[6] = {0, 0, 0, 0, 0, 0};
      eps[i] = 1e-3;
      double meps[6] = {0, 0, 0, 0, 0, 0};
      meps[i] = -1e-3;
      SE3 P = (evalPT * SE3::exp(eps)) * evalPT.inverse();
      SE3 M = (evalPT * SE3::exp(meps)) * evalPT.inverse();
      double lp[6], lm[6];
      P.log(lp); M.log(lm);
      for (int k = 0; k < 6; k++) nullspaces_pose[i][k] = (lp[k] - lm[k]) / (2e-3);
    }
    SE3 P = evalPT;
    for (int k = 0; k < 3; k++) P.t[k] *= 1.00001;
    P = P * evalPT.inverse();
    SE3 M = evalPT;
    for (int k = 0; k < 3; k++) M.t[k] /= 1.00001;
    M = M * evalPT.inverse();
    double lp[6], lm[6];
    P.log(lp); M.log(lm);
    for (int k = 0; k < 6; k++) nullspaces_scale[k] = (lp[k] - lm[k]) / (2e-3);
    for (int c = 0; c < 2; c++)
      for (int r = 0; r < 4; r++) nullspaces_affine[c][r] = 0;
    nullspaces_affine[0][0] = 1;
    nullspaces_affine[1][1] = std::exp((float)aff0_a()) * ab_exposure;  // expf(aff_g2l_0().a)*ab_exposure
  }
  void getPrior(const hs_params& P, double p[10]) const {
    for (int i = 0; i < 10; i++) p[i] = 0;
    if (id == 0) {
      for (int i = 0; i < 3; i++) p[i] = P.initialTransPrior;
      for (int i = 3; i < 6; i++) p[i] = P.initialRotPrior;
      p[6] = P.initialAffAPrior;
      p[7] = P.initialAffBPrior;
    } else {
      p[6] = P.affineOptModeA < 0 ? P.initialAffAPrior : P.affineOptModeA;
      p[7] = P.affineOptModeB < 0 ? P.initialAffBPrior : P.affineOptModeB;
    }
    p[8] = P.initialAffAPrior;
    p[9] = P.initialAffBPrior;
  }
  void takeData(const hs_params& P) {
    double p[10];
    getPrior(P, p);
    for (int i = 0; i < 8; i++) {
      prior[i] = p[i];
      delta[i] = state[i] - state_zero[i];
      delta_prior[i] = state[i] - 0.0;
    }
  }
};

struct PointO {
  float u, v, idepth;
  int host;
  float color[8], weights[8];
  bool hasDepthPrior;
  // MapPointOptimizationData
  float idepth_zero, step = 0, step_backup = 0, idepth_backup = 0, nullspaces_scale = 0;
  float priorF = 0, deltaF = 0, bdSumF = 0, HdiF = 0;
  float Hdd_accLF = 0, Hcd_accLF[4] = {0, 0, 0, 0}, bd_accLF = 0;
  float Hdd_accAF = 0, Hcd_accAF[4] = {0, 0, 0, 0}, bd_accAF = 0;
  float idepth_hessian = 0, maxRelBaseline = 0;
  int numGoodResiduals = 0;
  std::vector<int> residuals;
};

struct RawJ {
  float resF[8];
  float Jpdxi[2][6];
  float Jpdc[2][4];
  float Jpdd[2];
  float JIdx[2][8];
  float JabF[2][8];
  float JIdx2[4], JabJIdx[4], Jab2[4];  // 2x2 row-major
};

struct ResO {
  int point, host, target;
  int state_state = HS_RES_IN, state_NewState = HS_RES_OUT;
  double state_energy = 0, state_NewEnergy = 0, state_NewEnergyWithOutlier = -1;
  bool isNew = true, isLinearized = false, isActiveAndIsGoodNEW = false;
  RawJ J;
  float projectedTo[8][2];
  float centerProjectedTo[3];
  float res_toZeroF[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float JpJdF[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  void resetOOB() {
    state_NewEnergy = state_energy = 0;
    state_NewState = HS_RES_OUT;
    state_state = HS_RES_IN;
  }
  void takeData() {
    float a = J.JIdx2[0] * J.Jpdd[0] + J.JIdx2[1] * J.Jpdd[1];
    float b = J.JIdx2[2] * J.Jpdd[0] + J.JIdx2[3] * J.Jpdd[1];
    for (int i = 0; i < 6; i++) JpJdF[i] = J.Jpdxi[0][i] * a + J.Jpdxi[1][i] * b;
    JpJdF[6] = J.JabJIdx[0] * J.Jpdd[0] + J.JabJIdx[1] * J.Jpdd[1];
    JpJdF[7] = J.JabJIdx[2] * J.Jpdd[0] + J.JabJIdx[3] * J.Jpdd[1];
  }
  bool isActive() const { return isActiveAndIsGoodNEW; }
};

struct Precalc {
  float PRE_RTll[9], PRE_KRKiTll[9], PRE_RKiTll[9], PRE_RTll_0[9];
  float PRE_aff_mode[2];
  float PRE_b0_mode;
  float PRE_tTll[3], PRE_KtTll[3], PRE_tTll_0[3];
  float distanceLL;
};

struct M88 { double m[64]; };
struct M88f { float m[64]; };

// ---------------------------------------------------------------- small fp64 linear algebra
static void mm(const double* A, const double* B, double* C, int n, int k, int m) {
  for (int i = 0; i < n; i++)
    for (int j = 0; j < m; j++) {
      double s = 0;
      for (int l = 0; l < k; l++) s += A[i * k + l] * B[l * m + j];
      C[i * m + j] = s;
    }
}
static void mmT(const double* A, const double* B, double* C, int n, int k, int m) {  // A (n x k) * B^T (B is m x k)
  for (int i = 0; i < n; i++)
    for (int j = 0; j < m; j++) {
      double s = 0;
      for (int l = 0; l < k; l++) s += A[i * k + l] * B[j * k + l];
      C[i * m + j] = s;
    }
}


// Orthogonal projector onto span(N) with the reference's singular-value cut
// (Src/EnergyFunctional.cpp:668-690), via one-sided Jacobi SVD of N (n x m).
static void nullspace_projector(const std::vector<std::vector<double>>& ns, int n, double cut, std::vector<double>& P) {
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
  // Npi = U diag(1/S) V^T, with U = columns / S  ->  Npi(:,j) = sum_k Ucol_k/S_k^2 * V(j,k) ... projector N * Npi^T
  std::vector<double> Npi(n * m, 0.0);
  for (int k = 0; k < m; k++) {
    if (!(S[k] > cut * maxSv)) continue;
    double inv2 = 1.0 / (S[k] * S[k]);
    for (int i = 0; i < n; i++) {
      double uk = U[i * m + k] * inv2;  // (U_k / S_k) / S_k
      for (int j = 0; j < m; j++) Npi[i * m + j] += uk * V[j * m + k];
    }
  }
  P.assign(n * n, 0.0);
  std::vector<double> NNpiT(n * n);
  for (int i = 0; i < n; i++)
    for (int j = 0; j < n; j++) {
      double s = 0;
      for (int k = 0; k < m; k++) s += N[i * m + k] * Npi[j * m + k];
      NNpiT[i * n + j] = s;
    }
  for (int i = 0; i < n; i++)
    for (int j = 0; j < n; j++) P[i * n + j] = 0.5 * (NNpiT[i * n + j] + NNpiT[j * n + i]);
}

// ---------------------------------------------------------------- the BA window
struct BA {
  hs_params P;
  Calib calib;
  int nF = 0;
  std::vector<FrameO> frames;
  std::vector<PointO> points;
  std::vector<ResO> res;
  std::vector<int> activeResiduals;
  std::vector<Precalc> precalc;  // [h*nF + t]
  std::vector<M88> adHost, adTarget;
  std::vector<M88f> adHostF, adTargetF;
  std::vector<float> adHTdeltaF;  // [idx][8]
  double cPrior[4];
  float cDeltaF[4], cPriorF[4];
  std::vector<double> HM, bM;
  std::vector<double> lastX;
  std::vector<std::vector<double>> ns_pose, ns_scale;
  std::unique_ptr<Pool> pool;
  int T = 1;
  bool mt = false;
  int lastResInA = 0;

  // per-thread accumulators
  std::vector<std::vector<AccApprox>> accTopA, accTopL;
  std::vector<int> nresA, nresL;
  std::vector<std::vector<AccXX<8, 4>>> accE;
  std::vector<std::vector<AccX<8>>> accEB;
  std::vector<std::vector<AccXX<8, 8>>> accD;
  std::vector<AccXX<4, 4>> accHcc;
  std::vector<AccX<4>> accbc;

  int dim() const { return CP + 8 * nF; }

  // FrameFramePrecalc::set
  void setPrecalc(int h, int t) {
    Precalc& pc = precalc[h * nF + t];
    FrameO& H = frames[h];
    FrameO& Tg = frames[t];
    SE3 l2l0 = Tg.evalPT * H.evalPT.inverse();
    double R0[9];
    l2l0.rotationMatrix(R0);
    for (int i = 0; i < 9; i++) pc.PRE_RTll_0[i] = (float)R0[i];
    for (int i = 0; i < 3; i++) pc.PRE_tTll_0[i] = (float)l2l0.t[i];
    SE3 l2l = Tg.PRE_worldToCam * H.PRE_camToWorld;
    double R[9];
    l2l.rotationMatrix(R);
    for (int i = 0; i < 9; i++) pc.PRE_RTll[i] = (float)R[i];
    for (int i = 0; i < 3; i++) pc.PRE_tTll[i] = (float)l2l.t[i];
    pc.distanceLL = (float)std::sqrt(l2l.t[0] * l2l.t[0] + l2l.t[1] * l2l.t[1] + l2l.t[2] * l2l.t[2]);
    float K[9] = {calib.fxl(), 0, calib.cxl(), 0, calib.fyl(), calib.cyl(), 0, 0, 1};
    float Ki[9], KR[9];
    inv3f(K, Ki);
    mm3f(K, pc.PRE_RTll, KR);
    mm3f(KR, Ki, pc.PRE_KRKiTll);
    mm3f(pc.PRE_RTll, Ki, pc.PRE_RKiTll);
    mv3f(K, pc.PRE_tTll, pc.PRE_KtTll);
    double aff[2];
    fromToVecExposure(H.ab_exposure, Tg.ab_exposure, H.aff_a(), H.aff_b(), Tg.aff_a(), Tg.aff_b(), aff);
    pc.PRE_aff_mode[0] = (float)aff[0];
    pc.PRE_aff_mode[1] = (float)aff[1];
    pc.PRE_b0_mode = (float)H.aff0_b();
  }

  // EnergyFunctional::setAdjointsF
  void setAdjointsF() {
    adHost.assign(nF * nF, M88());
    adTarget.assign(nF * nF, M88());
    adHostF.assign(nF * nF, M88f());
    adTargetF.assign(nF * nF, M88f());
    for (int h = 0; h < nF; h++)
      for (int t = 0; t < nF; t++) {
        SE3 h2t = frames[t].evalPT * frames[h].evalPT.inverse();
        double AH[64], AT[64];
        for (int i = 0; i < 64; i++) AH[i] = AT[i] = (i % 9 == 0) ? 1.0 : 0.0;
        double Ad[36];
        h2t.Adj(Ad);
        for (int r = 0; r < 6; r++)
          for (int c = 0; c < 6; c++) {
            AH[r * 8 + c] = -Ad[c * 6 + r];
            AT[r * 8 + c] = (r == c) ? 1.0 : 0.0;
          }
        double affd[2];
        fromToVecExposure(frames[h].ab_exposure, frames[t].ab_exposure, frames[h].aff0_a(), frames[h].aff0_b(),
                          frames[t].aff0_a(), frames[t].aff0_b(), affd);
        float aff0 = (float)affd[0];
        AT[6 * 8 + 6] = -aff0;
        AH[6 * 8 + 6] = aff0;
        AT[7 * 8 + 7] = -1;
        AH[7 * 8 + 7] = aff0;
        for (int r = 0; r < 8; r++) {
          double s = r < 3 ? SCALE_XI_TRANS : (r < 6 ? SCALE_XI_ROT : (r == 6 ? SCALE_A : SCALE_B));
          for (int c = 0; c < 8; c++) { AH[r * 8 + c] *= s; AT[r * 8 + c] *= s; }
        }
        int idx = h + t * nF;
        for (int i = 0; i < 64; i++) {
          adHost[idx].m[i] = AH[i];
          adTarget[idx].m[i] = AT[i];
          adHostF[idx].m[i] = (float)AH[i];
          adTargetF[idx].m[i] = (float)AT[i];
        }
      }
    for (int i = 0; i < 4; i++) { cPrior[i] = P.initialCalibHessian; cPriorF[i] = (float)cPrior[i]; }
  }

  // EnergyFunctional::setDeltaF
  void setDeltaF() {
    adHTdeltaF.assign(nF * nF * 8, 0.f);
    for (int h = 0; h < nF; h++)
      for (int t = 0; t < nF; t++) {
        int idx = h + t * nF;
        float dh[8], dt[8];
        for (int i = 0; i < 8; i++) {
          dh[i] = (float)(frames[h].state[i] - frames[h].state_zero[i]);
          dt[i] = (float)(frames[t].state[i] - frames[t].state_zero[i]);
        }
        for (int c = 0; c < 8; c++) {
          float s1 = 0, s2 = 0;
          for (int r = 0; r < 8; r++) s1 += dh[r] * adHostF[idx].m[r * 8 + c];
          for (int r = 0; r < 8; r++) s2 += dt[r] * adTargetF[idx].m[r * 8 + c];
          adHTdeltaF[idx * 8 + c] = s1 + s2;
        }
      }
    for (int i = 0; i < 4; i++) cDeltaF[i] = (float)calib.value_minus_value_zero[i];
    for (auto& f : frames) {
      for (int i = 0; i < 8; i++) {
        f.delta[i] = f.state[i] - f.state_zero[i];
        f.delta_prior[i] = f.state[i] - 0.0;
      }
      for (int pi : f.points) points[pi].deltaF = points[pi].idepth - points[pi].idepth_zero;
    }
  }

  void setPrecalcValues() {
    precalc.resize(nF * nF);
    for (int h = 0; h < nF; h++)
      for (int t = 0; t < nF; t++) setPrecalc(h, t);
    setDeltaF();
  }

  // ------------------------------------------------------------ PointFrameResidual::linearize
  double linearize(ResO& r) {
    r.state_NewEnergyWithOutlier = -1;
    if (r.state_state == HS_RES_OOB) {
      r.state_NewState = HS_RES_OOB;
      return r.state_energy;
    }
    const PointO& p = points[r.point];
    const Precalc& pc = precalc[r.host * nF + r.target];
    float energyLeft = 0;
    const float* dIl = frames[r.target].img;
    const float* color = p.color;
    const float* weights = p.weights;
    const float affLL0 = pc.PRE_aff_mode[0], affLL1 = pc.PRE_aff_mode[1];
    const float b0 = pc.PRE_b0_mode;
    float d_xi_x[6], d_xi_y[6], d_C_x[4], d_C_y[4], d_d_x, d_d_y;
    {
      // projectPoint(u, v, idepth_zero, 0, 0, HCalib, R_0, t_0, ...)  Include/DirectProjection.h:20-38
      float KliP[3] = {(p.u + 0 - calib.cxl()) * calib.fxli(), (p.v + 0 - calib.cyl()) * calib.fyli(), 1};
      float ptp[3];
      {
        float Rk[3];
        mv3f(pc.PRE_RTll_0, KliP, Rk);
        for (int i = 0; i < 3; i++) ptp[i] = Rk[i] + pc.PRE_tTll_0[i] * p.idepth_zero;
      }
      float drescale = 1.0f / ptp[2];
      float new_idepth = p.idepth_zero * drescale;
      if (!(drescale > 0)) { r.state_NewState = HS_RES_OOB; return r.state_energy; }
      float u = ptp[0] * drescale;
      float v = ptp[1] * drescale;
      float Ku = u * calib.fxl() + calib.cxl();
      float Kv = v * calib.fyl() + calib.cyl();
      if (!(Ku > 1.1f && Kv > 1.1f && Ku < (calib.W - 3) && Kv < (calib.H - 3))) {
        r.state_NewState = HS_RES_OOB;
        return r.state_energy;
      }
      r.centerProjectedTo[0] = Ku; r.centerProjectedTo[1] = Kv; r.centerProjectedTo[2] = new_idepth;
      const float* R0 = pc.PRE_RTll_0;
      const float* t0 = pc.PRE_tTll_0;
      d_d_x = drescale * (t0[0] - t0[2] * u) * SCALE_IDEPTH * calib.fxl();
      d_d_y = drescale * (t0[1] - t0[2] * v) * SCALE_IDEPTH * calib.fyl();
      d_C_x[2] = drescale * (R0[2 * 3 + 0] * u - R0[0 * 3 + 0]);
      d_C_x[3] = calib.fxl() * drescale * (R0[2 * 3 + 1] * u - R0[0 * 3 + 1]) * calib.fyli();
      d_C_x[0] = KliP[0] * d_C_x[2];
      d_C_x[1] = KliP[1] * d_C_x[3];
      d_C_y[2] = calib.fyl() * drescale * (R0[2 * 3 + 0] * v - R0[1 * 3 + 0]) * calib.fxli();
      d_C_y[3] = drescale * (R0[2 * 3 + 1] * v - R0[1 * 3 + 1]);
      d_C_y[0] = KliP[0] * d_C_y[2];
      d_C_y[1] = KliP[1] * d_C_y[3];
      d_C_x[0] = (d_C_x[0] + u) * SCALE_F;
      d_C_x[1] *= SCALE_F;
      d_C_x[2] = (d_C_x[2] + 1) * SCALE_C;
      d_C_x[3] *= SCALE_C;
      d_C_y[0] *= SCALE_F;
      d_C_y[1] = (d_C_y[1] + v) * SCALE_F;
      d_C_y[2] *= SCALE_C;
      d_C_y[3] = (d_C_y[3] + 1) * SCALE_C;
      const float fx = calib.fxl(), fy = calib.fyl();
      d_xi_x[0] = new_idepth * fx;
      d_xi_x[1] = 0;
      d_xi_x[2] = -new_idepth * u * fx;
      d_xi_x[3] = -u * v * fx;
      d_xi_x[4] = (1 + u * u) * fx;
      d_xi_x[5] = -v * fx;
      d_xi_y[0] = 0;
      d_xi_y[1] = new_idepth * fy;
      d_xi_y[2] = -new_idepth * v * fy;
      d_xi_y[3] = -(1 + v * v) * fy;
      d_xi_y[4] = u * v * fy;
      d_xi_y[5] = u * fy;
    }
    RawJ& J = r.J;
    for (int i = 0; i < 6; i++) { J.Jpdxi[0][i] = d_xi_x[i]; J.Jpdxi[1][i] = d_xi_y[i]; }
    for (int i = 0; i < 4; i++) { J.Jpdc[0][i] = d_C_x[i]; J.Jpdc[1][i] = d_C_y[i]; }
    J.Jpdd[0] = d_d_x; J.Jpdd[1] = d_d_y;

    float JIdxJIdx_00 = 0, JIdxJIdx_11 = 0, JIdxJIdx_10 = 0;
    float JabJIdx_00 = 0, JabJIdx_01 = 0, JabJIdx_10 = 0, JabJIdx_11 = 0;
    float JabJab_00 = 0, JabJab_01 = 0, JabJab_11 = 0;
    float wJI2_sum = 0;
    for (int idx = 0; idx < PN; idx++) {
      float Ku, Kv;
      {
        float pt[3] = {p.u + kPattern[idx][0], p.v + kPattern[idx][1], 1};
        float q[3];
        mv3f(pc.PRE_KRKiTll, pt, q);
        for (int i = 0; i < 3; i++) q[i] = q[i] + pc.PRE_KtTll[i] * p.idepth;
        Ku = q[0] / q[2];
        Kv = q[1] / q[2];
        if (!(Ku > 1.1f && Kv > 1.1f && Ku < (calib.W - 3) && Kv < (calib.H - 3))) {
          r.state_NewState = HS_RES_OOB;
          return r.state_energy;
        }
      }
      r.projectedTo[idx][0] = Ku;
      r.projectedTo[idx][1] = Kv;
      V3f hit = interp33(dIl, Ku, Kv, calib.W);
      float residual = hit.x - (float)(affLL0 * color[idx] + affLL1);
      float drdA = (color[idx] - b0);
      if (!std::isfinite(hit.x)) { r.state_NewState = HS_RES_OOB; return r.state_energy; }
      float w = sqrtf(P.outlierTHSumComponent / (P.outlierTHSumComponent + (hit.y * hit.y + hit.z * hit.z)));
      w = 0.5f * (w + weights[idx]);
      float hw = fabsf(residual) < P.huberTH ? 1 : P.huberTH / fabsf(residual);
      energyLeft += w * w * hw * residual * residual * (2 - hw);
      {
        if (hw < 1) hw = sqrtf(hw);
        hw = hw * w;
        hit.y *= hw;
        hit.z *= hw;
        J.resF[idx] = residual * hw;
        J.JIdx[0][idx] = hit.y;
        J.JIdx[1][idx] = hit.z;
        J.JabF[0][idx] = drdA * hw;
        J.JabF[1][idx] = hw;
        JIdxJIdx_00 += hit.y * hit.y;
        JIdxJIdx_11 += hit.z * hit.z;
        JIdxJIdx_10 += hit.y * hit.z;
        JabJIdx_00 += drdA * hw * hit.y;
        JabJIdx_01 += drdA * hw * hit.z;
        JabJIdx_10 += hw * hit.y;
        JabJIdx_11 += hw * hit.z;
        JabJab_00 += drdA * drdA * hw * hw;
        JabJab_01 += drdA * hw * hw;
        JabJab_11 += hw * hw;
        wJI2_sum += hw * hw * (hit.y * hit.y + hit.z * hit.z);
        if (P.affineOptModeA < 0) J.JabF[0][idx] = 0;
        if (P.affineOptModeB < 0) J.JabF[1][idx] = 0;
      }
    }
    J.JIdx2[0] = JIdxJIdx_00; J.JIdx2[1] = JIdxJIdx_10; J.JIdx2[2] = JIdxJIdx_10; J.JIdx2[3] = JIdxJIdx_11;
    J.JabJIdx[0] = JabJIdx_00; J.JabJIdx[1] = JabJIdx_01; J.JabJIdx[2] = JabJIdx_10; J.JabJIdx[3] = JabJIdx_11;
    J.Jab2[0] = JabJab_00; J.Jab2[1] = JabJab_01; J.Jab2[2] = JabJab_01; J.Jab2[3] = JabJab_11;
    r.state_NewEnergyWithOutlier = energyLeft;
    float th = std::max<float>(frames[r.host].frameEnergyTH, frames[r.target].frameEnergyTH);
    if (energyLeft > th || wJI2_sum < 2) {
      energyLeft = th;
      r.state_NewState = HS_RES_OUT;
    } else {
      r.state_NewState = HS_RES_IN;
    }
    r.state_NewEnergy = energyLeft;
    return energyLeft;
  }

  void applyRes(ResO& r) {
    if (r.state_state == HS_RES_OOB) return;
    if (r.state_NewState == HS_RES_IN) {
      r.isActiveAndIsGoodNEW = true;
      r.takeData();
    } else {
      r.isActiveAndIsGoodNEW = false;
    }
    r.state_state = r.state_NewState;
    r.state_energy = r.state_NewEnergy;
  }

  void fixLinearizationF(ResO& r) {
    const float* dp = &adHTdeltaF[(r.host + nF * r.target) * 8];
    const PointO& p = points[r.point];
    float jx = 0, jy = 0, cx = 0, cy = 0;
    for (int i = 0; i < 6; i++) { jx += r.J.Jpdxi[0][i] * dp[i]; jy += r.J.Jpdxi[1][i] * dp[i]; }
    for (int i = 0; i < 4; i++) { cx += r.J.Jpdc[0][i] * cDeltaF[i]; cy += r.J.Jpdc[1][i] * cDeltaF[i]; }
    float Jp_delta_x = jx + cx + r.J.Jpdd[0] * p.deltaF;
    float Jp_delta_y = jy + cy + r.J.Jpdd[1] * p.deltaF;
    float da = dp[6], db = dp[7];
    for (int i = 0; i < PN; i++) {
      float rtz = r.J.resF[i];
      rtz = rtz - r.J.JIdx[0][i] * Jp_delta_x;
      rtz = rtz - r.J.JIdx[1][i] * Jp_delta_y;
      rtz = rtz - r.J.JabF[0][i] * da;
      rtz = rtz - r.J.JabF[1][i] * db;
      r.res_toZeroF[i] = rtz;
    }
    r.isLinearized = true;
  }

  // ------------------------------------------------------------ System::linearizeAll(false)
  double linearizeAll() {
    double E = 0;
    if (mt) {
      pool->reduce([this](int mn, int mx, double* s, int) {
        for (int k = mn; k < mx; k++) s[0] += linearize(res[activeResiduals[k]]);
      }, 0, (int)activeResiduals.size(), 0);
      E = pool->stats[0];
    } else {
      for (int k : activeResiduals) E += linearize(res[k]);
    }
    setNewFrameEnergyTH();
    return E;
  }

  void setNewFrameEnergyTH() {
    std::vector<float> all;
    all.reserve(activeResiduals.size());
    const int newest = nF - 1;
    for (int k : activeResiduals) {
      const ResO& r = res[k];
      if (r.state_NewEnergyWithOutlier >= 0 && r.target == newest) all.push_back((float)r.state_NewEnergyWithOutlier);
    }
    FrameO& nf = frames[newest];
    if (all.empty()) { nf.frameEnergyTH = 12 * 12 * PN; return; }
    int nthIdx = (int)(P.frameEnergyTHN * (float)all.size());
    std::nth_element(all.begin(), all.begin() + nthIdx, all.end());
    float nth = sqrtf(all[nthIdx]);
    nf.frameEnergyTH = nth * P.frameEnergyTHFacMedian;
    nf.frameEnergyTH = 26.0f * P.frameEnergyTHConstWeight + nf.frameEnergyTH * (1 - P.frameEnergyTHConstWeight);
    nf.frameEnergyTH = nf.frameEnergyTH * nf.frameEnergyTH;
    nf.frameEnergyTH *= P.overallEnergyTHWeight * P.overallEnergyTHWeight;
  }

  void applyResAll() {
    if (mt) {
      pool->reduce([this](int mn, int mx, double*, int) {
        for (int k = mn; k < mx; k++) applyRes(res[activeResiduals[k]]);
      }, 0, (int)activeResiduals.size(), 50);
    } else {
      for (int k : activeResiduals) applyRes(res[k]);
    }
  }

  // ------------------------------------------------------------ AccumulatedTopHessianSSE
  template <int mode>
  void topAddPoint(PointO& p, std::vector<AccApprox>& acc, int& nres) {
    float dd = p.deltaF;
    float bd_acc = 0, Hdd_acc = 0;
    float Hcd_acc[4] = {0, 0, 0, 0};
    for (int ri : p.residuals) {
      ResO& r = res[ri];
      if (mode == 0) { if (r.isLinearized || !r.isActive()) continue; }
      if (mode == 1) { if (!r.isLinearized || !r.isActive()) continue; }
      if (mode == 2) { if (!r.isActive()) continue; }
      const RawJ& J = r.J;
      int htIDX = r.host + r.target * nF;
      const float* dp = &adHTdeltaF[htIDX * 8];
      float resApprox[8];
      if (mode == 0) for (int i = 0; i < 8; i++) resApprox[i] = J.resF[i];
      if (mode == 2) for (int i = 0; i < 8; i++) resApprox[i] = r.res_toZeroF[i];
      if (mode == 1) {
        float jx = 0, jy = 0, cx = 0, cy = 0;
        for (int i = 0; i < 6; i++) { jx += J.Jpdxi[0][i] * dp[i]; jy += J.Jpdxi[1][i] * dp[i]; }
        for (int i = 0; i < 4; i++) { cx += J.Jpdc[0][i] * cDeltaF[i]; cy += J.Jpdc[1][i] * cDeltaF[i]; }
        float Jp_delta_x = jx + cx + J.Jpdd[0] * dd;
        float Jp_delta_y = jy + cy + J.Jpdd[1] * dd;
        float da = dp[6], db = dp[7];
        for (int i = 0; i < 8; i++) {
          float rtz = r.res_toZeroF[i];
          rtz = rtz + J.JIdx[0][i] * Jp_delta_x;
          rtz = rtz + J.JIdx[1][i] * Jp_delta_y;
          rtz = rtz + J.JabF[0][i] * da;
          rtz = rtz + J.JabF[1][i] * db;
          resApprox[i] = rtz;
        }
      }
      float JI_r0 = 0, JI_r1 = 0, Jab_r0 = 0, Jab_r1 = 0, rr = 0;
      for (int i = 0; i < PN; i++) {
        JI_r0 += resApprox[i] * J.JIdx[0][i];
        JI_r1 += resApprox[i] * J.JIdx[1][i];
        Jab_r0 += resApprox[i] * J.JabF[0][i];
        Jab_r1 += resApprox[i] * J.JabF[1][i];
        rr += resApprox[i] * resApprox[i];
      }
      acc[htIDX].update(J.Jpdc[0], J.Jpdxi[0], J.Jpdc[1], J.Jpdxi[1], J.JIdx2[0], J.JIdx2[1], J.JIdx2[3]);
      acc[htIDX].updateBotRight(J.Jab2[0], J.Jab2[1], Jab_r0, J.Jab2[3], Jab_r1, rr);
      acc[htIDX].updateTopRight(J.Jpdc[0], J.Jpdxi[0], J.Jpdc[1], J.Jpdxi[1], J.JabJIdx[0], J.JabJIdx[1],
                                J.JabJIdx[2], J.JabJIdx[3], JI_r0, JI_r1);
      float a = J.JIdx2[0] * J.Jpdd[0] + J.JIdx2[1] * J.Jpdd[1];
      float b = J.JIdx2[2] * J.Jpdd[0] + J.JIdx2[3] * J.Jpdd[1];
      bd_acc += JI_r0 * J.Jpdd[0] + JI_r1 * J.Jpdd[1];
      Hdd_acc += a * J.Jpdd[0] + b * J.Jpdd[1];
      for (int k = 0; k < 4; k++) Hcd_acc[k] += J.Jpdc[0][k] * a + J.Jpdc[1][k] * b;
      nres++;
    }
    if (mode == 0) {
      p.Hdd_accAF = Hdd_acc; p.bd_accAF = bd_acc;
      for (int k = 0; k < 4; k++) p.Hcd_accAF[k] = Hcd_acc[k];
    }
    if (mode == 1 || mode == 2) {
      p.Hdd_accLF = Hdd_acc; p.bd_accLF = bd_acc;
      for (int k = 0; k < 4; k++) p.Hcd_accLF[k] = Hcd_acc[k];
    }
    if (mode == 2) {
      for (int k = 0; k < 4; k++) p.Hcd_accAF[k] = 0;
      p.Hdd_accAF = 0; p.bd_accAF = 0;
    }
  }

  // stitchDoubleInternal over all threads' accumulators + stitchDoubleMT symmetrization
  void topStitch(std::vector<std::vector<AccApprox>>& acc, bool usePrior, std::vector<double>& H, std::vector<double>& b) {
    const int n = dim();
    const int toAgg = (int)acc.size();
    // per-"thread" partial H (reference: Hs[tid] via the pool, then summed serially)
    std::vector<std::vector<double>> Hs(T, std::vector<double>(n * n, 0.0)), bs(T, std::vector<double>(n, 0.0));
    auto internal = [&](int mn, int mx, int tid) {
      std::vector<double>& Ht = Hs[tid];
      std::vector<double>& bt = bs[tid];
      for (int k = mn; k < mx; k++) {
        int h = k % nF, t = k / nF;
        int hIdx = CP + h * 8, tIdx = CP + t * 8;
        int aidx = h + nF * t;
        double accH[169];
        for (int i = 0; i < 169; i++) accH[i] = 0;
        for (int tid2 = 0; tid2 < toAgg; tid2++) {
          acc[tid2][aidx].finish();
          if (acc[tid2][aidx].num == 0) continue;
          for (int i = 0; i < 169; i++) accH[i] += (double)acc[tid2][aidx].H[i];
        }
        double A88[64], A84[32], a8r[8], A44[16], a4r[4];
        for (int r = 0; r < 8; r++) {
          for (int c = 0; c < 8; c++) A88[r * 8 + c] = accH[(CP + r) * 13 + CP + c];
          for (int c = 0; c < 4; c++) A84[r * 4 + c] = accH[(CP + r) * 13 + c];
          a8r[r] = accH[(CP + r) * 13 + 12];
        }
        for (int r = 0; r < 4; r++) {
          for (int c = 0; c < 4; c++) A44[r * 4 + c] = accH[r * 13 + c];
          a4r[r] = accH[r * 13 + 12];
        }
        const double* aH = adHost[aidx].m;
        const double* aT = adTarget[aidx].m;
        double tmp[64], out[64], o84[32], o8[8];
        mm(aH, A88, tmp, 8, 8, 8);
        mmT(tmp, aH, out, 8, 8, 8);
        for (int r = 0; r < 8; r++) for (int c = 0; c < 8; c++) Ht[(hIdx + r) * n + hIdx + c] += out[r * 8 + c];
        mm(aT, A88, tmp, 8, 8, 8);
        mmT(tmp, aT, out, 8, 8, 8);
        for (int r = 0; r < 8; r++) for (int c = 0; c < 8; c++) Ht[(tIdx + r) * n + tIdx + c] += out[r * 8 + c];
        mm(aH, A88, tmp, 8, 8, 8);
        mmT(tmp, aT, out, 8, 8, 8);
        for (int r = 0; r < 8; r++) for (int c = 0; c < 8; c++) Ht[(hIdx + r) * n + tIdx + c] += out[r * 8 + c];
        mm(aH, A84, o84, 8, 8, 4);
        for (int r = 0; r < 8; r++) for (int c = 0; c < 4; c++) Ht[(hIdx + r) * n + c] += o84[r * 4 + c];
        mm(aT, A84, o84, 8, 8, 4);
        for (int r = 0; r < 8; r++) for (int c = 0; c < 4; c++) Ht[(tIdx + r) * n + c] += o84[r * 4 + c];
        for (int r = 0; r < 4; r++) for (int c = 0; c < 4; c++) Ht[r * n + c] += A44[r * 4 + c];
        mm(aH, a8r, o8, 8, 8, 1);
        for (int r = 0; r < 8; r++) bt[hIdx + r] += o8[r];
        mm(aT, a8r, o8, 8, 8, 1);
        for (int r = 0; r < 8; r++) bt[tIdx + r] += o8[r];
        for (int r = 0; r < 4; r++) bt[r] += a4r[r];
      }
      if (mn == 0 && usePrior) {
        for (int i = 0; i < CP; i++) {
          Ht[i * n + i] += cPrior[i];
          bt[i] += cPrior[i] * (double)cDeltaF[i];
        }
        for (int h = 0; h < nF; h++)
          for (int i = 0; i < 8; i++) {
            int j = CP + h * 8 + i;
            Ht[j * n + j] += frames[h].prior[i];
            bt[j] += frames[h].prior[i] * frames[h].delta_prior[i];
          }
      }
    };
    if (mt) pool->reduce([&](int mn, int mx, double*, int tid) { if (mn != mx) internal(mn, mx, tid); }, 0, nF * nF, 0);
    else internal(0, nF * nF, 0);
    H = Hs[0];
    b = bs[0];
    for (int t = 1; t < T; t++) {
      for (int i = 0; i < n * n; i++) H[i] += Hs[t][i];
      for (int i = 0; i < n; i++) b[i] += bs[t][i];
    }
    for (int h = 0; h < nF; h++) {
      int hIdx = CP + h * 8;
      for (int r = 0; r < 8; r++) for (int c = 0; c < 4; c++) H[c * n + hIdx + r] = H[(hIdx + r) * n + c];
      for (int t = h + 1; t < nF; t++) {
        int tIdx = CP + t * 8;
        for (int r = 0; r < 8; r++) for (int c = 0; c < 8; c++) H[(hIdx + r) * n + tIdx + c] += H[(tIdx + c) * n + hIdx + r];
        for (int r = 0; r < 8; r++) for (int c = 0; c < 8; c++) H[(tIdx + r) * n + hIdx + c] = H[(hIdx + c) * n + tIdx + r];
      }
    }
  }

  // mode 0: accumulateAF_MT, 1: accumulateLF_MT (Src/EnergyFunctional.cpp:155-220); 2: the marginalization pass of
  // marginalizePointsF over `subset` (Src/EnergyFunctional.cpp:572-583, accSSE_top_A->addPoint<2>)
  void accumulateTop(int mode, std::vector<double>& H, std::vector<double>& b, const std::vector<int>* subset = nullptr) {
    auto& acc = mode == 1 ? accTopL : accTopA;
    auto& nres = mode == 1 ? nresL : nresA;
    acc.assign(T, std::vector<AccApprox>(nF * nF));
    nres.assign(T, 0);
    for (auto& v : acc) for (auto& a : v) a.initialize();
    const int N = subset ? (int)subset->size() : (int)points.size();
    auto body = [&](int mn, int mx, int tid) {
      for (int q = mn; q < mx; q++) {
        PointO& pt = points[subset ? (*subset)[q] : q];
        if (mode == 0) topAddPoint<0>(pt, acc[tid], nres[tid]);
        else if (mode == 1) topAddPoint<1>(pt, acc[tid], nres[tid]);
        else topAddPoint<2>(pt, acc[tid], nres[tid]);
      }
    };
    if (mt) pool->reduce([&](int mn, int mx, double*, int tid) { body(mn, mx, tid); }, 0, N, 50);
    else body(0, N, 0);
    topStitch(acc, mode == 1, H, b);
    if (mode == 0) { lastResInA = 0; for (int v : nres) lastResInA += v; }
  }

  // ------------------------------------------------------------ AccumulatedSCHessianSSE
  void scAddPoint(PointO& p, bool shiftPriorToZero, int tid) {
    int ngoodres = 0;
    for (int ri : p.residuals) if (res[ri].isActive()) ngoodres++;
    if (ngoodres == 0) {
      p.HdiF = 0; p.bdSumF = 0; p.idepth_hessian = 0; p.maxRelBaseline = 0;
      return;
    }
    float H = p.Hdd_accAF + p.Hdd_accLF + p.priorF;
    if (H < 1e-10) H = 1e-10;
    p.idepth_hessian = H;
    p.HdiF = (float)(1.0 / H);
    p.bdSumF = p.bd_accAF + p.bd_accLF;
    if (shiftPriorToZero) p.bdSumF += p.priorF * p.deltaF;
    float Hcd[4];
    for (int k = 0; k < 4; k++) Hcd[k] = p.Hcd_accAF[k] + p.Hcd_accLF[k];
    accHcc[tid].update(Hcd, Hcd, p.HdiF);
    accbc[tid].update(Hcd, p.bdSumF * p.HdiF);
    const int nF2 = nF * nF;
    for (int r1i : p.residuals) {
      ResO& r1 = res[r1i];
      if (!r1.isActive()) continue;
      int r1ht = r1.host + r1.target * nF;
      for (int r2i : p.residuals) {
        ResO& r2 = res[r2i];
        if (!r2.isActive()) continue;
        accD[tid][r1ht + r2.target * nF2].update(r1.JpJdF, r2.JpJdF, p.HdiF);
      }
      accE[tid][r1ht].update(r1.JpJdF, Hcd, p.HdiF);
      accEB[tid][r1ht].update(r1.JpJdF, p.HdiF * p.bdSumF);
    }
  }

  void accumulateSC(std::vector<double>& H, std::vector<double>& b, const std::vector<int>* subset = nullptr,
                    bool shiftPriorToZero = true) {
    const int n = dim();
    accE.assign(T, std::vector<AccXX<8, 4>>(nF * nF));
    accEB.assign(T, std::vector<AccX<8>>(nF * nF));
    accD.assign(T, std::vector<AccXX<8, 8>>(nF * nF * nF));
    accHcc.assign(T, AccXX<4, 4>());
    accbc.assign(T, AccX<4>());
    for (int t = 0; t < T; t++) {
      for (auto& a : accE[t]) a.initialize();
      for (auto& a : accEB[t]) a.initialize();
      for (auto& a : accD[t]) a.initialize();
      accHcc[t].initialize();
      accbc[t].initialize();
    }
    const int N = subset ? (int)subset->size() : (int)points.size();
    auto body = [&](int mn, int mx, int tid) {
      for (int q = mn; q < mx; q++) scAddPoint(points[subset ? (*subset)[q] : q], shiftPriorToZero, tid);
    };
    if (mt) pool->reduce([&](int mn, int mx, double*, int tid) { body(mn, mx, tid); }, 0, N, 50);
    else body(0, N, 0);

    std::vector<std::vector<double>> Hs(T, std::vector<double>(n * n, 0.0)), bs(T, std::vector<double>(n, 0.0));
    const int nf = nF, nframes2 = nF * nF;
    auto internal = [&](int mn, int mx, int tid) {
      std::vector<double>& Ht = Hs[tid];
      std::vector<double>& bt = bs[tid];
      for (int k = mn; k < mx; k++) {
        int i = k % nf, j = k / nf;
        int iIdx = CP + i * 8, jIdx = CP + j * 8;
        int ijIdx = i + nf * j;
        double Hpc[32] = {0}, bp[8] = {0};
        for (int t2 = 0; t2 < T; t2++) {
          accE[t2][ijIdx].finish();
          accEB[t2][ijIdx].finish();
          for (int q = 0; q < 32; q++) Hpc[q] += (double)accE[t2][ijIdx].A1m[q];
          for (int q = 0; q < 8; q++) bp[q] += (double)accEB[t2][ijIdx].A1m[q];
        }
        double o84[32], o8[8];
        mm(adHost[ijIdx].m, Hpc, o84, 8, 8, 4);
        for (int r = 0; r < 8; r++) for (int c = 0; c < 4; c++) Ht[(iIdx + r) * n + c] += o84[r * 4 + c];
        mm(adTarget[ijIdx].m, Hpc, o84, 8, 8, 4);
        for (int r = 0; r < 8; r++) for (int c = 0; c < 4; c++) Ht[(jIdx + r) * n + c] += o84[r * 4 + c];
        mm(adHost[ijIdx].m, bp, o8, 8, 8, 1);
        for (int r = 0; r < 8; r++) bt[iIdx + r] += o8[r];
        mm(adTarget[ijIdx].m, bp, o8, 8, 8, 1);
        for (int r = 0; r < 8; r++) bt[jIdx + r] += o8[r];
        for (int kk = 0; kk < nf; kk++) {
          int kIdx = CP + kk * 8;
          int ijkIdx = ijIdx + kk * nframes2;
          int ikIdx = i + nf * kk;
          double D[64] = {0};
          bool any = false;
          for (int t2 = 0; t2 < T; t2++) {
            accD[t2][ijkIdx].finish();
            if (accD[t2][ijkIdx].num == 0) continue;
            any = true;
            for (int q = 0; q < 64; q++) D[q] += (double)accD[t2][ijkIdx].A1m[q];
          }
          (void)any;
          double tmp[64], out[64];
          mm(adHost[ijIdx].m, D, tmp, 8, 8, 8);
          mmT(tmp, adHost[ikIdx].m, out, 8, 8, 8);
          for (int r = 0; r < 8; r++) for (int c = 0; c < 8; c++) Ht[(iIdx + r) * n + iIdx + c] += out[r * 8 + c];
          mm(adTarget[ijIdx].m, D, tmp, 8, 8, 8);
          mmT(tmp, adTarget[ikIdx].m, out, 8, 8, 8);
          for (int r = 0; r < 8; r++) for (int c = 0; c < 8; c++) Ht[(jIdx + r) * n + kIdx + c] += out[r * 8 + c];
          mmT(tmp, adHost[ikIdx].m, out, 8, 8, 8);
          for (int r = 0; r < 8; r++) for (int c = 0; c < 8; c++) Ht[(jIdx + r) * n + iIdx + c] += out[r * 8 + c];
          mm(adHost[ijIdx].m, D, tmp, 8, 8, 8);
          mmT(tmp, adTarget[ikIdx].m, out, 8, 8, 8);
          for (int r = 0; r < 8; r++) for (int c = 0; c < 8; c++) Ht[(iIdx + r) * n + kIdx + c] += out[r * 8 + c];
        }
      }
      if (mn == 0) {
        for (int t2 = 0; t2 < T; t2++) {
          accHcc[t2].finish();
          accbc[t2].finish();
          for (int r = 0; r < 4; r++) for (int c = 0; c < 4; c++) Ht[r * n + c] += (double)accHcc[t2].A1m[r * 4 + c];
          for (int r = 0; r < 4; r++) bt[r] += (double)accbc[t2].A1m[r];
        }
      }
    };
    if (mt) pool->reduce([&](int mn, int mx, double*, int tid) { if (mn != mx) internal(mn, mx, tid); }, 0, nF * nF, 0);
    else internal(0, nF * nF, 0);
    H = Hs[0];
    b = bs[0];
    for (int t = 1; t < T; t++) {
      for (int i = 0; i < n * n; i++) H[i] += Hs[t][i];
      for (int i = 0; i < n; i++) b[i] += bs[t][i];
    }
    for (int h = 0; h < nF; h++) {
      int hIdx = CP + h * 8;
      for (int r = 0; r < 8; r++) for (int c = 0; c < 4; c++) H[c * n + hIdx + r] = H[(hIdx + r) * n + c];
    }
  }

  // ------------------------------------------------------------ marginalization of points
  // System::flagPointsForRemoval's per-point part for the points to marginalize (Src/Mapping.cpp:280-293:
  // resetOOB, linearize, isLinearized = false, applyRes, fixLinearizationF of the active residuals), then
  // EnergyFunctional::marginalizePointsF (Src/EnergyFunctional.cpp:545-609): priorF *= idepthFixPriorMargFac,
  // top addPoint<2> + SC addPoint(p, false), M - Msc, HM += margWeightFac (M - Msc), bM likewise
  // (SOLVER_ORTHOGONALIZE_POINTMARG is off in setting_solverMode, Src/Settings.cpp:114).
  void marginalizePoints(const std::vector<int>& pts, float priorMargFac, float margWeightFac) {
    setDeltaF();
    for (int pi : pts) {
      for (int ri : points[pi].residuals) {
        ResO& r = res[ri];
        r.resetOOB();
        linearize(r);
        r.isLinearized = false;
        applyRes(r);
        if (r.isActive()) fixLinearizationF(r);
      }
    }
    for (int pi : pts) points[pi].priorF *= priorMargFac;
    std::vector<double> M, Mb, Msc, Mbsc;
    accumulateTop(2, M, Mb, &pts);
    accumulateSC(Msc, Mbsc, &pts, false);
    const int n = dim();
    for (int i = 0; i < n * n; i++) HM[i] += margWeightFac * (M[i] - Msc[i]);
    for (int i = 0; i < n; i++) bM[i] += margWeightFac * (Mb[i] - Mbsc[i]);
  }

  // ------------------------------------------------------------ EnergyFunctional::marginalizeFrame
  // (Src/EnergyFunctional.cpp:456-543): move frame f's 8 rows / cols of HM / bM to the end, add its prior,
  // scale by 1/sqrt(|diag| + 10), Schur-complement the 8x8 block out (hpi = 0.5f*(hpi+hpi) kept as in the
  // reference: a no-op), unscale, symmetrize.  Outputs the (dim-8) prior; the window itself is not changed.
  void marginalizeFrame(int f, std::vector<double>& HMo, std::vector<double>& bMo) {
    setDeltaF();  // EFDeltaValid
    const int odim = dim(), ndim = odim - 8;
    std::vector<int> perm(odim);  // new position -> old index
    int q = 0;
    for (int i = 0; i < odim; i++)
      if (i < CP + 8 * f || i >= CP + 8 * f + 8) perm[q++] = i;
    for (int i = 0; i < 8; i++) perm[q++] = CP + 8 * f + i;
    std::vector<double> H(odim * odim), b(odim);
    for (int r = 0; r < odim; r++) {
      b[r] = bM[perm[r]];
      for (int c = 0; c < odim; c++) H[r * odim + c] = HM[perm[r] * odim + perm[c]];
    }
    const FrameO& fr = frames[f];
    for (int i = 0; i < 8; i++) {
      H[(ndim + i) * odim + ndim + i] += fr.prior[i];
      b[ndim + i] += fr.prior[i] * fr.delta_prior[i];
    }
    std::vector<double> S(odim), SI(odim);
    for (int i = 0; i < odim; i++) {
      S[i] = std::sqrt(std::fabs(H[i * odim + i]) + 10.0);
      SI[i] = 1.0 / S[i];
    }
    for (int r = 0; r < odim; r++) {
      for (int c = 0; c < odim; c++) H[r * odim + c] = SI[r] * H[r * odim + c] * SI[c];
      b[r] = SI[r] * b[r];
    }
    double hpi[64], inv[64];
    for (int r = 0; r < 8; r++)
      for (int c = 0; c < 8; c++) hpi[r * 8 + c] = H[(ndim + r) * odim + ndim + c];
    for (int i = 0; i < 64; i++) hpi[i] = 0.5f * (hpi[i] + hpi[i]);
    invert_pp(hpi, inv, 8);
    for (int i = 0; i < 64; i++) inv[i] = 0.5f * (inv[i] + inv[i]);
    // bli = H(bottom, left)^T * hpi  (ndim x 8)
    std::vector<double> bli(ndim * 8, 0.0);
    for (int r = 0; r < ndim; r++)
      for (int c = 0; c < 8; c++) {
        double acc = 0;
        for (int k = 0; k < 8; k++) acc += H[(ndim + k) * odim + r] * inv[k * 8 + c];
        bli[r * 8 + c] = acc;
      }
    for (int r = 0; r < ndim; r++) {
      for (int c = 0; c < ndim; c++) {
        double acc = 0;
        for (int k = 0; k < 8; k++) acc += bli[r * 8 + k] * H[(ndim + k) * odim + c];
        H[r * odim + c] -= acc;
      }
      double acc = 0;
      for (int k = 0; k < 8; k++) acc += bli[r * 8 + k] * b[ndim + k];
      b[r] -= acc;
    }
    HMo.assign(ndim * ndim, 0.0);
    bMo.assign(ndim, 0.0);
    for (int r = 0; r < ndim; r++) {
      bMo[r] = S[r] * b[r];
      for (int c = 0; c < ndim; c++) {
        const double u = S[r] * H[r * odim + c] * S[c], ut = S[c] * H[c * odim + r] * S[r];
        HMo[r * ndim + c] = 0.5 * (u + ut);
      }
    }
  }
  // inverse by Gauss-Jordan elimination with partial pivoting (Eigen's PartialPivLU-based inverse for 8x8)
  static void invert_pp(const double* A, double* X, int n) {
    std::vector<double> M(A, A + n * n);
    for (int i = 0; i < n * n; i++) X[i] = 0;
    for (int i = 0; i < n; i++) X[i * n + i] = 1;
    for (int c = 0; c < n; c++) {
      int pr = c;
      for (int r = c + 1; r < n; r++)
        if (std::fabs(M[r * n + c]) > std::fabs(M[pr * n + c])) pr = r;
      if (pr != c)
        for (int k = 0; k < n; k++) { std::swap(M[c * n + k], M[pr * n + k]); std::swap(X[c * n + k], X[pr * n + k]); }
      const double d = M[c * n + c];
      for (int k = 0; k < n; k++) { M[c * n + k] /= d; X[c * n + k] /= d; }
      for (int r = 0; r < n; r++) {
        if (r == c) continue;
        const double f = M[r * n + c];
        if (f == 0.0) continue;
        for (int k = 0; k < n; k++) { M[r * n + k] -= f * M[c * n + k]; X[r * n + k] -= f * X[c * n + k]; }
      }
    }
  }

  // ------------------------------------------------------------ nullspaces (System::getNullspaces)
  void getNullspaces() {
    const int n = dim();
    ns_pose.clear();
    ns_scale.clear();
    for (int i = 0; i < 6; i++) {
      std::vector<double> v(n, 0.0);
      for (auto& f : frames) {
        for (int k = 0; k < 6; k++) v[CP + f.idx * 8 + k] = f.nullspaces_pose[i][k];
        for (int k = 0; k < 3; k++) v[CP + f.idx * 8 + k] *= SCALE_XI_TRANS_INVERSE;
        for (int k = 3; k < 6; k++) v[CP + f.idx * 8 + k] *= SCALE_XI_ROT_INVERSE;
      }
      ns_pose.push_back(v);
    }
    std::vector<double> v(n, 0.0);
    for (auto& f : frames) {
      for (int k = 0; k < 6; k++) v[CP + f.idx * 8 + k] = f.nullspaces_scale[k];
      for (int k = 0; k < 3; k++) v[CP + f.idx * 8 + k] *= SCALE_XI_TRANS_INVERSE;
      for (int k = 3; k < 6; k++) v[CP + f.idx * 8 + k] *= SCALE_XI_ROT_INVERSE;
    }
    ns_scale.push_back(v);
  }

  void orthogonalize(std::vector<double>& x) {
    std::vector<std::vector<double>> ns = ns_pose;
    ns.insert(ns.end(), ns_scale.begin(), ns_scale.end());
    const int n = dim();
    std::vector<double> Pm;
    nullspace_projector(ns, n, P.solverModeDelta, Pm);
    std::vector<double> y(n, 0.0);
    for (int i = 0; i < n; i++) {
      double s = 0;
      for (int j = 0; j < n; j++) s += Pm[i * n + j] * x[j];
      y[i] = s;
    }
    for (int i = 0; i < n; i++) x[i] -= y[i];
  }

  // ------------------------------------------------------------ solveSystemF + resubstitute
  std::vector<double> HA, bA, HL, bL, Hsc, bsc;

  void solveSystemF(int iteration, std::vector<double>& xout) {
    double lambda = 1e-5;  // SOLVER_FIX_LAMBDA
    const int n = dim();
    accumulateTop(0, HA, bA);
    accumulateTop(1, HL, bL);
    accumulateSC(Hsc, bsc);
    // bM_top = bM + HM * getStitchedDeltaF()
    std::vector<double> delta(n);
    for (int i = 0; i < CP; i++) delta[i] = (double)cDeltaF[i];
    for (int h = 0; h < nF; h++) for (int i = 0; i < 8; i++) delta[CP + 8 * h + i] = frames[h].delta[i];
    std::vector<double> bMt(n);
    for (int i = 0; i < n; i++) {
      double s = 0;
      for (int j = 0; j < n; j++) s += HM[i * n + j] * delta[j];
      bMt[i] = bM[i] + s;
    }
    std::vector<double> Hf(n * n), bf(n);
    for (int i = 0; i < n * n; i++) Hf[i] = HL[i] + HM[i] + HA[i];
    for (int i = 0; i < n; i++) bf[i] = bL[i] + bMt[i] + bA[i] - bsc[i];
    for (int i = 0; i < n; i++) Hf[i * n + i] *= (1 + lambda);
    const double sc = (double)(1.0f / (1 + lambda));
    for (int i = 0; i < n * n; i++) Hf[i] -= Hsc[i] * sc;
    std::vector<double> S(n);
    for (int i = 0; i < n; i++) S[i] = 1.0 / std::sqrt(Hf[i * n + i] + 10);
    std::vector<double> Hs(n * n), bs(n);
    for (int i = 0; i < n; i++)
      for (int j = 0; j < n; j++) Hs[i * n + j] = S[i] * Hf[i * n + j] * S[j];
    for (int i = 0; i < n; i++) bs[i] = S[i] * bf[i];
    std::vector<double> y;
    ldlt_solve(Hs, n, bs, y);
    std::vector<double> x(n);
    for (int i = 0; i < n; i++) x[i] = S[i] * y[i];
    if (iteration >= 2) orthogonalize(x);
    lastX = x;
    resubstitute(x);
    xout = x;
  }

  void resubstitute(const std::vector<double>& x) {
    std::vector<float> xF(dim());
    for (int i = 0; i < dim(); i++) xF[i] = (float)x[i];
    for (int i = 0; i < 4; i++) calib.step[i] = -x[i];
    std::vector<float> xAd(nF * nF * 8);
    float cstep[4] = {xF[0], xF[1], xF[2], xF[3]};
    for (int h = 0; h < nF; h++) {
      for (int i = 0; i < 8; i++) frames[h].step[i] = -x[CP + 8 * h + i];
      frames[h].step[8] = frames[h].step[9] = 0;
      for (int t = 0; t < nF; t++) {
        const float* aH = adHostF[h + nF * t].m;
        const float* aT = adTargetF[h + nF * t].m;
        for (int c = 0; c < 8; c++) {
          float s1 = 0, s2 = 0;
          for (int r = 0; r < 8; r++) s1 += xF[CP + 8 * h + r] * aH[r * 8 + c];
          for (int r = 0; r < 8; r++) s2 += xF[CP + 8 * t + r] * aT[r * 8 + c];
          xAd[(nF * h + t) * 8 + c] = s1 + s2;
        }
      }
    }
    auto body = [&](int mn, int mx) {
      for (int k = mn; k < mx; k++) {
        PointO& p = points[k];
        int ngood = 0;
        for (int ri : p.residuals) if (res[ri].isActive()) ngood++;
        if (ngood == 0) { p.step = 0; continue; }
        float b = p.bdSumF;
        float dot = 0;
        for (int i = 0; i < 4; i++) dot += cstep[i] * (p.Hcd_accAF[i] + p.Hcd_accLF[i]);
        b -= dot;
        for (int ri : p.residuals) {
          ResO& r = res[ri];
          if (!r.isActive()) continue;
          const float* xa = &xAd[(r.host * nF + r.target) * 8];
          float d = 0;
          for (int i = 0; i < 8; i++) d += xa[i] * r.JpJdF[i];
          b -= d;
        }
        p.step = -b * p.HdiF;
      }
    };
    if (mt) pool->reduce([&](int mn, int mx, double*, int) { body(mn, mx); }, 0, (int)points.size(), 50);
    else body(0, (int)points.size());
  }

  // ------------------------------------------------------------ System::backupState / doStepFromBackup
  void backupState() {
    for (int i = 0; i < 4; i++) calib.value_backup[i] = calib.value[i];
    for (auto& f : frames) {
      for (int i = 0; i < 10; i++) f.state_backup[i] = f.state[i];
      for (int pi : f.points) points[pi].idepth_backup = points[pi].idepth;
    }
  }

  bool doStepFromBackup() {
    const float stepfacC = 1, stepfacD = 1;
    double pstepfac[10];
    for (int i = 0; i < 10; i++) pstepfac[i] = 1;
    float sumA = 0, sumB = 0, sumT = 0, sumR = 0, sumID = 0, numID = 0, sumNID = 0;
    double nv[4];
    for (int i = 0; i < 4; i++) nv[i] = calib.value_backup[i] + stepfacC * calib.step[i];
    calib.setValue(nv);
    for (auto& f : frames) {
      double s[10];
      for (int i = 0; i < 10; i++) s[i] = f.state_backup[i] + pstepfac[i] * f.step[i];
      f.setState(s);
      sumA += f.step[6] * f.step[6];
      sumB += f.step[7] * f.step[7];
      sumT += f.step[0] * f.step[0] + f.step[1] * f.step[1] + f.step[2] * f.step[2];
      sumR += f.step[3] * f.step[3] + f.step[4] * f.step[4] + f.step[5] * f.step[5];
      for (int pi : f.points) {
        PointO& p = points[pi];
        p.idepth = p.idepth_backup + stepfacD * p.step;
        sumID += p.step * p.step;
        sumNID += fabsf(p.idepth_backup);
        numID++;
        float nz = p.idepth_backup + stepfacD * p.step;
        p.idepth_zero = nz;
        p.nullspaces_scale = -(nz * 1.001 - nz / 1.001) * 500;
      }
    }
    sumA /= frames.size(); sumB /= frames.size(); sumR /= frames.size(); sumT /= frames.size();
    sumID /= numID; sumNID /= numID;
    setPrecalcValues();
    const float th = P.thOptIterations;
    return sqrtf(sumA) < 0.0005 * th && sqrtf(sumB) < 0.00005 * th && sqrtf(sumR) < 0.00005 * th &&
           sqrtf(sumT) * sumNID < 0.00005 * th;
  }

  // EnergyFunctional::calcLEnergyF_MT (Src/EnergyFunctional.cpp:289-368): frame priors, calib prior, and per
  // IndexThreadReduce chunk of 50 points an Accumulator11 over the linearized active residuals' (2 res_toZero +
  // J delta) J delta and the point prior deltaF^2 priorF
  double calcLEnergy() {
    double E = 0;
    for (const auto& f : frames) {
      double s = 0;
      for (int i = 0; i < 8; i++) s += f.delta_prior[i] * f.prior[i] * f.delta_prior[i];
      E += s;
    }
    {
      float s = 0.f;
      for (int i = 0; i < 4; i++) s += cDeltaF[i] * cPriorF[i] * cDeltaF[i];
      E += s;
    }
    auto body = [this](int mn, int mx, double* st, int) {
      float A = 0.f;  // Accumulator11, lane 0 (updateSingle / updateSingleNoShift); <= 50 updates: no shiftUp
      float lanes[4] = {0.f, 0.f, 0.f, 0.f};
      for (int i = mn; i < mx; i++) {
        const PointO& p = points[i];
        const float dd = p.deltaF;
        for (int ri : p.residuals) {
          const ResO& r = res[ri];
          if (!r.isLinearized || !r.isActive()) continue;
          const float* dp = &adHTdeltaF[(r.host + nF * r.target) * 8];
          float jx = 0, jy = 0, cx = 0, cy = 0;
          for (int k = 0; k < 6; k++) { jx += r.J.Jpdxi[0][k] * dp[k]; jy += r.J.Jpdxi[1][k] * dp[k]; }
          for (int k = 0; k < 4; k++) { cx += r.J.Jpdc[0][k] * cDeltaF[k]; cy += r.J.Jpdc[1][k] * cDeltaF[k]; }
          const float Jpx = jx + cx + r.J.Jpdd[0] * dd, Jpy = jy + cy + r.J.Jpdd[1] * dd;
          for (int k = 0; k < PN; k++) {  // updateSSENoShift over pattern quads: lane k % 4
            float Jd = r.J.JIdx[0][k] * Jpx;
            Jd = Jd + r.J.JIdx[1][k] * Jpy;
            Jd = Jd + r.J.JabF[0][k] * dp[6];
            Jd = Jd + r.J.JabF[1][k] * dp[7];
            float r0 = r.res_toZeroF[k];
            r0 = r0 + r0;
            r0 = r0 + Jd;
            lanes[k % 4] += Jd * r0;
          }
        }
        lanes[0] += p.deltaF * p.deltaF * p.priorF;  // updateSingle
      }
      (void)A;
      st[0] += (double)(((lanes[0] + lanes[1]) + lanes[2]) + lanes[3]);  // finish(): shiftUp(true), lane sum
    };
    if (mt) {
      pool->reduce([&](int mn, int mx, double* st, int t) { body(mn, mx, st, t); }, 0, (int)points.size(), 50);
      return E + pool->stats[0];
    }
    double s = 0;
    for (int i = 0; i < (int)points.size(); i += 50) {
      double st[1] = {0};
      body(i, std::min(i + 50, (int)points.size()), st, 0);
      s += st[0];
    }
    return E + s;
  }

  // EnergyFunctional::calcMEnergyF (Src/EnergyFunctional.cpp:277-286): delta . (2 bM + HM delta)
  double calcMEnergy() {
    const int n = dim();
    std::vector<double> d(n);
    for (int i = 0; i < 4; i++) d[i] = (double)cDeltaF[i];
    for (int f = 0; f < nF; f++)
      for (int i = 0; i < 8; i++) d[4 + 8 * f + i] = frames[f].delta[i];
    double E = 0;
    for (int r = 0; r < n; r++) {
      double hd = 0;
      for (int k = 0; k < n; k++) hd += HM[r * n + k] * d[k];
      E += d[r] * (2 * bM[r] + hd);
    }
    return E;
  }

  // System::optimize's tail (Src/FullSystemOptimize.cpp:498-509): the newest frame's setEvalPT(PRE_worldToCam,
  // (0,..,0, a, b, 0, 0)) (Include/Frame.h:213-218), setAdjointsF, setPrecalcValues, then linearizeAll(true)
  // (:19-52, :102-124): linearize + applyRes(true) per active residual; for residuals still active the point's
  // maxRelBaseline / numGoodResiduals (isNew is never cleared in the reference); setNewFrameEnergyTH.
  double fixLinearization(float* relBL, int* nGood, uint8_t* drop) {
    FrameO& f = frames[nF - 1];
    double nsz[10] = {0, 0, 0, 0, 0, 0, f.state[6], f.state[7], 0, 0};
    f.evalPT = f.PRE_worldToCam;
    f.setState(nsz);
    f.setStateZero(nsz);
    setAdjointsF();
    setPrecalcValues();
    double E = 0;
    for (int k : activeResiduals) {
      ResO& r = res[k];
      E += linearize(r);
      applyRes(r);
      if (r.isActive()) {
        const PointO& p = points[r.point];
        const Precalc& pc = precalc[r.host * nF + r.target];
        float pi[3], pt[3];
        for (int i = 0; i < 3; i++) {
          pi[i] = pc.PRE_KRKiTll[i * 3 + 0] * p.u + pc.PRE_KRKiTll[i * 3 + 1] * p.v + pc.PRE_KRKiTll[i * 3 + 2] * 1.f;
          pt[i] = pi[i] + pc.PRE_KtTll[i] * p.idepth;
        }
        const float dx = pi[0] / pi[2] - pt[0] / pt[2], dy = pi[1] / pi[2] - pt[1] / pt[2];
        const float relBS = 0.01 * std::sqrt(dx * dx + dy * dy);
        if (relBL && relBS > relBL[r.point]) relBL[r.point] = relBS;
        if (nGood) nGood[r.point]++;
      } else if (drop) {
        drop[k] = 1;
      }
    }
    setNewFrameEnergyTH();
    return E;
  }

  // K loop bodies of System::optimize continuing from the current linearization
  void iterate(int it0, int K, double* energies) {
    for (int k = 0; k < K; k++) {
      backupState();
      getNullspaces();
      std::vector<double> x;
      solveSystemF(it0 + k, x);
      doStepFromBackup();
      double E = linearizeAll();
      if (energies) energies[k] = E;
      applyResAll();
    }
  }

  // System::optimize core loop (Src/FullSystemOptimize.cpp:362-494), forceAcceptStep=true
  int optimize(int mnumOptIts, bool allowBreak, double* energies) {
    if (nF < 2) return 0;
    if (nF < 3) mnumOptIts = 20;
    if (nF < 4) mnumOptIts = 15;
    activeResiduals.clear();
    for (auto& f : frames)
      for (int pi : f.points)
        for (int ri : points[pi].residuals)
          if (!res[ri].isLinearized) { activeResiduals.push_back(ri); res[ri].resetOOB(); }
    double E = linearizeAll();
    if (energies) energies[0] = E;
    applyResAll();
    int it = 0;
    for (; it < mnumOptIts; it++) {
      backupState();
      getNullspaces();
      std::vector<double> x;
      solveSystemF(it, x);
      bool canbreak = doStepFromBackup();
      E = linearizeAll();
      if (energies) energies[it + 1] = E;
      applyResAll();
      if (allowBreak && canbreak && it >= P.minOptIterations) { it++; break; }
    }
    return it;
  }
};

}  // namespace hso

// ================================================================ C API
using namespace hso;

extern "C" {

void hso_params_default(hs_params* p) { params_default(p); }

void* hso_ba_create(const hs_params* params, const hs_camera* cam, int nF, const hs_frame* frames,
                    const float* const* images, const hs_points* pts, const hs_residuals* rs, int nthreads) {
  if (nF < 1 || nF > HS_MAX_FRAMES) return nullptr;
  BA* ba = new BA();
  if (params) ba->P = *params; else params_default(&ba->P);
  ba->T = nthreads < 1 ? 1 : nthreads;
  ba->mt = ba->T > 1;
  ba->pool.reset(new Pool(ba->T));
  ba->calib.W = cam->width;
  ba->calib.H = cam->height;
  double vs[4] = {cam->fx, cam->fy, cam->cx, cam->cy};
  for (int i = 0; i < 4; i++) ba->calib.value_zero[i] = 0;
  ba->calib.setValueScaled(vs);
  for (int i = 0; i < 4; i++) ba->calib.value_zero[i] = ba->calib.value[i];
  for (int i = 0; i < 4; i++) { ba->calib.value_minus_value_zero[i] = 0; ba->calib.step[i] = 0; }
  ba->nF = nF;
  ba->frames.resize(nF);
  for (int i = 0; i < nF; i++) {
    FrameO& f = ba->frames[i];
    f.id = frames[i].id;
    f.idx = i;
    f.ab_exposure = frames[i].ab_exposure;
    f.frameEnergyTH = frames[i].frameEnergyTH;
    f.evalPT = SE3::fromData(frames[i].worldToCam_evalPT);
    f.img = images[i];
    f.setState(frames[i].state);
    f.setStateZero(frames[i].state_zero);
    f.takeData(ba->P);
  }
  ba->points.resize(pts->n);
  for (int i = 0; i < pts->n; i++) {
    PointO& p = ba->points[i];
    p.u = pts->u[i]; p.v = pts->v[i];
    p.idepth = pts->idepth[i];
    p.idepth_zero = pts->idepth_zero[i];
    p.host = pts->host[i];
    for (int k = 0; k < 8; k++) { p.color[k] = pts->color[i * 8 + k]; p.weights[k] = pts->weights[i * 8 + k]; }
    p.hasDepthPrior = pts->has_depth_prior ? pts->has_depth_prior[i] != 0 : false;
    p.priorF = p.hasDepthPrior ? ba->P.idepthFixPrior * SCALE_IDEPTH * SCALE_IDEPTH : 0;
    p.deltaF = p.idepth - p.idepth_zero;
    ba->frames[p.host].points.push_back(i);
  }
  ba->res.resize(rs->n);
  for (int i = 0; i < rs->n; i++) {
    ResO& r = ba->res[i];
    r.point = rs->point[i];
    r.host = ba->points[r.point].host;
    r.target = rs->target[i];
    if (rs->state) r.state_state = rs->state[i];
    ba->points[r.point].residuals.push_back(i);
  }
  const int n = ba->dim();
  ba->HM.assign(n * n, 0.0);
  ba->bM.assign(n, 0.0);
  ba->setAdjointsF();
  ba->setPrecalcValues();
  return ba;
}

void hso_ba_destroy(void* h) { delete (BA*)h; }

int hso_ba_optimize(void* h, int iters, int allow_break, double* energies) {
  return ((BA*)h)->optimize(iters, allow_break != 0, energies);
}

void hso_ba_iterate(void* h, int it0, int K, double* energies) { ((BA*)h)->iterate(it0, K, energies); }

/* one linearizeAll(false) over all residuals (resetOOB semantics at first call) */
double hso_ba_linearize_all(void* h, int reset) {
  BA* ba = (BA*)h;
  if (reset || ba->activeResiduals.empty()) {
    ba->activeResiduals.clear();
    for (auto& f : ba->frames)
      for (int pi : f.points)
        for (int ri : ba->points[pi].residuals)
          if (!ba->res[ri].isLinearized) { ba->activeResiduals.push_back(ri); if (reset) ba->res[ri].resetOOB(); }
  }
  return ba->linearizeAll();
}
void hso_ba_apply_res(void* h) { ((BA*)h)->applyResAll(); }

/* calcLEnergyF_MT / calcMEnergyF on the current state (setDeltaF first, as the reference's EFDeltaValid asserts) */
void hso_ba_calc_energies(void* h, double* L, double* M) {
  BA* ba = (BA*)h;
  ba->setDeltaF();
  if (L) *L = ba->calcLEnergy();
  if (M) *M = ba->calcMEnergy();
}

/* System::optimize's tail + linearizeAll(true): returns its energy; relBL / nGood [n points] updated in place,
   drop [n residuals] set to 1 for the toRemove list (entries of other residuals untouched) */
double hso_ba_fix_linearization(void* h, float* relBL, int* nGood, uint8_t* drop) {
  return ((BA*)h)->fixLinearization(relBL, nGood, drop);
}

/* which: 0 = top A (mode 0), 1 = top L (mode 1 + priors), 2 = Schur complement */
void hso_ba_accumulate(void* h, int which, double* H, double* b) {
  BA* ba = (BA*)h;
  std::vector<double> HH, bb;
  if (which == 0) ba->accumulateTop(0, HH, bb);
  else if (which == 1) ba->accumulateTop(1, HH, bb);
  else ba->accumulateSC(HH, bb);
  std::memcpy(H, HH.data(), sizeof(double) * HH.size());
  std::memcpy(b, bb.data(), sizeof(double) * bb.size());
}

void hso_ba_solve_system(void* h, int iteration, double* x_out) {
  BA* ba = (BA*)h;
  ba->getNullspaces();
  std::vector<double> x;
  ba->solveSystemF(iteration, x);
  std::memcpy(x_out, x.data(), sizeof(double) * x.size());
}
// CalibHessian::setValue (Include/CalibData.h:60-91) of the current camera values (value_zero stays the create-time
// camera, as the reference's stays the initial calibration); the precalc records follow
void hso_ba_set_calib(void* h, const double* value4) {
  BA* ba = (BA*)h;
  ba->calib.setValue(value4);
  ba->setPrecalcValues();
}
// EnergyFunctional::HM / bM (the marginalization prior, Include/EnergyFunctional.h:62-63)
void hso_ba_set_marginal_prior(void* h, const double* HM, const double* bM) {
  BA* ba = (BA*)h;
  const size_t n = ba->HM.size();
  std::memcpy(ba->HM.data(), HM, sizeof(double) * n);
  std::memcpy(ba->bM.data(), bM, sizeof(double) * ba->bM.size());
}
void hso_ba_backup_state(void* h) { ((BA*)h)->backupState(); }
int hso_ba_do_step(void* h) { return ((BA*)h)->doStepFromBackup() ? 1 : 0; }

/* per-residual outputs (after linearize/applyRes) */
void hso_ba_get_residuals(void* h, uint8_t* state, uint8_t* new_state, double* energy, double* new_energy,
                          double* energy_with_outlier, float* resF /*n*8*/, float* J_extra /*n*28 nullable*/,
                          float* JpJdF /*n*8 nullable*/, float* center /*n*3 nullable*/) {
  BA* ba = (BA*)h;
  for (size_t i = 0; i < ba->res.size(); i++) {
    const ResO& r = ba->res[i];
    if (state) state[i] = (uint8_t)r.state_state;
    if (new_state) new_state[i] = (uint8_t)r.state_NewState;
    if (energy) energy[i] = r.state_energy;
    if (new_energy) new_energy[i] = r.state_NewEnergy;
    if (energy_with_outlier) energy_with_outlier[i] = r.state_NewEnergyWithOutlier;
    if (resF) for (int k = 0; k < 8; k++) resF[i * 8 + k] = r.J.resF[k];
    if (J_extra) {
      float* o = J_extra + i * 28;
      for (int k = 0; k < 6; k++) { o[k] = r.J.Jpdxi[0][k]; o[6 + k] = r.J.Jpdxi[1][k]; }
      for (int k = 0; k < 4; k++) { o[12 + k] = r.J.Jpdc[0][k]; o[16 + k] = r.J.Jpdc[1][k]; }
      o[20] = r.J.Jpdd[0]; o[21] = r.J.Jpdd[1];
      o[22] = r.J.JIdx2[0]; o[23] = r.J.JIdx2[1]; o[24] = r.J.JIdx2[3];
      o[25] = r.J.Jab2[0]; o[26] = r.J.Jab2[1]; o[27] = r.J.Jab2[3];
    }
    if (JpJdF) for (int k = 0; k < 8; k++) JpJdF[i * 8 + k] = r.JpJdF[k];
    if (center) for (int k = 0; k < 3; k++) center[i * 3 + k] = r.centerProjectedTo[k];
  }
}

void hso_ba_get_points(void* h, float* idepth, float* step, float* HdiF, float* bdSumF, float* Hdd_accAF) {
  BA* ba = (BA*)h;
  for (size_t i = 0; i < ba->points.size(); i++) {
    const PointO& p = ba->points[i];
    if (idepth) idepth[i] = p.idepth;
    if (step) step[i] = p.step;
    if (HdiF) HdiF[i] = p.HdiF;
    if (bdSumF) bdSumF[i] = p.bdSumF;
    if (Hdd_accAF) Hdd_accAF[i] = p.Hdd_accAF;
  }
}

/* frames: state[10], frameEnergyTH, PRE_worldToCam data[7] */
void hso_ba_get_frames(void* h, double* state, float* energyTH, double* pose7, double* calib_value4) {
  BA* ba = (BA*)h;
  for (int i = 0; i < ba->nF; i++) {
    const FrameO& f = ba->frames[i];
    if (state) for (int k = 0; k < 10; k++) state[i * 10 + k] = f.state[k];
    if (energyTH) energyTH[i] = f.frameEnergyTH;
    if (pose7) f.PRE_worldToCam.toData(pose7 + i * 7);
  }
  if (calib_value4) for (int k = 0; k < 4; k++) calib_value4[k] = ba->calib.value[k];
}

/* frames: evalPT data[7] and state_zero[10] (the linearization points; the optimize tail moves the newest one's) */
void hso_ba_get_frame_eval(void* h, double* eval7, double* state_zero) {
  BA* ba = (BA*)h;
  for (int i = 0; i < ba->nF; i++) {
    const FrameO& f = ba->frames[i];
    if (eval7) f.evalPT.toData(eval7 + i * 7);
    if (state_zero) for (int k = 0; k < 10; k++) state_zero[i * 10 + k] = f.state_zero[k];
  }
}

/* precalc records (for the device parity tests): per (h,t) 37 floats:
   KRKi[9] Kt[3] RTll_0[9] tTll_0[3] aff[2] b0 | RTll[9] tTll[3] -> 39 */
void hso_ba_get_precalc(void* h, float* out /*nF*nF*39*/) {
  BA* ba = (BA*)h;
  for (int i = 0; i < ba->nF * ba->nF; i++) {
    const Precalc& p = ba->precalc[i];
    float* o = out + i * 39;
    for (int k = 0; k < 9; k++) o[k] = p.PRE_KRKiTll[k];
    for (int k = 0; k < 3; k++) o[9 + k] = p.PRE_KtTll[k];
    for (int k = 0; k < 9; k++) o[12 + k] = p.PRE_RTll_0[k];
    for (int k = 0; k < 3; k++) o[21 + k] = p.PRE_tTll_0[k];
    o[24] = p.PRE_aff_mode[0]; o[25] = p.PRE_aff_mode[1]; o[26] = p.PRE_b0_mode;
    for (int k = 0; k < 9; k++) o[27 + k] = p.PRE_RTll[k];
    for (int k = 0; k < 3; k++) o[36 + k] = p.PRE_tTll[k];
  }
}

void hso_ba_get_nullspaces(void* h, double* N /* 7 x dim */) {
  BA* ba = (BA*)h;
  ba->getNullspaces();
  const int n = ba->dim();
  for (int i = 0; i < 6; i++) std::memcpy(N + i * n, ba->ns_pose[i].data(), sizeof(double) * n);
  std::memcpy(N + 6 * n, ba->ns_scale[0].data(), sizeof(double) * n);
}

int hso_ba_res_in_A(void* h) { return ((BA*)h)->lastResInA; }

// marginalizeFrame(f): the (dim-8) prior after removing frame f (the window is not changed)
void hso_ba_marginalize_frame(void* h, int f, double* HM_out, double* bM_out) {
  BA* ba = (BA*)h;
  std::vector<double> H, b;
  ba->marginalizeFrame(f, H, b);
  std::memcpy(HM_out, H.data(), sizeof(double) * H.size());
  std::memcpy(bM_out, b.data(), sizeof(double) * b.size());
}

// marginalize n points (window indices): HM / bM updated in place and returned (dim*dim, dim)
void hso_ba_marginalize_points(void* h, int n, const int* pts, float priorMargFac, float margWeightFac, double* HM_out,
                               double* bM_out) {
  BA* ba = (BA*)h;
  ba->marginalizePoints(std::vector<int>(pts, pts + n), priorMargFac, margWeightFac);
  std::memcpy(HM_out, ba->HM.data(), sizeof(double) * ba->HM.size());
  std::memcpy(bM_out, ba->bM.data(), sizeof(double) * ba->bM.size());
}

/* SE3 helpers for the Sophus-vector tests */
void hso_se3_exp(const double a[6], double out7[7]) { SE3::exp(a).toData(out7); }
void hso_se3_log(const double in7[7], double a[6]) { SE3::fromData(in7).log(a); }
void hso_se3_mul(const double a7[7], const double b7[7], double out7[7]) {
  (SE3::fromData(a7) * SE3::fromData(b7)).toData(out7);
}
void hso_se3_inverse(const double a7[7], double out7[7]) { SE3::fromData(a7).inverse().toData(out7); }
void hso_se3_adj(const double a7[7], double A[36]) { SE3::fromData(a7).Adj(A); }
void hso_se3_matrix(const double a7[7], double R9[9]) { SE3::fromData(a7).rotationMatrix(R9); }

}  // extern "C"
