// ORACLE — TEST INFRASTRUCTURE ONLY (see oracle_common.h for the parity status).
//
// CPU restatement of the initializer's direct two-frame refinement:
//   DirectRefinement ctor (point set-up)   Src/Initializer.cpp:1330-1385
//   DirectRefinement::Refine (LM, lvl 0)   Src/Initializer.cpp:1412-1564
//   resetPoints                            Src/Initializer.cpp:1897-1924
//   calcResAndGS                           Src/Initializer.cpp:1926-2153
//   doStep / applyStep                     Src/Initializer.cpp:2155-2205
//   calcEC / optReg                        Src/Initializer.cpp:2207-2270
// Accumulators in the reference's sequential order (Accumulator9 4-lane SSE + 1k/1m blocking,
// Accumulator11 lane 0, AccumulatorX<2>), fp32 expressions in the reference's operation order
// (built with -ffp-contract=off).  Reference quirks kept:
//   * EAlpha is never updated (the loop calls E.updateSingle), so alphaEnergy = alphaW*|t|^2*npts;
//   * the energy updates after E.finish() change E.num (returned as res[2] = 2*npts) but not E.A;
//   * maxstep is rewritten by every calcResAndGS, also by rejected ones, and doStep reads it;
//   * the rotation / translation scales of wM are applied to the Sophus (translation, rotation) order.
// The 6x6 fp32 LDLT follows Eigen's diagonal-pivoting LDLT (Eigen is not vendored: unpinned).
// The reference texel reads of the first frame at u+dx, v+dy are unchecked; the base index is clamped to
// the buffer here and in the kernel (it only changes reads outside the image buffer).
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <utility>
#include <vector>

#include "accum.h"
#include "oracle_common.h"
#include "se3.h"

namespace hso {

static inline int r_clamp_base(int ix, int iy, int W, int H) {
  long b = (long)ix + (long)iy * W;
  const long hi = (long)W * H - W - 2;
  return (int)(b < 0 ? 0 : (b > hi ? hi : b));
}
static inline float r_interp31(const float* img, float x, float y, int W, int H) {
  int ix = (int)x, iy = (int)y;
  float dx = x - ix, dy = y - iy, dxdy = dx * dy;
  const float* bp = img + 3 * r_clamp_base(ix, iy, W, H);
  return dxdy * bp[3 * (1 + W)] + (dy - dxdy) * bp[3 * W] + (dx - dxdy) * bp[3] + (1 - dx - dy + dxdy) * bp[0];
}

// Eigen compute_inverse_size3 in double (CalibData: pyrKi[0] = pyrK[0].inverse(), Include/CalibData.h:150)
static void inv3d(const double m[9], double r[9]) {
  auto M = [&](int i, int j) { return m[i * 3 + j]; };
  auto cof = [&](int i, int j) {
    int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
    return M(i1, j1) * M(i2, j2) - M(i1, j2) * M(i2, j1);
  };
  double c00 = cof(0, 0), c10 = cof(1, 0), c20 = cof(2, 0);
  double det = c00 * M(0, 0) + c10 * M(1, 0) + c20 * M(2, 0);
  double invdet = 1.0 / det;
  r[0] = c00 * invdet; r[1] = c10 * invdet; r[2] = c20 * invdet;
  r[3] = cof(0, 1) * invdet; r[4] = cof(1, 1) * invdet; r[5] = cof(2, 1) * invdet;
  r[6] = cof(0, 2) * invdet; r[7] = cof(1, 2) * invdet; r[8] = cof(2, 2) * invdet;
}

// Eigen::LDLT<Matrix<float,6,6>> (diagonal pivoting, left-looking) + solve
static void ldlt6f_solve(const float Ain[36], const float b[6], float x[6]) {
  const int n = 6;
  float A[36];
  std::memcpy(A, Ain, sizeof(A));
  int transp[6];
  float temp[6];
  auto at = [&](int i, int j) -> float& { return A[i * n + j]; };
  for (int k = 0; k < n; k++) {
    int idx = k;
    float best = std::fabs(at(k, k));
    for (int i = k + 1; i < n; i++)
      if (std::fabs(at(i, i)) > best) { best = std::fabs(at(i, i)); idx = i; }
    transp[k] = idx;
    if (k != idx) {
      for (int j = 0; j < n; j++) std::swap(at(k, j), at(idx, j));
      for (int i = 0; i < n; i++) std::swap(at(i, k), at(i, idx));
    }
    if (k > 0) {
      for (int j = 0; j < k; j++) temp[j] = at(j, j) * at(k, j);
      float s = 0;
      for (int j = 0; j < k; j++) s += at(k, j) * temp[j];
      at(k, k) -= s;
      for (int i = k + 1; i < n; i++) {
        float t = 0;
        for (int j = 0; j < k; j++) t += at(i, j) * temp[j];
        at(i, k) -= t;
      }
    }
    const float akk = at(k, k);
    if (std::fabs(akk) > std::numeric_limits<float>::min())
      for (int i = k + 1; i < n; i++) at(i, k) /= akk;
    for (int i = k + 1; i < n; i++) at(k, i) = at(i, k);
  }
  for (int i = 0; i < n; i++) x[i] = b[i];
  for (int k = 0; k < n; k++)
    if (transp[k] != k) std::swap(x[k], x[transp[k]]);
  for (int i = 0; i < n; i++)
    for (int j = 0; j < i; j++) x[i] -= at(i, j) * x[j];
  for (int i = 0; i < n; i++) x[i] = std::fabs(at(i, i)) > std::numeric_limits<float>::min() ? x[i] / at(i, i) : 0.0f;
  for (int i = n - 1; i >= 0; i--)
    for (int j = i + 1; j < n; j++) x[i] -= at(j, i) * x[j];
  for (int k = n - 1; k >= 0; k--)
    if (transp[k] != k) std::swap(x[k], x[transp[k]]);
}

// Vec8f dot product in Eigen's vectorized order: lane-wise sum of the two 4-float halves, then
// predux (l0 + l2) + (l1 + l3) (SSE movehl / shuffle; the 8-lane AVX packet reduces the same way)
static inline float dot8(const float* a, const float* b) {
  float s[4];
  for (int l = 0; l < 4; l++) s[l] = a[l] * b[l] + a[l + 4] * b[l + 4];
  return (s[0] + s[2]) + (s[1] + s[3]);
}

struct RPnt {  // struct Pnt (Include/Initializer.h:159-190), the fields DirectRefinement uses
  float u, v, idepth, idepth_new, iR;
  bool isGood, isGood_new;
  float energy[2], energy_new[2];
  float lastHessian, lastHessian_new, maxstep, outlierTH;
};

struct Refiner {
  int W, H;
  double Ki[9];
  float fx, fy, cx, cy;
  std::vector<float> img1, img2;  // FirstFrame / SecondFrame DirPyr[0], (I, dx, dy) per pixel
  float expo1 = 0, expo2 = 0;     // FrameShell::ab_exposure
  int n = 0;
  std::vector<RPnt> p;
  std::vector<uint8_t> tri;
  std::vector<float> invz;  // 1.0 / Pts3D[i].z as the ctor computes it
  std::vector<float> Jb, Jb_new;  // Vec10f per point
  float alphaK = 2.5f * 2.5f, alphaW = 150 * 150, regWeight = 0.8f, couplingWeight = 1;
  bool snapped = false;
  float huberTH = 9.f, outlierTH = 12 * 12;
  // LM log: per iteration {eTotalOld, eTotalNew, accept, lambda (before update), |inc|, resNew[0], resNew[1], regNew}
  std::vector<float> log;

  // ctor point set-up (Src/Initializer.cpp:1362-1382)
  void set_points(int n_, const float* u, const float* v, const uint8_t* t, const float* z) {
    n = n_;
    p.assign(n, RPnt{});
    tri.assign(t, t + n);
    invz.assign(n, 1.f);
    Jb.assign((size_t)n * 10, 0.f);
    Jb_new.assign((size_t)n * 10, 0.f);
    for (int i = 0; i < n; i++) {
      RPnt& q = p[i];
      q.u = u[i];
      q.v = v[i];
      invz[i] = tri[i] ? (float)(1.0 / z[i]) : 1.0f;
      q.idepth = q.iR = invz[i];
      q.idepth_new = q.idepth;
      q.isGood = true;
      q.isGood_new = false;
      q.energy[0] = q.energy[1] = 0;
      q.energy_new[0] = q.energy_new[1] = 0;
      q.lastHessian = q.lastHessian_new = 0;
      q.maxstep = 0;
      q.outlierTH = PN * outlierTH;
    }
    snapped = false;
  }

  void resetPoints() {
    for (int i = 0; i < n; i++) {
      p[i].energy[0] = p[i].energy[1] = 0;
      p[i].idepth_new = p[i].idepth;
    }
  }

  // calcResAndGS (Src/Initializer.cpp:1926-2153), lvl 0
  void calcResAndGS(const SE3& refToNew, double aff_a, double aff_b, float Hout[64], float bout[8], float Hsc[64],
                    float bsc[8], float res[3]) {
    const int wl = W, hl = H;
    const float* colorRef = img1.data();
    const float* colorNew = img2.data();
    double R[9], RKid[9];
    refToNew.rotationMatrix(R);
    SE3::mm3(R, Ki, RKid);
    float RKi[9];
    for (int q = 0; q < 9; q++) RKi[q] = (float)RKid[q];
    const float t[3] = {(float)refToNew.t[0], (float)refToNew.t[1], (float)refToNew.t[2]};
    const float r2a = (float)std::exp(aff_a), r2b = (float)aff_b;
    const float fxl = fx, fyl = fy, cxl = cx, cyl = cy;

    Acc11 E;
    Acc9 acc9;
    E.initialize();
    acc9.initialize();
    const int npts = n;
    for (int i = 0; i < npts; i++) {
      RPnt* point = &p[i];
      point->maxstep = 1e10;
      if (!point->isGood) {
        E.updateSingle((float)(point->energy[0]));
        point->energy_new[0] = point->energy[0];
        point->energy_new[1] = point->energy[1];
        point->isGood_new = false;
        continue;
      }
      float dp[8][PN], dd[PN], r[PN];
      float* jb = &Jb_new[(size_t)i * 10];
      for (int k = 0; k < 10; k++) jb[k] = 0;
      bool isGood = true;
      float energy = 0;
      for (int idx = 0; idx < PN; idx++) {
        const int dx = kPattern[idx][0], dy = kPattern[idx][1];
        const float x = point->u + dx, y = point->v + dy;
        float pt[3];
        for (int q = 0; q < 3; q++) pt[q] = (RKi[q * 3 + 0] * x + RKi[q * 3 + 1] * y + RKi[q * 3 + 2] * 1.f) + t[q] * point->idepth_new;
        const float u = pt[0] / pt[2];
        const float v = pt[1] / pt[2];
        const float Ku = fxl * u + cxl;
        const float Kv = fyl * v + cyl;
        const float new_idepth = point->idepth_new / pt[2];
        if (!(Ku > 1 && Kv > 1 && Ku < wl - 2 && Kv < hl - 2 && new_idepth > 0)) {
          isGood = false;
          break;
        }
        const V3f hitColor = interp33(colorNew, Ku, Kv, wl);
        const float rlR = r_interp31(colorRef, x, y, wl, hl);
        if (!std::isfinite(rlR) || !std::isfinite((float)hitColor.x)) {
          isGood = false;
          break;
        }
        const float residual = hitColor.x - r2a * rlR - r2b;
        float hw = std::fabs(residual) < huberTH ? 1 : huberTH / std::fabs(residual);
        if (!tri[i]) hw = (float)(hw * 0.1);
        energy += hw * residual * residual * (2 - hw);
        const float dxdd = (t[0] - t[2] * u) / pt[2];
        const float dydd = (t[1] - t[2] * v) / pt[2];
        if (hw < 1) hw = std::sqrt(hw);
        const float dxInterp = hw * hitColor.y * fxl;
        const float dyInterp = hw * hitColor.z * fyl;
        dp[0][idx] = new_idepth * dxInterp;
        dp[1][idx] = new_idepth * dyInterp;
        dp[2][idx] = -new_idepth * (u * dxInterp + v * dyInterp);
        dp[3][idx] = -u * v * dxInterp - (1 + v * v) * dyInterp;
        dp[4][idx] = (1 + u * u) * dxInterp + u * v * dyInterp;
        dp[5][idx] = -v * dxInterp + u * dyInterp;
        dp[6][idx] = -hw * r2a * rlR;
        dp[7][idx] = -hw * 1;
        dd[idx] = dxInterp * dxdd + dyInterp * dydd;
        r[idx] = hw * residual;
        const float nx = dxdd * fxl, ny = dydd * fyl;
        const float maxstep = 1.0f / std::sqrt(nx * nx + ny * ny);
        if (maxstep < point->maxstep) point->maxstep = maxstep;
        for (int k = 0; k < 8; k++) jb[k] += dp[k][idx] * dd[idx];
        jb[8] += r[idx] * dd[idx];
        jb[9] += dd[idx] * dd[idx];
      }
      if (!isGood || energy > point->outlierTH * 20) {
        E.updateSingle((float)(point->energy[0]));
        point->isGood_new = false;
        point->energy_new[0] = point->energy[0];
        point->energy_new[1] = point->energy[1];
        continue;
      }
      E.updateSingle(energy);
      point->isGood_new = true;
      point->energy_new[0] = energy;
      for (int g = 0; g + 3 < PN; g += 4) {
        float J[9][4];
        for (int l = 0; l < 4; l++) {
          for (int k = 0; k < 8; k++) J[k][l] = dp[k][g + l];
          J[8][l] = r[g + l];
        }
        acc9.updateSSE(J);
      }
    }
    E.finish();
    acc9.finish();

    // "alpha energy": the loop feeds E, not EAlpha (quirk kept)
    Acc11 EAlpha;
    EAlpha.initialize();
    for (int i = 0; i < npts; i++) {
      RPnt* point = &p[i];
      if (!point->isGood_new) {
        E.updateSingle((float)(point->energy[1]));
      } else {
        point->energy_new[1] = (point->idepth_new - 1) * (point->idepth_new - 1);
        E.updateSingle((float)(point->energy_new[1]));
      }
    }
    EAlpha.finish();
    const double tsq = refToNew.t[0] * refToNew.t[0] + refToNew.t[1] * refToNew.t[1] + refToNew.t[2] * refToNew.t[2];
    float alphaEnergy = (float)(alphaW * (EAlpha.A + tsq * npts));
    float alphaOpt;
    if (alphaEnergy > alphaK * npts) {
      alphaOpt = 0;
      alphaEnergy = alphaK * npts;
    } else {
      alphaOpt = alphaW;
    }

    Acc9 acc9SC;
    acc9SC.initialize();
    for (int i = 0; i < npts; i++) {
      RPnt* point = &p[i];
      if (!point->isGood_new) continue;
      float* jb = &Jb_new[(size_t)i * 10];
      point->lastHessian_new = jb[9];
      jb[8] += alphaOpt * (point->idepth_new - 1);
      jb[9] += alphaOpt;
      if (alphaOpt == 0) {
        jb[8] += couplingWeight * (point->idepth_new - point->iR);
        jb[9] += couplingWeight;
      }
      jb[9] = 1 / (1 + jb[9]);
      acc9SC.updateSingleWeighted(jb, jb[9]);
    }
    acc9SC.finish();

    for (int rr = 0; rr < 8; rr++) {
      for (int c = 0; c < 8; c++) {
        Hout[rr * 8 + c] = acc9.H[rr * 9 + c];
        Hsc[rr * 8 + c] = acc9SC.H[rr * 9 + c];
      }
      bout[rr] = acc9.H[rr * 9 + 8];
      bsc[rr] = acc9SC.H[rr * 9 + 8];
    }
    for (int k = 0; k < 3; k++) Hout[k * 8 + k] += alphaOpt * npts;
    double lg[6];
    refToNew.log(lg);
    for (int k = 0; k < 3; k++) bout[k] += (float)lg[k] * alphaOpt * npts;
    res[0] = E.A;
    res[1] = alphaEnergy;
    res[2] = (float)E.num;
  }

  // doStep (Src/Initializer.cpp:2155-2186)
  void doStep(float lambda, const float inc[8]) {
    const float maxPixelStep = 0.25f;
    const float idMaxStep = 1e10;
    for (int i = 0; i < n; i++) {
      if (!p[i].isGood) continue;
      const float* jb = &Jb[(size_t)i * 10];
      const float b = jb[8] + dot8(jb, inc);
      float step = -b * jb[9] / (1 + lambda);
      float maxstep = maxPixelStep * p[i].maxstep;
      if (maxstep > idMaxStep) maxstep = idMaxStep;
      if (step > maxstep) step = maxstep;
      if (step < -maxstep) step = -maxstep;
      float newIdepth = p[i].idepth + step;
      if (newIdepth < 1e-3) newIdepth = 1e-3;
      if (newIdepth > 50) newIdepth = 50;
      p[i].idepth_new = newIdepth;
    }
  }

  // applyStep (Src/Initializer.cpp:2188-2205)
  void applyStep() {
    for (int i = 0; i < n; i++) {
      if (!p[i].isGood) {
        p[i].idepth = p[i].idepth_new = p[i].iR;
        continue;
      }
      p[i].energy[0] = p[i].energy_new[0];
      p[i].energy[1] = p[i].energy_new[1];
      p[i].isGood = p[i].isGood_new;
      p[i].idepth = p[i].idepth_new;
      p[i].lastHessian = p[i].lastHessian_new;
    }
    std::swap(Jb, Jb_new);
  }

  // calcEC (Src/Initializer.cpp:2207-2227)
  void calcEC(float out[3]) {
    if (!snapped) {
      out[0] = 0; out[1] = 0; out[2] = (float)n;
      return;
    }
    AccX<2> E;
    E.initialize();
    for (int i = 0; i < n; i++) {
      const RPnt& q = p[i];
      if (!q.isGood_new) continue;
      const float rOld = q.idepth - q.iR;
      const float rNew = q.idepth_new - q.iR;
      const float L[2] = {rOld * rOld, rNew * rNew};
      E.updateNoWeight(L);
    }
    E.finish();
    out[0] = couplingWeight * E.A1m[0];
    out[1] = couplingWeight * E.A1m[1];
    out[2] = (float)E.num;
  }

  // optReg (Src/Initializer.cpp:2229-2270)
  void optReg() {
    if (!snapped) {
      for (int i = 0; i < n; i++) p[i].iR = tri[i] ? invz[i] : p[i].idepth;
      return;
    }
    for (int i = 0; i < n; i++)
      if (p[i].isGood) p[i].iR = p[i].idepth;
  }

  // Refine (Src/Initializer.cpp:1412-1564); T = thisToNext in/out, aff = thisToNext_aff in/out
  int refine(SE3& T, double aff[2]) {
    const int maxIterations0 = 1000;
    SE3 cur = T;
    double affc[2] = {aff[0], aff[1]};
    if (expo1 > 0 && expo2 > 0) {
      affc[0] = (double)logf(expo2 / expo1);
      affc[1] = 0;
    }
    float Hm[64], b[8], Hs[64], bs[8], resOld[3];
    resetPoints();
    calcResAndGS(cur, affc[0], affc[1], Hm, b, Hs, bs, resOld);
    applyStep();
    float lambda = 0.1f;
    const float eps = 1e-4f;
    int fails = 0;
    int iteration = 0;
    const float wM[8] = {SCALE_XI_ROT, SCALE_XI_ROT, SCALE_XI_ROT, SCALE_XI_TRANS, SCALE_XI_TRANS, SCALE_XI_TRANS,
                         SCALE_A, SCALE_B};
    const float sc = 0.01f / (W * H);
    log.clear();
    while (true) {
      float Hl[64], bl[8];
      for (int q = 0; q < 64; q++) Hl[q] = Hm[q];
      for (int i = 0; i < 8; i++) Hl[i * 8 + i] *= (1 + lambda);
      const float il = 1 / (1 + lambda);
      for (int q = 0; q < 64; q++) Hl[q] -= Hs[q] * il;
      for (int i = 0; i < 8; i++) bl[i] = b[i] - bs[i] * il;
      for (int r = 0; r < 8; r++)
        for (int c = 0; c < 8; c++) Hl[r * 8 + c] = ((wM[r] * Hl[r * 8 + c]) * wM[c]) * sc;
      for (int r = 0; r < 8; r++) bl[r] = (wM[r] * bl[r]) * sc;
      float H6[36], x6[6], inc[8];
      for (int r = 0; r < 6; r++)
        for (int c = 0; c < 6; c++) H6[r * 6 + c] = Hl[r * 8 + c];
      ldlt6f_solve(H6, bl, x6);  // fixAffine = true
      for (int k = 0; k < 6; k++) inc[k] = -(wM[k] * x6[k]);
      inc[6] = inc[7] = 0;
      double incd[6];
      for (int k = 0; k < 6; k++) incd[k] = (double)inc[k];
      const SE3 nw = SE3::exp(incd) * cur;
      double affn[2] = {affc[0] + inc[6], affc[1] + inc[7]};
      doStep(lambda, inc);
      float Hn[64], bn[8], Hsn[64], bsn[8], resNew[3], reg[3];
      calcResAndGS(nw, affn[0], affn[1], Hn, bn, Hsn, bsn, resNew);
      calcEC(reg);
      const float eTotalNew = resNew[0] + resNew[1] + reg[1];
      const float eTotalOld = resOld[0] + resOld[1] + reg[0];
      const bool accept = eTotalOld > eTotalNew;
      const float incNorm = std::sqrt(dot8(inc, inc));
      const float row[8] = {eTotalOld, eTotalNew, accept ? 1.f : 0.f, lambda, incNorm, resNew[0], resNew[1], reg[1]};
      log.insert(log.end(), row, row + 8);
      if (accept) {
        if (resNew[1] == alphaK * n) snapped = true;
        std::memcpy(Hm, Hn, sizeof(Hm)); std::memcpy(b, bn, sizeof(b));
        std::memcpy(Hs, Hsn, sizeof(Hs)); std::memcpy(bs, bsn, sizeof(bs));
        std::memcpy(resOld, resNew, sizeof(resOld));
        affc[0] = affn[0]; affc[1] = affn[1];
        cur = nw;
        applyStep();
        optReg();
        lambda *= 0.5;
        fails = 0;
        if (lambda < 0.0001) lambda = 0.0001;
      } else {
        fails++;
        lambda *= 4;
        if (lambda > 10000) lambda = 10000;
      }
      if (!(incNorm > eps) || iteration >= maxIterations0 || fails >= 2) break;
      iteration++;
    }
    T = cur;
    aff[0] = affc[0];
    aff[1] = affc[1];
    return iteration + 1;
  }
};

}  // namespace hso

using hso::Refiner;

extern "C" {

void* hso_ref_create(int W, int H, const double K4[4], const float* img1, const float* img2, float expo1, float expo2) {
  Refiner* r = new Refiner();
  r->W = W; r->H = H;
  const double K[9] = {K4[0], 0, K4[2], 0, K4[1], K4[3], 0, 0, 1};
  hso::inv3d(K, r->Ki);
  r->fx = (float)K4[0]; r->fy = (float)K4[1]; r->cx = (float)K4[2]; r->cy = (float)K4[3];
  r->img1.assign(img1, img1 + (size_t)W * H * 3);
  r->img2.assign(img2, img2 + (size_t)W * H * 3);
  r->expo1 = expo1; r->expo2 = expo2;
  return r;
}
void hso_ref_destroy(void* h) { delete (Refiner*)h; }
void hso_ref_set_points(void* h, int n, const float* u, const float* v, const uint8_t* tri, const float* z) {
  ((Refiner*)h)->set_points(n, u, v, tri, z);
}
// resetPoints + one calcResAndGS at (T, aff); per-point state readable with hso_ref_get_points
void hso_ref_calc(void* h, const double T7[7], const double aff[2], float* H64, float* b8, float* Hsc64, float* bsc8,
                  float* res3) {
  Refiner* r = (Refiner*)h;
  r->resetPoints();
  r->calcResAndGS(hso::SE3::fromData(T7), aff[0], aff[1], H64, b8, Hsc64, bsc8, res3);
}
int hso_ref_refine(void* h, double T7[7], double aff[2], int* snapped) {
  Refiner* r = (Refiner*)h;
  hso::SE3 T = hso::SE3::fromData(T7);
  const int it = r->refine(T, aff);
  T.toData(T7);
  if (snapped) *snapped = r->snapped;
  return it;
}
int hso_ref_get_log(void* h, int cap, float* out) {
  Refiner* r = (Refiner*)h;
  const int n = (int)r->log.size() / 8;
  for (int q = 0; q < n && q < cap; q++) std::memcpy(out + 8 * q, &r->log[8 * q], 8 * sizeof(float));
  return n;
}
// f32[n*7] = idepth, idepth_new, iR, energy_new0, energy_new1, maxstep, lastHessian_new; u8[n*2] = isGood, isGood_new;
// jb_new[n*10]
void hso_ref_get_points(void* h, float* f7, uint8_t* g2, float* jb_new) {
  Refiner* r = (Refiner*)h;
  for (int i = 0; i < r->n; i++) {
    const hso::RPnt& q = r->p[i];
    float* o = f7 + 7 * (size_t)i;
    o[0] = q.idepth; o[1] = q.idepth_new; o[2] = q.iR; o[3] = q.energy_new[0]; o[4] = q.energy_new[1];
    o[5] = q.maxstep; o[6] = q.lastHessian_new;
    g2[2 * i] = q.isGood; g2[2 * i + 1] = q.isGood_new;
  }
  if (jb_new) std::memcpy(jb_new, r->Jb_new.data(), sizeof(float) * 10 * r->n);
}

}  // extern "C"
