/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  CPU restatement of H-SLAM's CoarseTracker (parity unpinned:
 * the reference is unbuildable here and ships no tracker vectors; see oracle_common.h).
 *
 *   CoarseTracker ctor / makeK           Src/CoarseTracker.cpp:29-101
 *   makeCoarseDepthL0                    Src/CoarseTracker.cpp:105-263
 *   calcGSSSE (+ Accumulator9)           Src/CoarseTracker.cpp:267-324, Include/MatrixAccumulators.h:982-1345
 *   calcRes                              Src/CoarseTracker.cpp:329-485
 *   setCoarseTrackingRef                 Src/CoarseTracker.cpp:492-504
 *   trackNewestCoarse                    Src/CoarseTracker.cpp:506-683
 *   System::trackNewCoarse (try loop)    Src/System.cpp:413-481
 * Single-threaded, the reference's exact fp32 operation order (built with -ffp-contract=off).
 */
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <vector>

#include "accum.h"
#include "ldlt.h"
#include "oracle_common.h"
#include "se3.h"

namespace hso {

struct TrackerO {
  int sum_order = 0;  // 0: the reference's point order; 1: reversed (hso_trk_set_sum_order, the tests' order spread)
  hs_params P;
  int nlev = 0;
  int w[10], h[10];
  float fx[10], fy[10], cx[10], cy[10];
  float Ki[10][9];
  std::vector<float> idepth[10], wsum[10], wsum_bak[10];
  std::vector<float> pc_u[10], pc_v[10], pc_idepth[10], pc_color[10];
  int pc_n[10] = {0};
  std::vector<std::vector<float>> refPyr, newPyr;  // per level w*h*3 (I, dx, dy)
  float refExposure = 1, newExposure = 1;
  double refAff[2] = {0, 0};
  std::vector<float> bw_idepth, bw_u, bw_v, bw_dx, bw_dy, bw_res, bw_w, bw_ref;
  int bw_n = 0;
  Acc9 acc;
  double lastResiduals[5];
  double lastFlow[3];
  std::vector<int> log_lvl;           // per LM iteration of the last trackNewestCoarse: level,
  std::vector<double> log_new, log_old, log_inc;  // resNew/N, resOld/N (accept test), |inc| (break test)

  // CoarseTracker(ww, hh) + makeK(HCalib): fx[0] = HCalib->fxl() (float, scaled calib)
  void init(int W, int H, int levels, const float K4[4]) {
    nlev = levels;
    w[0] = W; h[0] = H;
    fx[0] = K4[0]; fy[0] = K4[1]; cx[0] = K4[2]; cy[0] = K4[3];
    for (int l = 1; l < nlev; l++) {
      w[l] = w[0] >> l;
      h[l] = h[0] >> l;
      fx[l] = fx[l - 1] * 0.5;
      fy[l] = fy[l - 1] * 0.5;
      cx[l] = (cx[0] + 0.5) / ((int)1 << l) - 0.5;
      cy[l] = (cy[0] + 0.5) / ((int)1 << l) - 0.5;
    }
    for (int l = 0; l < nlev; l++) {
      const float K[9] = {fx[l], 0, cx[l], 0, fy[l], cy[l], 0, 0, 1};
      inv3f(K, Ki[l]);
      const int n = w[l] * h[l];
      idepth[l].assign(n, 0.f); wsum[l].assign(n, 0.f); wsum_bak[l].assign(n, 0.f);
      pc_u[l].assign(n, 0.f); pc_v[l].assign(n, 0.f); pc_idepth[l].assign(n, 0.f); pc_color[l].assign(n, 0.f);
    }
    const int n0 = W * H;
    bw_idepth.assign(n0 + 4, 0.f); bw_u.assign(n0 + 4, 0.f); bw_v.assign(n0 + 4, 0.f); bw_dx.assign(n0 + 4, 0.f);
    bw_dy.assign(n0 + 4, 0.f); bw_res.assign(n0 + 4, 0.f); bw_w.assign(n0 + 4, 0.f); bw_ref.assign(n0 + 4, 0.f);
  }

  // makeCoarseDepthL0 over the points whose lastResiduals[0] (residual into lastRef) is IN, in the
  // reference's frame / point order: centre projection (u, v, new idepth) and the point's HdiF
  void makeCoarseDepthL0(int n, const float* cu, const float* cv, const float* cid, const float* hdi) {
    std::fill(idepth[0].begin(), idepth[0].end(), 0.f);
    std::fill(wsum[0].begin(), wsum[0].end(), 0.f);
    for (int i = 0; i < n; i++) {
      const int u = (int)(cu[i] + 0.5f);
      const int v = (int)(cv[i] + 0.5f);
      const float new_idepth = cid[i];
      const float weight = sqrtf(1e-3 / (hdi[i] + 1e-12));
      idepth[0][u + w[0] * v] += new_idepth * weight;
      wsum[0][u + w[0] * v] += weight;
    }
    for (int l = 1; l < nlev; l++) {
      const int wl = w[l], hl = h[l], wlm1 = w[l - 1];
      for (int y = 0; y < hl; y++)
        for (int x = 0; x < wl; x++) {
          const int b = 2 * x + 2 * y * wlm1;
          idepth[l][x + y * wl] = idepth[l - 1][b] + idepth[l - 1][b + 1] + idepth[l - 1][b + wlm1] + idepth[l - 1][b + wlm1 + 1];
          wsum[l][x + y * wl] = wsum[l - 1][b] + wsum[l - 1][b + 1] + wsum[l - 1][b + wlm1] + wsum[l - 1][b + wlm1 + 1];
        }
    }
    // dilate: levels 0-1 from the diagonal neighbours, levels >= 2 from the 4-neighbours
    for (int l = 0; l < nlev; l++) {
      const int wl = w[l], wh = w[l] * h[l] - w[l];
      wsum_bak[l] = wsum[l];
      float* id = idepth[l].data();
      float* ws = wsum[l].data();
      const float* wb = wsum_bak[l].data();
      int o[4];
      if (l < 2) { o[0] = 1 + wl; o[1] = -1 - wl; o[2] = wl - 1; o[3] = -wl + 1; }
      else { o[0] = 1; o[1] = -1; o[2] = wl; o[3] = -wl; }
      for (int i = wl; i < wh; i++) {
        if (wb[i] <= 0) {
          float sum = 0, num = 0, numn = 0;
          for (int q = 0; q < 4; q++)  // out-of-range reads of the reference (pixels (0,1), (w-1,h-2)) -> empty
            if (i + o[q] >= 0 && i + o[q] < wl * h[l] && wb[i + o[q]] > 0) { sum += id[i + o[q]]; num += wb[i + o[q]]; numn++; }
          if (numn > 0) { id[i] = sum / numn; ws[i] = num / numn; }
        }
      }
    }
    // normalize + compact in raster order
    for (int l = 0; l < nlev; l++) {
      const int wl = w[l], hl = h[l];
      const float* dI = refPyr[l].data();
      int n_ = 0;
      for (int y = 2; y < hl - 2; y++)
        for (int x = 2; x < wl - 2; x++) {
          const int i = x + y * wl;
          if (wsum[l][i] > 0) {
            idepth[l][i] /= wsum[l][i];
            pc_u[l][n_] = x;
            pc_v[l][n_] = y;
            pc_idepth[l][n_] = idepth[l][i];
            pc_color[l][n_] = dI[3 * i];
            if (!std::isfinite(pc_color[l][n_]) || !(idepth[l][i] > 0)) {
              idepth[l][i] = -1;
              continue;
            }
            n_++;
          } else {
            idepth[l][i] = -1;
          }
          wsum[l][i] = 1;
        }
      pc_n[l] = n_;
    }
  }

  void relAff(const double aff[2], double out[2]) const {
    fromToVecExposure(refExposure, newExposure, refAff[0], refAff[1], aff[0], aff[1], out);
  }

  // calcRes -> {E, N, flowT, 0, flowRT, saturated / N}
  void calcRes(int lvl, const SE3& T, const double aff[2], float cutoffTH, double rs[6]) {
    float E = 0;
    int numTermsInE = 0, numTermsInWarped = 0, numSaturated = 0;
    const int wl = w[lvl], hl = h[lvl];
    const float* dINew = newPyr[lvl].data();
    const float fxl = fx[lvl], fyl = fy[lvl], cxl = cx[lvl], cyl = cy[lvl];
    double Rd[9];
    T.rotationMatrix(Rd);
    float R[9], RKi[9];
    for (int i = 0; i < 9; i++) R[i] = (float)Rd[i];
    mm3f(R, Ki[lvl], RKi);
    const float t[3] = {(float)T.t[0], (float)T.t[1], (float)T.t[2]};
    double affd[2];
    relAff(aff, affd);
    const float affLL[2] = {(float)affd[0], (float)affd[1]};
    float sumSquaredShiftT = 0, sumSquaredShiftRT = 0, sumSquaredShiftNum = 0;
    const float maxEnergy = 2 * P.huberTH * cutoffTH - P.huberTH * P.huberTH;
    const int nl = pc_n[lvl];
    for (int ii = 0; ii < nl; ii++) {
      // order 1 (test spread only): the points in reverse order, so every fp32 sum (E, the flows, the warped
      // buffer that calcGSSSE sums) is formed in another order; the decisions per point are the same
      const int i = sum_order == 1 ? nl - 1 - ii : ii;
      const float id = pc_idepth[lvl][i], x = pc_u[lvl][i], y = pc_v[lvl][i];
      const float xy1[3] = {x, y, 1};
      float pt[3];
      mv3f(RKi, xy1, pt);
      for (int k = 0; k < 3; k++) pt[k] = pt[k] + t[k] * id;
      const float u = pt[0] / pt[2], v = pt[1] / pt[2];
      const float Ku = fxl * u + cxl, Kv = fyl * v + cyl;
      const float new_idepth = id / pt[2];
      if (lvl == 0 && i % 32 == 0) {
        float ptT[3], ptT2[3], pt3[3], kxy[3];
        mv3f(Ki[lvl], xy1, kxy);
        for (int k = 0; k < 3; k++) { ptT[k] = kxy[k] + t[k] * id; ptT2[k] = kxy[k] - t[k] * id; }
        mv3f(RKi, xy1, pt3);
        for (int k = 0; k < 3; k++) pt3[k] = pt3[k] - t[k] * id;
        const float uT = ptT[0] / ptT[2], vT = ptT[1] / ptT[2];
        const float KuT = fxl * uT + cxl, KvT = fyl * vT + cyl;
        const float uT2 = ptT2[0] / ptT2[2], vT2 = ptT2[1] / ptT2[2];
        const float KuT2 = fxl * uT2 + cxl, KvT2 = fyl * vT2 + cyl;
        const float u3 = pt3[0] / pt3[2], v3 = pt3[1] / pt3[2];
        const float Ku3 = fxl * u3 + cxl, Kv3 = fyl * v3 + cyl;
        sumSquaredShiftT += (KuT - x) * (KuT - x) + (KvT - y) * (KvT - y);
        sumSquaredShiftT += (KuT2 - x) * (KuT2 - x) + (KvT2 - y) * (KvT2 - y);
        sumSquaredShiftRT += (Ku - x) * (Ku - x) + (Kv - y) * (Kv - y);
        sumSquaredShiftRT += (Ku3 - x) * (Ku3 - x) + (Kv3 - y) * (Kv3 - y);
        sumSquaredShiftNum += 2;
      }
      if (!(Ku > 2 && Kv > 2 && Ku < wl - 3 && Kv < hl - 3 && new_idepth > 0)) continue;
      const float refColor = pc_color[lvl][i];
      const V3f hit = interp33(dINew, Ku, Kv, wl);
      if (!std::isfinite(hit.x)) continue;
      const float residual = hit.x - (float)(affLL[0] * refColor + affLL[1]);
      const float hw = std::fabs(residual) < P.huberTH ? 1 : P.huberTH / std::fabs(residual);
      if (std::fabs(residual) > cutoffTH) {
        E += maxEnergy;
        numTermsInE++;
        numSaturated++;
      } else {
        E += hw * residual * residual * (2 - hw);
        numTermsInE++;
        bw_idepth[numTermsInWarped] = new_idepth;
        bw_u[numTermsInWarped] = u;
        bw_v[numTermsInWarped] = v;
        bw_dx[numTermsInWarped] = hit.y;
        bw_dy[numTermsInWarped] = hit.z;
        bw_res[numTermsInWarped] = residual;
        bw_w[numTermsInWarped] = hw;
        bw_ref[numTermsInWarped] = refColor;
        numTermsInWarped++;
      }
    }
    while (numTermsInWarped % 4 != 0) {
      bw_idepth[numTermsInWarped] = 0; bw_u[numTermsInWarped] = 0; bw_v[numTermsInWarped] = 0;
      bw_dx[numTermsInWarped] = 0; bw_dy[numTermsInWarped] = 0; bw_res[numTermsInWarped] = 0;
      bw_w[numTermsInWarped] = 0; bw_ref[numTermsInWarped] = 0;
      numTermsInWarped++;
    }
    bw_n = numTermsInWarped;
    rs[0] = E;
    rs[1] = numTermsInE;
    rs[2] = sumSquaredShiftT / (sumSquaredShiftNum + 0.1);
    rs[3] = 0;
    rs[4] = sumSquaredShiftRT / (sumSquaredShiftNum + 0.1);
    rs[5] = numSaturated / (float)numTermsInE;
  }

  // calcGSSSE on the warped buffer of the last calcRes (4-lane SSE order, Accumulator9)
  void calcGSSSE(int lvl, double H[64], double b[8], const double aff[2]) {
    acc.initialize();
    const float fxl = fx[lvl], fyl = fy[lvl];
    const float b0 = (float)refAff[1];
    double affd[2];
    relAff(aff, affd);
    const float a = (float)affd[0];
    const int n = bw_n;
    for (int i = 0; i < n; i += 4) {
      float J[9][4], wgt[4];
      for (int l = 0; l < 4; l++) {
        const float dx = bw_dx[i + l] * fxl, dy = bw_dy[i + l] * fyl;
        const float u = bw_u[i + l], v = bw_v[i + l], id = bw_idepth[i + l];
        J[0][l] = id * dx;
        J[1][l] = id * dy;
        J[2][l] = 0.f - id * (u * dx + v * dy);
        J[3][l] = 0.f - ((u * v) * dx + dy * (1.f + v * v));
        J[4][l] = (u * v) * dy + dx * (1.f + u * u);
        J[5][l] = u * dy - v * dx;
        J[6][l] = a * (b0 - bw_ref[i + l]);
        J[7][l] = -1.f;
        J[8][l] = bw_res[i + l];
        wgt[l] = bw_w[i + l];
      }
      acc.updateSSE_eighted(J, wgt);
    }
    acc.finish();
    const double inv = (double)(1.0f / n);
    for (int r = 0; r < 8; r++) {
      for (int c = 0; c < 8; c++) H[r * 8 + c] = (double)acc.H[r * 9 + c] * inv;
      b[r] = (double)acc.H[r * 9 + 8] * inv;
    }
    const double s[8] = {SCALE_XI_ROT, SCALE_XI_ROT, SCALE_XI_ROT, SCALE_XI_TRANS, SCALE_XI_TRANS, SCALE_XI_TRANS,
                         SCALE_A, SCALE_B};
    for (int r = 0; r < 8; r++)
      for (int c = 0; c < 8; c++) H[r * 8 + c] *= s[c];
    for (int r = 0; r < 8; r++)
      for (int c = 0; c < 8; c++) H[r * 8 + c] *= s[r];
    for (int r = 0; r < 8; r++) b[r] *= s[r];
  }

  bool trackNewestCoarse(SE3& T_out, double aff_out[2], int coarsestLvl, const double minResForAbort[5],
                         int* iters_out) {
    for (int i = 0; i < 5; i++) lastResiduals[i] = NAN;
    for (int i = 0; i < 3; i++) lastFlow[i] = 1000;
    log_lvl.clear();
    log_new.clear();
    log_old.clear();
    log_inc.clear();
    const int maxIterations[] = {10, 20, 50, 50, 50};
    const float lambdaExtrapolationLimit = 0.001;
    SE3 cur = T_out;
    double aff[2] = {aff_out[0], aff_out[1]};
    bool haveRepeated = false;
    int its = 0;
    for (int lvl = coarsestLvl; lvl >= 0; lvl--) {
      double H[64], b[8];
      float levelCutoffRepeat = 1;
      double resOld[6];
      calcRes(lvl, cur, aff, P.coarseCutoffTH * levelCutoffRepeat, resOld);
      while (resOld[5] > 0.6 && levelCutoffRepeat < 50) {
        levelCutoffRepeat *= 2;
        calcRes(lvl, cur, aff, P.coarseCutoffTH * levelCutoffRepeat, resOld);
      }
      calcGSSSE(lvl, H, b, aff);
      float lambda = 0.01;
      for (int iteration = 0; iteration < maxIterations[lvl]; iteration++) {
        its++;
        std::vector<double> Hl(H, H + 64), mb(8), inc(8);
        for (int i = 0; i < 8; i++) Hl[i * 8 + i] *= (1 + lambda);
        for (int i = 0; i < 8; i++) mb[i] = -b[i];
        ldlt_solve(Hl, 8, mb, inc);
        // default setting_affineOptModeA/B >= 0: the full 8-dim step (the fixed-affine branches are off)
        float extrapFac = 1;
        if (lambda < lambdaExtrapolationLimit) extrapFac = sqrt(sqrt(lambdaExtrapolationLimit / lambda));
        for (int i = 0; i < 8; i++) inc[i] *= extrapFac;
        double incScaled[8];
        for (int i = 0; i < 8; i++) incScaled[i] = inc[i];
        for (int i = 0; i < 3; i++) incScaled[i] *= SCALE_XI_ROT;
        for (int i = 3; i < 6; i++) incScaled[i] *= SCALE_XI_TRANS;
        incScaled[6] *= SCALE_A;
        incScaled[7] *= SCALE_B;
        double ssum = 0;
        for (int i = 0; i < 8; i++) ssum += incScaled[i];
        if (!std::isfinite(ssum)) for (int i = 0; i < 8; i++) incScaled[i] = 0;
        const SE3 nw = SE3::exp(incScaled) * cur;
        double affn[2] = {aff[0] + incScaled[6], aff[1] + incScaled[7]};
        double resNew[6];
        calcRes(lvl, nw, affn, P.coarseCutoffTH * levelCutoffRepeat, resNew);
        const bool accept = (resNew[0] / resNew[1]) < (resOld[0] / resOld[1]);
        log_lvl.push_back(lvl);
        log_new.push_back(resNew[0] / resNew[1]);
        log_old.push_back(resOld[0] / resOld[1]);
        if (accept) {
          calcGSSSE(lvl, H, b, affn);
          for (int i = 0; i < 6; i++) resOld[i] = resNew[i];
          aff[0] = affn[0];
          aff[1] = affn[1];
          cur = nw;
          lambda *= 0.5;
        } else {
          lambda *= 4;
          if (lambda < lambdaExtrapolationLimit) lambda = lambdaExtrapolationLimit;
        }
        double nn = 0;
        for (int i = 0; i < 8; i++) nn += inc[i] * inc[i];
        log_inc.push_back(std::sqrt(nn));
        if (!(std::sqrt(nn) > 1e-3)) break;
      }
      lastResiduals[lvl] = sqrtf((float)(resOld[0] / resOld[1]));
      lastFlow[0] = resOld[2];
      lastFlow[1] = resOld[3];
      lastFlow[2] = resOld[4];
      if (iters_out) *iters_out = its;
      if (lastResiduals[lvl] > 1.5 * minResForAbort[lvl]) return false;
      if (levelCutoffRepeat > 1 && !haveRepeated) {
        lvl++;
        haveRepeated = true;
      }
    }
    T_out = cur;
    aff_out[0] = aff[0];
    aff_out[1] = aff[1];
    if ((P.affineOptModeA != 0 && (fabsf((float)aff_out[0]) > 1.2)) ||
        (P.affineOptModeB != 0 && (fabsf((float)aff_out[1]) > 200)))
      return false;
    double ra[2];
    relAff(aff_out, ra);
    if ((P.affineOptModeA == 0 && (fabsf(logf((float)ra[0])) > 1.5)) ||
        (P.affineOptModeB == 0 && (fabsf((float)ra[1]) > 200)))
      return false;
    if (P.affineOptModeA < 0) aff_out[0] = 0;
    if (P.affineOptModeB < 0) aff_out[1] = 0;
    return true;
  }
};

}  // namespace hso

using namespace hso;

extern "C" {

void* hso_trk_create(const hs_params* p, int W, int H, int levels, const float K4[4]) {
  TrackerO* t = new TrackerO();
  if (p) t->P = *p;
  else params_default(&t->P);
  t->init(W, H, levels, K4);
  return t;
}
void hso_trk_destroy(void* h) { delete (TrackerO*)h; }

static void load_pyr(TrackerO* t, std::vector<std::vector<float>>& dst, const float* const* pyr) {
  dst.resize(t->nlev);
  for (int l = 0; l < t->nlev; l++) dst[l].assign(pyr[l], pyr[l] + (size_t)t->w[l] * t->h[l] * 3);
}

// setCoarseTrackingRef: ref pyramid, exposure, aff_g2l and the IN residuals' centre projections + HdiF
void hso_trk_set_ref(void* h, const float* const* ref_pyr, float ab_exposure, const double aff[2], int n,
                     const float* cu, const float* cv, const float* cid, const float* hdi) {
  TrackerO* t = (TrackerO*)h;
  load_pyr(t, t->refPyr, ref_pyr);
  t->refExposure = ab_exposure;
  t->refAff[0] = aff[0];
  t->refAff[1] = aff[1];
  t->makeCoarseDepthL0(n, cu, cv, cid, hdi);
}
void hso_trk_set_frame(void* h, const float* const* new_pyr, float ab_exposure) {
  TrackerO* t = (TrackerO*)h;
  load_pyr(t, t->newPyr, new_pyr);
  t->newExposure = ab_exposure;
}
int hso_trk_get_ref(void* h, int lvl, float* u, float* v, float* id, float* color) {
  TrackerO* t = (TrackerO*)h;
  const int n = t->pc_n[lvl];
  if (u) std::memcpy(u, t->pc_u[lvl].data(), 4 * n);
  if (v) std::memcpy(v, t->pc_v[lvl].data(), 4 * n);
  if (id) std::memcpy(id, t->pc_idepth[lvl].data(), 4 * n);
  if (color) std::memcpy(color, t->pc_color[lvl].data(), 4 * n);
  return n;
}
// calcRes (+ calcGSSSE on its warped buffer): res6, H (8x8), b, warped count (padded)
void hso_trk_calc_res(void* h, int lvl, const double T7[7], const double aff[2], float cutoff, double res6[6],
                      double H64[64], double b8[8], int* n_warped) {
  TrackerO* t = (TrackerO*)h;
  const SE3 T = SE3::fromData(T7);
  t->calcRes(lvl, T, aff, cutoff, res6);
  if (n_warped) *n_warped = t->bw_n;
  if (H64 && b8) t->calcGSSSE(lvl, H64, b8, aff);
}
// test hook: the order the fp32 sums of calcRes / calcGSSSE are formed in (0 reference, 1 reversed point order),
// so tests can measure how far another summation order moves the LM trajectory
void hso_trk_set_sum_order(void* h, int order) { ((TrackerO*)h)->sum_order = order; }
int hso_trk_track(void* h, double T7[7], double aff[2], int coarsest, const double minRes[5], double lastRes[5],
                  double flow[3], int* iters) {
  TrackerO* t = (TrackerO*)h;
  SE3 T = SE3::fromData(T7);
  const bool ok = t->trackNewestCoarse(T, aff, coarsest, minRes, iters);
  T.toData(T7);
  for (int i = 0; i < 5; i++) lastRes[i] = t->lastResiduals[i];
  for (int i = 0; i < 3; i++) flow[i] = t->lastFlow[i];
  return ok ? 1 : 0;
}

// per-iteration LM log of the last trackNewestCoarse (accept test operands)
int hso_trk_get_log(void* h, int cap, int* lvl, double* new_ratio, double* old_ratio, double* inc_norm) {
  TrackerO* t = (TrackerO*)h;
  const int n = std::min<int>(cap, (int)t->log_lvl.size());
  for (int i = 0; i < n; i++) {
    lvl[i] = t->log_lvl[i];
    new_ratio[i] = t->log_new[i];
    old_ratio[i] = t->log_old[i];
    inc_norm[i] = t->log_inc[i];
  }
  return (int)t->log_lvl.size();
}

// System::trackNewCoarse try loop (Src/System.cpp:413-481): tries are lastF_2_fh candidates.
void hso_trk_track_tries(void* h, int n_tries, const double* tries7, const double aff_last[2],
                         const double lastCoarseRMSE[5], float reTrackThreshold, int coarsest, double T_out[7],
                         double aff_out[2], double achieved[5], double flow_out[3], int* have_one_good,
                         int* n_tried) {
  TrackerO* t = (TrackerO*)h;
  double achievedRes[5];
  for (int i = 0; i < 5; i++) achievedRes[i] = NAN;
  bool haveOneGood = false;
  double flowVecs[3] = {100, 100, 100};
  SE3 best;
  double bestAff[2] = {0, 0};
  int tried = 0;
  for (int i = 0; i < n_tries; i++) {
    double aff_this[2] = {aff_last[0], aff_last[1]};
    SE3 T = SE3::fromData(tries7 + 7 * i);
    const bool good = t->trackNewestCoarse(T, aff_this, coarsest, achievedRes, nullptr);
    tried++;
    if (good && std::isfinite((float)t->lastResiduals[0]) && !(t->lastResiduals[0] >= achievedRes[0])) {
      for (int k = 0; k < 3; k++) flowVecs[k] = t->lastFlow[k];
      bestAff[0] = aff_this[0];
      bestAff[1] = aff_this[1];
      best = T;
      haveOneGood = true;
    }
    if (haveOneGood)
      for (int k = 0; k < 5; k++)
        if (!std::isfinite((float)achievedRes[k]) || achievedRes[k] > t->lastResiduals[k])
          achievedRes[k] = t->lastResiduals[k];
    if (haveOneGood && achievedRes[0] < lastCoarseRMSE[0] * reTrackThreshold) break;
  }
  if (!haveOneGood) {
    flowVecs[0] = flowVecs[1] = flowVecs[2] = 0;
    bestAff[0] = aff_last[0];
    bestAff[1] = aff_last[1];
    best = SE3::fromData(tries7);
  }
  best.toData(T_out);
  aff_out[0] = bestAff[0];
  aff_out[1] = bestAff[1];
  for (int k = 0; k < 5; k++) achieved[k] = achievedRes[k];
  for (int k = 0; k < 3; k++) flow_out[k] = flowVecs[k];
  *have_one_good = haveOneGood ? 1 : 0;
  *n_tried = tried;
}

}  // extern "C"
