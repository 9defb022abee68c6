// ORACLE — TEST INFRASTRUCTURE ONLY (see oracle_common.h for the parity status).
//
// CPU restatement of the epipolar-search path:
//   ImmaturePoint::ImmaturePoint (ctor)   Src/ImmaturePoint.cpp:7-32
//   ImmaturePoint::traceOn                Src/ImmaturePoint.cpp:40-350
//   System::traceNewCoarse (the loop)     Src/Mapping.cpp:494-538
// Images are Frame::DirPyr[0]: AoS (I, dI/dx, dI/dy) floats, W*H*3.  Float expressions follow the
// reference's operation order; built with -ffp-contract=off (the reference's GCC default
// -ffp-contract=fast on an FMA host may fuse some of them — SURVEY.md §7 "Floating-point order").
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../include/hs_trace.h"
#include "oracle_common.h"

#define HS_TRC_MAXSLOT_ORACLE 64

namespace hso {

// The texel base index ix + iy*W is clamped to [0, W*H - W - 2] (the last base whose 2x2 taps lie in the
// buffer).  In-buffer reads, including the reference's row-wrapped ones at ix = W-1, are unchanged; the
// reference reads outside the image buffer (undefined behaviour) exactly where the clamp acts.
static inline int clamp_base(int ix, int iy, int W, int H) {
  long b = (long)ix + (long)iy * W;
  const long hi = (long)W * H - W - 2;
  return (int)(b < 0 ? 0 : (b > hi ? hi : b));
}
// getInterpolatedElement31 (Include/GlobalTypes.h:390-401) with the clamped base
static inline float t_interp31(const float* img, float x, float y, int W, int H) {
  int ix = (int)x, iy = (int)y;
  float dx = x - ix, dy = y - iy, dxdy = dx * dy;
  const float* bp = img + 3 * clamp_base(ix, iy, W, H);
  return dxdy * bp[3 * (1 + W)] + (dy - dxdy) * bp[3 * W] + (dx - dxdy) * bp[3] + (1 - dx - dy + dxdy) * bp[0];
}
// getInterpolatedElement33 (Include/GlobalTypes.h:377-388) with the clamped base
static inline V3f t_interp33(const float* img, float x, float y, int W, int H) {
  int ix = (int)x, iy = (int)y;
  float dx = x - ix, dy = y - iy, dxdy = dx * dy;
  const float* bp = img + 3 * clamp_base(ix, iy, W, H);
  const float w11 = dxdy, w01 = dy - dxdy, w10 = dx - dxdy, w00 = 1 - dx - dy + dxdy;
  const float *p11 = bp + 3 * (1 + W), *p01 = bp + 3 * W, *p10 = bp + 3;
  V3f r;
  r.x = w11 * p11[0] + w01 * p01[0] + w10 * p10[0] + w00 * bp[0];
  r.y = w11 * p11[1] + w01 * p01[1] + w10 * p10[1] + w00 * bp[1];
  r.z = w11 * p11[2] + w01 * p01[2] + w10 * p10[2] + w00 * bp[2];
  return r;
}
// getInterpolatedElement33BiLin (Include/GlobalTypes.h:355-375) with the clamped base
static inline V3f t_interp33BiLin(const float* img, float x, float y, int W, int H) {
  int ix = (int)x, iy = (int)y;
  const float* bp = img + 3 * clamp_base(ix, iy, W, H);
  float tl = bp[0], tr = bp[3], bl = bp[3 * W], br = bp[3 * W + 3];
  float dx = x - ix, dy = y - iy;
  float topInt = dx * tr + (1 - dx) * tl;
  float botInt = dx * br + (1 - dx) * bl;
  float leftInt = dy * bl + (1 - dy) * tl;
  float rightInt = dy * br + (1 - dy) * tr;
  V3f r;
  r.x = dx * rightInt + (1 - dx) * leftInt;
  r.y = rightInt - leftInt;
  r.z = botInt - topInt;
  return r;
}

// ImmaturePointStatus, Include/ImmaturePoint.h:25-31
enum { IPS_GOOD = 0, IPS_OOB, IPS_OUTLIER, IPS_SKIPPED, IPS_BADCONDITION, IPS_UNINITIALIZED };

struct ImmPt {
  int host;
  float u, v;
  float color[PN], weights[PN];
  float gradH[4];  // row-major Mat22f
  float energyTH;
  float quality;
  float idepth_min, idepth_max;
  int lastTraceStatus;
  float lastTraceUV[2];
  float lastTracePixelInterval;
  float my_type;
};

// ImmaturePoint ctor, Src/ImmaturePoint.cpp:7-32
static void immature_ctor(ImmPt& p, const float* hostImg, int W, int H, const hs_params& P) {
  p.idepth_min = 0;
  p.idepth_max = NAN;
  p.lastTraceStatus = IPS_UNINITIALIZED;
  p.lastTraceUV[0] = p.lastTraceUV[1] = 0;
  p.lastTracePixelInterval = 0;
  for (int k = 0; k < 4; k++) p.gradH[k] = 0;
  p.quality = NAN;  // the reference leaves it unset on the non-finite-colour early return
  for (int idx = 0; idx < PN; idx++) {
    const int dx = kPattern[idx][0], dy = kPattern[idx][1];
    V3f ptc = t_interp33BiLin(hostImg, p.u + dx, p.v + dy, W, H);
    p.color[idx] = ptc.x;
    if (!std::isfinite(p.color[idx])) {
      p.energyTH = NAN;
      return;
    }
    // gradH += g g^T  (Eigen: element (r,c) += g_r * g_c)
    p.gradH[0] = p.gradH[0] + ptc.y * ptc.y;
    p.gradH[1] = p.gradH[1] + ptc.y * ptc.z;
    p.gradH[2] = p.gradH[2] + ptc.z * ptc.y;
    p.gradH[3] = p.gradH[3] + ptc.z * ptc.z;
    p.weights[idx] = sqrtf(P.outlierTHSumComponent / (P.outlierTHSumComponent + (ptc.y * ptc.y + ptc.z * ptc.z)));
  }
  p.energyTH = PN * P.outlierTH;
  p.energyTH *= P.overallEnergyTHWeight * P.overallEnergyTHWeight;
  p.quality = 10000;
}

// Vec2f(x,y)^T * M * Vec2f(x,y): Eigen evaluates the row vector (v^T M) first, then the dot product
static inline float quad2(const float M[4], float x, float y) {
  const float r0 = x * M[0] + y * M[2];
  const float r1 = x * M[1] + y * M[3];
  return r0 * x + r1 * y;
}

// ImmaturePoint::traceOn, Src/ImmaturePoint.cpp:40-350.  KRKi row-major 3x3, Kt[3], aff[2] (Vec2f).
static int trace_on(ImmPt& p, const float* img, int W, int H, const float KRKi[9], const float Kt[3],
                    const float aff[2], const hs_params& P) {
  if (p.lastTraceStatus == IPS_OOB) return p.lastTraceStatus;
  const float maxPixSearch = (W + H) * P.maxPixSearch;
  auto oob = [&]() {
    p.lastTraceUV[0] = p.lastTraceUV[1] = -1;
    p.lastTracePixelInterval = 0;
    return p.lastTraceStatus = IPS_OOB;
  };
  // project min and max (:56-70)
  float pr[3];
  for (int r = 0; r < 3; r++) pr[r] = KRKi[r * 3 + 0] * p.u + KRKi[r * 3 + 1] * p.v + KRKi[r * 3 + 2] * 1.0f;
  float ptpMin[3];
  for (int r = 0; r < 3; r++) ptpMin[r] = pr[r] + Kt[r] * p.idepth_min;
  const float uMin = ptpMin[0] / ptpMin[2];
  const float vMin = ptpMin[1] / ptpMin[2];
  if (!(uMin > 4 && vMin > 4 && uMin < W - 5 && vMin < H - 5)) return oob();

  float dist, uMax, vMax, ptpMax[3];
  if (std::isfinite(p.idepth_max)) {  // :72-102
    for (int r = 0; r < 3; r++) ptpMax[r] = pr[r] + Kt[r] * p.idepth_max;
    uMax = ptpMax[0] / ptpMax[2];
    vMax = ptpMax[1] / ptpMax[2];
    if (!(uMax > 4 && vMax > 4 && uMax < W - 5 && vMax < H - 5)) return oob();
    dist = (uMin - uMax) * (uMin - uMax) + (vMin - vMax) * (vMin - vMax);
    dist = sqrtf(dist);
    if (dist < P.trace_slackInterval) {
      p.lastTraceUV[0] = (uMax + uMin) * 0.5f;
      p.lastTraceUV[1] = (vMax + vMin) * 0.5f;
      p.lastTracePixelInterval = dist;
      return p.lastTraceStatus = IPS_SKIPPED;
    }
  } else {  // :103-126
    dist = maxPixSearch;
    for (int r = 0; r < 3; r++) ptpMax[r] = pr[r] + Kt[r] * 0.01f;
    uMax = ptpMax[0] / ptpMax[2];
    vMax = ptpMax[1] / ptpMax[2];
    const float dx = uMax - uMin;
    const float dy = vMax - vMin;
    const float d = 1.0f / sqrtf(dx * dx + dy * dy);
    uMax = uMin + dist * dx * d;
    vMax = vMin + dist * dy * d;
    if (!(uMax > 4 && vMax > 4 && uMax < W - 5 && vMax < H - 5)) return oob();
  }
  // scale change (:130-137)
  if (!(p.idepth_min < 0 || (ptpMin[2] > 0.75f && ptpMin[2] < 1.5f))) return oob();

  // error bound in pixels (:140-157)
  float dx = P.trace_stepsize * (uMax - uMin);
  float dy = P.trace_stepsize * (vMax - vMin);
  const float a = quad2(p.gradH, dx, dy);
  const float b = quad2(p.gradH, dy, -dx);
  float errorInPixel = 0.2f + 0.2f * (a + b) / a;
  if (errorInPixel * P.trace_minImprovementFactor > dist && std::isfinite(p.idepth_max)) {
    p.lastTraceUV[0] = (uMax + uMin) * 0.5f;
    p.lastTraceUV[1] = (vMax + vMin) * 0.5f;
    p.lastTracePixelInterval = dist;
    return p.lastTraceStatus = IPS_BADCONDITION;
  }
  if (errorInPixel > 10) errorInPixel = 10;

  // discrete search (:161-233)
  dx /= dist;
  dy /= dist;
  if (dist > maxPixSearch) {
    uMax = uMin + maxPixSearch * dx;
    vMax = vMin + maxPixSearch * dy;
    dist = maxPixSearch;
  }
  int numSteps = 1.9999f + dist / P.trace_stepsize;
  const float R00 = KRKi[0], R01 = KRKi[1], R10 = KRKi[3], R11 = KRKi[4];  // Rplane = topLeftCorner<2,2>
  const float randShift = uMin * 1000 - floorf(uMin * 1000);
  float ptx = uMin - randShift * dx;
  float pty = vMin - randShift * dy;
  float rot[PN][2];
  for (int idx = 0; idx < PN; idx++) {
    const float px = (float)kPattern[idx][0], py = (float)kPattern[idx][1];
    rot[idx][0] = R00 * px + R01 * py;
    rot[idx][1] = R10 * px + R11 * py;
  }
  if (!std::isfinite(dx) || !std::isfinite(dy)) return oob();

  float errors[100];
  float bestU = 0, bestV = 0, bestEnergy = 1e10f;
  int bestIdx = -1;
  if (numSteps >= 100) numSteps = 99;
  for (int i = 0; i < numSteps; i++) {
    float energy = 0;
    for (int idx = 0; idx < PN; idx++) {
      const float hitColor = t_interp31(img, (float)(ptx + rot[idx][0]), (float)(pty + rot[idx][1]), W, H);
      if (!std::isfinite(hitColor)) {
        energy += 1e5f;
        continue;
      }
      const float residual = hitColor - (float)(aff[0] * p.color[idx] + aff[1]);
      const float hw = fabsf(residual) < P.huberTH ? 1 : P.huberTH / fabsf(residual);
      energy += hw * residual * residual * (2 - hw);
    }
    errors[i] = energy;
    if (energy < bestEnergy) {
      bestU = ptx;
      bestV = pty;
      bestEnergy = energy;
      bestIdx = i;
    }
    ptx += dx;
    pty += dy;
  }
  // second best outside +-radius (:236-244)
  float secondBest = 1e10f;
  for (int i = 0; i < numSteps; i++)
    if ((i < bestIdx - P.minTraceTestRadius || i > bestIdx + P.minTraceTestRadius) && errors[i] < secondBest)
      secondBest = errors[i];
  const float newQuality = secondBest / bestEnergy;
  if (newQuality < p.quality || numSteps > 10) p.quality = newQuality;

  // GN along the line (:247-305)
  float uBak = bestU, vBak = bestV, gnstepsize = 1, stepBack = 0;
  if (P.trace_GNIterations > 0) bestEnergy = 1e5f;
  for (int it = 0; it < P.trace_GNIterations; it++) {
    float Hs = 1, bs = 0, energy = 0;
    for (int idx = 0; idx < PN; idx++) {
      const V3f hc = t_interp33(img, (float)(bestU + rot[idx][0]), (float)(bestV + rot[idx][1]), W, H);
      if (!std::isfinite(hc.x)) {
        energy += 1e5f;
        continue;
      }
      const float residual = hc.x - (aff[0] * p.color[idx] + aff[1]);
      const float dResdDist = dx * hc.y + dy * hc.z;
      const float hw = fabsf(residual) < P.huberTH ? 1 : P.huberTH / fabsf(residual);
      Hs += hw * dResdDist * dResdDist;
      bs += hw * residual * dResdDist;
      energy += p.weights[idx] * p.weights[idx] * hw * residual * residual * (2 - hw);
    }
    if (energy > bestEnergy) {
      stepBack *= 0.5f;
      bestU = uBak + stepBack * dx;
      bestV = vBak + stepBack * dy;
    } else {
      float step = -gnstepsize * bs / Hs;
      if (step < -0.5f) step = -0.5f;
      else if (step > 0.5f) step = 0.5f;
      if (!std::isfinite(step)) step = 0;
      uBak = bestU;
      vBak = bestV;
      stepBack = step;
      bestU += step * dx;
      bestV += step * dy;
      bestEnergy = energy;
    }
    if (fabsf(stepBack) < P.trace_GNThreshold) break;
  }

  // energy-based outlier (:309-321)
  if (!(bestEnergy < p.energyTH * P.trace_extraSlackOnTH)) {
    p.lastTracePixelInterval = 0;
    p.lastTraceUV[0] = p.lastTraceUV[1] = -1;
    if (p.lastTraceStatus == IPS_OUTLIER) return p.lastTraceStatus = IPS_OOB;
    return p.lastTraceStatus = IPS_OUTLIER;
  }

  // new interval (:325-349)
  if (dx * dx > dy * dy) {
    p.idepth_min = (pr[2] * (bestU - errorInPixel * dx) - pr[0]) / (Kt[0] - Kt[2] * (bestU - errorInPixel * dx));
    p.idepth_max = (pr[2] * (bestU + errorInPixel * dx) - pr[0]) / (Kt[0] - Kt[2] * (bestU + errorInPixel * dx));
  } else {
    p.idepth_min = (pr[2] * (bestV - errorInPixel * dy) - pr[1]) / (Kt[1] - Kt[2] * (bestV - errorInPixel * dy));
    p.idepth_max = (pr[2] * (bestV + errorInPixel * dy) - pr[1]) / (Kt[1] - Kt[2] * (bestV + errorInPixel * dy));
  }
  if (p.idepth_min > p.idepth_max) std::swap(p.idepth_min, p.idepth_max);
  if (!std::isfinite(p.idepth_min) || !std::isfinite(p.idepth_max) || (p.idepth_max < 0)) {
    p.lastTracePixelInterval = 0;
    p.lastTraceUV[0] = p.lastTraceUV[1] = -1;
    return p.lastTraceStatus = IPS_OUTLIER;
  }
  p.lastTracePixelInterval = 2 * errorInPixel;
  p.lastTraceUV[0] = bestU;
  p.lastTraceUV[1] = bestV;
  return p.lastTraceStatus = IPS_GOOD;
}


// ============================================================================ point activation
// CoarseDistanceMap (Src/CoarseTracker.cpp:698-868): fwdWarpedIDDistFinal at pyramid level 1 and its BFS.
struct DistMap {
  int w1 = 0, h1 = 0;
  std::vector<float> d;
  std::vector<int> l1, l2;  // bfsList1 / bfsList2 as packed (x, y) pairs
  long long st_grows = 0, st_steps = 0, st_cells = 0;  // statistics: BFS calls, non-empty steps, frontier cells
  void grow(int bfsNum) {
    st_grows++;  // growDistBFS, :759-857 (k even: 4-neighbourhood, k odd: 8-neighbourhood)
    for (int k = 1; k < 40; k++) {
      int bfsNum2 = bfsNum;
      if (bfsNum2) st_steps++;
      st_cells += bfsNum2;
      std::swap(l1, l2);
      bfsNum = 0;
      for (int i = 0; i < bfsNum2; i++) {
        const int x = l2[2 * i], y = l2[2 * i + 1];
        if (x == 0 || y == 0 || x == w1 - 1 || y == h1 - 1) continue;
        const int idx = x + y * w1;
        const int nb = (k % 2 == 0) ? 4 : 8;
        static const int off[8][2] = {{1, 0}, {-1, 0}, {0, 1}, {0, -1}, {1, 1}, {-1, 1}, {-1, -1}, {1, -1}};
        for (int j = 0; j < nb; j++) {
          const int q = idx + off[j][0] + off[j][1] * w1;
          if (d[q] > k) {
            d[q] = k;
            l1[2 * bfsNum] = x + off[j][0];
            l1[2 * bfsNum + 1] = y + off[j][1];
            bfsNum++;
          }
        }
      }
    }
  }
  void add(int u, int v) {  // addIntoDistFinal, :860-866
    l1[0] = u;
    l1[1] = v;
    d[u + w1 * v] = 0;
    grow(1);
  }
};

// ImmaturePointTemporaryResidual (Include/ImmaturePoint.h:13-22)
struct TmpRes {
  int target;
  int state_state, state_NewState;
  float state_energy, state_NewEnergy;
};

struct ActCalib {
  int W, H;
  float fxl, fyl, cxl, cyl, fxli, fyli;
};

// ImmaturePoint::linearizeResidual, Src/ImmaturePoint.cpp:389-451
static double imm_linearize_residual(const ImmPt& p, float outlierTHSlack, TmpRes& r, float& Hdd, float& bd,
                                     float idepth, const float* dIl, const hs_act_pair& pc, const ActCalib& c,
                                     const hs_params& P) {
  if (r.state_state == HS_RES_OOB) {
    r.state_NewState = HS_RES_OOB;
    return r.state_energy;
  }
  float energyLeft = 0;
  const float affLL0 = pc.aff[0], affLL1 = pc.aff[1];
  for (int idx = 0; idx < PN; idx++) {
    const int dx = kPattern[idx][0], dy = kPattern[idx][1];
    // projectPoint(u, v, idepth, dx, dy, Calib, PRE_RTll, PRE_tTll, ...)  Include/DirectProjection.h:20-38
    float KliP[3] = {(p.u + dx - c.cxl) * c.fxli, (p.v + dy - c.cyl) * c.fyli, 1};
    float ptp[3], Rk[3];
    mv3f(pc.RTll, KliP, Rk);
    for (int i = 0; i < 3; i++) ptp[i] = Rk[i] + pc.tTll[i] * idepth;
    const float drescale = 1.0f / ptp[2];
    if (!(drescale > 0)) {
      r.state_NewState = HS_RES_OOB;
      return r.state_energy;
    }
    const float u = ptp[0] * drescale, v = ptp[1] * drescale;
    const float Ku = u * c.fxl + c.cxl, Kv = v * c.fyl + c.cyl;
    if (!(Ku > 1.1f && Kv > 1.1f && Ku < (c.W - 3) && Kv < (c.H - 3))) {
      r.state_NewState = HS_RES_OOB;
      return r.state_energy;
    }
    const V3f hit = interp33(dIl, Ku, Kv, c.W);
    if (!std::isfinite(hit.x)) {
      r.state_NewState = HS_RES_OOB;
      return r.state_energy;
    }
    const float residual = hit.x - (affLL0 * p.color[idx] + affLL1);
    float hw = fabsf(residual) < P.huberTH ? 1 : P.huberTH / fabsf(residual);
    energyLeft += p.weights[idx] * p.weights[idx] * hw * residual * residual * (2 - hw);
    const float dxInterp = hit.y * c.fxl;
    const float dyInterp = hit.z * c.fyl;
    // derive_idepth, Include/DirectProjection.h:7-10
    const float d_idepth =
        (dxInterp * drescale * (pc.tTll[0] - pc.tTll[2] * u) + dyInterp * drescale * (pc.tTll[1] - pc.tTll[2] * v)) *
        SCALE_IDEPTH;
    hw *= p.weights[idx] * p.weights[idx];
    Hdd += (hw * d_idepth) * d_idepth;
    bd += (hw * residual) * d_idepth;
  }
  if (energyLeft > p.energyTH * outlierTHSlack) {
    energyLeft = p.energyTH * outlierTHSlack;
    r.state_NewState = HS_RES_OUT;
  } else {
    r.state_NewState = HS_RES_IN;
  }
  r.state_NewEnergy = energyLeft;
  return energyLeft;
}

// System::optimizeImmaturePoint, Src/FullSystemOptPoint.cpp:24-175 (minObs = 1).  Returns true when a MapPoint is
// made; idepth / res_in (bit = target window frame, state IN) describe it.
static bool optimize_immature_point(const ImmPt& p, int hostF, int nF, const float* const* imgs,
                                    const hs_act_pair* pairs, const ActCalib& c, const hs_params& P, float& idepth_out,
                                    uint8_t& res_in) {
  TmpRes res[8];
  int nres = 0;
  for (int f = 0; f < nF; f++) {
    if (f == hostF) continue;
    TmpRes& r = res[nres++];
    r.state_NewEnergy = r.state_energy = 0;
    r.state_NewState = HS_RES_OUT;
    r.state_state = HS_RES_IN;
    r.target = f;
  }
  float lastEnergy = 0, lastHdd = 0, lastbd = 0;
  float currentIdepth = (p.idepth_max + p.idepth_min) * 0.5f;
  for (int i = 0; i < nres; i++) {
    lastEnergy += imm_linearize_residual(p, 1000, res[i], lastHdd, lastbd, currentIdepth, imgs[res[i].target],
                                         pairs[hostF * nF + res[i].target], c, P);
    res[i].state_state = res[i].state_NewState;
    res[i].state_energy = res[i].state_NewEnergy;
  }
  if (!std::isfinite(lastEnergy) || lastHdd < P.minIdepthH_act) return false;
  float lambda = 0.1;
  for (int iteration = 0; iteration < P.GNItsOnPointActivation; iteration++) {
    float H = lastHdd;
    H *= 1 + lambda;
    const float step = (1.0 / H) * lastbd;
    const float newIdepth = currentIdepth - step;
    float newHdd = 0, newbd = 0, newEnergy = 0;
    for (int i = 0; i < nres; i++)
      newEnergy += imm_linearize_residual(p, 1, res[i], newHdd, newbd, newIdepth, imgs[res[i].target],
                                          pairs[hostF * nF + res[i].target], c, P);
    if (!std::isfinite(lastEnergy) || newHdd < P.minIdepthH_act) return false;
    if (newEnergy < lastEnergy) {
      currentIdepth = newIdepth;
      lastHdd = newHdd;
      lastbd = newbd;
      lastEnergy = newEnergy;
      for (int i = 0; i < nres; i++) {
        res[i].state_state = res[i].state_NewState;
        res[i].state_energy = res[i].state_NewEnergy;
      }
      lambda *= 0.5;
    } else {
      lambda *= 5;
    }
    if (fabsf(step) < 0.0001 * currentIdepth) break;
  }
  if (!std::isfinite(currentIdepth)) return false;
  int numGoodRes = 0;
  res_in = 0;
  for (int i = 0; i < nres; i++)
    if (res[i].state_state == HS_RES_IN) {
      numGoodRes++;
      res_in |= (uint8_t)(1u << res[i].target);
    }
  if (numGoodRes < 1) return false;
  if (!std::isfinite(p.energyTH)) return false;  // MapPoint ctor copies energyTH (Include/MapPoint.h:92-115)
  idepth_out = currentIdepth;
  return true;
}

struct Tracer {
  hs_params P;
  int W, H;
  std::vector<ImmPt> pts;
  DistMap dm;
};

}  // namespace hso

using namespace hso;

extern "C" {

void* hso_trc_create(const hs_params* params, int W, int H) {
  Tracer* t = new Tracer();
  if (params) t->P = *params;
  else params_default(&t->P);
  t->W = W;
  t->H = H;
  return t;
}

void hso_trc_destroy(void* h) { delete (Tracer*)h; }

// new ImmaturePoints (ctor) on host keyframes: host_imgs[nH] AoS (I,dx,dy); points append in the given order
int hso_trc_add_points(void* h, int nH, const float* const* host_imgs, int n, const int* host, const float* u,
                       const float* v) {
  Tracer* t = (Tracer*)h;
  for (int i = 0; i < n; i++) {
    if (host[i] < 0 || host[i] >= nH) return -1;
    ImmPt p;
    std::memset(&p, 0, sizeof(p));
    p.host = host[i];
    p.u = u[i];
    p.v = v[i];
    p.my_type = 1;
    immature_ctor(p, host_imgs[host[i]], t->W, t->H, t->P);
    t->pts.push_back(p);
  }
  return 0;
}

// overwrite the search state (a point traced before): idepth_min/max, quality, lastTraceStatus (all nullable)
void hso_trc_set_state(void* h, const float* idepth_min, const float* idepth_max, const float* quality,
                       const uint8_t* status, const float* interval) {
  Tracer* t = (Tracer*)h;
  for (size_t i = 0; i < t->pts.size(); i++) {
    if (idepth_min) t->pts[i].idepth_min = idepth_min[i];
    if (idepth_max) t->pts[i].idepth_max = idepth_max[i];
    if (quality) t->pts[i].quality = quality[i];
    if (status) t->pts[i].lastTraceStatus = status[i];
    if (interval) t->pts[i].lastTracePixelInterval = interval[i];
  }
}

// System::traceNewCoarse loop body: every point traced on new_img with its host's (KRKi, Kt, aff).
// counts6[status]++ (IPS_* order).
void hso_trc_trace(void* h, const float* new_img, const hs_trace_host* hosts, int* counts6) {
  Tracer* t = (Tracer*)h;
  if (counts6) for (int k = 0; k < 6; k++) counts6[k] = 0;
  for (auto& p : t->pts) {
    const hs_trace_host& hh = hosts[p.host];
    trace_on(p, new_img, t->W, t->H, hh.KRKi, hh.Kt, hh.aff, t->P);
    if (counts6) counts6[p.lastTraceStatus]++;
  }
}

void hso_trc_get(void* h, uint8_t* status, float* idepth_min, float* idepth_max, float* quality, float* uv,
                 float* interval, float* energyTH, float* color, float* weights, float* gradH) {
  Tracer* t = (Tracer*)h;
  for (size_t i = 0; i < t->pts.size(); i++) {
    const ImmPt& p = t->pts[i];
    if (status) status[i] = (uint8_t)p.lastTraceStatus;
    if (idepth_min) idepth_min[i] = p.idepth_min;
    if (idepth_max) idepth_max[i] = p.idepth_max;
    if (quality) quality[i] = p.quality;
    if (uv) { uv[2 * i] = p.lastTraceUV[0]; uv[2 * i + 1] = p.lastTraceUV[1]; }
    if (interval) interval[i] = p.lastTracePixelInterval;
    if (energyTH) energyTH[i] = p.energyTH;
    for (int k = 0; k < PN; k++) {
      if (color) color[PN * i + k] = p.color[k];
      if (weights) weights[PN * i + k] = p.weights[k];
    }
    if (gradH) for (int k = 0; k < 4; k++) gradH[4 * i + k] = p.gradH[k];
  }
}

void hso_trc_set_types(void* h, const float* my_type) {
  Tracer* t = (Tracer*)h;
  for (size_t i = 0; i < t->pts.size(); i++) t->pts[i].my_type = my_type[i];
}

// System::activatePointsMT, Src/Mapping.cpp:330-480.  frame_imgs[nF]: DirPyr[0] of the window keyframes (AoS).
int hso_trc_activate(void* h, const float K4[4], int nF, const float* const* frame_imgs, const hs_act_frame* frames,
                     const hs_act_pair* pairs, int n_active, const int* act_frame, const float* act_u,
                     const float* act_v, const float* act_idepth, int ef_nPoints, float* currentMinActDist,
                     int n_order, const int* order, uint8_t* action, float* idepth, uint8_t* res_in, int* activated,
                     int* n_activated) {
  Tracer* t = (Tracer*)h;
  const hs_params& P = t->P;
  const int n = (int)t->pts.size();
  float& cmad = *currentMinActDist;
  // :332-352
  if (ef_nPoints < P.desiredPointDensity * 0.66) cmad -= 0.8;
  if (ef_nPoints < P.desiredPointDensity * 0.8) cmad -= 0.5;
  else if (ef_nPoints < P.desiredPointDensity * 0.9) cmad -= 0.2;
  else if (ef_nPoints < P.desiredPointDensity) cmad -= 0.1;
  if (ef_nPoints > P.desiredPointDensity * 1.5) cmad += 0.8;
  if (ef_nPoints > P.desiredPointDensity * 1.3) cmad += 0.5;
  if (ef_nPoints > P.desiredPointDensity * 1.15) cmad += 0.2;
  if (ef_nPoints > P.desiredPointDensity) cmad += 0.1;
  if (cmad < 0) cmad = 0;
  if (cmad > 4) cmad = 4;

  const int newest = nF - 1;
  DistMap& dm = t->dm;
  dm.w1 = t->W >> 1;
  dm.h1 = t->H >> 1;
  const int wh1 = dm.w1 * dm.h1;
  dm.d.assign(wh1, 1000.f);
  dm.l1.assign(2 * wh1, 0);
  dm.l2.assign(2 * wh1, 0);
  // makeDistanceMap, Src/CoarseTracker.cpp:726-756
  int numItems = 0;
  for (int i = 0; i < n_active; i++) {
    const int f = act_frame[i];
    if (f == newest) continue;
    const float* KRKi = frames[f].KRKi;
    const float* Kt = frames[f].Kt;
    float pt[3] = {act_u[i], act_v[i], 1}, ptp[3];
    mv3f(KRKi, pt, ptp);
    for (int k = 0; k < 3; k++) ptp[k] = ptp[k] + Kt[k] * act_idepth[i];
    const int u = ptp[0] / ptp[2] + 0.5f;
    const int v = ptp[1] / ptp[2] + 0.5f;
    if (!(u > 0 && v > 0 && u < dm.w1 && v < dm.h1)) continue;
    dm.d[u + dm.w1 * v] = 0;
    dm.l1[2 * numItems] = u;
    dm.l1[2 * numItems + 1] = v;
    numItems++;
  }
  dm.grow(numItems);

  ActCalib c{t->W, t->H, K4[0], K4[1], K4[2], K4[3], 1.0f / K4[0], 1.0f / K4[1]};
  std::vector<int> frame_of_slot(HS_TRC_MAXSLOT_ORACLE, -1);
  for (int f = 0; f < nF; f++) frame_of_slot[frames[f].slot] = f;
  for (int i = 0; i < n; i++) {
    if (action) action[i] = HS_ACT_KEEP;
    if (res_in) res_in[i] = 0;
  }
  std::vector<int> toOptimize;
  const int m = order ? n_order : n;
  for (int j = 0; j < m; j++) {  // :364-429
    const int i = order ? order[j] : j;
    ImmPt& ph = t->pts[i];
    const int f = frame_of_slot[ph.host];
    if (f < 0 || f == newest) continue;
    if (!std::isfinite(ph.idepth_max) || ph.lastTraceStatus == IPS_OUTLIER) {
      if (action) action[i] = HS_ACT_DELETED;
      continue;
    }
    const bool canActivate = (ph.lastTraceStatus == IPS_GOOD || ph.lastTraceStatus == IPS_SKIPPED ||
                              ph.lastTraceStatus == IPS_BADCONDITION || ph.lastTraceStatus == IPS_OOB) &&
                             ph.lastTracePixelInterval < 8 && ph.quality > P.minTraceQuality &&
                             (ph.idepth_max + ph.idepth_min) > 0;
    if (!canActivate) {
      if (frames[f].flagged_for_marg || ph.lastTraceStatus == IPS_OOB)
        if (action) action[i] = HS_ACT_DELETED;
      continue;
    }
    float pt[3] = {ph.u, ph.v, 1}, ptp[3];
    mv3f(frames[f].KRKi, pt, ptp);
    const float mid = 0.5f * (ph.idepth_max + ph.idepth_min);
    for (int k = 0; k < 3; k++) ptp[k] = ptp[k] + frames[f].Kt[k] * mid;
    const int u = ptp[0] / ptp[2] + 0.5f;
    const int v = ptp[1] / ptp[2] + 0.5f;
    if (u > 0 && v > 0 && u < dm.w1 && v < dm.h1) {
      const float dist = dm.d[u + dm.w1 * v] + (ptp[0] - floorf((float)(ptp[0])));
      if (dist >= cmad * ph.my_type) {
        dm.add(u, v);
        toOptimize.push_back(i);
      }
    } else {
      if (action) action[i] = HS_ACT_DELETED;
    }
  }
  // activatePointsMT_Reductor + the result loop, :434-480: every optimized point is either activated or deleted
  int na = 0;
  for (int i : toOptimize) {
    const ImmPt& ph = t->pts[i];
    const int f = frame_of_slot[ph.host];
    float id = 0;
    uint8_t mask = 0;
    const bool ok = optimize_immature_point(ph, f, nF, frame_imgs, pairs, c, P, id, mask);
    if (action) action[i] = ok ? HS_ACT_ACTIVATED : HS_ACT_DELETED;
    if (ok) {
      if (idepth) idepth[i] = id;
      if (res_in) res_in[i] = mask;
      if (activated) activated[na] = i;
      na++;
    }
  }
  if (n_activated) *n_activated = na;
  return 0;
}

void hso_trc_distance_map(void* h, float* out) {
  Tracer* t = (Tracer*)h;
  for (size_t i = 0; i < t->dm.d.size(); i++) out[i] = t->dm.d[i];
}

void hso_trc_bfs_stats(void* h, long long* out3) {
  Tracer* t = (Tracer*)h;
  out3[0] = t->dm.st_grows;
  out3[1] = t->dm.st_steps;
  out3[2] = t->dm.st_cells;
}

void hso_trc_compact(void* h, const uint8_t* keep) {
  Tracer* t = (Tracer*)h;
  std::vector<ImmPt> kept;
  for (size_t i = 0; i < t->pts.size(); i++)
    if (keep[i]) kept.push_back(t->pts[i]);
  t->pts.swap(kept);
}

}  // extern "C"
