// hs_trace_kernels.hip — ImmaturePoint ctor and traceOn as CDNA4 kernels.
//
// hs_k_imm_ctor   one thread per new point: 8 BiLin taps of the host KF (Src/ImmaturePoint.cpp:7-32).
// hs_k_trace_on   one wave64 per immature point (Src/ImmaturePoint.cpp:40-350):
//   * the scalar prelude (projection of idepth_min / idepth_max, OOB / SKIPPED / BADCONDITION decisions,
//     errorInPixel, numSteps, randShift, rotated pattern) is wave-uniform and computed in every lane;
//   * the discrete search puts step i on lane i (and i-64 on a second pass when numSteps > 64): 8 taps of
//     getInterpolatedElement31 each, summed in pattern order exactly as the reference;
//     the step positions are the reference's running sums ptx += dx (a uniform loop, not i*dx);
//   * best (first minimum) and second best (outside +-radius) are butterfly reductions over the wave;
//   * the 3 GN iterations put pattern pixel idx on lane idx; H, b and energy are summed in pattern order
//     from shuffles so every float matches the sequential reference.
// Images are level 0 as float4 (I, dI/dx, dI/dy, 0).  fp contraction is off: operation order as the oracle.
#include <hip/hip_runtime.h>

#include "hs_trace_kernels.h"

#pragma clang fp contract(off)
#include "hs_interp.h"

namespace {

using hs_img::clamp_base;
using hs_img::interp31;
using hs_img::interp33;
using hs_img::interp33BiLin;

constexpr int kPat[8][2] = {{0, -2}, {-1, -1}, {1, -1}, {-2, 0}, {0, 0}, {2, 0}, {-1, 1}, {0, 2}};

// v^T M v with Eigen's evaluation order (row vector first, then the dot product)
__device__ __forceinline__ float quad2(float g0, float g1, float g2, float g3, float x, float y) {
  const float r0 = x * g0 + y * g2;
  const float r1 = x * g1 + y * g3;
  return r0 * x + r1 * y;
}

__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o));
  return v;
}

}  // namespace

__global__ __launch_bounds__(256) void hs_k_imm_ctor(HsImmCtorArgs a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  const int p = a.first + i;
  const int h = a.host[p];
  const float4* img = a.host_img[h];
  const float u = a.u[p], v = a.v[p];
  float col[8], wgt[8];
  float g0 = 0, g1 = 0, g2 = 0, g3 = 0;
  float eTH = 0, q = 10000;
  bool bad = false;
#pragma unroll
  for (int idx = 0; idx < 8; idx++) {
    const float3 ptc = interp33BiLin(img, u + kPat[idx][0], v + kPat[idx][1], a.W, a.H);
    col[idx] = bad ? 0.f : ptc.x;
    wgt[idx] = 0;
    if (bad) continue;
    if (!isfinite(ptc.x)) {  // energyTH = NaN; return (quality left unset: NaN here, as the oracle)
      bad = true;
      continue;
    }
    g0 = g0 + ptc.y * ptc.y;
    g1 = g1 + ptc.y * ptc.z;
    g2 = g2 + ptc.z * ptc.y;
    g3 = g3 + ptc.z * ptc.z;
    wgt[idx] = sqrtf(a.outlierTHSumComponent / (a.outlierTHSumComponent + (ptc.y * ptc.y + ptc.z * ptc.z)));
  }
  if (bad) {
    eTH = __builtin_nanf("");
    q = __builtin_nanf("");
  } else {
    eTH = 8 * a.outlierTH;
    eTH *= a.overallEnergyTHWeight * a.overallEnergyTHWeight;
  }
  float4* c4 = reinterpret_cast<float4*>(a.color + 8 * (size_t)p);
  float4* w4 = reinterpret_cast<float4*>(a.weights + 8 * (size_t)p);
  c4[0] = make_float4(col[0], col[1], col[2], col[3]);
  c4[1] = make_float4(col[4], col[5], col[6], col[7]);
  w4[0] = make_float4(wgt[0], wgt[1], wgt[2], wgt[3]);
  w4[1] = make_float4(wgt[4], wgt[5], wgt[6], wgt[7]);
  reinterpret_cast<float4*>(a.gradH)[p] = make_float4(g0, g1, g2, g3);
  a.energyTH[p] = eTH;
  a.quality[p] = q;
  a.idepth_min[p] = 0;
  a.idepth_max[p] = __builtin_nanf("");
  a.status[p] = HS_IPS_UNINITIALIZED;
  a.uv[2 * p] = 0;
  a.uv[2 * p + 1] = 0;
  a.interval[p] = 0;
}

__global__ __launch_bounds__(256) void hs_k_trace_on(HsTraceArgs a) {
  const int lane = threadIdx.x & 63;
  const int p = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
  if (p >= a.n) return;
  const int W = a.W, H = a.H;
  int st = a.status[p];
  if (st == HS_IPS_OOB) {  // sticky (:42)
    if (lane == 0) a.steps[p] = 0;
    return;
  }

  const hs_trace_host hh = a.hosts[a.host[p]];
  const float u = a.u[p], v = a.v[p];
  const float4 gH = reinterpret_cast<const float4*>(a.gradH)[p];
  float idepth_min = a.idepth_min[p], idepth_max = a.idepth_max[p];
  float quality = a.quality[p];
  const float energyTH = a.energyTH[p];
  const float maxPixSearch = (W + H) * a.maxPixSearch;

  float outU = -1, outV = -1, outI = 0;
  int outS = HS_IPS_OOB;
  int searched = 0;
  bool write_interval = false;

  do {
    // project min and max (:56-70)
    float pr[3], ptpMin[3];
#pragma unroll
    for (int r = 0; r < 3; r++) pr[r] = hh.KRKi[r * 3 + 0] * u + hh.KRKi[r * 3 + 1] * v + hh.KRKi[r * 3 + 2] * 1.0f;
#pragma unroll
    for (int r = 0; r < 3; r++) ptpMin[r] = pr[r] + hh.Kt[r] * idepth_min;
    const float uMin = ptpMin[0] / ptpMin[2];
    const float vMin = ptpMin[1] / ptpMin[2];
    if (!(uMin > 4 && vMin > 4 && uMin < W - 5 && vMin < H - 5)) break;  // OOB

    float dist, uMax, vMax;
    const bool finiteMax = isfinite(idepth_max);
    if (finiteMax) {  // :72-102
      float ptpMax[3];
#pragma unroll
      for (int r = 0; r < 3; r++) ptpMax[r] = pr[r] + hh.Kt[r] * idepth_max;
      uMax = ptpMax[0] / ptpMax[2];
      vMax = ptpMax[1] / ptpMax[2];
      if (!(uMax > 4 && vMax > 4 && uMax < W - 5 && vMax < H - 5)) break;
      dist = (uMin - uMax) * (uMin - uMax) + (vMin - vMax) * (vMin - vMax);
      dist = sqrtf(dist);
      if (dist < a.slackInterval) {
        outU = (uMax + uMin) * 0.5f;
        outV = (vMax + vMin) * 0.5f;
        outI = dist;
        outS = HS_IPS_SKIPPED;
        break;
      }
    } else {  // :103-126
      dist = maxPixSearch;
      float ptpMax[3];
#pragma unroll
      for (int r = 0; r < 3; r++) ptpMax[r] = pr[r] + hh.Kt[r] * 0.01f;
      uMax = ptpMax[0] / ptpMax[2];
      vMax = ptpMax[1] / ptpMax[2];
      const float ddx = uMax - uMin;
      const float ddy = vMax - vMin;
      const float d = 1.0f / sqrtf(ddx * ddx + ddy * ddy);
      uMax = uMin + dist * ddx * d;
      vMax = vMin + dist * ddy * d;
      if (!(uMax > 4 && vMax > 4 && uMax < W - 5 && vMax < H - 5)) break;
    }
    if (!(idepth_min < 0 || (ptpMin[2] > 0.75f && ptpMin[2] < 1.5f))) break;  // scale change (:130-137)

    // error bound (:140-157)
    float dx = a.stepsize * (uMax - uMin);
    float dy = a.stepsize * (vMax - vMin);
    const float qa = quad2(gH.x, gH.y, gH.z, gH.w, dx, dy);
    const float qb = quad2(gH.x, gH.y, gH.z, gH.w, dy, -dx);
    float errorInPixel = 0.2f + 0.2f * (qa + qb) / qa;
    if (errorInPixel * a.minImprovementFactor > dist && finiteMax) {
      outU = (uMax + uMin) * 0.5f;
      outV = (vMax + vMin) * 0.5f;
      outI = dist;
      outS = HS_IPS_BADCONDITION;
      break;
    }
    if (errorInPixel > 10) errorInPixel = 10;

    // discrete search (:161-233)
    dx /= dist;
    dy /= dist;
    if (dist > maxPixSearch) dist = maxPixSearch;  // (uMax, vMax are not used past this point)
    int numSteps = 1.9999f + dist / a.stepsize;
    const float R00 = hh.KRKi[0], R01 = hh.KRKi[1], R10 = hh.KRKi[3], R11 = hh.KRKi[4];
    const float randShift = uMin * 1000 - floorf(uMin * 1000);
    const float ptx0 = uMin - randShift * dx;
    const float pty0 = vMin - randShift * dy;
    float rx[8], ry[8];
#pragma unroll
    for (int idx = 0; idx < 8; idx++) {
      const float px = (float)kPat[idx][0], py = (float)kPat[idx][1];
      rx[idx] = R00 * px + R01 * py;
      ry[idx] = R10 * px + R11 * py;
    }
    if (!isfinite(dx) || !isfinite(dy)) break;  // OOB
    if (numSteps >= 100) numSteps = 99;
    searched = numSteps;

    // step positions: the reference's running sums, lane i <- step i, lane i <- step i+64
    float x0 = 0, y0 = 0, x1 = 0, y1 = 0;
    {
      float x = ptx0, y = pty0;
      for (int j = 0; j < numSteps; j++) {
        if (j == lane) { x0 = x; y0 = y; }
        if (j == lane + 64) { x1 = x; y1 = y; }
        x += dx;
        y += dy;
      }
    }
    const float c0 = a.color[8 * (size_t)p + 0], c1 = a.color[8 * (size_t)p + 1], c2 = a.color[8 * (size_t)p + 2],
                c3 = a.color[8 * (size_t)p + 3], c4 = a.color[8 * (size_t)p + 4], c5 = a.color[8 * (size_t)p + 5],
                c6 = a.color[8 * (size_t)p + 6], c7 = a.color[8 * (size_t)p + 7];
    const float col[8] = {c0, c1, c2, c3, c4, c5, c6, c7};
    const float huberTH = a.huberTH;
    auto step_energy = [&](float sx, float sy) {
      float energy = 0;
#pragma unroll
      for (int idx = 0; idx < 8; idx++) {
        const float hitColor = interp31(a.img, (float)(sx + rx[idx]), (float)(sy + ry[idx]), W, H);
        if (!isfinite(hitColor)) {
          energy += 1e5f;
          continue;
        }
        const float residual = hitColor - (float)(hh.aff[0] * col[idx] + hh.aff[1]);
        const float hw = fabsf(residual) < huberTH ? 1 : huberTH / fabsf(residual);
        energy += hw * residual * residual * (2 - hw);
      }
      return energy;
    };
    const bool act0 = lane < numSteps, act1 = lane + 64 < numSteps;
    const float e0 = act0 ? step_energy(x0, y0) : __builtin_inff();
    const float e1 = act1 ? step_energy(x1, y1) : __builtin_inff();

    // best = first index of the minimum energy below 1e10 (:220-225)
    float be = fminf(e0, e1);
    be = wave_min(be);
    int bestIdx = -1;
    float bestEnergy = 1e10f, bestU = 0, bestV = 0;
    if (be < 1e10f) {
      const unsigned long long m0 = __ballot(act0 && e0 == be);
      const unsigned long long m1 = __ballot(act1 && e1 == be);
      bestIdx = m0 ? __builtin_ctzll(m0) : 64 + __builtin_ctzll(m1);
      const int src = bestIdx & 63;
      const float bx0 = __shfl(x0, src), by0 = __shfl(y0, src), bx1 = __shfl(x1, src), by1 = __shfl(y1, src);
      bestU = bestIdx < 64 ? bx0 : bx1;
      bestV = bestIdx < 64 ? by0 : by1;
      bestEnergy = be;
    }
    // second best outside +-radius (:236-244)
    const int rad = a.minTraceTestRadius;
    const int i0 = lane, i1 = lane + 64;
    const float s0 = (act0 && (i0 < bestIdx - rad || i0 > bestIdx + rad) && e0 < 1e10f) ? e0 : 1e10f;
    const float s1 = (act1 && (i1 < bestIdx - rad || i1 > bestIdx + rad) && e1 < 1e10f) ? e1 : 1e10f;
    const float secondBest = wave_min(fminf(s0, s1));
    const float newQuality = secondBest / bestEnergy;
    if (newQuality < quality || numSteps > 10) quality = newQuality;

    // GN along the line (:247-305): pattern pixel idx on lane idx
    const int li = lane & 7;
    const float wl = a.weights[8 * (size_t)p + li];
    float myCol = c0;
    myCol = li == 1 ? c1 : myCol;
    myCol = li == 2 ? c2 : myCol;
    myCol = li == 3 ? c3 : myCol;
    myCol = li == 4 ? c4 : myCol;
    myCol = li == 5 ? c5 : myCol;
    myCol = li == 6 ? c6 : myCol;
    myCol = li == 7 ? c7 : myCol;
    float myRx = rx[0], myRy = ry[0];
#pragma unroll
    for (int k = 1; k < 8; k++) {
      myRx = li == k ? rx[k] : myRx;
      myRy = li == k ? ry[k] : myRy;
    }
    float uBak = bestU, vBak = bestV, gnstepsize = 1, stepBack = 0;
    if (a.GNIterations > 0) bestEnergy = 1e5f;
    for (int it = 0; it < a.GNIterations; it++) {
      const float3 hc = interp33(a.img, (float)(bestU + myRx), (float)(bestV + myRy), W, H);
      const int fin = isfinite(hc.x) ? 1 : 0;
      const float residual = hc.x - (hh.aff[0] * myCol + hh.aff[1]);
      const float dResdDist = dx * hc.y + dy * hc.z;
      const float hw = fabsf(residual) < huberTH ? 1 : huberTH / fabsf(residual);
      const float tH = hw * dResdDist * dResdDist;
      const float tb = hw * residual * dResdDist;
      const float tE = wl * wl * hw * residual * residual * (2 - hw);
      float Hs = 1, bs = 0, energy = 0;
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const int fk = __shfl(fin, k);
        const float hk = __shfl(tH, k), bk = __shfl(tb, k), ek = __shfl(tE, k);
        if (!fk) {
          energy += 1e5f;
          continue;
        }
        Hs += hk;
        bs += bk;
        energy += ek;
      }
      if (energy > bestEnergy) {
        stepBack *= 0.5f;
        bestU = uBak + stepBack * dx;
        bestV = vBak + stepBack * dy;
      } else {
        float step = -gnstepsize * bs / Hs;
        if (step < -0.5f) step = -0.5f;
        else if (step > 0.5f) step = 0.5f;
        if (!isfinite(step)) step = 0;
        uBak = bestU;
        vBak = bestV;
        stepBack = step;
        bestU += step * dx;
        bestV += step * dy;
        bestEnergy = energy;
      }
      if (fabsf(stepBack) < a.GNThreshold) break;
    }

    // energy-based outlier (:309-321)
    if (!(bestEnergy < energyTH * a.extraSlackOnTH)) {
      outS = st == HS_IPS_OUTLIER ? HS_IPS_OOB : HS_IPS_OUTLIER;
      break;
    }
    // new interval (:325-349)
    float nmin, nmax;
    if (dx * dx > dy * dy) {
      nmin = (pr[2] * (bestU - errorInPixel * dx) - pr[0]) / (hh.Kt[0] - hh.Kt[2] * (bestU - errorInPixel * dx));
      nmax = (pr[2] * (bestU + errorInPixel * dx) - pr[0]) / (hh.Kt[0] - hh.Kt[2] * (bestU + errorInPixel * dx));
    } else {
      nmin = (pr[2] * (bestV - errorInPixel * dy) - pr[1]) / (hh.Kt[1] - hh.Kt[2] * (bestV - errorInPixel * dy));
      nmax = (pr[2] * (bestV + errorInPixel * dy) - pr[1]) / (hh.Kt[1] - hh.Kt[2] * (bestV + errorInPixel * dy));
    }
    if (nmin > nmax) {
      const float t = nmin;
      nmin = nmax;
      nmax = t;
    }
    idepth_min = nmin;
    idepth_max = nmax;
    write_interval = true;
    if (!isfinite(nmin) || !isfinite(nmax) || (nmax < 0)) {
      outS = HS_IPS_OUTLIER;
      break;
    }
    outI = 2 * errorInPixel;
    outU = bestU;
    outV = bestV;
    outS = HS_IPS_GOOD;
  } while (false);

  if (lane == 0) {
    a.steps[p] = searched;
    a.status[p] = (uint8_t)outS;
    a.uv[2 * p] = outU;
    a.uv[2 * p + 1] = outV;
    a.interval[p] = outI;
    a.quality[p] = quality;
    if (write_interval) {
      a.idepth_min[p] = idepth_min;
      a.idepth_max[p] = idepth_max;
    }
  }
}

// tallies of Src/Mapping.cpp:513-520 + the number of discrete-search steps evaluated (one workgroup;
// integer sums, order-free).  out[0..5] = counts per status, out[6..7] = steps as a 64-bit integer.
__global__ __launch_bounds__(1024) void hs_k_trace_count(int n, const uint8_t* __restrict__ status,
                                                         const int* __restrict__ steps, int* out) {
  __shared__ int c[6];
  __shared__ unsigned long long sc;
  if (threadIdx.x < 6) c[threadIdx.x] = 0;
  if (threadIdx.x == 0) sc = 0;
  __syncthreads();
  int l[6] = {0, 0, 0, 0, 0, 0};
  unsigned long long ls = 0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int s = status[i];
#pragma unroll
    for (int k = 0; k < 6; k++) l[k] += s == k;
    ls += (unsigned)steps[i];
  }
#pragma unroll
  for (int k = 0; k < 6; k++) {
    int x = l[k];
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    if ((threadIdx.x & 63) == 0) atomicAdd(&c[k], x);
  }
  for (int o = 32; o > 0; o >>= 1) ls += __shfl_xor(ls, o);
  if ((threadIdx.x & 63) == 0) atomicAdd(&sc, ls);
  __syncthreads();
  if (threadIdx.x < 6) out[threadIdx.x] = c[threadIdx.x];
  if (threadIdx.x == 0) *reinterpret_cast<unsigned long long*>(out + 6) = sc;
}
