// hs_ba_kernels.hip — gfx950 kernels of the windowed photometric BA hot path.
//
//   hs_k_linearize : PointFrameResidual::linearize + applyRes/takeData
//                    (Src/OptimizationClasses.cpp:43-256) fused with
//                    AccumulatedTopHessianSSE::addPoint<0> (Src/AccumulatedTopHessian.cpp:21-141)
//                    and AccumulatedSCHessianSSE::addPoint (Src/AccumulatedSCHessian.cpp:10-53).
//                    One wave64 per chunk of points of one host frame; lane = (target slot, pattern pixel).
//                    All accumulators live in VGPRs for the whole chunk; one partial slab per wave.
//   hs_k_reduce    : fixed-order sum of the wave partials per host (fp64) -> deterministic.
//   hs_k_stitch    : stitchDoubleInternal (top: Src/AccumulatedTopHessian.cpp:218-280,
//                    Schur: Src/AccumulatedSCHessian.cpp:54-133) in fp64, one workgroup per (host,target).
//   hs_k_resub     : EnergyFunctional::resubstituteFPt (Src/EnergyFunctional.cpp:249-274) fused with the
//                    point half of System::doStepFromBackup (Src/FullSystemOptimize.cpp:223-231).
//   hs_k_energy_th : System::setNewFrameEnergyTH (Src/FullSystemOptimize.cpp:60-101), exact k-th element
//                    by 4-pass radix select (nth_element's value is order independent).
//
// Per-residual arithmetic follows the reference operation order with fp contraction off, so
// categorical outputs (IN/OOB/OUT, energies, J) are bit-identical to the oracle.
#pragma clang fp contract(off)
#include <hip/hip_runtime.h>

#include "hs_kernels.h"

namespace {

__constant__ int c_pattern[8][2] = {{0, -2}, {-1, -1}, {1, -1}, {-2, 0}, {0, 0}, {2, 0}, {-1, 1}, {0, 2}};

constexpr float SCALE_F = 50.0f, SCALE_C = 50.0f, SCALE_IDEPTH = 1.0f;
constexpr int Q_N = 17;  // per-pixel quantities summed over the pattern (see k_linearize)

// getInterpolatedElement33 (Include/GlobalTypes.h:377-388) on float4 texels
__device__ __forceinline__ float3 interp33(const float4* __restrict__ img, float x, float y, int w) {
  int ix = (int)x, iy = (int)y;
  float dx = x - ix, dy = y - iy, dxdy = dx * dy;
  const float4* bp = img + ix + iy * w;
  const float4 p00 = bp[0], p10 = bp[1], p01 = bp[w], p11 = bp[w + 1];
  const float w11 = dxdy, w01 = dy - dxdy, w10 = dx - dxdy, w00 = 1 - dx - dy + dxdy;
  float3 r;
  r.x = w11 * p11.x + w01 * p01.x + w10 * p10.x + w00 * p00.x;
  r.y = w11 * p11.y + w01 * p01.y + w10 * p10.y + w00 * p00.y;
  r.z = w11 * p11.z + w01 * p01.z + w10 * p10.z + w00 * p00.z;
  return r;
}

// per-slot data exchanged through LDS (one slot = one residual = one target frame)
struct SlotData {
  float x[10], y[10];   // [Jpdc0(4) Jpdxi0(6)], [Jpdc1 Jpdxi1]
  float Jpdd[2];
  float JIdx2[3];       // 00, 01(=10), 11
  float Jab2[3];        // 00, 01, 11
  float JabJIdx[4];     // 00, 01, 10, 11
  float JIr[2], Jabr[2], rr;
  float JpJdF[8];
  float econ;           // contribution of this residual to linearizeAll's energy
  float active;         // isActiveAndIsGoodNEW after applyRes
  float pad[2];
};

struct WaveLds {
  float q[HS_MAXF][Q_N][8];
  float s[HS_MAXF][Q_N + 3];
  SlotData sd[HS_MAXF];
};

}  // namespace

__global__ __launch_bounds__(64) void hs_k_linearize(HsLinArgs a) {
  __shared__ WaveLds L;
  const int lane = threadIdx.x;
  const int t = lane >> 3;  // target slot
  const int k = lane & 7;   // pattern pixel
  const int chunk = blockIdx.x;
  const int pb = a.chunk_begin[chunk];
  const int pe = a.chunk_begin[chunk + 1];
  const int h = a.chunk_host[chunk];
  const int nF = a.nF;
  const HsCalib cal = a.calib;
  const float thH = a.frameTH[h];

  // ---- accumulator-lane roles (constant per lane)
  // top entry e0 = lane, e1 = 64 + lane (< 91)
  int er0 = 0, ec0 = 0, er1 = 0, ec1 = 0;
  {
    int e = lane, idx = 0;
    for (int r = 0; r < 10; r++)
      for (int c = r; c < 10; c++) {
        if (idx == e) { er0 = r; ec0 = c; }
        idx++;
      }
    if (e >= 55) { er0 = (e - 55) / 3; ec0 = (e - 55) % 3; }
    int e1 = 64 + lane;
    er1 = (e1 - 55) / 3; ec1 = (e1 - 55) % 3;
    if (e1 >= 85) { er1 = 0; ec1 = e1 - 85; }
  }
  float accTop0[HS_MAXF], accTop1[HS_MAXF], accD[HS_MAXF][HS_MAXF], accX[HS_MAXF];
  float accH = 0.f;
#pragma unroll
  for (int i = 0; i < HS_MAXF; i++) {
    accTop0[i] = 0.f; accTop1[i] = 0.f; accX[i] = 0.f;
#pragma unroll
    for (int j = 0; j < HS_MAXF; j++) accD[i][j] = 0.f;
  }
  int cnt = 0;           // lane < 8: residuals accumulated into top block (h, lane)
  double eSum = 0.0;     // lane 0

  const float4* __restrict__ imgT = (t < nF) ? a.img[t] : nullptr;
  const float thT = (t < nF) ? a.frameTH[t] : 0.f;
  const float thr = fmaxf(thH, thT);  // std::max<float>(host TH, target TH)

  for (int p = pb; p < pe; p++) {
    const float pu = a.u[p], pv = a.v[p];
    const float idep = a.idepth[p], idep0 = a.idepth_zero[p];
    const int r = a.res_of_slot[p * 8 + t];
    const bool has = r >= 0;
    int st = has ? (int)a.r_state[r] : HS_RES_OOB;

    // ---------------- linearize (one residual per slot, one pattern pixel per lane)
    bool oob = false;
    float Jx[10] = {0}, Jy[10] = {0}, Jd0 = 0.f, Jd1 = 0.f;
    float qv[Q_N];
#pragma unroll
    for (int qi = 0; qi < Q_N; qi++) qv[qi] = 0.f;
    float centre[3] = {0.f, 0.f, 0.f};
    bool centreOk = false;
    if (has && st != HS_RES_OOB) {
      const HsPrecalc& pc = a.pre[h * nF + t];
      // centre: projectPoint(u, v, idepth_zero, 0, 0, R_0, t_0)  Include/DirectProjection.h:20-38
      const float Kl0 = (pu + 0 - cal.cxl) * cal.fxli;
      const float Kl1 = (pv + 0 - cal.cyl) * cal.fyli;
      float pt0 = pc.R0[0] * Kl0 + pc.R0[1] * Kl1 + pc.R0[2] * 1.f;
      float pt1 = pc.R0[3] * Kl0 + pc.R0[4] * Kl1 + pc.R0[5] * 1.f;
      float pt2 = pc.R0[6] * Kl0 + pc.R0[7] * Kl1 + pc.R0[8] * 1.f;
      pt0 = pt0 + pc.t0[0] * idep0;
      pt1 = pt1 + pc.t0[1] * idep0;
      pt2 = pt2 + pc.t0[2] * idep0;
      const float drescale = 1.0f / pt2;
      const float new_idepth = idep0 * drescale;
      if (!(drescale > 0)) {
        oob = true;
      } else {
        const float u = pt0 * drescale, v = pt1 * drescale;
        const float Ku = u * cal.fxl + cal.cxl, Kv = v * cal.fyl + cal.cyl;
        if (!(Ku > 1.1f && Kv > 1.1f && Ku < (cal.W - 3) && Kv < (cal.H - 3))) {
          oob = true;
        } else {
          centreOk = true;
          centre[0] = Ku; centre[1] = Kv; centre[2] = new_idepth;
          const float* R0 = pc.R0;
          const float* t0 = pc.t0;
          Jd0 = drescale * (t0[0] - t0[2] * u) * SCALE_IDEPTH * cal.fxl;
          Jd1 = drescale * (t0[1] - t0[2] * v) * SCALE_IDEPTH * cal.fyl;
          float cx[4], cy[4];
          cx[2] = drescale * (R0[6] * u - R0[0]);
          cx[3] = cal.fxl * drescale * (R0[7] * u - R0[1]) * cal.fyli;
          cx[0] = Kl0 * cx[2];
          cx[1] = Kl1 * cx[3];
          cy[2] = cal.fyl * drescale * (R0[6] * v - R0[3]) * cal.fxli;
          cy[3] = drescale * (R0[7] * v - R0[4]);
          cy[0] = Kl0 * cy[2];
          cy[1] = Kl1 * cy[3];
          cx[0] = (cx[0] + u) * SCALE_F;
          cx[1] *= SCALE_F;
          cx[2] = (cx[2] + 1) * SCALE_C;
          cx[3] *= SCALE_C;
          cy[0] *= SCALE_F;
          cy[1] = (cy[1] + v) * SCALE_F;
          cy[2] *= SCALE_C;
          cy[3] = (cy[3] + 1) * SCALE_C;
          const float fx = cal.fxl, fy = cal.fyl;
          Jx[0] = cx[0]; Jx[1] = cx[1]; Jx[2] = cx[2]; Jx[3] = cx[3];
          Jy[0] = cy[0]; Jy[1] = cy[1]; Jy[2] = cy[2]; Jy[3] = cy[3];
          Jx[4] = new_idepth * fx;
          Jx[5] = 0;
          Jx[6] = -new_idepth * u * fx;
          Jx[7] = -u * v * fx;
          Jx[8] = (1 + u * u) * fx;
          Jx[9] = -v * fx;
          Jy[4] = 0;
          Jy[5] = new_idepth * fy;
          Jy[6] = -new_idepth * v * fy;
          Jy[7] = -(1 + v * v) * fy;
          Jy[8] = u * v * fy;
          Jy[9] = u * fy;

          // pattern pixel k
          const float px = pu + c_pattern[k][0], py = pv + c_pattern[k][1];
          float q0 = pc.KRKi[0] * px + pc.KRKi[1] * py + pc.KRKi[2] * 1.f;
          float q1 = pc.KRKi[3] * px + pc.KRKi[4] * py + pc.KRKi[5] * 1.f;
          float q2 = pc.KRKi[6] * px + pc.KRKi[7] * py + pc.KRKi[8] * 1.f;
          q0 = q0 + pc.Kt[0] * idep;
          q1 = q1 + pc.Kt[1] * idep;
          q2 = q2 + pc.Kt[2] * idep;
          const float PKu = q0 / q2, PKv = q1 / q2;
          if (!(PKu > 1.1f && PKv > 1.1f && PKu < (cal.W - 3) && PKv < (cal.H - 3))) {
            oob = true;
          } else {
            float3 hit = interp33(imgT, PKu, PKv, cal.W);
            const float color = a.color[p * 8 + k];
            const float residual = hit.x - (float)(pc.aff[0] * color + pc.aff[1]);
            const float drdA = (color - pc.b0);
            if (!isfinite(hit.x)) {
              oob = true;
            } else {
              float w = sqrtf(a.lp.outlierTHSumComponent /
                              (a.lp.outlierTHSumComponent + (hit.y * hit.y + hit.z * hit.z)));
              w = 0.5f * (w + a.weight[p * 8 + k]);
              float hw = fabsf(residual) < a.lp.huberTH ? 1 : a.lp.huberTH / fabsf(residual);
              qv[0] = w * w * hw * residual * residual * (2 - hw);
              if (hw < 1) hw = sqrtf(hw);
              hw = hw * w;
              const float hy = hit.y * hw, hz = hit.z * hw;
              const float resF = residual * hw;
              float jab0 = drdA * hw;
              float jab1 = hw;
              qv[1] = hy * hy;
              qv[2] = hz * hz;
              qv[3] = hy * hz;
              qv[4] = drdA * hw * hy;
              qv[5] = drdA * hw * hz;
              qv[6] = hw * hy;
              qv[7] = hw * hz;
              qv[8] = drdA * drdA * hw * hw;
              qv[9] = drdA * hw * hw;
              qv[10] = hw * hw;
              qv[11] = hw * hw * (hy * hy + hz * hz);
              if (a.lp.affineOptModeA < 0) jab0 = 0;
              if (a.lp.affineOptModeB < 0) jab1 = 0;
              // AccumulatedTopHessianSSE::addPoint<0>: JI_r, Jab_r, rr over resApprox = resF
              qv[12] = resF * hy;
              qv[13] = resF * hz;
              qv[14] = resF * jab0;
              qv[15] = resF * jab1;
              qv[16] = resF * resF;
            }
          }
        }
      }
    }
    const unsigned long long oobMask = __ballot(oob);
    const bool slotOob = ((oobMask >> (t * 8)) & 0xffull) != 0ull;

#pragma unroll
    for (int qi = 0; qi < Q_N; qi++) L.q[t][qi][k] = qv[qi];
    __syncthreads();
    // sequential (pattern-order) sums, exactly as the reference's running sums
    for (int qi = k; qi < Q_N; qi += 8) {
      float s = 0.f;
#pragma unroll
      for (int kk = 0; kk < 8; kk++) s += L.q[t][qi][kk];
      L.s[t][qi] = s;
    }
    __syncthreads();

    // ---------------- state decision + applyRes (lanes of a slot agree; lane k==0 writes)
    float JpJdF_k = 0.f;
    bool active = false;
    float econ = 0.f;
    if (has) {
      const float oldE = a.r_energy[r];
      if (st == HS_RES_OOB) {
        econ = oldE;  // linearize returns state_energy; applyRes returns early (sticky OOB)
        active = false;
        if (k == 0) a.r_ewo[r] = -1.f;
      } else if (slotOob) {
        econ = oldE;  // state_energy; NewEnergy unchanged
        if (k == 0) {
          a.r_ewo[r] = -1.f;
          a.r_state[r] = HS_RES_OOB;
          a.r_active[r] = 0;
          a.r_energy[r] = a.r_newEnergy[r];
        }
        active = false;
      } else {
        float energyLeft = L.s[t][0];
        const float wJI2 = L.s[t][11];
        int ns;
        if (k == 0) a.r_ewo[r] = energyLeft;
        if (energyLeft > thr || wJI2 < 2) {
          energyLeft = thr;
          ns = HS_RES_OUT;
        } else {
          ns = HS_RES_IN;
        }
        econ = energyLeft;
        active = ns == HS_RES_IN;
        if (active) {
          // takeData (Include/OptimizationClasses.h:195-201)
          const float J00 = L.s[t][1], J11 = L.s[t][2], J10 = L.s[t][3];
          const float aa = J00 * Jd0 + J10 * Jd1;
          const float bb = J10 * Jd0 + J11 * Jd1;
          if (k < 6) JpJdF_k = Jx[4 + k] * aa + Jy[4 + k] * bb;
          else if (k == 6) JpJdF_k = L.s[t][4] * Jd0 + L.s[t][5] * Jd1;
          else JpJdF_k = L.s[t][6] * Jd0 + L.s[t][7] * Jd1;
          a.r_JpJdF[r * 8 + k] = JpJdF_k;
        }
        if (k == 0) {
          a.r_state[r] = (uint8_t)ns;
          a.r_active[r] = active ? 1 : 0;
          a.r_energy[r] = energyLeft;
          a.r_newEnergy[r] = energyLeft;
        }
        if (ns == HS_RES_IN || ns == HS_RES_OUT) {
          if (a.newest_cand != nullptr && t == nF - 1 && k == 0) {
            const int slot = atomicAdd(a.newest_cnt, 1);
            a.newest_cand[slot] = L.s[t][0];
          }
        }
      }
      if (a.write_center && centreOk && k < 3) a.r_center[r * 3 + k] = centre[k];
    }
    // publish slot data for the accumulation lanes
    if (k == 0) {
      SlotData& sd = L.sd[t];
#pragma unroll
      for (int i = 0; i < 10; i++) { sd.x[i] = Jx[i]; sd.y[i] = Jy[i]; }
      sd.Jpdd[0] = Jd0; sd.Jpdd[1] = Jd1;
      sd.JIdx2[0] = L.s[t][1]; sd.JIdx2[1] = L.s[t][3]; sd.JIdx2[2] = L.s[t][2];
      sd.JabJIdx[0] = L.s[t][4]; sd.JabJIdx[1] = L.s[t][5]; sd.JabJIdx[2] = L.s[t][6]; sd.JabJIdx[3] = L.s[t][7];
      sd.Jab2[0] = L.s[t][8]; sd.Jab2[1] = L.s[t][9]; sd.Jab2[2] = L.s[t][10];
      sd.JIr[0] = L.s[t][12]; sd.JIr[1] = L.s[t][13];
      sd.Jabr[0] = L.s[t][14]; sd.Jabr[1] = L.s[t][15];
      sd.rr = L.s[t][16];
      sd.econ = econ;
      sd.active = active ? 1.f : 0.f;
    }
    L.sd[t].JpJdF[k] = JpJdF_k;
    __syncthreads();

    // ---------------- AccumulatedTopHessianSSE::addPoint<0> : block (h, tt) entries e0/e1 of this lane
#pragma unroll
    for (int tt = 0; tt < HS_MAXF; tt++) {
      const SlotData& sd = L.sd[tt];
      if (sd.active != 0.f) {
        // e0
        if (lane < 55) {
          const float xr = sd.x[er0], xc = sd.x[ec0], yr = sd.y[er0], yc = sd.y[ec0];
          accTop0[tt] += sd.JIdx2[0] * xc * xr + sd.JIdx2[2] * yc * yr + sd.JIdx2[1] * (xc * yr + yc * xr);
        } else {
          const float xr = sd.x[er0], yr = sd.y[er0];
          const float T0 = ec0 == 0 ? sd.JabJIdx[0] : (ec0 == 1 ? sd.JabJIdx[2] : sd.JIr[0]);
          const float T1 = ec0 == 0 ? sd.JabJIdx[1] : (ec0 == 1 ? sd.JabJIdx[3] : sd.JIr[1]);
          accTop0[tt] += xr * T0 + yr * T1;
        }
        // e1
        if (lane < 21) {
          const float xr = sd.x[er1], yr = sd.y[er1];
          const float T0 = ec1 == 0 ? sd.JabJIdx[0] : (ec1 == 1 ? sd.JabJIdx[2] : sd.JIr[0]);
          const float T1 = ec1 == 0 ? sd.JabJIdx[1] : (ec1 == 1 ? sd.JabJIdx[3] : sd.JIr[1]);
          accTop1[tt] += xr * T0 + yr * T1;
        } else if (lane < 27) {
          const int b = lane - 21;
          const float v = b == 0 ? sd.Jab2[0]
                        : b == 1 ? sd.Jab2[1]
                        : b == 2 ? sd.Jabr[0]
                        : b == 3 ? sd.Jab2[2]
                        : b == 4 ? sd.Jabr[1] : sd.rr;
          accTop1[tt] += v;
        }
        if (lane == tt) cnt++;
      }
    }

    // ---------------- per-point sums (residual-list order) + energy
    float Hdd = 0.f, bd = 0.f, Hcd[4] = {0.f, 0.f, 0.f, 0.f};
    int ngood = 0;
    for (int qn = 0; qn < 8; qn++) {
      const int tt = a.res_order[p * 8 + qn];
      if (tt < 0) break;
      const SlotData& sd = L.sd[tt];
      if (lane == 0) eSum += (double)sd.econ;
      if (sd.active == 0.f) continue;
      ngood++;
      const float aa = sd.JIdx2[0] * sd.Jpdd[0] + sd.JIdx2[1] * sd.Jpdd[1];
      const float bb = sd.JIdx2[1] * sd.Jpdd[0] + sd.JIdx2[2] * sd.Jpdd[1];
      bd += sd.JIr[0] * sd.Jpdd[0] + sd.JIr[1] * sd.Jpdd[1];
      Hdd += aa * sd.Jpdd[0] + bb * sd.Jpdd[1];
#pragma unroll
      for (int c = 0; c < 4; c++) Hcd[c] += sd.x[c] * aa + sd.y[c] * bb;
    }

    // ---------------- AccumulatedSCHessianSSE::addPoint(p, shiftPriorToZero=true)
    if (ngood == 0) {
      if (lane == 0) { a.p_HdiF[p] = 0.f; a.p_bdSumF[p] = 0.f; a.p_ngood[p] = 0; }
    } else {
      const float priorF = a.priorF[p];
      float Hh = Hdd + 0.f + priorF;
      if (Hh < 1e-10f) Hh = 1e-10f;
      const float HdiF = 1.0f / Hh;
      float bdSumF = bd + 0.f;
      bdSumF += priorF * (idep - idep0);
      if (lane == 0) { a.p_HdiF[p] = HdiF; a.p_bdSumF[p] = bdSumF; a.p_ngood[p] = (uint8_t)ngood; }
      if (lane < 4) a.p_Hcd[p * 4 + lane] = Hcd[lane];
      // accD: lane = (i, j)
      {
        const int i = lane >> 3, j = lane & 7;
        float Ji[HS_MAXF], Jj[HS_MAXF], act[HS_MAXF];
#pragma unroll
        for (int tt = 0; tt < HS_MAXF; tt++) {
          Ji[tt] = L.sd[tt].JpJdF[i];
          Jj[tt] = L.sd[tt].JpJdF[j];
          act[tt] = L.sd[tt].active;
        }
#pragma unroll
        for (int t1 = 0; t1 < HS_MAXF; t1++) {
          if (act[t1] == 0.f) continue;
          const float wl = HdiF * Ji[t1];
#pragma unroll
          for (int t2 = 0; t2 < HS_MAXF; t2++)
            if (act[t2] != 0.f) accD[t1][t2] += wl * Jj[t2];
        }
      }
      // accE (lanes 0..31), accEB (32..39), accHcc (40..55), accbc (56..59)
      {
        const float HcdSel0 = lane < 32 ? Hcd[lane & 3] : 0.f;
        float hr = 0.f, hc = 0.f;
        if (lane >= 40 && lane < 56) {
          const int m = lane - 40;
          hr = Hcd[m >> 2];
          hc = Hcd[m & 3];
          accH += HdiF * hr * hc;
        } else if (lane >= 56 && lane < 60) {
          accH += bdSumF * HdiF * Hcd[lane - 56];
        }
#pragma unroll
        for (int t1 = 0; t1 < HS_MAXF; t1++) {
          if (L.sd[t1].active == 0.f) continue;
          if (lane < 32) {
            accX[t1] += HdiF * L.sd[t1].JpJdF[lane >> 2] * HcdSel0;
          } else if (lane < 40) {
            accX[t1] += HdiF * bdSumF * L.sd[t1].JpJdF[lane - 32];
          }
        }
      }
    }
    __syncthreads();  // LDS is rewritten by the next point
  }

  // ---------------- write this wave's partial slab
  HsWavePartial* P = a.partials + chunk;
#pragma unroll
  for (int tt = 0; tt < HS_MAXF; tt++) {
    P->top[tt][lane] = accTop0[tt];
    if (lane < 27) P->top[tt][64 + lane] = accTop1[tt];
#pragma unroll
    for (int t2 = 0; t2 < HS_MAXF; t2++) P->D[tt][t2][lane] = accD[tt][t2];
    if (lane < 32) P->E[tt][lane] = accX[tt];
    else if (lane < 40) P->EB[tt][lane - 32] = accX[tt];
  }
  if (lane >= 40 && lane < 56) P->Hcc[lane - 40] = accH;
  if (lane >= 56 && lane < 60) P->bc[lane - 56] = accH;
  if (lane < HS_MAXF) P->cnt[lane] = cnt;
  if (lane == 0) { P->host = h; P->energy = eSum; }
}

// fixed-order reduction of wave partials into per-host fp64 slabs
__global__ void hs_k_reduce(HsReduceArgs a) {
  const int h = blockIdx.y;
  const int cb = a.host_chunk_begin[h], ce = a.host_chunk_begin[h + 1];
  HsHostSlab* S = a.slabs + h;
  const int NF = HS_WP_FLOATS;
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < NF + HS_MAXF; q += gridDim.x * blockDim.x) {
    if (q < NF) {
      double s = 0.0;
      for (int c = cb; c < ce; c++) s += (double)((const float*)(a.partials + c))[q];
      ((double*)S)[q] = s;
    } else {
      const int tt = q - NF;
      int s = 0;
      for (int c = cb; c < ce; c++) s += a.partials[c].cnt[tt];
      S->cnt[tt] = s;
    }
  }
  if (h == 0 && blockIdx.x == 0 && threadIdx.x == 0) {
    double e = 0.0;
    for (int c = 0; c < a.n_chunks; c++) e += a.partials[c].energy;
    *a.energy = e;
  }
}

namespace {
// out(8x8) = A(8x8) * M(8x8) * B(8x8)^T, 64 threads (r = tid>>3, c = tid&7), tmp in LDS
__device__ __forceinline__ double sandwich(const double* A, const double* M, const double* B, double* tmp, int tid) {
  const int r = tid >> 3, c = tid & 7;
  double s = 0.0;
  for (int l = 0; l < 8; l++) s += A[r * 8 + l] * M[l * 8 + c];
  __syncthreads();
  tmp[tid] = s;
  __syncthreads();
  double o = 0.0;
  for (int l = 0; l < 8; l++) o += tmp[r * 8 + l] * B[c * 8 + l];
  return o;
}
}  // namespace

// one block (64 threads) per (i = host, j = target) pair: top block aidx = i + nF*j and Schur rows (i, j, *)
__global__ __launch_bounds__(64) void hs_k_stitch(HsStitchArgs a) {
  const int nF = a.nF;
  const int i = blockIdx.x % nF, j = blockIdx.x / nF;
  const int tid = threadIdx.x;
  const int n = 4 + 8 * nF;
  const int iIdx = 4 + 8 * i, jIdx = 4 + 8 * j;
  const int ij = i + nF * j;
  const HsHostSlab* S = a.slabs + i;
  __shared__ double A88[64], A84[32], a8r[8], tmp[64], aH[64], aT[64], D[64], aH2[64], aT2[64], v8[8];
  __shared__ double Hpc[32];
  aH[tid] = a.adHost[ij * 64 + tid];
  aT[tid] = a.adTarget[ij * 64 + tid];
  // ---- top block (finish(): 13x13 from Data/TopRight/BotRight, AccumulatorApprox::finish)
  const bool haveTop = S->cnt[j] > 0;
  if (haveTop) {
    const double* e = S->top[j];
    // 13x13 symmetric from the 91 entries
    {
      const int r = tid >> 3, c = tid & 7;  // A88 = H[4+r][4+c]
      const int R = 4 + r, Cc = 4 + c;
      double v;
      if (R < 10 && Cc < 10) {
        const int rr = R < Cc ? R : Cc, cc = R < Cc ? Cc : R;
        const int idx = rr * 10 - (rr * (rr - 1)) / 2 + (cc - rr);
        v = e[idx];
      } else if (R < 10 || Cc < 10) {
        const int row = R < 10 ? R : Cc, col = (R < 10 ? Cc : R) - 10;
        v = e[55 + 3 * row + col];
      } else {
        const int rr = R - 10 < Cc - 10 ? R - 10 : Cc - 10, cc = R - 10 < Cc - 10 ? Cc - 10 : R - 10;
        const int map[3][3] = {{0, 1, 2}, {1, 3, 4}, {2, 4, 5}};
        v = e[85 + map[rr][cc]];
      }
      A88[tid] = v;
    }
    if (tid < 32) {  // A84 = H[4+r][c], r<8, c<4
      const int r = tid >> 2, c = tid & 3;
      const int R = 4 + r;
      double v;
      if (R < 10) {
        const int idx = c * 10 - (c * (c - 1)) / 2 + (R - c);
        v = e[idx];
      } else {
        v = e[55 + 3 * c + (R - 10)];
      }
      A84[tid] = v;
    }
    if (tid < 8) {  // a8r = H[4+r][12]
      const int R = 4 + tid;
      a8r[tid] = R < 10 ? e[55 + 3 * R + 2] : (R == 10 ? e[85 + 2] : e[85 + 4]);
    }
  }
  __syncthreads();
  const int r = tid >> 3, c = tid & 7;
  if (haveTop) {
    double o;
    o = sandwich(aH, A88, aH, tmp, tid);
    atomicAdd(&a.HA[(iIdx + r) * n + iIdx + c], o);
    o = sandwich(aT, A88, aT, tmp, tid);
    atomicAdd(&a.HA[(jIdx + r) * n + jIdx + c], o);
    o = sandwich(aH, A88, aT, tmp, tid);
    atomicAdd(&a.HA[(iIdx + r) * n + jIdx + c], o);
    if (tid < 32) {
      const int rr = tid >> 2, cc = tid & 3;
      double s1 = 0.0, s2 = 0.0;
      for (int l = 0; l < 8; l++) { s1 += aH[rr * 8 + l] * A84[l * 4 + cc]; s2 += aT[rr * 8 + l] * A84[l * 4 + cc]; }
      atomicAdd(&a.HA[(iIdx + rr) * n + cc], s1);
      atomicAdd(&a.HA[(jIdx + rr) * n + cc], s2);
    }
    if (tid < 16) {
      const int rr = tid >> 2, cc = tid & 3;
      const int idx = (rr < cc ? rr : cc) * 10 - ((rr < cc ? rr : cc) * ((rr < cc ? rr : cc) - 1)) / 2 +
                      ((rr < cc ? cc : rr) - (rr < cc ? rr : cc));
      atomicAdd(&a.HA[rr * n + cc], S->top[j][idx]);
    }
    if (tid < 8) {
      double s1 = 0.0, s2 = 0.0;
      for (int l = 0; l < 8; l++) { s1 += aH[tid * 8 + l] * a8r[l]; s2 += aT[tid * 8 + l] * a8r[l]; }
      atomicAdd(&a.bA[iIdx + tid], s1);
      atomicAdd(&a.bA[jIdx + tid], s2);
    }
    if (tid < 4) atomicAdd(&a.bA[tid], S->top[j][55 + 3 * tid + 2]);
  }
  // ---- Schur complement rows (i, j, k)
  if (tid < 32) Hpc[tid] = S->E[j][tid];
  if (tid < 8) v8[tid] = S->EB[j][tid];
  __syncthreads();
  if (tid < 32) {
    const int rr = tid >> 2, cc = tid & 3;
    double s1 = 0.0, s2 = 0.0;
    for (int l = 0; l < 8; l++) { s1 += aH[rr * 8 + l] * Hpc[l * 4 + cc]; s2 += aT[rr * 8 + l] * Hpc[l * 4 + cc]; }
    atomicAdd(&a.HSC[(iIdx + rr) * n + cc], s1);
    atomicAdd(&a.HSC[(jIdx + rr) * n + cc], s2);
  }
  if (tid < 8) {
    double s1 = 0.0, s2 = 0.0;
    for (int l = 0; l < 8; l++) { s1 += aH[tid * 8 + l] * v8[l]; s2 += aT[tid * 8 + l] * v8[l]; }
    atomicAdd(&a.bSC[iIdx + tid], s1);
    atomicAdd(&a.bSC[jIdx + tid], s2);
  }
  for (int kk = 0; kk < nF; kk++) {
    const int kIdx = 4 + 8 * kk;
    const int ik = i + nF * kk;
    __syncthreads();
    D[tid] = S->D[j][kk][tid];
    aH2[tid] = a.adHost[ik * 64 + tid];
    aT2[tid] = a.adTarget[ik * 64 + tid];
    __syncthreads();
    double o;
    o = sandwich(aH, D, aH2, tmp, tid);
    atomicAdd(&a.HSC[(iIdx + r) * n + iIdx + c], o);
    o = sandwich(aT, D, aT2, tmp, tid);
    atomicAdd(&a.HSC[(jIdx + r) * n + kIdx + c], o);
    o = sandwich(aT, D, aH2, tmp, tid);
    atomicAdd(&a.HSC[(jIdx + r) * n + iIdx + c], o);
    o = sandwich(aH, D, aT2, tmp, tid);
    atomicAdd(&a.HSC[(iIdx + r) * n + kIdx + c], o);
  }
  if (blockIdx.x == 0 && tid < 16) {
    double s = 0.0;
    for (int hh = 0; hh < nF; hh++) s += a.slabs[hh].Hcc[tid];
    atomicAdd(&a.HSC[(tid >> 2) * n + (tid & 3)], s);
  }
  if (blockIdx.x == 0 && tid < 4) {
    double s = 0.0;
    for (int hh = 0; hh < nF; hh++) s += a.slabs[hh].bc[tid];
    atomicAdd(&a.bSC[tid], s);
  }
}

// resubstituteFPt + point part of doStepFromBackup: one thread per point
__global__ void hs_k_resub(HsResubArgs a) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  double sID = 0.0, sNID = 0.0;
  if (p < a.n) {
    const int h = a.host[p];
    const float idb = a.idepth[p];  // idepth_backup (backupState copies idepth)
    float step = 0.f;
    if (a.ngood[p] != 0) {
      float b = a.bdSumF[p];
      float dot = 0.f;
      for (int c = 0; c < 4; c++) dot += a.cstep[c] * a.Hcd[p * 4 + c];
      b -= dot;
      for (int q = 0; q < 8; q++) {
        const int tt = a.res_order[p * 8 + q];
        if (tt < 0) break;
        const int r = a.res_of_slot[p * 8 + tt];
        if (!a.r_active[r]) continue;
        const float* xa = a.xAd + (h * a.nF + tt) * 8;
        float d = 0.f;
        for (int i = 0; i < 8; i++) d += xa[i] * a.JpJdF[r * 8 + i];
        b -= d;
      }
      step = -b * a.HdiF[p];
    }
    a.step[p] = step;
    if (a.apply) {
      const float nid = idb + 1.0f * step;
      a.idepth[p] = nid;
      a.idepth_zero[p] = nid;
    }
    sID = (double)step * (double)step;
    sNID = fabs((double)idb);
  }
  // block reduction of the step statistics (deterministic: fixed tree)
  __shared__ double r1[256], r2[256];
  r1[threadIdx.x] = sID;
  r2[threadIdx.x] = sNID;
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) { r1[threadIdx.x] += r1[threadIdx.x + s]; r2[threadIdx.x] += r2[threadIdx.x + s]; }
    __syncthreads();
  }
  if (threadIdx.x == 0) { a.stat_partial[blockIdx.x * 2] = r1[0]; a.stat_partial[blockIdx.x * 2 + 1] = r2[0]; }
}

// point half of doStepFromBackup when the step was computed without applying it
__global__ void hs_k_apply_step(int n, const float* step, float* idepth, float* idepth_zero) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < n) {
    const float nid = idepth[p] + 1.0f * step[p];
    idepth[p] = nid;
    idepth_zero[p] = nid;
  }
}

// setNewFrameEnergyTH: k-th smallest of the candidate energies by 4-pass radix select, one block of 1024.
// Multi-GPU: candidates of all ranks were all-gathered (rank r at cand + r*stride, cnt[r] values), so every
// rank selects the same element as the single-GPU nth_element over the union.
__global__ __launch_bounds__(1024) void hs_k_energy_th(HsEnergyThArgs a) {
  __shared__ unsigned int hist[256];
  __shared__ unsigned int s_prefix, s_mask, s_k;
  const int tid = threadIdx.x;
  int n = 0;
  for (int r = 0; r < a.nranks; r++) n += a.cnt[r];
  if (n == 0) {
    if (tid == 0) a.frameTH[a.newest] = 12 * 12 * 8;
    return;
  }
  if (tid == 0) {
    s_prefix = 0;
    s_mask = 0;
    s_k = (unsigned int)(int)(a.frameEnergyTHN * (float)n);
  }
  for (int pass = 0; pass < 4; pass++) {
    const int shift = 24 - 8 * pass;
    if (tid < 256) hist[tid] = 0;
    __syncthreads();
    const unsigned int prefix = s_prefix, mask = s_mask;
    for (int r = 0; r < a.nranks; r++) {
      const float* cr = a.cand + (size_t)r * a.stride;
      const int nr = a.cnt[r];
      for (int i = tid; i < nr; i += blockDim.x) {
        const unsigned int v = __float_as_uint(cr[i]);
        if ((v & mask) == prefix) atomicAdd(&hist[(v >> shift) & 255u], 1u);
      }
    }
    __syncthreads();
    if (tid == 0) {
      unsigned int kk = s_k, cum = 0;
      int b = 0;
      for (; b < 256; b++) {
        if (cum + hist[b] > kk) break;
        cum += hist[b];
      }
      s_k = kk - cum;
      s_prefix = prefix | ((unsigned int)b << shift);
      s_mask = mask | (255u << shift);
    }
    __syncthreads();
  }
  if (tid == 0) {
    const float nth = sqrtf(__uint_as_float(s_prefix));
    float th = nth * a.facMedian;
    th = 26.0f * a.constWeight + th * (1 - a.constWeight);
    th = th * th;
    th *= a.overallWeight * a.overallWeight;
    a.frameTH[a.newest] = th;
  }
}
