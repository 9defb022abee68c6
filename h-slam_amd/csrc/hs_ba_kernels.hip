// hs_ba_kernels.hip — gfx950 kernels of the windowed photometric BA hot path.
//
// One GN iteration of System::optimize is a device-only sequence (no host round trip):
//   hs_k_solve      EnergyFunctional::solveSystemF (Src/EnergyFunctional.cpp:705-817) in fp64 on one
//                   workgroup: stitchDoubleMT post-processing (Include/AccumulatedTopHessian.h:104-116), priors
//                   (Src/AccumulatedTopHessian.cpp:269-279), Schur, scaled LDLT in the Eigen pivot order,
//                   orthogonalize (Src/EnergyFunctional.cpp:648-702), resubstituteF_MT frame part (:222-247);
//                   then backupState + System::doStepFromBackup frame/calib part + setPrecalcValues
//                   (Src/FullSystemOptimize.cpp:171-264).
//   hs_k_linearize  one wave64 per point: resubstituteFPt + point step of the previous solve
//                   (Src/EnergyFunctional.cpp:249-274), then PointFrameResidual::linearize + applyRes/takeData
//                   (Src/OptimizationClasses.cpp:43-256) of its <= 7 residuals (lane = target slot x pattern
//                   pixel) and the per-point sums of AccumulatedTopHessianSSE::addPoint<0>
//                   (Src/AccumulatedTopHessian.cpp:21-141) / AccumulatedSCHessianSSE::addPoint (:10-53).
//   hs_k_accumulate one workgroup per (host, target[, split]): the AccumulatorApprox / AccumulatorXX / X
//                   updates (Include/MatrixAccumulators.h) in the reference's point order with the 1k/1m
//                   blocking, so an unsplit block equals the single-thread reference bit for bit; plus the
//                   energy sum, setNewFrameEnergyTH (Src/FullSystemOptimize.cpp:60-101) and accHcc/accbc.
//   hs_k_stitch     stitchDoubleInternal (top: Src/AccumulatedTopHessian.cpp:218-280, Schur:
//                   Src/AccumulatedSCHessian.cpp:54-133) in fp64, one workgroup per (host, target).
// Per-residual arithmetic follows the reference operation order with fp contraction off.
#pragma clang fp contract(off)
#include <hip/hip_runtime.h>

#include <cfloat>

#include "hs_kernels.h"

namespace {

__constant__ int c_pattern[8][2] = {{0, -2}, {-1, -1}, {1, -1}, {-2, 0}, {0, 0}, {2, 0}, {-1, 1}, {0, 2}};

constexpr float SCALE_F = 50.0f, SCALE_C = 50.0f, SCALE_IDEPTH = 1.0f;
constexpr int Q_N = 17;  // per-pixel quantities summed over the pattern

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

// One entry of a blocked fp32 accumulator: A (current), A1k, A1m (MatrixAccumulators.h shiftUp).
struct Blk {
  float A = 0.f, A1k = 0.f, A1m = 0.f;
  __device__ __forceinline__ void flush(int f) {
    if (f & 1) { A1k += A; A = 0.f; }
    if (f & 2) { A1m += A1k; A1k = 0.f; }
  }
  __device__ __forceinline__ float finish() {
    A1k += A;
    A1m += A1k;
    return A1m;
  }
};
// Update counters of one accumulator object (numIn1 / numIn1k / numIn1m).
struct BlkCnt {
  int n1 = 0, n1k = 0, n1m = 0;
  // numIn1++ then shiftUp(false); returns the flushed levels
  __device__ __forceinline__ int bump() {
    n1++;
    int f = 0;
    if (n1 > 1000) { f |= 1; n1k += n1; n1 = 0; }
    if (n1k > 1000) { f |= 2; n1m += n1k; n1k = 0; }
    return f;
  }
  __device__ __forceinline__ int total() const { return n1 + n1k + n1m; }
};

struct LinLds {
  float q[HS_MAXF][Q_N][8];
  float s[HS_MAXF][Q_N + 3];
  float econ[HS_MAXF];
  float act[HS_MAXF];
  float jx[HS_MAXF][4], jy[HS_MAXF][4], jd[HS_MAXF][2];
};

// resubstituteFPt: the point's idepth step from the previous linearization's per-point data
__device__ __forceinline__ float point_step(int p, int h, int nF, unsigned m, const float* cstep, const float* Hcd,
                                            float bdSumF, float HdiF, const int8_t* res_order, const float* xAd,
                                            const float* JpJdF) {
  if (m == 0u) return 0.f;
  float b = bdSumF;
  float dot = 0.f;
  for (int c = 0; c < 4; c++) dot += cstep[c] * Hcd[p * 4 + c];
  b -= dot;
  for (int q = 0; q < 8; q++) {
    const int tt = res_order[p * 8 + q];
    if (tt < 0) break;
    if (!((m >> tt) & 1u)) continue;
    const float* xa = xAd + (h * nF + tt) * 8;
    const float* jp = JpJdF + (p * 8 + tt) * 8;
    float d = 0.f;
    for (int i = 0; i < 8; i++) d += xa[i] * jp[i];
    b -= d;
  }
  return -b * HdiF;
}

}  // namespace

// =====================================================================================================
// linearize: one wave per point
// =====================================================================================================
__global__ __launch_bounds__(64) void hs_k_linearize(HsLinArgs a) {
  __shared__ LinLds L;
  const int lane = threadIdx.x;
  const int t = lane >> 3;  // target slot
  const int k = lane & 7;   // pattern pixel
  const int p = blockIdx.x;
  const int nF = a.nF;
  const int h = a.pt_host[p];
  const HsCalib cal = a.st->dcal;

  float idep = a.idepth[p], idep0 = a.idepth_zero[p];
  if (a.fuse_step) {
    // resubstituteFPt of the previous linearization + doStepFromBackup point part (stepfacD = 1)
    const float step = point_step(p, h, nF, a.p_actmask[p], a.st->cstep, a.p_Hcd, a.p_bdSumF[p], a.p_HdiF[p],
                                  a.res_order, a.xAd, a.p_JpJdF);
    idep = idep + 1.0f * step;
    idep0 = idep;
    __syncthreads();  // every lane has read the previous per-point data before it is overwritten
    if (lane == 0) {
      a.idepth[p] = idep;
      a.idepth_zero[p] = idep;
      a.p_step[p] = step;
    }
  }

  const float pu = a.u[p], pv = a.v[p];
  const int r = a.res_of_slot[p * 8 + t];
  const bool has = r >= 0;
  const int st = has ? (int)a.r_state[r] : HS_RES_OOB;

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
          const float3 hit = interp33(a.img[t], PKu, PKv, cal.W);
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
  // sequential (pattern-order) sums = the reference's running sums
  for (int qi = k; qi < Q_N; qi += 8) {
    float s = 0.f;
#pragma unroll
    for (int kk = 0; kk < 8; kk++) s += L.q[t][qi][kk];
    L.s[t][qi] = s;
  }
  __syncthreads();

  // ---------------- state decision + applyRes (the 8 lanes of a slot agree; lane k == 0 writes)
  bool active = false;
  float econ = 0.f;
  if (has) {
    const float oldE = a.r_energy[r];
    if (st == HS_RES_OOB) {
      econ = oldE;  // linearize returns state_energy; applyRes returns early (OOB is sticky)
      if (k == 0) a.r_ewo[r] = -1.f;
    } else if (slotOob) {
      econ = oldE;  // returns state_energy; applyRes: isActive = false, state = OOB, energy = NewEnergy
      if (k == 0) {
        a.r_ewo[r] = -1.f;
        a.r_state[r] = HS_RES_OOB;
        a.r_active[r] = 0;
        a.r_energy[r] = a.r_newEnergy[r];
      }
    } else {
      const float thr = fmaxf(a.frameTH[h], a.frameTH[t]);  // std::max<float>(host TH, target TH)
      float energyLeft = L.s[t][0];
      const float wJI2 = L.s[t][11];
      int ns;
      if (k == 0) a.r_ewo[r] = energyLeft;
      if (a.newest_cand != nullptr && t == nF - 1 && k == 0) {
        const int slot = atomicAdd(a.newest_cnt, 1);
        a.newest_cand[slot] = energyLeft;
      }
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
        float jj;
        if (k < 6) jj = Jx[4 + k] * aa + Jy[4 + k] * bb;
        else if (k == 6) jj = L.s[t][4] * Jd0 + L.s[t][5] * Jd1;
        else jj = L.s[t][6] * Jd0 + L.s[t][7] * Jd1;
        a.p_JpJdF[(p * 8 + t) * 8 + k] = jj;
        // Jacobian digest for the accumulate kernel (layout: hs_layout.h)
        float* jr = a.p_Jrec + (size_t)(p * 8 + t) * HS_JREC;
        for (int e = k; e < HS_JREC - 1; e += 8) {
          float v;
          if (e < 10) v = Jx[e];
          else if (e < 20) v = Jy[e - 10];
          else if (e == 20) v = J00;
          else if (e == 21) v = J10;
          else if (e == 22) v = J11;
          else if (e < 26) v = L.s[t][8 + (e - 23)];
          else if (e < 30) v = L.s[t][4 + (e - 26)];
          else v = L.s[t][12 + (e - 30)];
          jr[e] = v;
        }
      }
      if (k == 0) {
        a.r_state[r] = (uint8_t)ns;
        a.r_active[r] = active ? 1 : 0;
        a.r_energy[r] = energyLeft;
        a.r_newEnergy[r] = energyLeft;
      }
    }
    if (a.write_center && centreOk && k < 3) a.r_center[r * 3 + k] = centre[k];
  }
  if (k == 0) {
    L.econ[t] = econ;
    L.act[t] = active ? 1.f : 0.f;
    L.jd[t][0] = Jd0;
    L.jd[t][1] = Jd1;
  }
  if (k < 4) {
    L.jx[t][k] = Jx[k];
    L.jy[t][k] = Jy[k];
  }
  __syncthreads();

  // ---------------- per-point sums in the point's residual-list order (lane 0): addPoint<0> + SC prelude
  if (lane == 0) {
    double eSum = 0.0;
    float Hdd = 0.f, bd = 0.f, Hcd[4] = {0.f, 0.f, 0.f, 0.f};
    unsigned mask = 0u;
    for (int qn = 0; qn < 8; qn++) {
      const int tt = a.res_order[p * 8 + qn];
      if (tt < 0) break;
      eSum += (double)L.econ[tt];
      if (L.act[tt] == 0.f) continue;
      mask |= 1u << tt;
      const float J00 = L.s[tt][1], J11 = L.s[tt][2], J10 = L.s[tt][3];
      const float d0 = L.jd[tt][0], d1 = L.jd[tt][1];
      const float aa = J00 * d0 + J10 * d1;
      const float bb = J10 * d0 + J11 * d1;
      bd += L.s[tt][12] * d0 + L.s[tt][13] * d1;
      Hdd += aa * d0 + bb * d1;
#pragma unroll
      for (int c = 0; c < 4; c++) Hcd[c] += L.jx[tt][c] * aa + L.jy[tt][c] * bb;
    }
    a.p_energy[p] = eSum;
    a.p_actmask[p] = (uint8_t)mask;
    if (mask == 0u) {
      a.p_HdiF[p] = 0.f;
      a.p_bdSumF[p] = 0.f;
    } else {
      const float priorF = a.priorF[p];
      float Hh = Hdd + 0.f + priorF;  // Hdd_accAF + Hdd_accLF (no linearized residuals) + priorF
      if ((double)Hh < 1e-10) Hh = (float)1e-10;
      a.p_HdiF[p] = (float)(1.0 / (double)Hh);
      float bdSumF = bd + 0.f;
      bdSumF += priorF * (idep - idep0);
      a.p_bdSumF[p] = bdSumF;
    }
#pragma unroll
    for (int c = 0; c < 4; c++) a.p_Hcd[p * 4 + c] = Hcd[c] + 0.f;
  }
}

// =====================================================================================================
// accumulate: (host i, target slot j, split s) blocks + energy / Hcc,bc / energy threshold blocks
// =====================================================================================================
namespace {
constexpr int ACC_TILE = 64;
struct AccLds {
  float jp[ACC_TILE][64];
  float jr[ACC_TILE][HS_JREC];
  float hdi[ACC_TILE], bds[ACC_TILE], hcd[ACC_TILE][4];
  unsigned char m[ACC_TILE];
};

// linearizeAll's energy (+ the sumNID / numID statistics of doStepFromBackup); fixed-order tree in fp64
__device__ void acc_energy_block(const HsAccArgs& a) {
  __shared__ double red[256], red2[256];
  const int tid = threadIdx.x;
  double s = 0.0, s2 = 0.0;
  for (int p = tid; p < a.nP; p += 256) {
    s += a.p_energy[p];
    s2 += (double)fabsf(a.idepth[p]);
  }
  red[tid] = s;
  red2[tid] = s2;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) {
      red[tid] += red[tid + o];
      red2[tid] += red2[tid + o];
    }
    __syncthreads();
  }
  if (tid == 0) {
    a.energy_out[0] = red[0];
    a.energy_out[1] = red2[0];
    a.energy_out[2] = (double)a.nP;
  }
}

// accHcc / accbc over all points with an active residual (Src/AccumulatedSCHessian.cpp:32-33);
// 256 per-thread fp32 accumulators summed in fp64 in a fixed order (the reference sums its
// per-thread fp32 accumulators in fp64)
__device__ void acc_hcc_block(const HsAccArgs& a) {
  __shared__ float red[20][257];
  const int tid = threadIdx.x;
  float acc[20];
  for (int e = 0; e < 20; e++) acc[e] = 0.f;
  for (int p = tid; p < a.nP; p += 256) {
    if (a.actmask[p] == 0) continue;
    const float hdi = a.HdiF[p], bds = a.bdSumF[p];
    const float4 hc4 = reinterpret_cast<const float4*>(a.Hcd)[p];
    const float hc[4] = {hc4.x, hc4.y, hc4.z, hc4.w};
    for (int rr = 0; rr < 4; rr++) {
      const float wl = hdi * hc[rr];
      for (int c = 0; c < 4; c++) acc[rr * 4 + c] += wl * hc[c];
      acc[16 + rr] += bds * hdi * hc[rr];
    }
  }
  __shared__ double part[20][12];
  for (int e = 0; e < 20; e++) red[e][tid] = acc[e];
  __syncthreads();
  // 20 entries x 12 lanes partial sums, then a lane-ordered combine
  const int e = tid / 12, l = tid % 12;
  if (tid < 240) {
    double s = 0.0;
    for (int q = l; q < 256; q += 12) s += (double)red[e][q];
    part[e][l] = s;
  }
  __syncthreads();
  if (tid < 20) {
    double t = 0.0;
    for (int q = 0; q < 12; q++) t += part[tid][q];
    a.hccbc[tid] = t;
  }
}

// setNewFrameEnergyTH: k-th smallest candidate by 4-pass radix select with a parallel bin scan.
// Candidates of all ranks (all-gathered) are selected together, so every rank computes the same TH.
__device__ void acc_energy_th_block(const HsAccArgs& a) {
  __shared__ unsigned int hist[256], scan[256];
  __shared__ unsigned int s_prefix, s_mask, s_k, s_n;
  const int tid = threadIdx.x;
  if (tid == 0) {
    int n = 0;
    for (int r = 0; r < a.nranks; r++) n += a.cnt[r];
    s_n = (unsigned)n;
    s_prefix = 0;
    s_mask = 0;
    s_k = (unsigned int)(int)(a.frameEnergyTHN * (float)n);
  }
  __syncthreads();
  if (s_n == 0) {
    if (tid == 0) a.frameTH[a.newest] = 12 * 12 * 8;
    return;
  }
  for (int pass = 0; pass < 4; pass++) {
    const int shift = 24 - 8 * pass;
    hist[tid] = 0;
    __syncthreads();
    const unsigned int prefix = s_prefix, mask = s_mask;
    for (int r = 0; r < a.nranks; r++) {
      const float* cr = a.cand + (size_t)r * a.stride;
      const int nr = a.cnt[r];
      for (int i = tid; i < nr; i += 256) {
        const unsigned int v = __float_as_uint(cr[i]);
        if ((v & mask) == prefix) atomicAdd(&hist[(v >> shift) & 255u], 1u);
      }
    }
    __syncthreads();
    scan[tid] = hist[tid];
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {
      const unsigned int v = tid >= o ? scan[tid - o] : 0u;
      __syncthreads();
      scan[tid] += v;
      __syncthreads();
    }
    const unsigned int incl = scan[tid], excl = incl - hist[tid], kk = s_k;
    __syncthreads();
    if (excl <= kk && kk < incl) {
      s_k = kk - excl;
      s_prefix = prefix | ((unsigned int)tid << shift);
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
}  // namespace

__global__ __launch_bounds__(256) void hs_k_accumulate(HsAccArgs a) {
  const int nF = a.nF, S = a.S;
  const int nb = nF * nF * S;
  const int b = blockIdx.x;
  if (b == nb) { acc_energy_block(a); return; }
  if (b == nb + 1) { acc_hcc_block(a); return; }
  if (b == nb + 2) { acc_energy_th_block(a); return; }

  __shared__ AccLds T;
  const int tid = threadIdx.x;
  const int ij = b / S, s = b % S;
  const int i = ij % nF, j = ij / nF;  // host i, target j (accumulator index i + nF*j)
  const int hb = a.host_pt_begin[i], he = a.host_pt_begin[i + 1];
  const int span = he - hb;
  const int pb = hb + (int)((long long)span * s / S), pe = hb + (int)((long long)span * (s + 1) / S);

  // ---- thread roles
  // top entry (tid < 91): Data (r, c >= r) for e < 55, TopRight (r, col) for e < 85, BotRight for e < 91
  int er = 0, ec = 0, ttype = -1;
  if (tid < HS_TOP_N) {
    const int e = tid;
    if (e < 55) {
      int idx = 0;
      for (int rr = 0; rr < 10; rr++)
        for (int cc = rr; cc < 10; cc++) {
          if (idx == e) { er = rr; ec = cc; }
          idx++;
        }
      ttype = 0;
    } else if (e < 85) {
      er = (e - 55) / 3;
      ec = (e - 55) % 3;
      ttype = 1;
    } else {
      ec = e - 85;
      ttype = 2;
    }
  }
  // D entries (target j, target kD) [dr][dc] for kD = kD0 and kD0 + 4
  const int kD0 = tid >> 6, kD1 = kD0 + 4, dr = (tid & 63) >> 3, dc = tid & 7;
  // E entries: tid 91..122 (r = e >> 2, c = e & 3), EB: tid 123..130
  const int eE = tid - 91, eB = tid - 123;

  Blk top, d0, d1, ex;
  BlkCnt ctop, cd0, cd1, cex;

  for (int t0 = pb; t0 < pe; t0 += ACC_TILE) {
    const int tn = min(ACC_TILE, pe - t0);
    __syncthreads();
    for (int idx = tid; idx < tn * 16; idx += 256) {  // JpJdF of all slots, float4
      const int q = idx >> 4, w = idx & 15;
      reinterpret_cast<float4*>(T.jp[q])[w] = reinterpret_cast<const float4*>(a.JpJdF + (size_t)(t0 + q) * 64)[w];
    }
    for (int idx = tid; idx < tn * (HS_JREC / 4); idx += 256) {  // Jacobian digest of slot j, float4
      const int q = idx / (HS_JREC / 4), w = idx % (HS_JREC / 4);
      reinterpret_cast<float4*>(T.jr[q])[w] =
          reinterpret_cast<const float4*>(a.Jrec + ((size_t)(t0 + q) * 8 + j) * HS_JREC)[w];
    }
    for (int q = tid; q < tn; q += 256) {
      T.m[q] = a.actmask[t0 + q];
      T.hdi[q] = a.HdiF[t0 + q];
      T.bds[q] = a.bdSumF[t0 + q];
      reinterpret_cast<float4*>(T.hcd[q])[0] = reinterpret_cast<const float4*>(a.Hcd)[t0 + q];
    }
    __syncthreads();
    for (int q = 0; q < tn; q++) {
      const unsigned m = T.m[q];
      if (!((m >> j) & 1u)) continue;  // uniform
      const float* jr = T.jr[q];
      // ---- AccumulatedTopHessianSSE::addPoint<0>: update() (Data, then shiftUp), updateBotRight, updateTopRight
      if (ttype == 0) {
        const float xr = jr[HS_JR_X + er], xc = jr[HS_JR_X + ec], yr = jr[HS_JR_Y + er], yc = jr[HS_JR_Y + ec];
        top.A += jr[HS_JR_JIDX2 + 0] * xc * xr + jr[HS_JR_JIDX2 + 2] * yc * yr +
                 jr[HS_JR_JIDX2 + 1] * (xc * yr + yc * xr);
        top.flush(ctop.bump());
      } else if (ttype == 1) {
        top.flush(ctop.bump());
        const float xr = jr[HS_JR_X + er], yr = jr[HS_JR_Y + er];
        const float T0 = ec == 0 ? jr[HS_JR_JABJIDX + 0] : (ec == 1 ? jr[HS_JR_JABJIDX + 2] : jr[HS_JR_JIR + 0]);
        const float T1 = ec == 0 ? jr[HS_JR_JABJIDX + 1] : (ec == 1 ? jr[HS_JR_JABJIDX + 3] : jr[HS_JR_JIR + 1]);
        top.A += xr * T0 + yr * T1;
      } else if (ttype == 2) {
        top.flush(ctop.bump());
        const float v = ec == 0 ? jr[HS_JR_JAB2 + 0]
                      : ec == 1 ? jr[HS_JR_JAB2 + 1]
                      : ec == 2 ? jr[HS_JR_JABR + 0]
                      : ec == 3 ? jr[HS_JR_JAB2 + 2]
                      : ec == 4 ? jr[HS_JR_JABR + 1] : jr[HS_JR_RR];
        top.A += v;
      } else {
        ctop.bump();
      }
      // ---- AccumulatedSCHessianSSE::addPoint: accD[j][k] (both active), accE / accEB[j]
      const float hdi = T.hdi[q];
      const float wl = hdi * T.jp[q][j * 8 + dr];
      if ((m >> kD0) & 1u) {
        d0.A += wl * T.jp[q][kD0 * 8 + dc];
        d0.flush(cd0.bump());
      }
      if ((m >> kD1) & 1u) {
        d1.A += wl * T.jp[q][kD1 * 8 + dc];
        d1.flush(cd1.bump());
      }
      if (eE >= 0 && eE < 32) {
        ex.A += hdi * T.jp[q][j * 8 + (eE >> 2)] * T.hcd[q][eE & 3];
        ex.flush(cex.bump());
      } else if (eB >= 0 && eB < 8) {
        ex.A += hdi * T.bds[q] * T.jp[q][j * 8 + eB];
        ex.flush(cex.bump());
      } else {
        cex.bump();
      }
    }
  }
  float* P = a.part + ((size_t)ij * S + s) * HS_PART_N;
  int* PC = a.part_cnt + ((size_t)ij * S + s) * 16;
  if (tid < HS_TOP_N) P[tid] = top.finish();
  P[96 + kD0 * 64 + dr * 8 + dc] = d0.finish();
  P[96 + kD1 * 64 + dr * 8 + dc] = d1.finish();
  if (eE >= 0 && eE < 32) P[96 + 512 + eE] = ex.finish();
  else if (eB >= 0 && eB < 8) P[96 + 512 + 32 + eB] = ex.finish();
  if (tid == 0) {
    PC[0] = ctop.total();
    PC[9] = cex.total();
  }
  if ((tid & 63) == 0) {
    PC[1 + kD0] = cd0.total();
    PC[1 + kD1] = cd1.total();
  }
}

// =====================================================================================================
// stitch (fp64): one block (64 threads) per (host i, target j)
// =====================================================================================================
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
// index of (r, c) in the 10x10 upper-triangle Data block
__device__ __forceinline__ int tri_idx(int r, int c) {
  const int lo = r < c ? r : c, hi = r < c ? c : r;
  return lo * 10 - (lo * (lo - 1)) / 2 + (hi - lo);
}
}  // namespace

__global__ __launch_bounds__(64) void hs_k_stitch(HsStitchArgs a) {
  const int nF = a.nF, S = a.S;
  const int i = blockIdx.x % nF, j = blockIdx.x / nF;
  const int ij = i + nF * j;
  const int tid = threadIdx.x;
  const int n = 4 + 8 * nF;
  const int iIdx = 4 + 8 * i, jIdx = 4 + 8 * j;
  __shared__ double e[96], A88[64], A84[32], a8r[8], tmp[64], aH[64], aT[64], D[64], aH2[64], aT2[64], v8[8], Hpc[32];
  __shared__ int topCnt;
  aH[tid] = a.adHost[ij * 64 + tid];
  aT[tid] = a.adTarget[ij * 64 + tid];
  // sum of the split partials (stitchDoubleInternal: accH += acc[tid2].H.cast<double>() for num > 0)
  const float* P0 = a.part + (size_t)ij * S * HS_PART_N;
  const int* C0 = a.part_cnt + (size_t)ij * S * 16;
  if (tid == 0) {
    int c = 0;
    for (int s = 0; s < S; s++) c += C0[s * 16];
    topCnt = c;
  }
  for (int q = tid; q < 96; q += 64) {
    double sum = 0.0;
    for (int s = 0; s < S; s++)
      if (C0[s * 16] > 0) sum += (double)P0[s * HS_PART_N + q];
    e[q] = sum;
  }
  if (tid < 32) {
    double sum = 0.0;
    for (int s = 0; s < S; s++) sum += (double)P0[s * HS_PART_N + 96 + 512 + tid];
    Hpc[tid] = sum;
  }
  if (tid < 8) {
    double sum = 0.0;
    for (int s = 0; s < S; s++) sum += (double)P0[s * HS_PART_N + 96 + 512 + 32 + tid];
    v8[tid] = sum;
  }
  __syncthreads();
  const bool haveTop = topCnt > 0;
  if (haveTop) {  // AccumulatorApprox::finish -> 13x13 [calib4|xi6|a|b|r]
    const int r = tid >> 3, c = tid & 7;  // A88 = H[4+r][4+c]
    const int R = 4 + r, Cc = 4 + c;
    double v;
    if (R < 10 && Cc < 10) {
      v = e[tri_idx(R, Cc)];
    } else if (R < 10 || Cc < 10) {
      const int row = R < 10 ? R : Cc, col = (R < 10 ? Cc : R) - 10;
      v = e[55 + 3 * row + col];
    } else {
      const int bi = (R - 10) + (Cc - 10);  // (a,a) 0, (a,b) 1, (b,b) 3
      v = e[85 + (bi == 2 ? 3 : bi)];
    }
    A88[tid] = v;
    if (tid < 32) {  // A84 = H[4+r][c]
      const int rr = tid >> 2, cc = tid & 3;
      const int RR = 4 + rr;
      A84[tid] = RR < 10 ? e[tri_idx(cc, RR)] : e[55 + 3 * cc + (RR - 10)];
    }
    if (tid < 8) {  // a8r = H[4+r][12]
      const int RR = 4 + tid;
      a8r[tid] = RR < 10 ? e[55 + 3 * RR + 2] : (RR == 10 ? e[85 + 2] : e[85 + 4]);
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
      for (int l = 0; l < 8; l++) {
        s1 += aH[rr * 8 + l] * A84[l * 4 + cc];
        s2 += aT[rr * 8 + l] * A84[l * 4 + cc];
      }
      atomicAdd(&a.HA[(iIdx + rr) * n + cc], s1);
      atomicAdd(&a.HA[(jIdx + rr) * n + cc], s2);
    }
    if (tid < 16) atomicAdd(&a.HA[(tid >> 2) * n + (tid & 3)], e[tri_idx(tid >> 2, tid & 3)]);
    if (tid < 8) {
      double s1 = 0.0, s2 = 0.0;
      for (int l = 0; l < 8; l++) {
        s1 += aH[tid * 8 + l] * a8r[l];
        s2 += aT[tid * 8 + l] * a8r[l];
      }
      atomicAdd(&a.bA[iIdx + tid], s1);
      atomicAdd(&a.bA[jIdx + tid], s2);
    }
    if (tid < 4) atomicAdd(&a.bA[tid], e[55 + 3 * tid + 2]);
  }
  // ---- Schur complement rows (i, j, k)
  if (tid < 32) {
    const int rr = tid >> 2, cc = tid & 3;
    double s1 = 0.0, s2 = 0.0;
    for (int l = 0; l < 8; l++) {
      s1 += aH[rr * 8 + l] * Hpc[l * 4 + cc];
      s2 += aT[rr * 8 + l] * Hpc[l * 4 + cc];
    }
    atomicAdd(&a.HSC[(iIdx + rr) * n + cc], s1);
    atomicAdd(&a.HSC[(jIdx + rr) * n + cc], s2);
  }
  if (tid < 8) {
    double s1 = 0.0, s2 = 0.0;
    for (int l = 0; l < 8; l++) {
      s1 += aH[tid * 8 + l] * v8[l];
      s2 += aT[tid * 8 + l] * v8[l];
    }
    atomicAdd(&a.bSC[iIdx + tid], s1);
    atomicAdd(&a.bSC[jIdx + tid], s2);
  }
  for (int kk = 0; kk < nF; kk++) {
    const int kIdx = 4 + 8 * kk;
    const int ik = i + nF * kk;
    int dcnt = 0;
    for (int s = 0; s < S; s++) dcnt += C0[s * 16 + 1 + kk];
    if (dcnt == 0) continue;  // accD num == 0 (uniform)
    __syncthreads();
    double sum = 0.0;
    for (int s = 0; s < S; s++)
      if (C0[s * 16 + 1 + kk] > 0) sum += (double)P0[s * HS_PART_N + 96 + kk * 64 + tid];
    D[tid] = sum;
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
  if (blockIdx.x == 0 && tid < 16) atomicAdd(&a.HSC[(tid >> 2) * n + (tid & 3)], a.hccbc[tid]);
  if (blockIdx.x == 0 && tid < 4) atomicAdd(&a.bSC[tid], a.hccbc[16 + tid]);
}

// =====================================================================================================
// solve + step (fp64), one workgroup of 256 threads
// =====================================================================================================
__global__ __launch_bounds__(256) void hs_k_solve(HsSolveArgs a) {
  __shared__ double Hs[HS_MAXDIM * HS_MAXDIM];
  __shared__ double Hp[HS_MAXDIM * HS_MAXDIM];
  __shared__ double bf[HS_MAXDIM], Sv[HS_MAXDIM], xs[HS_MAXDIM], yv[HS_MAXDIM], px[HS_MAXDIM], dl[HS_MAXDIM];
  __shared__ float xF[HS_MAXDIM];
  __shared__ int pos[HS_MAXDIM];
  __shared__ int s_it;
  HsDevState* st = a.st;
  const int tid = threadIdx.x, nt = blockDim.x;
  const int nF = st->nF, n = 4 + 8 * nF;
  const double lambda = 1e-5;  // SOLVER_FIX_LAMBDA
  if (tid == 0) s_it = a.iteration >= 0 ? a.iteration : st->iteration;

  if (a.flags & HS_SOLVE) {
    if (tid == 0 && a.energy_log) {
      a.energy_log[st->log_count] = a.sysE[0];
      st->log_count = st->log_count + 1;
    }
    // getStitchedDeltaF for bM + HM * delta
    for (int q = tid; q < n; q += nt)
      dl[q] = q < 4 ? (double)(float)st->calib.value_minus_value_zero[q] : st->frames[(q - 4) / 8].delta[(q - 4) % 8];
    __syncthreads();
    // HFinal = (HL + HM) + HA ; diag *= (1+lambda) ; HFinal -= HSC / (1+lambda)
    const double sc = (double)(1.0f / (1 + lambda));
    for (int idx = tid; idx < n * n; idx += nt) {
      const int r = idx / n, c = idx % n;
      const int fr = r < 4 ? -1 : (r - 4) / 8, fc = c < 4 ? -1 : (c - 4) / 8;
      double ha = a.HA[idx];
      if (fr >= 0 && fc >= 0 && fr != fc) ha = a.HA[idx] + a.HA[c * n + r];  // stitchDoubleMT symmetrization
      else if (r < 4 && c >= 4) ha = a.HA[c * n + r];                          // calib row <- column
      double hsc = a.HSC[idx];
      if (r < 4 && c >= 4) hsc = a.HSC[c * n + r];
      double hl = 0.0;
      if (r == c) hl = r < 4 ? a.initialCalibHessian : st->frames[fr].prior[(r - 4) % 8];
      double hf = (hl + a.HM[idx]) + ha;
      if (r == c) hf *= (1 + lambda);
      hf = hf - hsc * sc;
      Hs[idx] = hf;
    }
    for (int q = tid; q < n; q += nt) {
      double bl;
      if (q < 4) {
        bl = a.initialCalibHessian * dl[q];
      } else {
        const hs::FrameH& f = st->frames[(q - 4) / 8];
        bl = f.prior[(q - 4) % 8] * f.delta_prior[(q - 4) % 8];
      }
      double hmd = 0.0;
      for (int c = 0; c < n; c++) hmd += a.HM[q * n + c] * dl[c];
      bf[q] = ((bl + (a.bM[q] + hmd)) + a.bA[q]) - a.bSC[q];
    }
    __syncthreads();
    // the consumed accumulation targets are zeroed for the next linearization
    for (int idx = tid; idx < n * n; idx += nt) {
      a.HA[idx] = 0.0;
      a.HSC[idx] = 0.0;
    }
    for (int q = tid; q < n; q += nt) {
      a.bA[q] = 0.0;
      a.bSC[q] = 0.0;
      Sv[q] = 1.0 / sqrt(Hs[q * n + q] + 10);
    }
    __syncthreads();
    for (int idx = tid; idx < n * n; idx += nt) {
      const int r = idx / n, c = idx % n;
      Hs[idx] = Sv[r] * Hs[idx] * Sv[c];
    }
    for (int q = tid; q < n; q += nt) bf[q] = Sv[q] * bf[q];
    __syncthreads();
    // Eigen LDLT pivot order: largest |diagonal| among the remaining (left-looking: the original diagonal),
    // first position on ties; equivalent to an unpivoted LDLT of P H P^T.
    if (tid < 64) {
      for (int q = tid; q < n; q += 64) pos[q] = q;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_wave_barrier();
      for (int kq = 0; kq < n; kq++) {
        double best = -1.0;
        int bi = n;
        for (int q = kq + tid; q < n; q += 64) {
          const double v = fabs(Hs[pos[q] * n + pos[q]]);
          if (v > best) { best = v; bi = q; }
        }
        for (int o = 32; o > 0; o >>= 1) {
          const double ob = __shfl_xor(best, o);
          const int oi = __shfl_xor(bi, o);
          if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
        }
        if (tid == 0 && bi != kq) {
          const int tq = pos[kq];
          pos[kq] = pos[bi];
          pos[bi] = tq;
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        __builtin_amdgcn_wave_barrier();
      }
    }
    __syncthreads();
    for (int idx = tid; idx < n * n; idx += nt) {
      const int r = idx / n, c = idx % n;
      Hp[idx] = Hs[pos[r] * n + pos[c]];
    }
    for (int q = tid; q < n; q += nt) yv[q] = bf[pos[q]];
    __syncthreads();
    // right-looking LDLT of the lower triangle; forward substitution L z = P b fused into the sweep
    for (int kq = 0; kq < n; kq++) {
      const double d = Hp[kq * n + kq];
      const bool valid = fabs(d) > DBL_MIN;
      if (valid)
        for (int q = kq + 1 + tid; q < n; q += nt) Hp[q * n + kq] /= d;
      __syncthreads();
      const double yk = yv[kq];
      for (int q = kq + 1 + tid; q < n; q += nt) yv[q] -= Hp[q * n + kq] * yk;
      const int m = n - kq - 1;
      const int ntri = m * (m + 1) / 2;
      for (int t = tid; t < ntri; t += nt) {
        // t -> (rr >= cc) in the trailing lower triangle
        int rr = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
        while (rr * (rr + 1) / 2 > t) rr--;
        while ((rr + 1) * (rr + 2) / 2 <= t) rr++;
        const int cc = t - rr * (rr + 1) / 2;
        const int R = kq + 1 + rr, Cc = kq + 1 + cc;
        Hp[R * n + Cc] -= Hp[R * n + kq] * (d * Hp[Cc * n + kq]);
      }
      __syncthreads();
    }
    for (int q = tid; q < n; q += nt) {
      const double d = Hp[q * n + q];
      yv[q] = fabs(d) > DBL_MIN ? yv[q] / d : 0.0;
    }
    __syncthreads();
    // backward substitution L^T x = z: one wave, a dot product per row
    if (tid < 64) {
      for (int kq = n - 1; kq >= 0; kq--) {
        double s = 0.0;
        for (int q = kq + 1 + tid; q < n; q += 64) s += Hp[q * n + kq] * yv[q];
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
        if (tid == 0) yv[kq] = yv[kq] - s;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        __builtin_amdgcn_wave_barrier();
      }
    }
    __syncthreads();
    for (int q = tid; q < n; q += nt) xs[pos[q]] = yv[q];
    __syncthreads();
    for (int q = tid; q < n; q += nt) xs[q] = Sv[q] * xs[q];
    __syncthreads();
    if (s_it >= 2) {  // SOLVER_ORTHOGONALIZE_X_LATER
      for (int q = tid; q < n; q += nt) {
        double s = 0.0;
        for (int c = 0; c < n; c++) s += a.Porth[q * n + c] * xs[c];
        px[q] = s;
      }
      __syncthreads();
      for (int q = tid; q < n; q += nt) xs[q] -= px[q];
      __syncthreads();
    }
    // resubstituteF_MT: frame / calib steps, xAd, cstep
    for (int q = tid; q < n; q += nt) {
      const double xv = xs[q];
      if (!isfinite(xv)) st->status = 1;
      xF[q] = (float)xv;
      st->lastX[q] = xv;
      if (a.x_out) a.x_out[q] = xv;
      if (q < 4) st->calib.step[q] = -xv;
      else st->frames[(q - 4) / 8].step[(q - 4) % 8] = -xv;
    }
    if (tid < nF) {
      st->frames[tid].step[8] = 0;
      st->frames[tid].step[9] = 0;
    }
    __syncthreads();
    if (tid < 4) st->cstep[tid] = xF[tid];
    for (int o = tid; o < nF * nF * 8; o += nt) {
      const int pair = o >> 3, c = o & 7;
      const int hh = pair / nF, tt = pair % nF;  // xAd[nF*h + t]
      const float* aHf = a.adHostF + (hh + nF * tt) * 64;
      const float* aTf = a.adTargetF + (hh + nF * tt) * 64;
      float s1 = 0.f, s2 = 0.f;
      for (int rr = 0; rr < 8; rr++) s1 += xF[4 + 8 * hh + rr] * aHf[rr * 8 + c];
      for (int rr = 0; rr < 8; rr++) s2 += xF[4 + 8 * tt + rr] * aTf[rr * 8 + c];
      a.xAd[o] = s1 + s2;
    }
  }
  __syncthreads();
  if (a.flags & HS_APPLY) {
    // backupState + doStepFromBackup(1, 1, 1, 1, 1): calib and frames, then setPrecalcValues
    if (tid == 0) {
      hs::CalibH& cal = st->calib;
      double nv[4];
      for (int q = 0; q < 4; q++) {
        cal.value_backup[q] = cal.value[q];
        nv[q] = cal.value_backup[q] + 1.0f * cal.step[q];
      }
      cal.setValue(nv);
      st->dcal = cal.device();
    }
    if (tid < nF) {
      hs::FrameH& f = st->frames[tid];
      double s[10];
      for (int q = 0; q < 10; q++) {
        f.state_backup[q] = f.state[q];
        s[q] = f.state_backup[q] + 1.0 * f.step[q];
      }
      f.setState(s);
      for (int q = 0; q < 8; q++) {
        f.delta[q] = f.state[q] - f.state_zero[q];
        f.delta_prior[q] = f.state[q] - 0.0;
      }
    }
    __syncthreads();
    for (int pr = tid; pr < nF * nF; pr += nt) {
      const int hh = pr / nF, tt = pr % nF;
      a.pre[pr] = hs::make_precalc(st->frames[hh], st->frames[tt], st->calib);
    }
    if (tid == 0) {
      float sumA = 0, sumB = 0, sumT = 0, sumR = 0;
      for (int f = 0; f < nF; f++) {
        const double* sp = st->frames[f].step;
        sumA += sp[6] * sp[6];
        sumB += sp[7] * sp[7];
        sumT += sp[0] * sp[0] + sp[1] * sp[1] + sp[2] * sp[2];
        sumR += sp[3] * sp[3] + sp[4] * sp[4] + sp[5] * sp[5];
      }
      const float nfr = (float)nF;
      sumA /= nfr; sumB /= nfr; sumR /= nfr; sumT /= nfr;
      const float sumNID = a.sysE[2] > 0 ? (float)(a.sysE[1] / a.sysE[2]) : 0.f;
      const float th = a.thOptIterations;
      st->canbreak = sqrtf(sumA) < 0.0005 * th && sqrtf(sumB) < 0.00005 * th && sqrtf(sumR) < 0.00005 * th &&
                     sqrtf(sumT) * sumNID < 0.00005 * th;
      st->iteration = s_it + 1;
    }
  }
  if (tid == 0 && a.cnt_reset) *a.cnt_reset = 0;
}

// =====================================================================================================
// granular API helpers
// =====================================================================================================
__global__ void hs_k_resub(HsResubArgs a) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= a.n) return;
  const float step = point_step(p, a.host[p], a.nF, a.actmask[p], a.st->cstep, a.Hcd, a.bdSumF[p], a.HdiF[p],
                                a.res_order, a.xAd, a.JpJdF);
  a.step[p] = step;
  if (a.apply) {
    const float nid = a.idepth[p] + 1.0f * step;
    a.idepth[p] = nid;
    a.idepth_zero[p] = nid;
  }
}

__global__ void hs_k_apply_step(int n, const float* step, float* idepth, float* idepth_zero) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < n) {
    const float nid = idepth[p] + 1.0f * step[p];
    idepth[p] = nid;
    idepth_zero[p] = nid;
  }
}
