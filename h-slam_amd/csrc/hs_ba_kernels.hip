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
//   stitch_pair     stitchDoubleInternal (top: Src/AccumulatedTopHessian.cpp:218-280, Schur:
//                   Src/AccumulatedSCHessian.cpp:54-133) in fp64, fused into hs_k_accumulate: the last
//                   split block of each (host, target) pair to finish stitches it.
// Per-residual arithmetic follows the reference operation order with fp contraction off.
#pragma clang fp contract(off)
#include <hip/hip_runtime.h>

#include <cfloat>
#include <type_traits>

#include "hs_kernels.h"

namespace {

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

// wall-clock checkpoint of a block (thread 0) when tracing is enabled
#define HS_TRACE(A, slot)                                                                          \
  do {                                                                                             \
    if ((A).trace && threadIdx.x == 0) (A).trace[(size_t)blockIdx.x * 16 + (slot)] = wall_clock64(); \
  } while (0)

struct LinLds {
  float s[HS_MAXF][Q_N + 3];
};

// lane l <- lane l-1 within each row of 16 (DPP row_shr:1; a row's lane 0 gets 0)
__device__ __forceinline__ float dpp_shr1(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x111, 0xf, 0xf, false));
}
// Left fold over the 8 lanes of each octet (= a target slot's pattern pixels): lane 8g+7 returns
// ((((0 + x[8g]) + x[8g+1]) + ...) + x[8g+7]), the reference's running sum in pattern order, bit for bit
// (step j: s[l] = s[l-1] + x[l], so after 7 steps lane 8g+7 holds the in-order fold of its octet).
__device__ __forceinline__ float octet_fold(float x) {
  float s = 0.f + x;
#pragma unroll
  for (int j = 0; j < 7; j++) s = dpp_shr1(s) + x;
  return s;
}
__device__ __forceinline__ float readlane_f(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

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
  int h = 0;  // points are sorted by host: the host is found from the kernel-argument boundaries, no load
#pragma unroll
  for (int i = 1; i < HS_MAXF; i++) h += (i < nF && p >= a.host_begin[i]) ? 1 : 0;
  const HsCalib cal = a.st->dcal;

  HS_TRACE(a, 0);
  // everything the linearization reads is loaded up front, unconditionally (clamped indices), so the
  // prologue is ONE memory round trip: residual state is in the slot layout [point][target slot] and the
  // host comes from the kernel arguments, so no load depends on another
  if (a.marg && a.marg[p] == 0) {  // marginalization pass, point not marginalized: no active residual
    if (lane == 0) {
      a.p_energy[p] = 0.0;
      a.p_actmask[p] = 0;
      a.p_HdiF[p] = 0.f;
      a.p_bdSumF[p] = 0.f;
      reinterpret_cast<float4*>(a.p_Hcd)[p] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (t == nF - 1 && k == 0) a.newest_cand[p] = -1.f;
    return;
  }
  const int sl = p * 8 + t;                 // this lane's residual slot
  const int tc_ = t < nF ? t : 0;
  float idep = a.idepth[p], idep0 = a.idepth_zero[p];
  const float pu = a.u[p], pv = a.v[p];
  const bool has = a.res_of_slot[sl] >= 0;
  const int st_raw = (int)a.r_state[sl];
  const float oldE_raw = a.r_energy[sl];
  const float oldNewE_raw = a.r_newEnergy[sl];
  const float thr = fmaxf(a.frameTH[h], a.frameTH[tc_]);  // std::max<float>(host TH, target TH)
  const float colorK = a.color[p * 8 + k], weightK = a.weight[p * 8 + k];
  const HsPrecalc pc = a.pre[h * nF + tc_];
  // the target's image: selected from the kernel-argument pointers (uniform SGPRs), not loaded per lane
  const float4* timg = a.img[0];
#pragma unroll
  for (int i = 1; i < HS_MAXF; i++) timg = (t == i) ? a.img[i] : timg;
  const uint2 ro2 = reinterpret_cast<const uint2*>(a.res_order)[p];  // the point's 8 residual-list slots
  auto res_slot = [&](int q) -> int { return (int)(int8_t)(((q < 4 ? ro2.x : ro2.y) >> (8 * (q & 3))) & 0xffu); };
  // the previous linearization's per-point data for the fused step (read unconditionally: one batch)
  const unsigned fm = a.p_actmask[p];
  const float xad = a.xAd[(h * nF + tc_) * 8 + k];
  const float jpj = a.p_JpJdF[sl * 8 + k];
  const float bds = a.p_bdSumF[p], hdi = a.p_HdiF[p];
  const float4 hcd = reinterpret_cast<const float4*>(a.p_Hcd)[p];
  const float4 cs4 = *reinterpret_cast<const float4*>(a.st->cstep);
  const float cs0 = cs4.x, cs1 = cs4.y, cs2 = cs4.z, cs3 = cs4.w;
  // pin the batch: without this the compiler sinks the fused-step loads into the fuse_step branch, behind
  // the wait for res_order (a second memory round trip)
  asm volatile("" ::"v"(fm), "v"(xad), "v"(jpj), "v"(bds), "v"(hdi), "v"(hcd.x), "v"(hcd.y), "v"(hcd.z), "v"(hcd.w),
               "v"(cs0), "v"(cs1), "v"(cs2), "v"(cs3), "v"(ro2.x), "v"(ro2.y));
  if (a.fuse_step) {
    // resubstituteFPt of the previous linearization (Src/EnergyFunctional.cpp:249-274) + the point part of
    // doStepFromBackup (stepfacD = 1).  Lane (t, k) forms xAd[h][t][k] * JpJdF[t][k]; the 8-term dot of a
    // residual is an in-order octet fold, the residual terms are then subtracted in list order (uniform).
    const unsigned m = fm;
    const float prod = ((m >> t) & 1u) ? xad * jpj : 0.f;
    const float dsum = octet_fold(prod);
    // branch-free (no load-dependent scalar control flow here, so every prologue load is one batch):
    // the list-order subtraction walks the point's residual slots with ds_bpermute reads of the folds
    float b = bds;
    float dot = 0.f;
    dot += cs0 * hcd.x;
    dot += cs1 * hcd.y;
    dot += cs2 * hcd.z;
    dot += cs3 * hcd.w;
    b -= dot;
    bool live = true;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const int tt = res_slot(q);
      live = live && tt >= 0;
      const int ts = tt < 0 ? 0 : tt;
      const float d = __shfl(dsum, ts * 8 + 7);
      if (live && ((m >> ts) & 1u)) b -= d;
    }
    const float step = m != 0u ? -b * hdi : 0.f;
    idep = idep + 1.0f * step;
    idep0 = idep;
    if (lane == 0) {
      a.idepth[p] = idep;
      a.idepth_zero[p] = idep;
      a.p_step[p] = step;
    }
  }
  // the marginalization pass starts from resetOOB (state IN, energies 0; Src/Mapping.cpp:285)
  const int st = has ? (a.marg ? HS_RES_IN : st_raw) : HS_RES_OOB;
  const float oldE = (has && !a.marg) ? oldE_raw : 0.f;
  const float oldNewE = (has && !a.marg) ? oldNewE_raw : 0.f;
  HS_TRACE(a, 1);

  bool oob = false;
  float Jx[10] = {0}, Jy[10] = {0}, Jd0 = 0.f, Jd1 = 0.f;
  float qv[Q_N];
#pragma unroll
  for (int qi = 0; qi < Q_N; qi++) qv[qi] = 0.f;
  float centre[3] = {0.f, 0.f, 0.f};
  bool centreOk = false;
  if (has && st != HS_RES_OOB) {
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

        // pattern pixel k (staticPattern[8], Include/GlobalTypes.h:181-184) as selects: a lane-indexed
        // constant-memory table would cost a dependent memory round trip here
        const int pdx = (k == 1 || k == 6) ? -1 : (k == 2) ? 1 : (k == 3) ? -2 : (k == 5) ? 2 : 0;
        const int pdy = (k == 0) ? -2 : (k <= 2) ? -1 : (k <= 5) ? 0 : (k == 6) ? 1 : 2;
        const float px = pu + pdx, py = pv + pdy;
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
          float3 hit = interp33(timg, PKu, PKv, cal.W);
          // all three channels are materialised here: otherwise the compiler sinks the dI/dx, dI/dy loads
          // under the isfinite(I) branch below, a second dependent memory round trip
          asm volatile("" : "+v"(hit.x), "+v"(hit.y), "+v"(hit.z));
          const float color = colorK;
          const float residual = hit.x - (float)(pc.aff[0] * color + pc.aff[1]);
          const float drdA = (color - pc.b0);
          if (!isfinite(hit.x)) {
            oob = true;
          } else {
            float w = sqrtf(a.lp.outlierTHSumComponent /
                            (a.lp.outlierTHSumComponent + (hit.y * hit.y + hit.z * hit.z)));
            w = 0.5f * (w + weightK);
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
            // AccumulatedTopHessianSSE::addPoint<0>: JI_r, Jab_r, rr over resApprox = resF; in the
            // marginalization pass addPoint<2> over res_toZeroF = resF - [JI Jp, Jab] delta
            // (fixLinearizationF, Src/OptimizationClasses.cpp:258-284)
            float rz = resF;
            if (a.marg) {
              const float* dp = a.adHTdelta + (h + nF * t) * 8;
              float jx = 0.f, jy = 0.f, cx = 0.f, cy = 0.f;
#pragma unroll
              for (int i = 0; i < 6; i++) {
                jx += Jx[4 + i] * dp[i];
                jy += Jy[4 + i] * dp[i];
              }
#pragma unroll
              for (int i = 0; i < 4; i++) {
                cx += Jx[i] * a.cDelta[i];
                cy += Jy[i] * a.cDelta[i];
              }
              const float dF = idep - idep0;
              const float Jpdx = jx + cx + Jd0 * dF;
              const float Jpdy = jy + cy + Jd1 * dF;
              rz = rz - hy * Jpdx;
              rz = rz - hz * Jpdy;
              rz = rz - jab0 * dp[6];
              rz = rz - jab1 * dp[7];
            }
            qv[12] = rz * hy;
            qv[13] = rz * hz;
            qv[14] = rz * jab0;
            qv[15] = rz * jab1;
            qv[16] = rz * rz;
          }
        }
      }
    }
  }
  const unsigned long long oobMask = __ballot(oob);
  const bool slotOob = ((oobMask >> (t * 8)) & 0xffull) != 0ull;
  HS_TRACE(a, 2);

  // sequential (pattern-order) sums = the reference's running sums: octet folds, published by lane k == 7
  {
    float sq[Q_N];
#pragma unroll
    for (int qi = 0; qi < Q_N; qi++) sq[qi] = octet_fold(qv[qi]);
    if (k == 7) {
#pragma unroll
      for (int qi = 0; qi < Q_N; qi++) L.s[t][qi] = sq[qi];
    }
  }
  __syncthreads();
  HS_TRACE(a, 4);

  // ---------------- state decision + applyRes (the 8 lanes of a slot agree; lane k == 0 writes).
  // Predicated rather than branched: the slot's sums are read from LDS in one batch and every store is
  // issued under a mask, so the divergent slot cases cost no serialised LDS round trips.
  float S[Q_N];
#pragma unroll
  for (int qi = 0; qi < Q_N; qi++) S[qi] = L.s[t][qi];
  const bool live = has && st != HS_RES_OOB;      // OOB is sticky: linearize returns state_energy
  const bool eval = live && !slotOob;             // a full linearization of this residual
  const bool isOut = S[0] > thr || S[11] < 2;
  const float energyLeft = isOut ? thr : S[0];
  const bool active = eval && !isOut;
  const float econ = eval ? energyLeft : oldE;
  if (has && k == 0) {
    a.r_ewo[sl] = eval ? S[0] : -1.f;
    if (live) {  // applyRes: OOB now -> inactive, state OOB, energy = NewEnergy; else the new state
      a.r_state[sl] = (uint8_t)(slotOob ? HS_RES_OOB : (isOut ? HS_RES_OUT : HS_RES_IN));
      a.r_active[sl] = active ? 1 : 0;
      a.r_energy[sl] = slotOob ? oldNewE : energyLeft;
      if (!slotOob) a.r_newEnergy[sl] = energyLeft;
    }
  }
  if (t == nF - 1 && k == 0) a.newest_cand[p] = eval ? S[0] : -1.f;
  if (has && a.write_center && centreOk && k < 3) a.r_center[sl * 3 + k] = centre[k];
  float tHdd = 0.f, tbd = 0.f, tc[4] = {0.f, 0.f, 0.f, 0.f};  // the slot's terms of the per-point sums
  {
    // takeData (Include/OptimizationClasses.h:195-201), computed unconditionally, stored when active
    const float J00 = S[1], J11 = S[2], J10 = S[3];
    const float aa = J00 * Jd0 + J10 * Jd1;
    const float bb = J10 * Jd0 + J11 * Jd1;
    // this residual's terms of the point sums (AccumulatedTopHessianSSE::addPoint<0> / SC prelude)
    tbd = S[12] * Jd0 + S[13] * Jd1;
    tHdd = aa * Jd0 + bb * Jd1;
#pragma unroll
    for (int c = 0; c < 4; c++) tc[c] = Jx[c] * aa + Jy[c] * bb;
    float jx4 = Jx[4], jy4 = Jy[4];
#pragma unroll
    for (int c = 5; c < 10; c++) {
      jx4 = k == c - 4 ? Jx[c] : jx4;
      jy4 = k == c - 4 ? Jy[c] : jy4;
    }
    const float jj = k < 6 ? jx4 * aa + jy4 * bb : (k == 6 ? S[4] * Jd0 + S[5] * Jd1 : S[6] * Jd0 + S[7] * Jd1);
    // Jacobian digest entries e = k + 8i (layout: hs_layout.h), selected with constant indices
    float v0 = Jx[0];
#pragma unroll
    for (int c = 1; c < 8; c++) v0 = k == c ? Jx[c] : v0;           // e = k
    float v1;
    {
      float y = Jy[0];
#pragma unroll
      for (int c = 1; c < 6; c++) y = k - 2 == c ? Jy[c] : y;      // e = k + 8 >= 10 -> Jy[k - 2]
      v1 = k == 0 ? Jx[8] : (k == 1 ? Jx[9] : y);
    }
    float v2 = Jy[6];                                               // e = k + 16
    v2 = k == 1 ? Jy[7] : v2;
    v2 = k == 2 ? Jy[8] : v2;
    v2 = k == 3 ? Jy[9] : v2;
    v2 = k == 4 ? J00 : v2;
    v2 = k == 5 ? J10 : v2;
    v2 = k == 6 ? J11 : v2;
    v2 = k == 7 ? S[8] : v2;
    float v3 = S[9];                                                // e = k + 24
    v3 = k == 1 ? S[10] : v3;
    v3 = k == 2 ? S[4] : v3;
    v3 = k == 3 ? S[5] : v3;
    v3 = k == 4 ? S[6] : v3;
    v3 = k == 5 ? S[7] : v3;
    v3 = k == 6 ? S[12] : v3;
    v3 = k == 7 ? S[13] : v3;
    float v4 = S[14];                                               // e = k + 32 (k < 3)
    v4 = k == 1 ? S[15] : v4;
    v4 = k == 2 ? S[16] : v4;
    if (active) {
      a.p_JpJdF[(p * 8 + t) * 8 + k] = jj;
      float* jr = a.p_Jrec + (size_t)(p * 8 + t) * HS_JREC;
      jr[k] = v0;
      jr[k + 8] = v1;
      jr[k + 16] = v2;
      jr[k + 24] = v3;
      if (k < 3) jr[k + 32] = v4;
    }
  }
  HS_TRACE(a, 5);
  // ---------------- per-point sums in the point's residual-list order (uniform; readlane from lane 8 * slot)
  {
    const unsigned long long actBits = __ballot(active);
    double eSum = 0.0;
    float Hdd = 0.f, bd = 0.f, Hcd[4] = {0.f, 0.f, 0.f, 0.f};
    unsigned mask = 0u;
    for (int qn = 0; qn < 8; qn++) {
      const int tt = res_slot(qn);
      if (tt < 0) break;
      const int src = tt * 8;
      eSum += (double)readlane_f(econ, src);
      if (!((actBits >> src) & 1ull)) continue;
      mask |= 1u << tt;
      bd += readlane_f(tbd, src);
      Hdd += readlane_f(tHdd, src);
#pragma unroll
      for (int c = 0; c < 4; c++) Hcd[c] += readlane_f(tc[c], src);
    }
    if (lane == 0) {
      a.p_energy[p] = eSum;
      a.p_actmask[p] = (uint8_t)mask;
      if (mask == 0u) {
        a.p_HdiF[p] = 0.f;
        a.p_bdSumF[p] = 0.f;
      } else {
        // marginalization pass: priorF *= idepthFixPriorMargFac, the sums are the LF ones (AF = 0), and
        // AccumulatedSCHessianSSE::addPoint(p, shiftPriorToZero = false) (Src/EnergyFunctional.cpp:563,577)
        const float priorF = a.marg ? a.priorF[p] * a.margPriorFac : a.priorF[p];
        float Hh = a.marg ? (0.f + Hdd) + priorF : Hdd + 0.f + priorF;  // Hdd_accAF + Hdd_accLF + priorF
        if ((double)Hh < 1e-10) Hh = (float)1e-10;
        a.p_HdiF[p] = (float)(1.0 / (double)Hh);
        float bdSumF = a.marg ? 0.f + bd : bd + 0.f;
        if (!a.marg) bdSumF += priorF * (idep - idep0);
        a.p_bdSumF[p] = bdSumF;
      }
      if (a.marg)
        reinterpret_cast<float4*>(a.p_Hcd)[p] = make_float4(0.f + Hcd[0], 0.f + Hcd[1], 0.f + Hcd[2], 0.f + Hcd[3]);
      else
        reinterpret_cast<float4*>(a.p_Hcd)[p] = make_float4(Hcd[0] + 0.f, Hcd[1] + 0.f, Hcd[2] + 0.f, Hcd[3] + 0.f);
    }
  }
  HS_TRACE(a, 3);
}

// =====================================================================================================
// accumulate: (host i, target slot j, split s) blocks + energy / Hcc,bc / energy threshold blocks
// =====================================================================================================
namespace {
constexpr int ACC_TILE = 64;  // points per LDS tile (one wave does the order-preserving compaction)
// per-point LDS record: Jacobian digest of residual (p, j) | 1 | 0 | HdiF | bdSumF | Hcd | JpJdF of all slots
constexpr int R_ONE = 36, R_ZERO = 37, R_HDI = 38, R_BDS = 39, R_HCD = 40, R_JP = 44, R_N = 108;
struct AccLds {
  float rec[ACC_TILE][R_N];  // also the staging of the waves' partials (4 x HS_PART_N floats)
  unsigned char m[ACC_TILE];
  unsigned char list[ACC_TILE];
  int cnt;
  int wcnt[4][16];
};
static_assert(ACC_TILE * R_N >= 4 * HS_PART_N, "partial staging fits in the tile records");

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
  __shared__ double part[20][12];
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
  for (int e = 0; e < 20; e++) red[e][tid] = acc[e];
  __syncthreads();
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
    // accHcc into the calib block of H_sc, accbc into b_sc (stitchDoubleMT, Include/AccumulatedSCHessian.h:92-99)
    const int n = 4 + 8 * a.nF;
    if (tid < 16) atomicAdd(&a.stitch.HSC[(tid >> 2) * n + (tid & 3)], t);
    else atomicAdd(&a.stitch.bSC[tid - 16], t);
  }
}

// setNewFrameEnergyTH: k-th smallest candidate by a 4-pass radix select with a parallel bin scan.
// Candidates: one float per point and rank (-1 / negative = none); the ranks' arrays are all-gathered so
// every rank selects over the same union and computes the same threshold.
__device__ void acc_energy_th_block(const HsAccArgs& a) {
  __shared__ unsigned int hist[256], scan[256];
  __shared__ unsigned int s_prefix, s_mask, s_k, s_n;
  const int tid = threadIdx.x;
  if (tid == 0) {
    s_prefix = 0;
    s_mask = 0;
  }
  for (int pass = 0; pass < 4; pass++) {
    const int shift = 24 - 8 * pass;
    hist[tid] = 0;
    __syncthreads();
    const unsigned int prefix = s_prefix, mask = s_mask;
    const int total = a.nranks * a.stride;
    for (int i = tid; i < total; i += 256) {
      const unsigned int v = __float_as_uint(a.cand[i]);
      if (v < 0x80000000u && (v & mask) == prefix) atomicAdd(&hist[(v >> shift) & 255u], 1u);
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
    if (pass == 0 && tid == 0) {
      s_n = scan[255];
      s_k = (unsigned int)(int)(a.frameEnergyTHN * (float)scan[255]);
    }
    __syncthreads();
    if (s_n == 0) break;
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
    if (s_n == 0) {
      a.frameTH[a.newest] = 12 * 12 * 8;
    } else {
      const float nth = sqrtf(__uint_as_float(s_prefix));
      float th = nth * a.facMedian;
      th = 26.0f * a.constWeight + th * (1 - a.constWeight);
      th = th * th;
      th *= a.overallWeight * a.overallWeight;
      a.frameTH[a.newest] = th;
    }
  }
}

// operand offsets of one AccumulatorApprox entry evaluated as ((a*xc)*xr + (c*yc)*yr) + b*((xc*yr) + (yc*xr));
// TopRight (xr*T0 + yr*T1) and BotRight (v) are that expression with 1 / 0 operands (same rounding)
struct TopRole {
  int oa = R_ZERO, ob = R_ZERO, oc = R_ZERO, oxr = R_ZERO, oxc = R_ZERO, oyr = R_ZERO, oyc = R_ZERO;
  bool isData = false;
};
__device__ __forceinline__ TopRole top_role(int e) {
  TopRole t;
  if (e < 55) {
    int er = 0, ec = 0, idx = 0;
    for (int rr = 0; rr < 10; rr++)
      for (int cc = rr; cc < 10; cc++) {
        if (idx == e) { er = rr; ec = cc; }
        idx++;
      }
    t.isData = true;
    t.oa = HS_JR_JIDX2 + 0; t.ob = HS_JR_JIDX2 + 1; t.oc = HS_JR_JIDX2 + 2;
    t.oxr = HS_JR_X + er; t.oxc = HS_JR_X + ec; t.oyr = HS_JR_Y + er; t.oyc = HS_JR_Y + ec;
  } else if (e < 85) {
    const int er = (e - 55) / 3, ec = (e - 55) % 3;
    t.oa = ec == 0 ? HS_JR_JABJIDX + 0 : (ec == 1 ? HS_JR_JABJIDX + 2 : HS_JR_JIR + 0);
    t.oc = ec == 0 ? HS_JR_JABJIDX + 1 : (ec == 1 ? HS_JR_JABJIDX + 3 : HS_JR_JIR + 1);
    t.oxr = HS_JR_X + er; t.oyr = HS_JR_Y + er; t.oxc = R_ONE; t.oyc = R_ONE;
  } else if (e < HS_TOP_N) {
    const int ec = e - 85;
    t.oa = ec == 0 ? HS_JR_JAB2 + 0
         : ec == 1 ? HS_JR_JAB2 + 1
         : ec == 2 ? HS_JR_JABR + 0
         : ec == 3 ? HS_JR_JAB2 + 2
         : ec == 4 ? HS_JR_JABR + 1 : HS_JR_RR;
    t.oxr = t.oxc = t.oyr = t.oyc = R_ONE;
  }
  return t;
}
struct AccOps {
  float t0[7], t1[7];  // top entry operands (lane, 64 + lane)
  float hdi, wj, x[HS_MAXF];  // accD: HdiF, JpJdF[j][dr], JpJdF[k][dc]
  float ex, ey;        // accE / accEB operands
  unsigned m;
};
}  // namespace

// Stages one tile of per-point records into LDS: all global loads are issued before any LDS store
// (clamped, always-valid addresses), then the order-preserving list of points active into j is built.
__device__ __forceinline__ void acc_load_tile(const HsAccArgs& a, AccLds& T, int t0, int tn, int j) {
  const int tid = threadIdx.x;
  const int qa0 = min((tid + 0) >> 4, tn - 1), qa1 = min((tid + 256) >> 4, tn - 1);
  const int qa2 = min((tid + 512) >> 4, tn - 1), qa3 = min((tid + 768) >> 4, tn - 1);
  const int w = tid & 15;
  const float4* jp = reinterpret_cast<const float4*>(a.JpJdF);
  const float4 j0 = jp[(size_t)(t0 + qa0) * 16 + w], j1 = jp[(size_t)(t0 + qa1) * 16 + w];
  const float4 j2 = jp[(size_t)(t0 + qa2) * 16 + w], j3 = jp[(size_t)(t0 + qa3) * 16 + w];
  constexpr int NW = HS_JREC / 4;
  const int r0 = tid, r1 = tid + 256, r2 = tid + 512;
  const float4* jr = reinterpret_cast<const float4*>(a.Jrec);
  const float4 k0 = jr[((size_t)(t0 + min(r0 / NW, tn - 1)) * 8 + j) * NW + r0 % NW];
  const float4 k1 = jr[((size_t)(t0 + min(r1 / NW, tn - 1)) * 8 + j) * NW + r1 % NW];
  const float4 k2 = jr[((size_t)(t0 + min(r2 / NW, tn - 1)) * 8 + j) * NW + r2 % NW];
  const int qs = min(tid, tn - 1);
  const unsigned char mk = a.actmask[t0 + qs];
  const float4 hcd = reinterpret_cast<const float4*>(a.Hcd)[t0 + qs];
  const float hdi = a.HdiF[t0 + qs], bds = a.bdSumF[t0 + qs];
  __syncthreads();  // the previous tile's records are no longer read
  // rows >= tn receive copies of the last point; they are never listed
  *reinterpret_cast<float4*>(&T.rec[(tid + 0) >> 4][R_JP + 4 * w]) = j0;
  *reinterpret_cast<float4*>(&T.rec[(tid + 256) >> 4][R_JP + 4 * w]) = j1;
  *reinterpret_cast<float4*>(&T.rec[(tid + 512) >> 4][R_JP + 4 * w]) = j2;
  *reinterpret_cast<float4*>(&T.rec[(tid + 768) >> 4][R_JP + 4 * w]) = j3;
  *reinterpret_cast<float4*>(&T.rec[r0 / NW][4 * (r0 % NW)]) = k0;
  *reinterpret_cast<float4*>(&T.rec[r1 / NW][4 * (r1 % NW)]) = k1;
  if (r2 < ACC_TILE * NW) *reinterpret_cast<float4*>(&T.rec[r2 / NW][4 * (r2 % NW)]) = k2;
  if (tid < ACC_TILE) {
    T.m[tid] = mk;
    *reinterpret_cast<float4*>(&T.rec[tid][R_HCD]) = hcd;
    T.rec[tid][R_HDI] = hdi;
    T.rec[tid][R_BDS] = bds;
    T.rec[tid][R_ONE] = 1.0f;
    T.rec[tid][R_ZERO] = 0.0f;
    const bool act = tid < tn && ((mk >> j) & 1u);
    const unsigned long long bal = __ballot(act);
    if (act) T.list[__popcll(bal & ((1ull << tid) - 1ull))] = (unsigned char)tid;
    if (tid == 0) T.cnt = __popcll(bal);
  }
  __syncthreads();
}

// One (host i, target j, split s) accumulator block.  kBlocked: the reference's 1k/1m flush blocking is
// emulated (needed when a block sums more than 1000 updates; below that shiftUp never fires and
// finish() returns the plain running sum, so the counters are dropped).
// One (host i, target j, split s) block: its 4 waves each accumulate a contiguous share of the split's
// points (a.W = 1: wave 0 takes all of them, i.e. the single-thread reference order) and write one partial
// each.  Lane roles: top entries lane / 64+lane, accD (j, k=0..7)[lane>>3][lane&7], accE / accEB lane < 40.
// kBlocked: the reference's 1k/1m flush blocking is emulated (needed above 1000 updates per partial;
// below that shiftUp never fires and finish() is the plain running sum, so the counters are dropped).
template <bool kBlocked>
__device__ __forceinline__ void acc_pair_block(const HsAccArgs& a, AccLds& T) {
  const int nF = a.nF, S = a.S, W = a.W;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int b = blockIdx.x;
  const int ij = b / S, s = b % S;
  const int i = ij % nF, j = ij / nF;  // host i, target j (accumulator index i + nF*j)
  const int hb = a.host_pt_begin[i], he = a.host_pt_begin[i + 1];
  const int span = he - hb;
  const int pb = hb + (int)((long long)span * s / S), pe = hb + (int)((long long)span * (s + 1) / S);

  const TopRole r0 = top_role(lane), r1 = top_role(64 + lane);
  const int dr = lane >> 3, dc = lane & 7;
  const int owj = R_JP + j * 8 + dr;
  int oex = R_ZERO, oey = R_ZERO;
  if (lane < 32) { oex = R_JP + j * 8 + (lane >> 2); oey = R_HCD + (lane & 3); }
  else if (lane < 40) { oex = R_BDS; oey = R_JP + j * 8 + (lane - 32); }

  Blk top0, top1, d[HS_MAXF], ex;
  BlkCnt ctop, cd[HS_MAXF], cex;
  int nTop = 0, nD[HS_MAXF];
#pragma unroll
  for (int k = 0; k < HS_MAXF; k++) nD[k] = 0;

  auto load = [&](int q, AccOps& o) {
    const float* R = T.rec[q];
    o.t0[0] = R[r0.oa]; o.t0[1] = R[r0.ob]; o.t0[2] = R[r0.oc]; o.t0[3] = R[r0.oxr]; o.t0[4] = R[r0.oxc];
    o.t0[5] = R[r0.oyr]; o.t0[6] = R[r0.oyc];
    o.t1[0] = R[r1.oa]; o.t1[1] = R[r1.ob]; o.t1[2] = R[r1.oc]; o.t1[3] = R[r1.oxr]; o.t1[4] = R[r1.oxc];
    o.t1[5] = R[r1.oyr]; o.t1[6] = R[r1.oyc];
    o.hdi = R[R_HDI]; o.wj = R[owj];
#pragma unroll
    for (int k = 0; k < HS_MAXF; k++) o.x[k] = R[R_JP + k * 8 + dc];
    o.ex = R[oex]; o.ey = R[oey];
    o.m = T.m[q];
  };
  auto topv = [](const float* t) {  // a b c xr xc yr yc
    return ((t[0] * t[4]) * t[3] + (t[2] * t[6]) * t[5]) + t[1] * ((t[4] * t[5]) + (t[6] * t[3]));
  };

  for (int t0 = pb; t0 < pe; t0 += ACC_TILE) {
    const int tn = min(ACC_TILE, pe - t0);
    acc_load_tile(a, T, t0, tn, j);
    HS_TRACE(a, 2);
    const int cnt = T.cnt;
    const int c0 = wv < W ? (cnt * wv) / W : cnt, c1 = wv < W ? (cnt * (wv + 1)) / W : cnt;
    AccOps nx;
    if (c0 < c1) load(T.list[c0], nx);
    for (int c = c0; c < c1; c++) {
      const AccOps o = nx;
      if (c + 1 < c1) load(T.list[c + 1], nx);
      // ---- AccumulatedTopHessianSSE::addPoint<0>: update() adds Data then shiftUp; BotRight / TopRight after
      const float u0 = topv(o.t0), u1 = topv(o.t1);
      const float wl = o.hdi * o.wj;
      if (kBlocked) {
        const int f = ctop.bump();
        if (r0.isData) top0.A += u0;
        if (r1.isData) top1.A += u1;
        if (f) { top0.flush(f); top1.flush(f); }
        if (!r0.isData) top0.A += u0;
        if (!r1.isData) top1.A += u1;
#pragma unroll
        for (int k = 0; k < HS_MAXF; k++)
          if ((o.m >> k) & 1u) {  // wave-uniform
            d[k].A += wl * o.x[k];
            d[k].flush(cd[k].bump());
          }
        ex.A += (o.hdi * o.ex) * o.ey;
        ex.flush(cex.bump());
      } else {
        top0.A += u0;
        top1.A += u1;
#pragma unroll
        for (int k = 0; k < HS_MAXF; k++) {
          const bool bk = (o.m >> k) & 1u;
          d[k].A = bk ? d[k].A + wl * o.x[k] : d[k].A;
          nD[k] += bk ? 1 : 0;
        }
        ex.A += (o.hdi * o.ex) * o.ey;
        nTop++;
      }
    }
  }
  HS_TRACE(a, 1);
  // the waves' partials are combined in wave order in fp64 (the reference sums its per-thread fp32
  // accumulators in fp64) into one partial of this split
  __syncthreads();  // tile records are no longer read
  float* stage = &T.rec[0][0];
  if (wv < W) {
    float* Ps = stage + wv * HS_PART_N;
    // finish(): A1m = (A1k + A) + A1m  (== A when nothing was flushed)
    Ps[lane] = top0.finish();
    if (64 + lane < 96) Ps[64 + lane] = 64 + lane < HS_TOP_N ? top1.finish() : 0.f;
#pragma unroll
    for (int k = 0; k < HS_MAXF; k++) Ps[96 + k * 64 + lane] = d[k].finish();
    if (lane < 40) Ps[96 + 512 + lane] = ex.finish();
    if (lane == 0) {
      T.wcnt[wv][0] = kBlocked ? ctop.total() : nTop;
      T.wcnt[wv][9] = kBlocked ? cex.total() : nTop;
    }
    if (lane < HS_MAXF) {
      int v = 0;
#pragma unroll
      for (int k = 0; k < HS_MAXF; k++) v = k == lane ? (kBlocked ? cd[k].total() : nD[k]) : v;
      T.wcnt[wv][1 + lane] = v;
    }
  }
  __syncthreads();
  double* P = a.part + ((size_t)ij * S + s) * HS_PART_N;
  int* PC = a.part_cnt + ((size_t)ij * S + s) * 16;
  // the partial is handed to the pair's stitching block (hs_k_accumulate): sc1 (write-through) stores
  for (int e = tid; e < HS_PART_N; e += 256) {
    double sum = 0.0;
    for (int w = 0; w < W; w++) sum += (double)stage[w * HS_PART_N + e];
    __hip_atomic_store(&P[e], sum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (tid < 10) {
    int c = 0;
    for (int w = 0; w < W; w++) c += T.wcnt[w][tid];
    __hip_atomic_store(&PC[tid], c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__device__ void stitch_pair(const HsStitchArgs& a, int ij, long long* trace);

// agent-scope relaxed load = global_load ... sc1 (bypasses this CU's L1; the L2 line of a write-through
// sc1 store is dropped, so the load is served from memory side)
template <typename T>
__device__ __forceinline__ T ld_sc1(const T* p) {
  return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(256) void hs_k_accumulate(HsAccArgs a) {
  const int nb = a.nF * a.nF * a.S;
  const int b = blockIdx.x;
  HS_TRACE(a, 0);
  if (b == nb) { acc_energy_block(a); HS_TRACE(a, 15); return; }
  if (b == nb + 1) { acc_hcc_block(a); HS_TRACE(a, 15); return; }
  if (b == nb + 2) {
    if (!a.skip_threshold) acc_energy_th_block(a);
    HS_TRACE(a, 15);
    return;
  }
  __shared__ AccLds T;
  __shared__ int s_last;
  if (a.blocked) acc_pair_block<true>(a, T);
  else acc_pair_block<false>(a, T);
  HS_TRACE(a, 11);
  // hand-off to the pair's stitch (MI355X_MICROARCH.md "Valid forms", counter row; cdna_hip_programming.md
  // §6 Guideline 16): the partial was stored sc1 (write-through, no L2 write-back fence needed); every
  // storing wave drains its stores, then after a barrier ONE lane adds to the pair's ticket; the block
  // whose add returns S - 1 (the last) stitches the pair with sc1 loads of the partials.  No block waits
  // on another (no spin), so any dispatch order and XCD placement is safe.
  const int ij = b / a.S;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    s_last = __hip_atomic_fetch_add(&a.ticket[ij], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == a.S - 1;
  __syncthreads();
  if (s_last) {
    stitch_pair(a.stitch, ij, a.trace ? a.trace + (size_t)blockIdx.x * 16 : nullptr);
    if (threadIdx.x == 0)  // ready for the next launch (the kernel boundary orders it)
      __hip_atomic_store(&a.ticket[ij], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  HS_TRACE(a, 15);
}

// =====================================================================================================
// stitch (fp64): one block (64 threads) per (host i, target j)
// =====================================================================================================
namespace {
// index of (r, c) in the 10x10 upper-triangle Data block
__device__ __forceinline__ int tri_idx(int r, int c) {
  const int lo = r < c ? r : c, hi = r < c ? c : r;
  return lo * 10 - (lo * (lo - 1)) / 2 + (hi - lo);
}
}  // namespace

// lane (r, c) of one wave: X(r, c) = sum_l PH(r, l) M(l, c) and Y(r, c) = sum_l PT(r, l) M(l, c) (rows r of PH / PT
// in registers), in l order as the reference's 8x8 products; staged to the wave's LDS scratch tx / ty
__device__ __forceinline__ void left2(const double ph[8], const double pt[8], const double* M, double* tx, double* ty,
                                      int lane) {
  const int c = lane & 7;
  double x = 0.0, y = 0.0;
#pragma unroll
  for (int l = 0; l < 8; l++) {
    const double m = M[l * 8 + c];
    x += ph[l] * m;
    y += pt[l] * m;
  }
  tx[lane] = x;
  ty[lane] = y;
}
// out(r, c) = sum_l T(r, l) B(c, l): the right product of a sandwich (T staged by left2)
__device__ __forceinline__ double right_t(const double* T, const double* B, int lane) {
  const int r = lane >> 3, c = lane & 7;
  double o = 0.0;
#pragma unroll
  for (int l = 0; l < 8; l++) o += T[r * 8 + l] * B[c * 8 + l];
  return o;
}

// stitch of one (host i, target j) pair by a 256-thread block (4 waves): fp64 sum of the split partials,
// then the top block (wave 0), the Schur rows (i, j, k) for k = wave, wave+4 (all waves) and the calib / b
// parts, atomically added into HA / bA / HSC / bSC.  trace: the block's checkpoint row (slots 12 / 14).
__device__ void stitch_pair(const HsStitchArgs& a, int ij, long long* trace) {
  const int nF = a.nF, S = a.S;
  const int i = ij % nF, j = ij / nF;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int n = 4 + 8 * nF;
  const int iIdx = 4 + 8 * i, jIdx = 4 + 8 * j;
  __shared__ double E[HS_PART_N];  // summed partial: top 96 | D 8x64 | E 32 | EB 8
  __shared__ double A88[64], A84[32], a8r[8], aH[64], aT[64];
  __shared__ double aH2[HS_MAXF][64], aT2[HS_MAXF][64], tmpw[4][128];
  __shared__ int cnt[16];
  // ---- everything this pair needs, all loads in flight together
  const double* P0 = a.part + (size_t)ij * S * HS_PART_N;
  const int* C0 = a.part_cnt + (size_t)ij * S * 16;
  if (tid < 64) {
    aH[tid] = a.adHost[ij * 64 + tid];
    aT[tid] = a.adTarget[ij * 64 + tid];
  }
#pragma unroll
  for (int u = 0; u < 4; u++) {  // adjoints of (i, k) for all k: 2 * 8 * 64 values
    const int q = tid + 256 * u, kk = q >> 7, w = q & 127;
    const int kc = min(kk, nF - 1);
    const double v = (w < 64 ? a.adHost : a.adTarget)[(i + nF * kc) * 64 + (w & 63)];
    if (kk < nF) (w < 64 ? aH2[kk] : aT2[kk])[w & 63] = v;
  }
  // split partials summed in fp64 in split order (stitchDoubleInternal: accH += acc[tid2].H.cast<double>()
  // for num > 0; a split with num == 0 made no update, so its partial is exactly +0 and adding it is the
  // same as skipping it).  sc1 loads (the partials were handed off without an acquire fence), four splits
  // per batch so the loads of a batch are in flight together.
  double sum[3] = {0.0, 0.0, 0.0};
  int csum = 0;
  for (int s0 = 0; s0 < S; s0 += 4) {
    double v[4][3];
    int cv[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int sq = min(s0 + q, S - 1);
      const double* Ps = P0 + (size_t)sq * HS_PART_N;
#pragma unroll
      for (int u = 0; u < 3; u++) v[q][u] = ld_sc1(&Ps[min(tid + 256 * u, HS_PART_N - 1)]);
      cv[q] = ld_sc1(&C0[sq * 16 + (tid & 15)]);
    }
#pragma unroll
    for (int q = 0; q < 4; q++)
      if (s0 + q < S) {
#pragma unroll
        for (int u = 0; u < 3; u++) sum[u] += v[q][u];
        csum += cv[q];
      }
  }
#pragma unroll
  for (int u = 0; u < 3; u++)
    if (tid + 256 * u < HS_PART_N) E[tid + 256 * u] = sum[u];
  if (tid < 16) cnt[tid] = csum;
  __syncthreads();
  if (trace && tid == 0) trace[12] = wall_clock64();
  const double* e = E;
  const double* Hpc = E + 96 + 512;
  const double* v8 = E + 96 + 512 + 32;
  const int r = lane >> 3, c = lane & 7;
  double* tmp = tmpw[wv];
  double ahr[8], atr[8];  // this lane's rows r of the adjoints, in registers for every left product
#pragma unroll
  for (int l = 0; l < 8; l++) {
    ahr[l] = aH[r * 8 + l];
    atr[l] = aT[r * 8 + l];
  }
  if (wv == 0 && cnt[0] > 0) {  // top block: AccumulatorApprox::finish -> 13x13 [calib4|xi6|a|b|r]
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
    A88[lane] = v;
    if (lane < 32) {  // A84 = H[4+r][c]
      const int rr = lane >> 2, cc = lane & 3;
      const int RR = 4 + rr;
      A84[lane] = RR < 10 ? e[tri_idx(cc, RR)] : e[55 + 3 * cc + (RR - 10)];
    }
    if (lane < 8) {  // a8r = H[4+r][12]
      const int RR = 4 + lane;
      a8r[lane] = RR < 10 ? e[55 + 3 * RR + 2] : (RR == 10 ? e[85 + 2] : e[85 + 4]);
    }
    __builtin_amdgcn_wave_barrier();
    // aH A aH^T, aT A aT^T, aH A aT^T: the two left products once, then three right products
    left2(ahr, atr, A88, tmp, tmp + 64, lane);
    __builtin_amdgcn_wave_barrier();
    const double o1 = right_t(tmp, aH, lane), o2 = right_t(tmp + 64, aT, lane), o3 = right_t(tmp, aT, lane);
    __builtin_amdgcn_wave_barrier();
    atomicAdd(&a.HA[(iIdx + r) * n + iIdx + c], o1);
    atomicAdd(&a.HA[(jIdx + r) * n + jIdx + c], o2);
    atomicAdd(&a.HA[(iIdx + r) * n + jIdx + c], o3);
    if (lane < 32) {
      const int rr = lane >> 2, cc = lane & 3;
      double s1 = 0.0, s2 = 0.0;
      for (int l = 0; l < 8; l++) {
        s1 += aH[rr * 8 + l] * A84[l * 4 + cc];
        s2 += aT[rr * 8 + l] * A84[l * 4 + cc];
      }
      atomicAdd(&a.HA[(iIdx + rr) * n + cc], s1);
      atomicAdd(&a.HA[(jIdx + rr) * n + cc], s2);
    }
    if (lane < 16) atomicAdd(&a.HA[(lane >> 2) * n + (lane & 3)], e[tri_idx(lane >> 2, lane & 3)]);
    if (lane < 8) {
      double s1 = 0.0, s2 = 0.0;
      for (int l = 0; l < 8; l++) {
        s1 += aH[lane * 8 + l] * a8r[l];
        s2 += aT[lane * 8 + l] * a8r[l];
      }
      atomicAdd(&a.bA[iIdx + lane], s1);
      atomicAdd(&a.bA[jIdx + lane], s2);
    }
    if (lane < 4) atomicAdd(&a.bA[lane], e[55 + 3 * lane + 2]);
  }
  if (wv == 1) {  // Schur calib columns and b: adH/adT * accE, * accEB
    if (lane < 32) {
      const int rr = lane >> 2, cc = lane & 3;
      double s1 = 0.0, s2 = 0.0;
      for (int l = 0; l < 8; l++) {
        s1 += aH[rr * 8 + l] * Hpc[l * 4 + cc];
        s2 += aT[rr * 8 + l] * Hpc[l * 4 + cc];
      }
      atomicAdd(&a.HSC[(iIdx + rr) * n + cc], s1);
      atomicAdd(&a.HSC[(jIdx + rr) * n + cc], s2);
    }
    if (lane < 8) {
      double s1 = 0.0, s2 = 0.0;
      for (int l = 0; l < 8; l++) {
        s1 += aH[lane * 8 + l] * v8[l];
        s2 += aT[lane * 8 + l] * v8[l];
      }
      atomicAdd(&a.bSC[iIdx + lane], s1);
      atomicAdd(&a.bSC[jIdx + lane], s2);
    }
  }
  for (int kk = wv; kk < nF; kk += 4) {  // Schur rows (i, j, k)
    if (cnt[1 + kk] == 0) continue;  // accD num == 0
    const int kIdx = 4 + 8 * kk;
    const double* D = E + 96 + kk * 64;
    // X = aH D, Y = aT D once; X aH2^T, Y aT2^T, Y aH2^T, X aT2^T (the reference's four sandwiches)
    left2(ahr, atr, D, tmp, tmp + 64, lane);
    __builtin_amdgcn_wave_barrier();
    const double o1 = right_t(tmp, aH2[kk], lane), o2 = right_t(tmp + 64, aT2[kk], lane);
    const double o3 = right_t(tmp + 64, aH2[kk], lane), o4 = right_t(tmp, aT2[kk], lane);
    __builtin_amdgcn_wave_barrier();
    atomicAdd(&a.HSC[(iIdx + r) * n + iIdx + c], o1);
    atomicAdd(&a.HSC[(jIdx + r) * n + kIdx + c], o2);
    atomicAdd(&a.HSC[(jIdx + r) * n + iIdx + c], o3);
    atomicAdd(&a.HSC[(iIdx + r) * n + kIdx + c], o4);
  }
  if (trace && tid == 0) trace[14] = wall_clock64();
}

// =====================================================================================================
// solve + step (fp64), one workgroup of 256 threads
// =====================================================================================================
namespace {
constexpr int SOLVE_NT = HS_SOLVE_NT;  // 4 waves, one per SIMD: one lower-triangle 4x4 tile per lane in the LDLT
constexpr int SOLVE_NU = (HS_MAXDIM * HS_MAXDIM + SOLVE_NT - 1) / SOLVE_NT;  // matrix entries per thread

__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), lane);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
}  // namespace


// Solves (L D L^T) y = z in place for the permuted, scaled system of one GN step (n = 4 + 8 nF, a multiple
// of 4): right-looking LDLT in 4-column blocks with one-block look-ahead, ONE workgroup barrier per block.
//  wave 0 (the panel wave): in phase k it applies block k's rank-4 update to the rows of column block
//    k + 1 (one row per lane), takes the updated 4x4 diagonal block from lanes 0-3 (readlane), factors it
//    uniformly, reduces its row to the (L D) / L entries of panel k + 1 and carries the forward substitution;
//  waves 1-3: every lower 4x4 tile right of the next panel (register-resident, one per lane) takes block
//    k's rank-4 update; the owners of column block k + 2 publish it for the panel wave's next phase.
// The panel chain (the critical path) thus overlaps the trailing update.  fp64 throughout, FMA-contracted,
// reciprocals by v_rcp_f64 + 2 Newton steps: the solve is checked against the oracle's Eigen-order LDLT by
// tolerance (the LDLT is parity-unpinned), not bitwise.  The pivot order is applied by the
// caller.  Then D^-1 and the backward substitution (one wave, 4x4 diagonal blocks solved uniformly).
//   M  : the permuted system (row-major, stride n), read only
//   LT : L transposed, LT[i * LSTR + k] = L(k, i); MUST be zero on entry (its upper part stays zero)
//   W  : scratch of 26 * HS_MAXDIM doubles;  yv : right-hand side in, solution out
constexpr int LSTR = HS_MAXDIM + 1;  // padded row stride of LT

// 1/d: v_rcp_f64 (~2^-26 relative) refined by ONE Newton step (~2^-50, 4e-15 relative) -- the pivots' error
// then sits ~1e11 below the 1e-3 tolerance on x, and the LDLT's critical path is 68 reciprocals long;
// 0 for a (near-)zero pivot
__device__ __forceinline__ double rcp_f64(double d) {
  double r = __builtin_amdgcn_rcp(d);
  const double e = __builtin_fma(-d, r, 1.0);
  r = __builtin_fma(r, e, r);
  return fabs(d) > DBL_MIN ? r : 0.0;
}

// The panel's uniform factors: pivots d, their reciprocals, the partially reduced diagonal-block entries
// q(jp, j) (after the columns < j) and the substituted right-hand side yd of the 4 diagonal rows.
struct Panel4 {
  double d[4], dinv[4], q[4][4], yd[4];
};
struct PanelOut {
  double lw[4], ls[4], yr;
};
// wave-cooperative panel factorization: lane l holds row K0 + l (lanes 0-3: the diagonal block's rows), a =
// its entries of the panel columns, yr its rhs; every lane of the wave executes this.  Column by column: the
// pivot and the reduced entries come from lanes 0-3 by readlane, so the critical path per column is one
// readlane, one reciprocal and one multiply-add.  A diagonal row l takes L entries only for j < l.
__device__ __forceinline__ void panel_coop(const double a[4], double yr, int l, Panel4& P, PanelOut& o) {
  double pr[4] = {a[0], a[1], a[2], a[3]};
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const double d = readlane_f64(pr[j], j);
    const double dinv = rcp_f64(d);
    const double ydj = readlane_f64(yr, j);
    P.d[j] = d;
    P.dinv[j] = dinv;
    P.yd[j] = ydj;
#pragma unroll
    for (int jp = j + 1; jp < 4; jp++) P.q[jp][j] = readlane_f64(pr[j], jp);
    const double lj = pr[j] * dinv;
    o.lw[j] = l > j ? pr[j] : 0.0;
    o.ls[j] = l > j ? lj : 0.0;
#pragma unroll
    for (int jp = j + 1; jp < 4; jp++) pr[jp] = __builtin_fma(-o.ls[j], P.q[jp][j], pr[jp]);
    yr = __builtin_fma(-o.ls[j], ydj, yr);
  }
  o.yr = yr;
}
// a further (non-diagonal) row with the panel's factors: the same operations as panel_coop's lanes l >= 4
__device__ __forceinline__ void panel_row_uniform(const double a[4], double yr, const Panel4& P, PanelOut& o) {
  double pr[4] = {a[0], a[1], a[2], a[3]};
#pragma unroll
  for (int j = 0; j < 4; j++) {
    o.lw[j] = pr[j];
    o.ls[j] = pr[j] * P.dinv[j];
#pragma unroll
    for (int jp = j + 1; jp < 4; jp++) pr[jp] = __builtin_fma(-o.ls[j], P.q[jp][j], pr[jp]);
    yr = __builtin_fma(-o.ls[j], P.yd[j], yr);
  }
  o.yr = yr;
}

// publishes one panel row r (l = r - K0): LW / LS (zero for the diagonal rows, which take no part in the
// trailing update), its L entries, and the substituted rhs; lane j < 4 also stores pivot j
__device__ __forceinline__ void panel_row_store(const PanelOut& o, const Panel4& P, int r, int l, int K0, double* LWn,
                                                double* LSn, double* LT, double* Dv, double* yf, double* yv) {
  constexpr int MD = HS_MAXDIM;
  const bool diag = l < 4;
#pragma unroll
  for (int j = 0; j < 4; j++) {
    LWn[j * MD + r] = diag ? 0.0 : o.lw[j];
    LSn[j * MD + r] = diag ? 0.0 : o.ls[j];
    LT[(K0 + j) * LSTR + r] = o.ls[j];  // zero on and above the diagonal
  }
  if (diag) {
    Dv[r] = l == 0 ? P.d[0] : l == 1 ? P.d[1] : l == 2 ? P.d[2] : P.d[3];
    yf[r] = o.yr;
  } else {
    yv[r] = o.yr;
  }
}

__device__ __forceinline__ void ldlt_solve_blocked(const double* M, double* LT, double* W, double* yv, int n, int tid,
                                                   long long* trace) {
  constexpr int MD = HS_MAXDIM;
  static_assert((HS_MAXDIM / 4 - 2) * (HS_MAXDIM / 4 - 1) / 2 <= SOLVE_NT - 64, "one trailing tile per lane");
  const int nb = n >> 2;
  double* PBq = W;            // [2][4][MD] column block k+1 before block k's update, column-major
  double* LWb = W + 8 * MD;   // [2][4][MD] (L D) of panel k
  double* LSb = W + 16 * MD;  // [2][4][MD] L of panel k
  double* Dv = W + 24 * MD;   // [MD] pivots
  double* yf = W + 25 * MD;   // [MD] forward-substituted rhs of the diagonal rows
  const bool pw = tid < 64;   // the panel wave
  // waves 1-3: trailing tile (tr, tc), tc >= 2, row-major over the lower triangle
  const int u = tid - 64;
  int trp = 0;
  while ((trp + 1) * (trp + 2) / 2 <= u) trp++;
  const int tr = 2 + trp, tc = 2 + (u - trp * (trp + 1) / 2);
  const bool tile = !pw && tr < nb;
  double v[4][4];
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int c = 0; c < 4; c++) v[i][c] = tile ? M[(4 * tr + i) * n + 4 * tc + c] : 0.0;
  if (tid < n)
#pragma unroll
    for (int c = 0; c < 4; c++) PBq[4 * MD + c * MD + tid] = M[tid * n + 4 + c];  // column block 1
  // prologue: panel 0 over rows 0 .. n-1 by the panel wave (lanes 0-3 also take rows 64 .. n-1)
  if (pw) {
    const int r = min(tid, n - 1);
    double a4[4];
#pragma unroll
    for (int c = 0; c < 4; c++) a4[c] = M[r * n + c];
    Panel4 P;
    PanelOut o;
    panel_coop(a4, yv[r], tid, P, o);
    if (tid < n) panel_row_store(o, P, tid, tid, 0, LWb, LSb, LT, Dv, yf, yv);
    if (tid + 64 < n) {
      const int r2 = tid + 64;
#pragma unroll
      for (int c = 0; c < 4; c++) a4[c] = M[r2 * n + c];
      panel_row_uniform(a4, yv[r2], P, o);
      panel_row_store(o, P, r2, r2, 0, LWb, LSb, LT, Dv, yf, yv);
    }
  }
  __syncthreads();
  for (int k = 0; k + 1 < nb; k++) {
    const int K0 = 4 * (k + 1);
    const double* LWk = LWb + (k & 1) * 4 * MD;
    const double* LSk = LSb + (k & 1) * 4 * MD;
    if (trace && tid == 0 && k == 4) trace[16] = clock64();
    if (pw) {  // panel k+1: row r = K0 + lane
      const int l = tid, r = min(K0 + l, n - 1);
      const double* PBc = PBq + ((k + 1) & 1) * 4 * MD;
      double a4[4], lwk[4], lsd[4][4];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        a4[j] = PBc[j * MD + r];
        lwk[j] = LWk[j * MD + r];
#pragma unroll
        for (int c = 0; c < 4; c++) lsd[c][j] = LSk[j * MD + K0 + c];
      }
      const double yr = yv[r];
#pragma unroll
      for (int j = 0; j < 4; j++)  // block k's update of this row of column block k+1
#pragma unroll
        for (int c = 0; c < 4; c++) a4[c] = __builtin_fma(-lwk[j], lsd[c][j], a4[c]);
      Panel4 P;
      PanelOut o;
      panel_coop(a4, yr, l, P, o);
      if (K0 + l < n)
        panel_row_store(o, P, r, l, K0, LWb + ((k + 1) & 1) * 4 * MD, LSb + ((k + 1) & 1) * 4 * MD, LT, Dv, yf, yv);
      if (trace && tid == 0 && k == 4) trace[17] = clock64();
    } else if (tile && tc >= k + 2) {  // block k's rank-4 update of a trailing tile
      double lw[4][4], ls[4][4];
#pragma unroll
      for (int j = 0; j < 4; j++)
#pragma unroll
        for (int i = 0; i < 4; i++) {
          lw[i][j] = LWk[j * MD + 4 * tr + i];
          ls[i][j] = LSk[j * MD + 4 * tc + i];
        }
#pragma unroll
      for (int j = 0; j < 4; j++)
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
          for (int c = 0; c < 4; c++) v[i][c] = __builtin_fma(-lw[i][j], ls[c][j], v[i][c]);
      if (tc == k + 2) {
        double* PBn = PBq + (k & 1) * 4 * MD;
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
          for (int c = 0; c < 4; c++) PBn[c * MD + 4 * tr + i] = v[i][c];
      }
    }
    if (trace && tid == 64 && k == 4) trace[18] = clock64();
    __syncthreads();
    if (trace && tid == 0 && k == 4) trace[19] = clock64();
    if (trace && tid == 0 && k == 4) trace[12] = wall_clock64();
    if (trace && tid == 0 && k == 8) trace[14] = wall_clock64();  // mid-factorization checkpoint
  }
  // D^-1 z, then L^T x = D^-1 z by wave 0: lane i owns row i (< 64); rows 64 .. n-1 (at most the last block)
  // are solved uniformly first.  Per 4-row block the unknowns are solved uniformly from the block's diagonal
  // L entries, then every lane updates its row in decreasing k; LT is zero on and above the diagonal, so the
  // updates need no masks and a row of the block ends equal to its unknown.
  if (pw) {
    const int i = tid;
    const int ci = min(i, n - 1);
    double y = i < n ? yf[ci] * rcp_f64(Dv[ci]) : 0.0;
    int kb = nb - 1;
    if (n > 64) {  // the last block (rows 64 .. 67)
      const int k0 = 64;
      double x[4];
#pragma unroll
      for (int j = 3; j >= 0; j--) {
        double zz = yf[k0 + j] * rcp_f64(Dv[k0 + j]);
#pragma unroll
        for (int jj = 3; jj > j; jj--) zz = __builtin_fma(-LT[(k0 + j) * LSTR + k0 + jj], x[jj], zz);
        x[j] = zz;
      }
#pragma unroll
      for (int j = 3; j >= 0; j--) y = __builtin_fma(-LT[i * LSTR + k0 + j], x[j], y);
      if (i < 4) yv[k0 + i] = i == 0 ? x[0] : i == 1 ? x[1] : i == 2 ? x[2] : x[3];
      kb = 15;
    }
    for (; kb >= 0; kb--) {
      const int k0 = 4 * kb;
      double z[4], Li[4], Ld[4][4];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        z[j] = readlane_f64(y, k0 + j);
        Li[j] = LT[i * LSTR + k0 + j];
#pragma unroll
        for (int jj = j + 1; jj < 4; jj++) Ld[jj][j] = LT[(k0 + j) * LSTR + k0 + jj];
      }
      double x[4];
#pragma unroll
      for (int j = 3; j >= 0; j--) {
        double zz = z[j];
#pragma unroll
        for (int jj = 3; jj > j; jj--) zz = __builtin_fma(-Ld[jj][j], x[jj], zz);
        x[j] = zz;
      }
#pragma unroll
      for (int j = 3; j >= 0; j--) y = __builtin_fma(-Li[j], x[j], y);
    }
    if (i < n && i < 64) yv[i] = y;
    if (trace && tid == 0) trace[13] = wall_clock64();
  }
}

__global__ __launch_bounds__(SOLVE_NT) void hs_k_solve(HsSolveArgs a) {
  __shared__ double A[HS_MAXDIM * HS_MAXDIM];  // raw HA, then the scaled system, then LDLT scratch
  __shared__ double B[HS_MAXDIM * (HS_MAXDIM + 1)];  // raw HSC, then the permuted system, then L
  __shared__ double LT[HS_MAXDIM * (HS_MAXDIM + 1)];  // L^T of the factorization (zeroed at entry)
  __shared__ double Nf[2 * HS_MAXDIM * HS_NNS];  // nullspace factors N | Npi (prefetched at entry)
  __shared__ double tk[2 * HS_NNS];
  __shared__ double bf[HS_MAXDIM], Sv[HS_MAXDIM], xs[HS_MAXDIM], yv[HS_MAXDIM], px[HS_MAXDIM], dl[HS_MAXDIM];
  __shared__ double dgs[HS_MAXDIM];  // |diagonal| of the scaled system (pivot keys)
  __shared__ float xF[HS_MAXDIM];
  __shared__ double dgr[HS_MAXDIM];  // raw diagonal of the assembled system
  __shared__ int pos[HS_MAXDIM], rk[HS_MAXDIM];
  __shared__ int s_it;
  // the window state lives in LDS for the whole kernel: every field is touched by dependent scalar code
  // (steps, SE3 updates, precalc), which would otherwise pay a global-memory round trip per access
  __shared__ __align__(16) unsigned char st_raw[sizeof(HsDevState)];
  static_assert(sizeof(HsDevState) % 8 == 0, "HsDevState is copied as 8-byte words");
  HsDevState* st = reinterpret_cast<HsDevState*>(st_raw);
  const int tid = threadIdx.x, nt = SOLVE_NT;
  HS_TRACE(a, 0);
  if (a.trace && threadIdx.x == 0) a.trace[24] = clock64();  // shader clock (effective-clock probe)
  // entry prefetch: every global input (window state, systems, nullspace factors, b vectors, adjoints) is
  // requested into registers before the first LDS store, so the kernel pays ONE memory round trip here
  // instead of one per dependent load-store loop iteration
  constexpr int ST_WORDS = (int)(sizeof(HsDevState) / 8);
  constexpr int ST_NU = (ST_WORDS + SOLVE_NT - 1) / SOLVE_NT;
  constexpr int NF_NU = (2 * HS_MAXDIM * HS_NNS + SOLVE_NT - 1) / SOLVE_NT;
  const bool solve = (a.flags & HS_SOLVE) != 0;
  const int nF = a.nF, n = 4 + 8 * nF, nn = n * n;
  const unsigned inv_n = (unsigned)((0x100000000ull + n - 1) / n);  // idx / n == umulhi(idx, inv_n) for idx < n*n
  uint2 stw[ST_NU];
  {
    const uint2* gs = reinterpret_cast<const uint2*>(a.st);
#pragma unroll
    for (int u = 0; u < ST_NU; u++) stw[u] = gs[min(tid + u * SOLVE_NT, ST_WORDS - 1)];
  }
  double ha[SOLVE_NU], hs[SOLVE_NU], nfv[NF_NU];
  double bA_q = 0.0, bSC_q = 0.0, bM_q = 0.0;
  const double sysE0 = a.sysE[0], sysE1 = a.sysE[1], sysE2 = a.sysE[2];  // energy, sum |idepth|, #points
  if (solve) {
#pragma unroll
    for (int u = 0; u < SOLVE_NU; u++) {
      const int idx = min(tid + u * nt, nn - 1);
      ha[u] = a.HA[idx];
      hs[u] = a.HSC[idx];
    }
#pragma unroll
    for (int u = 0; u < NF_NU; u++) nfv[u] = a.Nproj[min(tid + u * SOLVE_NT, 2 * n * HS_NNS - 1)];
    if (tid < n) {
      bA_q = a.bA[tid];
      bSC_q = a.bSC[tid];
      bM_q = a.bM[tid];
    }
  }
  {
    uint2* ls = reinterpret_cast<uint2*>(st_raw);
#pragma unroll
    for (int u = 0; u < ST_NU; u++)
      if (tid + u * SOLVE_NT < ST_WORDS) ls[tid + u * SOLVE_NT] = stw[u];
  }
  if (solve) {
#pragma unroll
    for (int u = 0; u < NF_NU; u++)
      if (tid + u * SOLVE_NT < 2 * n * HS_NNS) Nf[tid + u * SOLVE_NT] = nfv[u];
  }
  __syncthreads();
  if (tid == 0) s_it = a.iteration >= 0 ? a.iteration : st->iteration;
  const double lambda = 1e-5;  // SOLVER_FIX_LAMBDA

  if (solve) {
    if (tid == 0 && a.energy_log) {
      a.energy_log[st->log_count] = sysE0;
      st->log_count = st->log_count + 1;
    }
#pragma unroll
    for (int u = 0; u < SOLVE_NU; u++)
      if (tid + u * nt < nn) {
        // raw HA -> B, raw HSC -> LT, both at the padded row stride n + 1 so the transposed reads of the
        // symmetrization below are (nearly) bank-conflict free; LT is cleared for the LDLT afterwards
        const int ix = tid + u * nt, r = (int)__umulhi((unsigned)ix, inv_n), c = ix - r * n;
        B[r * (n + 1) + c] = ha[u];
        LT[r * (n + 1) + c] = hs[u];
      }
    if (tid < n) {
      const int q = tid;
      dl[q] = q < 4 ? (double)(float)st->calib.value_minus_value_zero[q] : st->frames[(q - 4) / 8].delta[(q - 4) % 8];
      double bl, pr;
      if (q < 4) {
        pr = a.initialCalibHessian;
        bl = a.initialCalibHessian * dl[q];
      } else {
        const hs::FrameH& f = st->frames[(q - 4) / 8];
        pr = f.prior[(q - 4) % 8];
        bl = f.prior[(q - 4) % 8] * f.delta_prior[(q - 4) % 8];
      }
      px[q] = pr;  // HL diagonal (priors); staging only: these four arrays are reused below
      xs[q] = bl;
      yv[q] = bA_q;
      Sv[q] = bSC_q;
    }
    __syncthreads();
    HS_TRACE(a, 7);
    // HFinal = (HL + HM) + HA' ; diag *= (1+lambda) ; HFinal -= HSC' / (1+lambda)   (' = stitchDoubleMT
    // post-processing: frame off-diagonal blocks symmetrized, calib rows copied from the calib columns)
    const double sc = (double)(1.0f / (1 + lambda));
    double v[SOLVE_NU];
    // HM (the marginalization prior) is usually absent: two instances of the loop, chosen by one uniform
    // branch, so the common one carries no HM registers or loads
    auto assemble = [&](auto withHM) {
#pragma unroll
      for (int u = 0; u < SOLVE_NU; u++) {
        const int ix = min(tid + u * nt, nn - 1), r = (int)__umulhi((unsigned)ix, inv_n), c = ix - r * n;
        const int idx = r * (n + 1) + c, tdx = c * (n + 1) + r;
        const int fr = r < 4 ? -1 : (r - 4) >> 3, fc = c < 4 ? -1 : (c - 4) >> 3;
        const double a0 = B[idx], a1 = B[tdx], b0 = LT[idx], b1 = LT[tdx], hl0 = px[r];
        const double hm = decltype(withHM)::value ? a.HM[r * n + c] : 0.0;
        const bool sym = (fr >= 0) & (fc >= 0) & (fr != fc), calrow = (r < 4) & (c >= 4);
        const double ha_ = sym ? a0 + a1 : (calrow ? a1 : a0);
        const double hsc = calrow ? b1 : b0;
        const double hl = r == c ? hl0 : 0.0;
        double hv = (hl + hm) + ha_;
        hv = r == c ? hv * (1 + lambda) : hv;
        v[u] = hv - hsc * sc;
      }
    };
    if (a.HM) assemble(std::integral_constant<bool, true>{});
    else assemble(std::integral_constant<bool, false>{});
    if (tid < n) {
      const int q = tid;
      double hmd = 0.0;
      if (a.HM)
        for (int c = 0; c < n; c++) hmd += a.HM[q * n + c] * dl[c];
      // ((bL + (bM + HM delta)) + bA) - bSC
      bf[q] = ((xs[q] + (bM_q + hmd)) + yv[q]) - Sv[q];
    }
    // the diagonal of the assembled system (held in registers by its owners) is staged for the scaling
#pragma unroll
    for (int u = 0; u < SOLVE_NU; u++) {
      const int ix = tid + u * nt, r = (int)__umulhi((unsigned)ix, inv_n), c = ix - r * n;
      if (ix < nn && r == c) dgr[r] = v[u];
    }
    if (tid < HS_MAXDIM) rk[tid] = 0;
    __syncthreads();
    HS_TRACE(a, 8);
    for (int idx = tid; idx < HS_MAXDIM * (HS_MAXDIM + 1); idx += nt) LT[idx] = 0.0;  // L^T: zero on entry
    // scaling S = 1/sqrt(diag + 10); the pivot keys |S H S|_qq in the scaling's own operation order
    if (tid < n) {
      const double hqq = dgr[tid];
      const double sq = 1.0 / sqrt(hqq + 10);
      Sv[tid] = sq;
      dgs[tid] = fabs(sq * hqq * sq);
      bf[tid] = sq * bf[tid];
    }
    __syncthreads();
    HS_TRACE(a, 9);
    // the scaled system S H S, straight from the registers (no LDS round trip of the raw system)
#pragma unroll
    for (int u = 0; u < SOLVE_NU; u++) {  // all reads first (unconditional), then the predicated stores
      const int ix = min(tid + u * nt, nn - 1), r = (int)__umulhi((unsigned)ix, inv_n), c = ix - r * n;
      v[u] = Sv[r] * v[u] * Sv[c];
    }
#pragma unroll
    for (int u = 0; u < SOLVE_NU; u++)
      if (tid + u * nt < nn) A[tid + u * nt] = v[u];
    HS_TRACE(a, 10);
    // Pivot order: descending |diagonal| of the scaled system, Eigen's LDLT rule (left-looking: the largest
    // remaining |original diagonal| is the next pivot).  Exact ties are broken by the original index; Eigen
    // breaks them by the current position after its own swaps, which permutes tied rows only: x differs by
    // rounding, far inside the tolerance on x (the LDLT is parity-unpinned).  Ranks are counted
    // by all four waves (wave w compares against keys 17w .. 17w + 16) and combined with LDS atomics.
    {
      const int ln = tid & 63, w4 = __builtin_amdgcn_readfirstlane(tid >> 6);
      const int p0 = w4 * (HS_MAXDIM / 4), p1 = min(n, p0 + HS_MAXDIM / 4);
      double wk[HS_MAXDIM / 4];  // this wave's 17 keys: uniform LDS reads, all issued before any compare
#pragma unroll
      for (int q = 0; q < HS_MAXDIM / 4; q++) wk[q] = dgs[min(p0 + q, n - 1)];
#pragma unroll
      for (int half = 0; half < 2; half++) {
        const int e = ln + 64 * half;
        const double w0 = dgs[min(e, n - 1)];
        int cnt_ = 0;
#pragma unroll
        for (int q = 0; q < HS_MAXDIM / 4; q++) {  // branch-free (& / |, no short-circuit control flow)
          const int pp = p0 + q;
          cnt_ += (int)((pp < p1) & ((wk[q] > w0) | ((wk[q] == w0) & (pp < e))));
        }
        if (e < n) atomicAdd(&rk[e], cnt_);
      }
    }
    HS_TRACE(a, 11);
    __syncthreads();
    if (tid < n) pos[rk[tid]] = tid;
    __syncthreads();
    HS_TRACE(a, 1);
    // the permuted system P S H S P^T and right-hand side for the factorization
    {  // branch-free gather: all index and value reads first (clamped), then the predicated stores
      int pr_[SOLVE_NU], pc_[SOLVE_NU];
#pragma unroll
      for (int u = 0; u < SOLVE_NU; u++) {
        const int ix = min(tid + u * nt, nn - 1), r = (int)__umulhi((unsigned)ix, inv_n), c = ix - r * n;
        pr_[u] = pos[r];
        pc_[u] = pos[c];
      }
#pragma unroll
      for (int u = 0; u < SOLVE_NU; u++) v[u] = A[pr_[u] * n + pc_[u]];
#pragma unroll
      for (int u = 0; u < SOLVE_NU; u++)
        if (tid + u * nt < nn) B[tid + u * nt] = v[u];
    }
    if (tid < n) yv[tid] = bf[pos[tid]];
    __syncthreads();
    HS_TRACE(a, 2);
    ldlt_solve_blocked(B, LT, A, yv, n, tid, a.trace);
    __syncthreads();
    HS_TRACE(a, 3);
    if (tid < n) xs[pos[tid]] = Sv[pos[tid]] * yv[tid];
    __syncthreads();
    HS_TRACE(a, 4);
    // the fp32 adjoints for xAd: requested here so their latency overlaps orthogonalize (holding them in
    // registers across the LDLT costs 32 VGPRs of a kernel at the register limit)
    float adh[2][8], adt[2][8];
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const int o = min(tid + k * nt, nF * nF * 8 - 1);
      const int pair = o >> 3, c = o & 7, hh = pair / nF, tt = pair - hh * nF;
      const float* aHf = a.adHostF + (hh + nF * tt) * 64;
      const float* aTf = a.adTargetF + (hh + nF * tt) * 64;
#pragma unroll
      for (int rr = 0; rr < 8; rr++) {
        adh[k][rr] = aHf[rr * 8 + c];
        adt[k][rr] = aTf[rr * 8 + c];
      }
    }
    if (s_it >= 2) {  // SOLVER_ORTHOGONALIZE_X_LATER: x -= P x, P = (N Npi^T + Npi N^T) / 2 (orthogonalize)
      // t1 = Npi^T x, t2 = N^T x: 14 dot products over n, 4 lanes each
      const int d = tid >> 2, part = tid & 3, len = n >> 2;
      if (d < 2 * HS_NNS) {
        const double* col = Nf + (d < HS_NNS ? n * HS_NNS : 0);  // Npi for t1, N for t2
        const int kk = d % HS_NNS;
        double sacc = 0.0;
        for (int c = part * len; c < (part + 1) * len; c++) sacc = __builtin_fma(col[c * HS_NNS + kk], xs[c], sacc);
        sacc += __shfl_xor(sacc, 1);
        sacc += __shfl_xor(sacc, 2);
        if (part == 0) tk[d] = sacc;
      }
      __syncthreads();
      if (tid < n) {
        double s1 = 0.0, s2 = 0.0;
#pragma unroll
        for (int kk = 0; kk < HS_NNS; kk++) {
          s1 = __builtin_fma(Nf[tid * HS_NNS + kk], tk[kk], s1);
          s2 = __builtin_fma(Nf[n * HS_NNS + tid * HS_NNS + kk], tk[HS_NNS + kk], s2);
        }
        xs[tid] -= 0.5 * (s1 + s2);
      }
      __syncthreads();
    }
    // resubstituteF_MT: frame / calib steps, xAd, cstep
    if (tid < n) {
      const int q = tid;
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
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const int o = tid + k * nt;
      if (o < nF * nF * 8) {
        const int pair = o >> 3, hh = pair / nF, tt = pair - hh * nF;  // xAd[nF*h + t]
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int rr = 0; rr < 8; rr++) s1 += xF[4 + 8 * hh + rr] * adh[k][rr];
#pragma unroll
        for (int rr = 0; rr < 8; rr++) s2 += xF[4 + 8 * tt + rr] * adt[k][rr];
        a.xAd[o] = s1 + s2;
      }
    }
    // the consumed accumulation targets are zeroed for the next linearization (no barrier waits on these)
    for (int idx = tid; idx < nn; idx += nt) {
      a.HA[idx] = 0.0;
      a.HSC[idx] = 0.0;
    }
    if (tid < n) {
      a.bA[tid] = 0.0;
      a.bSC[tid] = 0.0;
    }
    HS_TRACE(a, 5);
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
    if (tid >= 64 && tid < 64 + nF) {
      hs::FrameH& f = st->frames[tid - 64];
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
    HS_TRACE(a, 6);
    for (int pr = tid; pr < nF * nF; pr += nt) {
      const int hh = pr / nF, tt = pr % nF;
      a.pre[pr] = hs::make_precalc(st->frames[hh], st->frames[tt], st->calib);
    }
    if (tid == 128) {
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
      const float sumNID = sysE2 > 0 ? (float)(sysE1 / sysE2) : 0.f;
      const float th = a.thOptIterations;
      st->canbreak = sqrtf(sumA) < 0.0005 * th && sqrtf(sumB) < 0.00005 * th && sqrtf(sumR) < 0.00005 * th &&
                     sqrtf(sumT) * sumNID < 0.00005 * th;
      st->iteration = s_it + 1;
    }
  }
  __syncthreads();
  {  // write the window state back
    const uint2* ls = reinterpret_cast<const uint2*>(st_raw);
    uint2* gs = reinterpret_cast<uint2*>(a.st);
    for (int i = tid; i < (int)(sizeof(HsDevState) / 8); i += nt) gs[i] = ls[i];
  }
  if (a.trace && threadIdx.x == 0) a.trace[25] = clock64();
  HS_TRACE(a, 15);
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
