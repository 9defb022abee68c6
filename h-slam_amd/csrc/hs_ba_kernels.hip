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
#include "hs_se3_dev.h"


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

// the same on the packed 12-byte (I, dx, dy) texels of an image slot (HsLinArgs.img3): the 2x2 taps span fewer
// cache lines than the float4 texels
__device__ __forceinline__ float3 interp33p(const float* __restrict__ img3, float x, float y, int w) {
  int ix = (int)x, iy = (int)y;
  float dx = x - ix, dy = y - iy, dxdy = dx * dy;
  const float* bp = img3 + 3 * (ix + iy * w);
  const float* bq = bp + 3 * w;
  const float3 p00 = make_float3(bp[0], bp[1], bp[2]), p10 = make_float3(bp[3], bp[4], bp[5]);
  const float3 p01 = make_float3(bq[0], bq[1], bq[2]), p11 = make_float3(bq[3], bq[4], bq[5]);
  const float w11 = dxdy, w01 = dy - dxdy, w10 = dx - dxdy, w00 = 1 - dx - dy + dxdy;
  float3 r;
  r.x = w11 * p11.x + w01 * p01.x + w10 * p10.x + w00 * p00.x;
  r.y = w11 * p11.y + w01 * p01.y + w10 * p10.y + w00 * p00.y;
  r.z = w11 * p11.z + w01 * p01.z + w10 * p10.z + w00 * p00.z;
  return r;
}
#ifndef LIN_ONE_PATH
#define LIN_ONE_PATH 1
#endif
#ifndef LIN_TEXEL12
#define LIN_TEXEL12 1  // hs_k_lin's taps from the packed 12-byte texels
#endif

// wall-clock checkpoint of a block (thread 0) when tracing is enabled
#define HS_TRACE(A, slot)                                                                          \
  do {                                                                                             \
    if ((A).trace && threadIdx.x == 0) (A).trace[(size_t)blockIdx.x * 16 + (slot)] = wall_clock64(); \
  } while (0)

// a double moved between lanes of a row of 16 by one DPP control (quad_perm / row_half_mirror / row_mirror)
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

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

// doStepFromBackup -> FrameOptimizationData::setState's pose of one frame (Src/FullSystemOptimize.cpp:212-233,
// Include/Frame.h:151-170): PRE_worldToCam = exp(scaled state) * evalPT and its inverse, into o[0..6] | o[7..13]
// (SE3 data); o[14], o[15] = the scaled affine a, b.  The solve's step stage and the fused loop's linearize prologue
// both run this, so their poses are bit-identical.
__device__ __forceinline__ void frame_pose_stage(const double sc[10], const hs::SE3& evalPT, double* o,
                                                 hs::SE3* PWo = nullptr, hs::SE3* PCo = nullptr) {
  const hs::SE3 PW = se3_mul_step(se3_exp_step(sc), evalPT);
  const hs::SE3 PC = PW.inverse();
  PW.toData(o);
  PC.toData(o + 7);
  o[14] = sc[6];
  o[15] = sc[7];
  if (PWo) *PWo = PW;
  if (PCo) *PCo = PC;
}

// FrameFramePrecalc::set's state-dependent part for pair (host h, target t) (Src/OptimizationClasses.cpp:13-39) from
// the two frames' frame_pose_stage records: PRE_KRKiTll, PRE_KtTll, PRE_aff_mode (AffLight::fromToVecExposure of the
// scaled a / b) and PRE_b0_mode (the host's aff0_b); vsf = the calib's value_scaledf.  PRE_RTll_0 / PRE_tTll_0
// depend on evalPT only and are not touched.
template <typename PC>
__device__ __forceinline__ void pair_precalc_stage(const double* oh, const double* ot, float exp_h, float exp_t,
                                                   double state_zero7_h, const float vsf[4], PC& pc) {
  double aff[2];
  hs::fromToVecExposure(exp_h, exp_t, oh[14], oh[15], ot[14], ot[15], aff);
  pc.aff[0] = (float)aff[0];
  pc.aff[1] = (float)aff[1];
  pc.b0 = (float)(state_zero7_h * hs::SCALE_B);
  const float K[9] = {vsf[0], 0, vsf[2], 0, vsf[1], vsf[3], 0, 0, 1};
  float Ki[9];
  hs::inv3f(K, Ki);
  hs::SE3 PWt, PCh;
  PWt.q = hs::Quat{ot[0], ot[1], ot[2], ot[3]};
  PWt.t[0] = ot[4]; PWt.t[1] = ot[5]; PWt.t[2] = ot[6];
  PCh.q = hs::Quat{oh[7], oh[8], oh[9], oh[10]};
  PCh.t[0] = oh[11]; PCh.t[1] = oh[12]; PCh.t[2] = oh[13];
  const hs::SE3 l2l = se3_mul_step(PWt, PCh);
  double R[9];
  l2l.rotationMatrix(R);
  float RT[9], tT[3];
#pragma unroll
  for (int i = 0; i < 9; i++) RT[i] = (float)R[i];
#pragma unroll
  for (int i = 0; i < 3; i++) tT[i] = (float)l2l.t[i];
  float KR[9], KRKi[9], Kt[3];
  hs::mm3f(K, RT, KR);
  hs::mm3f(KR, Ki, KRKi);
  hs::mv3f(K, tT, Kt);
#pragma unroll
  for (int i = 0; i < 9; i++) pc.KRKi[i] = KRKi[i];
#pragma unroll
  for (int i = 0; i < 3; i++) pc.Kt[i] = Kt[i];
}

}  // namespace

// =====================================================================================================
// linearize + accumulate: a block = 4 waves over an equal share of ONE host's points, one wave per point
// =====================================================================================================
namespace {

// One point's linearization as lane (target slot t, pattern pixel k) holds it.
struct LinPt {
  float Jx[10], Jy[10];  // [Jpdc(4) Jpdxi(6)] rows of the lane's residual (when the slot was evaluated)
  float S[Q_N];          // the slot's pattern-order sums (octet fold at lane 8t+7, broadcast to the octet)
  float jj;              // JpJdF[t][k] of an active residual, else 0
  bool active;           // the lane's residual is active after this linearization
  unsigned mask;         // the point's active slots (uniform)
  float HdiF, bdSumF, Hcd[4];  // the point's Schur prelude (uniform)
  double eSum;           // the point's share of linearizeAll's energy (uniform)
  float idep;            // idepth after the fused step (uniform)
  // lane-selected accumulator operands (acc_point's layout), formed here from SSA values: select chains over
  // the struct's arrays would be folded into dynamically indexed loads and keep the struct in scratch
  float xk, yk;                // Jx[k], Jy[k]
  float xr10, yr10, xc10, yc10;  // Data (8,8) / (8,9) / (9,9) operands of lanes 0 / 1 / 2
  float xr14, yr14, t014, t114;  // TopRight (8 + k/3, k%3) operands of lanes 0..5
  float br15;                  // BotRight[k] of lanes 0..5
  float hcr, hcc;              // Hcd[r], Hcd[c] of the accHcc / accbc lane
};

// PointFrameResidual::linearize + applyRes / takeData (Src/OptimizationClasses.cpp:43-256) of point p's <= 7
// residuals (lane = target slot x pattern pixel), preceded by the fused resubstituteFPt + point step of the
// previous solve (Src/EnergyFunctional.cpp:249-274), followed by the point sums of
// AccumulatedTopHessianSSE::addPoint<0> / AccumulatedSCHessianSSE::addPoint (Src/AccumulatedTopHessian.cpp:21-141,
// Src/AccumulatedSCHessian.cpp:10-33).  Writes the per-residual / per-point state; returns what the
// accumulators need.  Wave-uniform p.
// The per-point global inputs of lin_point (lane (t, k)'s view), loaded one point ahead by lin_block so the loads
// of point p + W are in flight while point p is linearized; every load is unconditional (clamped indices).
struct LinIn {
  float idep, idep0, pu, pv;
  int res;            // res_of_slot of the lane's slot (< 0: none)
  int st_raw;         // ResState of the slot
  float oldE_raw, oldNewE_raw;
  float colorK, weightK;
  uint2 ro2;          // the point's 8 residual-list slots (int8 each)
  unsigned fm;        // previous linearization's active mask
  float jpj, bds, hdi;
  float4 hcd;
  float priorF;       // the point's idepth prior (its load would otherwise sit in the middle of the point sums)
};
__device__ __forceinline__ void lin_load(const HsLinArgs& a, int p, int lane, LinIn& in) {
  const int t = lane >> 3, k = lane & 7, sl = p * 8 + t;
  in.idep = a.idepth[p];
  in.idep0 = a.idepth_zero[p];
  in.pu = a.u[p];
  in.pv = a.v[p];
  in.res = a.res_of_slot[sl];
  in.st_raw = (int)a.r_state[sl];
  in.oldE_raw = a.r_energy[sl];
  in.oldNewE_raw = a.r_newEnergy[sl];
  in.colorK = a.color[p * 8 + k];
  in.weightK = a.weight[p * 8 + k];
  in.ro2 = reinterpret_cast<const uint2*>(a.res_order)[p];
  in.fm = a.p_actmask[p];
  in.jpj = a.p_JpJdF[sl * 8 + k];
  in.bds = a.p_bdSumF[p];
  in.hdi = a.p_HdiF_prev[p];
  in.hcd = reinterpret_cast<const float4*>(a.p_Hcd)[p];
  in.priorF = a.priorF[p];
}

// per-block constants of lin_point, staged in LDS once per block: the host's precalc records (by target slot),
// the frames' thresholds, xAd[h][t][k] and the calib step
struct LinConst {
  HsCalib cal;  // the scaled calib (staged with the rest: a load in lin_point would follow the block barrier)
  HsPrecalc pre[HS_MAXF];
  float th[HS_MAXF];
  float xad[HS_MAXF * 8];
  float cs[4];
};

// kFix: System::linearizeAll(true)'s bookkeeping (Src/FullSystemOptimize.cpp:26-50): for every residual still active
// after applyRes the point's maxRelBaseline = max(relBS) and numGoodResiduals++ (isNew is never cleared in the
// reference, Include/OptimizationClasses.h:98,112), in the point's residual-list order.
// per-wave LDS scratch of lin_point / acc_point (inside the wave's own partials area, which is written only after
// the wave's last point): the pattern values [Q_N][64], the slot sums [8][LW_SS] and the Schur rows [8][8]
constexpr int LW_SS = 20;  // slot-sum row stride (floats): 16 B aligned rows for ds_read_b128
constexpr int LW_QR = 68;  // pattern-value row stride: the 16 lanes of a 16 B read cover distinct banks
constexpr int LW_QS = 0, LW_SUM = Q_N * LW_QR, LW_JJ = LW_SUM + 8 * LW_SS, LW_FLOATS = LW_JJ + 64;
static_assert(LW_SUM % 4 == 0 && LW_JJ % 4 == 0, "16 B aligned scratch rows");
static_assert(LW_FLOATS <= hs_ne(false) * 64, "lin scratch fits the wave's partials area");

// kMarg: the marginalization pass (hs_k_lin_marg*): production launches compile its branches and arguments out
// kProd: the production launch (hs_k_lin): the fused point step on, no trace -- both compile-time, so their
// branches and arguments leave the kernel (hs_k_lin_gen keeps them at run time)
template <bool kFix, bool kMarg, bool kProd>
__device__ __forceinline__ void lin_point(const HsLinArgs& a, int p, int h, int lane, const LinIn& in,
                                          const LinConst& K, float* ws, LinPt& o) {
  long long* const trc = kProd ? nullptr : a.trace;
  const int t = lane >> 3;  // target slot
  const int k = lane & 7;   // pattern pixel
  const int nF = a.nF;
  const HsCalib cal = K.cal;
  if (kMarg && a.marg && a.marg[p] == 0) {  // marginalization pass, point not marginalized: no active residual
    if (lane == 0) {
      a.p_actmask[p] = 0;
      a.p_HdiF[p] = 0.f;
      a.p_bdSumF[p] = 0.f;
      reinterpret_cast<float4*>(a.p_Hcd)[p] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (t == nF - 1 && k == 0) a.newest_cand[p] = -1.f;
#pragma unroll
    for (int i = 0; i < 10; i++) o.Jx[i] = o.Jy[i] = 0.f;
#pragma unroll
    for (int i = 0; i < Q_N; i++) o.S[i] = 0.f;
    o.jj = 0.f; o.active = false; o.mask = 0u; o.HdiF = 0.f; o.bdSumF = 0.f;
    o.Hcd[0] = o.Hcd[1] = o.Hcd[2] = o.Hcd[3] = 0.f;
    o.eSum = 0.0;
    o.idep = in.idep;
    o.xk = o.yk = o.xr10 = o.yr10 = o.xc10 = o.yc10 = o.xr14 = o.yr14 = o.t014 = o.t114 = o.br15 = 0.f;
    o.hcr = o.hcc = 0.f;
    return;
  }
  // the point's inputs arrived with lin_load (one point ahead); the block constants are in LDS
  const int sl = p * 8 + t;                 // this lane's residual slot
  const int tc_ = t < nF ? t : 0;
  float idep = in.idep, idep0 = in.idep0;
  const float pu = in.pu, pv = in.pv;
  const bool has = in.res >= 0;
  const int st_raw = in.st_raw;
  const float oldE_raw = in.oldE_raw;
  const float oldNewE_raw = in.oldNewE_raw;
  const float thr = fmaxf(K.th[h], K.th[tc_]);  // std::max<float>(host TH, target TH)
  const float colorK = in.colorK, weightK = in.weightK;
  const HsPrecalc pc = K.pre[tc_];
  // the target's image: selected from the kernel-argument pointers (uniform SGPRs), not loaded per lane
  const float4* timg = a.img + (long long)hs_img_slot(a.img_slot, tc_) * a.img_stride;  // past the window: frame 0
  const float* timg3 = a.img3 + (long long)hs_img_slot(a.img_slot, tc_) * a.img_stride * 3;
  // the point's 8 residual-list slots and previous active mask, as scalars (uniform per point)
  const uint2 ro2 = make_uint2(__builtin_amdgcn_readfirstlane(in.ro2.x), __builtin_amdgcn_readfirstlane(in.ro2.y));
  auto res_slot = [&](int q) -> int { return (int)(int8_t)(((q < 4 ? ro2.x : ro2.y) >> (8 * (q & 3))) & 0xffu); };
  // the previous linearization's per-point data for the fused step
  const unsigned fm = __builtin_amdgcn_readfirstlane(in.fm);
  const float xad = K.xad[tc_ * 8 + k];
  const float jpj = in.jpj;
  const float bds = in.bds, hdi = in.hdi;
  const float4 hcd = in.hcd;
  const float cs0 = K.cs[0], cs1 = K.cs[1], cs2 = K.cs[2], cs3 = K.cs[3];
  if (kProd || a.fuse_step) {
    // resubstituteFPt of the previous linearization + the point part of doStepFromBackup (stepfacD = 1).
    // Lane (t, k) forms xAd[h][t][k] * JpJdF[t][k]; the 8-term dot of a residual is an in-order octet fold, the
    // residual terms are then subtracted in list order (uniform).
    const unsigned m = fm;
    const float prod = ((m >> t) & 1u) ? xad * jpj : 0.f;
    const float dsum = octet_fold(prod);
    float b = bds;
    float dot = 0.f;
    dot += cs0 * hcd.x;
    dot += cs1 * hcd.y;
    dot += cs2 * hcd.z;
    dot += cs3 * hcd.w;
    b -= dot;
    // lane q gathers the dot of list entry q (one ds_bpermute), then the terms are subtracted in list order
    const int tq = res_slot(k);
    const float dq = __shfl(dsum, (tq < 0 ? 0 : tq) * 8 + 7);
    float dl[8];
#pragma unroll
    for (int q = 0; q < 8; q++) dl[q] = readlane_f(dq, q);  // independent, ahead of the ordered subtractions
    bool live = true;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const int tt = res_slot(q);
      live = live && tt >= 0;
      const int ts = tt < 0 ? 0 : tt;
      const float bq = b - dl[q];
      b = (live && ((m >> ts) & 1u)) ? bq : b;
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
  const int st = has ? ((kMarg && a.marg) ? HS_RES_IN : st_raw) : HS_RES_OOB;
  const float oldE = (has && !(kMarg && a.marg)) ? oldE_raw : 0.f;
  const float oldNewE = (has && !(kMarg && a.marg)) ? oldNewE_raw : 0.f;

  // Branch-free: every lane evaluates the whole chain (a wave's lanes diverge here anyway, so branches would run
  // both sides and re-materialise the zeroed values at every merge); the reference's early exits become the
  // validity flags okC (centre projection in the image), okP (pattern pixel in the image) and okI (finite
  // intensity).  Values of a lane whose slot is not fully evaluated are never read: everything downstream is gated
  // by eval / active, and the texel fetch of an out-of-image pixel is redirected to (2, 2).
  const bool live0 = has && st != HS_RES_OOB;
  float Jx[10], Jy[10], Jd0, Jd1;
  float qv[Q_N];
  float centre[3];
  bool okC, okI;
  {
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
    const float u = pt0 * drescale, v = pt1 * drescale;
    const float Ku = u * cal.fxl + cal.cxl, Kv = v * cal.fyl + cal.cyl;
    okC = (drescale > 0) && (Ku > 1.1f && Kv > 1.1f && Ku < (cal.W - 3) && Kv < (cal.H - 3));
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
    const bool okP = okC && (PKu > 1.1f && PKv > 1.1f && PKu < (cal.W - 3) && PKv < (cal.H - 3));
    float3 hit = LIN_TEXEL12 ? interp33p(timg3, okP ? PKu : 2.f, okP ? PKv : 2.f, cal.W)
                             : interp33(timg, okP ? PKu : 2.f, okP ? PKv : 2.f, cal.W);
    if (trc && threadIdx.x == 0 && hit.x != -12345.f) trc[(size_t)blockIdx.x * 16 + 13] = wall_clock64();
    const float color = colorK;
    const float residual = hit.x - (float)(pc.aff[0] * color + pc.aff[1]);
    const float drdA = (color - pc.b0);
    okI = okP && isfinite(hit.x);
    float w = sqrtf(a.lp.outlierTHSumComponent / (a.lp.outlierTHSumComponent + (hit.y * hit.y + hit.z * hit.z)));
    w = 0.5f * (w + weightK);
    float hw = fabsf(residual) < a.lp.huberTH ? 1 : a.lp.huberTH / fabsf(residual);
    qv[0] = w * w * hw * residual * residual * (2 - hw);
    hw = hw < 1 ? sqrtf(hw) : hw;
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
    if (kMarg && a.marg) {
      const float* dp = a.adHTdelta + (h + nF * t) * 8;
      float jx = 0.f, jy = 0.f, cxx = 0.f, cyy = 0.f;
#pragma unroll
      for (int i = 0; i < 6; i++) {
        jx += Jx[4 + i] * dp[i];
        jy += Jy[4 + i] * dp[i];
      }
      const float* cd = a.adHTdelta + nF * nF * 8;  // cDeltaF after the pairs (hs_k_marg_delta)
#pragma unroll
      for (int i = 0; i < 4; i++) {
        cxx += Jx[i] * cd[i];
        cyy += Jy[i] * cd[i];
      }
      const float dF = idep - idep0;
      const float Jpdx = jx + cxx + Jd0 * dF;
      const float Jpdy = jy + cyy + Jd1 * dF;
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
  const bool oob = live0 && !okI;
  const bool centreOk = live0 && okC;
  const unsigned long long oobMask = __ballot(oob);
  const bool slotOob = ((oobMask >> (t * 8)) & 0xffull) != 0ull;

  // sequential (pattern-order) sums = the reference's running sums: octet folds at lane 8t+7, broadcast to the
  // octet by ds_bpermute (no LDS round trip, no barrier: the waves of a block run their points independently)
  // through the wave's LDS scratch: the pattern values are transposed so that one lane folds one (quantity, slot)
  // pair over its 8 pixels in order (two 16 B reads, 8 adds), the 136 sums go back to LDS and every lane reads
  // the 17 sums of its slot (same-address reads within an octet)
  float S[Q_N];
  {
    float* qs = ws + LW_QS;
    float* ss = ws + LW_SUM;
#pragma unroll
    for (int qi = 0; qi < Q_N; qi++) qs[qi * LW_QR + lane] = qv[qi];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int r = 0; r < 3; r++) {  // pairs lane + 64 r = (quantity qi, slot ts), 136 of them
      const int pr = lane + 64 * r;
      if (r < 2 || pr < Q_N * 8) {
        const int qi = pr >> 3, ts = pr & 7;
        const float4 x0 = *reinterpret_cast<const float4*>(qs + qi * LW_QR + ts * 8);
        const float4 x1 = *reinterpret_cast<const float4*>(qs + qi * LW_QR + ts * 8 + 4);
        float f = 0.f + x0.x;
        f = f + x0.y;
        f = f + x0.z;
        f = f + x0.w;
        f = f + x1.x;
        f = f + x1.y;
        f = f + x1.z;
        f = f + x1.w;
        ss[ts * LW_SS + qi] = f;
      }
    }
    __builtin_amdgcn_wave_barrier();
    const float4* sr = reinterpret_cast<const float4*>(ss + t * LW_SS);
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const float4 v4 = sr[i];
      S[4 * i] = v4.x;
      S[4 * i + 1] = v4.y;
      S[4 * i + 2] = v4.z;
      S[4 * i + 3] = v4.w;
    }
    S[16] = ss[t * LW_SS + 16];
  }
  if (trc && threadIdx.x == 0 && S[0] != -12345.f) trc[(size_t)blockIdx.x * 16 + 14] = wall_clock64();

  // ---------------- state decision + applyRes (the 8 lanes of a slot agree; lane k == 0 writes)
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
  float tHdd, tbd, tc[4];  // the slot's terms of the per-point sums
  {
    // takeData (Include/OptimizationClasses.h:155-161), computed unconditionally, stored when active
    const float J00 = S[1], J11 = S[2], J10 = S[3];
    const float aa = J00 * Jd0 + J10 * Jd1;
    const float bb = J10 * Jd0 + J11 * Jd1;
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
    if (active) a.p_JpJdF[(p * 8 + t) * 8 + k] = jj;
    o.jj = active ? jj : 0.f;
  }
  // ---------------- per-point sums in the point's residual-list order (uniform; readlane from lane 8 * slot)
  {
    const unsigned long long actBits = __ballot(active);
    // lane 8t + i carries quantity i of slot t (tbd, tHdd, tc[0..3], -, econ); lane i of every octet gathers
    // quantity i of the listed residuals (one ds_bpermute per list entry, all in flight), then sums them in list
    // order: the reference's sequential sums, one lane per quantity
    const float X = k == 0 ? tbd : k == 1 ? tHdd : k == 2 ? tc[0] : k == 3 ? tc[1] : k == 4 ? tc[2] : k == 5 ? tc[3] : econ;
    float g[8];
    int nres = 8;
#pragma unroll
    for (int qn = 0; qn < 8; qn++) {
      const int tt = res_slot(qn);
      nres = (tt < 0 && qn < nres) ? qn : nres;
      g[qn] = __shfl(X, (tt < 0 ? 0 : tt) * 8 + k);
    }
    float qsum = 0.f;
    double eAcc = 0.0;
    unsigned mask = 0u;
#pragma unroll
    for (int qn = 0; qn < 8; qn++) {  // fully unrolled, predicated (g stays in registers)
      const bool listed = qn < nres;  // uniform
      const int tt = res_slot(qn) & 7;
      const double e1 = eAcc + (double)g[qn];  // econ: every listed residual (read from lane 7)
      eAcc = listed ? e1 : eAcc;
      const bool act = listed && ((actBits >> (tt * 8)) & 1ull);
      mask |= act ? 1u << tt : 0u;
      const float q1 = qsum + g[qn];
      qsum = act ? q1 : qsum;
    }
    const double eSum = __longlong_as_double(((long long)__builtin_amdgcn_readlane((int)(__double_as_longlong(eAcc) >> 32), 7) << 32) |
                                             (unsigned int)__builtin_amdgcn_readlane((int)__double_as_longlong(eAcc), 7));
    const float bd = readlane_f(qsum, 0), Hdd = readlane_f(qsum, 1);
    float Hcd[4];
#pragma unroll
    for (int c = 0; c < 4; c++) Hcd[c] = readlane_f(qsum, 2 + c);
    float HdiF = 0.f, bdSumF = 0.f;
    if (mask != 0u) {
      // marginalization pass: priorF *= idepthFixPriorMargFac, the sums are the LF ones (AF = 0), and
      // AccumulatedSCHessianSSE::addPoint(p, shiftPriorToZero = false) (Src/EnergyFunctional.cpp:563,577)
      const float priorF = (kMarg && a.marg) ? in.priorF * a.margPriorFac : in.priorF;
      float Hh = (kMarg && a.marg) ? (0.f + Hdd) + priorF : Hdd + 0.f + priorF;  // Hdd_accAF + Hdd_accLF + priorF
      if ((double)Hh < 1e-10) Hh = (float)1e-10;
      HdiF = (float)(1.0 / (double)Hh);
      bdSumF = (kMarg && a.marg) ? 0.f + bd : bd + 0.f;
      if (!(kMarg && a.marg)) bdSumF += priorF * (idep - idep0);
    }
    float4 hc4;
    if (kMarg && a.marg) hc4 = make_float4(0.f + Hcd[0], 0.f + Hcd[1], 0.f + Hcd[2], 0.f + Hcd[3]);
    else hc4 = make_float4(Hcd[0] + 0.f, Hcd[1] + 0.f, Hcd[2] + 0.f, Hcd[3] + 0.f);
    if (lane == 0) {
      a.p_actmask[p] = (uint8_t)mask;
      a.p_HdiF[p] = HdiF;
      a.p_bdSumF[p] = bdSumF;
      reinterpret_cast<float4*>(a.p_Hcd)[p] = hc4;
    }
    if (kFix) {
      // relBS = 0.01 |ptp_inf.xy / ptp_inf.z - ptp.xy / ptp.z| with ptp_inf = KRKi (u, v, 1), ptp = ptp_inf + Kt
      // idepth (:35-37; 0.01 is a double), uniform per slot
      float q0 = pc.KRKi[0] * pu + pc.KRKi[1] * pv + pc.KRKi[2] * 1.f;
      float q1 = pc.KRKi[3] * pu + pc.KRKi[4] * pv + pc.KRKi[5] * 1.f;
      float q2 = pc.KRKi[6] * pu + pc.KRKi[7] * pv + pc.KRKi[8] * 1.f;
      const float r0 = q0 + pc.Kt[0] * idep, r1 = q1 + pc.Kt[1] * idep, r2 = q2 + pc.Kt[2] * idep;
      const float dx = q0 / q2 - r0 / r2, dy = q1 / q2 - r1 / r2;
      const float relBS = (float)(0.01 * (double)sqrtf(dx * dx + dy * dy));
      float mr = a.fix_relBL[p];
      int ng = a.fix_nGood[p];
      for (int qn = 0; qn < 8; qn++) {
        const int tt = res_slot(qn);
        if (tt < 0) break;
        if (!((actBits >> (tt * 8)) & 1ull)) continue;
        const float rb = readlane_f(relBS, tt * 8);
        if (rb > mr) mr = rb;
        ng++;
      }
      if (lane == 0) {
        a.fix_relBL[p] = mr;
        a.fix_nGood[p] = ng;
      }
    }
    o.mask = mask;
    o.HdiF = HdiF;
    o.bdSumF = bdSumF;
    o.Hcd[0] = hc4.x; o.Hcd[1] = hc4.y; o.Hcd[2] = hc4.z; o.Hcd[3] = hc4.w;
    o.eSum = eSum;
  }
  if (trc && threadIdx.x == 0 && o.eSum != -12345.0) trc[(size_t)blockIdx.x * 16 + 15] = wall_clock64();
#pragma unroll
  for (int i = 0; i < 10; i++) {
    o.Jx[i] = Jx[i];
    o.Jy[i] = Jy[i];
  }
#pragma unroll
  for (int i = 0; i < Q_N; i++) o.S[i] = S[i];
  o.active = active;
  o.idep = idep;
  {
    float xk = Jx[0], yk = Jy[0];
#pragma unroll
    for (int c = 1; c < 8; c++) {
      xk = k == c ? Jx[c] : xk;
      yk = k == c ? Jy[c] : yk;
    }
    o.xk = xk;
    o.yk = yk;
    o.xr10 = k == 2 ? Jx[9] : Jx[8];
    o.yr10 = k == 2 ? Jy[9] : Jy[8];
    o.xc10 = k == 0 ? Jx[8] : Jx[9];
    o.yc10 = k == 0 ? Jy[8] : Jy[9];
    const int kk = k < 3 ? k : k - 3;
    o.xr14 = k < 3 ? Jx[8] : Jx[9];
    o.yr14 = k < 3 ? Jy[8] : Jy[9];
    o.t014 = kk == 0 ? S[4] : (kk == 1 ? S[6] : S[12]);
    o.t114 = kk == 0 ? S[5] : (kk == 1 ? S[7] : S[13]);
    o.br15 = k == 0 ? S[8] : k == 1 ? S[9] : k == 2 ? S[14] : k == 3 ? S[10] : k == 4 ? S[15] : S[16];
    const int r = (lane >> 2) & 3, c = lane & 3;
    o.hcr = r == 0 ? o.Hcd[0] : r == 1 ? o.Hcd[1] : r == 2 ? o.Hcd[2] : o.Hcd[3];
    o.hcc = c == 0 ? o.Hcd[0] : c == 1 ? o.Hcd[1] : c == 2 ? o.Hcd[2] : o.Hcd[3];
  }
}

// index of the (o1 <= o2) pair of non-host slots in the production accD layout
__host__ __device__ constexpr int dpair(int o1, int o2) { return o1 * 7 - (o1 * (o1 - 1)) / 2 + (o2 - o1); }

// The lane's accumulators of its block (see hs_kernels.h, HS_E_TOP).  fp32, the reference's per-update
// expressions (Include/MatrixAccumulators.h), in the wave's point order.
template <bool kExact>
struct LinAcc {
  static constexpr int ND = kExact ? HS_ND_EXACT : HS_ND_PROD;
  float T[HS_E_TOP];  // AccumulatorApprox entries of (host, t): see acc_point
  float D[ND];        // accD[host + t1 nF + t2 nF^2][row][col], lane = 8 row + col
  float E[5];         // accE[host + t nF][k][0..3], accEB[host + t nF][k]
  float C;            // accHcc[r][c] (lanes 0..15, lane = 4r + c), accbc[r] (lanes 16..19)
  double e, sid, np;  // energy, sum |idepth|, points
};

template <bool kExact>
__device__ __forceinline__ void acc_point(LinAcc<kExact>& A, const LinPt& P, int h, int lane, float* ws) {
  // ---- AccumulatedTopHessianSSE::addPoint<0> of the lane's residual: AccumulatorApprox::update / updateTopRight /
  // updateBotRight (Include/MatrixAccumulators.h:754-915).  Lane (t, k) owns, of the 13x13 (host, t) block:
  //   T[j]  Data (j, k), j <= k (x/y column k, the rows uniform)      T[8], T[9]  Data (k, 8), (k, 9)
  //   T[10] Data (8,8) / (8,9) / (9,9) on lanes 0 / 1 / 2            T[11..13]   TopRight (k, a / b / r)
  //   T[14] TopRight (8 + k/3, k%3) on lanes 0..5                     T[15]       BotRight[k] on lanes 0..5
  // Entries a lane computes for j > k / k >= 3 / k >= 6 are never read (hs_k_reduce decodes the owners only).
  if (P.active) {
    const float a_ = P.S[1], b_ = P.S[3], c_ = P.S[2];  // JIdx2 00, 01, 11
    const float xk = P.xk, yk = P.yk;
    // Data[(r, c >= r)] += a x_c x_r + c y_c y_r + b (x_c y_r + y_c x_r), left to right
    auto dat = [&](float xr, float yr, float xc, float yc) {
      return ((a_ * xc) * xr + (c_ * yc) * yr) + b_ * ((xc * yr) + (yc * xr));
    };
#pragma unroll
    for (int j = 0; j < 8; j++) A.T[j] += dat(P.Jx[j], P.Jy[j], xk, yk);
    A.T[8] += dat(xk, yk, P.Jx[8], P.Jy[8]);
    A.T[9] += dat(xk, yk, P.Jx[9], P.Jy[9]);
    A.T[10] += dat(P.xr10, P.yr10, P.xc10, P.yc10);
    // TopRight[3 r + c] += x_r TR0c + y_r TR1c with (TR00, TR10, TR01, TR11, TR02, TR12) = (JabJIdx 00, 01, 10, 11,
    // JI_r 0, 1)
    A.T[11] += xk * P.S[4] + yk * P.S[5];
    A.T[12] += xk * P.S[6] + yk * P.S[7];
    A.T[13] += xk * P.S[12] + yk * P.S[13];
    A.T[14] += P.xr14 * P.t014 + P.yr14 * P.t114;
    // BotRight (Jab2 00, 01, Jab_r 0, Jab2 11, Jab_r 1, rr)
    A.T[15] += P.br15;
    // ---- AccumulatedSCHessianSSE::addPoint (Src/AccumulatedSCHessian.cpp:50-51): accE update(JpJdF, Hcd, HdiF),
    // accEB update(JpJdF, HdiF * bdSumF)
    const float wl = P.HdiF * P.jj;
#pragma unroll
    for (int c = 0; c < 4; c++) A.E[c] += wl * P.Hcd[c];
    A.E[4] += (P.HdiF * P.bdSumF) * P.jj;
  }
  // ---- accD[host + t1 nF + t2 nF^2].update(JpJdF_t1, JpJdF_t2, HdiF) (Src/AccumulatedSCHessian.cpp:38-48): lane
  // (row, col) = (lane >> 3, lane & 7); JpJdF[t][i] sits in lane 8t + i (zero unless active)
  {
    // rows of the non-host slots through the wave's LDS scratch: jb[i][o] = JpJdF[slot of o][i]
    const int dr = lane >> 3, dc = lane & 7;
    float* jb = ws + LW_JJ;
    const int t = lane >> 3, k = lane & 7;
    if (t != h) jb[k * 8 + t - (t > h ? 1 : 0)] = P.jj;
    __builtin_amdgcn_wave_barrier();
    const float4 r0 = *reinterpret_cast<const float4*>(jb + dr * 8), r1 = *reinterpret_cast<const float4*>(jb + dr * 8 + 4);
    const float4 c0 = *reinterpret_cast<const float4*>(jb + dc * 8), c1 = *reinterpret_cast<const float4*>(jb + dc * 8 + 4);
    const float j1[7] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z};
    const float j2[7] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z};
#pragma unroll
    for (int o1 = 0; o1 < 7; o1++) {
      const float wl = P.HdiF * j1[o1];
#pragma unroll
      for (int o2 = kExact ? 0 : o1; o2 < 7; o2++) A.D[kExact ? o1 * 7 + o2 : dpair(o1, o2)] += wl * j2[o2];
    }
  }
  // ---- accHcc.update(Hcd, Hcd, HdiF), accbc.update(Hcd, bdSumF * HdiF) (Src/AccumulatedSCHessian.cpp:32-33)
  if (P.mask != 0u) A.C += lane < 16 ? (P.HdiF * P.hcr) * P.hcc : (P.bdSumF * P.HdiF) * P.hcc;
  A.e += P.eSum;
  A.sid += (double)fabsf(P.idep);
  A.np += 1.0;
}

template <bool kExact, bool kFix, bool kMarg = false, bool kProd = false>
__device__ __forceinline__ void lin_block(const HsLinArgs& a) {
  struct { long long* trace; } const T{kProd ? nullptr : a.trace};  // HS_TRACE's view
  extern __shared__ float lin_stage[];  // [HS_LIN_NW waves][ne][64] fp32 partials, then [HS_LIN_NW][3] fp64 energies
  // the wave index as a scalar: the point index and everything per point then stays uniform (scalar loads,
  // scalar branches) instead of being treated as divergent
  if (a.brk && a.st->stop) return;
  const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int b = blockIdx.x;
  int h = 0;  // the block's host: from the kernel-argument block boundaries, no load
#pragma unroll
  for (int i = 1; i < HS_MAXF; i++) h += (i < a.nF && b >= a.blk_begin[i]) ? 1 : 0;
  const int nb = a.blk_begin[h + 1] - a.blk_begin[h], q = b - a.blk_begin[h];
  const int hb = a.host_begin[h], nh = a.host_begin[h + 1] - hb;
  const int pb = hb + (int)((long long)nh * q / nb), pe = hb + (int)((long long)nh * (q + 1) / nb);
  HS_TRACE(T, 0);
  __shared__ LinConst K;
  {  // the block's constants: precalc records of host h (by target), thresholds, xAd[h][.][.], calib step
    const int nF = a.nF;
    constexpr int PW = (int)(sizeof(HsPrecalc) / 4);
    static_assert(sizeof(HsPrecalc) % 4 == 0, "precalc staged as words");
    const int* src = reinterpret_cast<const int*>(a.pre + h * nF);
    int* dst = reinterpret_cast<int*>(K.pre);
    for (int i = tid; i < nF * PW; i += HS_LIN_NT) dst[i] = src[i];
    if (tid < nF) K.th[tid] = a.frameTH[tid];
    if ((kProd || a.fuse_step) && tid < nF * 8) {
      // xAd[h][t][c] of the last solve (EnergyFunctional::resubstituteF_MT): the frame steps (float)lastX and the
      // fp32 adjoints of the pair, in the solve's summation order
      const int t = tid >> 3, c = tid & 7;
      const float* aH = a.adHostF + (h + nF * t) * 64;
      const float* aT = a.adTargetF + (h + nF * t) * 64;
      const double* lx = a.st->lastX;
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int rr = 0; rr < 8; rr++) s1 += (float)lx[4 + 8 * h + rr] * aH[rr * 8 + c];
#pragma unroll
      for (int rr = 0; rr < 8; rr++) s2 += (float)lx[4 + 8 * t + rr] * aT[rr * 8 + c];
      K.xad[tid] = s1 + s2;
    }
    if (tid < 4) K.cs[tid] = a.st->cstep[tid];
    constexpr int CW = (int)(sizeof(HsCalib) / 4);
    static_assert(sizeof(HsCalib) % 4 == 0, "calib staged as words");
    if (tid >= 64 && tid < 64 + CW)
      reinterpret_cast<int*>(&K.cal)[tid - 64] = reinterpret_cast<const int*>(&a.st->dcal)[tid - 64];
  }
  LinAcc<kExact> A;
#pragma unroll
  for (int i = 0; i < HS_E_TOP; i++) A.T[i] = 0.f;
#pragma unroll
  for (int i = 0; i < LinAcc<kExact>::ND; i++) A.D[i] = 0.f;
#pragma unroll
  for (int i = 0; i < 5; i++) A.E[i] = 0.f;
  A.C = 0.f;
  A.e = A.sid = A.np = 0.0;
  float* ws = lin_stage + wv * hs_ne(kExact) * 64;  // the wave's LDS scratch (its partials area)
  LinIn cur;
  const bool work = wv < a.W && pb + wv < pe;
  if (work) lin_load(a, pb + wv, lane, cur);  // in flight across the barrier
  __syncthreads();
  HS_TRACE(T, 12);
  if (work && LIN_ONE_PATH && pb + wv + a.W >= pe) {
    // the wave's only point (the 2k headline: one point per wave): no loop, so nothing is hoisted out of one and
    // kept live (spilled) across the point's work
    LinPt P;
    lin_point<kFix, kMarg, kProd>(a, pb + wv, h, lane, cur, K, ws, P);
    if (a.accumulate) acc_point<kExact>(A, P, h, lane, ws);
  } else if (work) {
    for (int p = pb + wv; p < pe; p += a.W) {  // wave-uniform
      LinIn nxt;
      if (p + a.W < pe) lin_load(a, p + a.W, lane, nxt);  // the next point's loads overlap this point's work
      else nxt = cur;  // last point of the wave (a wave-uniform branch): no duplicate loads
      LinPt P;
      lin_point<kFix, kMarg, kProd>(a, p, h, lane, cur, K, ws, P);
      if (a.accumulate) acc_point<kExact>(A, P, h, lane, ws);
      cur = nxt;
    }
  }
  HS_TRACE(T, 1);
  if (T.trace && lane == 0) T.trace[(size_t)blockIdx.x * 16 + 4 + wv] = wall_clock64();  // each wave's finish
  if (!a.accumulate) return;
  // the waves' partials, summed in wave order (fp32) into the block partial; the energies in fp64
  constexpr int NE = hs_ne(kExact);
  float* my = lin_stage + wv * NE * 64;
#pragma unroll
  for (int i = 0; i < HS_E_TOP; i++) my[i * 64 + lane] = A.T[i];
#pragma unroll
  for (int i = 0; i < LinAcc<kExact>::ND; i++) my[(HS_E_TOP + i) * 64 + lane] = A.D[i];
#pragma unroll
  for (int i = 0; i < 5; i++) my[(HS_E_TOP + LinAcc<kExact>::ND + i) * 64 + lane] = A.E[i];
  my[(NE - 1) * 64 + lane] = A.C;
  double* se = reinterpret_cast<double*>(lin_stage + HS_LIN_NW * NE * 64);
  if (lane == 0) {
    se[wv * 3 + 0] = A.e;
    se[wv * 3 + 1] = A.sid;
    se[wv * 3 + 2] = A.np;
  }
  __syncthreads();
  HS_TRACE(T, 3);
  // 16 B per thread and step, every wave's value loaded before the in-order sum (a runtime-bound loop would wait
  // for each LDS load in turn); waves past W hold no points and are not added
  static_assert((NE * 64) % 4 == 0, "partials staged as float4");
  float4* out4 = reinterpret_cast<float4*>(a.part + (size_t)b * NE * 64);
  const float4* st4 = reinterpret_cast<const float4*>(lin_stage);
  // both rounds' loads issued together (the round count is a compile-time constant), then the sums
  constexpr int NI = (NE * 16 + HS_LIN_NT - 1) / HS_LIN_NT;
  float4 v[NI][HS_LIN_NW];
#pragma unroll
  for (int k = 0; k < NI; k++)
#pragma unroll
    for (int w = 0; w < HS_LIN_NW; w++) v[k][w] = st4[w * NE * 16 + min(tid + k * HS_LIN_NT, NE * 16 - 1)];
#pragma unroll
  for (int k = 0; k < NI; k++) {
    const int i = tid + k * HS_LIN_NT;
    float4 s = v[k][0];
#pragma unroll
    for (int w = 1; w < HS_LIN_NW; w++)
      if (w < a.W) {
        s.x += v[k][w].x;
        s.y += v[k][w].y;
        s.z += v[k][w].z;
        s.w += v[k][w].w;
      }
    if (i < NE * 16) out4[i] = s;
  }
  if (tid < 3) {
    double s = se[tid];
    for (int w = 1; w < a.W; w++) s += se[w * 3 + tid];
    a.part_e[(size_t)b * 4 + tid] = s;
  }
  HS_TRACE(T, 2);
}
}  // namespace

__global__ __launch_bounds__(HS_LIN_NT) void hs_k_lin(HsLinArgs a) { lin_block<false, false, false, true>(a); }
__global__ __launch_bounds__(HS_LIN_NT) void hs_k_lin_gen(HsLinArgs a) { lin_block<false, false>(a); }
__global__ __launch_bounds__(HS_LIN_NT) void hs_k_lin_exact(HsLinArgs a) { lin_block<true, false>(a); }
__global__ __launch_bounds__(HS_LIN_NT) void hs_k_lin_fix(HsLinArgs a) { lin_block<false, true>(a); }
__global__ __launch_bounds__(HS_LIN_NT) void hs_k_lin_exact_fix(HsLinArgs a) { lin_block<true, true>(a); }
__global__ __launch_bounds__(HS_LIN_NT) void hs_k_lin_marg(HsLinArgs a) { lin_block<false, false, true>(a); }
__global__ __launch_bounds__(HS_LIN_NT) void hs_k_lin_exact_marg(HsLinArgs a) { lin_block<true, false, true>(a); }

// =====================================================================================================
// reduce + stitch: (host, chunk) blocks sum the host's block partials in block order; the last chunk block of a
// host stitches the host (fp64) into the host's slot.  Two more blocks: the energy, setNewFrameEnergyTH.
// =====================================================================================================
namespace {
// linearizeAll's energy (+ the sumNID / numID statistics of doStepFromBackup): block partials in block order
// (threads 0..255 sum; a larger block's other threads only take part in the barriers)
__device__ void red_energy_block(const HsRedArgs& a) {
  __shared__ double red[3][256];
  const int tid = threadIdx.x;
  if (tid < 256) {
    double s[3] = {0.0, 0.0, 0.0};
    const int per = (a.nblk + 255) / 256, b0 = tid * per, b1 = min(a.nblk, b0 + per);  // contiguous runs
    for (int b = b0; b < b1; b++)
#pragma unroll
      for (int k = 0; k < 3; k++) s[k] += a.part_e[(size_t)b * 4 + k];
#pragma unroll
    for (int k = 0; k < 3; k++) red[k][tid] = s[k];
  }
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o)
#pragma unroll
      for (int k = 0; k < 3; k++) red[k][tid] += red[k][tid + o];
    __syncthreads();
  }
  if (tid < 3) a.sysE[tid] = red[tid][0];
}

// setNewFrameEnergyTH (Src/FullSystemOptimize.cpp:60-101): the k-th smallest candidate, k = (int)(THN * count), by
// a 3-pass radix select over the candidates' bit patterns (non-negative floats order like their bits).  Candidates:
// one float per point and rank (negative or NaN = none); the ranks' arrays are all-gathered, so every rank
// selects over the same union and computes the same threshold.  Pass 1 (bits 30..19) is counted by the nhist
// histogram blocks of hs_k_reduce (red_th_hist_block, spread over the chip); the stitch launch's last block
// (red_energy_th_block) selects the bin, then counts bits 18..9 and 8..0 of the survivors, which it compacts into
// LDS on the way.  All counts are integer: the result is order-independent.
__device__ void red_th_hist_block(const HsRedArgs& a, int j) {
  __shared__ unsigned int hh[HS_TH_BINS];
  const int tid = threadIdx.x, nt = blockDim.x;
  for (int i = tid; i < HS_TH_BINS; i += nt) hh[i] = 0u;
  __syncthreads();
  const int total = a.nranks * a.stride;
  const int per = (total + a.nhist - 1) / a.nhist, i0 = j * per, i1 = min(total, i0 + per);
  for (int i = i0 + tid; i < i1; i += nt) {
    const unsigned int v = __float_as_uint(a.cand[i]);
    if (v <= 0x7f800000u) atomicAdd(&hh[v >> 19], 1u);  // >= 0 and not NaN (state_NewEnergyWithOutlier >= 0)
  }
  __syncthreads();
  for (int i = tid; i < HS_TH_BINS; i += nt)
    if (hh[i]) atomicAdd(&a.th_hist[i], hh[i]);
}

// inclusive block prefix sum (wave scans + the waves' totals through wsum[16]); total = the block's sum
__device__ __forceinline__ unsigned int block_incl_scan(unsigned int x, unsigned int* wsum, unsigned int& total) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[wv] = x;
  __syncthreads();
  unsigned int off = 0, tot = 0;
  for (int w = 0; w < nw; w++) {
    const unsigned int v = wsum[w];
    off += w < wv ? v : 0u;
    tot += v;
  }
  __syncthreads();
  total = tot;
  return x + off;
}

constexpr int TH_CAP = 24576;  // survivors of pass 1 kept in LDS (else pass 3 re-reads the candidates)

// The bin of hist[0 .. nbins) that holds the k-th smallest counted element and k's rank inside it (every thread of
// the block calls it; any block size with nbins <= 8 * blockDim.x).  k = (int)(thn * total) when thn >= 0, else kin;
// total = the histogram's sum (0: bin / krem are not set).  zero: the histogram is re-zeroed after it is read.
__device__ __forceinline__ void hist_pick(unsigned int* hist, int nbins, bool zero, float thn, unsigned int kin,
                                          unsigned int* wsum, unsigned int* ctl, unsigned int& bin,
                                          unsigned int& krem, unsigned int& total) {
  const int tid = threadIdx.x, nt = blockDim.x;
  const int bpt = (nbins + nt - 1) / nt, b0 = tid * bpt;
  unsigned int hv[8], s = 0u;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    hv[j] = (j < bpt && b0 + j < nbins) ? hist[b0 + j] : 0u;
    s += hv[j];
  }
  if (zero)
#pragma unroll
    for (int j = 0; j < 8; j++)
      if (j < bpt && b0 + j < nbins) hist[b0 + j] = 0u;
  const unsigned int incl = block_incl_scan(s, wsum, total);
  if (total == 0u) return;
  const unsigned int k = thn >= 0.f ? (unsigned int)(int)(thn * (float)total) : kin;
  if (s != 0u && incl - s <= k && k < incl) {
    unsigned int run = incl - s;
    int r = 0;
#pragma unroll
    for (int j = 0; j < 7; j++)
      if (r == j && j + 1 < bpt && k >= run + hv[j]) {
        run += hv[j];
        r = j + 1;
      }
    ctl[0] = (unsigned int)(b0 + r);
    ctl[1] = k - run;
  }
  __syncthreads();
  bin = ctl[0];
  krem = ctl[1];
  __syncthreads();  // ctl is rewritten by the next pick
}

// pass 1's bin: the pass-1 histogram's bin b1 holding the k-th smallest candidate (k = (int)(THN * n)) and the
// rank kk of the wanted value inside b1; n = number of candidates (0: no candidate).  zero: re-zero the histogram for
// the next launch (its last reader does).  Every thread of the block calls it.
__device__ __forceinline__ void th_pass1(const HsRedArgs& a, unsigned int* wsum, unsigned int* ctl, bool zero,
                                         unsigned int& b1, unsigned int& kk, unsigned int& n) {
  hist_pick(a.th_hist, HS_TH_BINS, zero, a.frameEnergyTHN, 0u, wsum, ctl, b1, kk, n);
}

// Multi-block pass 2 (large windows; the stitch launch's np2 extra blocks): block q counts bits 18..9 of its chunk's
// candidates in bin b1 into the global pass-2 histogram and appends them to the global survivor list (LDS
// histogram and LDS compaction first: one global atomic per non-empty bin and one per block for the list range).
// The pass-3 select (red_energy_th_block with th_hist2 set) runs after the stitch.
__device__ void red_th_pass2_block(const HsRedArgs& a, int q, unsigned int* sm) {
  unsigned int* hist2 = sm;          // [1024]
  unsigned int* wsum = sm + 1024;    // [16]
  unsigned int* ctl = sm + 1040;     // bin, k, block survivors, list base
  unsigned int* buf = sm + 1088;     // [TH_CAP]
  const int tid = threadIdx.x, nt = blockDim.x;
  for (int i = tid; i < 1024; i += nt) hist2[i] = 0u;
  if (tid == 0) ctl[2] = 0u;
  unsigned int b1 = 0, kk = 0, n = 0;
  th_pass1(a, wsum, ctl, false, b1, kk, n);
  if (n == 0) return;
  const int total = a.nranks * a.stride;
  const int per = (total + a.np2 - 1) / a.np2, i0 = q * per, i1 = min(total, i0 + per);
  constexpr int TH_U = 16;
  for (int c0 = i0; c0 < i1; c0 += TH_U * nt) {
    unsigned int v[TH_U];
#pragma unroll
    for (int u = 0; u < TH_U; u++) {
      const int i = c0 + u * nt + tid;
      v[u] = i < i1 ? __float_as_uint(a.cand[i]) : 0xffffffffu;
    }
#pragma unroll
    for (int u = 0; u < TH_U; u++)
      if (v[u] <= 0x7f800000u && (v[u] >> 19) == b1) {
        atomicAdd(&hist2[(v[u] >> 9) & 1023u], 1u);
        const unsigned int pos = atomicAdd(&ctl[2], 1u);
        if (pos < (unsigned int)TH_CAP) buf[pos] = v[u];
      }
  }
  __syncthreads();
  const bool over = ctl[2] > (unsigned int)TH_CAP;
  const unsigned int ns = over ? 0u : ctl[2];
  if (tid == 0) {
    // the block's survivors go to the global list; a chunk beyond TH_CAP, or a list that would pass HS_TH_SURV, sets
    // the overflow word (th_nsurv[1]) instead: pass 3 then re-scans the candidates (the count stays a plain sum)
    const unsigned int base = atomicAdd(&a.th_nsurv[0], ns);
    if (over || base + ns > (unsigned int)HS_TH_SURV) atomicOr(&a.th_nsurv[1], 1u);
    ctl[3] = base;
  }
  for (int i = tid; i < 1024; i += nt)
    if (hist2[i]) atomicAdd(&a.th_hist2[i], hist2[i]);
  __syncthreads();
  const unsigned int base = ctl[3];
  for (unsigned int i = tid; i < ns; i += nt)
    if (base + i < (unsigned int)HS_TH_SURV) a.th_surv[base + i] = buf[i];
}

// The select block: passes 2 and 3 over the candidates in pass 1's bin (any block size).
// sm: hist2 [1024] | hist3 [512] | wsum [16] | ctl [48] | buf [cap] (survivors of pass 1 kept in LDS; more: pass 3
// re-scans the candidates) | local: hist1 [HS_TH_BINS].
// local = false: pass 1 is the global histogram of hs_k_reduce's histogram blocks (read and re-zeroed here); with
// a.th_hist2 set, pass 2 is the stitch launch's multi-block one (its histogram and survivor list are read and
// re-zeroed here instead of re-scanning the candidates).  local = true: the block counts pass 1 itself into LDS
// (the multi-rank path's select beside the solve, over the all-gathered candidates; a.th_hist2 unused).
__device__ void th_select_block(const HsRedArgs& a, unsigned int* sm, int cap, bool local) {
  unsigned int* hist2 = sm;          // [1024]
  unsigned int* hist3 = sm + 1024;   // [512]
  unsigned int* wsum = sm + 1536;    // [16]
  unsigned int* ctl = sm + 1552;     // bin, k, survivors, count
  unsigned int* buf = sm + 1600;     // [cap]
  unsigned int* hist1 = sm + 1600 + cap;  // local: [HS_TH_BINS]
  const int tid = threadIdx.x, nt = blockDim.x;
  const int total = a.nranks * a.stride;
  const bool multi = !local && a.th_hist2 != nullptr;
  for (int i = tid; i < 1024 + 512; i += nt) sm[i] = 0u;
  if (local)
    for (int i = tid; i < HS_TH_BINS; i += nt) hist1[i] = 0u;
  if (tid == 0) {
    ctl[2] = 0u;
    ctl[3] = 0u;
  }
  constexpr int TH_U = 16;  // candidates in flight per thread (the scans are latency-bound: one block)
  if (local) {  // ---- pass 1 (bits 30..19) of every candidate into LDS
    __syncthreads();
    for (int i0 = 0; i0 < total; i0 += TH_U * nt) {
      unsigned int v[TH_U];
#pragma unroll
      for (int u = 0; u < TH_U; u++) {
        const int i = i0 + u * nt + tid;
        v[u] = i < total ? __float_as_uint(a.cand[i]) : 0xffffffffu;
      }
#pragma unroll
      for (int u = 0; u < TH_U; u++)
        if (v[u] <= 0x7f800000u) atomicAdd(&hist1[v[u] >> 19], 1u);  // >= 0 and not NaN
    }
    __syncthreads();
  }
  // ---- pass 1's bin (the global histogram is re-zeroed for the next launch)
  unsigned int b1 = 0, kk = 0, n = 0;
  hist_pick(local ? hist1 : a.th_hist, HS_TH_BINS, !local, a.frameEnergyTHN, 0u, wsum, ctl, b1, kk, n);
  unsigned int ns = 0, srcn = 0;
  const unsigned int* src = nullptr;  // the survivors pass 3 reads (nullptr: re-scan the candidates)
  if (multi) {
    const unsigned int gs = a.th_nsurv[0], over = a.th_nsurv[1];
    for (int i = tid; i < 1024; i += nt) {
      hist2[i] = a.th_hist2[i];
      a.th_hist2[i] = 0u;
    }
    __syncthreads();
    if (tid == 0) {
      a.th_nsurv[0] = 0u;
      a.th_nsurv[1] = 0u;
    }
    if (over == 0u && gs <= (unsigned int)HS_TH_SURV) {
      src = a.th_surv;
      srcn = gs;
    }
  }
  if (n == 0) {
    if (tid == 0) a.frameTH[a.newest] = 12 * 12 * 8;
    return;
  }
  if (!multi) {
    // ---- pass 2: bits 18..9 of the candidates in bin b1; survivors compacted into LDS (order irrelevant: counts)
    for (int i0 = 0; i0 < total; i0 += TH_U * nt) {
      unsigned int v[TH_U];
#pragma unroll
      for (int u = 0; u < TH_U; u++) {
        const int i = i0 + u * nt + tid;
        v[u] = i < total ? __float_as_uint(a.cand[i]) : 0xffffffffu;
      }
#pragma unroll
      for (int u = 0; u < TH_U; u++)
        if (v[u] <= 0x7f800000u && (v[u] >> 19) == b1) {
          atomicAdd(&hist2[(v[u] >> 9) & 1023u], 1u);
          const unsigned int pos = atomicAdd(&ctl[2], 1u);
          if (pos < (unsigned int)cap) buf[pos] = v[u];
        }
    }
    __syncthreads();
    ns = ctl[2];
    if (ns <= (unsigned int)cap) {
      src = buf;
      srcn = ns;
    }
  }
  unsigned int b2 = 0, tot2 = 0;
  hist_pick(hist2, 1024, false, -1.f, kk, wsum, ctl, b2, kk, tot2);
  const unsigned int p2 = (b1 << 10) | b2;
  // ---- pass 3: bits 8..0 of the survivors with prefix p2
  if (src) {
    for (unsigned int i = tid; i < srcn; i += nt) {
      const unsigned int v = src[i];
      if ((v >> 9) == p2) atomicAdd(&hist3[v & 511u], 1u);
    }
  } else {
    for (int i0 = 0; i0 < total; i0 += TH_U * nt) {
      unsigned int v[TH_U];
#pragma unroll
      for (int u = 0; u < TH_U; u++) {
        const int i = i0 + u * nt + tid;
        v[u] = i < total ? __float_as_uint(a.cand[i]) : 0xffffffffu;
      }
#pragma unroll
      for (int u = 0; u < TH_U; u++)
        if (v[u] <= 0x7f800000u && (v[u] >> 9) == p2) atomicAdd(&hist3[v[u] & 511u], 1u);
    }
  }
  __syncthreads();
  unsigned int b3 = 0, k3 = 0, tot3 = 0;
  hist_pick(hist3, 512, false, -1.f, kk, wsum, ctl, b3, k3, tot3);
  if (tid == 0) {
    const float nth = sqrtf(__uint_as_float((p2 << 9) | b3));
    float th = nth * a.facMedian;
    th = 26.0f * a.constWeight + th * (1 - a.constWeight);
    th = th * th;
    th *= a.overallWeight * a.overallWeight;
    a.frameTH[a.newest] = th;
  }
}
__device__ __forceinline__ void red_energy_th_block(const HsRedArgs& a, unsigned int* sm) {
  th_select_block(a, sm, TH_CAP, false);
}

// the (R, C) entry (R <= C) of one (host, target) pair's 13x13 AccumulatorApprox block [calib 4 | xi 6 | a | b | r]
// from its octet of the host sums, oct[e * 8 + k] = entry e of lane k (the owner layout of acc_point)
__device__ __forceinline__ int top_oct_index(int R, int C) {
  int e, k;
  if (C < 8) { e = R; k = C; }                                     // Data (R, C <= 7): lane C, T[R]
  else if (C < 10) {
    if (R < 8) { e = C; k = R; }                                   // Data (R, 8 | 9): lane R, T[8 | 9]
    else { e = 10; k = (R == 8 && C == 8) ? 0 : (R == 8 ? 1 : 2); }  // (8,8) (8,9) (9,9): lanes 0 1 2, T[10]
  } else if (R < 10) {
    const int col = C - 10;                                        // TopRight (R, col)
    if (R < 8) { e = 11 + col; k = R; }
    else { e = 14; k = (R - 8) * 3 + col; }
  } else {                                                         // BotRight
    e = 15;
    k = R == 10 ? C - 10 : (R == 11 ? 2 + C - 10 : 5);
  }
  return e * 8 + k;
}
__device__ __forceinline__ double top_oct(const double* oct, int R, int C) { return oct[top_oct_index(R, C)]; }
// the octet offset of entry `ln` (lane (r, c)) of a pair's A88 block ([xi a b] x [xi a b], symmetric)
__device__ __forceinline__ int a88_index(int ln) {
  const int R = 4 + (ln >> 3), C = 4 + (ln & 7);
  return top_oct_index(min(R, C), max(R, C));
}

// 8x8 block products by one wave, lane (r, c): out = L M (L row r, M column c) / out = L M^T
__device__ __forceinline__ double mm8(const double* L, const double* M, int r, int c) {
  double s0 = 0.0, s1 = 0.0;
#pragma unroll
  for (int l = 0; l < 8; l += 2) {
    s0 = __builtin_fma(L[r * 8 + l], M[l * 8 + c], s0);
    s1 = __builtin_fma(L[r * 8 + l + 1], M[(l + 1) * 8 + c], s1);
  }
  return s0 + s1;
}
__device__ __forceinline__ double mm8t(const double* L, const double* M, int r, int c) {
  double s0 = 0.0, s1 = 0.0;
#pragma unroll
  for (int l = 0; l < 8; l += 2) {
    s0 = __builtin_fma(L[r * 8 + l], M[c * 8 + l], s0);
    s1 = __builtin_fma(L[r * 8 + l + 1], M[c * 8 + l + 1], s1);
  }
  return s0 + s1;
}
// L M R^T by one wave through the wave's LDS scratch (64 doubles)
__device__ __forceinline__ double sandwich8(const double* L, const double* M, const double* R, double* scr, int lane) {
  const int r = lane >> 3, c = lane & 7;
  scr[lane] = mm8(L, M, r, c);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const double v = mm8t(scr, R, r, c);
  __builtin_amdgcn_wave_barrier();
  return v;
}

constexpr int ST_NT = HS_STITCH_NT, ST_NW = ST_NT / 64;  // stitch block: 16 waves, one 8x8 term per wave at a time
constexpr int ST_LDS = 12288 + ST_NW * 64;  // doubles of the stitch block's LDS (the f == g frame block)
static_assert(2 * ST_LDS >= 1600 + TH_CAP, "the threshold select's LDS lives in the stitch block's scratch");
}  // namespace

// host sums of chunk q of host h (blockDim entries of the host's [ne][64] accumulators per block)
__device__ __forceinline__ void red_host_chunk(const HsRedArgs& a, int h, int q) {
  const int NE64 = a.ne * 64;
  const int e = q * (int)blockDim.x + (int)threadIdx.x;  // entry of the host's [ne][64] accumulators
  const int b0 = a.blk_begin[h], b1 = a.blk_begin[h + 1];
  if (e < NE64) {
    // the host's block partials in block order, fp64 (the reference sums its per-thread fp32 accumulators in
    // fp64); up to 64 loads in flight per batch (one batch for <= 64 blocks per host)
    double s = 0.0;
    if (b1 - b0 <= 32) {  // the headline's 32 blocks per host: one 32-wide batch (no clamped duplicate loads)
      float v[32];
#pragma unroll
      for (int u = 0; u < 32; u++) v[u] = a.part[(size_t)min(b0 + u, b1 - 1) * NE64 + e];
#pragma unroll
      for (int u = 0; u < 32; u++)
        if (b0 + u < b1) s += (double)v[u];
    } else {
      for (int bb = b0; bb < b1; bb += 64) {
        float v[64];
#pragma unroll
        for (int u = 0; u < 64; u++) v[u] = a.part[(size_t)min(bb + u, b1 - 1) * NE64 + e];
#pragma unroll
        for (int u = 0; u < 64; u++)
          if (bb + u < b1) s += (double)v[u];
      }
    }
    a.hostsum[(size_t)h * NE64 + e] = s;
  }
}

__global__ __launch_bounds__(256) void hs_k_reduce(HsRedArgs a) {
  if (a.stop && *a.stop) return;
  const int nred = a.nF * a.Q;
  const int b = blockIdx.x;
  if (a.hist_only) {  // multi-rank large windows: pass 1 over the all-gathered candidates
    red_th_hist_block(a, b);
    return;
  }
  HS_TRACE(a, 0);
  if (b == nred) { red_energy_block(a); HS_TRACE(a, 15); return; }
  if (b > nred) { red_th_hist_block(a, b - nred - 1); HS_TRACE(a, 15); return; }
  red_host_chunk(a, b / a.Q, b % a.Q);
  HS_TRACE(a, 15);
}

// the multi-block pass 2 alone (test hook hs_debug_threshold; production runs it inside the stitch launch)
__global__ __launch_bounds__(HS_STITCH_NT) void hs_k_th_pass2(HsRedArgs a) {
  __shared__ unsigned int sm[1600 + TH_CAP];
  if (a.stop && *a.stop) return;
  red_th_pass2_block(a, blockIdx.x, sm);
}

__global__ __launch_bounds__(HS_STITCH_NT) void hs_k_th_select(HsRedArgs a) {
  __shared__ unsigned int sm[1600 + TH_CAP];
  if (a.stop && *a.stop) return;
  red_energy_th_block(a, sm);
}

// stitchDoubleMT (Include/AccumulatedTopHessian.h:69-117, Include/AccumulatedSCHessian.h:70-111) with
// stitchDoubleInternal (Src/AccumulatedTopHessian.cpp:218-280, Src/AccumulatedSCHessian.cpp:54-133) in fp64, one
// block per output block:
//   frame block (f, g), f <= g: top  (f,f): sum_t adH[f,t] A[f,t] adH[f,t]^T + sum_h adT[h,f] A[h,f] adT[h,f]^T,
//                                     (f,g): adH[f,g] A[f,g] adT[f,g]^T + (adH[g,f] A[g,f] adT[g,f]^T)^T;
//                               Schur: sum over hosts h of host h's four-sandwich sum, which is A_h D_h A_h^T with
//                                     A_h(f, t) = [f = h] adH[h,t] + [f = t] adT[h,t]: host h not f, g contributes
//                                     adT[h,f] D_h(f,g) adT[h,g]^T, host f (Y_f(f,g) = sum_t1 adH[f,t1] D_f(t1,g))
//                                     Y_f adT[f,g]^T, host g adT[g,f] sum_t2 D_g(f,t2) adH[g,t2]^T (f == g: host f
//                                     sum_t1 adH[f,t1] sum_t2 D_f(t1,t2) adH[f,t2]^T);
//   calib x frame f: top adH / adT A84, Schur adH / adT accE, b adH / adT a8r and accEB;
//   calib x calib: A44 and accHcc, b a4r and accbc, summed over every host and pair.
// Every term is an 8x8 block formed by one wave (lane (r, c)) and kept in LDS; the terms of an output are summed
// in one fixed order (hosts, then targets), so the system is bit-reproducible.  The vector holds the upper
// triangle of HA - sc HSC (diagonal: HA (1 + lambda) - sc HSC; the solve adds the priors) and bA - bSC;
// `sep` HA | bA and HSC | bSC separately.
// The heavy part of a diagonal frame block (f, f): host f's own Schur term sum_t1 adH[f,t1] sum_t2 D_f(t1,t2)
// adH[f,t2]^T (7 terms of 8 products each), in a block of its own (the first nF blocks of the stitch launch) so the
// diagonal blocks' terms no longer share one CU's LDS bandwidth with the other 21 sandwiches: its sum goes to aux
// [f][64] (full 8x8), which the consumers fold into (f, f): out -= sc aux (the solve's prefetch, the host read-backs),
// sepS += aux.
__device__ void stitch_diag_schur(const HsStitchArgs& a, const int f, double* lds) {
  const int nF = a.nF;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, r = lane >> 3, c = lane & 7;
  const int NE64 = a.ne * 64;
  const double* HSf = a.hostsum + (size_t)f * NE64;
  double* aHf = lds;         // [8][64] adH[f, t]
  double* Dq = aHf + 512;    // [8][8][64] D_f(t1, t2)
  double* tS = Dq + 4096;    // [8][64] the term of t1
  double* scr = tS + 512;    // per-wave scratch [ST_NW][64]
  {  // one load batch: adjoints | D blocks (power-of-two strides; slots t >= nF or == f skipped)
    constexpr int SU = (512 + 4096 + ST_NT - 1) / ST_NT;
    double v[SU];
    int dst[SU];
#pragma unroll
    for (int u = 0; u < SU; u++) {
      const int q = tid + ST_NT * u;
      const double* src = a.adHost;
      int d = -1;
      if (q < 512) {
        const int t = q >> 6, ln = q & 63;
        if (t < nF) {
          src = a.adHost + (size_t)(f + nF * t) * 64 + ln;
          d = q;
        }
      } else if (q < 512 + 4096) {
        const int qd = q - 512, x1 = qd >> 9, x2 = (qd >> 6) & 7, ln = qd & 63, rr = ln >> 3, cc = ln & 7;
        if (x1 < nF && x2 < nF && x1 != f && x2 != f) {
          const int o1 = x1 - (x1 > f ? 1 : 0), o2 = x2 - (x2 > f ? 1 : 0);
          int base, ls, cs;
          if (a.exact) { base = (HS_E_TOP + o1 * 7 + o2) * 64; ls = 8; cs = 1; }
          else if (o1 <= o2) { base = (HS_E_TOP + dpair(o1, o2)) * 64; ls = 8; cs = 1; }
          else { base = (HS_E_TOP + dpair(o2, o1)) * 64; ls = 1; cs = 8; }
          src = HSf + base + rr * ls + cc * cs;
          d = 512 + qd;
        }
      }
      v[u] = *src;
      dst[u] = d;
    }
#pragma unroll
    for (int u = 0; u < SU; u++)
      if (dst[u] >= 0) lds[dst[u]] = v[u];
  }
  __syncthreads();
  HS_TRACE(a, 1);
  double* sw = scr + wv * 64;
  for (int x = wv; x < nF - 1; x += ST_NW) {
    const int y = x + (x >= f ? 1 : 0);
    double v0 = 0.0, v1 = 0.0;
#pragma unroll
    for (int t2 = 0; t2 < HS_MAXF; t2++) {  // unrolled, the skipped slots masked: the LDS reads issue together
      const double pv = mm8t(Dq + (y * 8 + t2) * 64, aHf + t2 * 64, r, c);
      const bool on = t2 < nF && t2 != f;
      if (t2 & 1) v1 = on ? v1 + pv : v1;
      else v0 = on ? v0 + pv : v0;
    }
    sw[lane] = v0 + v1;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    tS[y * 64 + lane] = mm8(aHf + y * 64, sw, r, c);
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  HS_TRACE(a, 2);
  if (tid < 64) {
    double vS[HS_MAXF];
#pragma unroll
    for (int i = 0; i < HS_MAXF; i++) vS[i] = tS[i * 64 + lane];
    double hf = 0.0;
#pragma unroll
    for (int t1 = 0; t1 < HS_MAXF; t1++) hf = (t1 < nF && t1 != f) ? hf + vS[t1] : hf;
    if (a.aux_out) a.aux_out[f * 64 + lane] = hf;
    if (a.aux_sep) a.aux_sep[f * 64 + lane] = hf;
  }
}

__device__ __forceinline__ void stitch_block(const HsStitchArgs& a, int j, double* lds) {
  const int nF = a.nF, n = 4 + 8 * nF, nn = n * n, SL = nn + n;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, r = lane >> 3, c = lane & 7;
  const int NE64 = a.ne * 64;
  const int ND = a.exact ? HS_ND_EXACT : HS_ND_PROD;
  const int oE = (HS_E_TOP + ND) * 64;  // accE / accEB / Hcc entries of a host sum
  const int nFB = nF * (nF + 1) / 2;
  HS_TRACE(a, 0);
  if (j < nF) {  // the first nF blocks: the diagonal blocks' host-f Schur terms
    stitch_diag_schur(a, j, lds);
    HS_TRACE(a, 15);
    return;
  }
  j -= nF;
  if (j == nFB + nF + 1) {  // setNewFrameEnergyTH for the next linearization, beside the stitch
    if (!a.red.skip_threshold) red_energy_th_block(a.red, reinterpret_cast<unsigned int*>(lds));
    HS_TRACE(a, 15);
    return;
  }
  if (j > nFB + nF + 1) {  // large windows: the select's pass 2, spread over np2 blocks (pass 3 runs after)
    red_th_pass2_block(a.red, j - (nFB + nF + 2), reinterpret_cast<unsigned int*>(lds));
    return;
  }
  auto adH = [&](int h, int t) { return a.adHost + (size_t)(h + nF * t) * 64; };
  auto adT = [&](int h, int t) { return a.adTarget + (size_t)(h + nF * t) * 64; };
  auto HS = [&](int h) { return a.hostsum + (size_t)h * NE64; };
  // D_h(t1, t2)[l][cc] at HS(h)[base + l ls + cc cs] (production stores t1 <= t2 only: D(t2, t1) = D(t1, t2)^T)
  auto Dat = [&](int h, int t1, int t2, int& base, int& ls, int& cs) {
    const int o1 = t1 - (t1 > h ? 1 : 0), o2 = t2 - (t2 > h ? 1 : 0);
    if (a.exact) { base = (HS_E_TOP + o1 * 7 + o2) * 64; ls = 8; cs = 1; }
    else if (o1 <= o2) { base = (HS_E_TOP + dpair(o1, o2)) * 64; ls = 8; cs = 1; }
    else { base = (HS_E_TOP + dpair(o2, o1)) * 64; ls = 1; cs = 8; }
  };
  double* out = a.out;
  double* sepA = a.sep;
  double* sepS = a.sep ? a.sep + SL : nullptr;
  auto put = [&](int R, int C, double ha, double hs, bool diag) {
    if (out) out[R * n + C] = diag ? ha * a.lambda1 - hs * a.sc : ha - hs * a.sc;
    if (sepA) {
      sepA[R * n + C] = ha;
      sepS[R * n + C] = hs;
    }
  };

  if (j < nFB) {
    // ------------------------------------------------------------ frame block (f, g), f <= g
    int f = 0, g = 0;
    {
      int q = j;
      while (q >= nF - f) { q -= nF - f; f++; }
      g = f + q;
    }
    double* aHf = lds;             // [8][64] adH[f, t]
    double* aTf = aHf + 512;       // [8][64] adT[h, f]
    double* aHg = aTf + 512;       // [8][64] adH[g, t]
    double* aTg = aHg + 512;       // [8][64] adT[h, g]
    double* Dx = aTg + 512;        // [8][64] D_h(f, g) by host h
    double* Dq = Dx + 512;         // f < g: [8][64] D_f(t1, g) by t1 | [8][64] D_g(f, t2) by t2 (f == g: unused)
    double* A8 = Dq + 4096;        // A88 blocks [16][64]: f < g: (f, g) | (g, f); f == g: (f, t) by t | (h, f) by 8 + h
    double* tS = A8 + 1024;        // Schur terms [16][64]
    double* tA = tS + 1024;        // top terms [16][64]
    double* scr = tA + 1024;       // per-wave scratch [ST_NW][64]
    // ---- loads: a flat table (adjoints | D blocks | octets), every thread's loads issued in one batch at
    // clamped addresses, then the LDS stores (a load per table row would be a dependent round trip each)
    {
      // table rows at power-of-two strides (slot index t < 8 = HS_MAXF; rows with t >= nF are skipped), so the
      // index math is shifts and masks, not runtime divisions
      const int nAdj = (f < g ? 4 : 2) * 512;        // [kind][t][64]
      const int nD = f < g ? 3 * 512 : 512;          // f < g: [kind][x][64]; f == g: Dx [h][64] (D_f: its own block)
      const int nOct = f < g ? 128 : 16 * 64;        // A88 blocks [slot][64], gathered from the pairs' octets
      const int total = nAdj + nD + nOct;
      constexpr int SU = (512 * 4 + 3 * 512 + 128 + ST_NT - 1) / ST_NT;  // the largest table: f < g
      double v[SU];
      int dst[SU];
#pragma unroll
      for (int u = 0; u < SU; u++) {
        const int q = tid + ST_NT * u;
        const double* src = a.adHost;
        int d = -1;
        if (q < nAdj) {  // aHf | aTf | aHg | aTg
          const int kind = q >> 9, t = (q >> 6) & 7, ln = q & 63;
          const bool host = (kind & 1) == 0;
          const int fg = kind < 2 ? f : g, hh = host ? fg : t, tt = host ? t : fg;
          if (t < nF) {
            src = (host ? a.adHost : a.adTarget) + (size_t)(hh + nF * tt) * 64 + ln;
            d = q;
          }
        } else if (q < nAdj + nD) {
          const int qd = q - nAdj, ln = qd & 63, rr = ln >> 3, cc = ln & 7;
          int h = -1, t1 = 0, t2 = 0;
          if (f < g) {
            const int kind = qd >> 9, x = (qd >> 6) & 7;
            if (x < nF) {
              if (kind == 0 && x != f && x != g) { h = x; t1 = f; t2 = g; d = (int)(Dx - lds) + x * 64 + ln; }
              if (kind == 1 && x != f) { h = f; t1 = x; t2 = g; d = (int)(Dq - lds) + x * 64 + ln; }
              if (kind == 2 && x != g) { h = g; t1 = f; t2 = x; d = (int)(Dq - lds) + 512 + x * 64 + ln; }
            }
          } else {
            const int x = qd >> 6;
            if (x < nF && x != f) { h = x; t1 = f; t2 = f; d = (int)(Dx - lds) + qd; }
          }
          if (h >= 0) {
            int base, ls, cs;
            Dat(h, t1, t2, base, ls, cs);
            src = HS(h) + base + rr * ls + cc * cs;
          }
        } else if (q < total) {
          const int qo = q - nAdj - nD, oi = qo >> 6, w = a88_index(qo & 63), e = w >> 3, k = w & 7;
          int hh = -1, tt = 0;
          if (f < g) {
            if (oi == 0) { hh = f; tt = g; } else { hh = g; tt = f; }
          } else {
            const int x = oi & 7;  // octet slots: (f, t) at t, (h, f) at 8 + h
            if (x < nF && x != f) {
              hh = oi < 8 ? f : x;
              tt = oi < 8 ? x : f;
            }
          }
          if (hh >= 0) {
            src = HS(hh) + e * 64 + tt * 8 + k;
            d = (int)(A8 - lds) + qo;
          }
        }
        v[u] = *src;
        dst[u] = d;
      }
#pragma unroll
      for (int u = 0; u < SU; u++)
        if (dst[u] >= 0) lds[dst[u]] = v[u];
    }
    __syncthreads();
    HS_TRACE(a, 1);
    double* sw = scr + wv * 64;
    if (f < g) {
      // terms: tS[h] for every host h (the host f / g terms in their host slot), tA[0] and tA[1]
      for (int h = wv; h < nF; h += ST_NW) {
        double v;
        if (h != f && h != g) {
          v = sandwich8(aTf + h * 64, Dx + h * 64, aTg + h * 64, sw, lane);  // adT[h,f] D_h(f,g) adT[h,g]^T
        } else if (h == f) {  // (sum_t1 adH[f,t1] D_f(t1, g)) adT[f,g]^T
          double y0 = 0.0, y1 = 0.0;
#pragma unroll
          for (int t1 = 0; t1 < HS_MAXF; t1++) {
            const double pv = mm8(aHf + t1 * 64, Dq + t1 * 64, r, c);
            const bool on = t1 < nF && t1 != f;
            if (t1 & 1) y1 = on ? y1 + pv : y1;
            else y0 = on ? y0 + pv : y0;
          }
          sw[lane] = y0 + y1;
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          v = mm8t(sw, aTg + f * 64, r, c);
          __builtin_amdgcn_wave_barrier();
        } else {  // adT[g,f] (sum_t2 D_g(f, t2) adH[g,t2]^T)
          double y0 = 0.0, y1 = 0.0;
#pragma unroll
          for (int t2 = 0; t2 < HS_MAXF; t2++) {
            const double pv = mm8t(Dq + 512 + t2 * 64, aHg + t2 * 64, r, c);
            const bool on = t2 < nF && t2 != g;
            if (t2 & 1) y1 = on ? y1 + pv : y1;
            else y0 = on ? y0 + pv : y0;
          }
          sw[lane] = y0 + y1;
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          v = mm8(aTf + g * 64, sw, r, c);
          __builtin_amdgcn_wave_barrier();
        }
        tS[h * 64 + lane] = v;
      }
      if (wv == ST_NW - 2) tA[lane] = sandwich8(aHf + g * 64, A8, aTg + f * 64, sw, lane);       // adH[f,g] A adT[f,g]^T
      if (wv == ST_NW - 1) tA[64 + lane] = sandwich8(aHg + f * 64, A8 + 64, aTf + g * 64, sw, lane);  // (g,f) pair, transposed below
      __syncthreads();
      HS_TRACE(a, 2);
      if (tid < 64) {
        double hs = 0.0;
#pragma unroll
        for (int h = 0; h < HS_MAXF; h++) {  // unrolled with masked slots: the LDS reads issue together
          const double v = tS[h * 64 + lane];
          hs = h < nF ? hs + v : hs;
        }
        const double ha = tA[lane] + tA[64 + c * 8 + r];
        put(4 + 8 * f + r, 4 + 8 * g + c, ha, hs, false);
      }
    } else {
      // Schur terms: tS[h] = adT[h,f] D_h(f,f) adT[h,f]^T (h != f); host f's own term (adH[f,t1] sum_t2 D_f(t1,t2)
      // adH[f,t2]^T, 56 products) is formed by block f of the launch (stitch_diag_schur) and folded in by the
      // consumers; top terms: tA[t] host pairs (f, t), tA[8 + h] target pairs (h, f).  The 21 two-product
      // sandwiches round-robin over the 16 waves; every term is formed by one wave
      const int nSmall = 3 * (nF - 1);
      for (int x = wv; x < nSmall; x += ST_NW) {
        const int yi = x % (nF - 1), kind = x / (nF - 1) == 0 ? 0 : (x / (nF - 1) == 1 ? 2 : 3);
        const int y = yi + (yi >= f ? 1 : 0);
        if (kind == 0) {
          tS[y * 64 + lane] = sandwich8(aTf + y * 64, Dx + y * 64, aTf + y * 64, sw, lane);
        } else if (kind == 2) {
          tA[y * 64 + lane] = sandwich8(aHf + y * 64, A8 + y * 64, aHf + y * 64, sw, lane);
        } else {
          tA[(8 + y) * 64 + lane] = sandwich8(aTf + y * 64, A8 + (8 + y) * 64, aTf + y * 64, sw, lane);
        }
      }
      __syncthreads();
      HS_TRACE(a, 2);
      if (tid < 64 && r <= c) {
        // hosts in order, host f's term its t1 partials in order; then the top terms.  Unrolled over the 8 slots
        // with the unused ones masked, so the 32 LDS reads issue together instead of one round trip per term
        double vS[HS_MAXF], vA[2 * HS_MAXF];
#pragma unroll
        for (int i = 0; i < 2 * HS_MAXF; i++) {
          if (i < HS_MAXF) vS[i] = tS[i * 64 + lane];
          vA[i] = tA[i * 64 + lane];
        }
        double hs = 0.0, ha = 0.0;
#pragma unroll
        for (int h = 0; h < HS_MAXF; h++) hs = (h < nF && h != f) ? hs + vS[h] : hs;  // host f: aux (folded later)
#pragma unroll
        for (int t = 0; t < HS_MAXF; t++) ha = (t < nF && t != f) ? ha + vA[t] : ha;
#pragma unroll
        for (int h = 0; h < HS_MAXF; h++) ha = (h < nF && h != f) ? ha + vA[HS_MAXF + h] : ha;
        put(4 + 8 * f + r, 4 + 8 * f + c, ha, hs, r == c);
      }
    }
  } else if (j < nFB + nF) {
    // ------------------------------------------------------------ calib x frame f, b of frame f
    const int f = j - nFB;
    double* aHf = lds;          // [8][64]
    double* aTf = aHf + 512;    // [8][64]
    double* oc = aTf + 512;     // [16][128]: (f, t) by t | (h, f) by 8 + h
    double* Ee = oc + 2048;     // [16][40]: accE (32, [k][c]) | accEB (8) of pair (f, t) by t | (h, f) by 8 + h
    double* pt = Ee + 640;      // [8][40] partials
    {  // flat load table, slots m < 16 (m < 8: pair (f, m), m >= 8: pair (m - 8, f)): adjoints [m][64] | octets
       // [m][128] | accE / accEB [m][40], one batch, power-of-two strides
      constexpr int nAdj = 16 * 64, nOct = 16 * 128, total = nAdj + nOct + 16 * 64;
      constexpr int SU = (total + ST_NT - 1) / ST_NT;
      double v[SU];
      int dst[SU];
#pragma unroll
      for (int u = 0; u < SU; u++) {
        const int q = tid + ST_NT * u;
        const double* src = a.adHost;
        int d = -1;
        if (q < nAdj) {
          const int m = q >> 6, ln = q & 63, t = m & 7;
          if (t < nF) {
            src = (m < 8 ? adH(f, t) : adT(t, f)) + ln;
            d = q;
          }
        } else if (q < nAdj + nOct) {
          const int qo = q - nAdj, m = qo >> 7, w = qo & 127, e = w >> 3, k = w & 7, t = m & 7;
          if (t < nF && t != f) {
            src = HS(m < 8 ? f : t) + e * 64 + (m < 8 ? t : f) * 8 + k;
            d = (int)(oc - lds) + qo;
          }
        } else if (q < total) {
          const int qe = q - nAdj - nOct, m = qe >> 6, ln = qe & 63, t = m & 7;
          if (t < nF && t != f && ln < 40) {
            const int k = ln < 32 ? ln >> 2 : ln - 32, cc = ln < 32 ? (ln & 3) : 4;
            src = HS(m < 8 ? f : t) + oE + cc * 64 + (m < 8 ? t : f) * 8 + k;  // accE [k][c] (4k + c), accEB [k]
            d = (int)(Ee - lds) + m * 40 + ln;
          }
        }
        v[u] = *src;
        dst[u] = d;
      }
#pragma unroll
      for (int u = 0; u < SU; u++)
        if (dst[u] >= 0) lds[dst[u]] = v[u];
    }
    __syncthreads();
    // thread (output o < 40, quarter q): o < 32: H(4 + 8f + rr, cc), o >= 32: b(4 + 8f + rr); pairs m = q, q + 4, ..
    if (tid < 160) {
      const int o = tid % 40, q = tid / 40;
      const int rr = o < 32 ? o >> 2 : o - 32, cc = o < 32 ? (o & 3) : -1;
      double ha = 0.0, hs = 0.0;
      for (int m = q; m < 16; m += 4) {
        const int t = m & 7;
        if (t >= nF || t == f) continue;
        const double* L = (m < 8 ? aHf : aTf) + t * 64 + rr * 8;
        const double* octm = oc + m * 128;
        const double* Em = Ee + m * 40;
        double x = 0.0, y = 0.0;
#pragma unroll
        for (int k = 0; k < 8; k++) {
          const double tv = cc >= 0 ? top_oct(octm, cc, 4 + k) : top_oct(octm, 4 + k, 12);  // A84[k][cc] | a8r[k]
          const double ev = cc >= 0 ? Em[k * 4 + cc] : Em[32 + k];                        // accE[k][cc] | accEB[k]
          x = __builtin_fma(L[k], tv, x);
          y = __builtin_fma(L[k], ev, y);
        }
        ha += x;
        hs += y;
      }
      pt[q * 40 + o] = ha;
      pt[160 + q * 40 + o] = hs;
    }
    __syncthreads();
    if (tid < 40) {
      const int rr = tid < 32 ? tid >> 2 : tid - 32, cc = tid < 32 ? (tid & 3) : -1;
      const double ha = ((pt[tid] + pt[40 + tid]) + pt[80 + tid]) + pt[120 + tid];
      const double hs = ((pt[160 + tid] + pt[200 + tid]) + pt[240 + tid]) + pt[280 + tid];
      if (cc >= 0) {
        put(cc, 4 + 8 * f + rr, ha, hs, false);
      } else {
        if (out) out[nn + 4 + 8 * f + rr] = ha - hs;
        if (sepA) {
          sepA[nn + 4 + 8 * f + rr] = ha;
          sepS[nn + 4 + 8 * f + rr] = hs;
        }
      }
    }
  } else {
    // ------------------------------------------------------------ calib x calib (A44, accHcc) and calib b (a4r, accbc)
    double* pt = lds;  // [8 hosts][20] top sums | [8][20] Schur
    if (tid < 160) {
      const int o = tid % 20, h = tid / 20;
      double ta = 0.0, ts = 0.0;
      if (h < nF) {
        const double* src = HS(h);
        for (int t = 0; t < nF; t++) {
          if (t == h) continue;
          // A44 (R, C <= 3): lane C, T[R]; a4r (R, 12): TopRight (R, r) -> lane R, T[13]
          const int R = o < 16 ? min(o >> 2, o & 3) : o - 16, C = o < 16 ? max(o >> 2, o & 3) : 0;
          ta += o < 16 ? src[R * 64 + t * 8 + C] : src[13 * 64 + t * 8 + R];
        }
        ts = src[oE + 5 * 64 + o];  // accHcc (lanes 0..15) / accbc (16..19) of host h
      }
      pt[h * 20 + o] = ta;
      pt[160 + h * 20 + o] = ts;
    }
    __syncthreads();
    if (tid < 20) {
      double ta = 0.0, ts = 0.0;
      for (int h = 0; h < nF; h++) {
        ta += pt[h * 20 + tid];
        ts += pt[160 + h * 20 + tid];
      }
      if (tid < 16) {
        const int rr = tid >> 2, cc = tid & 3;
        if (rr <= cc) put(rr, cc, ta, ts, rr == cc);
      } else {
        if (out) out[nn + tid - 16] = ta - ts;
        if (sepA) {
          sepA[nn + tid - 16] = ta;
          sepS[nn + tid - 16] = ts;
        }
      }
    }
  }
  HS_TRACE(a, 15);
}

// hs_k_result's work (below) for the stitch launch's extra block: every input was written by earlier launches
__device__ void stitch_result_block(const HsStitchArgs& a) {
  const int k = a.res_k;
  double* out = a.res_out;
  for (int i = threadIdx.x; i < k; i += blockDim.x) out[i] = a.res_elog[i];
  if (threadIdx.x == 0) {
    out[k] = a.red.sysE[0];
    out[k + 1] = (double)a.res_st->status;
    out[a.res_slot] = (double)k;
  }
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(out + a.res_slot + 1), a.res_seq, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(ST_NT) void hs_k_stitch(HsStitchArgs a) {
  __shared__ double lds[ST_LDS];
  __shared__ int s_last;
  // the fp64 adjoints' stamp (HS_ADJ_STAMP), requested before the block's work and compared after it
  // (a launch stopped by the device-side break stitches nothing and checks nothing)
  const bool run = !(a.red.stop && *a.red.stop);
  const bool chk = run && a.status && blockIdx.x == 0 && threadIdx.x == 0;
  double sH = 0.0, sT = 0.0;
  unsigned int ex = 0u;
  if (chk) {
    sH = a.adHost[HS_ADJ_STAMP];
    sT = a.adTarget[HS_ADJ_STAMP];
    ex = *a.adj_expect;
  }
  if (run) stitch_block(a, blockIdx.x, lds);
  if (chk) {
    if (sH != (double)ex || sT != (double)ex) atomicOr(a.status, (int)HS_STATUS_STALE64);
    else atomicAnd(a.status, ~(int)HS_STATUS_STALE64);
  }
  if (!a.res_out) return;
  // the GN loop call's results: written by the launch's last block to retire (a ticket), after every block's stores
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    s_last = atomicAdd(a.res_ticket, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (!s_last) return;
  __threadfence();
  if (threadIdx.x == 0) atomicExch(a.res_ticket, 0u);
  stitch_result_block(a);
}


// =====================================================================================================
// solve + step (fp64), one workgroup of 256 threads
// =====================================================================================================
#include "hs_solve_ldlt.h"
using namespace hs_solve;

namespace {
constexpr int SOLVE_NT = HS_SOLVE_NT;  // 8 waves: the LDLT's panel wave + 7 waves of trailing half-tiles

}  // namespace


// Solves (L D L^T) y = z in place for the permuted, scaled system of one GN step (n = 4 + 8 nF, a multiple
// of 4): right-looking LDLT in 4-column blocks with one-block look-ahead, ONE workgroup barrier per block.
//  wave 0 (the panel wave): lane l owns row l + 4 for the whole factorization and carries its (L D) entries of
//    the last panel and its forward-substituted rhs in registers.  In phase k it applies block k's rank-4
//    update to its row of column block k + 1, takes the updated 4x4 diagonal block from lanes 4k .. 4k+3
//    (readlane), factors it uniformly and reduces its row to the (L D) / L entries of panel k + 1; it publishes
//    only L (LT), the pivots and the diagonal rows' rhs;
//  waves 1-7: every lower 4x4 tile right of the next panel (register-resident, one per lane) takes block
//    k's rank-4 update (its L D rows formed from LT and the pivots); the owners of column block k + 2 publish it
//    (row-major, 32 B per row) for the panel wave's next phase.
// The panel chain (the critical path) thus overlaps the trailing update.  fp64 throughout, FMA-contracted,
// reciprocals by v_rcp_f64 + 2 Newton steps: the solve is checked against the oracle's Eigen-order LDLT by
// tolerance (the LDLT is parity-unpinned), not bitwise.  The pivot order is applied by the
// caller.  Then D^-1 and the backward substitution (one wave, 4x4 diagonal blocks solved uniformly).
//   M  : the permuted system (row-major, stride n), read only
//   LT : L transposed, LT[i * LSTR + k] = L(k, i); MUST be zero on entry (its upper part stays zero)
//   W  : scratch of 26 * HS_MAXDIM doubles;  yv : right-hand side in, solution out
// the multi-rank select block of the solve / combine launches lives in the solve's LDS matrix A
constexpr int SOLVE_TH_CAP = 2 * HS_MAXDIM * HS_MAXDIM - 1600 - HS_TH_BINS;
static_assert(SOLVE_TH_CAP >= 1024, "survivor space of the multi-rank select");
constexpr int LDLT_SCRATCH = 26 * HS_MAXDIM;

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
// pivot and the reduced entries come from lanes 0-3 by readlane.  The later columns are reduced as
// a(jp) -= (a(j) q(jp, j)) / d(j), the product formed beside the reciprocal, so the critical path per column is
// one readlane, the reciprocal (+ Newton step) and one multiply-add; L = a(j) / d(j) and its row mask stay off
// it (rows l <= j of the diagonal block take garbage updates of entries no later column reads).  A diagonal row
// l takes L entries only for j < l.
__device__ __forceinline__ void panel_coop(const double a[4], double yr, int l, Panel4& P, PanelOut& o, int base = 0) {
  double pr[4] = {a[0], a[1], a[2], a[3]};
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const double d = readlane_f64(pr[j], base + j);
    const double dinv = rcp_f64(d);
    const double ydj = readlane_f64(yr, base + j);
    P.d[j] = d;
    P.dinv[j] = dinv;
    P.yd[j] = ydj;
#pragma unroll
    for (int jp = j + 1; jp < 4; jp++) P.q[jp][j] = readlane_f64(pr[j], base + jp);
    const double lj = pr[j] * dinv;
    o.lw[j] = l > j ? pr[j] : 0.0;
    o.ls[j] = l > j ? lj : 0.0;
#pragma unroll
    for (int jp = j + 1; jp < 4; jp++) pr[jp] = __builtin_fma(-(pr[j] * P.q[jp][j]), dinv, pr[jp]);
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
    for (int jp = j + 1; jp < 4; jp++) pr[jp] = __builtin_fma(-(pr[j] * P.q[jp][j]), P.dinv[j], pr[jp]);
    yr = __builtin_fma(-o.ls[j], P.yd[j], yr);
  }
  o.yr = yr;
}

// publishes one panel row r (l = r - K0): its (L D) entries LW (zero for the diagonal rows, which take no part in
// the trailing update), its L entries into LT (which the next phase reads back), and the substituted rhs; lane
// j < 4 also stores pivot j
__device__ __forceinline__ void panel_row_store(const PanelOut& o, const Panel4& P, int r, int l, int K0, double* LWn,
                                                double* LT, double* Dv, double* yf, double* yv) {
  constexpr int MD = HS_MAXDIM;
  const bool diag = l < 4;
#pragma unroll
  for (int j = 0; j < 4; j++) {
    LWn[j * MD + r] = diag ? 0.0 : o.lw[j];
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
                                                   long long* trace, int dbg = 0) {
  constexpr int MD = HS_MAXDIM;
  static_assert((HS_MAXDIM / 4 - 2) * (HS_MAXDIM / 4 - 1) / 2 <= SOLVE_NT - 64, "one trailing tile per lane");
  static_assert(LSTR % 2 == 0, "16 B aligned LT groups");
  const int nb = n >> 2;
  double* PBq = W;            // [2][MD][4] column block k+1 before block k's update, row-major (32 B per row)
  double* LWb = W + 8 * MD;   // [4][MD] (L D) of panel 0 (the panel wave's initial carry)
  double* Dv = W + 24 * MD;   // [MD] pivots
  double* yf = W + 25 * MD;   // [MD] forward-substituted rhs of the diagonal rows
  const bool pw = tid < 64;   // the panel wave
  // waves 1-7: trailing tile (tr, tc), tc >= 2, row-major over the lower triangle
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
    for (int c = 0; c < 4; c++) PBq[4 * MD + tid * 4 + c] = M[tid * n + 4 + c];  // column block 1
  // prologue: panel 0 over rows 0 .. n-1 by the panel wave (lanes 0-3 also take rows 64 .. n-1)
  if (pw) {
    const int r = min(tid, n - 1);
    double a4[4];
#pragma unroll
    for (int c = 0; c < 4; c++) a4[c] = M[r * n + c];
    Panel4 P;
    PanelOut o;
    panel_coop(a4, yv[r], tid, P, o);
    if (tid < n) panel_row_store(o, P, tid, tid, 0, LWb, LT, Dv, yf, yv);
    if (tid + 64 < n) {
      const int r2 = tid + 64;
#pragma unroll
      for (int c = 0; c < 4; c++) a4[c] = M[r2 * n + c];
      panel_row_uniform(a4, yv[r2], P, o);
      panel_row_store(o, P, r2, r2, 0, LWb, LT, Dv, yf, yv);
    }
  }
  __syncthreads();
  // the panel wave's carry: lane l owns row rw = l + 4 (clamped; rows >= n are never stored)
  const int rw = min(tid + 4, n - 1);
  double lwc[4] = {0.0, 0.0, 0.0, 0.0}, ycar = 0.0;
  if (pw) {
#pragma unroll
    for (int j = 0; j < 4; j++) lwc[j] = LWb[j * MD + rw];
    ycar = yv[rw];
  }
  for (int k = 0; k + 1 < nb; k++) {
    const int K0 = 4 * (k + 1);
    const double* LSk = LT + 4 * k * LSTR;  // LSk[j * LSTR + row] = L(row, 4k + j)
    if (trace && tid == 0 && k == 4) trace[16] = clock64();
    if (pw) {  // panel k+1: lane l owns row rw; the diagonal rows are lanes 4k .. 4k+3
      const double* PBc = PBq + ((k + 1) & 1) * 4 * MD;
      const double4 pb = *reinterpret_cast<const double4*>(PBc + rw * 4);
      double a4[4] = {pb.x, pb.y, pb.z, pb.w};
      double lsd[4][4];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const double4 q4 = *reinterpret_cast<const double4*>(LSk + j * LSTR + K0);  // L(K0 + c, 4k + j)
        lsd[0][j] = q4.x;
        lsd[1][j] = q4.y;
        lsd[2][j] = q4.z;
        lsd[3][j] = q4.w;
      }
#pragma unroll
      for (int j = 0; j < 4; j++)  // block k's update of this row of column block k+1
#pragma unroll
        for (int c = 0; c < 4; c++) a4[c] = __builtin_fma(-lwc[j], lsd[c][j], a4[c]);
      const int l = tid - 4 * k;  // row rw - K0 (< 0: a row of an earlier panel, inert)
      Panel4 P;
      PanelOut o;
      panel_coop(a4, ycar, l, P, o, 4 * k);
      if (l >= 0 && tid + 4 < n) {
#pragma unroll
        for (int j = 0; j < 4; j++) LT[(K0 + j) * LSTR + rw] = o.ls[j];  // zero on and above the diagonal
        if (l < 4) {
          Dv[rw] = l == 0 ? P.d[0] : l == 1 ? P.d[1] : l == 2 ? P.d[2] : P.d[3];
          yf[rw] = o.yr;
        }
      }
#pragma unroll
      for (int j = 0; j < 4; j++) lwc[j] = o.lw[j];
      ycar = o.yr;
      if (trace && tid == 0 && k == 4) trace[17] = clock64();
    } else if (tile && tc >= k + 2) {  // block k's rank-4 update of a trailing tile
      double lw[4][4], ls[4][4], dk[4];
#pragma unroll
      for (int j = 0; j < 4; j++) dk[j] = Dv[4 * k + j];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const double4 r4 = *reinterpret_cast<const double4*>(LSk + j * LSTR + 4 * tr);
        const double4 c4 = *reinterpret_cast<const double4*>(LSk + j * LSTR + 4 * tc);
        lw[0][j] = r4.x * dk[j];
        lw[1][j] = r4.y * dk[j];
        lw[2][j] = r4.z * dk[j];
        lw[3][j] = r4.w * dk[j];
        ls[0][j] = c4.x;
        ls[1][j] = c4.y;
        ls[2][j] = c4.z;
        ls[3][j] = c4.w;
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
          *reinterpret_cast<double4*>(PBn + (4 * tr + i) * 4) = make_double4(v[i][0], v[i][1], v[i][2], v[i][3]);
      }
    }
    if (trace && tid == 64 && k == 4) trace[18] = clock64();
    __syncthreads();
    if (trace && tid == 0 && k == 4) trace[19] = clock64();
    if (trace && tid == 0 && k == 4) trace[12] = wall_clock64();
    if (trace && tid == 0 && k == 8) trace[14] = wall_clock64();  // mid-factorization checkpoint
  }
  ldlt_backward(LT, W, yv, n, tid, trace);
}

// FrameOptimizationData::setState's scaling (Include/Frame.h:151-170)
__device__ __forceinline__ void scale_state(const double s[10], double o[10]) {
#pragma unroll
  for (int i = 0; i < 3; i++) o[i] = hs::SCALE_XI_TRANS * s[i];
#pragma unroll
  for (int i = 3; i < 6; i++) o[i] = hs::SCALE_XI_ROT * s[i];
  o[6] = hs::SCALE_A * s[6];
  o[7] = hs::SCALE_B * s[7];
  o[8] = hs::SCALE_A * s[8];
  o[9] = hs::SCALE_B * s[9];
}

// test hook (hs_debug_se3): the product SE3 of hs_se3.h and the solve's step forms on the device, one element per
// thread.  op 0 exp | 1 se3_exp_step (the doStep's series exp) | 2 log | 3 Adj | 4 product | 5 inverse |
// 6 se3_mul_step (the doStep's product) | 7 rotation matrix.  in: [n][14] (tangent6 or data7, second data7 at +7),
// out: [n][36].
__global__ void hs_k_debug_se3(int op, int n, const double* in, double* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double* x = in + 14 * i;
  double* o = out + 36 * i;
  hs::SE3 r;
  switch (op) {
    case 0: r = hs::SE3::exp(x); r.toData(o); break;
    case 1: r = se3_exp_step(x); r.toData(o); break;
    case 2: hs::SE3::fromData(x).log(o); break;
    case 3: hs::SE3::fromData(x).Adj(o); break;
    case 4: r = hs::SE3::fromData(x) * hs::SE3::fromData(x + 7); r.toData(o); break;
    case 5: r = hs::SE3::fromData(x).inverse(); r.toData(o); break;
    case 6: r = se3_mul_step(hs::SE3::fromData(x), hs::SE3::fromData(x + 7)); r.toData(o); break;
    default: hs::SE3::fromData(x).rotationMatrix(o); break;
  }
}

__global__ __launch_bounds__(SOLVE_NT) void hs_k_solve(HsSolveArgs a) {
  __shared__ double A[HS_MAXDIM * HS_MAXDIM];  // the scaled system S H S (row-major, stride n)
  __shared__ __align__(16) double B[LDLT_SCRATCH];  // LDLT scratch
  __shared__ __align__(16) double LT[HS_MAXDIM * LSTR];  // L^T of the factorization (zeroed at entry)
  __shared__ double Nf[2 * HS_MAXDIM * HS_NNS];  // nullspace factors N | Npi (prefetched at entry)
  __shared__ double tk[2 * HS_NNS];
  __shared__ double Sv[HS_MAXDIM], xs[HS_MAXDIM], yv[HS_MAXDIM];
  __shared__ double dgv[2 * HS_MAXDIM], dgm[2 * HS_MAXDIM];  // raw diagonal | b, and HM's diagonal | bM
  __shared__ float xF[HS_MAXDIM];
  __shared__ double AUXs[HS_MAXF * 64];  // the diagonal blocks' host-f Schur terms (stitch aux_out)
  __shared__ int s_it;
  // the window state lives in LDS for the whole kernel: every field is touched by dependent scalar code
  // (steps, SE3 updates, precalc), which would otherwise pay a global-memory round trip per access
  __shared__ __align__(16) unsigned char st_raw[sizeof(HsDevState)];
  static_assert(sizeof(HsDevState) % 8 == 0, "HsDevState is copied as 8-byte words");
  HsDevState* st = reinterpret_cast<HsDevState*>(st_raw);
  const int tid = threadIdx.x, nt = SOLVE_NT;
  if (a.brk && a.reset_it < 0 && blockIdx.x == 0) {
    const HsDevState* g = a.st;
    if (g->stop || (g->log_count > 0 && g->canbreak && g->iteration - 1 >= a.minOpt)) {
      if (tid == 0) a.st->stop = 1;  // every thread stops whichever value of stop it read
      return;
    }
  }
  if (blockIdx.x == 1) {  // setNewFrameEnergyTH over the (gathered) candidates, beside the solve (th_local 1: the
                          // whole select; 2: pass 3 of the multi-block select, passes 1 and 2 ran before)
    th_select_block(a.th, reinterpret_cast<unsigned int*>(A), SOLVE_TH_CAP, a.th_local == 1);
    return;
  }
  HS_TRACE(a, 0);
  if (a.trace && threadIdx.x == 0) a.trace[24] = clock64();  // shader clock (effective-clock probe)
  // entry prefetch: every global input (window state, system vector, HM / bM, nullspace factors, energies) is
  // requested into registers before the first LDS store, so the kernel pays ONE memory round trip here
  constexpr int ST_WORDS = (int)(sizeof(HsDevState) / 8);
  constexpr int ST_NU = (ST_WORDS + SOLVE_NT - 1) / SOLVE_NT;
  constexpr int NF_NU = (2 * HS_MAXDIM * HS_NNS + SOLVE_NT - 1) / SOLVE_NT;
  const bool solve = (a.flags & HS_SOLVE) != 0;
  const int nF = a.nF, n = 4 + 8 * nF, nn = n * n;
  uint2 stw[ST_NU];
  {
    const uint2* gst = reinterpret_cast<const uint2*>(a.st);
#pragma unroll
    for (int u = 0; u < ST_NU; u++) stw[u] = gst[min(tid + u * SOLVE_NT, ST_WORDS - 1)];
  }
  // the system vector: thread slots q = tid + 512 u of the packed upper triangle (then b), read at their place
  // (r, c) of the n x n layout.  The triangle is walked as an (n / 2) x (n + 1) rectangle (n = 4 + 8 nF is even):
  // rectangle row i holds triangle row i (n - i entries) followed by triangle row n - 1 - i (i + 1 entries), so
  // (r, c) follows from one reciprocal and selects (24-bit multiplies: full-rate integer ops)
  constexpr int NUQ = (hs_nt(HS_MAXDIM) + HS_MAXDIM + SOLVE_NT - 1) / SOLVE_NT;
  const int ntri = hs_nt(n);
  const float w1inv = 1.0f / (float)(n + 1);
  int qaddr[NUQ], qr[NUQ], qc[NUQ];
#pragma unroll
  for (int u = 0; u < NUQ; u++) {
    const int q = tid + SOLVE_NT * u;
    const int i = (int)(((float)q + 0.5f) * w1inv);  // exact: (q + 0.5) / (n + 1) stays >= 0.5 / 69 from an integer
    const int j = q - __mul24(i, n + 1);
    const bool upper = j < n - i;
    const int r = upper ? i : n - 1 - i, c = upper ? i + j : j - 1;
    const bool tri = q < ntri, isb = !tri && q < ntri + n;
    qr[u] = tri ? r : (isb ? -2 : -1);
    qc[u] = tri ? c : (isb ? q - ntri : -1);
    qaddr[u] = tri ? __mul24(r, n) + c : (isb ? nn + (q - ntri) : -1);
  }
  // the diagonal frame blocks' host-f Schur terms after the energies (hs_k_stitch's aux_out, [nF][64]): staged into
  // LDS (one coalesced load per thread, in the batch below); entry (qr, qc) of a block (f, f) folds in
  // aux [f][qr - 4 - 8 f][qc - 4 - 8 f] (aaddr: its LDS index, -1: none)
  const int AUX0 = nn + n + 3;
  int aaddr[NUQ];
#pragma unroll
  for (int u = 0; u < NUQ; u++) {
    const int fr = (qr[u] - 4) >> 3, fc = (qc[u] - 4) >> 3;
    aaddr[u] = (qr[u] >= 4 && fr == fc) ? fr * 64 + ((qr[u] - 4) & 7) * 8 + ((qc[u] - 4) & 7) : -1;
  }
  double gs[NUQ], hmq[NUQ], hml[NUQ], nfv[NF_NU], axv = 0.0;
  // energy, sum |idepth|, #points as vector loads (a uniform address would make them scalar loads, whose wait
  // shares lgkmcnt with the LDS stores below)
  int vz;
  asm volatile("v_mov_b32 %0, 0" : "=v"(vz));
  double sysE0 = a.sysE[vz], sysE1 = a.sysE[vz + 1], sysE2 = a.sysE[vz + 2];
  // the fp32 adjoints' stamps (HS_ADJ_STAMP), checked after the counters' reset below
  const unsigned int sHF = a.chk_adj ? reinterpret_cast<const unsigned int*>(a.adHostF)[HS_ADJ_STAMP + vz] : 0u;
  const unsigned int sTF = a.chk_adj ? reinterpret_cast<const unsigned int*>(a.adTargetF)[HS_ADJ_STAMP + vz] : 0u;
  const unsigned int sEx = a.chk_adj ? a.adj_expect[vz] : 0u;
  const bool hasHM = a.HM != nullptr;
  if (solve) {
    axv = a.sys[AUX0 + min(tid, nF * 64 - 1)];
    if (hasHM) {  // HM at the entry (r, c) and at its mirror (c, r) (the latter for HM delta's rows), bM for b
#pragma unroll
      for (int u = 0; u < NUQ; u++) {
        gs[u] = a.sys[max(qaddr[u], 0)];
        hmq[u] = qr[u] == -2 ? a.bM[qc[u]] : a.HM[qr[u] >= 0 ? qaddr[u] : 0];
        hml[u] = a.HM[qr[u] >= 0 ? __mul24(qc[u], n) + qr[u] : 0];
      }
    } else {  // no marginalization prior (a uniform branch): only bM is read beside the system
#pragma unroll
      for (int u = 0; u < NUQ; u++) {
        gs[u] = a.sys[max(qaddr[u], 0)];
        hmq[u] = qr[u] == -2 ? a.bM[qc[u]] : 0.0;
        hml[u] = 0.0;
      }
    }
#pragma unroll
    for (int u = 0; u < NF_NU; u++) nfv[u] = a.Nproj[min(tid + u * SOLVE_NT, 2 * n * HS_NNS - 1)];
  }
  HS_TRACE(a, 1);  // every load of the prefetch issued
  if (a.gsys) {  // multi-rank: the gathered vectors (a.sys = rank 0's) summed in rank order, the raw sums kept
    const double* ge = a.gsys + nn + n;
    sysE0 = ge[0];  // rank 0's (a.sysE is this rank's own)
    sysE1 = ge[1];
    sysE2 = ge[2];
    for (int r = 1; r < a.nranks; r++) {
      sysE0 += ge[r * a.gstride];
      sysE1 += ge[r * a.gstride + 1];
      sysE2 += ge[r * a.gstride + 2];
    }
    if (tid < 3) a.sys_out[nn + n + tid] = tid == 0 ? sysE0 : (tid == 1 ? sysE1 : sysE2);
    if (solve) {
#pragma unroll
      for (int u = 0; u < NUQ; u++) {
        const int ad = max(qaddr[u], 0);
        for (int r = 1; r < a.nranks; r++) gs[u] += a.gsys[r * a.gstride + ad];
        if (qaddr[u] >= 0) a.sys_out[ad] = gs[u];
      }
      for (int r = 1; r < a.nranks; r++) axv += a.gsys[r * a.gstride + AUX0 + min(tid, nF * 64 - 1)];
      if (tid < nF * 64) a.sys_out[AUX0 + tid] = axv;
    }
  }
  // L^T must be zero on entry to the LDLT: stored while the prefetch above is in flight (with a marginalization
  // prior, LT first holds HM for the per-row HM delta products and is zeroed after them)
  if (solve && !hasHM)
    for (int idx = tid; idx < HS_MAXDIM * LSTR; idx += nt) LT[idx] = 0.0;
  {
    uint2* ls = reinterpret_cast<uint2*>(st_raw);
#pragma unroll
    for (int u = 0; u < ST_NU; u++)
      if (tid + u * SOLVE_NT < ST_WORDS) ls[tid + u * SOLVE_NT] = stw[u];
  }
  HS_TRACE(a, 9);  // the window state arrived (thread 0's words)
  if (solve && tid < nF * 64) AUXs[tid] = axv;
  if (solve) {  // the raw diagonal (+ HM's) and b (+ bM) entries to LDS for the per-row scaling below
#pragma unroll
    for (int u = 0; u < NUQ; u++) {
      if (qr[u] >= 0 && qr[u] == qc[u]) {
        dgv[qc[u]] = gs[u];
        dgm[qc[u]] = hmq[u];
      } else if (qr[u] == -2) {
        dgv[HS_MAXDIM + qc[u]] = gs[u];
        dgm[HS_MAXDIM + qc[u]] = hmq[u];
      }
      if (hasHM && qr[u] >= 0) {
        LT[qr[u] * LSTR + qc[u]] = hmq[u];
        LT[qc[u] * LSTR + qr[u]] = hml[u];
      }
    }
#pragma unroll
    for (int u = 0; u < NF_NU; u++)
      if (tid + u * SOLVE_NT < 2 * n * HS_NNS) Nf[tid + u * SOLVE_NT] = nfv[u];
  }
  HS_TRACE(a, 11);  // thread 0's system entries arrived
  __syncthreads();
  HS_TRACE(a, 8);
  if (tid == 0) {
    if (a.reset_it >= 0) {  // the first launch of a GN loop call (no separate host-to-device copy of the counters)
      st->iteration = a.reset_it;
      st->status = 0;
      st->log_count = 0;
      st->stop = 0;
    }
    s_it = a.iteration >= 0 ? a.iteration : st->iteration;
    if (a.chk_adj)
      st->status = (st->status & ~(int)HS_STATUS_STALE32) | ((sHF != sEx || sTF != sEx) ? HS_STATUS_STALE32 : 0);
  }
  const double lambda = 1e-5;  // SOLVER_FIX_LAMBDA

  if (solve) {
    if (tid == 0 && a.energy_log) {
      a.energy_log[st->log_count] = sysE0;
      st->log_count = st->log_count + 1;
    }
    // HFinal = (HL + HM + HA) diag (1+lambda) - HSC / (1+lambda) and b = (bL + (bM + HM delta)) + (bA - bSC)
    // (Src/EnergyFunctional.cpp:728-764): the system vector carries HA - sc HSC with the diagonal
    // HA (1+lambda) - sc HSC and bA - bSC (hs_k_stitch); the priors HL / bL (the frames' prior and the calib prior,
    // Src/AccumulatedTopHessian.cpp:269-279) and the marginalization prior HM / bM are added here, each entry by
    // the thread that loaded it.  The owner of a diagonal entry also forms the scaling S = 1 / sqrt(diag + 10)
    // (:799-801).
    const double lam1 = 1 + lambda;
    auto delta = [&](int q) -> double {  // the reference's prior deltas: calib value - value_zero (as float), frame delta
      return q < 4 ? (double)(float)st->calib.value_minus_value_zero[q] : st->frames[(q - 4) >> 3].delta[(q - 4) & 7];
    };
    // per row q (one thread each): the assembled diagonal, the scaling S = 1 / sqrt(diag + 10) (reciprocal square
    // root + Newton: rounding-level from the IEEE quotient) and the scaled right-hand side
    if (tid < n) {
      const int q = tid;
      const double pr = q < 4 ? a.initialCalibHessian : st->frames[(q - 4) >> 3].prior[(q - 4) & 7];
      // (frame rows: the diagonal block's host-f Schur term folded in first, as for the off-diagonal entries)
      const double dq = q < 4 ? dgv[q] : dgv[q] - a.aux_sc * AUXs[((q - 4) >> 3) * 64 + ((q - 4) & 7) * 9];
      const double hv = dq + (pr + dgm[q]) * lam1;
      const double sq = rsqrt_step(hv + 10);
      Sv[q] = sq;
      A[q * n + q] = sq * hv * sq;
      const double bl = q < 4 ? a.initialCalibHessian * delta(q)
                              : pr * st->frames[(q - 4) >> 3].delta_prior[(q - 4) & 7];
      double hmd = 0.0;  // (HM delta)_q in the reference's order, HM's row q staged in LT
      if (hasHM)
        for (int k = 0; k < n; k++) hmd += LT[q * LSTR + k] * delta(k);
      yv[q] = sq * ((bl + (dgm[HS_MAXDIM + q] + hmd)) + dgv[HS_MAXDIM + q]);
    }
    __syncthreads();
    HS_TRACE(a, 7);
    if (hasHM)  // LT's HM rows are read: zero for the LDLT (the barrier after the off-diagonal pass orders it)
      for (int idx = tid; idx < HS_MAXDIM * LSTR; idx += nt) LT[idx] = 0.0;
    // the scaled off-diagonal entries S H S, mirrored from the upper triangle
#pragma unroll
    for (int u = 0; u < NUQ; u++) {
      const int r = qr[u], c = qc[u];
      if (r >= 0 && r != c) {
        const double gf = aaddr[u] >= 0 ? gs[u] - a.aux_sc * AUXs[aaddr[u]] : gs[u];
        const double w = Sv[r] * (gf + hmq[u]) * Sv[c];
        A[r * n + c] = w;
        A[c * n + r] = w;
      }
    }
    __syncthreads();
    HS_TRACE(a, 2);
    // scaled LDLT without pivoting: the damped system is symmetric positive definite, for which the
    // factorization is backward stable without pivoting; Eigen's LDLT (Src/EnergyFunctional.cpp:801) pivots on
    // the diagonal, which changes x by rounding only (the LDLT is parity-unpinned; tests bound x by
    // the reference's own 1- vs 8-thread spread)
    if ((a.dbg & 8) && a.trace && tid == 0) a.trace[20] = clock64();
    for (int rep = 0; rep < ((a.dbg & 8) ? 2 : 1); rep++) {
      ldlt_solve_blocked(A, LT, B, yv, n, tid, a.trace, a.dbg);
      __syncthreads();
      if ((a.dbg & 8) && a.trace && tid == 0) a.trace[21 + rep] = clock64();
    }
    __syncthreads();
    HS_TRACE(a, 3);
    if (tid < n) xs[tid] = Sv[tid] * yv[tid];
    __syncthreads();
    HS_TRACE(a, 4);
    if ((a.dbg & 32) && a.trace && tid == 0) a.trace[26] = clock64();
    // xAd (EnergyFunctional::resubstituteF_MT's per-pair adjoint products) for the granular path only: in the
    // fused GN loop (HS_APPLY) the linearize kernel forms its host's xAd itself from lastX.  The fp32 adjoints
    // are requested here so their latency overlaps orthogonalize.
    const bool wxad = !(a.flags & HS_APPLY);
    float adh[2][8], adt[2][8];
    if (wxad) {  // a uniform branch: the fused path issues none of these loads (a barrier would wait for them)
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
    }
    if (s_it >= 2) {  // SOLVER_ORTHOGONALIZE_X_LATER: x -= P x, P = (N Npi^T + Npi N^T) / 2 (orthogonalize)
      // t1 = Npi^T x, t2 = N^T x: 14 dot products over n, 16 lanes each (at most 5 terms per lane, then an xor
      // tree: a short dependent chain)
      const int d = tid >> 4, part = tid & 15;
      constexpr int LEN = (HS_MAXDIM + 15) / 16;
      if (d < 2 * HS_NNS) {
        const double* col = Nf + (d < HS_NNS ? n * HS_NNS : 0);  // Npi for t1, N for t2
        const int kk = d % HS_NNS;
        double sacc = 0.0;
#pragma unroll
        for (int cc = 0; cc < LEN; cc++) {
          const int c = part * LEN + cc;
          const int cl = min(c, n - 1);
          const double t = __builtin_fma(col[cl * HS_NNS + kk], xs[cl], sacc);
          sacc = c < n ? t : sacc;
        }
        // the 16 lanes' butterfly in DPP (no LDS round trip): xor 1, xor 2 (quad_perm), then the 8- and 16-lane
        // mirrors, which pair the already-equal quads and halves
        sacc += dpp_f64<0xB1>(sacc);
        sacc += dpp_f64<0x4E>(sacc);
        sacc += dpp_f64<0x141>(sacc);
        sacc += dpp_f64<0x140>(sacc);
        if (part == 0) tk[d] = sacc;
      }
      __syncthreads();
      if ((a.dbg & 32) && a.trace && tid == 0) a.trace[27] = clock64();
    }
    // resubstituteF_MT: frame / calib steps, xAd, cstep; row q's thread first applies its own orthogonalize
    // update (x_q -= (P x)_q), so no barrier separates the two
    if (tid < n) {
      const int q = tid;
      double xv = xs[q];
      if (s_it >= 2) {
        double s1 = 0.0, s2 = 0.0;
#pragma unroll
        for (int kk = 0; kk < HS_NNS; kk++) {
          s1 = __builtin_fma(Nf[q * HS_NNS + kk], tk[kk], s1);
          s2 = __builtin_fma(Nf[n * HS_NNS + q * HS_NNS + kk], tk[HS_NNS + kk], s2);
        }
        xv -= 0.5 * (s1 + s2);
      }
      if (!isfinite(xv)) st->status |= HS_STATUS_NONFINITE;
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
    if ((a.dbg & 32) && a.trace && tid == 0) a.trace[28] = clock64();
    if (tid < 4) st->cstep[tid] = xF[tid];
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const int o = tid + k * nt;
      if (wxad && o < nF * nF * 8) {
        const int pair = o >> 3, hh = pair / nF, tt = pair - hh * nF;  // xAd[nF*h + t]
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int rr = 0; rr < 8; rr++) s1 += xF[4 + 8 * hh + rr] * adh[k][rr];
#pragma unroll
        for (int rr = 0; rr < 8; rr++) s2 += xF[4 + 8 * tt + rr] * adt[k][rr];
        a.xAd[o] = s1 + s2;
      }
    }
    if ((a.dbg & 32) && a.trace && tid == 0) a.trace[29] = clock64();
    HS_TRACE(a, 5);
  }
  __syncthreads();
  if (a.flags & HS_APPLY) {
    // backupState + doStepFromBackup(1, 1, 1, 1, 1) + setPrecalcValues (Src/FullSystemOptimize.cpp:171-314) in two
    // register-resident stages: lane 64 + f (wave 1) steps frame f (new state, its scaled copy, PRE_worldToCam
    // = exp(scaled xi) * evalPT and its inverse: frame_pose_stage) into LDS; after one barrier lane (h, t) of wave 0
    // reads both frames' poses and forms the pair's FrameFramePrecalc::set (pair_precalc_stage) while wave 1 writes
    // the frames and the calib back.  PRE_RTll_0 / PRE_tTll_0 depend on evalPT only and stay as uploaded.
    const int np = nF * nF;
    double* fx = B;  // LDLT scratch (free now): per frame PRE_worldToCam (7) | PRE_camToWorld (7) | scaled a, b
    double cv[4];
#pragma unroll
    for (int q = 0; q < 4; q++) cv[q] = st->calib.value[q] + 1.0f * st->calib.step[q];
    if ((a.dbg & 16) && a.trace && tid == 0) a.trace[20] = clock64();
    // stage 1 on wave 1 (lane 64 + f): frame f's new pose into LDS; its write-back waits until after the barrier,
    // beside wave 0's pair stage
    const int fw = tid - 64;
    const bool fl = fw >= 0 && fw < nF;
    double sh[10], ns[10], sc[10];
    hs::SE3 PW, PC;
    if (fl) {
      const hs::FrameH& F = st->frames[fw];
#pragma unroll
      for (int q = 0; q < 10; q++) {
        sh[q] = F.state[q];
        ns[q] = sh[q] + 1.0 * F.step[q];
      }
      scale_state(ns, sc);
      double ev[7];
      F.evalPT.toData(ev);
      frame_pose_stage(sc, hs::SE3::fromData(ev), fx + 16 * fw, &PW, &PC);
    }
    if (tid >= 128 && tid < 192) {  // canbreak on wave 2, beside the frame stage (it reads the steps only)
      // lane f forms frame f's terms (fp64, the reference's expressions), lane 0 adds them in frame order into the
      // float sums (float += double, as the reference's loop): no chain of dependent LDS reads
      const int f = min(tid - 128, nF - 1);
      const double* sp = st->frames[f].step;
      const double tA = sp[6] * sp[6], tB = sp[7] * sp[7];
      const double tT = sp[0] * sp[0] + sp[1] * sp[1] + sp[2] * sp[2];
      const double tR = sp[3] * sp[3] + sp[4] * sp[4] + sp[5] * sp[5];
      float sumA = 0, sumB = 0, sumT = 0, sumR = 0;
      for (int g = 0; g < nF; g++) {
        sumA += readlane_f64(tA, g);
        sumB += readlane_f64(tB, g);
        sumT += readlane_f64(tT, g);
        sumR += readlane_f64(tR, g);
      }
      const float nfr = (float)nF;
      sumA /= nfr; sumB /= nfr; sumR /= nfr; sumT /= nfr;
      const float sumNID = sysE2 > 0 ? (float)(sysE1 / sysE2) : 0.f;
      const float th = a.thOptIterations;
      if (tid == 128) {
        st->canbreak = sqrtf(sumA) < 0.0005 * th && sqrtf(sumB) < 0.00005 * th && sqrtf(sumR) < 0.00005 * th &&
                       sqrtf(sumT) * sumNID < 0.00005 * th;
        st->iteration = s_it + 1;
      }
    }
    // the pair stage's inputs that no stage writes, read before the barrier
    const float vsf[4] = {(float)(hs::SCALE_F * cv[0]), (float)(hs::SCALE_F * cv[1]), (float)(hs::SCALE_C * cv[2]),
                          (float)(hs::SCALE_C * cv[3])};
    float exh = 0.f, ext = 0.f;
    double sz7 = 0.0;
    if (tid < np) {
      const int hh = tid / nF, tt = tid - hh * nF;
      exh = st->frames[hh].ab_exposure;
      ext = st->frames[tt].ab_exposure;
      sz7 = st->frames[hh].state_zero[7];
    }
    if ((a.dbg & 16) && a.trace && tid == 0) a.trace[22] = clock64();
    __syncthreads();
    if ((a.dbg & 16) && a.trace && tid == 0) a.trace[23] = clock64();
    if (tid == 192) {  // the calib on wave 3, beside the pair stage (every lane read cv before the barrier)
      hs::CalibH& cal = st->calib;
#pragma unroll
      for (int q = 0; q < 4; q++) cal.value_backup[q] = cal.value[q];
      cal.setValue(cv);
      st->dcal = cal.device();
    }
    if (tid < np) {
      const int hh = tid / nF, tt = tid - hh * nF;
      pair_precalc_stage(fx + 16 * hh, fx + 16 * tt, exh, ext, sz7, vsf, a.pre[tid]);
    }
    if (fl) {  // frame fw: backupState, setState, setDeltaF's delta / delta_prior
      hs::FrameH& F = st->frames[fw];
#pragma unroll
      for (int q = 0; q < 10; q++) {
        F.state_backup[q] = sh[q];
        F.state[q] = ns[q];
        F.state_scaled[q] = sc[q];
      }
      F.PRE_worldToCam = PW;
      F.PRE_camToWorld = PC;
#pragma unroll
      for (int q = 0; q < 8; q++) {
        F.delta[q] = ns[q] - F.state_zero[q];
        F.delta_prior[q] = ns[q] - 0.0;
      }
    }
    if ((a.dbg & 16) && a.trace && tid == 0) a.trace[21] = clock64();
    HS_TRACE(a, 6);
    if (tid == 0) HS_TRACE(a, 10);
  }
  __syncthreads();
  {  // write the window state back: every word by the whole workgroup (the window's frames; HS_MAXF slots beyond
     // them are untouched by the solve and skipped)
    constexpr int F0 = (int)(offsetof(HsDevState, frames) / 8), FW1 = (int)(sizeof(hs::FrameH) / 8);
    constexpr int FW = (int)(sizeof(HsDevState::frames) / 8), SW = (int)(sizeof(HsDevState) / 8);
    static_assert(offsetof(HsDevState, frames) % 8 == 0 && sizeof(hs::FrameH) % 8 == 0, "word copies");
    const int fend = F0 + nF * FW1;
    const uint2* ls = reinterpret_cast<const uint2*>(st_raw);
    uint2* gs = reinterpret_cast<uint2*>(a.st);
    constexpr int NU = (SW + SOLVE_NT - 1) / SOLVE_NT;
#pragma unroll
    for (int u = 0; u < NU; u++) {
      const int i = tid + u * SOLVE_NT;
      if (i < SW && (i < fend || i >= F0 + FW)) gs[i] = ls[i];
    }
  }
  if (a.trace && threadIdx.x == 0) a.trace[25] = clock64();
  HS_TRACE(a, 15);
}

// multi-rank exchange without a following solve (granular calls, the last GN iteration, optimize's break test):
// block 0 sums the gathered system vectors in rank order into sys_out (the solve's prefetch forms the same sums),
// block 1 (th_local) selects the threshold over the gathered candidates
__global__ __launch_bounds__(SOLVE_NT) void hs_k_combine(HsSolveArgs a) {
  __shared__ double A[HS_MAXDIM * HS_MAXDIM];
  if (blockIdx.x == 1) {
    th_select_block(a.th, reinterpret_cast<unsigned int*>(A), SOLVE_TH_CAP, a.th_local == 1);
    return;
  }
  if (!a.gsys) return;  // test hook: the select block alone
  const int n = 4 + 8 * a.nF, len = n * n + n + 3 + 64 * a.nF;  // + the diagonal blocks' host-f Schur terms
  for (int i = threadIdx.x; i < len; i += SOLVE_NT) {
    double s = a.gsys[i];
    for (int r = 1; r < a.nranks; r++) s += a.gsys[r * a.gstride + i];
    a.sys_out[i] = s;
  }
}

// brk (optimize's device-side break): the iterations done are the solves that ran (st->log_count), written to
// out[done_slot]; st->stop is cleared for the next call
__global__ void hs_k_result(const double* elog, int k, const double* sysE, HsDevState* st, double* out, int brk,
                            int done_slot, unsigned long long seq) {
  if (brk) k = min(k, st->log_count);
  for (int i = threadIdx.x; i < k; i += blockDim.x) out[i] = elog[i];
  if (threadIdx.x == 0) {
    out[k] = sysE[0];
    out[k + 1] = (double)st->status;
    out[done_slot] = (double)k;
    if (brk) st->stop = 0;
  }
  __syncthreads();  // every thread's log stores before the done word (the release below orders them)
  if (threadIdx.x == 0)
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(out + done_slot + 1), seq, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
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

__global__ void hs_k_reset_res(int n8, uint8_t* st, uint8_t* act, float* en, float* nen) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n8) {
    st[i] = HS_RES_IN;
    act[i] = 0;
    en[i] = 0.f;
    nen[i] = 0.f;
  }
}

// EnergyFunctional::setDeltaF (Src/EnergyFunctional.cpp:128-152) in fp32: adHTdeltaF[h + nF t] = delta_h^T adHostF +
// delta_t^T adTargetF (each dot product in index order), cDeltaF = (float) calib.value_minus_value_zero.  One thread
// per (pair, entry).
__global__ void hs_k_marg_delta(const HsDevState* st, const float* adHF, const float* adTF, float* adHTd) {
  const int nF = st->nF, o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o < nF * nF * 8) {
    const int idx = o >> 3, q = o & 7, h = idx % nF, t = idx / nF;
    float s1 = 0, s2 = 0;
    for (int r = 0; r < 8; r++) s1 += (float)(st->frames[h].state[r] - st->frames[h].state_zero[r]) * adHF[idx * 64 + r * 8 + q];
    for (int r = 0; r < 8; r++) s2 += (float)(st->frames[t].state[r] - st->frames[t].state_zero[r]) * adTF[idx * 64 + r * 8 + q];
    adHTd[o] = s1 + s2;
  } else if (o < nF * nF * 8 + 4) {
    adHTd[o] = (float)st->calib.value_minus_value_zero[o - nF * nF * 8];
  }
}

// EnergyFunctional::marginalizePointsF's prior update (Src/EnergyFunctional.cpp:596-606): HM += w (M - Msc),
// bM += w (Mb - Mbsc) with M | Mb = HA | bA and Msc | Mbsc = HSC | bSC of the separate stitch (upper triangles,
// mirrored; HSC's diagonal blocks plus their host-f Schur terms), the same fp64 operations as the host form
__global__ void hs_k_marg_update(const double* sep, const double* sep_aux, double* HM, double* bM, int nF, int SL,
                                 double w) {
  const int n = 4 + 8 * nF, o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o < n * n) {
    const int r = o / n, q = o - r * n, lo = min(r, q), hi = max(r, q);
    const double m = sep[lo * n + hi];
    double msc = sep[SL + lo * n + hi];
    if (lo >= 4 && (lo - 4) / 8 == (hi - 4) / 8) {
      const int f = (lo - 4) / 8;
      msc += sep_aux[f * 64 + (lo - 4 - 8 * f) * 8 + (hi - 4 - 8 * f)];
    }
    HM[o] += w * (m - msc);
  } else if (o < n * n + n) {
    const int r = o - n * n;
    bM[r] += w * (sep[n * n + r] - sep[SL + n * n + r]);
  }
}

// fix = 1: the optimize tail's setEvalPT of the newest frame first; then (both) every frame pair's precalc and
// adjoints (System::setPrecalcValues, EnergyFunctional::setAdjointsF) from the device state
__global__ __launch_bounds__(64) void hs_k_fix_frames(HsDevState* st, HsPrecalc* pre, double* adH, double* adT,
                                                      float* adHF, float* adTF, hs_params P, int fix,
                                                      unsigned int seq, unsigned int* expect) {
  const int nF = st->nF, tid = threadIdx.x;
  if (fix && tid == 0) {  // newStateZero = 0 except segment(6, 2) = the newest frame's a / b; setEvalPT(PRE_worldToCam, .)
    hs::FrameH& f = st->frames[nF - 1];
    double nsz[10] = {0, 0, 0, 0, 0, 0, f.state[6], f.state[7], 0, 0};
    f.evalPT = f.PRE_worldToCam;
    f.setState(nsz);
    for (int i = 0; i < 10; i++) f.state_zero[i] = nsz[i];  // setStateZero's nullspaces: on the host, when read
    f.takeData(P);
  }
  __syncthreads();
  for (int idx = tid; idx < nF * nF; idx += blockDim.x) {  // idx = h + t nF (adjoints); precalc at h nF + t
    const int h = idx % nF, t = idx / nF;
    const hs::FrameH& H = st->frames[h];
    const hs::FrameH& T = st->frames[t];
    pre[h * nF + t] = hs::make_precalc(H, T, st->calib);
    double AH[64], AT[64];
    hs::make_adjoints(H, T, AH, AT);
    for (int i = 0; i < 64; i++) {
      adH[(size_t)idx * 64 + i] = AH[i];
      adT[(size_t)idx * 64 + i] = AT[i];
      adHF[(size_t)idx * 64 + i] = (float)AH[i];
      adTF[(size_t)idx * 64 + i] = (float)AT[i];
    }
  }
  if (tid == 0) {  // this upload's stamp (HS_ADJ_STAMP), checked by the stitch / solve launches that read the adjoints
    adH[HS_ADJ_STAMP] = (double)seq;
    adT[HS_ADJ_STAMP] = (double)seq;
    reinterpret_cast<unsigned int*>(adHF)[HS_ADJ_STAMP] = seq;
    reinterpret_cast<unsigned int*>(adTF)[HS_ADJ_STAMP] = seq;
    *expect = seq;
  }
}

// test hook: spins for `ticks` of the 100 MHz wall clock and exits (every wave reaches the bound), standing in for a
// collective whose peer stalls: the host's bounded wait (wait_stream) must return HS_ERR_RCCL while it runs
__global__ void hs_k_debug_stall(long long ticks) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

// image slot texels (I, dx, dy, |grad|^2) -> packed (I, dx, dy) triplets for hs_k_lin8's taps: 12 instead of 16 bytes
// per texel, so a pattern row's taps span fewer cache lines
__global__ void hs_k_pack_texels(long long n, const float4* src, float* dst3) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 t = src[i];
  dst3[3 * i + 0] = t.x;
  dst3[3 * i + 1] = t.y;
  dst3[3 * i + 2] = t.z;
}

__global__ void hs_k_apply_step(int n, const float* step, float* idepth, float* idepth_zero) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < n) {
    const float nid = idepth[p] + 1.0f * step[p];
    idepth[p] = nid;
    idepth_zero[p] = nid;
  }
}

// EnergyFunctional::calcLEnergyPt's point term (Src/EnergyFunctional.cpp:289-347) for the window's points: per
// IndexThreadReduce chunk of 50 points an Accumulator11 sums deltaF^2 priorF in fp32 (at most 50 updates: no
// shiftUp; finish() adds three zero lanes), and the chunk values add up in fp64 in chunk order -- the
// single-thread reference's result.  One block; the window holds no linearized residuals (the marginalization
// pass consumes them), so the residual terms are empty.
__global__ __launch_bounds__(256) void hs_k_lenergy(int n, const float* idepth, const float* idepth_zero,
                                                    const float* priorF, float* chunk, double* out) {
  const int tid = threadIdx.x;
  const int nc = (n + 49) / 50;
  for (int c = tid; c < nc; c += 256) {
    float A = 0.f;
    for (int i = 50 * c; i < min(n, 50 * c + 50); i++) {
      const float dF = idepth[i] - idepth_zero[i];
      A += dF * dF * priorF[i];
    }
    chunk[c] = A;
  }
  __syncthreads();
  if (tid == 0) {
    double s = 0.0;
    for (int c = 0; c < nc; c++) s += (double)chunk[c];
    out[0] = s;
  }
}
