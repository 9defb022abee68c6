// hs_refine_kernels.hip — gfx950 kernel of H-SLAM's initializer refinement DirectRefinement (SURVEY.md §8f
// rank 4, the second Accumulator9 user).
//
//   hs_k_refine_step   one LM iteration of DirectRefinement::Refine (Src/Initializer.cpp:1412-1564) per launch,
//                      grid = ceil(n / 32) blocks of 256 threads: 8 lanes per point, one lane per pattern pixel.
//     prologue   (the point's leader lane) applyStep (:2188-2205) + optReg (:2229-2270) of the previous pass if it
//                was accepted, then doStep (:2155-2186) with the increment the previous launch solved for;
//                resetPoints (:1897-1924) in the first launch
//     pass       calcResAndGS (:1926-2153): every lane projects / samples / differentiates its pixel; the leader
//                folds its group's 8 values in pattern order (energy, maxstep, JbBuffer_new: bit-identical to the
//                reference's sequential loop, including the prefix before the first failing pixel), decides
//                isGood_new and adds its acc9SC row (updateSingleWeighted order) and calcEC terms (:2207-2227);
//                the lanes of good points add their pixel's 9x9 acc9 products
//     reduction  fixed-order LDS sums (acc9 over each wave's lanes, then the 4 waves; acc9SC / E / calcEC over the
//                block's 32 points) -> block partials
//                (release fence + acq_rel ticket) -> the last block to take the ticket acquires and sums the partials in block
//                order (no block waits on another)
//     LM         the last block: the sums unpacked by 45 threads; thread 0 the accept test and the lambda / fails /
//                snapped bookkeeping; the block copies H -> Hm and builds the scaled 6x6 system; thread 0 the
//                fixAffine fp32 LDLT step, SE3 exp * refToNew and the next pass's constants; or done
//   The host enqueues launches in batches and polls `done`; launches after it return at entry.  A final launch
//   applies the last accepted step.  Per-point state stays in HBM (structure of arrays); the
//   JbBuffer / JbBuffer_new swap is a plane-index flip carried in the control block.
//
// Per-point arithmetic follows the reference's fp32 operation order (fp contraction off).  The normal-equation
// and energy sums are fixed-order parallel reductions (the reference sums sequentially in 4 SSE lanes): those
// compare within tolerance.
#pragma clang fp contract(off)
#include <hip/hip_runtime.h>

#include <cfloat>

#include "hs_refine_kernels.h"

namespace {

constexpr int RB = 256;             // threads per block
constexpr int RW = RB / 64;         // waves per block
constexpr int NACC = 45;            // upper triangle of the 9x9 [J | r] system
constexpr int NX = 12;              // per-lane values folded by the leader: e, maxstep, dp_j * dd (8), r * dd, dd * dd
__constant__ int kPat[8][2] = {{0, -2}, {-1, -1}, {1, -1}, {-2, 0}, {0, 0}, {2, 0}, {-1, 1}, {0, 2}};

__device__ __forceinline__ float3 ref_interp33(const float4* __restrict__ img, float x, float y, int w) {
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
// getInterpolatedElement31 of the first frame; the base texel index is clamped to the buffer (the reference
// reads outside it, undefined behaviour, exactly where the clamp acts)
__device__ __forceinline__ float ref_interp31(const float4* __restrict__ img, float x, float y, int w, int h) {
  int ix = (int)x, iy = (int)y;
  float dx = x - ix, dy = y - iy, dxdy = dx * dy;
  long b = (long)ix + (long)iy * w;
  const long hi = (long)w * h - w - 2;
  b = b < 0 ? 0 : (b > hi ? hi : b);
  const float4* bp = img + b;
  return dxdy * bp[1 + w].x + (dy - dxdy) * bp[w].x + (dx - dxdy) * bp[1].x + (1 - dx - dy + dxdy) * bp[0].x;
}

// Vec8f dot in Eigen's vectorized order (lane-wise halves, then (l0 + l2) + (l1 + l3))
__device__ __forceinline__ float dot8(const float* a, const float* b) {
  float s[4];
#pragma unroll
  for (int l = 0; l < 4; l++) s[l] = a[l] * b[l] + a[l + 4] * b[l + 4];
  return (s[0] + s[2]) + (s[1] + s[3]);
}

#define REF_TRACE(slot)                                                                        \
  do {                                                                                         \
    if (a.trace && threadIdx.x == 0) a.trace[(size_t)blockIdx.x * 16 + (slot)] = wall_clock64(); \
  } while (0)

// thread 0's LDS workspace for the LM step (dynamically indexed arrays in private memory would live in scratch)
struct RefWork {
  float Hn[64], bn[8], Hsn[64], bsn[8];  // this pass's H_out / b_out / H_out_sc / b_out_sc
  float H6[36], bl[8], x6[8];
};

// Eigen::LDLT<Matrix<float,6,6>> (diagonal pivoting, left-looking) + solve, one thread, the factor in registers
__device__ __forceinline__ void ldlt6f_solve(const float* __restrict__ A, const float* __restrict__ rhs, float* __restrict__ x) {
  float dg[6];
  int pm[6];
#pragma unroll
  for (int i = 0; i < 6; i++) {
    dg[i] = fabsf(A[i * 6 + i]);
    pm[i] = i;
  }
#pragma unroll
  for (int k = 0; k < 6; k++) {
    float best = dg[k];
    int bi = k;
#pragma unroll
    for (int j = k + 1; j < 6; j++)
      if (dg[j] > best) { best = dg[j]; bi = j; }
#pragma unroll
    for (int j = k + 1; j < 6; j++)
      if (j == bi) {
        const float td = dg[k]; dg[k] = dg[j]; dg[j] = td;
        const int tp = pm[k]; pm[k] = pm[j]; pm[j] = tp;
      }
  }
  float M[6][6], y[6], D[6];
#pragma unroll
  for (int i = 0; i < 6; i++) {
#pragma unroll
    for (int j = 0; j < 6; j++) M[i][j] = A[pm[i] * 6 + pm[j]];
    y[i] = rhs[pm[i]];
  }
#pragma unroll
  for (int k = 0; k < 6; k++) {
    float temp[6];
#pragma unroll
    for (int j = 0; j < k; j++) temp[j] = D[j] * M[k][j];
    float s = 0;
#pragma unroll
    for (int j = 0; j < k; j++) s += M[k][j] * temp[j];
    M[k][k] -= s;
#pragma unroll
    for (int i = k + 1; i < 6; i++) {
      float t = 0;
#pragma unroll
      for (int j = 0; j < k; j++) t += M[i][j] * temp[j];
      M[i][k] -= t;
    }
    const float d = M[k][k];
    D[k] = d;
    if (fabsf(d) > FLT_MIN) {
#pragma unroll
      for (int i = k + 1; i < 6; i++) M[i][k] /= d;
    }
  }
#pragma unroll
  for (int i = 0; i < 6; i++)
#pragma unroll
    for (int k = 0; k < i; k++) y[i] = y[i] - M[i][k] * y[k];
#pragma unroll
  for (int i = 0; i < 6; i++) y[i] = fabsf(D[i]) > FLT_MIN ? y[i] / D[i] : 0.0f;
#pragma unroll
  for (int i = 5; i >= 0; i--)
#pragma unroll
    for (int j = i + 1; j < 6; j++) y[i] = y[i] - M[j][i] * y[j];
#pragma unroll
  for (int i = 0; i < 6; i++) x[pm[i]] = y[i];
}

// the LM step of Refine (Src/Initializer.cpp:1447-1466) from the control block's Hm / Hs / bm / bs / lambda.
// prep (threads 0..35 of the last block): Hl = H with the diagonal * (1 + lambda), minus Hsc / (1 + lambda),
// then wM Hl wM * (0.01 / (w h)); fixAffine reads the top-left 6x6 block and the first 6 entries of bl only
__device__ __forceinline__ void lm_solve_prep(const HsRefArgs& a, const HsRefCtl* C, RefWork* W, int t) {
  const float wM[8] = {1.0f, 1.0f, 1.0f, 0.5f, 0.5f, 0.5f, 10.0f, 1000.0f};  // SCALE_XI_ROT x3, _TRANS x3, A, B
  const float scl = 0.01f / (a.W * a.H);
  const float lambda = C->lambda;
  const float il = 1 / (1 + lambda);
  if (t < 36) {
    const int r = t / 6, c = t - 6 * r;
    float h = C->Hm[r * 8 + c];
    if (r == c) h *= (1 + lambda);
    h -= C->Hs[r * 8 + c] * il;
    W->H6[t] = ((wM[r] * h) * wM[c]) * scl;
  } else if (t < 44) {
    const int r = t - 36;
    W->bl[r] = (wM[r] * (C->bm[r] - C->bs[r] * il)) * scl;
  }
}

// tail (thread 0): the 6x6 LDLT, inc, Tn = exp(inc) * T, affn and the constants of the pass at Tn
__device__ __forceinline__ void lm_solve_tail(const HsRefArgs& a, HsRefCtl* C, RefWork* W) {
  const float wM[6] = {1.0f, 1.0f, 1.0f, 0.5f, 0.5f, 0.5f};
  REF_TRACE(11);
  ldlt6f_solve(W->H6, W->bl, W->x6);  // fixAffine = true
  REF_TRACE(12);
  double incd[6];
#pragma unroll
  for (int k = 0; k < 6; k++) {
    C->inc[k] = -(wM[k] * W->x6[k]);
    incd[k] = (double)C->inc[k];
  }
  C->inc[6] = C->inc[7] = 0.f;
  double T[7], Tn[7];
#pragma unroll
  for (int q = 0; q < 7; q++) T[q] = C->T[q];
  const hs::SE3 nw = hs::SE3::exp(incd) * hs::SE3::fromData(T);
  nw.toData(Tn);
#pragma unroll
  for (int q = 0; q < 7; q++) C->Tn[q] = Tn[q];
  double affn[2] = {C->aff[0] + C->inc[6], C->aff[1] + C->inc[7]};
  C->affn[0] = affn[0];
  C->affn[1] = affn[1];
  REF_TRACE(13);
  HsRefPass pc;
  hs_ref_pass_consts(Tn, affn, a.Ki, a.n, &pc);
  C->pc = pc;
  REF_TRACE(14);
}

enum { LM_COPY = 1, LM_SOLVE = 2, LM_OUT = 4 };

// last block, thread 0, after the parallel unpack of the sums into W->Hn / bn / Hsn / bsn: the alpha terms,
// res / calcEC, and the mode's LM logic.  Returns what the block does next: LM_COPY (H -> Hm etc.), LM_OUT (the
// single pass's H / b into the control block), LM_SOLVE (the next step)
__device__ __forceinline__ int lm_decide(const HsRefArgs& a, HsRefCtl* C, RefWork* W, const double* R,
                                         const HsRefPass& pc, int sel) {
  const int n = a.n;
  float* H = W->Hn;
  float* b = W->bn;
  float res[3], ec[2];
#pragma unroll
  for (int k = 0; k < 3; k++) {
    H[k * 8 + k] += pc.alphaOpt * n;
    b[k] += pc.tlog[k] * pc.alphaOpt * n;
  }
  res[0] = (float)R[2 * NACC];
  res[1] = pc.alphaEnergy;
  res[2] = (float)(2 * n);  // E.num: npts updates in each of the two energy loops
  ec[0] = hs_ref_coupling * (float)R[2 * NACC + 1];
  ec[1] = hs_ref_coupling * (float)R[2 * NACC + 2];
  if (a.mode == HS_REF_CALC) {
#pragma unroll
    for (int k = 0; k < 3; k++) C->res[k] = res[k];
    C->jb_sel = sel;
    C->done = 1;
    return LM_OUT;
  }
  if (a.mode == HS_REF_INIT) {  // the first calcResAndGS + applyStep(0) (Src/Initializer.cpp:1424-1426)
#pragma unroll
    for (int k = 0; k < 3; k++) C->resOld[k] = res[k];
#pragma unroll
    for (int k = 0; k < 7; k++) C->T[k] = a.T0[k];
    C->aff[0] = a.aff0[0];
    C->aff[1] = a.aff0[1];
    C->lambda = 0.1f;
    C->fails = 0;
    C->iteration = 0;
    C->snapped = 0;
    C->apply_prev = 1;   // applyStep without optReg
    C->optreg_prev = 0;
    C->jb_sel = sel;
    C->done = 0;
    return LM_COPY | LM_SOLVE;
  }
  REF_TRACE(9);
  // HS_REF_ITER: calcEC + the accept test (Src/Initializer.cpp:1470-1540)
  const int it = C->iteration;
  const float reg0 = C->snapped ? ec[0] : 0.f, reg1 = C->snapped ? ec[1] : 0.f;
  const float eTotalNew = res[0] + res[1] + reg1;
  const float eTotalOld = C->resOld[0] + C->resOld[1] + reg0;
  const bool accept = eTotalOld > eTotalNew;
  float inc[8];
#pragma unroll
  for (int k = 0; k < 8; k++) inc[k] = C->inc[k];
  const float incNorm = sqrtf(dot8(inc, inc));
  if (it < HS_REF_MAXLOG) {
    float* L = a.log + (size_t)it * HS_REF_LOGW;
    L[0] = eTotalOld; L[1] = eTotalNew; L[2] = accept ? 1.f : 0.f; L[3] = C->lambda; L[4] = incNorm;
    L[5] = res[0]; L[6] = res[1]; L[7] = reg1;
  }
  int fails = C->fails;
  if (accept) {
    if (res[1] == hs_ref_alphaK * n) C->snapped = 1;
#pragma unroll
    for (int k = 0; k < 3; k++) C->resOld[k] = res[k];
    C->aff[0] = C->affn[0];
    C->aff[1] = C->affn[1];
#pragma unroll
    for (int k = 0; k < 7; k++) C->T[k] = C->Tn[k];
    C->lambda *= 0.5f;
    fails = 0;
    if (C->lambda < 0.0001f) C->lambda = 0.0001f;
  } else {
    fails++;
    C->lambda *= 4;
    if (C->lambda > 10000) C->lambda = 10000;
  }
  C->fails = fails;
  C->apply_prev = accept;
  C->optreg_prev = accept;
  C->jb_sel = sel;
  const int cp = accept ? LM_COPY : 0;
  if (!(incNorm > 1e-4f) || it >= 1000 || fails >= 2) {
    C->done = 1;
    return cp;
  }
  C->iteration = it + 1;
  REF_TRACE(10);
  return cp | LM_SOLVE;
}

// one pattern pixel of calcResAndGS (Src/Initializer.cpp:1970-2039); false = the point is bad.  xv: the values the
// leader folds in pattern order; J: this pixel's acc9 row
__device__ __forceinline__ bool ref_pixel(const HsRefArgs& a, const HsRefPass& S, int idx, float pu, float pv,
                                          float idn, bool tri, float* xv, float J[9]) {
  const float x = pu + kPat[idx][0], y = pv + kPat[idx][1];
  float pt[3];
#pragma unroll
  for (int q = 0; q < 3; q++) pt[q] = (S.RKi[q * 3 + 0] * x + S.RKi[q * 3 + 1] * y + S.RKi[q * 3 + 2] * 1.f) + S.t[q] * idn;
  const float u = pt[0] / pt[2];
  const float v = pt[1] / pt[2];
  const float Ku = a.fx * u + a.cx;
  const float Kv = a.fy * v + a.cy;
  const float new_idepth = idn / pt[2];
  if (!(Ku > 1 && Kv > 1 && Ku < a.W - 2 && Kv < a.H - 2 && new_idepth > 0)) return false;
  const float3 hit = ref_interp33(a.img2, Ku, Kv, a.W);
  const float rlR = ref_interp31(a.img1, x, y, a.W, a.H);
  if (!isfinite(rlR) || !isfinite(hit.x)) return false;
  const float residual = hit.x - S.r2a * rlR - S.r2b;
  float hw = fabsf(residual) < a.huberTH ? 1 : a.huberTH / fabsf(residual);
  if (!tri) hw = (float)(hw * 0.1);
  xv[0] = hw * residual * residual * (2 - hw);
  const float dxdd = (S.t[0] - S.t[2] * u) / pt[2];
  const float dydd = (S.t[1] - S.t[2] * v) / pt[2];
  if (hw < 1) hw = sqrtf(hw);
  const float dxI = hw * hit.y * a.fx;
  const float dyI = hw * hit.z * a.fy;
  J[0] = new_idepth * dxI;
  J[1] = new_idepth * dyI;
  J[2] = -new_idepth * (u * dxI + v * dyI);
  J[3] = -u * v * dxI - (1 + v * v) * dyI;
  J[4] = (1 + u * u) * dxI + u * v * dyI;
  J[5] = -v * dxI + u * dyI;
  J[6] = -hw * S.r2a * rlR;
  J[7] = -hw * 1;
  const float dd = dxI * dxdd + dyI * dydd;
  J[8] = hw * residual;
  const float nx = dxdd * a.fx, ny = dydd * a.fy;
  xv[1] = 1.0f / sqrtf(nx * nx + ny * ny);
#pragma unroll
  for (int k = 0; k < 8; k++) xv[2 + k] = J[k] * dd;
  xv[10] = J[8] * dd;
  xv[11] = dd * dd;
  return true;
}



struct RefLds {
  HsRefCtl ctl;          // the device-resident LM state, copied in at entry (the last block writes it back)
  RefWork wk;
  float xv[RB][NX + 1];  // per-lane values for the leader's in-order fold (+1: bank padding)
  int pgood[HS_REF_PPB];
  float Pl[HS_REF_PPB][13];  // each point's acc9SC row (JbBuffer_new after the alpha / coupling terms), E, calcEC
  float Jl[RB][10];      // each lane's acc9 row [J | r] (zero unless its point is good)
  float pa[NACC][RW];    // acc9 per wave
  double red[HS_REF_NRED];
  int last, lmflags;
};
__constant__ unsigned char kQr[NACC] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1, 2, 2, 2, 2, 2, 2, 2,
                                        3, 3, 3, 3, 3, 3, 4, 4, 4, 4, 4, 5, 5, 5, 5, 6, 6, 6, 7, 7, 8};
__constant__ unsigned char kQc[NACC] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 1, 2, 3, 4, 5, 6, 7, 8, 2, 3, 4, 5, 6, 7, 8,
                                        3, 4, 5, 6, 7, 8, 4, 5, 6, 7, 8, 5, 6, 7, 8, 6, 7, 8, 7, 8, 8};

}  // namespace

__global__ __launch_bounds__(RB) void hs_k_refine_step(HsRefArgs a) {
  HsRefCtl* C = a.ctl;
  const int mode = a.mode;
  __shared__ RefLds S;
  const int tid = threadIdx.x, lane = tid & 63;
  const int slot = tid >> 3, k = tid & 7;
  const int i = blockIdx.x * HS_REF_PPB + slot;
  const int n = a.n;
  const bool valid = i < n;
  const bool leader = k == 0;
  const HsRefPoints& P = a.p;
  REF_TRACE(0);
  // every lane's point coordinates, issued before the control-block round trip
  float pu = 0.f, pv = 0.f;
  int tri = 0;
  if (valid) {
    pu = P.u[i];
    pv = P.v[i];
    tri = P.tri[i];
  }
  {  // the control block into LDS: one 8-byte word per thread, one round trip
    constexpr int CW = (int)(sizeof(HsRefCtl) / 8);
    static_assert(sizeof(HsRefCtl) % 8 == 0, "HsRefCtl is copied as 8-byte words");
    const uint2* gs = reinterpret_cast<const uint2*>(C);
    uint2* ls = reinterpret_cast<uint2*>(&S.ctl);
    for (int w = tid; w < CW; w += RB) ls[w] = gs[w];
  }
  __syncthreads();
  if (mode == HS_REF_ITER && S.ctl.done) return;  // the LM has stopped: launches queued after it do nothing (uniform)
  if (tid == 0 && (mode == HS_REF_CALC || mode == HS_REF_INIT)) {
    S.ctl.pc = a.pc0;
    S.ctl.apply_prev = 0;
    S.ctl.optreg_prev = 0;
    S.ctl.snapped = 0;
    S.ctl.jb_sel = a.jb_sel0;
  }
  __syncthreads();
  REF_TRACE(1);
  const int sel = S.ctl.jb_sel ^ S.ctl.apply_prev;  // JbBuffer plane after this launch's applyStep
  float* __restrict__ Jbn = P.jb[sel ^ 1];
  // ---- prologue (the point's leader lane): every load first (the arrays may alias as far as the compiler
  // knows, so loads after a store would serialize), then applyStep / optReg / doStep in registers
  float idn = 0.f, idp = 0.f, iR = 0.f, e0 = 0.f, e1 = 0.f;
  int g = 0;
  if (valid && leader) {
    const int g_old = P.good[i];
    const float id_old = P.idepth[i], iR_old = P.iR[i];
    if (mode == HS_REF_CALC || mode == HS_REF_INIT) {  // resetPoints
      g = g_old;
      idp = id_old;
      idn = id_old;
      iR = iR_old;
      P.energy[i] = 0.f;
      P.energy[n + i] = 0.f;
      P.idepth_new[i] = idn;
    } else {
      const int gn_prev = P.good_new[i];
      const float en0 = P.energy_new[i], en1 = P.energy_new[n + i], idn_prev = P.idepth_new[i];
      const float lhn = P.lastH_new[i], invz = P.invz[i], ms_prev = P.maxstep[i];
      const float eo0 = P.energy[i], eo1 = P.energy[n + i];
      const float* Jb = P.jb[sel];
      float jb[10];
#pragma unroll
      for (int q = 0; q < 10; q++) jb[q] = Jb[(size_t)q * n + i];
      g = g_old;
      idp = id_old;
      iR = iR_old;
      e0 = eo0;
      e1 = eo1;
      float idn_w = idn_prev;
      if (S.ctl.apply_prev) {  // applyStep (+ optReg)
        if (!g_old) {
          idp = iR_old;
          idn_w = iR_old;
          if (S.ctl.optreg_prev && !S.ctl.snapped) iR = tri ? invz : iR_old;
        } else {
          e0 = en0;
          e1 = en1;
          g = gn_prev;
          idp = idn_prev;
          if (S.ctl.optreg_prev) {
            if (!S.ctl.snapped) iR = tri ? invz : idp;
            else if (g) iR = idp;
          }
          P.energy[i] = e0;
          P.energy[n + i] = e1;
          P.good[i] = (uint8_t)g;
          P.lastH[i] = lhn;
        }
        P.idepth[i] = idp;
        P.iR[i] = iR;
      }
      if (mode == HS_REF_ITER && g) {  // doStep with JbBuffer = plane sel (its rows were written by a pass
        // whose point was good, which this point is)
        const float b = jb[8] + dot8(jb, S.ctl.inc);
        float step = -b * jb[9] / (1 + S.ctl.lambda);
        float maxstep = 0.25f * ms_prev;
        if (maxstep > 1e10f) maxstep = 1e10f;
        if (step > maxstep) step = maxstep;
        if (step < -maxstep) step = -maxstep;
        float newIdepth = idp + step;
        if (newIdepth < 1e-3f) newIdepth = 1e-3f;
        if (newIdepth > 50) newIdepth = 50;
        idn_w = newIdepth;
      }
      idn = idn_w;
      if (S.ctl.apply_prev || (mode == HS_REF_ITER && g)) P.idepth_new[i] = idn;
    }
  }
  if (mode == HS_REF_FINAL) return;
  REF_TRACE(2);
  const int base = lane & ~7;
  idn = __shfl(idn, base);
  g = __shfl(g, base);
  // ---- pass: one pixel per lane
  float J[9];
  bool ok = false;
  const bool live = valid && g;
  if (live) ok = ref_pixel(a, S.ctl.pc, k, pu, pv, idn, tri != 0, S.xv[tid], J);
  const unsigned long long failm = __ballot(live && !ok);
  const unsigned int fb = (unsigned int)(failm >> base) & 0xffu;
  const int f = fb ? __builtin_ctz(fb) : 8;  // first failing pixel: the reference's loop breaks there
  __syncthreads();
  REF_TRACE(3);
  float E = 0.f, ec0 = 0.f, ec1 = 0.f;
  float* prow = S.Pl[slot];
  if (valid && leader) {
    int gn = 0;
    if (!g) {
      P.maxstep[i] = 1e10f;
      E = e0;
      P.energy_new[i] = e0;
      P.energy_new[n + i] = e1;
    } else {
      float energy = 0.f, maxstep = 1e10f, jb[10];
#pragma unroll
      for (int q = 0; q < 10; q++) jb[q] = 0.f;
#pragma unroll
      for (int kk = 0; kk < 8; kk++) {
        if (kk < f) {
          const float* x = S.xv[tid + kk];
          energy += x[0];
          if (x[1] < maxstep) maxstep = x[1];
#pragma unroll
          for (int q = 0; q < 10; q++) jb[q] += x[2 + q];
        }
      }
      P.maxstep[i] = maxstep;
      if (f < 8 || energy > 8 * a.outlierTH * 20) {
        E = e0;
        P.energy_new[i] = e0;
        P.energy_new[n + i] = e1;
      } else {
        gn = 1;
        E = energy;
        P.energy_new[i] = energy;
        P.energy_new[n + i] = (idn - 1) * (idn - 1);
        // acc9SC row (Src/Initializer.cpp:2114-2124)
        const float alphaOpt = S.ctl.pc.alphaOpt;
        P.lastH_new[i] = jb[9];
        jb[8] += alphaOpt * (idn - 1);
        jb[9] += alphaOpt;
        if (alphaOpt == 0) {
          jb[8] += hs_ref_coupling * (idn - iR);
          jb[9] += hs_ref_coupling;
        }
        jb[9] = 1 / (1 + jb[9]);
        // calcEC terms (Src/Initializer.cpp:2214-2220)
        const float rOld = idp - iR, rNew = idn - iR;
        ec0 = rOld * rOld;
        ec1 = rNew * rNew;
      }
#pragma unroll
      for (int q = 0; q < 10; q++) {
        Jbn[(size_t)q * n + i] = jb[q];
        prow[q] = gn ? jb[q] : 0.f;
      }
    }
    if (!g) {
#pragma unroll
      for (int q = 0; q < 10; q++) prow[q] = 0.f;
    }
    prow[10] = E;
    prow[11] = ec0;
    prow[12] = ec1;
    P.good_new[i] = (uint8_t)gn;
    S.pgood[slot] = gn;
  } else if (leader) {
    S.pgood[slot] = 0;
#pragma unroll
    for (int q = 0; q < 13; q++) prow[q] = 0.f;
  }
  __syncthreads();
  REF_TRACE(4);
  {  // this lane's acc9 row (zero unless its point is good)
    const bool pg = S.pgood[slot] != 0;
#pragma unroll
    for (int q = 0; q < 9; q++) S.Jl[tid][q] = pg ? J[q] : 0.f;
  }
  __syncthreads();
  // ---- block sums in a fixed order: acc9 entry q over each wave's 64 lanes in lane order, then the 4 waves;
  // acc9SC (updateSingleWeighted form: diagonal (J_r J_r) w, off-diagonal J_c (J_r w)) and E / calcEC over the
  // 32 points in point order
  if (tid < NACC * RW) {
    const int q = tid >> 2, w = tid & 3, r = kQr[q], c = kQc[q];
    float s = 0.f;
    const int l0 = w * 64;
#pragma unroll 16
    for (int l = 0; l < 64; l++) s += S.Jl[l0 + l][r] * S.Jl[l0 + l][c];
    S.pa[q][w] = s;
  } else if (tid < NACC * RW + NACC) {
    const int q = tid - NACC * RW, r = kQr[q], c = kQc[q];
    float s = 0.f;
#pragma unroll 8
    for (int p = 0; p < HS_REF_PPB; p++) {
      const float* row = S.Pl[p];
      const float w = row[9];
      s += r == c ? row[r] * row[r] * w : row[c] * (row[r] * w);
    }
    S.red[NACC + q] = (double)s;
  } else if (tid < NACC * RW + NACC + 3) {
    const int q = tid - NACC * RW - NACC;
    float s = 0.f;
    for (int p = 0; p < HS_REF_PPB; p++) s += S.Pl[p][10 + q];
    S.red[2 * NACC + q] = (double)s;
  }
  __syncthreads();
  if (tid < HS_REF_NRED) {
    double s;
    if (tid < NACC) {
      s = 0.0;
#pragma unroll
      for (int w = 0; w < RW; w++) s += (double)S.pa[tid][w];
    } else {
      s = S.red[tid];
    }
    __hip_atomic_store(&a.part[(size_t)blockIdx.x * HS_REF_NRED + tid], s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  REF_TRACE(5);
  // hand-off (HIP memory model, no reliance on write-through behaviour): every thread's partial store is ordered
  // before the ticket by an agent-scope release fence, the ticket is an acq_rel read-modify-write, and the block
  // whose add returns nblocks - 1 takes an agent-scope acquire fence before it reads the other blocks' partials
  // (no block waits on another)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __syncthreads();
  if (tid == 0)
    S.last = __hip_atomic_fetch_add(a.ticket, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == a.nblocks - 1;
  __syncthreads();
  REF_TRACE(6);
  if (!S.last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  if (tid < HS_REF_NRED) {  // block order, up to 64 independent write-through loads in flight per thread
    double s = 0.0;
    const double* pp = a.part + tid;
    for (int b = 0; b < a.nblocks; b += 64) {
      double t[64];
#pragma unroll
      for (int j = 0; j < 64; j++)
        t[j] = __hip_atomic_load(pp + (size_t)min(b + j, a.nblocks - 1) * HS_REF_NRED, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int j = 0; j < 64; j++)
        if (b + j < a.nblocks) s += t[j];
    }
    S.red[tid] = s;  // only this thread reads slot tid before the sum
  }
  __syncthreads();
  if (tid < NACC) {  // unpack entry tid of acc9 / acc9SC into H_out / b_out / H_out_sc / b_out_sc
    const int r = kQr[tid], c = kQc[tid];
    const float v = (float)S.red[tid], w = (float)S.red[NACC + tid];
    if (c < 8) {
      S.wk.Hn[r * 8 + c] = S.wk.Hn[c * 8 + r] = v;
      S.wk.Hsn[r * 8 + c] = S.wk.Hsn[c * 8 + r] = w;
    } else if (r < 8) {  // column 8 = [b; r'r]: the (8, 8) entry is not part of b
      S.wk.bn[r] = v;
      S.wk.bsn[r] = w;
    }
  }
  __syncthreads();
  if (tid == 0) {
    REF_TRACE(8);
    const HsRefPass pc = S.ctl.pc;
    S.lmflags = lm_decide(a, &S.ctl, &S.wk, S.red, pc, sel);
  }
  __syncthreads();
  const int fl = S.lmflags;
  if (tid < 64) {
    if (fl & LM_COPY) {
      S.ctl.Hm[tid] = S.wk.Hn[tid];
      S.ctl.Hs[tid] = S.wk.Hsn[tid];
      if (tid < 8) {
        S.ctl.bm[tid] = S.wk.bn[tid];
        S.ctl.bs[tid] = S.wk.bsn[tid];
      }
    }
    if (fl & LM_OUT) {
      S.ctl.H[tid] = S.wk.Hn[tid];
      S.ctl.Hsc[tid] = S.wk.Hsn[tid];
      if (tid < 8) {
        S.ctl.b[tid] = S.wk.bn[tid];
        S.ctl.bsc[tid] = S.wk.bsn[tid];
      }
    }
  }
  __syncthreads();
  if (fl & LM_SOLVE) {
    lm_solve_prep(a, &S.ctl, &S.wk, tid);
    __syncthreads();
    if (tid == 0) lm_solve_tail(a, &S.ctl, &S.wk);
  }
  if (tid == 0) __hip_atomic_store(a.ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // ready for the next launch
  __syncthreads();
  {  // the control block back (the next launch reads it after the kernel boundary)
    constexpr int CW = (int)(sizeof(HsRefCtl) / 8);
    const uint2* ls = reinterpret_cast<const uint2*>(&S.ctl);
    uint2* gs = reinterpret_cast<uint2*>(a.ctl);
    for (int w = tid; w < CW; w += RB) gs[w] = ls[w];
  }
  REF_TRACE(7);
}
