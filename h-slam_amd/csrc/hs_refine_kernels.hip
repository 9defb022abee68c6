// hs_refine_kernels.hip — gfx950 kernel of H-SLAM's initializer refinement DirectRefinement (SURVEY.md §8f
// rank 4, the second Accumulator9 user):
//
//   hs_k_refine   one workgroup (512 threads, 8 waves) runs the whole level-0 LM loop of
//                 DirectRefinement::Refine (Src/Initializer.cpp:1412-1564) on the device:
//                   resetPoints (:1897-1924), calcResAndGS (:1926-2153) with its Accumulator9 normal equations,
//                   the Schur part acc9SC and the calcEC regularizer energy fused in one pass over the points,
//                   the fixAffine 6x6 fp32 LDLT step + SE3 update on thread 0, doStep (:2155-2186),
//                   applyStep (:2188-2205) and optReg (:2229-2270) as per-point passes.
//                 Point state stays in HBM as structure-of-arrays (one thread owns a fixed point set), the
//                 JbBuffer / JbBuffer_new swap is a plane-index flip.
//
// Per-point arithmetic follows the reference's fp32 operation order (fp contraction off): every per-point
// output of a pass (isGood_new, energy_new, maxstep, JbBuffer_new, lastHessian_new, idepth_new) is
// bit-identical to the CPU restatement.  The normal-equation and energy sums are fixed-order parallel
// reductions (wave xor trees, then the 8 waves in order in fp64) where the reference sums sequentially in
// 4 SSE lanes: those compare within tolerance.  Each point's accumulator contribution is computed in a
// second sweep over its pattern once the point is known to be good, so the 9x9 sums stay in registers.
#pragma clang fp contract(off)
#include <hip/hip_runtime.h>

#include <cfloat>

#include "hs_refine_kernels.h"
#include "hs_se3.h"

namespace {

constexpr int REF_NT = 512;
constexpr int REF_NW = REF_NT / 64;
constexpr int REF_NACC = 45;                         // upper triangle of the 9x9 [J | r] system
constexpr int REF_NRED = 2 * REF_NACC + 3;           // acc9, acc9SC, E, calcEC old / new
constexpr float kAlphaK = 2.5f * 2.5f, kAlphaW = 150 * 150, kCoupling = 1;
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

// Eigen::LDLT<Matrix<float,6,6>> (diagonal pivoting, left-looking) + solve, one thread, register-resident
__device__ __noinline__ void ldlt6f_solve(const float* __restrict__ A, const float* __restrict__ rhs, float* __restrict__ x) {
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

struct RefShared {
  // pass inputs (thread 0 writes)
  float RKi[9], t[3], r2a, r2b, alphaOpt, alphaEnergy, tlog[3];
  // pass outputs
  double red[REF_NW][REF_NRED];
  float H[64], b[8], Hsc[64], bsc[8], res[3], ec[2];
  // LM state
  double T[7], Tn[7], aff[2], affn[2];
  float Hm[64], bm[8], Hs[64], bs[8], resOld[3];
  float inc[8], lambda;
  int snapped, accept, brk;
};

// thread 0: the pass constants at (T, aff) (out of line: keeps the fp64 SE3 code out of the pass's registers)
__device__ __noinline__ void ref_setup(const HsRefArgs& a, RefShared& S, const double T7[7], const double aff[2]) {
  const hs::SE3 T = hs::SE3::fromData(T7);
  double R[9];
  T.rotationMatrix(R);
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++)
      S.RKi[r * 3 + c] = (float)(R[r * 3 + 0] * a.Ki[0 * 3 + c] + R[r * 3 + 1] * a.Ki[1 * 3 + c] + R[r * 3 + 2] * a.Ki[2 * 3 + c]);
  for (int q = 0; q < 3; q++) S.t[q] = (float)T.t[q];
  S.r2a = (float)exp(aff[0]);
  S.r2b = (float)aff[1];
  // EAlpha never receives an update in the reference (its loop feeds E): alphaEnergy = alphaW * |t|^2 * npts
  const double tsq = T.t[0] * T.t[0] + T.t[1] * T.t[1] + T.t[2] * T.t[2];
  const float EAlphaA = 0.f;
  float alphaEnergy = (float)(kAlphaW * (EAlphaA + tsq * a.n));
  float alphaOpt;
  if (alphaEnergy > kAlphaK * a.n) {
    alphaOpt = 0;
    alphaEnergy = kAlphaK * a.n;
  } else {
    alphaOpt = kAlphaW;
  }
  S.alphaOpt = alphaOpt;
  S.alphaEnergy = alphaEnergy;
  double lg[6];
  T.log(lg);
  for (int q = 0; q < 3; q++) S.tlog[q] = (float)lg[q];
}

struct PixOut {
  float e, dd, r, ms, dp[8];
};

// one pattern pixel of calcResAndGS (Src/Initializer.cpp:1970-2039); false = the point is bad
__device__ __forceinline__ bool ref_pixel(const HsRefArgs& a, const RefShared& S, int idx, float pu, float pv,
                                          float idn, bool tri, PixOut& o) {
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
  o.e = hw * residual * residual * (2 - hw);
  const float dxdd = (S.t[0] - S.t[2] * u) / pt[2];
  const float dydd = (S.t[1] - S.t[2] * v) / pt[2];
  if (hw < 1) hw = sqrtf(hw);
  const float dxI = hw * hit.y * a.fx;
  const float dyI = hw * hit.z * a.fy;
  o.dp[0] = new_idepth * dxI;
  o.dp[1] = new_idepth * dyI;
  o.dp[2] = -new_idepth * (u * dxI + v * dyI);
  o.dp[3] = -u * v * dxI - (1 + v * v) * dyI;
  o.dp[4] = (1 + u * u) * dxI + u * v * dyI;
  o.dp[5] = -v * dxI + u * dyI;
  o.dp[6] = -hw * S.r2a * rlR;
  o.dp[7] = -hw * 1;
  o.dd = dxI * dxdd + dyI * dydd;
  o.r = hw * residual;
  const float nx = dxdd * a.fx, ny = dydd * a.fy;
  o.ms = 1.0f / sqrtf(nx * nx + ny * ny);
  return true;
}

// calcResAndGS + calcEC sums at the constants in S; reads JbBuffer_new plane `nsel`
__device__ void ref_pass(const HsRefArgs& a, RefShared& S, int nsel) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const HsRefPoints& P = a.p;
  float* __restrict__ Jbn = P.jb[nsel];
  const int n = a.n;
  const float alphaOpt = S.alphaOpt, thr = 8 * a.outlierTH * 20;
  float acc[REF_NACC];
#pragma unroll
  for (int q = 0; q < REF_NACC; q++) acc[q] = 0.f;
  float E = 0.f;
  for (int i = tid; i < n; i += REF_NT) {
    const float e0 = P.energy[i], e1 = P.energy[n + i];
    if (!P.good[i]) {
      P.maxstep[i] = 1e10f;
      E += e0;
      P.energy_new[i] = e0;
      P.energy_new[n + i] = e1;
      P.good_new[i] = 0;
      continue;
    }
    const float pu = P.u[i], pv = P.v[i], idn = P.idepth_new[i];
    const bool tri = P.tri[i] != 0;
    float jb[10];
#pragma unroll
    for (int k = 0; k < 10; k++) jb[k] = 0.f;
    float energy = 0.f, maxstep = 1e10f;
    bool ok = true;
    for (int idx = 0; idx < 8; idx++) {
      PixOut o;
      if (!ref_pixel(a, S, idx, pu, pv, idn, tri, o)) {
        ok = false;
        break;
      }
      energy += o.e;
      if (o.ms < maxstep) maxstep = o.ms;
#pragma unroll
      for (int k = 0; k < 8; k++) jb[k] += o.dp[k] * o.dd;
      jb[8] += o.r * o.dd;
      jb[9] += o.dd * o.dd;
    }
    P.maxstep[i] = maxstep;
    if (!ok || energy > thr) {
      E += e0;
      P.energy_new[i] = e0;
      P.energy_new[n + i] = e1;
      P.good_new[i] = 0;
#pragma unroll
      for (int k = 0; k < 10; k++) Jbn[(size_t)k * n + i] = jb[k];
      continue;
    }
    E += energy;
    P.good_new[i] = 1;
    P.energy_new[i] = energy;
    P.energy_new[n + i] = (idn - 1) * (idn - 1);
    // acc9 contribution: the same per-pixel values again (deterministic), 9x9 upper triangle
    for (int idx = 0; idx < 8; idx++) {
      PixOut o;
      ref_pixel(a, S, idx, pu, pv, idn, tri, o);
      float J[9];
#pragma unroll
      for (int k = 0; k < 8; k++) J[k] = o.dp[k];
      J[8] = o.r;
      int q = 0;
#pragma unroll
      for (int r = 0; r < 9; r++)
#pragma unroll
        for (int c = r; c < 9; c++) acc[q++] += J[r] * J[c];
    }
    // acc9SC input (Src/Initializer.cpp:2114-2124): JbBuffer_new[8..9] with the alpha / coupling terms
    const float iR = P.iR[i];
    P.lastH_new[i] = jb[9];
    jb[8] += alphaOpt * (idn - 1);
    jb[9] += alphaOpt;
    if (alphaOpt == 0) {
      jb[8] += kCoupling * (idn - iR);
      jb[9] += kCoupling;
    }
    jb[9] = 1 / (1 + jb[9]);
#pragma unroll
    for (int k = 0; k < 10; k++) Jbn[(size_t)k * n + i] = jb[k];
  }
  // wave xor trees, then the waves in order in fp64
#pragma unroll
  for (int q = 0; q < REF_NACC + 1; q++) {
    float v = q < REF_NACC ? acc[q] : E;
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (lane == 0) S.red[wv][q < REF_NACC ? q : 2 * REF_NACC] = (double)v;
  }
  // phase 2: acc9SC (updateSingleWeighted order, Src/Initializer.cpp:2125-2130) and the calcEC terms
  // (:2214-2220) of the points good in this pass, from the JbBuffer_new rows just written (same thread)
  {
    float sc[REF_NACC];
#pragma unroll
    for (int q = 0; q < REF_NACC; q++) sc[q] = 0.f;
    float ec0 = 0.f, ec1 = 0.f;
    for (int i = tid; i < n; i += REF_NT) {
      if (!P.good_new[i]) continue;
      float J[9];
#pragma unroll
      for (int k = 0; k < 9; k++) J[k] = Jbn[(size_t)k * n + i];
      const float w = Jbn[(size_t)9 * n + i];
      int q = 0;
#pragma unroll
      for (int r = 0; r < 9; r++) {
        sc[q++] += J[r] * J[r] * w;
        J[r] *= w;
#pragma unroll
        for (int c = r + 1; c < 9; c++) sc[q++] += J[c] * J[r];
      }
      const float iR = P.iR[i];
      const float rOld = P.idepth[i] - iR, rNew = P.idepth_new[i] - iR;
      ec0 += rOld * rOld;
      ec1 += rNew * rNew;
    }
#pragma unroll
    for (int q = 0; q < REF_NACC + 2; q++) {
      float v = q < REF_NACC ? sc[q] : (q == REF_NACC ? ec0 : ec1);
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
      if (lane == 0) S.red[wv][q < REF_NACC ? REF_NACC + q : 2 * REF_NACC + 1 + (q - REF_NACC)] = (double)v;
    }
  }
  __syncthreads();
  if (tid < REF_NRED) {
    double s = 0.0;
    for (int w = 0; w < REF_NW; w++) s += S.red[w][tid];
    S.red[0][tid] = s;  // wave 0's slot is only read by this thread before the sum
  }
  __syncthreads();
  if (tid == 0) {
    const double* R = S.red[0];
    int q = 0;
    for (int r = 0; r < 9; r++)
      for (int c = r; c < 9; c++, q++) {
        const float v = (float)R[q], w = (float)R[REF_NACC + q];
        if (c < 8) {
          S.H[r * 8 + c] = S.H[c * 8 + r] = v;
          S.Hsc[r * 8 + c] = S.Hsc[c * 8 + r] = w;
        } else if (r < 8) {
          S.b[r] = v;
          S.bsc[r] = w;
        }
      }
    for (int k = 0; k < 3; k++) {
      S.H[k * 8 + k] += alphaOpt * n;
      S.b[k] += S.tlog[k] * alphaOpt * n;
    }
    S.res[0] = (float)R[2 * REF_NACC];
    S.res[1] = S.alphaEnergy;
    S.res[2] = (float)(2 * n);  // E.num: npts updates in each of the two loops
    S.ec[0] = kCoupling * (float)R[2 * REF_NACC + 1];
    S.ec[1] = kCoupling * (float)R[2 * REF_NACC + 2];
  }
  __syncthreads();
}

}  // namespace

__global__ __launch_bounds__(REF_NT) void hs_k_refine(HsRefArgs a) {
  __shared__ RefShared S;
  const int tid = threadIdx.x;
  const HsRefPoints& P = a.p;
  const int n = a.n;
  int sel = a.jb_sel;  // plane holding JbBuffer (uniform)
  // resetPoints
  for (int i = tid; i < n; i += REF_NT) {
    P.energy[i] = 0.f;
    P.energy[n + i] = 0.f;
    P.idepth_new[i] = P.idepth[i];
  }
  if (tid == 0) {
    for (int q = 0; q < 7; q++) S.T[q] = a.T_in[q];
    S.aff[0] = a.aff_in[0];
    S.aff[1] = a.aff_in[1];
    ref_setup(a, S, S.T, S.aff);
  }
  __syncthreads();
  ref_pass(a, S, sel ^ 1);
  if (a.single_pass) {
    if (tid == 0) {
      HsRefOut& o = *a.out;
      for (int q = 0; q < 64; q++) { o.H[q] = S.H[q]; o.Hsc[q] = S.Hsc[q]; }
      for (int q = 0; q < 8; q++) { o.b[q] = S.b[q]; o.bsc[q] = S.bsc[q]; }
      for (int q = 0; q < 3; q++) o.res[q] = S.res[q];
      o.jb_sel = sel;
    }
    return;
  }
  // applyStep of the initial evaluation (unconditional)
  for (int i = tid; i < n; i += REF_NT) {
    if (!P.good[i]) {
      P.idepth[i] = P.idepth_new[i] = P.iR[i];
      continue;
    }
    P.energy[i] = P.energy_new[i];
    P.energy[n + i] = P.energy_new[n + i];
    P.good[i] = P.good_new[i];
    P.idepth[i] = P.idepth_new[i];
    P.lastH[i] = P.lastH_new[i];
  }
  sel ^= 1;
  if (tid == 0) {
    for (int q = 0; q < 64; q++) { S.Hm[q] = S.H[q]; S.Hs[q] = S.Hsc[q]; }
    for (int q = 0; q < 8; q++) { S.bm[q] = S.b[q]; S.bs[q] = S.bsc[q]; }
    for (int q = 0; q < 3; q++) S.resOld[q] = S.res[q];
    S.lambda = 0.1f;
    S.snapped = 0;
  }
  const float wM[8] = {1.0f, 1.0f, 1.0f, 0.5f, 0.5f, 0.5f, 10.0f, 1000.0f};  // SCALE_XI_ROT x3, SCALE_XI_TRANS x3, A, B
  const float scl = 0.01f / (a.W * a.H);
  int fails = 0, iteration = 0;
  __syncthreads();
  while (true) {
    if (tid == 0) {
      const float lambda = S.lambda;
      float Hl[64], bl[8];
      for (int q = 0; q < 64; q++) Hl[q] = S.Hm[q];
      for (int i = 0; i < 8; i++) Hl[i * 8 + i] *= (1 + lambda);
      const float il = 1 / (1 + lambda);
      for (int q = 0; q < 64; q++) Hl[q] -= S.Hs[q] * il;
      for (int i = 0; i < 8; i++) bl[i] = S.bm[i] - S.bs[i] * il;
      float H6[36], x6[6];
      for (int r = 0; r < 6; r++)
        for (int c = 0; c < 6; c++) H6[r * 6 + c] = ((wM[r] * Hl[r * 8 + c]) * wM[c]) * scl;
      for (int r = 0; r < 8; r++) bl[r] = (wM[r] * bl[r]) * scl;
      ldlt6f_solve(H6, bl, x6);  // fixAffine = true
      double incd[6];
      for (int k = 0; k < 6; k++) {
        S.inc[k] = -(wM[k] * x6[k]);
        incd[k] = (double)S.inc[k];
      }
      S.inc[6] = S.inc[7] = 0.f;
      const hs::SE3 nw = hs::SE3::exp(incd) * hs::SE3::fromData(S.T);
      nw.toData(S.Tn);
      S.affn[0] = S.aff[0] + S.inc[6];
      S.affn[1] = S.aff[1] + S.inc[7];
      ref_setup(a, S, S.Tn, S.affn);
    }
    __syncthreads();
    {  // doStep (Src/Initializer.cpp:2155-2186) with JbBuffer = plane sel
      const float* Jb = P.jb[sel];
      float inc[8];
#pragma unroll
      for (int k = 0; k < 8; k++) inc[k] = S.inc[k];
      const float lambda = S.lambda;
      for (int i = tid; i < n; i += REF_NT) {
        if (!P.good[i]) continue;
        float jb[10];
#pragma unroll
        for (int k = 0; k < 10; k++) jb[k] = Jb[(size_t)k * n + i];
        const float b = jb[8] + dot8(jb, inc);
        float step = -b * jb[9] / (1 + lambda);
        float maxstep = 0.25f * P.maxstep[i];
        if (maxstep > 1e10f) maxstep = 1e10f;
        if (step > maxstep) step = maxstep;
        if (step < -maxstep) step = -maxstep;
        float newIdepth = P.idepth[i] + step;
        if (newIdepth < 1e-3f) newIdepth = 1e-3f;
        if (newIdepth > 50) newIdepth = 50;
        P.idepth_new[i] = newIdepth;
      }
    }
    __syncthreads();
    ref_pass(a, S, sel ^ 1);
    if (tid == 0) {
      const float reg0 = S.snapped ? S.ec[0] : 0.f, reg1 = S.snapped ? S.ec[1] : 0.f;  // calcEC
      const float eTotalNew = S.res[0] + S.res[1] + reg1;
      const float eTotalOld = S.resOld[0] + S.resOld[1] + reg0;
      const bool accept = eTotalOld > eTotalNew;
      const float incNorm = sqrtf(dot8(S.inc, S.inc));
      if (iteration < HS_REF_MAXLOG) {
        float* L = a.log + (size_t)iteration * HS_REF_LOGW;
        L[0] = eTotalOld; L[1] = eTotalNew; L[2] = accept ? 1.f : 0.f; L[3] = S.lambda; L[4] = incNorm;
        L[5] = S.res[0]; L[6] = S.res[1]; L[7] = reg1;
      }
      if (accept) {
        if (S.res[1] == kAlphaK * n) S.snapped = 1;
        for (int q = 0; q < 64; q++) { S.Hm[q] = S.H[q]; S.Hs[q] = S.Hsc[q]; }
        for (int q = 0; q < 8; q++) { S.bm[q] = S.b[q]; S.bs[q] = S.bsc[q]; }
        for (int q = 0; q < 3; q++) S.resOld[q] = S.res[q];
        S.aff[0] = S.affn[0];
        S.aff[1] = S.affn[1];
        for (int q = 0; q < 7; q++) S.T[q] = S.Tn[q];
        S.lambda *= 0.5f;
        fails = 0;
        if (S.lambda < 0.0001f) S.lambda = 0.0001f;
      } else {
        fails++;
        S.lambda *= 4;
        if (S.lambda > 10000) S.lambda = 10000;
      }
      S.accept = accept;
      S.brk = !(incNorm > 1e-4f) || iteration >= 1000 || fails >= 2;
    }
    __syncthreads();
    if (S.accept) {  // applyStep + optReg (uniform branch)
      const bool snapped = S.snapped != 0;
      for (int i = tid; i < n; i += REF_NT) {
        if (!P.good[i]) {
          const float r = P.iR[i];
          P.idepth[i] = P.idepth_new[i] = r;
          if (!snapped) P.iR[i] = P.tri[i] ? P.invz[i] : r;
          continue;
        }
        P.energy[i] = P.energy_new[i];
        P.energy[n + i] = P.energy_new[n + i];
        const uint8_t g = P.good_new[i];
        P.good[i] = g;
        const float idp = P.idepth_new[i];
        P.idepth[i] = idp;
        P.lastH[i] = P.lastH_new[i];
        if (!snapped) P.iR[i] = P.tri[i] ? P.invz[i] : idp;
        else if (g) P.iR[i] = idp;
      }
      sel ^= 1;
    }
    const bool brk = S.brk != 0;
    __syncthreads();  // every thread has read S.accept / S.brk before thread 0 rewrites them
    if (brk) break;
    iteration++;
  }
  if (tid == 0) {
    HsRefOut& o = *a.out;
    for (int q = 0; q < 7; q++) o.T[q] = S.T[q];
    o.aff[0] = S.aff[0];
    o.aff[1] = S.aff[1];
    o.iterations = iteration + 1;
    o.snapped = S.snapped;
    o.jb_sel = sel;
    for (int q = 0; q < 3; q++) o.res[q] = S.resOld[q];
  }
}
