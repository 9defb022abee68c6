// hs_track_kernels.hip — gfx950 kernels of H-SLAM's CoarseTracker.
//
//   makeCoarseDepthL0 (Src/CoarseTracker.cpp:105-263), once per keyframe:
//     hs_k_trk_scatter      point -> level-0 idepth / weight sums, in the reference's point order (1 thread:
//                           colliding points add in order, so the sums are the reference's)
//     hs_k_trk_down         2x2 sums up the pyramid
//     hs_k_trk_dilate       one dilation pass (diagonal neighbours on levels 0-1, 4-neighbours above)
//     hs_k_trk_count / hs_k_trk_scan / hs_k_trk_compact
//                           normalisation + order-preserving (raster order) compaction into pc_* arrays
//   trackNewestCoarse (Src/CoarseTracker.cpp:506-683), per frame:
//     hs_k_track            one workgroup (1024 threads) runs the whole coarse-to-fine LM loop of one
//                           pose hypothesis: calcRes (Src/CoarseTracker.cpp:329-485) and the calcGSSSE
//                           normal equations (:267-324) fused in one pass over the reference points,
//                           block reductions, the 8x8 fp64 LDLT step (Eigen pivot order) and SE3 update.
//                           A grid of N workgroups runs N hypotheses of System::trackNewCoarse at once.
// Per-point arithmetic follows the reference's fp32 operation order (fp contraction off), so the
// in-bounds / saturation / warped-set decisions of a pass are bit-identical; the energy and Hessian
// sums are fixed-order parallel reductions (the reference sums in 4 SSE lanes).
#pragma clang fp contract(off)
#include <hip/hip_runtime.h>

#include <cfloat>

#include "hs_track_kernels.h"
#include "hs_se3_dev.h"

namespace {

constexpr int TRK_NT = 512;
constexpr int TRK_B = 4;
#ifndef TRK_MEET_F32
#define TRK_MEET_F32 1  // member meetings exchange fp32 block totals (one granule per value) instead of fp64 (two)
#endif              // points per thread whose loads are in flight together
constexpr int TRK_NACC = 45;          // upper triangle of the 9x9 [J | r] normal equations
constexpr int TRK_NRED = TRK_NACC + 4 + 3;  // + E, flowT, flowRT, flowNum | numE, numSat, numWarped
static_assert(TRK_NRED == HS_TRK_NRED, "pass partial layout");

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

#define HS_TRACE(A, slot)                                                                          \
  do {                                                                                             \
    if ((A).trace && threadIdx.x == 0) (A).trace[(size_t)blockIdx.x * 16 + (slot)] = wall_clock64(); \
  } while (0)

__device__ __forceinline__ double trk_readlane_f64(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), lane);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// Eigen LDLT (diagonal pivoting) solve of an 8x8 system on one wave: the pivot order is the swap sequence on the
// original diagonal (left-looking LDLT, Eigen's ldlt_inplace::unblocked: column k is updated with the finished
// columns j < k, temp_j = D_j L_kj, then scaled by the pivot).  Lane i (mod 8) holds row i of the pivoted matrix, so
// column k's dot products run on the 8 row lanes at once (row k's L entries come by readlane) with the operations of
// the single-thread form in the same order (the same result bit for bit); a single thread ran it as one ~140-
// operation dependent fp64 chain.  One reciprocal per pivot (v_rcp_f64 + two Newton steps, within an ulp of 1 / d)
// instead of Eigen's divisions.  A's diagonal is read scaled by dscale (the LM damping (1 + lambda)).  Every lane
// of the wave calls it; x is uniform.
__device__ __forceinline__ void ldlt8_solve_wave(const double* __restrict__ A, const double* __restrict__ rhs,
                                                 double* __restrict__ x, double dscale, int lane) {
  double dg[8];
  int pm[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    dg[i] = fabs(A[i * 8 + i] * dscale);
    pm[i] = i;
  }
#pragma unroll
  for (int k = 0; k < 8; k++) {
    double best = dg[k];
    int bi = k;
#pragma unroll
    for (int j = k + 1; j < 8; j++)
      if (dg[j] > best) { best = dg[j]; bi = j; }
#pragma unroll
    for (int j = k + 1; j < 8; j++)
      if (j == bi) {
        const double td = dg[k]; dg[k] = dg[j]; dg[j] = td;
        const int tp = pm[k]; pm[k] = pm[j]; pm[j] = tp;
      }
  }
  const int i = lane & 7;
  int pi = pm[0];
#pragma unroll
  for (int q = 1; q < 8; q++) pi = i == q ? pm[q] : pi;
  double m[8];
#pragma unroll
  for (int j = 0; j < 8; j++) m[j] = pm[j] == pi ? A[pi * 9] * dscale : A[pi * 8 + pm[j]];
  double y = rhs[pi];
  double D[8], Dinv[8];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    double temp[8];
#pragma unroll
    for (int j = 0; j < k; j++) temp[j] = D[j] * trk_readlane_f64(m[j], k);
    double t = 0;
#pragma unroll
    for (int j = 0; j < k; j++) t += m[j] * temp[j];
    if (i >= k) m[k] -= t;  // row k: the pivot's own update (the single-thread form's s)
    const double d = trk_readlane_f64(m[k], k);
    D[k] = d;
    double rinv = __builtin_amdgcn_rcp(d);
    rinv = __builtin_fma(rinv, __builtin_fma(-d, rinv, 1.0), rinv);
    rinv = __builtin_fma(rinv, __builtin_fma(-d, rinv, 1.0), rinv);
    Dinv[k] = fabs(d) > DBL_MIN ? rinv : 0.0;
    if (fabs(d) > DBL_MIN && i > k) m[k] *= Dinv[k];
  }
#pragma unroll
  for (int k = 0; k < 8; k++) {  // forward: y_i -= L(i, k) y_k for k < i, in k order
    const double yk = trk_readlane_f64(y, k);
    if (i > k) y = y - m[k] * yk;
  }
  double yy[8];
#pragma unroll
  for (int q = 0; q < 8; q++) yy[q] = trk_readlane_f64(y, q) * Dinv[q];
#pragma unroll
  for (int q = 7; q >= 0; q--)
#pragma unroll
    for (int j = q + 1; j < 8; j++) yy[q] = yy[q] - trk_readlane_f64(m[q], j) * yy[j];
#pragma unroll
  for (int q = 0; q < 8; q++) {
    double v = yy[0];
#pragma unroll
    for (int r = 1; r < 8; r++) v = pm[r] == q ? yy[r] : v;
    x[q] = pm[0] == q ? yy[0] : v;
  }
}

__device__ __forceinline__ double trk_bperm_f64(double v, int src_lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_ds_bpermute(src_lane << 2, (int)(b & 0xffffffffll));
  const int hi = __builtin_amdgcn_ds_bpermute(src_lane << 2, (int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// The same damped 8x8 solve by Gauss-Jordan elimination on the whole wave: lane 8 i + j holds A(i, j) (the diagonal
// scaled by dscale) and rhs(i).  Per pivot k every lane fetches A(k, j) and A(i, k) by ds_bpermute and A(k, k),
// rhs(k) by readlane; row k is scaled by 1 / A(k, k) and every other row loses A(i, k) / A(k, k) times row k.  After
// eight pivots rhs holds x.  The system is the LM-damped H + lambda diag(H) (symmetric positive semi-definite), so
// elimination in the natural order is stable without Eigen's diagonal pivoting; an exactly zero pivot (a zero row
// and column: an affine parameter held fixed) gives x_k = 0 as Eigen's LDLT solve does.  Depth: 8 x (one LDS
// exchange, a reciprocal, an fma) against the LDLT's 8 dependent dot products plus two substitutions; the result
// differs from the LDLT's by rounding only (tests/test_gpu_track.py: the LM logs and poses within the oracle's own
// summation-order spread).  Every lane of the wave calls it; x is uniform.
__device__ __forceinline__ void gj8_solve_wave(const double* __restrict__ A, const double* __restrict__ rhs,
                                               double* __restrict__ x, double dscale, int lane) {
  const int i = lane >> 3, j = lane & 7;
  double a = A[i * 8 + j];
  if (i == j) a *= dscale;
  double r = rhs[i];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const double akj = trk_bperm_f64(a, k * 8 + j);
    const double aik = trk_bperm_f64(a, i * 8 + k);
    const double d = trk_readlane_f64(a, k * 9);
    const double rk = trk_readlane_f64(r, k * 8);
    double rinv = __builtin_amdgcn_rcp(d);
    rinv = __builtin_fma(rinv, __builtin_fma(-d, rinv, 1.0), rinv);
    rinv = __builtin_fma(rinv, __builtin_fma(-d, rinv, 1.0), rinv);
    rinv = fabs(d) > DBL_MIN ? rinv : 0.0;
    if (i == k) {
      a *= rinv;
      r *= rinv;
    } else {
      const double f = aik * rinv;
      a = __builtin_fma(-f, akj, a);
      r = __builtin_fma(-f, rk, r);
    }
  }
#pragma unroll
  for (int q = 0; q < 8; q++) x[q] = trk_readlane_f64(r, q * 8);
}

struct TrkShared {
  // pass inputs (thread 0 writes)
  float RKi[9], t[3], affLL[2], a_gs, b0, cutoff, maxEnergy;
  int lvl, npts;  // npts: the level's reference points (*pc_n)
  // pass outputs
  double red[TRK_NT / 64][TRK_NRED];
  double res[6];
  double H[64], b[8];
  int nWarped;
  // LM state
  double T[7], Tn[7];
  double Tq[4];  // T's quaternion normalized (T as given until the first accepted step, whose Tn is normalized)
  double aff[2], affn[2];
  double Hs[64], bs[8], resOld[6];
  double incNorm;
  float lambda, cutoffRep;
  int brk[2];
  int Gl;    // the level's members (trk_setup_part: 1 below a.gmin points, else a.G)
  int lvseq;  // level ends so far (the level-end record's slot and tag)
  int dead;  // a member meeting timed out: the launch's results are void (the host reruns with G = 1), so every later
             // meeting is skipped and the LM / level loops end at once
  int passes;
  int npass, iters, nchecks;  // this workgroup's pass count (partial parity, counter target), LM iterations, checks
  long long pointPasses;
  // lane q < 45 of the pass tail: its normal-equation entry (r, c) (H (r, c) at hp & 255, (c, r) at (hp >> 8) & 255,
  // c == 8: b (r) at hp & 255 with bit 16 set; (8, 8): -1) and the two scales, formed once per launch
  int hpos[64];
  double hsr[64], hsc[64];
  long long prof[13];  // HS_KTRACE: thread-0 cycles: point loop, reductions, LM step, passes, wave reduce, barrier,
                      // the LM step's solve, its exp + product
  HsTryOut out;       // the lead's output record (thread 0 writes), copied out by trk_publish
};

// Wave reduce-scatter of 64 values (v[i], i < 64) over the 64 lanes: afterwards lane l holds the sum of v[l] over
// all lanes.  Each step pairs every lane with one partner, keeps half of its remaining values (the upper half when
// its bit of the step is set) and adds the partner's copies of them: permlane32 swap (bit 5), permlane16 swap
// (bit 4), DPP row_ror:8 (bit 3), row_half_mirror (pairs l, l ^ 7 within 8: bit 2 decides), quad_perm [2,3,0,1]
// (bit 1) and [1,0,3,2] (bit 0): 63 exchanges + 63 adds for 64 values, against 64 x 6 exchanges of per-value trees.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float wave_reduce_scatter64(const float (&v)[64], int lane) {
  float a[32];
#pragma unroll
  for (int i = 0; i < 32; i++) {  // lanes < 32: v_i + v_i(lane + 32); lanes >= 32: v_(32+i)(lane - 32) + v_(32+i)
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[i]), __float_as_uint(v[32 + i]), false, false);
    a[i] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
  float b[16];
#pragma unroll
  for (int i = 0; i < 16; i++) {  // rows 0, 2 keep a[i], rows 1, 3 keep a[16 + i]
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a[i]), __float_as_uint(a[16 + i]), false, false);
    b[i] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
  const bool b3 = (lane & 8) != 0, b2 = (lane & 4) != 0, b1 = (lane & 2) != 0, b0 = (lane & 1) != 0;
  float c[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {  // partner l ^ 8 (row_ror:8)
    const float keep = b3 ? b[8 + i] : b[i], send = b3 ? b[i] : b[8 + i];
    c[i] = keep + dpp_mov<0x128>(send);
  }
  float d[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {  // partner (l & ~7) | (7 - (l & 7)) (row_half_mirror): bit 2 differs
    const float keep = b2 ? c[4 + i] : c[i], send = b2 ? c[i] : c[4 + i];
    d[i] = keep + dpp_mov<0x141>(send);
  }
  float e[2];
#pragma unroll
  for (int i = 0; i < 2; i++) {  // partner l ^ 2 (quad_perm [2,3,0,1])
    const float keep = b1 ? d[2 + i] : d[i], send = b1 ? d[i] : d[2 + i];
    e[i] = keep + dpp_mov<0x4E>(send);
  }
  const float keep = b0 ? e[1] : e[0], send = b0 ? e[0] : e[1];  // partner l ^ 1 (quad_perm [1,0,3,2])
  return keep + dpp_mov<0xB1>(send);
}

// calcRes + calcGSSSE at S.RKi / S.t / S.affLL for level S.lvl; results in S.res / S.H / S.b / S.nWarped, or (lm:
// an LM iteration's pass) the accept test and, on accept, the new state and Hs / bs / resOld
__device__ void trk_pass(const HsTrackArgs& a, TrkShared& S, int h, int g, bool lm = false) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int G = S.Gl, GT = G * TRK_NT;  // the level's workgroups take points g TRK_NT + tid (mod G TRK_NT)
  const int lvl = S.lvl;
  const HsTrkLevel& L = a.lv[lvl];
  const int n = S.npts, wl = L.w, hl = L.h;
  const float fxl = L.fx, fyl = L.fy, cxl = L.cx, cyl = L.cy;
  float RKi[9], Ki[9];
#pragma unroll
  for (int q = 0; q < 9; q++) { RKi[q] = S.RKi[q]; Ki[q] = L.Ki[q]; }
  const float t0 = S.t[0], t1 = S.t[1], t2 = S.t[2];
  const float aff0 = S.affLL[0], aff1 = S.affLL[1], ags = S.a_gs, b0 = S.b0;
  const float cutoff = S.cutoff, maxEnergy = S.maxEnergy, huberTH = a.huberTH;
  const long long pc0 = (a.trace && tid == 0) ? clock64() : 0;
  float E = 0.f, sT = 0.f, sRT = 0.f, sN = 0.f;
  int nE = 0, nSat = 0, nW = 0;
  float acc[TRK_NACC];
#pragma unroll
  for (int q = 0; q < TRK_NACC; q++) acc[q] = 0.f;
  // the thread's points i = tid + k TRK_NT in order, TRK_B at a time: every load of a batch (point data, then the
  // bilinear taps) is issued before any is used, so a batch costs two memory round trips instead of two per point.
  // A wave's lanes hold consecutive points, so "slot b of this batch holds a point for some lane" is wave-uniform
  // (wb + b GT < n): empty slots are skipped whole, loads and projection included.
  const int wb0 = g * TRK_NT + (tid & ~63);
  for (int i0 = g * TRK_NT + tid, wb = wb0; wb < n; i0 += TRK_B * GT, wb += TRK_B * GT) {
    float id[TRK_B], x[TRK_B], y[TRK_B], refColor[TRK_B];
#pragma unroll
    for (int b = 0; b < TRK_B; b++) {
      id[b] = x[b] = y[b] = refColor[b] = 0.f;
      if (wb + b * GT < n) {
        const int i = min(i0 + b * GT, n - 1);
        id[b] = L.pc_id[i];
        x[b] = L.pc_u[i];
        y[b] = L.pc_v[i];
        refColor[b] = L.pc_col[i];
      }
    }
    float u[TRK_B], v[TRK_B], Ku[TRK_B], Kv[TRK_B], new_idepth[TRK_B];
    bool inb[TRK_B];
    float4 tap[TRK_B][4];
    float fdx[TRK_B], fdy[TRK_B];
#pragma unroll
    for (int b = 0; b < TRK_B; b++) {
      inb[b] = false;
      fdx[b] = fdy[b] = u[b] = v[b] = Ku[b] = Kv[b] = new_idepth[b] = 0.f;
      if (wb + b * GT >= n) continue;  // wave-uniform
      const int i = i0 + b * GT;
      float pt0 = RKi[0] * x[b] + RKi[1] * y[b] + RKi[2] * 1.f;
      float pt1 = RKi[3] * x[b] + RKi[4] * y[b] + RKi[5] * 1.f;
      float pt2 = RKi[6] * x[b] + RKi[7] * y[b] + RKi[8] * 1.f;
      pt0 = pt0 + t0 * id[b];
      pt1 = pt1 + t1 * id[b];
      pt2 = pt2 + t2 * id[b];
      u[b] = pt0 / pt2;
      v[b] = pt1 / pt2;
      Ku[b] = fxl * u[b] + cxl;
      Kv[b] = fyl * v[b] + cyl;
      new_idepth[b] = id[b] / pt2;
      inb[b] = i < n && (Ku[b] > 2 && Kv[b] > 2 && Ku[b] < wl - 3 && Kv[b] < hl - 3 && new_idepth[b] > 0);
      // bilinear taps (interp33), requested for every point of the slot; out-of-bounds points read pixel 0
      const float sx = inb[b] ? Ku[b] : 0.f, sy = inb[b] ? Kv[b] : 0.f;
      const int ix = (int)sx, iy = (int)sy;
      fdx[b] = sx - ix;
      fdy[b] = sy - iy;
      const float4* bp = L.img + ix + iy * wl;
      tap[b][0] = bp[0];
      tap[b][1] = bp[1];
      tap[b][2] = bp[wl];
      tap[b][3] = bp[wl + 1];
    }
#pragma unroll
    for (int b = 0; b < TRK_B; b++) {
      if (!inb[b]) continue;
      const float dx = fdx[b], dy = fdy[b], dxdy = dx * dy;
      const float w11 = dxdy, w01 = dy - dxdy, w10 = dx - dxdy, w00 = 1 - dx - dy + dxdy;
      const float4 p00 = tap[b][0], p10 = tap[b][1], p01 = tap[b][2], p11 = tap[b][3];
      float3 hit;
      hit.x = w11 * p11.x + w01 * p01.x + w10 * p10.x + w00 * p00.x;
      hit.y = w11 * p11.y + w01 * p01.y + w10 * p10.y + w00 * p00.y;
      hit.z = w11 * p11.z + w01 * p01.z + w10 * p10.z + w00 * p00.z;
      if (!isfinite(hit.x)) continue;
      const float residual = hit.x - (float)(aff0 * refColor[b] + aff1);
      const float hw = fabsf(residual) < huberTH ? 1 : huberTH / fabsf(residual);
      if (fabsf(residual) > cutoff) {
        E += maxEnergy;
        nE++;
        nSat++;
      } else {
        E += hw * residual * residual * (2 - hw);
        nE++;
        nW++;
        // calcGSSSE Jacobian of this warped point (Src/CoarseTracker.cpp:282-306)
        const float gx = hit.y * fxl, gy = hit.z * fyl;
        const float uu = u[b], vv = v[b], ni = new_idepth[b];
        float J[9];
        J[0] = ni * gx;
        J[1] = ni * gy;
        J[2] = 0.f - ni * (uu * gx + vv * gy);
        J[3] = 0.f - ((uu * vv) * gx + gy * (1.f + vv * vv));
        J[4] = (uu * vv) * gy + gx * (1.f + uu * uu);
        J[5] = uu * gy - vv * gx;
        J[6] = ags * (b0 - refColor[b]);
        J[7] = -1.f;
        J[8] = residual;
        // the normal-equation sums with fused multiply-adds (their order and rounding are free: the reference sums
        // in four SSE lanes, the parity bar is relative)
        int q = 0;
#pragma unroll
        for (int r = 0; r < 9; r++) {
          const float Jw = J[r] * hw;
#pragma unroll
          for (int c = r; c < 9; c++, q++) acc[q] = __builtin_fmaf(Jw, J[c], acc[q]);
        }
      }
    }
  }
  // the flow indicators (Src/CoarseTracker.cpp:370-401: level 0, every point with i % 32 == 0): flow point
  // j = tid G + g of the hypothesis' threads is point 32 j, so they sit on the first waves of every member, away
  // from the point loop (where the two flow lanes of each wave made the whole wave run the branch per slot)
  if (lvl == 0) {
    for (int j = tid * G + g; 32 * j < n; j += GT) {
      const int i = 32 * j;
      const float xf = L.pc_u[i], yf = L.pc_v[i], idf = L.pc_id[i];
      float pt0 = RKi[0] * xf + RKi[1] * yf + RKi[2] * 1.f;
      float pt1 = RKi[3] * xf + RKi[4] * yf + RKi[5] * 1.f;
      float pt2 = RKi[6] * xf + RKi[7] * yf + RKi[8] * 1.f;
      const float ra0 = pt0, ra1 = pt1, ra2 = pt2;
      pt0 = pt0 + t0 * idf;
      pt1 = pt1 + t1 * idf;
      pt2 = pt2 + t2 * idf;
      const float uu = pt0 / pt2, vv = pt1 / pt2;
      const float Kuf = fxl * uu + cxl, Kvf = fyl * vv + cyl;
      const float k0 = Ki[0] * xf + Ki[1] * yf + Ki[2] * 1.f;
      const float k1 = Ki[3] * xf + Ki[4] * yf + Ki[5] * 1.f;
      const float k2 = Ki[6] * xf + Ki[7] * yf + Ki[8] * 1.f;
      const float pT0 = k0 + t0 * idf, pT1 = k1 + t1 * idf, pT2 = k2 + t2 * idf;
      const float pS0 = k0 - t0 * idf, pS1 = k1 - t1 * idf, pS2 = k2 - t2 * idf;
      const float p30 = ra0 - t0 * idf, p31 = ra1 - t1 * idf, p32 = ra2 - t2 * idf;
      const float uT = pT0 / pT2, vT = pT1 / pT2;
      const float KuT = fxl * uT + cxl, KvT = fyl * vT + cyl;
      const float uT2 = pS0 / pS2, vT2 = pS1 / pS2;
      const float KuT2 = fxl * uT2 + cxl, KvT2 = fyl * vT2 + cyl;
      const float u3 = p30 / p32, v3 = p31 / p32;
      const float Ku3 = fxl * u3 + cxl, Kv3 = fyl * v3 + cyl;
      float sf = (KuT - xf) * (KuT - xf) + (KvT - yf) * (KvT - yf);
      sT += sf;
      sf = (KuT2 - xf) * (KuT2 - xf) + (KvT2 - yf) * (KvT2 - yf);
      sT += sf;
      sf = (Kuf - xf) * (Kuf - xf) + (Kvf - yf) * (Kvf - yf);
      sRT += sf;
      sf = (Ku3 - xf) * (Ku3 - xf) + (Kv3 - yf) * (Kv3 - yf);
      sRT += sf;
      sN += 2;
    }
  }
  const long long pc1 = (a.trace && tid == 0) ? clock64() + (long long)(acc[0] * 0.f + acc[44] * 0.f) : 0;
  // wave reductions (one reduce-scatter: lane q ends with value q's wave sum; the counts are small integers, exact in
  // fp32), then the waves in order in fp64
  float vals[64];
#pragma unroll
  for (int q = 0; q < TRK_NACC; q++) vals[q] = acc[q];
  vals[TRK_NACC + 0] = E;
  vals[TRK_NACC + 1] = sT;
  vals[TRK_NACC + 2] = sRT;
  vals[TRK_NACC + 3] = sN;
  vals[TRK_NACC + 4] = (float)nE;
  vals[TRK_NACC + 5] = (float)nSat;
  vals[TRK_NACC + 6] = (float)nW;
#pragma unroll
  for (int q = TRK_NRED; q < 64; q++) vals[q] = 0.f;
  const float mine = wave_reduce_scatter64(vals, lane);
  if (lane < TRK_NRED) S.red[wv][lane] = (double)mine;
  const long long pcw = (a.trace && tid == 0) ? clock64() + (long long)(mine * 0.f) : 0;
  __syncthreads();
  if (a.trace && tid == 0) {
    S.prof[4] += pcw - pc1;
    S.prof[5] += clock64() - pcw;
  }
  if (wv == 0) {
    // Wave 0 from here to the pass's end, lane q holding value q: the block total (the 8 wave sums, loaded together,
    // added as a fixed tree), the member meeting, then the pass's results from registers (readlane broadcasts), so
    // the only barrier left is the one that publishes them.
    const int q = min(lane, TRK_NRED - 1);
    double r8[TRK_NT / 64];
#pragma unroll
    for (int w = 0; w < TRK_NT / 64; w++) r8[w] = S.red[w][q];
    const long long pt0 = (a.trace && lane == 0) ? clock64() : 0;
    double tot = ((r8[0] + r8[1]) + (r8[2] + r8[3])) + ((r8[4] + r8[5]) + (r8[6] + r8[7]));
    static_assert(TRK_NT / 64 == 8, "block tree");
    const long long pt1 = (a.trace && lane == 0) ? clock64() + (long long)(tot * 0.0) : 0;
    if (G > 1) {
      // The hypothesis' workgroups meet by granules (cdna_hip_programming.md §6 Guideline 16, R2: the data is the
      // flag): every fp64 partial goes out as two 8-byte {tag, 32-bit half} granules (sc1 stores), and lane q
      // re-reads the 2 G granules of its value (sc1 loads) until every tag matches, then sums the G partials in
      // workgroup order.  One memory round trip per poll, no counter, no fences.  The tag carries the launch's epoch
      // and the pass, so granules left by earlier launches never match; the pass parity keeps a fast member off a
      // slow member's buffer (it cannot write pass k + 2 before every member has read pass k).
      typedef unsigned long long u64;
      u64* P = reinterpret_cast<u64*>(a.part) + ((size_t)h * 2 + (S.npass & 1)) * HS_TRK_MAXG * TRK_NRED * 2;
      const unsigned int tg = (a.epoch << HS_TRK_PASS_BITS) | (unsigned int)(S.npass + 1);
      const u64 tag = (u64)tg << 32;
#if TRK_MEET_F32
      // one granule per value: the member's block total rounded to fp32 (every consumer below reads the pass totals
      // as fp32: H / b from (float) tot, the energies and counts as floats / small integers), summed over the
      // members in fp64 in member order: half the stores and polled loads of the fp64 form
      if (lane < TRK_NRED)
        __hip_atomic_store(P + g * TRK_NRED + lane, tag | (u64)__float_as_uint((float)tot), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      u64 v[HS_TRK_MAXG];
      const long long pm0 = (a.trace && lane == 0) ? clock64() : 0;
      const unsigned long long t_end = wall_clock64() + (S.dead ? 0ull : (unsigned long long)a.spin_limit);
      for (;;) {
#pragma unroll
        for (int gg = 0; gg < HS_TRK_MAXG; gg++)
          if (gg < G) v[gg] = __hip_atomic_load(P + gg * TRK_NRED + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bool ok = true;
#pragma unroll
        for (int gg = 0; gg < HS_TRK_MAXG; gg++) ok &= gg >= G || (unsigned int)(v[gg] >> 32) == tg;
        if (__all(ok)) break;
        __builtin_amdgcn_s_sleep(1);
        if (wall_clock64() >= t_end) {  // a member never arrived (not co-resident): flag the hypothesis, go on
          if (lane == 0) {
            __hip_atomic_store(a.cnt + h, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            S.dead = 1;
          }
          break;
        }
      }
      if (a.trace && lane == 0) {
        S.prof[8] += clock64() - pm0;  // the meeting: own stores to every member's granules seen
        S.prof[9] += 1;
      }
      tot = 0.0;
#pragma unroll
      for (int gg = 0; gg < HS_TRK_MAXG; gg++)
        if (gg < G) tot += (double)__uint_as_float((unsigned int)(v[gg] & 0xffffffffull));
    }
#else
      if (lane < TRK_NRED) {
        const u64 bits = (u64)__double_as_longlong(tot);
        __hip_atomic_store(P + (g * TRK_NRED + lane) * 2, tag | (bits & 0xffffffffull), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(P + (g * TRK_NRED + lane) * 2 + 1, tag | (bits >> 32), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
      u64 v[2 * HS_TRK_MAXG];
      const long long pm0 = (a.trace && lane == 0) ? clock64() : 0;
      // the poll's time bound on the constant 100 MHz wall clock (spin_limit ticks, set by the host from the clock
      // rate); after a timeout (S.dead) a meeting polls once
      const unsigned long long t_end = wall_clock64() + (S.dead ? 0ull : (unsigned long long)a.spin_limit);
      for (;;) {
        bool ok = true;
#pragma unroll
        for (int gg = 0; gg < HS_TRK_MAXG; gg++)
          if (gg < G) {
            v[2 * gg] = __hip_atomic_load(P + (gg * TRK_NRED + q) * 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            v[2 * gg + 1] = __hip_atomic_load(P + (gg * TRK_NRED + q) * 2 + 1, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
          }
#pragma unroll
        for (int gg = 0; gg < HS_TRK_MAXG; gg++)
          if (gg < G) ok = ok && (unsigned int)(v[2 * gg] >> 32) == tg && (unsigned int)(v[2 * gg + 1] >> 32) == tg;
        if (__all(ok)) break;
        __builtin_amdgcn_s_sleep(1);
        if (wall_clock64() >= t_end) {  // a member never arrived (not co-resident): flag the hypothesis, go on
          if (lane == 0) {
            __hip_atomic_store(a.cnt + h, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            S.dead = 1;
          }
          break;
        }
      }
      if (a.trace && lane == 0) {
        S.prof[8] += clock64() - pm0;  // the meeting: own stores to every member's granules seen
        S.prof[9] += 1;
      }
      tot = 0.0;
      if (G == HS_TRK_MAXG) {  // (uniform) the production member count: no per-slot masks
#pragma unroll
        for (int gg = 0; gg < HS_TRK_MAXG; gg++)
          tot += __longlong_as_double((long long)((v[2 * gg] & 0xffffffffull) | (v[2 * gg + 1] << 32)));
      } else {
#pragma unroll
        for (int gg = 0; gg < HS_TRK_MAXG; gg++)
          if (gg < G) tot += __longlong_as_double((long long)((v[2 * gg] & 0xffffffffull) | (v[2 * gg + 1] << 32)));
      }
    }
#endif
    const float Ef = (float)trk_readlane_f64(tot, TRK_NACC + 0);
    const float fT = (float)trk_readlane_f64(tot, TRK_NACC + 1), fRT = (float)trk_readlane_f64(tot, TRK_NACC + 2);
    const float fN = (float)trk_readlane_f64(tot, TRK_NACC + 3);
    const int numE = (int)trk_readlane_f64(tot, TRK_NACC + 4), numSat = (int)trk_readlane_f64(tot, TRK_NACC + 5);
    const int numW = (int)trk_readlane_f64(tot, TRK_NACC + 6);
    // res[6] (Src/CoarseTracker.cpp:402-409), lane k < 6 forming res[k] alone: its quotient in parallel with the
    // other lanes' instead of three quotients in series on every lane
    const double r0 = Ef, r1 = numE;
    double rl;
    {
      const float q5 = numSat / (float)numE;
      const double q24 = (double)(lane == 4 ? fRT : fT) / (fN + 0.1);
      rl = lane == 0 ? r0 : lane == 1 ? r1 : lane == 3 ? 0.0 : lane == 5 ? (double)q5 : q24;
    }
    const int npad = (numW + 3) & ~3;  // buf_warped_n includes the zero padding (quirk kept)
    // lm: the LM iteration's accept test (Src/CoarseTracker.cpp:611-640) -- an accepted pass's normal equations
    // and residuals go straight to Hs / bs / resOld; a plain pass leaves them in H / b / res
    const double oldRatio = S.resOld[0] / S.resOld[1];
    const double newRatio = r0 / r1;
    const bool accept = lm && newRatio < oldRatio;
    double* Hd = accept ? S.Hs : S.H;
    double* bd = accept ? S.bs : S.b;
    if (lane < 6 && (!lm || accept)) (accept ? S.resOld : S.res)[lane] = rl;
    if (lane < 45 && (!lm || accept)) {  // H / b from the 45 upper-triangle sums (row-major), one entry per lane
      const int hp = S.hpos[lane];
      const double inv = (double)(1.0f / npad);
      const double vv = (double)(float)tot;
      const double sr = S.hsr[lane], scc = S.hsc[lane];
      if (hp >= 0 && !(hp & 0x10000)) {
        Hd[hp & 255] = ((vv * inv) * scc) * sr;
        Hd[(hp >> 8) & 255] = ((vv * inv) * sr) * scc;
      } else if (hp >= 0) {  // (8, 8) is the residual square sum, not part of H / b
        bd[hp & 255] = (vv * inv) * sr;
      }
    }
    const long long pt2 = (a.trace && lane == 0) ? clock64() : 0;
    if (lane == 0) {
      S.passes += 1;
      S.npass += 1;
      S.pointPasses += n;
      S.nWarped = npad;
      if (lm) {
        const int it = S.iters - 1;
        if (g == 0 && it < HS_TRK_MAXLOG) {
          a.lm_log[((size_t)h * HS_TRK_MAXLOG + it) * 3 + 0] = newRatio;
          a.lm_log[((size_t)h * HS_TRK_MAXLOG + it) * 3 + 1] = oldRatio;
          a.lm_log[((size_t)h * HS_TRK_MAXLOG + it) * 3 + 2] = S.incNorm;
          a.lm_lvl[(size_t)h * HS_TRK_MAXLOG + it] = lvl;
        }
        if (accept) {
          S.aff[0] = S.affn[0];
          S.aff[1] = S.affn[1];
          for (int k = 0; k < 7; k++) S.T[k] = S.Tn[k];
          for (int k = 0; k < 4; k++) S.Tq[k] = S.Tn[k];
          S.lambda *= 0.5;
        } else {
          S.lambda *= 4;
          if (S.lambda < 0.001f) S.lambda = 0.001f;  // lambdaExtrapolationLimit
        }
      }
      if (a.trace) {
        const long long pc2 = clock64() + (long long)(S.nWarped * 0);
        S.prof[0] += pc1 - pc0;
        S.prof[1] += pc2 - pc1;
        S.prof[3] += 1;
        S.prof[10] += pt1 - pt0;  // the 8-wave tree (LDS loads + adds)
        S.prof[11] += pt2 - pt1;  // the meeting (if any) + results to the H / b stores
        S.prof[12] += pc2 - pt2;  // lane 0's bookkeeping
      }
    }
  }
  __syncthreads();
}

// the pose part of the pass inputs from a unit quaternion (RKi) and / or a translation (t)
__device__ void trk_setup_pose(const HsTrackArgs& a, TrkShared& S, const hs::Quat* q, const double* t, int lvl) {
  if (q) {
    hs::SE3 T;
    T.q = *q;
    double Rd[9];
    T.rotationMatrix(Rd);
    float R[9];
    for (int k = 0; k < 9; k++) R[k] = (float)Rd[k];
    const float* Ki = a.lv[lvl].Ki;
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) S.RKi[r * 3 + c] = R[r * 3 + 0] * Ki[0 * 3 + c] + R[r * 3 + 1] * Ki[1 * 3 + c] + R[r * 3 + 2] * Ki[2 * 3 + c];
  }
  if (t)
    for (int k = 0; k < 3; k++) S.t[k] = (float)t[k];
}

// the pass inputs for state (T, aff) at level lvl: the pose part (pose = true: RKi, t) and / or the affine part
// (pose = false: the relative affine transfer, the cutoff); one thread each, or one thread both
__device__ void trk_setup_part(const HsTrackArgs& a, TrkShared& S, const double T7[7], const double aff[2], int lvl,
                               float cutoff, bool pose) {
  if (!pose) {
    double rel[2];
    hs::fromToVecExposure(a.refExposure, a.newExposure, a.refAff[0], a.refAff[1], aff[0], aff[1], rel);
    S.affLL[0] = (float)rel[0];
    S.affLL[1] = (float)rel[1];
    S.a_gs = (float)rel[0];
    S.b0 = (float)a.refAff[1];
    S.cutoff = cutoff;
    S.maxEnergy = 2 * a.huberTH * cutoff - a.huberTH * a.huberTH;
    S.lvl = lvl;
    S.npts = *a.lv[lvl].pc_n;
    S.Gl = S.npts < a.gmin ? 1 : a.G;
    return;
  }
  const hs::SE3 T = hs::SE3::fromData(T7);
  trk_setup_pose(a, S, &T.q, T.t, lvl);
}
__device__ void trk_setup(const HsTrackArgs& a, TrkShared& S, const double T7[7], const double aff[2], int lvl,
                          float cutoff) {
  trk_setup_part(a, S, T7, aff, lvl, cutoff, true);
  trk_setup_part(a, S, T7, aff, lvl, cutoff, false);
}

// the lead's output record, LDS -> a.out[h] (device) and, when the caller asked for it, a.hout[h] (mapped pinned
// host memory: the host reads it once the launch has completed, with no copy behind the kernel); wave 0, 8 B a lane
__device__ void trk_publish(const HsTrackArgs& a, TrkShared& S, int h, bool lead) {
  __syncthreads();
  if (!lead || threadIdx.x >= 64) return;
  constexpr int NW = sizeof(HsTryOut) / 8;
  static_assert(sizeof(HsTryOut) % 8 == 0, "output record in 8-B words");
  const unsigned long long* src = reinterpret_cast<const unsigned long long*>(&S.out);
  unsigned long long* dd = reinterpret_cast<unsigned long long*>(a.out + h);
  unsigned long long* dh = a.hout ? reinterpret_cast<unsigned long long*>(a.hout + h) : nullptr;
  for (int k = threadIdx.x; k < NW; k += 64) {
    const unsigned long long w = src[k];
    dd[k] = w;
    if (dh) dh[k] = w;
  }
  // the record (and any timeout flag this wave stored) before the done word: the release orders the wave's stores
  if (a.hdone && threadIdx.x == 0) __hip_atomic_store(a.hdone + h, a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace

// The end of a level that some members sat out (S.Gl < a.G): member 0 publishes the state the next level starts from
// -- T, its normalized quaternion, aff, the pass count (the pass meetings' parity and tags), the cutoff repeat
// factor (REPEAT LEVEL) and the LM iteration count -- as 32 tagged granules (two per value, as the pass meetings'
// partials); the other members poll them (bounded by the wall clock, as the pass meetings) and take them over.
__device__ void trk_level_meet(const HsTrackArgs& a, TrkShared& S, int h, int g) {
  typedef unsigned long long u64;
  __syncthreads();  // member 0: the level's last pass is in S
  if (threadIdx.x < 64) {
    // the lane index read here (volatile: not hoisted to the kernel's entry, where the lane terms of this rare path
    // were kept live across the whole kernel -- spilled to scratch -- and reloaded at every level meeting)
    int lane;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
    const int q = lane >> 1;
    u64* R = a.lvrec + ((size_t)h * HS_TRK_MAXLVSEQ + min(S.lvseq, HS_TRK_MAXLVSEQ - 1)) * 32;
    const unsigned int tg = (a.epoch << 8) | (unsigned int)(S.lvseq + 1);
    if (g == 0) {
      if (lane < 32) {
        const double v = q < 7 ? S.T[q] : q < 11 ? S.Tq[q - 7] : q < 13 ? S.aff[q - 11] : q == 13 ? (double)S.npass
                         : q == 14 ? (double)S.cutoffRep : (double)S.iters;
        const u64 bits = (u64)__double_as_longlong(v);
        __hip_atomic_store(R + lane, ((u64)tg << 32) | ((lane & 1) ? (bits >> 32) : (bits & 0xffffffffull)),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    } else if (g >= S.Gl) {  // (the level's other members hold the same state already)
      const unsigned long long t_end = wall_clock64() + (S.dead ? 0ull : (unsigned long long)a.spin_limit);
      u64 w = 0;
      for (;;) {
        w = __hip_atomic_load(R + min(lane, 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (__all((unsigned int)(w >> 32) == tg)) break;
        __builtin_amdgcn_s_sleep(1);
        if (wall_clock64() >= t_end) {
          if (lane == 0) {
            __hip_atomic_store(a.cnt + h, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            S.dead = 1;
          }
          break;
        }
      }
      // lane 2 q + 1 holds value q's high half: pair it with the low half of lane 2 q
      const unsigned int lo = (unsigned int)(w & 0xffffffffull);
      const unsigned int hi = (unsigned int)__builtin_amdgcn_ds_bpermute((lane + 1) << 2, (int)lo);
      const double v = __longlong_as_double((long long)(((u64)hi << 32) | lo));
      if (!S.dead && lane < 32 && !(lane & 1)) {
        if (q < 7) S.T[q] = v;
        else if (q < 11) S.Tq[q - 7] = v;
        else if (q < 13) S.aff[q - 11] = v;
        else if (q == 13) S.npass = (int)v;
        else if (q == 14) S.cutoffRep = (float)v;
        else S.iters = (int)v;
      }
    }
  }
  if (threadIdx.x == 0) S.lvseq += 1;
  __syncthreads();
}

__global__ __launch_bounds__(TRK_NT) void hs_k_track(HsTrackArgs a) {
  __shared__ TrkShared S;
  const int tid = threadIdx.x;
  const int h = blockIdx.x / a.G, g = blockIdx.x - h * a.G;  // hypothesis, member workgroup
  if (a.trace && tid == 0) {  // placement probe: the XCD (HW_REG_XCC_ID) and CU (HW_REG_HW_ID bits 11:8) of the block
    const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 15u;
    const unsigned cu = (__builtin_amdgcn_s_getreg((31 << 11) | 4) >> 8) & 15u;
    a.trace[(size_t)blockIdx.x * 16 + 14] = (long long)(xcc | (cu << 4) | ((unsigned)h << 8) | ((unsigned)g << 16));
  }
  const bool lead = g == 0;  // the workgroup that writes the hypothesis' outputs (every member computes them)
  HsTryOut& out = S.out;  // staged in LDS, published by trk_publish
  HS_TRACE(a, 0);
  if (tid < 64) {  // the pass tail's per-lane normal-equation entry and scales (S.hpos; ordered by the first barrier)
    int qq = tid, r = 0;
    while (r < 9 && qq >= 9 - r) {
      qq -= 9 - r;
      r++;
    }
    const int c = r + qq;
    S.hpos[tid] = tid >= 45 || (r == 8 && c == 8) ? -1 : (c < 8 ? (r * 8 + c) | ((c * 8 + r) << 8) : r | 0x10000);
    S.hsr[tid] = r < 3 ? hs_trk_scale_rot : r < 6 ? hs_trk_scale_trans : r == 6 ? hs_trk_scale_a : hs_trk_scale_b;
    S.hsc[tid] = c < 3 ? hs_trk_scale_rot : c < 6 ? hs_trk_scale_trans : c == 6 ? hs_trk_scale_a : hs_trk_scale_b;
  }
  if (a.single_pass) {  // hs_tracker_calc_res
    if (tid == 0) {
      S.dead = 0;
      S.passes = 0;
      S.npass = 0;
      S.pointPasses = 0;
      double T7[7], aff[2];
      for (int q = 0; q < 7; q++) T7[q] = a.n_inl ? a.inl[7 * h + q] : a.T_in[7 * h + q];
      for (int q = 0; q < 2; q++) aff[q] = a.n_inl ? a.inl[7 * a.n_inl + 2 * h + q] : a.aff_in[2 * h + q];
      trk_setup(a, S, T7, aff, a.pass_lvl, a.pass_cutoff);
    }
    __syncthreads();
    trk_pass(a, S, h, g);
    if (tid == 0 && lead) {
      for (int q = 0; q < 6; q++) out.res6[q] = S.res[q];
      for (int q = 0; q < 64; q++) out.H[q] = S.H[q];
      for (int q = 0; q < 8; q++) out.b[q] = S.b[q];
      out.n_warped = S.nWarped;
    }
    trk_publish(a, S, h, lead);
    return;
  }
  const int maxIterations[5] = {10, 20, 50, 50, 50};
  const float lambdaExtrapolationLimit = 0.001f;
  if (tid == 0) {
    for (int q = 0; q < 7; q++) S.T[q] = a.n_inl ? a.inl[7 * h + q] : a.T_in[7 * h + q];
    const hs::SE3 T0 = hs::SE3::fromData(S.T);
    S.Tq[0] = T0.q.x;
    S.Tq[1] = T0.q.y;
    S.Tq[2] = T0.q.z;
    S.Tq[3] = T0.q.w;
    S.aff[0] = a.n_inl ? a.inl[7 * a.n_inl + 2 * h + 0] : a.aff_in[2 * h + 0];
    S.aff[1] = a.n_inl ? a.inl[7 * a.n_inl + 2 * h + 1] : a.aff_in[2 * h + 1];
    S.nchecks = 0;
    S.lvseq = 0;
    S.dead = 0;
    S.iters = 0;
    S.npass = 0;
    S.passes = 0;
    S.pointPasses = 0;
    for (int q = 0; q < 13; q++) S.prof[q] = 0;
  }
  __syncthreads();
  bool haveRepeated = false;
  for (int lvl = a.coarsest; lvl >= 0 && !S.dead; lvl--) {  // (S.dead: uniform, read after a pass' barrier)
    if (tid == 0) {
      S.cutoffRep = 1;
      trk_setup(a, S, S.T, S.aff, lvl, a.coarseCutoffTH * S.cutoffRep);
    }
    __syncthreads();
    const bool active = g < S.Gl;  // uniform: the level's members
    if (active) {
    trk_pass(a, S, h, g);
    while (S.res[5] > 0.6 && S.cutoffRep < 50 && !S.dead) {  // uniform: S.res / S.cutoffRep are shared
      __syncthreads();
      if (tid == 0) {
        S.cutoffRep *= 2;
        trk_setup(a, S, S.T, S.aff, lvl, a.coarseCutoffTH * S.cutoffRep);
      }
      __syncthreads();
      trk_pass(a, S, h, g);
    }
    if (tid == 0) {  // calcGSSSE of the last calcRes; lambda = 0.01
      for (int q = 0; q < 64; q++) S.Hs[q] = S.H[q];
      for (int q = 0; q < 8; q++) S.bs[q] = S.b[q];
      for (int q = 0; q < 6; q++) S.resOld[q] = S.res[q];
      S.lambda = 0.01f;
    }
    __syncthreads();
    for (int iteration = 0; iteration < maxIterations[lvl]; iteration++) {
      // the LM step on four waves, each solving the same 8x8 system (same inputs, same increment), then lane 0 of
      // each takes a part: wave 0 the rotation (exp, product: the new quaternion, RKi), wave 2 the translation
      // (exp's V a plus the rotated old translation; it recomputes the exp quaternion), wave 3 the increment norm /
      // break test, wave 1 the affine part (fromToVecExposure).  A rotation beyond the series range (theta^2 >= 1e-2)
      // runs the whole reference exp and product on wave 0.  S.Tq is S.T's quaternion normalized (once at the start;
      // every product normalizes its own).
      if (tid < 256) {
        const int wv = tid >> 6;
        const long long lm0 = a.trace ? clock64() : 0;
        double mb[8], inc[8];
#pragma unroll
        for (int i = 0; i < 8; i++) mb[i] = -S.bs[i];
        if (a.solve == 0)
          gj8_solve_wave(S.Hs, mb, inc, 1 + S.lambda, tid & 63);
        else
          ldlt8_solve_wave(S.Hs, mb, inc, 1 + S.lambda, tid & 63);
        if ((tid & 63) == 0) {
          const long long lm1 = a.trace ? clock64() + (long long)(inc[7] * 0.0) : 0;
          float extrapFac = 1;
          if (S.lambda < lambdaExtrapolationLimit) extrapFac = sqrtf(sqrtf(lambdaExtrapolationLimit / S.lambda));
          for (int i = 0; i < 8; i++) inc[i] *= extrapFac;
          double incScaled[8];
          for (int i = 0; i < 8; i++) incScaled[i] = inc[i];
          for (int i = 0; i < 3; i++) incScaled[i] *= hs_trk_scale_rot;
          for (int i = 3; i < 6; i++) incScaled[i] *= hs_trk_scale_trans;
          incScaled[6] *= hs_trk_scale_a;
          incScaled[7] *= hs_trk_scale_b;
          double ssum = 0;
          for (int i = 0; i < 8; i++) ssum += incScaled[i];
          if (!isfinite(ssum))
            for (int i = 0; i < 8; i++) incScaled[i] = 0;
          const double u = se3_step_u(incScaled);
          const bool series = u < 1e-2;
          if (wv == 0) {
            S.iters++;
            const hs::Quat Tq{S.Tq[0], S.Tq[1], S.Tq[2], S.Tq[3]};
            if (series) {
              const hs::Quat q = se3_mul_step_q(se3_exp_step_q(incScaled, u), Tq);
              S.Tn[0] = q.x;
              S.Tn[1] = q.y;
              S.Tn[2] = q.z;
              S.Tn[3] = q.w;
              trk_setup_pose(a, S, &q, nullptr, lvl);
            } else {
              hs::SE3 T;
              T.q = Tq;
              for (int k = 0; k < 3; k++) T.t[k] = S.T[4 + k];
              const hs::SE3 nw = se3_mul_step(se3_exp_step(incScaled), T);
              nw.toData(S.Tn);
              trk_setup_pose(a, S, &nw.q, nw.t, lvl);
            }
            if (a.trace) {
              const long long lm2 = clock64() + (long long)(S.RKi[4] * 0.f);
              S.prof[6] += lm1 - lm0;
              S.prof[7] += lm2 - lm1;
              S.prof[2] += lm2 - lm0;
            }
          } else if (wv == 2) {
            if (series) {
              const hs::Quat qe = se3_exp_step_q(incScaled, u);
              double te[3], rt[3], tn[3];
              se3_exp_step_t(incScaled, u, te);
              const double tT[3] = {S.T[4], S.T[5], S.T[6]};
              hs::qrot(qe, tT, rt);
              for (int k = 0; k < 3; k++) tn[k] = te[k] + rt[k];
              S.Tn[4] = tn[0];
              S.Tn[5] = tn[1];
              S.Tn[6] = tn[2];
              trk_setup_pose(a, S, nullptr, tn, lvl);
            }
          } else if (wv == 3) {
            double nn = 0;
            for (int i = 0; i < 8; i++) nn += inc[i] * inc[i];
            S.incNorm = sqrt(nn);
            S.brk[iteration & 1] = !(S.incNorm > 1e-3);
          } else {
            double affn[2] = {S.aff[0] + incScaled[6], S.aff[1] + incScaled[7]};
            S.affn[0] = affn[0];
            S.affn[1] = affn[1];
            trk_setup_part(a, S, nullptr, affn, lvl, a.coarseCutoffTH * S.cutoffRep, false);
          }
        }
      }
      __syncthreads();
      trk_pass(a, S, h, g, true);  // the pass, the accept test and the state update; ends with a barrier
      if (S.brk[iteration & 1] || S.dead) break;  // (parity: the next step writes the other slot while slow waves read)
    }
    if (tid == 0) {  // lastResiduals[lvl] / lastFlowIndicators: logged for the caller's abort replay
      const int c = S.nchecks;
      if (lead && c < HS_TRK_MAXCHECK) {
        out.check_lvl[c] = lvl;
        out.check_res[c] = sqrtf((float)(S.resOld[0] / S.resOld[1]));
        out.check_flow[c][0] = S.resOld[2];
        out.check_flow[c][1] = S.resOld[3];
        out.check_flow[c][2] = S.resOld[4];
      }
      S.nchecks = c < HS_TRK_MAXCHECK ? c + 1 : c;
    }
    }  // active
    if (S.Gl < a.G) trk_level_meet(a, S, h, g);  // the members that sat the level out take member 0's state
    const bool rep = S.cutoffRep > 1 && !haveRepeated;
    __syncthreads();
    if (rep) {  // REPEAT LEVEL
      lvl++;
      haveRepeated = true;
    }
  }
  if (tid == 0 && lead) {
    out.iters = S.iters;
    out.n_checks = S.nchecks;
    for (int q = 0; q < 7; q++) out.T[q] = S.T[q];
    out.aff[0] = S.aff[0];
    out.aff[1] = S.aff[1];
    bool ok = true;
    if ((a.affineOptModeA != 0 && (fabsf((float)S.aff[0]) > 1.2f)) ||
        (a.affineOptModeB != 0 && (fabsf((float)S.aff[1]) > 200)))
      ok = false;
    double rel[2];
    hs::fromToVecExposure(a.refExposure, a.newExposure, a.refAff[0], a.refAff[1], S.aff[0], S.aff[1], rel);
    if ((a.affineOptModeA == 0 && (fabsf(logf((float)rel[0])) > 1.5f)) ||
        (a.affineOptModeB == 0 && (fabsf((float)rel[1]) > 200)))
      ok = false;
    if (a.affineOptModeA < 0) out.aff[0] = 0;
    if (a.affineOptModeB < 0) out.aff[1] = 0;
    out.ok = ok ? 1 : 0;
    out.passes = S.passes;
    out.point_passes = S.pointPasses;
    if (a.trace) {
      for (int q = 0; q < 10; q++) a.trace[(size_t)blockIdx.x * 16 + 4 + q] = S.prof[q];
      for (int q = 0; q < 3; q++) a.trace[(size_t)blockIdx.x * 16 + 1 + q] = S.prof[10 + q];
    }
  }
  trk_publish(a, S, h, lead);
  HS_TRACE(a, 15);
}

// ---------------------------------------------------------------- makeCoarseDepthL0
__device__ void hs_k_trk_scatter_seq(int n, const float* cu, const float* cv, const float* cid, const float* hdi,
                                     int w, int h, float* idepth0, float* wsum0) {
  for (int i = 0; i < n; i++) {  // the reference's order: colliding points add in sequence
    const int u = (int)(cu[i] + 0.5f);
    const int v = (int)(cv[i] + 0.5f);
    if (u < 0 || v < 0 || u >= w || v >= h) continue;  // the reference assumes in-image centres
    const float new_idepth = cid[i];
    const float weight = sqrtf(1e-3 / (hdi[i] + 1e-12));
    idepth0[u + w * v] += new_idepth * weight;
    wsum0[u + w * v] += weight;
  }
}

__global__ void hs_k_trk_scatter(int n, const float* cu, const float* cv, const float* cid, const float* hdi, int w,
                                 int h, float* idepth0, float* wsum0) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  hs_k_trk_scatter_seq(n, cu, cv, cid, hdi, w, h, idepth0, wsum0);
}

// makeCoarseDepthL0's point loop in parallel with the sequential loop's sums: the points are sorted by (pixel,
// point index) in LDS (bitonic, one workgroup), and the first point of every pixel's run adds the run in point order,
// starting from the memset zero -- the very additions of the sequential loop, so the maps are bit-identical.  n comes
// from the device (d_n, the BA hand-off's count) or the argument; more than kScatCap points fall back to the loop.
constexpr int kScatCap = 8192;
__global__ __launch_bounds__(1024) void hs_k_trk_scatter_sorted(const int* d_n, int n_arg, const float* cu,
                                                                const float* cv, const float* cid, const float* hdi,
                                                                int w, int h, float* idepth0, float* wsum0) {
  extern __shared__ unsigned long long skey[];
  const int n = d_n ? *d_n : n_arg;
  const int tid = threadIdx.x;
  if (n > kScatCap) {
    if (tid == 0) hs_k_trk_scatter_seq(n, cu, cv, cid, hdi, w, h, idepth0, wsum0);
    return;
  }
  int N = 64;
  while (N < n) N <<= 1;
  for (int i = tid; i < N; i += 1024) {
    unsigned long long k = ~0ull;
    if (i < n) {
      const int u = (int)(cu[i] + 0.5f);
      const int v = (int)(cv[i] + 0.5f);
      if (!(u < 0 || v < 0 || u >= w || v >= h))
        k = ((unsigned long long)(unsigned)(u + w * v) << 32) | (unsigned)i;
    }
    skey[i] = k;
  }
  __syncthreads();
  for (int kk = 2; kk <= N; kk <<= 1)
    for (int j = kk >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < N; i += 1024) {
        const int l = i ^ j;
        if (l > i) {
          const unsigned long long a = skey[i], b = skey[l];
          if ((a > b) == ((i & kk) == 0)) {
            skey[i] = b;
            skey[l] = a;
          }
        }
      }
      __syncthreads();
    }
  for (int i = tid; i < n; i += 1024) {
    const unsigned long long k = skey[i];
    if (k == ~0ull) continue;
    const unsigned pix = (unsigned)(k >> 32);
    if (i > 0 && (unsigned)(skey[i - 1] >> 32) == pix) continue;  // not the first point of its pixel
    float s = 0.f, sw = 0.f;
    for (int q = i; q < n && (unsigned)(skey[q] >> 32) == pix; q++) {
      const int p = (int)(skey[q] & 0xffffffffull);
      const float weight = sqrtf(1e-3 / (hdi[p] + 1e-12));
      s += cid[p] * weight;
      sw += weight;
    }
    idepth0[pix] = s;
    wsum0[pix] = sw;
  }
}

__global__ void hs_k_trk_down(int wl, int hl, int wlm1, const float* idm, const float* wsm, float* idl, float* wsl) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= wl * hl) return;
  const int y = i / wl, x = i - y * wl;
  const int b = 2 * x + 2 * y * wlm1;
  idl[i] = idm[b] + idm[b + 1] + idm[b + wlm1] + idm[b + wlm1 + 1];
  wsl[i] = wsm[b] + wsm[b + 1] + wsm[b + wlm1] + wsm[b + wlm1 + 1];
}

// reads only pixels with bak > 0 and writes only pixels with bak <= 0: race free in parallel
__global__ void hs_k_trk_dilate(int wl, int hl, int diag, const float* bak, float* id, float* ws) {
  const int i = wl + blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= wl * hl - wl) return;
  if (bak[i] > 0) return;
  int o[4];
  if (diag) { o[0] = 1 + wl; o[1] = -1 - wl; o[2] = wl - 1; o[3] = -wl + 1; }
  else { o[0] = 1; o[1] = -1; o[2] = wl; o[3] = -wl; }
  float sum = 0, num = 0, numn = 0;
  const int n = wl * hl;
#pragma unroll
  for (int q = 0; q < 4; q++)
    // the reference reads one element past either end at pixels (0,1) / (w-1,h-2) (CoarseTracker.cpp:175-178);
    // those two pixels never reach pc_* (border 2), so out-of-range neighbours count as empty
    if (i + o[q] >= 0 && i + o[q] < n && bak[i + o[q]] > 0) {
      sum += id[i + o[q]];
      num += bak[i + o[q]];
      numn++;
    }
  if (numn > 0) {
    id[i] = sum / numn;
    ws[i] = num / numn;
  }
}

namespace {
__device__ __forceinline__ bool trk_keep(int i, int wl, int hl, const float* id, const float* ws, const float4* ref,
                                         float* idn) {
  const int y = i / wl, x = i - y * wl;
  if (y < 2 || y >= hl - 2 || x < 2 || x >= wl - 2) return false;
  if (!(ws[i] > 0)) return false;
  const float v = id[i] / ws[i];
  *idn = v;
  return isfinite(ref[i].x) && v > 0;
}
}  // namespace

__global__ __launch_bounds__(256) void hs_k_trk_count(int wl, int hl, const float* id, const float* ws,
                                                       const float4* ref, int* blockCount) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  float idn;
  const bool k = i < wl * hl && trk_keep(i, wl, hl, id, ws, ref, &idn);
  const int c = __syncthreads_count(k);
  if (threadIdx.x == 0) blockCount[blockIdx.x] = c;
}

// exclusive scan of the block counts (one workgroup); total -> *pc_n
__global__ __launch_bounds__(1024) void hs_k_trk_scan(int nb, const int* blockCount, int* blockOff, int* pc_n) {
  __shared__ int s[1024];
  __shared__ int carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int base = 0; base < nb; base += 1024) {
    const int i = base + threadIdx.x;
    const int v = i < nb ? blockCount[i] : 0;
    s[threadIdx.x] = v;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
      const int t = threadIdx.x >= o ? s[threadIdx.x - o] : 0;
      __syncthreads();
      s[threadIdx.x] += t;
      __syncthreads();
    }
    if (i < nb) blockOff[i] = carry + s[threadIdx.x] - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry += s[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) *pc_n = carry;
}

__global__ __launch_bounds__(256) void hs_k_trk_compact(int wl, int hl, const float* id, const float* ws,
                                                         const float4* ref, const int* blockOff, float* pu, float* pv,
                                                         float* pid, float* pcol) {
  __shared__ int waveCnt[4];
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float idn = 0.f;
  const bool k = i < wl * hl && trk_keep(i, wl, hl, id, ws, ref, &idn);
  const unsigned long long bal = __ballot(k);
  if (lane == 0) waveCnt[wv] = __popcll(bal);
  __syncthreads();
  int off = blockOff[blockIdx.x];
  for (int w = 0; w < wv; w++) off += waveCnt[w];
  off += __popcll(bal & ((1ull << lane) - 1ull));
  if (k) {
    const int y = i / wl, x = i - y * wl;
    pu[off] = (float)x;
    pv[off] = (float)y;
    pid[off] = idn;
    pcol[off] = ref[i].x;
  }
}
