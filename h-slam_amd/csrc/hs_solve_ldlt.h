// hs_solve_ldlt.h -- the fp64 LDLT pieces of hs_k_solve shared with tools/micro/ldlt_wave.hip: the single-wave
// factorization (lane = frame row) and the backward pass.  Device code; include after hip_runtime.h.
#pragma once
#include <cfloat>

#include "hs_kernels.h"

namespace hs_solve {

constexpr int LSTR = HS_MAXDIM + 2;  // padded row stride of LT (even: 16 B aligned 4-entry groups)

__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), lane);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// 1/d: v_rcp_f64 (~2^-26 relative) refined by ONE Newton step (~2^-50, 4e-15 relative) -- the pivots' error
// then sits ~1e11 below the 1e-3 tolerance on x, and the LDLT's critical path is 68 reciprocals long;
// 0 for a (near-)zero pivot
__device__ __forceinline__ double rcp_f64(double d) {
  double r = __builtin_amdgcn_rcp(d);
  const double e = __builtin_fma(-d, r, 1.0);
  r = __builtin_fma(r, e, r);
  return fabs(d) > DBL_MIN ? r : 0.0;
}

// D^-1 z, then L^T x = D^-1 z by wave 0 from LT, the pivots Dv = W + 24 MD and the forward-substituted rhs
// yf = W + 25 MD: lane i owns row i (< 64); rows 64 .. n-1 (at most the last block) are solved uniformly first.
// Per 4-row block the unknowns are solved uniformly from the block's diagonal L entries, then every lane updates
// its row in decreasing k; LT is zero on and above the diagonal, so the updates need no masks and a row of the
// block ends equal to its unknown.
__device__ __forceinline__ void ldlt_backward(const double* LT, double* W, double* yv, int n, int tid, long long* trace) {
  constexpr int MD = HS_MAXDIM;
  const double* Dv = W + 24 * MD;
  const double* yf = W + 25 * MD;
  const bool pw = tid < 64;
  if (pw) {
    const int i = tid;
    const int ci = min(i, n - 1);
    double y = i < n ? yf[ci] * rcp_f64(Dv[ci]) : 0.0;
    int kb = (n >> 2) - 1;
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
    }
    (void)kb;
    // blocks 15 .. 0 unrolled (no loop-carried branches, so the LT loads of later blocks are issued early); the
    // blocks at and beyond nb (n <= 64) are all zero (LT zeroed at entry, y = 0 past n) and leave y unchanged
#pragma unroll
    for (int kb2 = 15; kb2 >= 0; kb2--) {
      const int kb = kb2;
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

// Single-wave right-looking LDLT (no workgroup barrier): lane l holds row l + 4 of the scaled system in registers
// (68 doubles), the calib rows 0..3 are uniform and go first.  Per pivot k: the pivot by readlane (uniform for the
// calib pivots), its reciprocal, the column A(m, k) broadcast through 64 doubles of LDS (one wave: LDS operations
// complete in order, so the next pivot's store cannot overtake this pivot's loads), then one FMA per trailing
// column on every lane, 8 columns per scheduling group (the loads of a group in flight together, no more: the row
// already takes 136 registers); the rhs is forward-substituted alongside.  L goes to LT as it is formed
// (LT[k * LSTR + r] = L(r, k)), with the pivots Dv and the forward-substituted rhs yf, for ldlt_backward.
// Wave 0 only.
template <int K, int MD>
__device__ __forceinline__ void ldlt_wave_update(double (&a)[MD], double lk, const double* colb) {
  // a[m] -= lk A(m, K) for m = K+1 .. MD-1, in groups of 8 columns
#pragma unroll
  for (int c0 = K + 1; c0 < MD; c0 += 8) {
    asm volatile("" ::: "memory");
    double cv[8];
#pragma unroll
    for (int q = 0; q < 8; q++)
      if (c0 + q < MD) cv[q] = colb[c0 + q - 4];
#pragma unroll
    for (int q = 0; q < 8; q++)
      if (c0 + q < MD) a[c0 + q] = __builtin_fma(-lk, cv[q], a[c0 + q]);
    // the group's updates happen here: without these pins the scheduler runs ahead on the pivot chain and keeps
    // the deferred groups' loaded columns live (thousands of spilled registers)
#pragma unroll
    for (int q = 0; q < 8; q++)
      if (c0 + q < MD) asm volatile("" : "+v"(a[c0 + q]));
  }
}

template <int K, int MD>
__device__ __forceinline__ void ldlt_wave_frames(double (&a)[MD], double& y, double* colb, double* LT, double* Dv,
                                                 int n, int lane, int r, bool live) {
  if constexpr (K < MD) {
    {  // K >= n: the pivot lane is past the window (zero row): d = 0, dinv = 0, lk = 0, nothing changes
      constexpr int p = K - 4;
      const double d = readlane_f64(a[K], p);
      const double yk = readlane_f64(y, p);
      colb[lane] = a[K];
      const double dinv = rcp_f64(d);
      const bool below = lane > p;
      const double lk = below ? a[K] * dinv : 0.0;
      y = __builtin_fma(-lk, yk, y);
      if (below && live) LT[K * LSTR + r] = lk;
      if (lane == 0) Dv[K] = d;
      ldlt_wave_update<K, MD>(a, lk, colb);
      ldlt_wave_frames<K + 1, MD>(a, y, colb, LT, Dv, n, lane, r, live);
    }
  }
}

static __device__ __attribute__((noinline)) void ldlt_factor_wave(const double* M, double* LT, double* W, const double* yv, int n,
                                                 int lane) {
  constexpr int MD = HS_MAXDIM;
  static_assert(MD == 68, "lane = frame row: 64 frame rows + 4 calib rows");
  double* colb = W;  // [64]
  double* Dv = W + 24 * MD;
  double* yf = W + 25 * MD;
  const int r = lane + 4;
  const bool live = r < n;
  const int rr = live ? r : 4;
  double a[MD];
#pragma unroll
  for (int j = 0; j < MD; j++) a[j] = (live && j < n) ? M[rr * n + j] : 0.0;
  double y = live ? yv[rr] : 0.0;
  double C[4][4], yc[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    yc[i] = yv[i];
#pragma unroll
    for (int j = 0; j < 4; j++) C[i][j] = M[i * n + j];
  }
#pragma unroll
  for (int k = 0; k < 4; k++) {  // the calib pivots (uniform)
    const double d = C[k][k];
    const double dinv = rcp_f64(d);
    colb[lane] = a[k];
    const double lk = a[k] * dinv;
    double lc[4];
#pragma unroll
    for (int j = k + 1; j < 4; j++) lc[j] = C[j][k] * dinv;
    y = __builtin_fma(-lk, yc[k], y);
#pragma unroll
    for (int j = k + 1; j < 4; j++) yc[j] = __builtin_fma(-lc[j], yc[k], yc[j]);
#pragma unroll
    for (int m = k + 1; m < 4; m++) a[m] = __builtin_fma(-lk, C[m][k], a[m]);
#pragma unroll
    for (int j = k + 1; j < 4; j++)
#pragma unroll
      for (int m = k + 1; m <= j; m++) C[j][m] = __builtin_fma(-lc[j], C[m][k], C[j][m]);
    if (live) LT[k * LSTR + r] = lk;
    if (lane == 0) {
      Dv[k] = d;
      yf[k] = yc[k];
#pragma unroll
      for (int j = k + 1; j < 4; j++) LT[k * LSTR + j] = lc[j];
    }
    ldlt_wave_update<3, MD>(a, lk, colb);  // columns 4 .. MD-1 (the calib columns m < 4 were updated above)
  }
  ldlt_wave_frames<4, MD>(a, y, colb, LT, Dv, n, lane, r, live);
  if (live) yf[r] = y;
}

// The same factorization software-pipelined by one pivot: step K first applies its update to column K + 1 and the
// rhs, publishes column K + 1 (the other of two LDS column buffers) and forms pivot K + 1 (readlane, reciprocal)
// -- that dependent chain then overlaps step K's remaining column groups instead of following them.
template <int K, int MD>
__device__ __forceinline__ void ldlt_wave_pipe(double (&a)[MD], double& y, double* colb, double* LT, double* Dv,
                                               int lane, int r, bool live, double lk, double yk) {
  if constexpr (K < MD) {
    const double* cb = colb + (K & 1) * 64;  // column K: A(m, K) of rows m > K (lane m - 4)
    double* cn = colb + ((K + 1) & 1) * 64;
    y = __builtin_fma(-lk, yk, y);
    double lk1 = 0.0, yk1 = 0.0;
    if constexpr (K + 1 < MD) {
      a[K + 1] = __builtin_fma(-lk, cb[K + 1 - 4], a[K + 1]);
      constexpr int p1 = K + 1 - 4;
      const double d1 = readlane_f64(a[K + 1], p1);
      yk1 = readlane_f64(y, p1);
      cn[lane] = a[K + 1];
      const double dinv1 = rcp_f64(d1);
      lk1 = lane > p1 ? a[K + 1] * dinv1 : 0.0;
      if (lane == 0) Dv[K + 1] = d1;
      asm volatile("" : "+v"(a[K + 1]), "+v"(lk1), "+v"(y));
    }
    if (lane > K - 4 && live) LT[K * LSTR + r] = lk;
    ldlt_wave_update<K + 1, MD>(a, lk, cb);  // columns K + 2 .. MD - 1
    ldlt_wave_pipe<K + 1, MD>(a, y, colb, LT, Dv, lane, r, live, lk1, yk1);
  }
}

static __device__ __attribute__((noinline)) void ldlt_factor_wave_pipe(const double* M, double* LT, double* W, const double* yv, int n,
                                                      int lane) {
  constexpr int MD = HS_MAXDIM;
  double* colb = W;  // [2][64]
  double* Dv = W + 24 * MD;
  double* yf = W + 25 * MD;
  const int r = lane + 4;
  const bool live = r < n;
  const int rr = live ? r : 4;
  double a[MD];
#pragma unroll
  for (int j = 0; j < MD; j++) a[j] = (live && j < n) ? M[rr * n + j] : 0.0;
  double y = live ? yv[rr] : 0.0;
  double C[4][4], yc[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    yc[i] = yv[i];
#pragma unroll
    for (int j = 0; j < 4; j++) C[i][j] = M[i * n + j];
  }
  double* cb = colb + 64;  // the calib steps' column buffer (the frame steps start at buffer 0)
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const double d = C[k][k];
    const double dinv = rcp_f64(d);
    cb[lane] = a[k];
    const double lk = a[k] * dinv;
    double lc[4];
#pragma unroll
    for (int j = k + 1; j < 4; j++) lc[j] = C[j][k] * dinv;
    y = __builtin_fma(-lk, yc[k], y);
#pragma unroll
    for (int j = k + 1; j < 4; j++) yc[j] = __builtin_fma(-lc[j], yc[k], yc[j]);
#pragma unroll
    for (int m = k + 1; m < 4; m++) a[m] = __builtin_fma(-lk, C[m][k], a[m]);
#pragma unroll
    for (int j = k + 1; j < 4; j++)
#pragma unroll
      for (int m = k + 1; m <= j; m++) C[j][m] = __builtin_fma(-lc[j], C[m][k], C[j][m]);
    if (live) LT[k * LSTR + r] = lk;
    if (lane == 0) {
      Dv[k] = d;
      yf[k] = yc[k];
#pragma unroll
      for (int j = k + 1; j < 4; j++) LT[k * LSTR + j] = lc[j];
    }
    ldlt_wave_update<3, MD>(a, lk, cb);
  }
  // pivot 4 (lane 0), then the pipelined frame steps
  const double d4 = readlane_f64(a[4], 0);
  const double yk4 = readlane_f64(y, 0);
  colb[lane] = a[4];
  const double lk4 = lane > 0 ? a[4] * rcp_f64(d4) : 0.0;
  if (lane == 0) Dv[4] = d4;
  ldlt_wave_pipe<4, MD>(a, y, colb, LT, Dv, lane, r, live, lk4, yk4);
  if (live) yf[r] = y;
}

}  // namespace hs_solve
