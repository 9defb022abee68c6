// hs_solve_ldlt.h -- fp64 pieces of hs_k_solve's LDLT shared with tools/micro/ldlt_wave.hip: readlane / reciprocal
// helpers and the backward pass.  Device code; include after hip_runtime.h.
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

}  // namespace hs_solve
