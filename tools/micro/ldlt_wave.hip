// Round-4 EXPERIMENT (not used by the product): a single-wave, barrier-free LDLT for hs_k_solve (lane = frame row,
// 68 doubles of the row in registers, the pivot column broadcast through LDS, plain and software-pipelined by one
// pivot), + hs_solve_ldlt.h's backward pass, on a random SPD system of the GN step's size n = 4 + 8 nF, against a
// host fp64 unpivoted LDLT.  Measured on MI355X (gpurun_out/r04_ab1, r04_ab2): factorization 44-56k cycles against
// ~31k for the product's panel LDLT (factor + backward): one wave issues the ~2000 trailing-update FMAs at ~20
// cycles each (LDS column reads in 8-column groups, 2 groups of prefetch); in the solve kernel the step went
// 44.7 -> 53-55 us.  Kept for the record.
// build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -I../../h-slam_amd/csrc -o ldlt_wave ldlt_wave.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "hs_solve_ldlt.h"

using namespace hs_solve;

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
  // a[m] -= lk A(m, K) for m = K+1 .. MD-1, in groups of 8 columns; the column loads run kPre groups ahead of the
  // FMAs that use them (the LDS latency of a group is ~8 FMAs' issue time)
  constexpr int C0 = K + 1;
  constexpr int NG = (MD - C0 + 7) / 8;
  constexpr int kPre = 2;
  if constexpr (NG > 0) {
    double cv[NG][8];
    auto load = [&](int g) {
#pragma unroll
      for (int q = 0; q < 8; q++)
        if (C0 + 8 * g + q < MD) cv[g][q] = colb[C0 + 8 * g + q - 4];
    };
#pragma unroll
    for (int g = 0; g < kPre && g < NG; g++) load(g);
#pragma unroll
    for (int g = 0; g < NG; g++) {
      if (g + kPre < NG) load(g + kPre);
#pragma unroll
      for (int q = 0; q < 8; q++)
        if (C0 + 8 * g + q < MD) a[C0 + 8 * g + q] = __builtin_fma(-lk, cv[g][q], a[C0 + 8 * g + q]);
      // the group's updates happen here: without these pins the scheduler runs ahead on the pivot chain and keeps
      // the deferred groups' loaded columns live (thousands of spilled registers)
#pragma unroll
      for (int q = 0; q < 8; q++)
        if (C0 + 8 * g + q < MD) asm volatile("" : "+v"(a[C0 + 8 * g + q]));
    }
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


template <bool PIPE>
__global__ __launch_bounds__(512) void k(const double* Ag, const double* bg, double* xg, int n, long long* tr) {
  __shared__ double A[HS_MAXDIM * HS_MAXDIM], LT[HS_MAXDIM * LSTR], W[26 * HS_MAXDIM], y[HS_MAXDIM];
  const int tid = threadIdx.x, nt = blockDim.x;
  for (int q = tid; q < n * n; q += nt) A[q] = Ag[q];
  for (int q = tid; q < HS_MAXDIM * LSTR; q += nt) LT[q] = 0.0;
  if (tid < n) y[tid] = bg[tid];
  __syncthreads();
  if (tid < 64) {
    const long long c0 = clock64();
    if (PIPE) ldlt_factor_wave_pipe(A, LT, W, y, n, tid);
    else ldlt_factor_wave(A, LT, W, y, n, tid);
    const long long c1 = clock64();
    ldlt_backward(LT, W, y, n, tid, nullptr);
    const long long c2 = clock64();
    if (tid == 0) {
      tr[0] = c1 - c0;
      tr[1] = c2 - c1;
    }
  }
  __syncthreads();
  if (tid < n) xg[tid] = y[tid];
}

static void host_solve(const std::vector<double>& A, const std::vector<double>& b, int n, std::vector<double>& x) {
  std::vector<double> L(n * n, 0.0), D(n);
  for (int j = 0; j < n; j++) {
    double s = A[j * n + j];
    for (int q = 0; q < j; q++) s -= L[j * n + q] * L[j * n + q] * D[q];
    D[j] = s;
    for (int i = j + 1; i < n; i++) {
      double t = A[i * n + j];
      for (int q = 0; q < j; q++) t -= L[i * n + q] * L[j * n + q] * D[q];
      L[i * n + j] = t / s;
    }
  }
  std::vector<double> z(b);
  for (int i = 0; i < n; i++)
    for (int q = 0; q < i; q++) z[i] -= L[i * n + q] * z[q];
  for (int i = 0; i < n; i++) z[i] /= D[i];
  x = z;
  for (int i = n - 1; i >= 0; i--)
    for (int q = i + 1; q < n; q++) x[i] -= L[q * n + i] * x[q];
}

template <bool PIPE>
static int run() {
  int bad = 0;
  for (int nF = 1; nF <= 8; nF++) {
    const int n = 4 + 8 * nF;
    std::vector<double> R(n * n), A(n * n, 0.0), b(n), x, xg(n);
    srand(7 + nF);
    for (auto& v : R) v = (rand() / (double)RAND_MAX - 0.5);
    for (int i = 0; i < n; i++)
      for (int j = 0; j < n; j++) {
        double s = 0;
        for (int q = 0; q < n; q++) s += R[i * n + q] * R[j * n + q];
        A[i * n + j] = s + (i == j ? 0.5 * n : 0.0);
      }
    for (auto& v : b) v = rand() / (double)RAND_MAX - 0.5;
    host_solve(A, b, n, x);
    double *dA, *db, *dx;
    long long* dt;
    if (hipMalloc(&dA, sizeof(double) * n * n) != hipSuccess || hipMalloc(&db, sizeof(double) * n) != hipSuccess ||
        hipMalloc(&dx, sizeof(double) * n) != hipSuccess || hipMalloc(&dt, sizeof(long long) * 2) != hipSuccess)
      return 2;
    (void)hipMemcpy(dA, A.data(), sizeof(double) * n * n, hipMemcpyHostToDevice);
    (void)hipMemcpy(db, b.data(), sizeof(double) * n, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int r = 0; r < 3; r++) hipLaunchKernelGGL(k<PIPE>, dim3(1), dim3(512), 0, 0, dA, db, dx, n, dt);
    (void)hipEventRecord(e0, 0);
    const int reps = 50;
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k<PIPE>, dim3(1), dim3(512), 0, 0, dA, db, dx, n, dt);
    (void)hipEventRecord(e1, 0);
    if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 1; }
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    long long t[2];
    (void)hipMemcpy(xg.data(), dx, sizeof(double) * n, hipMemcpyDeviceToHost);
    (void)hipMemcpy(t, dt, sizeof(t), hipMemcpyDeviceToHost);
    double num = 0, den = 0;
    for (int i = 0; i < n; i++) {
      num += (xg[i] - x[i]) * (xg[i] - x[i]);
      den += x[i] * x[i];
    }
    const double rel = std::sqrt(num / den);
    bad |= !(rel < 1e-10);
    printf("%s nF=%d n=%d: rel err %.3e  factor %lld cycles  backward %lld cycles  launch avg %.2f us\n", PIPE ? "pipe" : "plain", nF, n, rel,
           t[0], t[1], ms * 1e3 / reps);
    (void)hipFree(dA); (void)hipFree(db); (void)hipFree(dx); (void)hipFree(dt);
  }
  return bad;
}

int main() { return run<false>() | run<true>(); }
