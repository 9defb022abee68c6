// micro-benchmark + correctness check (gfx950) of hs_ldlt.h's barrier-free LDLT solve of the GN step's system
// (n = 4 + 8 nF), against a host fp64 unpivoted LDLT.  Prints per-phase shader cycles of the last launch.
// build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o ldlt8 ldlt8.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ldlt_blocks.h"

template <int W>
__global__ __launch_bounds__(64 * W) void k(const double* Ag, const double* bg, double* xg, int nF,
                                                   long long* tr, int* err) {
  __shared__ double A[68 * 68], y[68];
  __shared__ hs_ldlt::Lds L;
  __shared__ long long lt[64 * 4];
  const int tid = threadIdx.x, nt = blockDim.x, n = 4 + 8 * nF;
  for (int q = tid; q < n * n; q += nt) A[q] = Ag[q];
  if (tid < n) y[tid] = bg[tid];
  __syncthreads();
  if (tid == 0) tr[0] = clock64();
  if (tid == 0) tr[5] = wall_clock64();
  hs_ldlt::solve<W>(A, y, nF, L, tid, tr, lt);
  __syncthreads();
  for (int q = tid; q < 64 * 4; q += nt) tr[64 + q] = lt[q];
  if (tid == 0) tr[6] = wall_clock64();
  if (tid < n) xg[tid] = y[tid];
  if (tid == 0) *err = 0;
}

static void host_solve(const std::vector<double>& A, const std::vector<double>& b, int n, std::vector<double>& x) {
  std::vector<double> L(n * n, 0.0), D(n);
  for (int j = 0; j < n; j++) {
    double s = A[j * n + j];
    for (int k = 0; k < j; k++) s -= L[j * n + k] * L[j * n + k] * D[k];
    D[j] = s;
    for (int i = j + 1; i < n; i++) {
      double t = A[i * n + j];
      for (int k = 0; k < j; k++) t -= L[i * n + k] * L[j * n + k] * D[k];
      L[i * n + j] = t / s;
    }
  }
  std::vector<double> z(b);
  for (int i = 0; i < n; i++)
    for (int k = 0; k < i; k++) z[i] -= L[i * n + k] * z[k];
  for (int i = 0; i < n; i++) z[i] /= D[i];
  x = z;
  for (int i = n - 1; i >= 0; i--)
    for (int k = i + 1; k < n; k++) x[i] -= L[k * n + i] * x[k];
}

template <int W>
static int run(int nF, int reps) {
  const int n = 4 + 8 * nF;
  std::vector<double> R(n * n), A(n * n, 0.0), b(n);
  srand(7 + nF);
  for (auto& v : R) v = (rand() / (double)RAND_MAX - 0.5);
  for (int i = 0; i < n; i++)
    for (int j = 0; j < n; j++) {
      double s = 0;
      for (int k = 0; k < n; k++) s += R[i * n + k] * R[j * n + k] * std::pow(10.0, -5.0 * k / n);
      A[i * n + j] = s;
    }
  for (int i = 0; i < n; i++) A[i * n + i] += 1e-5;
  for (int i = 0; i < n; i++) b[i] = std::sin(1.0 + i);
  std::vector<double> xr;
  host_solve(A, b, n, xr);
  double *dA, *db, *dx;
  long long* dt;
  int* de;
  (void)hipMalloc(&dA, sizeof(double) * n * n);
  (void)hipMalloc(&db, sizeof(double) * n);
  (void)hipMalloc(&dx, sizeof(double) * n);
  (void)hipMalloc(&dt, sizeof(long long) * 512);
  (void)hipMemset(dt, 0, sizeof(long long) * 512);
  (void)hipMalloc(&de, sizeof(int));
  (void)hipMemcpy(dA, A.data(), sizeof(double) * n * n, hipMemcpyHostToDevice);
  (void)hipMemcpy(db, b.data(), sizeof(double) * n, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int r = 0; r < 3; r++) hipLaunchKernelGGL((k<W>), dim3(1), dim3(64 * W), 0, 0, dA, db, dx, nF, dt, de);
  (void)hipEventRecord(e0, 0);
  for (int r = 0; r < reps; r++) hipLaunchKernelGGL((k<W>), dim3(1), dim3(64 * W), 0, 0, dA, db, dx, nF, dt, de);
  (void)hipEventRecord(e1, 0);
  if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 1; }
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  std::vector<double> x(n);
  long long t[512];
  int err;
  (void)hipMemcpy(x.data(), dx, sizeof(double) * n, hipMemcpyDeviceToHost);
  (void)hipMemcpy(t, dt, sizeof(t), hipMemcpyDeviceToHost);
  (void)hipMemcpy(&err, de, sizeof(int), hipMemcpyDeviceToHost);
  double e2 = 0, r2 = 0;
  for (int i = 0; i < n; i++) { e2 += (x[i] - xr[i]) * (x[i] - xr[i]); r2 += xr[i] * xr[i]; }
  printf("W=%d nF=%d: rel err %.3e  err=%d  cycles: calib %lld  factor %lld  barrier %lld  back %lld  total %lld  "
         "wall %.2f us  launch avg %.2f us\n", W, nF, std::sqrt(e2 / r2), err, t[1] - t[0], t[2] - t[1], t[3] - t[2],
         t[4] - t[3], t[4] - t[0], (t[6] - t[5]) / 100.0, ms * 1e3 / reps);
  printf("   phase: start / apply done / own done / holder done (cycles from solve start)\n");
  for (int p = 0; p < 2 * nF; p++)
    printf("     %2d: %6lld %6lld %6lld %6lld\n", p, t[64 + p * 4] - t[0], t[65 + p * 4] - t[0], t[66 + p * 4] - t[0],
           t[67 + p * 4] - t[0]);
  return 0;
}

int main() {
  int rc = 0;
  for (int nF : {8}) {
    rc |= run<8>(nF, 200);
    rc |= run<16>(nF, 200);
  }
  return rc;
}
