// micro-benchmark + correctness check (gfx950) of hs_k_solve's single-wave LDLT (h-slam_amd/csrc/hs_solve_ldlt.h:
// ldlt_factor_wave + ldlt_backward) on a random SPD system of the GN step's size n = 4 + 8 nF, against a host fp64
// unpivoted LDLT.  Prints the factorization / backward shader cycles of the last launch.
// build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -I../../h-slam_amd/csrc -o ldlt_wave ldlt_wave.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "hs_solve_ldlt.h"

using namespace hs_solve;

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
