// ldlt_rl.hip — round-6 measured attempt: a right-looking LDLT of the GN step's 68 x 68 fp64
// system with the trailing matrix in registers across the whole 512-thread workgroup and ONE LDS broadcast +
// barrier per column, against the product's panel LDLT (hs_k_solve's ldlt_solve_blocked, 17 4-column panels with
// one-panel look-ahead), both followed by the same backward pass (hs_solve_ldlt.h ldlt_backward), in the same
// harness, on random SPD systems scaled like the solve's S H S (unit diagonal).
//
// Right-looking form: thread t owns a segment of up to 5 consecutive entries (i, j0 .. j0+4) of one row of the lower
// triangle, the rhs as row n (its entries y_j); 512 threads cover n (n + 1) / 2 + n = 2414 entries at n = 68.  Per
// column k, after the barrier: every thread reads the published column k (col[k & 1][row]) and 1 / d_k, updates its
// entries j > k (a_ij -= a_ik a_jk / d_k), and the owners of column k + 1 update that entry first and publish it
// (the diagonal's owner also its reciprocal); the owners of column k write L(i, k) = a_ik / d_k into LT, the
// pivot and the rhs' final y_k; barrier.  68 phases of one dependent chain each: LDS read -> fma -> (rcp) -> LDS write
// -> barrier.
// build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -I../../h-slam_amd/csrc -o ldlt_rl ldlt_rl.hip
#include "../../h-slam_amd/csrc/hs_ba_kernels.hip"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace {
constexpr int MD = HS_MAXDIM;
constexpr int SEG = 5;

// the segment of thread t: row i (n = the rhs row), first column j0, count cnt (0: idle)
__device__ __forceinline__ void rl_segment(int t, int n, int& i, int& j0, int& cnt) {
  int s = t;
  for (int r = 0; r <= n; r++) {
    const int len = r < n ? r + 1 : n;  // lower triangle incl. diagonal; the rhs row: j < n
    const int ns = (len + SEG - 1) / SEG;
    if (s < ns) {
      i = r;
      j0 = s * SEG;
      cnt = min(SEG, len - j0);
      return;
    }
    s -= ns;
  }
  i = -1;
  j0 = 0;
  cnt = 0;
}

// forward part of the right-looking LDLT; outputs as ldlt_solve_blocked's factorization: LT (L transposed, zero on
// and above the diagonal, zero on entry), pivots Dv = W + 24 MD, forward-substituted rhs yf = W + 25 MD
__device__ void ldlt_rl(const double* M, double* LT, double* W, double* yv, int n, int tid, int i, int j0, int cnt) {
  double* col = W;                 // [2][MD + 2] published column, rows 0 .. n (n: the rhs), 1 / d at [MD + 1]
  double* Dv = W + 24 * MD;
  double* yf = W + 25 * MD;
  double a[SEG];
#pragma unroll
  for (int c = 0; c < SEG; c++) a[c] = c < cnt ? (i < n ? M[i * n + j0 + c] : yv[j0 + c]) : 0.0;
  // column 0 and 1 / d_0
  if (cnt > 0 && j0 == 0) {
    col[i] = a[0];
    if (i == 0) col[MD + 1] = hs_solve::rcp_f64(a[0]);
  }
  __syncthreads();
  const int jl = j0 + cnt - 1;  // my last column
  for (int k = 0; k < n; k++) {
    const double* cp = col + (k & 1) * (MD + 2);
    double* cn = col + ((k + 1) & 1) * (MD + 2);
    if (cnt > 0 && jl >= k && i >= k) {
      const double dinv = cp[MD + 1];
      const double ci = cp[i];
      const double t = ci * dinv;  // L(i, k) (i > k), or 1 (i == k)
      // column k + 1 first (the next phase's chain), then the rest
#pragma unroll
      for (int c = 0; c < SEG; c++) {
        const int j = j0 + c;
        if (c < cnt && j == k + 1 && i >= j) {
          a[c] = __builtin_fma(-t, cp[j], a[c]);
          cn[i] = a[c];
          if (i == j) cn[MD + 1] = hs_solve::rcp_f64(a[c]);
        }
      }
#pragma unroll
      for (int c = 0; c < SEG; c++) {
        const int j = j0 + c;
        if (c < cnt && j > k + 1) a[c] = __builtin_fma(-t, cp[j], a[c]);
        if (c < cnt && j == k) {  // column k is final: L, the pivot, the rhs
          if (i == n) yf[k] = a[c];
          else if (i == k) Dv[k] = a[c];
          else LT[k * hs_solve::LSTR + i] = t;
        }
      }
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(512) void k_solve(const double* Mg, const double* bg, double* xg, int n, int mode, int reps,
                                               long long* cyc) {
  __shared__ double A[MD * MD], LTs[MD * hs_solve::LSTR], Ws[LDLT_SCRATCH], y[MD];
  const int tid = threadIdx.x;
  long long best = 1LL << 62, bestw = 1LL << 62;
  int si, sj0, scnt;  // the right-looking form's segment (a constant table in a product kernel)
  rl_segment(tid, n, si, sj0, scnt);
  for (int r = 0; r < reps; r++) {
    for (int q = tid; q < n * n; q += 512) A[q] = Mg[q];
    for (int q = tid; q < MD * hs_solve::LSTR; q += 512) LTs[q] = 0.0;
    if (tid < n) y[tid] = bg[tid];
    __syncthreads();
    const long long c0 = clock64(), w0 = wall_clock64();
    if (mode == 0) {
      ldlt_solve_blocked(A, LTs, Ws, y, n, tid, nullptr, 0);
    } else {
      ldlt_rl(A, LTs, Ws, y, n, tid, si, sj0, scnt);
      hs_solve::ldlt_backward(LTs, Ws, y, n, tid, nullptr);
    }
    __syncthreads();
    const long long c1 = clock64(), w1 = wall_clock64();
    if (c1 - c0 < best) best = c1 - c0;
    if (w1 - w0 < bestw) bestw = w1 - w0;
    __syncthreads();
  }
  if (tid < n) xg[tid] = y[tid];
  if (tid == 0) {
    cyc[0] = best;
    cyc[1] = bestw;
  }
}
}  // namespace

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                         \
      return 1;                                                                            \
    }                                                                                      \
  } while (0)

int main(int argc, char** argv) {
  const int n = MD, reps = argc > 1 ? std::atoi(argv[1]) : 20;
  int khz = 0;
  CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
  std::srand(7);
  for (int trial = 0; trial < 3; trial++) {
    // SPD, scaled to a unit diagonal like S H S: B B^T + n I, then D^-1/2 . D^-1/2
    std::vector<double> B((size_t)n * n), H((size_t)n * n), b(n), x(n);
    for (auto& v : B) v = (std::rand() / (double)RAND_MAX - 0.5);
    for (int r = 0; r < n; r++)
      for (int c = 0; c < n; c++) {
        double s = r == c ? (trial + 1) * 0.05 * n : 0.0;
        for (int k = 0; k < n; k++) s += B[r * n + k] * B[c * n + k];
        H[r * n + c] = s;
      }
    for (int r = 0; r < n; r++) b[r] = std::rand() / (double)RAND_MAX - 0.5;
    std::vector<double> sq(n);
    for (int r = 0; r < n; r++) sq[r] = 1.0 / std::sqrt(H[r * n + r]);
    for (int r = 0; r < n; r++)
      for (int c = 0; c < n; c++) H[r * n + c] *= sq[r] * sq[c];
    // host reference: unpivoted LDLT in fp64
    std::vector<double> L((size_t)n * n, 0.0), D(n), z(b);
    for (int j = 0; j < n; j++) {
      double d = H[j * n + j];
      for (int k = 0; k < j; k++) d -= L[j * n + k] * L[j * n + k] * D[k];
      D[j] = d;
      L[j * n + j] = 1.0;
      for (int r = j + 1; r < n; r++) {
        double s = H[r * n + j];
        for (int k = 0; k < j; k++) s -= L[r * n + k] * L[j * n + k] * D[k];
        L[r * n + j] = s / d;
      }
    }
    for (int r = 0; r < n; r++)
      for (int k = 0; k < r; k++) z[r] -= L[r * n + k] * z[k];
    for (int r = 0; r < n; r++) z[r] /= D[r];
    for (int r = n - 1; r >= 0; r--) {
      x[r] = z[r];
      for (int k = r + 1; k < n; k++) x[r] -= L[k * n + r] * x[k];
    }
    double *dM, *db, *dx;
    long long* dc;
    CK(hipMalloc(&dM, sizeof(double) * n * n));
    CK(hipMalloc(&db, sizeof(double) * n));
    CK(hipMalloc(&dx, sizeof(double) * n));
    CK(hipMalloc(&dc, sizeof(long long) * 2));
    CK(hipMemcpy(dM, H.data(), sizeof(double) * n * n, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, b.data(), sizeof(double) * n, hipMemcpyHostToDevice));
    for (int mode = 0; mode < 2; mode++) {
      hipLaunchKernelGGL(k_solve, dim3(1), dim3(512), 0, 0, dM, db, dx, n, mode, reps, dc);
      CK(hipGetLastError());
      CK(hipDeviceSynchronize());
      std::vector<double> g(n);
      long long cy[2];
      CK(hipMemcpy(g.data(), dx, sizeof(double) * n, hipMemcpyDeviceToHost));
      CK(hipMemcpy(cy, dc, sizeof(cy), hipMemcpyDeviceToHost));
      double en = 0, xn = 0;
      for (int r = 0; r < n; r++) {
        en += (g[r] - x[r]) * (g[r] - x[r]);
        xn += x[r] * x[r];
      }
      std::printf("{\"trial\": %d, \"form\": \"%s\", \"n\": %d, \"cycles\": %lld, \"us\": %.3f, \"rel_err\": %.3e}\n",
                  trial, mode == 0 ? "panel (product)" : "right-looking, 1 barrier per column", n, cy[0],
                  cy[1] * 1e3 / (khz > 0 ? khz : 100000), std::sqrt(en / xn));
    }
    (void)hipFree(dM);
    (void)hipFree(db);
    (void)hipFree(dx);
    (void)hipFree(dc);
  }
  return 0;
}
