// micro-benchmark (gfx950): cycles per LDLT panel phase of hs_k_solve's panel wave, by component.
// One 64-thread workgroup runs 16 phases of {LDS loads, rank-4 update, diagonal-block gather, uniform 4x4 LDLT,
// row reduction, LDS stores, barrier}; modes drop one component at a time.
// build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o panel panel.hip
#include <hip/hip_runtime.h>
#include <cfloat>
#include <cstdio>

__device__ __forceinline__ double rl(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), lane);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double rcp_f64(double d) {
  double r = __builtin_amdgcn_rcp(d);
  const double e = __builtin_fma(-d, r, 1.0);
  r = __builtin_fma(r, e, r);
  return fabs(d) > DBL_MIN ? r : 0.0;
}

template <int MODE>
__global__ void k(double* out, long long* cyc, int nph) {
  constexpr int MD = 68;
  __shared__ double PB[4 * MD], LW[4 * MD], LS[4 * MD], Y[MD], D[MD], LT[MD * 69];
  const int l = threadIdx.x;
  for (int i = l; i < 4 * MD; i += 64) {
    PB[i] = 1.0 + 0.01 * i;
    LW[i] = 0.001 * (i % 7);
    LS[i] = 0.002 * (i % 5);
  }
  for (int i = l; i < MD; i += 64) Y[i] = 0.5 + i;
  __syncthreads();
  double acc = 0.0;
  long long t0 = clock64();
  for (int k = 0; k < nph; k++) {
    const int K0 = 4 * (k & 7) + 4, r = min(K0 + l, MD - 1);
    double a4[4], lwk[4], lsd[4][4], yr;
    if (MODE != 2) {
#pragma unroll
      for (int j = 0; j < 4; j++) {
        a4[j] = PB[j * MD + r];
        lwk[j] = LW[j * MD + r];
#pragma unroll
        for (int c = 0; c < 4; c++) lsd[c][j] = LS[j * MD + K0 + c];
      }
      yr = Y[r];
    } else {
#pragma unroll
      for (int j = 0; j < 4; j++) {
        a4[j] = 1.0 + l + j + acc;
        lwk[j] = 0.001 * j;
#pragma unroll
        for (int c = 0; c < 4; c++) lsd[c][j] = 0.002 * (c + j);
      }
      yr = 0.5 + l;
    }
#pragma unroll
    for (int j = 0; j < 4; j++)
#pragma unroll
      for (int c = 0; c < 4; c++) a4[c] = __builtin_fma(-lwk[j], lsd[c][j], a4[c]);
    double A[4][4], Yv[4];
    if (MODE == 4) {  // gather through LDS
      if (l < 4) {
#pragma unroll
        for (int c = 0; c < 4; c++) D[l * 4 + c] = a4[c];
        D[16 + l] = yr;
      }
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int i = 0; i < 4; i++) {
#pragma unroll
        for (int j = 0; j <= i; j++) A[i][j] = D[i * 4 + j];
        Yv[i] = D[16 + i];
      }
    } else if (MODE != 1) {
#pragma unroll
      for (int i = 0; i < 4; i++) {
#pragma unroll
        for (int j = 0; j <= i; j++) A[i][j] = rl(a4[j], i);
        Yv[i] = rl(yr, i);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; i++) {
#pragma unroll
        for (int j = 0; j <= i; j++) A[i][j] = 1.0 + i + j + k;
        Yv[i] = 1.0 + i;
      }
    }
    double rr[4], q[4][4], yd[4];
    {
      double B[4][4];
#pragma unroll
      for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j <= i; j++) B[i][j] = A[i][j];
      double y[4] = {Yv[0], Yv[1], Yv[2], Yv[3]};
#pragma unroll
      for (int j = 0; j < 4; j++) {
        rr[j] = MODE == 5 ? 1.0 / (B[j][j] + 3.0) : rcp_f64(B[j][j]);
        yd[j] = y[j];
#pragma unroll
        for (int i = j + 1; i < 4; i++) q[i][j] = B[i][j];
#pragma unroll
        for (int i = j + 1; i < 4; i++) {
          const double lv = B[i][j] * rr[j];
#pragma unroll
          for (int jp = j + 1; jp <= i; jp++) B[i][jp] = __builtin_fma(-lv, B[jp][j], B[i][jp]);
          y[i] = __builtin_fma(-lv, y[j], y[i]);
        }
      }
    }
    double pr[4] = {a4[0], a4[1], a4[2], a4[3]}, lw[4], ls[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      lw[j] = pr[j];
      ls[j] = pr[j] * rr[j];
#pragma unroll
      for (int jp = j + 1; jp < 4; jp++) pr[jp] = __builtin_fma(-ls[j], q[jp][j], pr[jp]);
      yr = __builtin_fma(-ls[j], yd[j], yr);
    }
    if (MODE != 3) {
#pragma unroll
      for (int j = 0; j < 4; j++) {
        LW[j * MD + r] = lw[j];
        LS[j * MD + r] = ls[j];
        LT[(K0 + j) * 69 + r] = l > j ? ls[j] : 0.0;
      }
      if (l == 0)
#pragma unroll
        for (int j = 0; j < 4; j++) D[K0 + j] = yd[j];
      Y[r] = yr;
    } else {
      acc += lw[0] + lw[1] + lw[2] + lw[3] + ls[0] + ls[1] + ls[2] + ls[3] + yr + yd[0] + yd[3];
    }
    __syncthreads();
  }
  long long t1 = clock64();
  out[l] = acc + LW[l] + D[l & 7];
  if (l == 0) cyc[0] = t1 - t0;
}

int main() {
  double* d;
  long long* c;
  (void)hipMalloc(&d, 1024 * 8);
  (void)hipMalloc(&c, 8);
  const char* names[] = {"full phase", "no gather / factor inputs constant", "no LDS loads", "no LDS stores",
                         "gather through LDS", "IEEE 1/x pivots"};
  for (int mode = 0; mode < 6; mode++) {
    long long cy = 0;
    for (int rep = 0; rep < 3; rep++) {
      switch (mode) {
        case 0: hipLaunchKernelGGL(k<0>, dim3(1), dim3(64), 0, 0, d, c, 160); break;
        case 1: hipLaunchKernelGGL(k<1>, dim3(1), dim3(64), 0, 0, d, c, 160); break;
        case 2: hipLaunchKernelGGL(k<2>, dim3(1), dim3(64), 0, 0, d, c, 160); break;
        case 3: hipLaunchKernelGGL(k<3>, dim3(1), dim3(64), 0, 0, d, c, 160); break;
        case 4: hipLaunchKernelGGL(k<4>, dim3(1), dim3(64), 0, 0, d, c, 160); break;
        case 5: hipLaunchKernelGGL(k<5>, dim3(1), dim3(64), 0, 0, d, c, 160); break;
      }
      (void)hipDeviceSynchronize();
      (void)hipMemcpy(&cy, c, 8, hipMemcpyDeviceToHost);
    }
    printf("%-40s %7.1f cycles/phase\n", names[mode], (double)cy / 160);
  }
  return 0;
}
