// micro-benchmark (gfx950): latency of the GN step's frame update + FrameFramePrecalc::set chain (hs_k_solve's
// HS_APPLY section) on one wave, cold (first call) and warm (repeated), with the series SE3::exp and with Sophus'.
// build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I../../h-slam_amd/csrc -o step step.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#include "hs_host_math.h"

__device__ __forceinline__ hs::SE3 exp_series(const double a[6]) {
  const double w0 = a[3], w1 = a[4], w2 = a[5];
  const double u = w0 * w0 + w1 * w1 + w2 * w2;
  if (!(u < 1e-2)) return hs::SE3::exp(a);
  auto poly = [u](double c0, double c1, double c2, double c3, double c4, double c5) {
    return __builtin_fma(__builtin_fma(__builtin_fma(__builtin_fma(__builtin_fma(c5, u, c4), u, c3), u, c2), u, c1), u,
                         c0);
  };
  const double imag = poly(1.0 / 2, -1.0 / 48, 1.0 / 3840, -1.0 / 645120, 1.0 / 185794560, -1.0 / 81749606400.0);
  const double real = poly(1.0, -1.0 / 8, 1.0 / 384, -1.0 / 46080, 1.0 / 10321920, -1.0 / 3715891200.0);
  const double c1 = poly(1.0 / 2, -1.0 / 24, 1.0 / 720, -1.0 / 40320, 1.0 / 3628800, -1.0 / 479001600);
  const double c2 = poly(1.0 / 6, -1.0 / 120, 1.0 / 5040, -1.0 / 362880, 1.0 / 39916800, -1.0 / 6227020800.0);
  hs::SE3 r;
  const double qx = imag * w0, qy = imag * w1, qz = imag * w2;
  const double inv = 1.0 / sqrt(qx * qx + qy * qy + qz * qz + real * real);
  r.q = hs::Quat{qx * inv, qy * inv, qz * inv, real * inv};
  double O[9], O2[9], V[9];
  hs::SE3::hat3(a + 3, O);
  hs::SE3::mm3(O, O, O2);
  for (int i = 0; i < 9; i++) V[i] = ((i % 4 == 0) ? 1.0 : 0.0) + c1 * O[i] + c2 * O2[i];
  for (int i = 0; i < 3; i++) r.t[i] = V[i * 3 + 0] * a[0] + V[i * 3 + 1] * a[1] + V[i * 3 + 2] * a[2];
  return r;
}

template <int MODE>
__global__ void k(const double* in, double* out, long long* cyc) {
  const int l = threadIdx.x;
  double acc = 0.0;
  long long t[4];
  for (int rep = 0; rep < 2; rep++) {
    t[2 * rep] = clock64();
    double a[6];
    for (int i = 0; i < 6; i++) a[i] = in[(l * 6 + i + rep) & 255] * 1e-3;
    hs::SE3 E = MODE == 0 ? exp_series(a) : hs::SE3::exp(a);
    hs::SE3 ev = hs::SE3::fromData(in + 8);
    hs::SE3 PW = E * ev;
    hs::SE3 PC = PW.inverse();
    hs::SE3 l2l = PW * PC;
    double R[9];
    l2l.rotationMatrix(R);
    acc += R[0] + R[4] + l2l.t[2];
    if (MODE == 2) {  // + precalc's exp of the affine difference
      acc += exp(a[0] - a[1]);
    }
    t[2 * rep + 1] = clock64() + (long long)(acc * 0.0);
  }
  out[l] = acc;
  if (l == 0) {
    cyc[0] = t[1] - t[0];
    cyc[1] = t[3] - t[2];
  }
}

int main() {
  double *in, *out;
  long long* c;
  (void)hipMalloc(&in, 256 * 8);
  (void)hipMalloc(&out, 1024 * 8);
  (void)hipMalloc(&c, 16);
  double h[256];
  for (int i = 0; i < 256; i++) h[i] = 0.1 + 0.01 * (i % 17);
  h[8] = 0.1; h[9] = 0.2; h[10] = 0.3; h[11] = 0.9; h[12] = 1; h[13] = 2; h[14] = 3;
  (void)hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  const char* names[] = {"series exp + mul + inverse + mul + R", "Sophus exp + mul + inverse + mul + R",
                         "Sophus chain + fp64 exp"};
  for (int mode = 0; mode < 3; mode++) {
    long long cy[2] = {0, 0};
    for (int rep = 0; rep < 3; rep++) {
      if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(1), dim3(64), 0, 0, in, out, c);
      if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(1), dim3(64), 0, 0, in, out, c);
      if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(1), dim3(64), 0, 0, in, out, c);
      (void)hipDeviceSynchronize();
      (void)hipMemcpy(cy, c, 16, hipMemcpyDeviceToHost);
    }
    printf("%-40s first %6lld  second %6lld cycles\n", names[mode], cy[0], cy[1]);
  }
  return 0;
}
