// hs_se3_dev.h — device-only SE(3) forms of a GN / LM step (shared by the BA solve's doStep and the tracker's LM
// step): Sophus' exp and product with the transcendental / IEEE-division chains replaced by series and reciprocal
// square roots.  They differ from hs_se3.h (Sophus) by rounding only (tests/test_gpu_se3.py pins both to the Sophus
// test sets).
#pragma once
#include <hip/hip_runtime.h>

#include "hs_se3.h"

// 1 / sqrt(x) for a quaternion norm near 1: v_rsq_f64 refined by two Newton steps (no IEEE square root and division
// on the doStep chain); differs from 1.0 / sqrt(x) by rounding only
__device__ __forceinline__ double rsqrt_step(double x) {
  double r = __builtin_amdgcn_rsq(x);
  r = r * __builtin_fma(-0.5 * x, r * r, 1.5);
  r = r * __builtin_fma(-0.5 * x, r * r, 1.5);
  return r;
}

// Sophus SE3::exp (hs_se3.h) for a GN step: for theta^2 < 1e-2 the so3 / V coefficients sin(x/2)/x, cos(x/2),
// (1 - cos x)/x^2 and (x - sin x)/x^3 come from their Taylor series in u = x^2 (6 terms: truncation < 1e-20
// relative; no sqrt, trig or division on the chain); the quaternion is normalized with one reciprocal square
// root.  Larger tangents take the reference formulas.  Differs from Sophus by rounding only.
// the two halves of the series form (u = |w|^2 < 1e-2), so a caller can run them on different waves: the unit
// quaternion, and the translation V a
// An fp64 constant materialized where it is used (two v_mov_b32 the compiler may not hoist): kernels with long
// loops around the step (the tracker's LM loop) otherwise keep the series coefficients live across the loop in
// registers, and at 256 VGPRs spill them to scratch.
template <unsigned long long B>
__device__ __forceinline__ double kd() {
  unsigned int lo, hi;
  asm volatile("v_mov_b32 %0, %1" : "=v"(lo) : "i"((unsigned int)(B & 0xffffffffull)));
  asm volatile("v_mov_b32 %0, %1" : "=v"(hi) : "i"((unsigned int)(B >> 32)));
  return __hiloint2double((int)hi, (int)lo);
}
#define HS_KD(x) kd<__builtin_bit_cast(unsigned long long, (double)(x))>()

__device__ __forceinline__ double se3_step_poly(double u, double c0, double c1, double c2, double c3, double c4,
                                                double c5) {
  return __builtin_fma(__builtin_fma(__builtin_fma(__builtin_fma(__builtin_fma(c5, u, c4), u, c3), u, c2), u, c1), u,
                       c0);
}
__device__ __forceinline__ hs::Quat se3_exp_step_q(const double a[6], double u) {
  const double imag = se3_step_poly(u, 1.0 / 2, HS_KD(-1.0 / 48), HS_KD(1.0 / 3840), HS_KD(-1.0 / 645120),
                                    HS_KD(1.0 / 185794560), HS_KD(-1.0 / 81749606400.0));
  const double real = se3_step_poly(u, 1.0, HS_KD(-1.0 / 8), HS_KD(1.0 / 384), HS_KD(-1.0 / 46080),
                                    HS_KD(1.0 / 10321920), HS_KD(-1.0 / 3715891200.0));
  const double qx = imag * a[3], qy = imag * a[4], qz = imag * a[5];
  const double inv = rsqrt_step(qx * qx + qy * qy + qz * qz + real * real);
  return hs::Quat{qx * inv, qy * inv, qz * inv, real * inv};
}
__device__ __forceinline__ void se3_exp_step_t(const double a[6], double u, double t[3]) {
  const double c1 = se3_step_poly(u, 1.0 / 2, HS_KD(-1.0 / 24), HS_KD(1.0 / 720), HS_KD(-1.0 / 40320),
                                  HS_KD(1.0 / 3628800), HS_KD(-1.0 / 479001600));
  const double c2 = se3_step_poly(u, HS_KD(1.0 / 6), HS_KD(-1.0 / 120), HS_KD(1.0 / 5040), HS_KD(-1.0 / 362880),
                                  HS_KD(1.0 / 39916800), HS_KD(-1.0 / 6227020800.0));
  double O[9], O2[9], V[9];
  hs::SE3::hat3(a + 3, O);
  hs::SE3::mm3(O, O, O2);
#pragma unroll
  for (int i = 0; i < 9; i++) V[i] = ((i % 4 == 0) ? 1.0 : 0.0) + c1 * O[i] + c2 * O2[i];
#pragma unroll
  for (int i = 0; i < 3; i++) t[i] = V[i * 3 + 0] * a[0] + V[i * 3 + 1] * a[1] + V[i * 3 + 2] * a[2];
}
__device__ __forceinline__ double se3_step_u(const double a[6]) { return a[3] * a[3] + a[4] * a[4] + a[5] * a[5]; }

__device__ __forceinline__ hs::SE3 se3_exp_step(const double a[6]) {
  const double u = se3_step_u(a);
  if (!(u < 1e-2)) return hs::SE3::exp(a);
  hs::SE3 r;
  r.q = se3_exp_step_q(a, u);
  se3_exp_step_t(a, u, r.t);
  return r;
}

// SE3 product (Sophus fastMultiply: quaternion product + normalize), normalized with one reciprocal square root;
// se3_mul_step_q is its rotation half
__device__ __forceinline__ hs::Quat se3_mul_step_q(const hs::Quat& a, const hs::Quat& b) {
  const hs::Quat q = hs::qmul(a, b);
  const double inv = rsqrt_step(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
  return hs::Quat{q.x * inv, q.y * inv, q.z * inv, q.w * inv};
}
__device__ __forceinline__ hs::SE3 se3_mul_step(const hs::SE3& A, const hs::SE3& B) {
  hs::SE3 r;
  double rt[3];
  hs::qrot(A.q, B.t, rt);
  r.t[0] = A.t[0] + rt[0];
  r.t[1] = A.t[1] + rt[1];
  r.t[2] = A.t[2] + rt[2];
  r.q = se3_mul_step_q(A.q, B.q);
  return r;
}

