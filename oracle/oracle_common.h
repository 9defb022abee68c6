/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (CPU restatement of the reference path).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load liboracle*.so; the product (h-slam_amd/) never links it.
 *
 * PARITY STATUS: the reference (AUBVRL/H-SLAM) cannot be compiled here (it
 * needs Eigen3/Boost/OpenCV/DBoW3) and ships no golden vectors
 * or tests for this path.  This restatement is therefore
 * "parity unpinned" against the reference itself: it is pinned only by the
 * vendored Sophus test vectors (SE3), finite-difference Jacobian checks,
 * H symmetry / PSD / gauge-nullspace properties and zero residual at ground
 * truth on noise-free synthetic scenes (tests/test_oracle_*.py).
 *
 * Constants and primitives restated from:
 *   pattern 8            Include/GlobalTypes.h:33,181-184,225-228
 *   SCALE_*              Include/GlobalTypes.h:34-50
 *   interpolators        Include/GlobalTypes.h:355-401
 *   projectPoint         Include/DirectProjection.h:12-38
 *   AffLight             Include/GlobalTypes.h:326-352
 */
#pragma once
#include <cmath>
#include <cstdint>
#include "../include/hs_types.h"

namespace hso {

static const int PN = 8;            // patternNum
static const int CP = 4;            // CPARS
static const int kPattern[8][2] = {{0, -2}, {-1, -1}, {1, -1}, {-2, 0}, {0, 0}, {2, 0}, {-1, 1}, {0, 2}};

static const float SCALE_IDEPTH = 1.0f;
static const float SCALE_XI_ROT = 1.0f;
static const float SCALE_XI_TRANS = 0.5f;
static const float SCALE_F = 50.0f;
static const float SCALE_C = 50.0f;
static const float SCALE_A = 10.0f;
static const float SCALE_B = 1000.0f;
static const float SCALE_XI_ROT_INVERSE = 1.0f / SCALE_XI_ROT;
static const float SCALE_XI_TRANS_INVERSE = 1.0f / SCALE_XI_TRANS;
static const float SCALE_F_INVERSE = 1.0f / SCALE_F;
static const float SCALE_C_INVERSE = 1.0f / SCALE_C;
static const float SCALE_A_INVERSE = 1.0f / SCALE_A;
static const float SCALE_B_INVERSE = 1.0f / SCALE_B;

struct V3f { float x, y, z; };

// getInterpolatedElement33 (Include/GlobalTypes.h:377-388): img is AoS (I,dx,dy) per pixel.
inline V3f interp33(const float* img, float x, float y, int width) {
  int ix = (int)x, iy = (int)y;
  float dx = x - ix, dy = y - iy, dxdy = dx * dy;
  const float* bp = img + 3 * (ix + iy * width);
  const float w11 = dxdy, w01 = dy - dxdy, w10 = dx - dxdy, w00 = 1 - dx - dy + dxdy;
  const float* p11 = bp + 3 * (1 + width);
  const float* p01 = bp + 3 * width;
  const float* p10 = bp + 3;
  V3f r;
  r.x = w11 * p11[0] + w01 * p01[0] + w10 * p10[0] + w00 * bp[0];
  r.y = w11 * p11[1] + w01 * p01[1] + w10 * p10[1] + w00 * bp[1];
  r.z = w11 * p11[2] + w01 * p01[2] + w10 * p10[2] + w00 * bp[2];
  return r;
}

// getInterpolatedElement31 (Include/GlobalTypes.h:390-401)
inline float interp31(const float* img, float x, float y, int width) {
  int ix = (int)x, iy = (int)y;
  float dx = x - ix, dy = y - iy, dxdy = dx * dy;
  const float* bp = img + 3 * (ix + iy * width);
  return dxdy * bp[3 * (1 + width)] + (dy - dxdy) * bp[3 * width] + (dx - dxdy) * bp[3] +
         (1 - dx - dy + dxdy) * bp[0];
}

// getInterpolatedElement33BiLin (Include/GlobalTypes.h:355-375)
inline V3f interp33BiLin(const float* img, float x, float y, int width) {
  int ix = (int)x, iy = (int)y;
  const float* bp = img + 3 * (ix + iy * width);
  float tl = bp[0], tr = bp[3], bl = bp[3 * width], br = bp[3 * width + 3];
  float dx = x - ix, dy = y - iy;
  float topInt = dx * tr + (1 - dx) * tl;
  float botInt = dx * br + (1 - dx) * bl;
  float leftInt = dy * bl + (1 - dy) * tl;
  float rightInt = dy * br + (1 - dy) * tr;
  V3f r;
  r.x = dx * rightInt + (1 - dx) * leftInt;
  r.y = rightInt - leftInt;
  r.z = botInt - topInt;
  return r;
}

// AffLight::fromToVecExposure (Include/GlobalTypes.h:334-346)
inline void fromToVecExposure(float exposureF, float exposureT, double g2Fa, double g2Fb, double g2Ta,
                              double g2Tb, double out[2]) {
  if (exposureF == 0 || exposureT == 0) exposureT = exposureF = 1;
  double a = std::exp(g2Ta - g2Fa) * exposureT / exposureF;
  double b = g2Tb - a * g2Fb;
  out[0] = a; out[1] = b;
}

// 3x3 float helpers, Eigen-like evaluation order (sum over k in order)
inline void mm3f(const float A[9], const float B[9], float C[9]) {
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++)
      C[r * 3 + c] = A[r * 3 + 0] * B[0 * 3 + c] + A[r * 3 + 1] * B[1 * 3 + c] + A[r * 3 + 2] * B[2 * 3 + c];
}
inline void mv3f(const float A[9], const float v[3], float o[3]) {
  for (int r = 0; r < 3; r++) o[r] = A[r * 3 + 0] * v[0] + A[r * 3 + 1] * v[1] + A[r * 3 + 2] * v[2];
}
// Eigen compute_inverse_size3 (cofactor / determinant) in float
inline void inv3f(const float m[9], float r[9]) {
  auto M = [&](int i, int j) { return m[i * 3 + j]; };
  auto cof = [&](int i, int j) {
    int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
    return M(i1, j1) * M(i2, j2) - M(i1, j2) * M(i2, j1);
  };
  float c00 = cof(0, 0), c10 = cof(1, 0), c20 = cof(2, 0);
  float det = c00 * M(0, 0) + c10 * M(1, 0) + c20 * M(2, 0);
  float invdet = 1.0f / det;
  r[0] = c00 * invdet; r[1] = c10 * invdet; r[2] = c20 * invdet;
  r[3] = cof(0, 1) * invdet; r[4] = cof(1, 1) * invdet; r[5] = cof(2, 1) * invdet;
  r[6] = cof(0, 2) * invdet; r[7] = cof(1, 2) * invdet; r[8] = cof(2, 2) * invdet;
}

inline void params_default(hs_params* p) {
  p->huberTH = 9;
  p->outlierTHSumComponent = 50 * 50;
  p->frameEnergyTHN = 0.7f;
  p->frameEnergyTHFacMedian = 1.5;
  p->frameEnergyTHConstWeight = 0.5;
  p->overallEnergyTHWeight = 1;
  p->idepthFixPrior = 50 * 50;
  p->initialCalibHessian = 5e9;
  p->affineOptModeA = 1e12;
  p->affineOptModeB = 1e8;
  p->initialRotPrior = 1e11;
  p->initialTransPrior = 1e10;
  p->initialAffAPrior = 1e14;
  p->initialAffBPrior = 1e14;
  p->solverModeDelta = 0.00001;
  p->thOptIterations = 1.2;
  p->coarseCutoffTH = 20;
  p->minOptIterations = 1;
  p->pad = 0;
  p->outlierTH = 12 * 12;
  p->maxPixSearch = 0.027f;
  p->trace_slackInterval = 1.5f;
  p->trace_stepsize = 1.0f;
  p->trace_minImprovementFactor = 2;
  p->trace_GNThreshold = 0.1f;
  p->trace_extraSlackOnTH = 1.2f;
  p->minTraceTestRadius = 2;
  p->trace_GNIterations = 3;
  p->idepthFixPriorMargFac = 600 * 600;
  p->margWeightFac = 0.5f * 0.5f;
  p->desiredPointDensity = 2000;
  p->minTraceQuality = 3;
  p->minIdepthH_act = 100;
  p->GNItsOnPointActivation = 3;
  p->minGradHistCut = 0.5f;
  p->minGradHistAdd = 7;
  p->gradDownweightPerLevel = 0.75f;
  p->selectDirectionDistribution = 1;
}

}  // namespace hso
