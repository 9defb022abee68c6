// hs_refine_kernels.h — argument block of the DirectRefinement kernel (hs_refine_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hs_se3.h"

#define HS_REF_MAXLOG 1001  // Refine's level-0 iteration cap (maxIterations[0] = 1000) + 1
#define HS_REF_LOGW 8       // per LM iteration: eTotalOld, eTotalNew, accept, lambda, |inc|, resNew0, resNew1, regNew
#define HS_REF_PPB 32       // points per block (8 lanes per point, one lane per pattern pixel)
#define HS_REF_NRED 93      // acc9 (45), acc9SC (45), E, calcEC old / new

// per-point state (struct Pnt, Include/Initializer.h:159-190) as structure-of-arrays in HBM;
// JbBuffer / JbBuffer_new are two [10][n] planes, swapped by applyStep
struct HsRefPoints {
  const float* u;
  const float* v;
  const float* invz;       // 1 / Pts3D.z of triangulated points, 1 otherwise
  const uint8_t* tri;      // Triangulated[i]
  float* idepth;
  float* idepth_new;
  float* iR;
  float* energy;           // [2][n]
  float* energy_new;       // [2][n]
  float* lastH;
  float* lastH_new;
  float* maxstep;
  uint8_t* good;
  uint8_t* good_new;
  float* jb[2];            // [10][n] each
};

// the constants of one calcResAndGS pass at (refToNew, aff)
struct HsRefPass {
  float RKi[9], t[3], r2a, r2b, alphaOpt, alphaEnergy, tlog[3];
};

// device-resident LM state of Refine, carried from one step kernel to the next (the last block of a step writes it)
struct HsRefCtl {
  HsRefPass pc;                 // constants of the next pass
  float inc[8], lambda;         // the next doStep
  int apply_prev, optreg_prev;  // the previous pass was accepted: applyStep (+ optReg) in the next prologue
  int snapped, jb_sel, done, iteration, fails;
  double T[7], Tn[7], aff[2], affn[2];
  float Hm[64], bm[8], Hs[64], bs[8], resOld[3];
  // outputs of a single calcResAndGS (hs_refiner_calc_res)
  float H[64], b[8], Hsc[64], bsc[8], res[3];
};

enum { HS_REF_CALC = 0, HS_REF_INIT = 1, HS_REF_ITER = 2, HS_REF_FINAL = 3 };

struct HsRefArgs {
  HsRefPoints p;
  int n, W, H, mode, nblocks;
  float fx, fy, cx, cy;
  double Ki[9];
  const float4* img1;      // FirstFrame DirPyr[0] (I, dx, dy, 0)
  const float4* img2;      // SecondFrame DirPyr[0]
  float huberTH, outlierTH;
  int jb_sel0;             // CALC / INIT: the JbBuffer plane at entry
  HsRefPass pc0;           // CALC / INIT: the pass constants at the caller's (T, aff), computed on the host
  double T0[7], aff0[2];   // INIT: the starting pose
  HsRefCtl* ctl;
  double* part;            // [nblocks][HS_REF_NRED] block partial sums
  int* ticket;
  float* log;              // [HS_REF_MAXLOG][HS_REF_LOGW]
  long long* trace;        // [nblocks][16] wall-clock stamps (HS_REF_TRACE=1), nullable
};

__global__ void hs_k_refine_step(HsRefArgs a);

constexpr float hs_ref_alphaK = 2.5f * 2.5f, hs_ref_alphaW = 150 * 150, hs_ref_coupling = 1;

// the pass constants at (T, aff) (Src/Initializer.cpp:1930-1940, 2086-2101, 2146): RKi = (R * Ki).cast<float>(),
// t, exp(a), b, the alpha regularizer terms (EAlpha never receives an update in the reference, so
// alphaEnergy = alphaW * |t|^2 * npts) and log(T).head<3>()
inline __host__ __device__ void hs_ref_pass_consts(const double T7[7], const double aff[2], const double Ki[9], int n,
                                                   HsRefPass* pc) {
  const hs::SE3 T = hs::SE3::fromData(T7);
  double R[9];
  T.rotationMatrix(R);
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++)
      pc->RKi[r * 3 + c] = (float)(R[r * 3 + 0] * Ki[0 * 3 + c] + R[r * 3 + 1] * Ki[1 * 3 + c] + R[r * 3 + 2] * Ki[2 * 3 + c]);
  for (int q = 0; q < 3; q++) pc->t[q] = (float)T.t[q];
  pc->r2a = (float)exp(aff[0]);
  pc->r2b = (float)aff[1];
  const double tsq = T.t[0] * T.t[0] + T.t[1] * T.t[1] + T.t[2] * T.t[2];
  const float EAlphaA = 0.f;
  float alphaEnergy = (float)(hs_ref_alphaW * (EAlphaA + tsq * n));
  float alphaOpt;
  if (alphaEnergy > hs_ref_alphaK * n) {
    alphaOpt = 0;
    alphaEnergy = hs_ref_alphaK * n;
  } else {
    alphaOpt = hs_ref_alphaW;
  }
  pc->alphaOpt = alphaOpt;
  pc->alphaEnergy = alphaEnergy;
  double lg[6];
  T.log(lg);
  for (int q = 0; q < 3; q++) pc->tlog[q] = (float)lg[q];
}
