// hs_refine_kernels.h — argument block of the DirectRefinement kernel (hs_refine_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define HS_REF_MAXLOG 1001  // Refine's level-0 iteration cap (maxIterations[0] = 1000) + 1
#define HS_REF_LOGW 8       // per LM iteration: eTotalOld, eTotalNew, accept, lambda, |inc|, resNew0, resNew1, regNew

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

struct HsRefOut {
  double T[7];
  double aff[2];
  int iterations, snapped, jb_sel;
  float res[3];            // resOld at exit (single pass: this pass's res)
  float H[64], b[8], Hsc[64], bsc[8];
};

struct HsRefArgs {
  HsRefPoints p;
  int n, W, H;
  float fx, fy, cx, cy;
  double Ki[9];
  const float4* img1;      // FirstFrame DirPyr[0] (I, dx, dy, 0)
  const float4* img2;      // SecondFrame DirPyr[0]
  double T_in[7];
  double aff_in[2];
  float huberTH, outlierTH;
  int single_pass;         // hs_refiner_calc_res: resetPoints + one calcResAndGS
  int jb_sel;              // which plane is JbBuffer at entry
  HsRefOut* out;
  float* log;              // [HS_REF_MAXLOG][HS_REF_LOGW]
};

__global__ void hs_k_refine(HsRefArgs a);
