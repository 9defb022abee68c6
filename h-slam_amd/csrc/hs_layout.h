// hs_layout.h — device-resident data layout of the BA window (shared by the
// HIP kernels and the C++ host layer).  Everything is structure-of-arrays in
// HBM; the reference's shared_ptr graph never exists on the
// device.
//
//   images   : per frame, per level, float4 (I, dI/dx, dI/dy, 0) row-major
//              (Frame::DirPyr, Include/Frame.h:39; 16-B texels so a bilinear
//              tap is one dwordx4 load)
//   points   : u, v, idepth, idepth_zero, priorF, host   [n]
//              color, weight                           [n][8]
//              res_of_slot                             [n][8]  residual index per
//                                                      target frame (-1 = none)
//              res_order                               [n][8]  target frames in the
//                                                      point's residual-list order
//   residuals: state / energy / new energy / energy-with-outlier / active,
//              JpJdF [m][8], centre projection [m][3]
//   precalc  : HsPrecalc [nF*nF] indexed host*nF + target (Frame::targetPrecalc)
//   partials : one HsWavePartial per BA wave (per-host chunk of points)
#pragma once
#include <stdint.h>

#define HS_PN 8
#define HS_MAXF 8
#define HS_TOP_N 91   // 55 (10x10 upper) + 30 (10 x {a,b,r}) + 6 (3x3 upper)

// FrameFramePrecalc restricted to what the linearize kernel reads
// (Include/OptimizationClasses.h:55-86)
struct HsPrecalc {
  float KRKi[9];   // PRE_KRKiTll
  float Kt[3];     // PRE_KtTll
  float R0[9];     // PRE_RTll_0
  float t0[3];     // PRE_tTll_0
  float aff[2];    // PRE_aff_mode
  float b0;        // PRE_b0_mode
  float pad;
};

// CalibData scaled values used on the device (Include/CalibData.h:93-100)
struct HsCalib {
  float fxl, fyl, cxl, cyl, fxli, fyli;
  int W, H;
};

// settings read inside the linearize kernel
struct HsLinParams {
  float huberTH;
  float outlierTHSumComponent;
  float affineOptModeA;
  float affineOptModeB;
};

// one BA wave's accumulators (fp32), host frame = chunk host.
// layout of top[t][e]: e < 55 : Data (upper-tri of [calib4|xi6]),
//                      e < 85 : TopRight[3*r + {a,b,r}], e < 91 : BotRight
struct HsWavePartial {
  float top[HS_MAXF][96];              // [target][entry] (91 used)
  float D[HS_MAXF][HS_MAXF][64];       // [t1][t2][8x8]   (accD host fixed)
  float E[HS_MAXF][32];                // [t1][8x4]
  float EB[HS_MAXF][8];                // [t1][8]
  float Hcc[16];
  float bc[4];
  int cnt[HS_MAXF];                    // residuals accumulated per target (AccumulatorApprox::num)
  int host;
  int pad[3];
  double energy;                       // sum of linearize() energies of the chunk's residuals
  double pad2;
};

#define HS_WP_FLOATS (HS_MAXF * 96 + HS_MAXF * HS_MAXF * 64 + HS_MAXF * 32 + HS_MAXF * 8 + 16 + 4)

// reduced per-host slab (fp64)
struct HsHostSlab {
  double top[HS_MAXF][96];
  double D[HS_MAXF][HS_MAXF][64];
  double E[HS_MAXF][32];
  double EB[HS_MAXF][8];
  double Hcc[16];
  double bc[4];
  int cnt[HS_MAXF];
};
