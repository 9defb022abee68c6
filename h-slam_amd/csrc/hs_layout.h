// hs_layout.h — device-resident data layout of the BA window (shared by the
// HIP kernels and the C++ host layer).  Everything is structure-of-arrays in
// HBM; the reference's shared_ptr graph never exists on the
// device.
//
//   images    : per frame float4 (I, dI/dx, dI/dy, 0) row-major (Frame::DirPyr[0], Include/Frame.h:39;
//               16-B texels: a bilinear tap is one dwordx4 load)
//   points    : u, v, idepth, idepth_zero, priorF, host                       [n]
//               color, weight                                                [n][8]
//               res_of_slot  residual index per target frame slot (-1 none)  [n][8]
//               res_order    target slots in the point's residual-list order [n][8]
//   per point outputs of a linearization (slot layout, read by the next iteration's fused point step and
//               the granular resubstitute): actmask (bit t = residual into frame t is active), HdiF, bdSumF,
//               Hcd[4], JpJdF [n][8 slots][8], step
//   block partials of the fused linearize (hs_k_lin): [block][entry][64 lanes] fp32 accumulators + fp64
//               energies; per-host sums [host][entry][64] fp64; per-host system slots (upper triangles)
//   residuals : state / energy / new energy / energy-with-outlier / active, centre projection [m][3]
//   precalc   : HsPrecalc [nF*nF] indexed host*nF + target (Frame::targetPrecalc)
#pragma once
#include <stdint.h>

#define HS_PN 8
#define HS_MAXF 8
#define HS_MAXDIM (4 + 8 * HS_MAXF)
#define HS_TOP_N 91    // 55 (10x10 upper) + 30 (10 x {a,b,r}) + 6 (3x3 upper)

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
