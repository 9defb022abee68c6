// hs_trace_kernels.h — argument blocks of the ImmaturePoint kernels (hs_trace_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hs_trace.h"

#define HS_TRC_MAXHOST 64

// ImmaturePoint ctor for points [first, first + n)
struct HsImmCtorArgs {
  int n, first, W, H;
  const float4* const* host_img;  // device array of [HS_TRC_MAXHOST] level-0 images
  const int* host;
  const float* u;
  const float* v;
  float outlierTHSumComponent, outlierTH, overallEnergyTHWeight;
  float* color;     // [n][8]
  float* weights;   // [n][8]
  float* gradH;     // [n][4]
  float* energyTH;
  float* quality;
  float* idepth_min;
  float* idepth_max;
  uint8_t* status;
  float* uv;        // [n][2]
  float* interval;
};

struct HsTraceArgs {
  int n, W, H;
  const float4* img;            // the new frame, level 0
  const hs_trace_host* hosts;   // per host slot
  const int* host;
  const float* u;
  const float* v;
  const float* color;
  const float* weights;
  const float* gradH;
  const float* energyTH;
  float* quality;
  float* idepth_min;
  float* idepth_max;
  uint8_t* status;
  float* uv;
  float* interval;
  int* steps;                   // [n] discrete-search steps evaluated (0 = no search)
  float huberTH, maxPixSearch, slackInterval, stepsize, minImprovementFactor, GNThreshold, extraSlackOnTH;
  int minTraceTestRadius, GNIterations;
};

__global__ void hs_k_imm_ctor(HsImmCtorArgs a);
__global__ void hs_k_trace_on(HsTraceArgs a);
__global__ void hs_k_trace_count(int n, const uint8_t* status, const int* steps, int* out);
