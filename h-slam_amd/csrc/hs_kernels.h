// hs_kernels.h — kernel argument blocks and launch declarations (host <-> device).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hs_types.h"
#include "hs_layout.h"

struct HsLinArgs {
  const float4* img[HS_MAXF];  // level-0 texels per window frame
  HsCalib calib;
  HsLinParams lp;
  int nF;
  int write_center;
  const HsPrecalc* pre;        // [nF*nF] host*nF + target
  const float* frameTH;        // [nF]
  // points
  const float* u;
  const float* v;
  const float* idepth;
  const float* idepth_zero;
  const float* priorF;
  const float* color;          // [n][8]
  const float* weight;         // [n][8]
  const int* res_of_slot;      // [n][8]
  const int8_t* res_order;     // [n][8]
  const int* chunk_begin;      // [n_chunks+1]
  const int* chunk_host;       // [n_chunks]
  // residual state (in/out)
  uint8_t* r_state;
  uint8_t* r_active;
  float* r_energy;
  float* r_newEnergy;
  float* r_ewo;
  float* r_JpJdF;              // [m][8]
  float* r_center;             // [m][3]
  // point outputs
  float* p_HdiF;
  float* p_bdSumF;
  float* p_Hcd;                // [n][4]
  uint8_t* p_ngood;
  // accumulators
  HsWavePartial* partials;
  float* newest_cand;          // energies of residuals into the newest frame (setNewFrameEnergyTH)
  int* newest_cnt;
};

struct HsReduceArgs {
  const HsWavePartial* partials;
  const int* host_chunk_begin;  // [nF+1]
  int n_chunks;
  HsHostSlab* slabs;            // [nF]
  double* energy;
};

struct HsStitchArgs {
  int nF;
  const HsHostSlab* slabs;
  const double* adHost;         // [nF*nF][64]  index h + nF*t
  const double* adTarget;
  double* HA;                   // [n*n] zeroed
  double* bA;
  double* HSC;
  double* bSC;
};

struct HsResubArgs {
  int n, nF, apply;
  float cstep[4];
  const int* host;
  const float* xAd;             // [nF*nF][8] index h*nF + t
  const float* bdSumF;
  const float* HdiF;
  const float* Hcd;
  const uint8_t* ngood;
  const int* res_of_slot;
  const int8_t* res_order;
  const uint8_t* r_active;
  const float* JpJdF;
  float* idepth;
  float* idepth_zero;
  float* step;
  double* stat_partial;         // [blocks][2]
};

struct HsEnergyThArgs {
  const float* cand;            // [nranks][stride]
  const int* cnt;               // [nranks]
  int nranks;
  int stride;
  float* frameTH;
  int newest;
  float frameEnergyTHN, facMedian, constWeight, overallWeight;
};

__global__ void hs_k_linearize(HsLinArgs a);
__global__ void hs_k_reduce(HsReduceArgs a);
__global__ void hs_k_stitch(HsStitchArgs a);
__global__ void hs_k_resub(HsResubArgs a);
__global__ void hs_k_energy_th(HsEnergyThArgs a);
__global__ void hs_k_apply_step(int n, const float* step, float* idepth, float* idepth_zero);
