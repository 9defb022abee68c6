// hs_win_kernels.h — argument blocks of the incremental-window kernels (hs_win_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hs_types.h"
#include "hs_layout.h"

// slot codes of a commit's residual table [n][8]
constexpr unsigned HS_WIN_KEEP = 0xFF;  // a committed residual: state / centre from the old column of its frame
constexpr unsigned HS_WIN_NONE = 0xFE;  // no residual in this slot
// (any other value: a residual inserted since the last commit, starting in that ResState)

// a point inserted since the last commit (uploaded with the commit's structure)
struct HsStagedPoint {
  float u, v, idepth, idepth_zero, priorF, relBL;
  int nGood;
  float color[8], weight[8];
};

struct HsWinPointSet {
  float *u, *v, *idepth, *idepth_zero, *priorF, *color, *weight, *relBL;
  int* nGood;
  uint8_t* r_state;
  float* r_center;
};

struct HsWinGatherArgs {
  int n;                        // points of the new layout
  int nF;                       // frames of the new layout
  int col_src[HS_MAXF];         // new frame column -> old column (-1: inserted since the last commit)
  float th_init[HS_MAXF];       // frameEnergyTH of the inserted frames
  const int* src;               // [n] old position, or -(1 + k) for staged point k
  const uint8_t* newres;        // [n][8] slot codes
  const HsStagedPoint* staged;
  HsWinPointSet from, to;
  const float* hdif_from;       // the last solve's HdiF (old layout)
  float* hdif_to;
  float* frameTH;               // [HS_MAXF] permuted in place
};

__global__ void hs_k_win_gather(HsWinGatherArgs a);
__global__ void hs_k_win_newest(int n, int newest, const int* res_of_slot, const uint8_t* r_state,
                                const float* r_center, const float* hdif, float* out, int cap, int* n_out);
