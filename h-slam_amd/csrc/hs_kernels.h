// hs_kernels.h — kernel argument blocks, the device-resident window state and launch declarations.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hs_types.h"
#include "hs_host_math.h"
#include "hs_layout.h"

constexpr int HS_SOLVE_NT = 256;  // hs_k_solve workgroup size
constexpr int HS_NNS = 7;         // gauge nullspaces: 6 pose + 1 scale (System::getNullspaces)

// Window state owned by the device between GN iterations (updated by hs_k_solve).
struct HsDevState {
  hs::FrameH frames[HS_MAXF];
  hs::CalibH calib;
  HsCalib dcal;             // scaled calib read by the linearize kernel
  float cstep[4];           // xF.head<CPARS>() of the last solve (resubstituteF_MT)
  double lastX[HS_MAXDIM];
  int nF;
  int iteration;            // next GN iteration index (orthogonalize from 2)
  int status;               // != 0: non-finite system / step
  int log_count;            // number of energies written to the log
  int canbreak;
  int pad[3];
};

struct HsLinArgs {
  const float4* img[HS_MAXF];  // level-0 texels per window frame
  const HsDevState* st;
  HsLinParams lp;
  int nF;
  int write_center;
  int fuse_step;               // apply resubstitute + point step of the previous solve first
  int host_begin[HS_MAXF + 1]; // first point of each host (points are sorted by host)
  // marginalization pass (hs_ba_marginalize_points): only points with marg[p] != 0 are linearized (after
  // resetOOB), their active residuals take fixLinearizationF, the SC prelude uses priorF * margPriorFac and no
  // prior shift; every other point reports no active residual.  nullptr = the normal pass.
  const uint8_t* marg;
  const float* adHTdelta;      // [nF*nF][8] index host + nF*target (EnergyFunctional::adHTdeltaF)
  float cDelta[4];             // EnergyFunctional::cDeltaF
  float margPriorFac;          // setting_idepthFixPriorMargFac
  const HsPrecalc* pre;        // [nF*nF] host*nF + target
  const float* frameTH;        // [nF]
  const float* xAd;            // [nF*nF][8] index h*nF + t (fuse_step)
  // points
  const int* pt_host;
  const float* u;
  const float* v;
  float* idepth;
  float* idepth_zero;
  const float* priorF;
  const float* color;          // [n][8]
  const float* weight;         // [n][8]
  const int* res_of_slot;      // [n][8]
  const int8_t* res_order;     // [n][8]
  // residual state (in/out)
  uint8_t* r_state;
  uint8_t* r_active;
  float* r_energy;
  float* r_newEnergy;
  float* r_ewo;
  float* r_center;             // [m][3]
  // per point outputs (slot layout)
  uint8_t* p_actmask;
  float* p_HdiF;
  float* p_bdSumF;
  float* p_Hcd;                // [n][4]
  float* p_JpJdF;              // [n][8][8]
  float* p_Jrec;               // [n][8][HS_JREC]
  double* p_energy;            // [n]
  float* p_step;               // [n]
  float* newest_cand;          // [n] energy of the point's residual into the newest frame, -1 = none
  long long* trace;            // nullable: per-block wall-clock checkpoints [grid][16]
};

struct HsStitchArgs {
  int nF, S;
  const double* part;
  const int* part_cnt;
  const double* hccbc;
  const double* adHost;        // [nF*nF][64]  index h + nF*t
  const double* adTarget;
  double* HA;                  // [n*n] zeroed
  double* bA;
  double* HSC;
  double* bSC;
  long long* trace;
};

struct HsAccArgs {
  int nF, S, nP;
  int W;                       // waves of a block that accumulate (1: one wave, the reference's point order)
  int blocked;                 // a (host, target, split) block can exceed 1000 updates: emulate shiftUp
  const int* host_pt_begin;    // [nF+1]
  const uint8_t* actmask;
  const float* HdiF;
  const float* bdSumF;
  const float* Hcd;
  const float* JpJdF;
  const float* Jrec;
  double* part;                // [nF*nF][S][HS_PART_N] (fp64 sums of the waves' fp32 partials)
  int* part_cnt;               // [nF*nF][S][16]: top count, D counts (per k), E count
  const double* p_energy;
  const float* idepth;         // |idepth| sum for doStepFromBackup's sumNID
  double* energy_out;          // [3]: energy, sum |idepth|, number of points
  double* hccbc;               // [20] finished Hcc (16) + bc (4), fp64
  // setNewFrameEnergyTH over the candidates of all ranks (rank r at cand + r*stride, -1 = none)
  const float* cand;
  int nranks, stride;
  float* frameTH;
  int newest;
  float frameEnergyTHN, facMedian, constWeight, overallWeight;
  int skip_threshold;          // marginalization pass: setNewFrameEnergyTH is not part of it
  long long* trace;
  // stitch fused into the accumulate launch: the last split block of a (host, target) pair to finish
  // (ticket counter) stitches that pair; the Hcc block adds accHcc / accbc itself
  HsStitchArgs stitch;
  int* ticket;                 // [nF*nF] zero between launches (the stitching block resets its counter)
};


enum { HS_SOLVE = 1, HS_APPLY = 2 };

struct HsSolveArgs {
  int flags;
  int iteration;               // < 0: use st->iteration
  int nF;                      // window size (== st->nF)
  HsDevState* st;
  double* HA;                  // HA | bA | HSC | bSC, consumed then zeroed (SOLVE)
  double* bA;
  double* HSC;
  double* bSC;
  const double* HM;            // nullable: marginalization prior is zero
  const double* bM;
  const double* Nproj;         // [2][n][HS_NNS] nullspace factors N | Npi (P = (N Npi^T + Npi N^T) / 2)
  const float* adHostF;        // [nF*nF][64]
  const float* adTargetF;
  float* xAd;                  // out [nF*nF][8]
  HsPrecalc* pre;              // out [nF*nF]
  double* x_out;               // [n]
  const double* sysE;          // [3] energy, sum |idepth|, #points of the consumed linearization
  double* energy_log;          // SOLVE appends sysE[0] at st->log_count
  long long* trace;
  double initialCalibHessian;
  float thOptIterations;
};

struct HsResubArgs {
  int n, nF, apply;
  const HsDevState* st;
  const int* host;
  const float* xAd;            // [nF*nF][8] index h*nF + t
  const uint8_t* actmask;
  const float* bdSumF;
  const float* HdiF;
  const float* Hcd;
  const float* JpJdF;          // [n][8][8]
  const int8_t* res_order;
  float* idepth;
  float* idepth_zero;
  float* step;
};

__global__ void hs_k_linearize(HsLinArgs a);
__global__ void hs_k_accumulate(HsAccArgs a);
__global__ void hs_k_solve(HsSolveArgs a);
__global__ void hs_k_resub(HsResubArgs a);
__global__ void hs_k_apply_step(int n, const float* step, float* idepth, float* idepth_zero);
