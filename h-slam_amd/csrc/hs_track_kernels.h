// hs_track_kernels.h — argument blocks of the CoarseTracker kernels (hs_track_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hs_track.h"
#include "hs_host_math.h"

#define HS_TRK_MAXCHECK 12
#define HS_TRK_MAXLOG 256  // LM iterations logged per hypothesis (10+20+3*50 + one repeated level <= 230)

constexpr double hs_trk_scale_rot = 1.0, hs_trk_scale_trans = 0.5, hs_trk_scale_a = 10.0, hs_trk_scale_b = 1000.0;

// one pyramid level: CoarseTracker's K / Ki (makeK) and the device images / reference points
struct HsTrkLevel {
  int w, h;
  float fx, fy, cx, cy;
  float Ki[9];
  const float4* img;    // new frame (I, dx, dy, 0)
  const float* pc_u;
  const float* pc_v;
  const float* pc_id;
  const float* pc_col;
  const int* pc_n;
};

// per hypothesis: the outcome without abort + the per-level residual log for the caller's replay
struct HsTryOut {
  double T[7];
  double aff[2];
  int ok, n_checks, iters, n_warped;
  int passes;                 // calcRes(+calcGSSSE) passes run
  long long point_passes;     // sum over the passes of the level's reference points (the roofline's units)
  int check_lvl[HS_TRK_MAXCHECK];
  double check_res[HS_TRK_MAXCHECK];
  double check_flow[HS_TRK_MAXCHECK][3];
  double res6[6];
  double H[64];
  double b[8];
};

constexpr int HS_TRK_INL = 4;  // hypotheses passed in the kernel arguments

struct HsTrackArgs {
  HsTrkLevel lv[HS_TRK_MAXLEV];
  int coarsest;
  float huberTH, coarseCutoffTH, affineOptModeA, affineOptModeB;
  float refExposure, newExposure;
  double refAff[2];
  const double* T_in;   // [n][7]
  const double* aff_in; // [n][2]
  int n_inl;            // n <= HS_TRK_INL: the hypotheses come in the arguments (inl: T [n][7] | aff [n][2])
  double inl[9 * HS_TRK_INL];
  HsTryOut* out;        // [n]
  HsTryOut* hout;       // [n] or null: the same records in mapped pinned host memory (written at the end)
  int single_pass, pass_lvl;
  float pass_cutoff;
  unsigned int spin_limit;  // polls of the G-member meeting before a hypothesis is flagged (then rerun with G = 1)
  double* lm_log;       // [n][HS_TRK_MAXLOG][3]: resNew/N, resOld/N (accept test), |inc| (break test) per LM iteration
  int* lm_lvl;          // [n][HS_TRK_MAXLOG]
  long long* trace;
  // G workgroups per hypothesis (blocks h G .. h G + G - 1): each pass's points are spread over them; their sums
  // meet as tagged granules in part [n][2 (pass parity)][HS_TRK_MAXG][HS_TRK_NRED][2] (u64), and every workgroup
  // forms the same totals (in workgroup order) and runs the same LM step.  A granule's tag is (epoch << 12) |
  // (pass + 1): the launch's epoch (1 .. 2^20 - 1, one per launch, the buffers zeroed when it wraps) keeps the
  // granules of earlier launches from matching, so no per-launch memset is needed
  int G, nhyp;
  // per-level member count: a level with fewer than gmin reference points (one workgroup's batch: 512 threads x 4
  // points) runs on member 0 alone, with no per-pass meeting, and member 0 hands the state to the other members once
  // at the level's end (lvrec [n][HS_TRK_MAXLVSEQ][32] tagged granules, (epoch << 8) | (level sequence + 1))
  int gmin;
  unsigned long long* lvrec;
  unsigned int epoch;
  int solve;            // the LM step's 8x8 solve: 0 Gauss-Jordan on 64 lanes, 1 Eigen-order LDLT on 8 row lanes
  double* part;
  unsigned int* cnt;    // [nhyp] timeout flags (a member never arrived): the epoch of the launch that timed out
  // [nhyp] or null: the lead of hypothesis h stores seq here (system scope, release) after its record (hout) and
  // flags, so the host may read the results without waiting for the launch's end (hs_track.cpp, run_tries)
  unsigned int* hdone;
  unsigned int seq;
};
constexpr int HS_TRK_PASS_BITS = 12;  // passes per launch < 4096 (<= 5 levels x (50 + 1 + 6 cutoff repeats) x 2)
constexpr int HS_TRK_NRED = 52;  // the reduced values of a pass (45 normal-equation entries, 4 energies / flows, 3 counts)
constexpr int HS_TRK_MAXG = 16;
constexpr int HS_TRK_MAXLVSEQ = 8;  // level ends per track (<= 5 levels + one repeated level)

__global__ void hs_k_track(HsTrackArgs a);
__global__ void hs_k_trk_scatter(int n, const float* cu, const float* cv, const float* cid, const float* hdi, int w,
                                 int h, float* idepth0, float* wsum0);
constexpr int HS_TRK_SCAT_CAP = 8192;  // points sorted in LDS by hs_k_trk_scatter_sorted (dynamic LDS: 8 B each)
__global__ void hs_k_trk_scatter_sorted(const int* d_n, int n_arg, const float* cu, const float* cv, const float* cid,
                                        const float* hdi, int w, int h, float* idepth0, float* wsum0);
__global__ void hs_k_trk_down(int wl, int hl, int wlm1, const float* idm, const float* wsm, float* idl, float* wsl);
__global__ void hs_k_trk_dilate(int wl, int hl, int diag, const float* bak, float* id, float* ws);
__global__ void hs_k_trk_count(int wl, int hl, const float* id, const float* ws, const float4* ref, int* blockCount);
__global__ void hs_k_trk_scan(int nb, const int* blockCount, int* blockOff, int* pc_n);
__global__ void hs_k_trk_compact(int wl, int hl, const float* id, const float* ws, const float4* ref,
                                 const int* blockOff, float* pu, float* pv, float* pid, float* pcol);
