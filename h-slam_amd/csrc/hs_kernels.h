// hs_kernels.h — kernel argument blocks, the device-resident window state and launch declarations.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hs_types.h"
#include "hs_host_math.h"
#include "hs_layout.h"

constexpr int HS_SOLVE_NT = 512;   // hs_k_solve workgroup size
constexpr int HS_STITCH_NT = 1024; // hs_k_stitch workgroup size
constexpr int HS_LIN_NW = 8;       // hs_k_lin waves per block (production: each takes points; exact mode: wave 0)
constexpr int HS_LIN_NT = 64 * HS_LIN_NW;
#ifndef HS_LIN8_WAVES
#define HS_LIN8_WAVES 8  // one workgroup per CU (its LDS): waves wv and wv + 4 share a SIMD (hs_k_lin8's L8_PRIO)
#endif
constexpr int HS_LIN8_NT = 64 * HS_LIN8_WAVES;  // hs_k_lin8 workgroup size (8 points per wave at a time)
constexpr int HS_NNS = 7;         // gauge nullspaces: 6 pose + 1 scale (System::getNullspaces)
// The adjoint buffers (fp64 d_adHost / d_adTarget, fp32 d_adHostF / d_adTargetF: [HS_MAXF^2][64]) carry one stamp word
// after the adjoints: hs_k_fix_frames writes the upload's sequence number there (the fp32 buffers its bits) and into
// a separate expectation word, and every reader launch (hs_k_stitch: fp64, hs_k_solve: fp32) compares the two.  A
// mismatch -- a zero fill or any other write landing on the buffers after the upload -- sets HS_STATUS_STALE in
// HsDevState::status, which the C-ABI returns as HS_ERR_STATE instead of a system with zero frame rows.  The
// expectation lives in device memory, not in the launch arguments, so a captured GN loop graph stays valid across
// uploads (hs_ba_fix_linearization uploads once per keyframe).
constexpr int HS_ADJ_STAMP = HS_MAXF * HS_MAXF * 64;
// status bits: each stamp check owns its bit and sets / clears it at every launch (the stitch the fp64 one, the
// solve the fp32 one), so the bits describe the adjoints the last launches read
enum { HS_STATUS_NONFINITE = 1, HS_STATUS_STALE64 = 2, HS_STATUS_STALE32 = 4, HS_STATUS_STALE = 6 };

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
  int stop;                 // optimize's device-side break: set by the first solve launch that stops, read by the
                            // iteration's other launches (HsLinArgs.brk, HsRedArgs.stop); cleared by hs_k_result
  int pad[2];
};

// Per-lane accumulator entries of the fused linearize kernel (hs_k_lin): lane (slot t, pattern k) of a wave
// keeps, for the (host, t) pair of its block, 16 AccumulatorApprox entries (HS_E_TOP, decoded in hs_k_reduce's
// stitch), HS_ND(exact) AccumulatorXX<8,8> accD entries (lane = (row, col) of every (t1, t2) block), 4 accE +
// 1 accEB entries (lane (t, k): row k of accE[host, t]) and one accHcc / accbc entry (lanes 0..19).
constexpr int HS_E_TOP = 16;
constexpr int HS_ND_PROD = 28;   // (t1 <= t2) over the 7 non-host slots; D(t2, t1) = D(t1, t2)^T
constexpr int HS_ND_EXACT = 49;  // every ordered (t1, t2): the single-thread reference's own sums
__host__ __device__ constexpr int hs_ne(bool exact) { return HS_E_TOP + (exact ? HS_ND_EXACT : HS_ND_PROD) + 5 + 1; }
__host__ __device__ constexpr int hs_nt(int n) { return n * (n + 1) / 2; }  // upper triangle of the n x n system

// image slot of window frame t (per lane): a select chain over the uniform kernel arguments, so no per-lane load
// sits in front of the bilinear taps
__device__ __forceinline__ int hs_img_slot(const int (&slot)[HS_MAXF], int t) {
  int r = slot[0];
#pragma unroll
  for (int i = 1; i < HS_MAXF; i++) r = (t == i) ? slot[i] : r;
  return r;
}

struct HsLinArgs {
  const float4* img;           // level-0 texels of the image slots, slot s at img + s * img_stride
  const float* img3;           // the same texels packed as 12-byte (I, dx, dy) triplets (hs_k_lin8)
  long long img_stride;
  int img_slot[HS_MAXF];       // window frame -> image slot (frames keep their slot while the window slides)
  const HsDevState* st;
  HsLinParams lp;
  int nF;
  int write_center;
  int fuse_step;               // apply resubstitute + point step of the previous solve first
  int accumulate;              // 1: the per-lane accumulators and the block partials (0: linearize + applyRes only)
  int host_begin[HS_MAXF + 1]; // first point of each host (points are sorted by host)
  int blk_begin[HS_MAXF + 1];  // first block of each host: block b of host h covers an equal share of its points
  int W;                       // waves of a block that take points (1 = the single-thread reference's point order)
  // marginalization pass (hs_ba_marginalize_points): only points with marg[p] != 0 are linearized (after
  // resetOOB), their active residuals take fixLinearizationF, the SC prelude uses priorF * margPriorFac and no
  // prior shift; every other point reports no active residual.  nullptr = the normal pass.
  const uint8_t* marg;
  const float* adHTdelta;      // [nF*nF][8] index host + nF*target (EnergyFunctional::adHTdeltaF), then cDeltaF [4]
  float margPriorFac;          // setting_idepthFixPriorMargFac
  const HsPrecalc* pre;        // [nF*nF] host*nF + target
  const float* frameTH;        // [nF]
  const float* adHostF;        // [nF*nF][64] index h + nF*t: fp32 adjoints (fuse_step: xAd formed per block)
  const float* adTargetF;
  // points
  float* idepth;
  float* idepth_zero;
  const float* u;
  const float* v;
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
  float* p_HdiF;               // written (this linearization's SC prelude)
  const float* p_HdiF_prev;    // read by the fused step: the previous linearization's (ping-pong with p_HdiF)
  float* p_bdSumF;
  float* p_Hcd;                // [n][4]
  float* p_JpJdF;              // [n][8][8]
  float* p_step;               // [n]
  // linearizeAll(true) bookkeeping (hs_k_lin_fix only): maxRelBaseline / numGoodResiduals per point, in / out
  float* fix_relBL;
  int* fix_nGood;
  float* newest_cand;          // [n] energy of the point's residual into the newest frame, -1 = none
  // nullable (hs_k_lin8, large single-rank windows): setNewFrameEnergyTH's pass-1 histogram (HsRedArgs::th_hist) of
  // the candidates, counted as they are written (an LDS histogram per block, its nonzero bins added at the end), in
  // place of hs_k_reduce's histogram blocks
  unsigned int* th_hist;
  // block partials: part[blk][ne][64] (fp32, waves summed in wave order), part_e[blk][4] (fp64 energy,
  // sum |idepth|, #points)
  float* part;
  double* part_e;
  long long* trace;            // nullable: per-block wall-clock checkpoints [grid][16]
  int brk;                     // optimize's device-side break: return at entry when st->stop is set
};

// hs_k_reduce: (host, chunk) blocks sum the host's block partials in block order (fp64) into the host sums; + one
// energy block (writes the energies behind the system vector).  The setNewFrameEnergyTH fields are read by the
// extra block of hs_k_stitch.
struct HsRedArgs {
  int nF, ne, Q, nblk;
  int blk_begin[HS_MAXF + 1];
  const float* part;
  const double* part_e;
  double* hostsum;             // [nF][ne][64]
  double* sysE;                // [3] energy, sum |idepth|, number of points
  // setNewFrameEnergyTH over the candidates of all ranks (rank r at cand + r*stride, -1 = none)
  const float* cand;
  int nranks, stride;
  float* frameTH;
  int newest;
  float frameEnergyTHN, facMedian, constWeight, overallWeight;
  int skip_threshold;          // marginalization pass: setNewFrameEnergyTH is not part of it
  // the select's first radix pass (candidate bits 30..19) as a 4096-bin histogram, counted by nhist blocks of
  // hs_k_reduce into th_hist (integer atomics: order-independent); consumed and re-zeroed by hs_k_stitch
  unsigned int* th_hist;
  int nhist;
  // large windows: the select's pass 2 by np2 blocks of the stitch launch (nullptr / 0: the select block scans the
  // candidates itself): pass-2 histogram [1024], survivor list [HS_TH_SURV] and its length (zero between launches)
  unsigned int* th_hist2;
  unsigned int* th_surv;
  unsigned int* th_nsurv;      // [2]: survivor count, overflow flag
  int np2;
  int hist_only;               // hs_k_reduce: only the nhist histogram blocks (multi-rank path, after the exchange)
  long long* trace;
  const int* stop;             // nullable: &st->stop (optimize's device-side break; the launch returns when set)
};
constexpr int HS_TH_BINS = 4096;
constexpr int HS_TH_SURV = 1 << 20;

// hs_k_stitch: stitchDoubleMT of the top and Schur systems from the host sums, one block per output block of the
// system (8x8 frame blocks f <= g, calib x frame f, calib x calib), every output entry summed over the
// contributing (host, target) pairs in a fixed order and written once.
struct HsStitchArgs {
  int nF, exact, ne;
  const double* hostsum;
  const double* adHost;        // [nF*nF][64]  index h + nF*t
  const double* adTarget;
  double* out;                 // system vector [SL]: upper triangle of HA - sc HSC (diagonal HA (1+lambda) - sc HSC)
                               // in the n x n layout, then bA - bSC
  double* sep;                 // nullable: [2][SL] HA | bA, HSC | bSC (granular read-back)
  // the diagonal frame blocks' host-f Schur terms, [nF][64] each (written by the launch's first nF blocks; their
  // consumers fold them in: out(f, f) -= sc aux_out[f], sepS(f, f) += aux_sep[f]); nullable
  double* aux_out;
  double* aux_sep;
  double lambda1, sc;          // 1 + lambda, 1 / (1 + lambda)
  HsRedArgs red;               // setNewFrameEnergyTH (the launch's last block)
  long long* trace;
  // non-null: the GN loop call's results (hs_k_result's work: elog, the last energy, status, iteration count, then
  // the done word) by one extra block at the end of the grid -- the call's last stitch launch, instead of a launch
  // of their own
  double* res_out;
  const double* res_elog;
  const HsDevState* res_st;
  int res_k, res_slot;
  unsigned long long res_seq;
  unsigned int* res_ticket;    // with res_out: blocks retired so far (zero between launches); the last one writes the
                               // results, so the done word means the whole launch has finished
  int* status;                 // nullable: &HsDevState::status, HS_STATUS_STALE when the fp64 adjoints' stamp is not
  const unsigned int* adj_expect;  // the sequence of the last adjoint upload (written by hs_k_fix_frames)
};

enum { HS_SOLVE = 1, HS_APPLY = 2 };

struct HsSolveArgs {
  int flags;
  int iteration;               // < 0: use st->iteration
  int nF;                      // window size (== st->nF)
  HsDevState* st;
  const double* sys;           // the system vector of hs_k_stitch (all-reduced over the ranks): [n*n] | [n]

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
  int dbg;                     // experiments (env HS_SOLVE_DBG); 0 in production
  // multi-rank exchange (hs_ba.cpp exchange()): gsys = [nranks][gstride] the ranks' system vectors + energies as
  // all-gathered, summed here in rank order (every rank the same sums) in place of sys / sysE; sys_out receives the
  // sum.  th_local: the launch's block 1 runs setNewFrameEnergyTH's select over the gathered candidates (th): 1 the
  // whole select (pass 1 counted in LDS), 2 pass 3 of the multi-block select (th_hist / th_hist2 / th_surv filled by
  // the reduce and stitch launches).
  const double* gsys;
  int nranks, gstride;
  double* sys_out;
  int th_local;
  HsRedArgs th;
  double aux_sc;               // the stitch's sc: the diagonal blocks' host-f Schur terms (after the energies) fold in
  int reset_it;                // >= 0: the first launch of a GN loop call sets iteration = reset_it, status = log_count = 0
  // optimize's canbreak on the device (Src/FullSystemOptimize.cpp:493): a launch after the call's first stops (block
  // 0 returns at entry and sets st->stop) when the previous step allowed it (st->canbreak) and the previous
  // iteration index was >= minOpt; block 1's threshold select runs anyway (same candidates, same result)
  int brk, minOpt;
  int chk_adj;                 // compare the fp32 adjoints' stamp with *adj_expect (HS_STATUS_STALE on a mismatch)
  const unsigned int* adj_expect;
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

__global__ void hs_k_lin(HsLinArgs a);        // production partitioning
__global__ void hs_k_lin_exact(HsLinArgs a);  // HS_ACC_EXACT: one wave per host, the reference's sums
__global__ void hs_k_lin_fix(HsLinArgs a);        // + linearizeAll(true)'s per-point bookkeeping
__global__ void hs_k_lin_exact_fix(HsLinArgs a);
__global__ void hs_k_lin_gen(HsLinArgs a);         // hs_k_lin with the point step and the trace as run-time flags
__global__ void hs_k_lin_marg(HsLinArgs a);        // the marginalization pass (HsLinArgs.marg set)
__global__ void hs_k_lin_exact_marg(HsLinArgs a);
__global__ void hs_k_lin8(HsLinArgs a);       // production: lane = (point, target slot), 8 points per wave
__global__ void hs_k_reduce(HsRedArgs a);
__global__ void hs_k_th_select(HsRedArgs a);
__global__ void hs_k_th_pass2(HsRedArgs a);     // the multi-block pass 2 alone (test hook; multi-rank large windows)
__global__ void hs_k_stitch(HsStitchArgs a);
__global__ void hs_k_solve(HsSolveArgs a);
__global__ void hs_k_combine(HsSolveArgs a);
// the GN loop's results in one zero-copy write to pinned host memory: out[0, k) = elog, out[k] = energy of the last
// linearization, out[k + 1] = status, out[done_slot] = iterations run; then seq into the 64-bit word at
// out[done_slot + 1] (system scope, release: the host may take the results from it without the stream's end)
__global__ void hs_k_result(const double* elog, int k, const double* sysE, HsDevState* st, double* out, int brk,
                            int done_slot, unsigned long long seq);   // multi-rank: the gathered systems summed into sys_out (+ block 1: select)
__global__ void hs_k_resub(HsResubArgs a);
__global__ void hs_k_debug_se3(int op, int n, const double* in, double* out);  // test hook
__global__ void hs_k_debug_fastmath(int n, const float* a, const float* b, float* out);  // test hook (hs_lin8)
__global__ void hs_k_apply_step(int n, const float* step, float* idepth, float* idepth_zero);
__global__ void hs_k_pack_texels(long long n, const float4* src, float* dst3);  // float4 texels -> (I, dx, dy)
// System::optimize's tail, frame part (Src/FullSystemOptimize.cpp:498-506) on the device: the newest frame's
// setEvalPT(PRE_worldToCam, (0,..,0, a, b, 0, 0)) + takeData, then setAdjointsF + setPrecalcValues of every pair (one
// thread per pair).  The nullspaces of the moved frame are left to the host (hs_ctx::frames_stale).  One block of 64.
// PointFrameResidual::resetOOB of every slot: state IN, inactive, energies 0
__global__ void hs_k_reset_res(int n8, uint8_t* st, uint8_t* act, float* en, float* nen);
// hs_ba_marginalize_points on the device: EnergyFunctional::setDeltaF's adHTdeltaF [nF*nF][8] + cDeltaF [4] (after
// them) from the window state; then HM += w (M - Msc), bM += w (Mb - Mbsc) from the separate stitch outputs
__global__ void hs_k_marg_delta(const HsDevState* st, const float* adHF, const float* adTF, float* adHTd);
__global__ void hs_k_marg_update(const double* sep, const double* sep_aux, double* HM, double* bM, int nF, int SL,
                                 double w);
__global__ void hs_k_fix_frames(HsDevState* st, HsPrecalc* pre, double* adH, double* adT, float* adHF, float* adTF,
                                hs_params P, int fix, unsigned int seq, unsigned int* expect);
__global__ void hs_k_debug_stall(long long ticks);  // test hook: a bounded spin on the wall clock (a stalled peer)
__global__ void hs_k_lenergy(int n, const float* idepth, const float* idepth_zero, const float* priorF, float* chunk,
                             double* out);
