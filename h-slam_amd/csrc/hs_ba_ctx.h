// hs_ba_ctx.h — the BA context (private to the library): device buffers allocated to capacity once, the
// committed window layout, and the host mirror of the window's structure that the incremental keyframe API
// (include/hs_ba.h, "incremental window") edits between commits.  Shared by hs_ba.cpp (GN loop, legacy
// whole-window set-up, read-back), hs_ba_window.cpp (insert / drop / remove / commit) and hs_track.cpp (the
// BA -> tracker hand-off of makeCoarseDepthL0's inputs).
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <string>
#include <thread>
#include <vector>

#include "../../include/hs_ba.h"
#include "hs_host_math.h"
#include "hs_kernels.h"
#include "hs_win_kernels.h"

namespace hs {
extern thread_local std::string g_err;  // hs_last_error(), shared by every entry point of the library
inline int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
}  // namespace hs

#define HS_HIP(x)                                                                                          \
  do {                                                                                                     \
    hipError_t e_ = (x);                                                                                   \
    if (e_ != hipSuccess) return hs::fail(HS_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_));     \
  } while (0)

#define HS_NCCL(x)                                                                                            \
  do {                                                                                                        \
    ncclResult_t r_ = (x);                                                                                    \
    if (r_ != ncclSuccess) return hs::fail(HS_ERR_RCCL, std::string(#x) + ": " + ncclGetErrorString(r_));     \
  } while (0)

#define HS_TRY(x)        \
  do {                   \
    int rc_ = (x);       \
    if (rc_) return rc_; \
  } while (0)

namespace hs {

constexpr int kLogCap = 4096;          // energies logged on the device per optimize / iterate call
constexpr int kEventIters = 128;       // iterations timed with HIP events per call
constexpr int kLinBlocksTarget = 256;  // linearize blocks of a window (points per wave grows beyond that)
// hs_k_lin8 (lane = (point, target slot), 8 points per wave at a time) takes the production linearization from this
// many points up: its wave issues ~2.3x fewer instructions per point (throughput), while hs_k_lin's one-point waves
// finish a small window sooner (latency).  Measured (r03_b3, per launch): 2k 10.6 vs 16.5 us, 5k 21.1 vs 18.4,
// 10k 30.2 vs 25.7, 20k 53.8 vs 43.6 (hs_k_lin vs hs_k_lin8).  Env HS_LIN8=0 / 1 forces either.
constexpr int kLin8MinPoints = 4000;
constexpr int kThMultiMinPoints = 60000;  // the multi-block threshold select (below: one block beside the solve)
constexpr int kLin8BlocksTarget = 256;  // hs_k_lin8 blocks of a window (one 8-wave block per CU)
// hs_k_lin8's taps address the packed slots through one buffer resource with 32-bit offsets: the texel index is formed
// by 24-bit multiplies (W * H < 2^23) and slot * W * H * 12 + offset must stay below 2^31 over all HS_MAXF slots.
// Larger images run hs_k_lin (64-bit addressing) at every point count.
inline bool lin8_supported(int W, int H) {
  const long long px = (long long)W * H;
  return px < (1LL << 23) && (long long)HS_MAXF * px * 12 + 12 * (long long)W <= 0x7fffffffLL;
}

// Allocate and zero-fill n elements; the fill is enqueued on `s`, the stream every later user of the buffer runs on.
// (A null-stream hipMemset returns before the fill lands and does not order against a hipStreamNonBlocking stream:
// a context's first kernel could store into a buffer that the fill then zeroed -- tools/micro/memset_order.hip.)
template <typename T>
inline int dalloc(T** p, size_t n, hipStream_t s) {
  if (n == 0) n = 1;
  HS_HIP(hipMalloc((void**)p, n * sizeof(T)));
  HS_HIP(hipMemsetAsync(*p, 0, n * sizeof(T), s));
  return HS_OK;
}

// Per-point state that survives a structural commit (double-buffered: the commit gathers set A into set B in the new
// point order, then the two swap).  The last solve's HdiF survives too, through the HdiF ping-pong pair.
struct PointSet {
  float *u = nullptr, *v = nullptr, *idepth = nullptr, *idepth_zero = nullptr, *priorF = nullptr;
  float *color = nullptr, *weight = nullptr;  // [cap][8]
  float* relBL = nullptr;                     // maxRelBaseline (linearizeAll(true) bookkeeping)
  int* nGood = nullptr;                       // numGoodResiduals
  uint8_t* r_state = nullptr;                // [cap][8] residual state, slot layout
  float* r_center = nullptr;                  // [cap][8][3] centerProjectedTo
};

// host mirror of the window's structure (the reference's frameHessians / pointHessians / residual lists)
struct WinFrame {
  int key = 0;            // stable frame handle (insertion counter)
  int slot = 0;           // image slot in d_img_all
  int committed = -1;     // window index in the committed device layout (-1: inserted since the last commit)
  hs_frame init{};        // the hs_frame it was inserted with (new frames only)
};
struct WinPoint {
  int handle = 0;
  int src = 0;            // committed device position, or -(1 + k): the k-th point staged since the last commit
  int nres = 0;
  int tgt[HS_MAXF];       // residual list (PointHessian::residuals order): target frame keys
  uint8_t st[HS_MAXF];    // 0xFF: a committed residual; else the initial ResState of a residual inserted since
};

}  // namespace hs

struct hs_ctx {
  hs_params P;
  int device = 0;
  hipStream_t stream = nullptr;
  std::vector<hipEvent_t> ev;  // 4 per timed iteration
  hipEvent_t ev_ready = nullptr;  // cross-stream hand-off (BA -> tracker)
  hipEvent_t ev_upload = nullptr; // the last asynchronous upload from the pinned staging buffers (h_fstage, h_stage,
                                  // h_state, h_raw): waited on before the host rewrites them
  uint8_t* h_fstage = nullptr;    // pinned: the projector of upload_frames
  int events = 0;              // HS_EVENT_TIMING: 0 none (default), 1 linearize kernel only, 2 every phase

  // ---- capacity (allocated once; hs_ba_reserve or the first hs_ba_set_window that needs more)
  int cap_P = 0, cap_blk = 0, cap_W = 0, cap_H = 0, cap_stride = 0;
  hs_camera cam{};
  bool haveCam = false;

  // ---- committed window (host side)
  int nF = 0, nP = 0, nR = 0;
  // hs_k_lin partitioning: blk_begin[h] = first block of host h; W waves per block take points; exact: one wave
  // per host in point order (HS_ACC_EXACT=1, the single-thread reference's fp32 sums)
  std::vector<int> blk_begin;
  int nblk = 0, W = 4, ne = 0, Q = 0;
  bool exact = false;
  bool lin8 = false;              // production linearizations run hs_k_lin8 (8-wave blocks, W = 8)
  // large windows: setNewFrameEnergyTH's select as a multi-block pass 2 (np2 extra blocks of the stitch launch) and a
  // one-block pass 3 over pass 2's survivors, instead of the stitch's single select block scanning every candidate
  // twice (env HS_TH_MULTI=0 / 1 forces it off / on)
  bool th_multi = false;
  bool hist_in_lin = false;       // the last linearize launch counted the select's pass-1 histogram (hs_k_lin8)
  bool sepValid = false;          // d_sep holds the separate HA / HSC of the last linearization
  std::vector<int> pt_host, res_point, res_target, host_pt_begin;
  std::vector<int> res_of_slot;   // [nP*8]
  std::vector<int8_t> res_order;  // [nP*8]
  std::vector<double> HM, bM, Porth, Nproj;
  int img_slot[HS_MAXF] = {0, 1, 2, 3, 4, 5, 6, 7};  // window frame -> image slot
  HsDevState* h_state = nullptr;  // pinned staging of the device state
  bool h_state_valid = false;     // h_state equals the device state (no solve since the last fetch / upload)
  bool brk_active = false;        // gn_iterations' device-side break: the launches carry the stop checks
  bool tail_pending = false;      // hs_k_fix_frames moved the newest frame on the device: the next fetch_state
                                  // recomputes its nullspaces on the host and leaves the projector stale
  bool proj_stale = false;        // Nproj predates the frames' nullspaces: the next solve launch recomputes it
  bool hm_host_stale = false;     // d_HM / d_bM are newer than HM / bM (device marginalization): sync_hm
  int* h_ctl = nullptr;           // pinned: iteration, status, log_count
  bool haveSystem = false;        // a stitched, not yet solved system is in the slots

  // ---- incremental window (hs_ba_insert_* / drop / remove; applied to the device by the commit)
  bool incremental = false;       // the window is edited through the incremental API (host mirror valid)
  bool dirty = false;             // structural edits not yet committed
  bool tail_valid = false;        // d_r_active holds the last hs_ba_fix_linearization's activity (toRemove)
  std::vector<hs::WinFrame> wframes;              // window order
  std::vector<std::vector<hs::WinPoint>> wpts;    // per window frame: its points (pointHessians order)
  std::vector<HsStagedPoint> staged;              // points inserted since the last commit
  std::vector<int> loc_key, loc_idx;              // handle -> (host frame key, index in its list); key -1 = gone
  int next_handle = 0, next_frame_key = 0;
  std::vector<int> pt_handle;                     // committed: handle of the point at each device position
  uint8_t* h_stage = nullptr;                     // pinned upload staging of a commit
  size_t h_stage_cap = 0;
  uint8_t* d_stage = nullptr;                     // its device copy
  size_t d_stage_cap = 0;

  // ---- device
  float* d_img3 = nullptr;        // the same slots packed as (I, dI/dx, dI/dy) triplets: hs_k_lin8's taps (pack_slot)
  float4* d_img_all = nullptr;    // HS_MAXF image slots of level-0 texels
  size_t img_px = 0;
  float* d_raw = nullptr;         // raw level-0 staging for hs_ba_set_frame_image_raw
  float* h_raw = nullptr;         // pinned host staging of a raw image
  HsDevState* d_state = nullptr;
  HsPrecalc* d_pre = nullptr;
  float* d_frameTH = nullptr;
  hs::PointSet ps[2];             // ps[cur]: the committed point state; ps[cur ^ 1]: the commit's gather target
  int cur = 0;
  float *d_u = nullptr, *d_v = nullptr, *d_idepth = nullptr, *d_idepth_zero = nullptr, *d_priorF = nullptr;
  float *d_color = nullptr, *d_weight = nullptr;
  int *d_res_of_slot = nullptr, *d_pt_host = nullptr, *d_host_pt_begin = nullptr;
  int8_t* d_res_order = nullptr;
  uint8_t *d_r_state = nullptr, *d_r_active = nullptr;
  float *d_r_energy = nullptr, *d_r_newEnergy = nullptr, *d_r_ewo = nullptr, *d_r_center = nullptr;
  uint8_t* d_p_actmask = nullptr;
  float *d_p_HdiF = nullptr, *d_p_bdSumF = nullptr, *d_p_Hcd = nullptr, *d_p_JpJdF = nullptr;
  float* d_p_step = nullptr;
  // HdiF ping-pong: a linearization reads the previous one's HdiF (fused step) from d_p_HdiF and writes its own into
  // d_p_HdiF_alt, then the two swap; hdif_solved = the buffer the last point step read (the last solve's SC prelude)
  float* d_p_HdiF_alt = nullptr;
  float* hdif_solved = nullptr;
  float* d_fix_relBL = nullptr;      // [nP] maxRelBaseline in / out of hs_ba_fix_linearization
  int* d_fix_nGood = nullptr;        // [nP] numGoodResiduals in / out
  float* d_part = nullptr;       // [nblk][ne][64] block partials of hs_k_lin
  double* d_part_e = nullptr;    // [nblk][4] block energies
  double* d_hostsum = nullptr;   // [nF][ne][64] per-host sums (hs_k_reduce)
  double* d_sys = nullptr;       // [SX] system vector (upper triangle of HA - sc HSC | bA - bSC) + energy,
                                 // sum |idepth|, #points + the diagonal blocks' host-f Schur terms (see SX)
  double* d_sep = nullptr;       // [2][SL] HA | bA, HSC | bSC (granular read-back)
  double* d_sep_aux = nullptr;   // [HS_MAXF][64] the diagonal blocks' host-f Schur terms of the last sep stitch
  double *d_adHost = nullptr, *d_adTarget = nullptr;  // [HS_MAXF^2][64] + the stamp word (HS_ADJ_STAMP)
  float *d_adHostF = nullptr, *d_adTargetF = nullptr;
  unsigned int adj_seq = 0;        // sequence of the last adjoint upload enqueued (hs_k_fix_frames' stamp)
  unsigned int* d_ticket = nullptr;  // [0] hs_k_stitch's retire ticket (zero between launches), [1] the sequence
                                     // of the last adjoint upload on the device (hs_k_fix_frames; HS_ADJ_STAMP)
  double *d_HM = nullptr, *d_bM = nullptr, *d_Nproj = nullptr;
  float* d_xAd = nullptr;
  double* d_x = nullptr;
  double* d_elog = nullptr;
  unsigned int* d_th_hist = nullptr;  // [HS_TH_BINS] threshold select pass-1 histogram (zero between launches)
  unsigned int *d_th_hist2 = nullptr, *d_th_surv = nullptr, *d_th_nsurv = nullptr;  // multi-block pass 2
  float* d_cand = nullptr;  // [nranks][cand_stride] newest-frame energy per point (-1 / NaN = none)
  int cand_stride = 0;
  bool hm_zero = true;      // marginalization prior not set: the solve skips HM
  uint8_t* d_marg = nullptr;     // [nP] marginalization flags (hs_ba_marginalize_points)
  float* d_adHTdelta = nullptr;  // [nF*nF][8] EnergyFunctional::adHTdeltaF for fixLinearizationF
  float* d_le_chunk = nullptr;   // hs_ba_calc_energies: per-chunk sums
  double* d_le_out = nullptr;
  // BA -> tracker hand-off (hs_tracker_set_ref_ba): points with an IN residual into the newest frame, compacted in
  // point order: cu | cv | cid | HdiF, and their count
  float* d_ref_pts = nullptr;
  int* d_ref_n = nullptr;
  // kernel tracing (env HS_KTRACE=1): per-block wall-clock checkpoints of the last iteration
  bool tracing = false;
  long long *d_tr_lin = nullptr, *d_tr_acc = nullptr, *d_tr_solve = nullptr, *d_tr_st = nullptr;

  // two GN iterations captured as one hipGraph (gn_iterations; env HS_GRAPH=1 enables it: measured 60.2 vs 58.8 us
  // per step eager at the 2k headline, so eager launches stay the default): valid while the launch
  // arguments are unchanged (dropped by every structural change / hs_ba_set_marginal_prior) and the HdiF ping-pong is
  // at the parity it was captured at
  hipGraphExec_t gexec = nullptr;
  const float* graph_hdif = nullptr;

  // RCCL
  ncclComm_t comm = nullptr;
  int rank = 0, nranks = 1;
  // the bounded wait of a multi-rank context (wait_stream): a collective that fails or does not finish within
  // comm_timeout_ms aborts the communicator; every later call then returns HS_ERR_RCCL (comm_lost)
  int comm_timeout_ms = 60000;
  bool comm_lost = false;
  std::thread abort_thread;  // ncclCommAbort of a lost communicator (joined by hs_destroy)
  int dbg_stall_ms = 0;  // test hook hs_debug_stall: the next GN loop call's stream stalls before its results
  // the multi-rank exchange (launch_reduce / exchange in hs_ba.cpp): one all-gather per linearization of every
  // rank's system vector + energies into d_gsys [nranks][SL + 3] and of its newest-frame candidates into d_cand.
  // gath_pending: a gather whose sums are formed by the next solve launch (the fused GN loop); gath_th: the
  // threshold select is still to run (block 1 of that launch; single-rank windows below kLin8MinPoints too)
  double* d_gsys = nullptr;
  // gath_th: setNewFrameEnergyTH's select still to run as block 1 of the next solve / combine launch: 1 the one-block
  // select over every candidate (pass 1 in LDS), 2 only pass 3 of the multi-block select (passes 1 and 2 ran in the
  // reduce / stitch launches: large windows, instead of a launch of its own after the stitch)
  bool gath_pending = false;
  int gath_th = 0;
  // in-process rank group (test hook hs_ba_debug_group): the same exchange by device copies between the contexts of
  // one process, driven by hs_ba_group_linearize / hs_ba_group_iterate
  std::vector<hs_ctx*> group;
  int group_stride = 0;
  bool xch_local = false, xch_th = false, xch_defer = false;  // group: a local reduce awaits the exchange
  hipEvent_t ev_xch[2] = {nullptr, nullptr};

  bool multi_rank() const { return comm != nullptr || !group.empty(); }
  // the GN loop call's counters, reset by its first solve launch (reset_it; -1: none pending), and its results,
  // written by hs_k_result into pinned host memory [kLogCap + 2] (one zero-copy write instead of three copies)
  int pending_reset = -1;
  // pinned staging of per-point / per-slot read-backs (hs_ba_fix_linearization, hs_ba_get_point_state), grown on
  // demand (rb_stage)
  unsigned char* h_rb = nullptr;
  size_t h_rb_cap = 0;
  bool rb_pending = false;  // an asynchronous copy from / into h_rb may still be in flight (a call left early)
  hipError_t rb_stage(size_t bytes) {
    if (rb_pending) {  // the last user returned before its stream sync (an error path): drain before reuse
      const hipError_t e = hipStreamSynchronize(stream);
      if (e != hipSuccess) return e;
      rb_pending = false;
    }
    if (bytes <= h_rb_cap) return hipSuccess;
    if (h_rb) (void)hipHostFree(h_rb);
    h_rb = nullptr;
    h_rb_cap = 0;
    const hipError_t e = hipHostMalloc((void**)&h_rb, bytes);
    if (e == hipSuccess) h_rb_cap = bytes;
    return e;
  }
  double* h_res = nullptr;
  double* d_res = nullptr;  // the device view of h_res
  unsigned long long res_seq = 0;  // hs_k_result's done-word sequence (h_res[kLogCap + 2])

  // timings of the last optimize / iterate
  double t_lin = 0, t_acc = 0, t_solve = 0, t_timed = 0, t_wall = 0, t_iters = 0;

  int dim() const { return 4 + 8 * nF; }
  int SL() const { return dim() * dim() + dim(); }  // slot: n x n (upper triangle used) + b
  // the whole raw system vector: SL | 3 energies | the diagonal blocks' host-f Schur terms [nF][64] (folded in by
  // its consumers); what a multi-rank exchange moves
  int SX() const { return SL() + 3 + 64 * nF; }
  double* sysE() const { return d_sys + SL(); }
};

namespace hs {
// hs_ba.cpp
void drop_graph(hs_ctx* c);
int ensure_capacity(hs_ctx* c, int W, int H, int capP, int capBlk);
void bind_point_set(hs_ctx* c);   // d_u ... d_r_center = ps[cur]
int sync_hm(hs_ctx* c);          // HM / bM <- d_HM / d_bM after a device marginalization
int fetch_state(hs_ctx* c);
void compute_projector(hs_ctx* c);
int make_partition(hs_ctx* c);    // blk_begin / nblk / W / lin8 / th_multi from host_pt_begin
int pack_slot(hs_ctx* c, int s);  // image slot s's packed (I, dx, dy) copy from its texels (after every slot write)
int copy_frame_image_device(hs_ctx* c, int frame, const void* d_texels);
int upload_frames(hs_ctx* c);     // adjoints, projector, precalc of c->h_state's frames -> device (async)
int wait_uploads(hs_ctx* c);      // the pinned staging buffers are free for the host again
size_t fstage_bytes();
int cand_stride_for(hs_ctx* c, int nP, int* stride);
size_t stage_bytes(int capP);     // hs_ba_window.cpp: pinned commit blob for capP points
int marginalize_frame_prior(hs_ctx* c, int frame, std::vector<double>& HMn, std::vector<double>& bMn);
int commit(hs_ctx* c);            // hs_ba_window.cpp: apply pending structural edits (no-op when clean)
inline int commit_if_dirty(hs_ctx* c) { return c->dirty ? commit(c) : HS_OK; }
int max_blocks_for(int capP);
// everything enqueued on the context's stream has finished: hipStreamSynchronize on a single-rank context; on a
// multi-rank one a bounded poll of the stream and the communicator's asynchronous error (HS_ERR_RCCL + abort on a
// failure or after comm_timeout_ms)
int wait_stream(hs_ctx* c);
int comm_fail(hs_ctx* c, const std::string& msg);  // abort the communicator, HS_ERR_RCCL
// HsDevState::status of a finished launch chain -> the C-ABI code (HS_STATUS_STALE first: HS_ERR_STATE)
int status_error(int status);
}  // namespace hs
