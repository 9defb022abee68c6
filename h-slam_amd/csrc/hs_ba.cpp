// hs_ba.cpp — C-ABI implementation (include/hs_ba.h): context, device memory and the
// device-resident GN loop of System::optimize.  The window state (frames, calib, precalc,
// systems, steps) lives in HBM between iterations; one GN iteration is the launch sequence
//   hs_k_solve(SOLVE|APPLY) -> hs_k_lin (fused point step, linearize, per-lane accumulation, block partials)
//   -> hs_k_reduce (per-host fixed-order sums) -> hs_k_stitch (one block per output block of the system,
//   fixed-order sums) -> [multi-rank: one all-gather of the system vectors + candidates; the next solve launch sums
//   them in rank order and selects the threshold in its second block]
// with no host synchronisation and no order-dependent atomics (bit-reproducible).  The host only prepares the window (adjoints, nullspace
// projector, initial precalc — the reference's once-per-window Eigen/Sophus work) and reads
// results back.  Device memory is allocated to capacity once per context (hs_ba_reserve, or the first window that
// needs more); the incremental keyframe API (hs_ba_window.cpp) edits the window in place.  Compiled by hipcc as HIP
// together with hs_ba_kernels.hip; no torch, no Eigen.
#include <algorithm>
#include <chrono>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "hs_ba_ctx.h"

using namespace hs;

namespace hs {
thread_local std::string g_err;  // hs_last_error(), shared by every entry point of the library
}

namespace hs {

void drop_graph(hs_ctx* c) {
  if (c->gexec) (void)hipGraphExecDestroy(c->gexec);
  c->gexec = nullptr;
  c->graph_hdif = nullptr;
}

// upper bound of the linearize blocks of any window of at most capP points (make_partition below): every host's
// points split into blocks of bw * ppw points, ppw chosen so the grid stays near the target; env HS_LIN_PPW forces a
// ppw (more blocks), HS_ACC_EXACT one block per host
int max_blocks_for(int capP) {
  int m = std::max(kLinBlocksTarget, kLin8BlocksTarget) + HS_MAXF;
  if (const char* e = std::getenv("HS_LIN8_BLOCKS")) m = std::max(m, std::atoi(e) + HS_MAXF);
  if (const char* e = std::getenv("HS_LIN_PPW")) {
    const int ppw = std::max(1, std::atoi(e));
    m = std::max(m, capP / (HS_LIN_NW * ppw) + 1 + HS_MAXF);
  }
  return m;
}

static void free_buffers(hs_ctx* c) {
  drop_graph(c);
  std::vector<void*> ptrs = {
      c->d_img_all, c->d_img3, c->d_raw, c->d_state, c->d_pre, c->d_frameTH, c->d_res_of_slot, c->d_pt_host,
      c->d_host_pt_begin, c->d_res_order, c->d_r_active, c->d_r_energy, c->d_r_newEnergy, c->d_r_ewo,
      c->d_p_actmask, c->d_p_HdiF, c->d_p_bdSumF, c->d_p_Hcd, c->d_p_JpJdF, c->d_p_step, c->d_part, c->d_part_e,
      c->d_hostsum, c->d_sys, c->d_sep, c->d_adHost, c->d_adTarget, c->d_adHostF, c->d_adTargetF, c->d_HM, c->d_bM,
      c->d_Nproj, c->d_xAd, c->d_x, c->d_elog, c->d_cand, c->d_tr_lin, c->d_tr_acc, c->d_tr_solve, c->d_tr_st,
      c->d_marg, c->d_adHTdelta, c->d_p_HdiF_alt, c->d_th_hist, c->d_th_hist2, c->d_th_surv, c->d_th_nsurv,
      c->d_le_chunk, c->d_le_out, c->d_ref_pts, c->d_ref_n, c->d_stage, c->d_gsys, c->d_sep_aux, c->d_ticket};
  for (auto& s : c->ps) {
    for (void* p : {(void*)s.u, (void*)s.v, (void*)s.idepth, (void*)s.idepth_zero, (void*)s.priorF, (void*)s.color,
                    (void*)s.weight, (void*)s.relBL, (void*)s.nGood, (void*)s.r_state, (void*)s.r_center})
      ptrs.push_back(p);
    s = PointSet();
  }
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (c->h_stage) (void)hipHostFree(c->h_stage);
  if (c->h_raw) (void)hipHostFree(c->h_raw);
  c->h_stage = nullptr;
  c->h_stage_cap = 0;
  c->h_raw = nullptr;
  c->d_img_all = nullptr; c->d_img3 = nullptr; c->d_raw = nullptr;
  c->d_state = nullptr; c->d_pre = nullptr; c->d_frameTH = nullptr;
  c->d_res_of_slot = c->d_pt_host = c->d_host_pt_begin = nullptr;
  c->d_res_order = nullptr;
  c->d_r_active = nullptr;
  c->d_r_energy = c->d_r_newEnergy = c->d_r_ewo = nullptr;
  c->d_p_actmask = nullptr;
  c->d_p_HdiF = c->d_p_bdSumF = c->d_p_Hcd = c->d_p_JpJdF = c->d_p_step = nullptr;
  c->d_part = nullptr; c->d_part_e = nullptr; c->d_hostsum = nullptr; c->d_sys = nullptr; c->d_sep = nullptr;
  c->d_adHost = c->d_adTarget = nullptr; c->d_adHostF = c->d_adTargetF = nullptr;
  c->d_HM = c->d_bM = c->d_Nproj = nullptr;
  c->d_xAd = nullptr; c->d_x = nullptr; c->d_elog = nullptr; c->d_cand = nullptr;
  c->d_tr_lin = c->d_tr_acc = c->d_tr_solve = c->d_tr_st = nullptr;
  c->d_marg = nullptr;
  c->d_adHTdelta = nullptr;
  c->d_p_HdiF_alt = nullptr;
  c->hdif_solved = nullptr;
  c->d_th_hist = nullptr;
  c->d_th_hist2 = c->d_th_surv = c->d_th_nsurv = nullptr;
  c->d_le_chunk = nullptr; c->d_le_out = nullptr;
  c->d_ref_pts = nullptr; c->d_ref_n = nullptr;
  c->d_stage = nullptr;
  c->d_gsys = nullptr;
  c->d_sep_aux = nullptr;
  c->d_ticket = nullptr;
  c->gath_pending = false;
  c->gath_th = 0;
  c->d_stage_cap = 0;
  c->cap_P = c->cap_blk = c->cap_W = c->cap_H = c->cap_stride = 0;
  bind_point_set(c);
  c->nF = c->nP = c->nR = 0;
  c->haveSystem = false;
  c->sepValid = false;
}

void bind_point_set(hs_ctx* c) {
  const PointSet& s = c->ps[c->cur];
  c->d_u = s.u; c->d_v = s.v; c->d_idepth = s.idepth; c->d_idepth_zero = s.idepth_zero; c->d_priorF = s.priorF;
  c->d_color = s.color; c->d_weight = s.weight;
  c->d_fix_relBL = s.relBL; c->d_fix_nGood = s.nGood;
  c->d_r_state = s.r_state; c->d_r_center = s.r_center;
}

// the communicator is aborted off the calling thread (ncclCommAbort releases the collectives still spinning on the
// stream, and its frees wait for the device): the call returns HS_ERR_RCCL at once; hs_destroy joins the abort
int comm_fail(hs_ctx* c, const std::string& msg) {
  if (c->comm) {
    ncclComm_t cm = c->comm;
    const int dev = c->device;
    c->comm = nullptr;
    c->abort_thread = std::thread([cm, dev] {
      (void)hipSetDevice(dev);
      (void)ncclCommAbort(cm);
    });
  }
  c->comm_lost = true;
  return fail(HS_ERR_RCCL, msg);
}

int wait_stream(hs_ctx* c) {
  if (!c->comm) {
    if (c->comm_lost) return fail(HS_ERR_RCCL, "communicator aborted by an earlier call");
    HS_HIP(hipStreamSynchronize(c->stream));
    return HS_OK;
  }
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t q = hipStreamQuery(c->stream);
    if (q == hipSuccess) return HS_OK;
    if (q != hipErrorNotReady) return fail(HS_ERR_HIP, std::string("hipStreamQuery: ") + hipGetErrorString(q));
    ncclResult_t ar = ncclSuccess;
    const ncclResult_t r = ncclCommGetAsyncError(c->comm, &ar);
    if (r != ncclSuccess) return comm_fail(c, std::string("ncclCommGetAsyncError: ") + ncclGetErrorString(r));
    if (ar != ncclSuccess && ar != ncclInProgress)
      return comm_fail(c, std::string("collective failed: ") + ncclGetErrorString(ar));
    const auto el = std::chrono::steady_clock::now() - t0;
    if (el > std::chrono::milliseconds(c->comm_timeout_ms))
      return comm_fail(c, "collective did not complete within " + std::to_string(c->comm_timeout_ms) +
                              " ms (a peer rank stalled or died); communicator aborted");
    if (el > std::chrono::microseconds(200)) std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

int status_error(int status) {
  if (status & HS_STATUS_STALE)
    return fail(HS_ERR_STATE, "stale frame adjoints: the stamp of the last upload did not reach the device buffers");
  if (status) return fail(HS_ERR_NONFINITE, "non-finite GN step");
  return HS_OK;
}

// candidate-buffer stride: the same on every rank (max point count over the ranks; one small all-reduce)
int cand_stride_for(hs_ctx* c, int nP, int* stride) {
  int s = nP > 0 ? nP : 1;
  if (!c->group.empty()) {  // in-process group: the stride fixed at hs_ba_debug_group
    if (s > c->group_stride) return fail(HS_ERR_INVALID, "shard exceeds the group's candidate stride");
    s = c->group_stride;
  } else if (c->comm) {
    int* d_tmp = nullptr;
    HS_TRY(dalloc(&d_tmp, 1, c->stream));
    // every step on the context's stream (a null-stream copy would not order against it); h_ctl[6]: pinned scratch
    c->h_ctl[6] = s;
    HS_HIP(hipMemcpyAsync(d_tmp, &c->h_ctl[6], sizeof(int), hipMemcpyHostToDevice, c->stream));
    HS_NCCL(ncclAllReduce(d_tmp, d_tmp, 1, ncclInt, ncclMax, c->comm, c->stream));
    HS_HIP(hipMemcpyAsync(&c->h_ctl[6], d_tmp, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    const int rc = wait_stream(c);
    (void)hipFree(d_tmp);
    if (rc != HS_OK) return rc;
    s = c->h_ctl[6];
  }
  *stride = s;
  return HS_OK;
}

// Every device buffer of a window of up to HS_MAXF frames of W x H and capP points, allocated (zeroed) once.  A
// context keeps its allocation while later windows fit; a window that needs more reallocates (hs_ba_set_window
// only: the incremental API fails instead, hs_ba_reserve sizes it).
int ensure_capacity(hs_ctx* c, int W, int H, int capP, int capBlk) {
  capP = std::max(capP, 1);
  capBlk = std::max(capBlk, 1);
  if (c->d_state && W == c->cap_W && H == c->cap_H && capP <= c->cap_P && capBlk <= c->cap_blk) return HS_OK;
  HS_TRY(wait_stream(c));
  free_buffers(c);
  const size_t npx = (size_t)W * H, P8 = (size_t)capP * 8;
  const int nmax = HS_MAXDIM, SLmax = nmax * nmax + nmax, ne = hs_ne(true), FF = HS_MAXF * HS_MAXF;
  HS_TRY(dalloc(&c->d_img_all, npx * HS_MAXF, c->stream));
  HS_TRY(dalloc(&c->d_img3, npx * HS_MAXF * 3, c->stream));
  c->img_px = npx;
  HS_TRY(dalloc(&c->d_state, 1, c->stream));
  HS_TRY(dalloc(&c->d_pre, FF, c->stream));
  HS_TRY(dalloc(&c->d_frameTH, HS_MAXF, c->stream));
  for (auto& s : c->ps) {
    HS_TRY(dalloc(&s.u, capP, c->stream)); HS_TRY(dalloc(&s.v, capP, c->stream));
    HS_TRY(dalloc(&s.idepth, capP, c->stream)); HS_TRY(dalloc(&s.idepth_zero, capP, c->stream)); HS_TRY(dalloc(&s.priorF, capP, c->stream));
    HS_TRY(dalloc(&s.color, P8, c->stream)); HS_TRY(dalloc(&s.weight, P8, c->stream));
    HS_TRY(dalloc(&s.relBL, capP, c->stream)); HS_TRY(dalloc(&s.nGood, capP, c->stream));
    HS_TRY(dalloc(&s.r_state, P8, c->stream)); HS_TRY(dalloc(&s.r_center, P8 * 3, c->stream));
  }
  c->cur = 0;
  HS_TRY(dalloc(&c->d_res_of_slot, P8, c->stream)); HS_TRY(dalloc(&c->d_res_order, P8, c->stream));
  HS_TRY(dalloc(&c->d_pt_host, capP, c->stream)); HS_TRY(dalloc(&c->d_host_pt_begin, HS_MAXF + 1, c->stream));
  // residual state in the slot layout [point][target slot] (P8 entries; slots without a residual unused)
  HS_TRY(dalloc(&c->d_r_active, P8, c->stream));
  HS_TRY(dalloc(&c->d_r_energy, P8, c->stream)); HS_TRY(dalloc(&c->d_r_newEnergy, P8, c->stream)); HS_TRY(dalloc(&c->d_r_ewo, P8, c->stream));
  HS_TRY(dalloc(&c->d_p_actmask, capP, c->stream)); HS_TRY(dalloc(&c->d_p_HdiF, capP, c->stream)); HS_TRY(dalloc(&c->d_p_bdSumF, capP, c->stream));
  HS_TRY(dalloc(&c->d_p_Hcd, (size_t)capP * 4, c->stream)); HS_TRY(dalloc(&c->d_p_JpJdF, P8 * 8, c->stream));
  HS_TRY(dalloc(&c->d_p_step, capP, c->stream)); HS_TRY(dalloc(&c->d_p_HdiF_alt, capP, c->stream));
  c->hdif_solved = c->d_p_HdiF;
  HS_TRY(dalloc(&c->d_part, (size_t)capBlk * ne * 64, c->stream));
  HS_TRY(dalloc(&c->d_part_e, (size_t)capBlk * 4, c->stream));
  HS_TRY(dalloc(&c->d_hostsum, (size_t)HS_MAXF * ne * 64, c->stream));
  HS_TRY(dalloc(&c->d_sys, (size_t)SLmax + 3 + HS_MAXF * 64, c->stream));
  HS_TRY(dalloc(&c->d_sep, (size_t)2 * SLmax, c->stream));
  HS_TRY(dalloc(&c->d_sep_aux, (size_t)HS_MAXF * 64, c->stream));
  // the adjoints + one stamp word each (HS_ADJ_STAMP: hs_k_fix_frames' upload sequence, checked by their readers)
  HS_TRY(dalloc(&c->d_adHost, FF * 64 + 1, c->stream)); HS_TRY(dalloc(&c->d_adTarget, FF * 64 + 1, c->stream));
  HS_TRY(dalloc(&c->d_adHostF, FF * 64 + 1, c->stream)); HS_TRY(dalloc(&c->d_adTargetF, FF * 64 + 1, c->stream));
  HS_TRY(dalloc(&c->d_HM, (size_t)nmax * nmax, c->stream)); HS_TRY(dalloc(&c->d_bM, nmax, c->stream));
  HS_TRY(dalloc(&c->d_Nproj, (size_t)2 * nmax * HS_NNS, c->stream));
  HS_TRY(dalloc(&c->d_xAd, FF * 8, c->stream)); HS_TRY(dalloc(&c->d_x, nmax, c->stream)); HS_TRY(dalloc(&c->d_elog, kLogCap, c->stream));
  int stride = capP;
  HS_TRY(cand_stride_for(c, capP, &stride));
  c->cap_stride = stride;
  HS_TRY(dalloc(&c->d_cand, (size_t)stride * c->nranks, c->stream));
  HS_HIP(hipMemsetAsync(c->d_cand, 0xff, sizeof(float) * (size_t)stride * c->nranks, c->stream));  // NaN: none
  if (c->multi_rank()) HS_TRY(dalloc(&c->d_gsys, ((size_t)SLmax + 3 + HS_MAXF * 64) * c->nranks, c->stream));
  HS_TRY(dalloc(&c->d_th_hist, HS_TH_BINS, c->stream));
  HS_TRY(dalloc(&c->d_th_hist2, 1024, c->stream));
  HS_TRY(dalloc(&c->d_th_nsurv, 2, c->stream));
  HS_TRY(dalloc(&c->d_th_surv, HS_TH_SURV, c->stream));
  HS_TRY(dalloc(&c->d_marg, capP, c->stream));
  HS_TRY(dalloc(&c->d_adHTdelta, FF * 8 + 4, c->stream));  // + cDeltaF
  HS_TRY(dalloc(&c->d_le_chunk, (size_t)(capP + 49) / 50, c->stream));
  HS_TRY(dalloc(&c->d_le_out, 1, c->stream));
  HS_TRY(dalloc(&c->d_ref_pts, (size_t)4 * capP, c->stream));
  HS_TRY(dalloc(&c->d_ref_n, 1, c->stream));
  HS_TRY(dalloc(&c->d_ticket, 2, c->stream));  // [0] the stitch's retire ticket, [1] the adjoint expectation
  // incremental window: the commit blob (pinned + device) and a raw level-0 image's staging
  c->h_stage_cap = c->d_stage_cap = stage_bytes(capP);
  HS_HIP(hipHostMalloc((void**)&c->h_stage, c->h_stage_cap));
  HS_TRY(dalloc(&c->d_stage, c->d_stage_cap, c->stream));
  HS_HIP(hipHostMalloc((void**)&c->h_raw, sizeof(float) * npx));
  HS_TRY(dalloc(&c->d_raw, npx, c->stream));
  const char* tr = std::getenv("HS_KTRACE");
  c->tracing = tr && tr[0] == '1';
  if (c->tracing) {
    HS_TRY(dalloc(&c->d_tr_lin, (size_t)capBlk * 16, c->stream));
    HS_TRY(dalloc(&c->d_tr_acc, (size_t)(HS_MAXF * ((ne * 64 + 255) / 256) + 1 + 64) * 16, c->stream));
    HS_TRY(dalloc(&c->d_tr_st, (size_t)(HS_MAXF * (HS_MAXF + 1) / 2 + 2 * HS_MAXF + 2 + 64) * 16, c->stream));  // + np2 <= 64
    HS_TRY(dalloc(&c->d_tr_solve, 32, c->stream));
  }
  c->cap_W = W; c->cap_H = H; c->cap_P = capP; c->cap_blk = capBlk;
  bind_point_set(c);
  return HS_OK;
}

// ---------------------------------------------------------------- window preparation (host, once per window)
void compute_projector(hs_ctx* c) {
  // System::getNullspaces (pose 6 + scale 1; affine nullspaces are not used by orthogonalize)
  const int n = c->dim();
  const std::vector<FrameH> frames(c->h_state->frames, c->h_state->frames + c->nF);
  std::vector<std::vector<double>> ns;
  for (int i = 0; i < 6; i++) {
    std::vector<double> v(n, 0.0);
    for (const auto& f : frames) {
      for (int k = 0; k < 6; k++) v[4 + f.idx * 8 + k] = f.nullspaces_pose[i][k];
      for (int k = 0; k < 3; k++) v[4 + f.idx * 8 + k] *= SCALE_XI_TRANS_INVERSE;
      for (int k = 3; k < 6; k++) v[4 + f.idx * 8 + k] *= SCALE_XI_ROT_INVERSE;
    }
    ns.push_back(v);
  }
  std::vector<double> v(n, 0.0);
  for (const auto& f : frames) {
    for (int k = 0; k < 6; k++) v[4 + f.idx * 8 + k] = f.nullspaces_scale[k];
    for (int k = 0; k < 3; k++) v[4 + f.idx * 8 + k] *= SCALE_XI_TRANS_INVERSE;
    for (int k = 3; k < 6; k++) v[4 + f.idx * 8 + k] *= SCALE_XI_ROT_INVERSE;
  }
  ns.push_back(v);
  nullspace_projector(ns, n, c->P.solverModeDelta, c->Porth, &c->Nproj);
}

// the device state -> h_state.  After an optimize tail (hs_k_fix_frames) the newest frame's setStateZero nullspaces
// (Include/Frame.h:166-190) are recomputed here on the host; the projector built from them is left to the next
// solve launch (proj_stale) -- a window edit re-uploads every frame (upload_frames) and builds it anyway.
int fetch_state(hs_ctx* c) {
  HS_HIP(hipMemcpyAsync(c->h_state, c->d_state, sizeof(HsDevState), hipMemcpyDeviceToHost, c->stream));
  if (c->hm_host_stale) {  // the device marginal prior comes along (one sync for both)
    const int n = c->dim();
    c->HM.resize((size_t)n * n);
    c->bM.resize(n);
    HS_HIP(hipMemcpyAsync(c->HM.data(), c->d_HM, sizeof(double) * n * n, hipMemcpyDeviceToHost, c->stream));
    HS_HIP(hipMemcpyAsync(c->bM.data(), c->d_bM, sizeof(double) * n, hipMemcpyDeviceToHost, c->stream));
  }
  HS_TRY(wait_stream(c));
  c->hm_host_stale = false;
  c->h_state_valid = true;
  if (c->tail_pending) {
    c->tail_pending = false;
    FrameH& f = c->h_state->frames[c->nF - 1];
    double sz[10];
    std::memcpy(sz, f.state_zero, sizeof(sz));
    f.setStateZero(sz);
    c->proj_stale = true;
    // the device copy gets the new nullspaces too: a later fetch_state (after a solve) copies the device frame over
    // h_state, and upload_frames / compute_projector would otherwise rebuild the projector from the old ones
    HS_TRY(wait_uploads(c));
    std::memcpy(c->h_fstage, &f, sizeof(FrameH));
    HS_HIP(hipMemcpyAsync(&c->d_state->frames[c->nF - 1], c->h_fstage, sizeof(FrameH), hipMemcpyHostToDevice,
                          c->stream));
    HS_HIP(hipEventRecord(c->ev_upload, c->stream));
  }
  return HS_OK;
}

// the projector of the current frames' nullspaces -> device (before a solve, after an optimize tail)
static int settle_projector(hs_ctx* c) {
  if (c->tail_pending) HS_TRY(fetch_state(c));
  if (!c->proj_stale) return HS_OK;
  compute_projector(c);
  HS_HIP(hipMemcpyAsync(c->d_Nproj, c->Nproj.data(), sizeof(double) * 2 * c->dim() * HS_NNS, hipMemcpyHostToDevice,
                        c->stream));
  HS_TRY(wait_stream(c));
  c->proj_stale = false;
  return HS_OK;
}

// HM / bM <- d_HM / d_bM after hs_ba_marginalize_points updated them on the device
int sync_hm(hs_ctx* c) {
  if (!c->hm_host_stale) return HS_OK;
  const int n = c->dim();
  c->HM.resize((size_t)n * n);
  c->bM.resize(n);
  HS_HIP(hipMemcpyAsync(c->HM.data(), c->d_HM, sizeof(double) * n * n, hipMemcpyDeviceToHost, c->stream));
  HS_HIP(hipMemcpyAsync(c->bM.data(), c->d_bM, sizeof(double) * n, hipMemcpyDeviceToHost, c->stream));
  HS_TRY(wait_stream(c));
  c->hm_host_stale = false;
  return HS_OK;
}

size_t fstage_bytes() {
  const int FF = HS_MAXF * HS_MAXF;
  return FF * sizeof(HsPrecalc) + (size_t)FF * 64 * (2 * sizeof(double) + 2 * sizeof(float)) +
         (size_t)2 * HS_MAXDIM * HS_NNS * sizeof(double);
}

// the stamp of a new adjoint upload (hs_k_fix_frames also writes it to the expectation word, d_ticket[1], which the
// readers compare with: no launch argument carries it, so a captured GN loop graph survives the upload)
static unsigned int next_adj_seq(hs_ctx* c) { return ++c->adj_seq; }

int wait_uploads(hs_ctx* c) {
  HS_HIP(hipEventSynchronize(c->ev_upload));
  return HS_OK;
}

// getNullspaces' projector of the frames in c->h_state (fp64 host algebra), the state and the projector to the
// device (asynchronous copies from the pinned h_state / h_fstage; the event ev_upload marks their completion, the
// host waits on it before it rewrites either), then EnergyFunctional::setAdjointsF + System::setPrecalcValues of
// every frame pair on the device (hs_k_fix_frames, fix = 0).
int upload_frames(hs_ctx* c) {
  const int nF = c->nF, n = c->dim();
  HS_TRY(wait_uploads(c));
  HsDevState& S = *c->h_state;
  S.nF = nF;
  c->tail_pending = false;  // every frame's adjoints, precalc and the projector are rewritten from h_state
  c->proj_stale = false;
  compute_projector(c);
  uint8_t* p = c->h_fstage;
  auto put = [&](void* dst, const void* src, size_t bytes) -> hipError_t {
    std::memcpy(p, src, bytes);
    hipError_t e = hipMemcpyAsync(dst, p, bytes, hipMemcpyHostToDevice, c->stream);
    p += (bytes + 15) & ~(size_t)15;
    return e;
  };
  HS_HIP(hipMemcpyAsync(c->d_state, c->h_state, sizeof(HsDevState), hipMemcpyHostToDevice, c->stream));
  HS_HIP(put(c->d_Nproj, c->Nproj.data(), sizeof(double) * 2 * n * HS_NNS));
  HS_HIP(hipEventRecord(c->ev_upload, c->stream));
  // the pairs' precalc and adjoints on the device from the uploaded state (the expressions of the host forms)
  hipLaunchKernelGGL(hs_k_fix_frames, dim3(1), dim3(64), 0, c->stream, c->d_state, c->d_pre, c->d_adHost,
                     c->d_adTarget, c->d_adHostF, c->d_adTargetF, c->P, 0, next_adj_seq(c), c->d_ticket + 1);
  HS_HIP(hipGetLastError());
  c->h_state_valid = true;
  return HS_OK;
}

// refresh image slot s's packed copy (d_img3) from its float4 texels, on the context's stream: every write of a slot
// (the window upload, hs_ba_set_frame_image / _raw / _device) ends with it
int pack_slot(hs_ctx* c, int s) {
  const long long n = (long long)c->img_px;
  hipLaunchKernelGGL(hs_k_pack_texels, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream, n,
                     c->d_img_all + (size_t)s * c->img_px, c->d_img3 + (size_t)s * c->img_px * 3);
  HS_HIP(hipGetLastError());
  return HS_OK;
}

// hs_k_lin partitioning of the committed window (host_pt_begin).  Production: every host's points are split into
// blocks of HS_LIN_NW waves x ppw points (ppw grows with the window so the grid stays near kLinBlocksTarget blocks;
// env HS_LIN_PPW overrides).  HS_ACC_EXACT=1: one block per host whose wave 0 takes every point in order = the
// single-thread reference's fp32 accumulator sums (no shiftUp emulation: at most 1000 points per host).
int make_partition(hs_ctx* c) {
  const int nF = c->nF, nP = c->nP;
  const char* ex = std::getenv("HS_ACC_EXACT");
  c->exact = ex && ex[0] == '1';
  c->ne = hs_ne(c->exact);
  c->Q = (c->ne * 64 + 255) / 256;
  c->blk_begin.assign(nF + 1, 0);
  c->lin8 = !c->exact && nP >= kLin8MinPoints;
  if (const char* e = std::getenv("HS_LIN8")) c->lin8 = !c->exact && e[0] == '1';
  c->lin8 = c->lin8 && lin8_supported(c->cap_W, c->cap_H);  // its 32-bit tap offsets
  // the extra launch of pass 3 costs more than a one-block scan of a small window's candidates
  c->th_multi = nP >= kThMultiMinPoints;
  if (const char* e = std::getenv("HS_TH_MULTI")) c->th_multi = e[0] == '1';
  // points per block: hs_k_lin HS_LIN_NW waves x ppw points; hs_k_lin8 HS_LIN8_NT / 64 = 8 waves x ppw groups of 8
  // points (its partition also serves hs_k_lin's marginalization / linearizeAll(true) passes, with W = 8 waves)
  const int bw = c->lin8 ? (HS_LIN8_NT / 64) * 8 : HS_LIN_NW;
  int target = c->lin8 ? kLin8BlocksTarget : kLinBlocksTarget;
  if (const char* e = std::getenv("HS_LIN8_BLOCKS"); e && c->lin8) target = std::max(1, std::atoi(e));
  int ppw = std::max(1, (nP + bw * target - 1) / (bw * target));
  const char* pe = std::getenv("HS_LIN_PPW");
  if (pe) ppw = std::max(1, std::atoi(pe));
  // hs_k_lin8 with more than one point group per wave: every CU a block.  ceil(nh / (bw ppw)) blocks per host leave
  // CUs idle (200k points: 31 per host, 248 of 256) and rotate the host's image bands over the XCDs from host to host
  // (workgroup w runs on XCD w mod 8); floor(target nh / nP) blocks per host fill the grid (Σ <= target + nF, within
  // the block capacity) and, at 32 per host, give XCD x the same bands q = x mod 8 of every host (its L2 holds them):
  // 200k 160 -> 137 us per launch (hs_k_lin8 round 6)
  const bool fill = c->lin8 && ppw > 1 && !pe && !std::getenv("HS_LIN8_BLOCKS") && !std::getenv("HS_LIN8_NOFILL");
  c->W = c->exact ? 1 : (c->lin8 ? HS_LIN8_NT / 64 : HS_LIN_NW);
  for (int h = 0; h < nF; h++) {
    const int nh = c->host_pt_begin[h + 1] - c->host_pt_begin[h];
    if (c->exact && nh > 1000) return fail(HS_ERR_INVALID, "HS_ACC_EXACT supports at most 1000 points per host");
    int nb = nh == 0 ? 0 : (c->exact ? 1 : (nh + bw * ppw - 1) / (bw * ppw));
    if (fill && nh > 0) nb = std::max(nb, (int)((long long)target * nh / nP));
    c->blk_begin[h + 1] = c->blk_begin[h] + nb;
  }
  c->nblk = c->blk_begin[nF];
  if (c->nblk > c->cap_blk) return fail(HS_ERR_NOMEM, "linearize partition exceeds the block capacity");
  return HS_OK;
}

}  // namespace hs

// ---------------------------------------------------------------- launches (asynchronous)
static size_t lin_lds(const hs_ctx* c) {
  return (size_t)HS_LIN_NW * c->ne * 64 * sizeof(float) + 3 * HS_LIN_NW * sizeof(double);
}

static int launch_linearize(hs_ctx* c, int fuse, bool marg = false, bool accumulate = true, bool fix = false) {
  // a pass without the fused point step reads no HdiF: it writes into the buffer that does not hold the last solve's
  // (efPoint->HdiF stays that of the last accumulateSCF_MT until the next solve: the tail's linearizeAll(true) and a
  // marginalization pass do not change it, and makeCoarseDepthL0 reads it afterwards)
  if (!fuse && c->d_p_HdiF_alt == c->hdif_solved) std::swap(c->d_p_HdiF, c->d_p_HdiF_alt);
  HsLinArgs a;
  std::memset(&a, 0, sizeof(a));
  if (marg) {  // hs_ba_marginalize_points: flags uploaded, adHTdeltaF and cDeltaF formed by hs_k_marg_delta
    a.marg = c->d_marg;
    a.adHTdelta = c->d_adHTdelta;
    a.margPriorFac = c->P.idepthFixPriorMargFac;
  }
  a.img = c->d_img_all;
  a.img3 = c->d_img3;
  a.img_stride = (long long)c->img_px;
  for (int f = 0; f < HS_MAXF; f++) a.img_slot[f] = c->img_slot[f];
  a.st = c->d_state;
  a.lp.huberTH = c->P.huberTH;
  a.lp.outlierTHSumComponent = c->P.outlierTHSumComponent;
  a.lp.affineOptModeA = c->P.affineOptModeA;
  a.lp.affineOptModeB = c->P.affineOptModeB;
  a.nF = c->nF;
  a.write_center = 1;
  a.fuse_step = fuse;
  a.accumulate = accumulate ? 1 : 0;
  for (int i = 0; i <= c->nF; i++) {
    a.host_begin[i] = c->host_pt_begin[i];
    a.blk_begin[i] = c->blk_begin[i];
  }
  for (int i = c->nF + 1; i <= HS_MAXF; i++) {
    a.host_begin[i] = c->nP;
    a.blk_begin[i] = c->nblk;
  }
  a.W = c->W;
  a.pre = c->d_pre;
  a.frameTH = c->d_frameTH;
  a.adHostF = c->d_adHostF;
  a.adTargetF = c->d_adTargetF;
  a.u = c->d_u; a.v = c->d_v; a.idepth = c->d_idepth; a.idepth_zero = c->d_idepth_zero; a.priorF = c->d_priorF;
  a.color = c->d_color; a.weight = c->d_weight;
  a.res_of_slot = c->d_res_of_slot; a.res_order = c->d_res_order;
  a.r_state = c->d_r_state; a.r_active = c->d_r_active; a.r_energy = c->d_r_energy;
  a.r_newEnergy = c->d_r_newEnergy; a.r_ewo = c->d_r_ewo; a.r_center = c->d_r_center;
  a.p_actmask = c->d_p_actmask; a.p_HdiF = c->d_p_HdiF_alt; a.p_HdiF_prev = c->d_p_HdiF;
  a.p_bdSumF = c->d_p_bdSumF; a.p_Hcd = c->d_p_Hcd;
  a.p_JpJdF = c->d_p_JpJdF; a.p_step = c->d_p_step;
  a.fix_relBL = c->d_fix_relBL; a.fix_nGood = c->d_fix_nGood;
  a.newest_cand = c->d_cand + (size_t)c->rank * c->cand_stride;
  // large single-rank windows: hs_k_lin8 counts setNewFrameEnergyTH's pass-1 histogram itself (env HS_LIN8_HIST=0:
  // hs_k_reduce's histogram blocks, as before)
  const char* lh = std::getenv("HS_LIN8_HIST");
  const bool lin_hist = c->lin8 && !marg && !fix && accumulate && c->th_multi && !c->multi_rank() &&
                        !(lh && lh[0] == '0');
  a.th_hist = lin_hist ? c->d_th_hist : nullptr;
  c->hist_in_lin = lin_hist;
  a.part = c->d_part; a.part_e = c->d_part_e;
  a.trace = c->d_tr_lin;
  a.brk = c->brk_active ? 1 : 0;
  if (c->nblk > 0) {
    if (c->lin8 && !marg && !fix) {
      hipLaunchKernelGGL(hs_k_lin8, dim3(c->nblk), dim3(HS_LIN8_NT), 0, c->stream, a);
    } else {
      auto k = marg ? (c->exact ? hs_k_lin_exact_marg : hs_k_lin_marg)
                    : c->exact ? (fix ? hs_k_lin_exact_fix : hs_k_lin_exact)
                    : fix ? hs_k_lin_fix : (fuse && !a.trace) ? hs_k_lin : hs_k_lin_gen;
      hipLaunchKernelGGL(k, dim3(c->nblk), dim3(HS_LIN_NT), lin_lds(c), c->stream, a);
    }
  }
  HS_HIP(hipGetLastError());
  c->tail_valid = fix;  // d_r_active = linearizeAll(true)'s activity: the toRemove list
  std::swap(c->d_p_HdiF, c->d_p_HdiF_alt);
  if (fuse) c->hdif_solved = c->d_p_HdiF_alt;
  if (accumulate) c->sepValid = false;
  return HS_OK;
}

static HsRedArgs red_args(hs_ctx* c, bool skip_threshold) {
  HsRedArgs a;
  std::memset(&a, 0, sizeof(a));
  a.nF = c->nF; a.ne = c->ne; a.Q = c->Q; a.nblk = c->nblk;
  for (int i = 0; i <= c->nF; i++) a.blk_begin[i] = c->blk_begin[i];
  a.part = c->d_part; a.part_e = c->d_part_e; a.hostsum = c->d_hostsum;
  a.sysE = c->sysE();
  a.cand = c->d_cand; a.nranks = c->nranks; a.stride = c->cand_stride;
  a.frameTH = c->d_frameTH; a.newest = c->nF - 1;
  a.frameEnergyTHN = c->P.frameEnergyTHN; a.facMedian = c->P.frameEnergyTHFacMedian;
  a.constWeight = c->P.frameEnergyTHConstWeight; a.overallWeight = c->P.overallEnergyTHWeight;
  a.skip_threshold = skip_threshold ? 1 : 0;
  a.th_hist = c->d_th_hist;
  a.th_hist2 = c->d_th_hist2;
  a.th_surv = c->d_th_surv;
  a.th_nsurv = c->d_th_nsurv;
  // pass-1 histogram blocks / pass-2 blocks of the multi-block select: ~4k candidates each, at most 64
  a.nhist = a.np2 = std::min(64, std::max(1, (c->nranks * c->cand_stride + 4095) / 4096));
  a.trace = c->d_tr_acc;
  return a;
}

static const int* stop_flag(hs_ctx* c) {
  return reinterpret_cast<const int*>((const char*)c->d_state + offsetof(HsDevState, stop));
}

// what a solve launch would have done beside the solve, when none follows: hs_k_combine's block 0 sums the gathered
// systems (multi-rank), block 1 selects the threshold (when it is pending)
static int launch_combine(hs_ctx* c) {
  if (!c->gath_pending && !c->gath_th) return HS_OK;
  HsSolveArgs a;
  std::memset(&a, 0, sizeof(a));
  a.nF = c->nF;
  if (c->gath_pending) {
    a.gsys = c->d_gsys; a.nranks = c->nranks; a.gstride = c->SX(); a.sys_out = c->d_sys;
  }
  a.th_local = c->gath_th;
  a.th = red_args(c, false);
  hipLaunchKernelGGL(hs_k_combine, dim3(c->gath_th ? 2 : 1), dim3(HS_SOLVE_NT), 0, c->stream, a);
  HS_HIP(hipGetLastError());
  c->gath_pending = false;
  c->gath_th = 0;
  return HS_OK;
}

// after the exchange: large windows run the multi-block select over the gathered candidates now (three launches:
// a 1-block select over 10^5..10^6 candidates would outlast the solve beside it); then either the sums are left to
// the next solve launch (defer, the fused GN loop) or hs_k_combine forms them now
static int post_exchange(hs_ctx* c, bool th, bool defer) {
  c->gath_th = th ? 1 : 0;
  c->gath_pending = true;
  if (th && c->th_multi) {
    HsRedArgs a = red_args(c, false);
    a.hist_only = 1;
    hipLaunchKernelGGL(hs_k_reduce, dim3(a.nhist), dim3(256), 0, c->stream, a);
    hipLaunchKernelGGL(hs_k_th_pass2, dim3(a.np2), dim3(HS_STITCH_NT), 0, c->stream, a);
    HS_HIP(hipGetLastError());
    c->gath_th = 2;  // pass 3 as block 1 of the solve / combine launch that follows
  }
  if (!defer) HS_TRY(launch_combine(c));
  return HS_OK;
}

// the one collective of a linearization: every rank's system vector + energies and its candidates, all-gathered in
// one RCCL group (the sums are formed in rank order on every rank, so every rank solves the same system)
static int exchange(hs_ctx* c, bool th) {
  const size_t len = (size_t)c->SX();
  HS_NCCL(ncclGroupStart());
  HS_NCCL(ncclAllGather(c->d_sys, c->d_gsys, len, ncclDouble, c->comm, c->stream));
  if (th)
    HS_NCCL(ncclAllGather(c->d_cand + (size_t)c->rank * c->cand_stride, c->d_cand, c->cand_stride, ncclFloat,
                          c->comm, c->stream));
  HS_NCCL(ncclGroupEnd());
  return HS_OK;
}

// per-host sums (+ energy, threshold), stitch; multi-rank: then the exchange.
// readback = true: only the separate HA / HSC of the last linearization (d_sep) are re-formed from its host sums;
// no exchange, the system vector and the energies are left as they are.
// defer (multi-rank, the fused GN loop): the gathered sums and the threshold select run in the next solve launch.
static int launch_reduce(hs_ctx* c, bool skip_threshold = false, bool sep = false, bool readback = false,
                         bool defer = false, unsigned long long res_seq = 0, int res_k = 0) {
  const bool xch = c->multi_rank() && !readback;
  HsRedArgs a = red_args(c, skip_threshold);
  if (c->brk_active) a.stop = stop_flag(c);
  // setNewFrameEnergyTH: windows below kLin8MinPoints (and every multi-rank window) select in block 1 of the next
  // solve launch (or hs_k_combine), beside the solve: the select only feeds the next linearize, and as the stitch
  // launch's last block it outlasted the stitch's blocks by ~1.5 us at 2k.  Large single-rank windows: pass 1 in
  // hs_k_reduce's histogram blocks, pass 2 in the stitch launch, pass 3 after it.
  const bool beside = !skip_threshold && !readback && (xch || !c->th_multi);
  const bool lin_hist = c->hist_in_lin && !readback;  // the linearization counted pass 1 (hs_k_lin8)
  if (!readback) c->hist_in_lin = false;
  a.nhist = (skip_threshold || beside || lin_hist) ? 0 : a.nhist;
  if (lin_hist && skip_threshold)  // counted but not consumed: the histogram must be zero for the next select
    HS_HIP(hipMemsetAsync(c->d_th_hist, 0, sizeof(unsigned int) * HS_TH_BINS, c->stream));
  if (!readback) {
    hipLaunchKernelGGL(hs_k_reduce, dim3(c->nF * c->Q + 1 + a.nhist), dim3(256), 0, c->stream, a);
    HS_HIP(hipGetLastError());
  }
  const bool multi = c->th_multi && !skip_threshold && !readback && !xch;
  if (!multi) {  // pass 2 by np2 extra blocks of the stitch launch, pass 3 by one block after it (multi only)
    a.th_hist2 = nullptr;
    a.np2 = 0;
  }
  HsStitchArgs st;
  std::memset(&st, 0, sizeof(st));
  st.nF = c->nF; st.exact = c->exact ? 1 : 0; st.ne = c->ne;
  st.hostsum = c->d_hostsum; st.adHost = c->d_adHost; st.adTarget = c->d_adTarget;
  st.out = readback ? nullptr : c->d_sys;
  st.sep = sep ? c->d_sep : nullptr;
  st.aux_out = readback ? nullptr : c->d_sys + c->SL() + 3;
  st.aux_sep = sep ? c->d_sep_aux : nullptr;
  st.lambda1 = 1 + 1e-5;       // SOLVER_FIX_LAMBDA (Src/EnergyFunctional.cpp:707-708)
  st.sc = 1.0f / (1 + 1e-5);   // H -= H_sc * (1.0f / (1 + lambda)) (:763)
  st.trace = c->d_tr_st;
  st.red = a;
  st.red.skip_threshold = (skip_threshold || readback || multi || beside) ? 1 : 0;
  // the first nF blocks: the diagonal blocks' host-f Schur terms (hs_ba_kernels.hip stitch_diag_schur)
  const int nS = c->nF + c->nF * (c->nF + 1) / 2 + c->nF + 2 + (multi ? a.np2 : 0);
  if (res_seq) {  // the GN loop call's results by one more block of this launch (hs_ba_iterate's last iteration)
    st.res_out = c->d_res;
    st.res_elog = c->d_elog;
    st.res_st = c->d_state;
    st.res_k = res_k;
    st.res_slot = kLogCap + 1;
    st.res_seq = res_seq;
    st.res_ticket = c->d_ticket;
  }
  st.status = reinterpret_cast<int*>((char*)c->d_state + offsetof(HsDevState, status));
  st.adj_expect = c->d_ticket + 1;
  hipLaunchKernelGGL(hs_k_stitch, dim3(nS), dim3(HS_STITCH_NT), 0, c->stream, st);
  HS_HIP(hipGetLastError());
  if (multi) {  // pass 3: the select over pass 2's histogram and survivors.  It only feeds the next linearize: in the
                // fused GN loop it runs as block 1 of the next solve launch, beside the solve (defer), else as a
                // one-block launch now (env HS_TH_BESIDE=0: always the launch)
    // (not under the device-side break: a launch after the break would rerun pass 3 on the consumed histograms,
    // where hs_k_th_select's own launch returns at entry)
    const char* tb = std::getenv("HS_TH_BESIDE");
    if (defer && !c->brk_active && !(tb && tb[0] == '0')) {
      c->gath_th = 2;
    } else {
      hipLaunchKernelGGL(hs_k_th_select, dim3(1), dim3(HS_STITCH_NT), 0, c->stream, a);
      HS_HIP(hipGetLastError());
    }
  }
  if (sep) c->sepValid = true;
  if (beside && !xch) {
    c->gath_th = 1;
    if (!defer) HS_TRY(launch_combine(c));
  }
  if (xch) {
    if (!c->group.empty()) {  // the group driver exchanges once every member has reduced
      c->xch_local = true;
      c->xch_th = !skip_threshold;
      c->xch_defer = defer;
      return HS_OK;
    }
    HS_TRY(exchange(c, !skip_threshold));
    HS_TRY(post_exchange(c, !skip_threshold, defer));
  }
  return HS_OK;
}

static int launch_solve(hs_ctx* c, int flags, int iteration, bool log) {
  if (c->tail_pending || c->proj_stale) HS_TRY(settle_projector(c));  // the moved newest frame's projector
  HsSolveArgs a;
  std::memset(&a, 0, sizeof(a));
  a.flags = flags;
  a.iteration = iteration;
  a.nF = c->nF;
  a.st = c->d_state;
  a.sys = c->d_sys;
  a.sysE = c->sysE();
  int grid = 1;
  if (c->gath_pending || c->gath_th) {
    if (!(flags & HS_SOLVE)) {
      HS_TRY(launch_combine(c));
    } else {  // the fused GN loop: the gathered sums in the solve's prefetch, the select as block 1 beside it
      if (c->gath_pending) {
        a.sys = c->d_gsys;
        a.gsys = c->d_gsys; a.nranks = c->nranks; a.gstride = c->SX(); a.sys_out = c->d_sys;
      }
      a.th_local = c->gath_th;
      a.th = red_args(c, false);
      grid = c->gath_th ? 2 : 1;
      c->gath_pending = false;
      c->gath_th = 0;
    }
  }
  a.HM = c->hm_zero ? nullptr : c->d_HM;
  a.bM = c->d_bM; a.Nproj = c->d_Nproj;
  a.adHostF = c->d_adHostF; a.adTargetF = c->d_adTargetF;
  a.xAd = c->d_xAd; a.pre = c->d_pre; a.x_out = c->d_x;
  a.energy_log = log ? c->d_elog : nullptr;
  a.aux_sc = (double)(1.0f / (1 + 1e-5));  // hs_k_stitch's sc
  a.reset_it = c->pending_reset;
  c->pending_reset = -1;
  a.trace = c->d_tr_solve;
  a.initialCalibHessian = c->P.initialCalibHessian;
  a.thOptIterations = c->P.thOptIterations;
  a.brk = c->brk_active ? 1 : 0;
  a.minOpt = c->P.minOptIterations;
  a.chk_adj = 1;
  a.adj_expect = c->d_ticket + 1;
  if (const char* e = std::getenv("HS_SOLVE_DBG")) a.dbg = std::atoi(e);
  hipLaunchKernelGGL(hs_k_solve, dim3(grid), dim3(HS_SOLVE_NT), 0, c->stream, a);
  HS_HIP(hipGetLastError());
  c->h_state_valid = false;
  return HS_OK;
}

static int reset_states(hs_ctx* c) {  // PointFrameResidual::resetOOB on every active residual (one launch)
  const int P8 = c->nP * 8;  // slot layout
  if (P8 == 0) return HS_OK;
  hipLaunchKernelGGL(hs_k_reset_res, dim3((P8 + 255) / 256), dim3(256), 0, c->stream, P8, c->d_r_state,
                     c->d_r_active, c->d_r_energy, c->d_r_newEnergy);
  HS_HIP(hipGetLastError());
  return HS_OK;
}

// a full linearizeAll pass from a clean accumulation target (granular API / optimize entry)
static int linearize_pass(hs_ctx* c, bool reset) {
  if (reset) HS_TRY(reset_states(c));
  HS_TRY(launch_linearize(c, 0));
  HS_TRY(launch_reduce(c, false, true));
  c->haveSystem = true;
  return HS_OK;
}

// via_solve: the next solve launch resets them (its kernel argument); else one host-to-device copy (a captured graph
// replays its launches' arguments, so the graph path copies)
static int set_loop_counters(hs_ctx* c, int iteration, bool via_solve = false) {
  if (via_solve) {
    c->pending_reset = iteration;
    return HS_OK;
  }
  c->h_ctl[0] = iteration;  // iteration
  c->h_ctl[1] = 0;          // status
  c->h_ctl[2] = 0;          // log_count
  HS_HIP(hipMemcpyAsync((char*)c->d_state + offsetof(HsDevState, iteration), c->h_ctl, 3 * sizeof(int),
                        hipMemcpyHostToDevice, c->stream));
  return HS_OK;
}

// per-kernel checkpoint summary of the last traced launch (stderr): for every checkpoint the
// min / median / max over blocks of (checkpoint - the block's start) and the launch span, in us
static int dump_one(const char* name, const long long* d, int nblocks, double tick_us, hipStream_t s,
                    long long* first = nullptr, long long* last = nullptr, const std::vector<int>* groups = nullptr) {
  const bool solve = std::string(name) == "solve";
  std::vector<long long> h(solve ? 32 : (size_t)nblocks * 16);  // the solve row has 32 slots (16..25: probes)
  HS_HIP(hipMemcpyAsync(h.data(), d, sizeof(long long) * h.size(), hipMemcpyDeviceToHost, s));
  HS_HIP(hipStreamSynchronize(s));
  long long t0 = -1, t1 = 0;
  for (int b = 0; b < nblocks; b++) {
    if (h[b * 16] == 0) continue;
    t0 = t0 < 0 ? h[b * 16] : std::min(t0, h[b * 16]);
    for (int k = 1; k < 16; k++) t1 = std::max(t1, h[b * 16 + k]);
  }
  std::fprintf(stderr, "[hs trace] %-12s blocks %5d span %8.2f us\n", name, nblocks, t0 < 0 ? 0.0 : (t1 - t0) * tick_us);
  if (first) *first = t0;
  if (last) *last = t1;
  if (solve && h[0] && h[24] && h[25] && h[15] > h[0])  // slots 24/25: shader clock
    std::fprintf(stderr, "[hs trace] %-12s shader clock %.0f MHz\n", name,
                 (double)(h[25] - h[24]) / ((h[15] - h[0]) * tick_us));
  if (std::string(name) == "stitch") {  // per block: start offset and end of the block (us from the first start)
    std::fprintf(stderr, "[hs trace] stitch blocks (start..end us):");
    for (int b = 0; b < nblocks; b++)
      if (h[b * 16] && h[b * 16 + 15])
        std::fprintf(stderr, " %d:%.1f/%.1f/%.1f/%.1f", b, (h[b * 16] - t0) * tick_us,
                     h[b * 16 + 1] ? (h[b * 16 + 1] - t0) * tick_us : -1.0, h[b * 16 + 2] ? (h[b * 16 + 2] - t0) * tick_us : -1.0,
                     (h[b * 16 + 15] - t0) * tick_us);
    std::fprintf(stderr, "\n");
  }
  if (groups && groups->size() > 1) {  // per block group (the linearize launch: per host): start and cp1 spread
    for (size_t gi = 0; gi + 1 < groups->size(); gi++) {
      std::vector<double> st, e1;
      for (int b = (*groups)[gi]; b < (*groups)[gi + 1]; b++)
        if (h[b * 16] && h[b * 16 + 1]) {
          st.push_back((h[b * 16] - t0) * tick_us);
          e1.push_back((h[b * 16 + 1] - t0) * tick_us);
        }
      if (st.empty()) continue;
      std::sort(st.begin(), st.end());
      std::sort(e1.begin(), e1.end());
      std::fprintf(stderr, "[hs trace] %-12s group %zu: %zu blocks, start %.1f..%.1f, cp1 end min %.1f med %.1f max %.1f us\n",
                   name, gi, st.size(), st.front(), st.back(), e1.front(), e1[e1.size() / 2], e1.back());
    }
  }
  for (int k = 1; k < 16; k++) {
    std::vector<double> v;
    for (int b = 0; b < nblocks; b++)
      if (h[b * 16] && h[b * 16 + k]) v.push_back((h[b * 16 + k] - h[b * 16]) * tick_us);
    if (v.empty()) continue;
    std::sort(v.begin(), v.end());
    std::fprintf(stderr, "[hs trace] %-12s cp%-2d n %5zu  min %8.2f  med %8.2f  max %8.2f us (start spread %.2f)\n",
                 name, k, v.size(), v.front(), v[v.size() / 2], v.back(), 0.0);
  }
  return HS_OK;
}

static int dump_traces(hs_ctx* c) {
  int khz = 0;
  HS_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device));
  const double tick_us = khz > 0 ? 1e3 / khz : 0.01;
  long long f[4] = {0, 0, 0, 0}, l[4] = {0, 0, 0, 0};
  HS_TRY(dump_one("solve", c->d_tr_solve, 1, tick_us, c->stream, &f[0], &l[0]));
  {  // in-loop shader-clock stamps of the solve (slots 16..23, cycles after slot 16)
    long long h[32];
    HS_HIP(hipMemcpy(h, c->d_tr_solve, sizeof(h), hipMemcpyDeviceToHost));
    std::fprintf(stderr, "[hs trace] solve kb4 cycles:");
    for (int k = 17; k < 30; k++)
      if (k < 24 || k > 25) std::fprintf(stderr, " s%d=%lld", k, h[k] ? h[k] - h[16] : -1);
    std::fprintf(stderr, "\n");
  }
  HS_TRY(dump_one("linearize", c->d_tr_lin, c->nblk, tick_us, c->stream, &f[1], &l[1], &c->blk_begin));
  HS_TRY(dump_one("reduce", c->d_tr_acc, c->nF * c->Q + 1, tick_us, c->stream, &f[2], &l[2]));
  HS_TRY(dump_one("stitch", c->d_tr_st, c->nF + c->nF * (c->nF + 1) / 2 + c->nF + 2, tick_us, c->stream, &f[3],
                  &l[3]));
  // the last iteration's launch chain on the wall clock: each kernel's first block start -> last checkpoint, and the
  // gap from one kernel's last checkpoint to the next kernel's first block (launch + end-of-kernel release)
  if (f[0] > 0 && f[1] > 0 && f[2] > 0 && f[3] > 0)
    std::fprintf(stderr, "[hs trace] chain us: solve %.2f | gap %.2f | lin %.2f | gap %.2f | reduce %.2f | gap %.2f | "
                 "stitch %.2f\n", (l[0] - f[0]) * tick_us, (f[1] - l[0]) * tick_us, (l[1] - f[1]) * tick_us,
                 (f[2] - l[1]) * tick_us, (l[2] - f[2]) * tick_us, (f[3] - l[2]) * tick_us, (l[3] - f[3]) * tick_us);
  return HS_OK;
}

// K fused GN iterations continuing from the current (stitched) linearization.
// energies_out[k] = energy of the linearization after iteration k.
static int gn_iterations(hs_ctx* c, int it0, int K, bool allow_break, double* energies_out, int* done,
                         double* e0 = nullptr) {
  if (K > kLogCap - 1) return fail(HS_ERR_INVALID, "too many iterations per call");
  int k = 0;
  const int nev = c->events ? std::min(K, kEventIters) : 0;
  const bool all = c->events >= 2;
  // hipGraph replay of iteration pairs: no per-iteration host work (no break test, no events, no tracing, no
  // collectives inside a capture)
  const char* ge = std::getenv("HS_GRAPH");
  const bool graph = (ge && ge[0] == '1') && !allow_break && nev == 0 && !c->tracing && !c->multi_rank() && K >= 2;
  // allow_break on one rank: the break test runs on the device (hs_k_solve), so the K iterations are enqueued with
  // no host round trip between them; launches after the break return at entry.  Multi-rank windows, tracing and
  // HS_HOST_BREAK=1 read canbreak back after every iteration instead.
  const char* hb = std::getenv("HS_HOST_BREAK");
  const bool dev_brk = allow_break && !c->multi_rank() && !c->tracing && !(hb && hb[0] == '1');
  // before any capture: launch_solve must not sync inside one
  if (c->tail_pending || c->proj_stale) HS_TRY(settle_projector(c));
  HS_TRY(set_loop_counters(c, it0, !graph));
  if (graph) {
    if (c->gexec && c->graph_hdif != c->d_p_HdiF) drop_graph(c);
    if (!c->gexec) {
      const float* hd = c->d_p_HdiF;
      float *sv_h = c->d_p_HdiF, *sv_a = c->d_p_HdiF_alt, *sv_s = c->hdif_solved;
      hipGraph_t g = nullptr;
      HS_HIP(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
      int rc = HS_OK;
      for (int q = 0; q < 2 && rc == HS_OK; q++) {
        if ((rc = launch_solve(c, HS_SOLVE | HS_APPLY, -1, true)) != HS_OK) break;
        if ((rc = launch_linearize(c, 1)) != HS_OK) break;
        rc = launch_reduce(c);
      }
      if (rc != HS_OK) {  // leave the stream out of capture mode and the ping-pong as it was
        hipGraph_t partial = nullptr;
        (void)hipStreamEndCapture(c->stream, &partial);
        if (partial) (void)hipGraphDestroy(partial);
        c->d_p_HdiF = sv_h;
        c->d_p_HdiF_alt = sv_a;
        c->hdif_solved = sv_s;
        return rc;
      }
      HS_HIP(hipStreamEndCapture(c->stream, &g));
      const hipError_t ie = hipGraphInstantiate(&c->gexec, g, nullptr, nullptr, 0);
      (void)hipGraphDestroy(g);
      if (ie != hipSuccess) {
        c->gexec = nullptr;
        return fail(HS_ERR_HIP, "hipGraphInstantiate failed");
      }
      c->graph_hdif = hd;  // two linearizations: the ping-pong is back at its parity
    }
    for (; k + 2 <= K; k += 2) HS_HIP(hipGraphLaunch(c->gexec, c->stream));
  }
  c->brk_active = dev_brk;
  // the call's results: written by an extra block of the last iteration's stitch launch when the last iteration is
  // known in advance (no break test) and launched eagerly on one rank, else by hs_k_result after the loop
  const unsigned long long seq = ++c->res_seq;
  const bool fold_res = !allow_break && !c->multi_rank() && k < K;
  for (; k < K; k++) {
    const bool timed = k < nev;
    if (timed && all) HS_HIP(hipEventRecord(c->ev[4 * k + 0], c->stream));
    int rc = launch_solve(c, HS_SOLVE | HS_APPLY, -1, true);
    if (rc == HS_OK && timed) rc = hipEventRecord(c->ev[4 * k + 1], c->stream) == hipSuccess ? HS_OK : HS_ERR_HIP;
    if (rc == HS_OK) rc = launch_linearize(c, 1);
    if (rc == HS_OK && timed) rc = hipEventRecord(c->ev[4 * k + 2], c->stream) == hipSuccess ? HS_OK : HS_ERR_HIP;
    // the next iteration's solve launch sums the gathered systems (multi-rank) and selects the threshold
    const bool last = fold_res && k + 1 == K;
    if (rc == HS_OK)
      rc = launch_reduce(c, false, false, false, (k + 1 < K && !allow_break) || dev_brk, last ? seq : 0, last ? K : 0);
    if (rc == HS_OK && timed && all)
      rc = hipEventRecord(c->ev[4 * k + 3], c->stream) == hipSuccess ? HS_OK : HS_ERR_HIP;
    if (rc != HS_OK) {
      c->brk_active = false;
      return rc == HS_ERR_HIP ? fail(HS_ERR_HIP, "event record failed") : rc;
    }
    if (allow_break && !dev_brk) {
      int cb = 0;
      HS_HIP(hipMemcpyAsync(&c->h_ctl[3], (char*)c->d_state + offsetof(HsDevState, canbreak), sizeof(int),
                            hipMemcpyDeviceToHost, c->stream));
      HS_TRY(wait_stream(c));
      cb = c->h_ctl[3];
      if (cb && it0 + k >= c->P.minOptIterations) {
        k++;
        break;
      }
    }
  }
  c->brk_active = false;
  c->haveSystem = true;
  if (c->pending_reset >= 0) HS_TRY(set_loop_counters(c, it0));  // K == 0: no solve took the reset
  c->pending_reset = -1;
  if (dev_brk) HS_TRY(launch_combine(c));  // the last linearization's deferred threshold select
  // read back: energy log (E of the linearizations consumed by each solve) + the last energy + status, written by
  // one small kernel straight into pinned host memory
  if (c->dbg_stall_ms > 0) {  // test hook hs_debug_stall (one-shot)
    int khz = 0;
    HS_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device));
    const long long ticks = (long long)c->dbg_stall_ms * (khz > 0 ? khz : 100000);
    c->dbg_stall_ms = 0;
    hipLaunchKernelGGL(hs_k_debug_stall, dim3(1), dim3(64), 0, c->stream, ticks);
    HS_HIP(hipGetLastError());
  }
  if (!fold_res) {
    hipLaunchKernelGGL(hs_k_result, dim3(1), dim3(256), 0, c->stream, c->d_elog, k, c->sysE(), c->d_state, c->d_res,
                       dev_brk ? 1 : 0, kLogCap + 1, seq);
    HS_HIP(hipGetLastError());
  }
  // the results are complete once the result kernel's done word shows this call (its release orders them): poll it
  // (bounded) instead of waiting for the stream's end; the synchronize after the bound surfaces any error.  With
  // per-iteration events the event reads below wait for the stream anyway.
  {
    bool seen = false;
    if (nev == 0) {
      const auto t_start = std::chrono::steady_clock::now();
      const unsigned long long* dw = reinterpret_cast<const unsigned long long*>(c->h_res + kLogCap + 2);
      // a multi-rank context leaves the spin after 1 ms for wait_stream's bounded poll of the communicator
      const auto bound = c->comm ? std::chrono::microseconds(1000) : std::chrono::microseconds(2000000);
      for (int spins = 0;; spins++) {
        if (__atomic_load_n(dw, __ATOMIC_ACQUIRE) == seq) {
          seen = true;
          break;
        }
        if ((spins & 1023) == 1023 && std::chrono::steady_clock::now() - t_start > bound) break;
      }
    }
    if (!seen) HS_TRY(wait_stream(c));
  }
  if (dev_brk) {  // launch_linearize swapped the HdiF ping-pong for every launch; the skipped ones wrote nothing
    const int d = (int)c->h_res[kLogCap + 1];
    if ((k - d) & 1) {
      std::swap(c->d_p_HdiF, c->d_p_HdiF_alt);
      c->hdif_solved = c->d_p_HdiF_alt;
    }
    k = d;
  }
  if (e0) *e0 = c->h_res[0];
  std::vector<double> elog(c->h_res, c->h_res + k + 1);
  c->h_ctl[1] = (int)c->h_res[k + 1];
  double tl = 0, ta = 0, ts = 0;
  for (int q = 0; q < std::min(k, nev); q++) {
    float ms;
    HS_HIP(hipEventElapsedTime(&ms, c->ev[4 * q + 1], c->ev[4 * q + 2]));
    tl += ms;
    if (!all) continue;
    HS_HIP(hipEventElapsedTime(&ms, c->ev[4 * q + 0], c->ev[4 * q + 1]));
    ts += ms;
    HS_HIP(hipEventElapsedTime(&ms, c->ev[4 * q + 2], c->ev[4 * q + 3]));
    ta += ms;
  }
  c->t_lin = tl; c->t_acc = ta; c->t_solve = ts; c->t_timed = std::min(k, nev); c->t_iters = k;
  if (c->tracing) HS_TRY(dump_traces(c));
  if (done) *done = k;
  if (energies_out)
    for (int q = 0; q < k; q++) energies_out[q] = elog[q + 1];
  HS_TRY(status_error(c->h_ctl[1]));
  for (int q = 0; q <= k; q++)
    if (!std::isfinite(elog[q])) return fail(HS_ERR_NONFINITE, "non-finite energy (isLost)");
  return HS_OK;
}

// in-process rank group (hs_ba_debug_group): every member has enqueued its local reduce; each member's system vector +
// energies (and candidates) are copied into every member's gather buffers on the receiver's stream after the
// sender's reduce, then every member waits until all copies out of its own buffers are enqueued before it goes on
// (so no member overwrites d_sys / its candidates while a peer still copies them) and finishes like an RCCL rank
static int group_exchange(const std::vector<hs_ctx*>& g) {
  for (hs_ctx* s : g) {
    if (!s->xch_local) return fail(HS_ERR_STATE, "group member without a pending reduce");
    HS_HIP(hipEventRecord(s->ev_xch[0], s->stream));
  }
  for (hs_ctx* r : g) {
    const size_t len = (size_t)r->SX();
    for (hs_ctx* s : g) {
      HS_HIP(hipStreamWaitEvent(r->stream, s->ev_xch[0], 0));
      HS_HIP(hipMemcpyAsync(r->d_gsys + (size_t)s->rank * len, s->d_sys, sizeof(double) * len, hipMemcpyDeviceToDevice,
                            r->stream));
      if (r->xch_th && r != s)
        HS_HIP(hipMemcpyAsync(r->d_cand + (size_t)s->rank * r->cand_stride, s->d_cand + (size_t)s->rank * s->cand_stride,
                              sizeof(float) * r->cand_stride, hipMemcpyDeviceToDevice, r->stream));
    }
    HS_HIP(hipEventRecord(r->ev_xch[1], r->stream));
  }
  for (hs_ctx* s : g)
    for (hs_ctx* r : g)
      if (r != s) HS_HIP(hipStreamWaitEvent(s->stream, r->ev_xch[1], 0));
  for (hs_ctx* r : g) {
    r->xch_local = false;
    HS_TRY(post_exchange(r, r->xch_th, r->xch_defer));
  }
  return HS_OK;
}

// every entry point that needs the device window: pending incremental edits are committed first
static int begin_call(hs_ctx* c) {
  if (!c) return fail(HS_ERR_INVALID, "null context");
  if (c->comm_lost) return fail(HS_ERR_RCCL, "communicator aborted by an earlier call (a peer rank failed)");
  HS_HIP(hipSetDevice(c->device));
  HS_TRY(commit_if_dirty(c));
  if (c->nF == 0) return fail(HS_ERR_STATE, "no window");
  return HS_OK;
}

// ================================================================ C-ABI
extern "C" {

int hs_params_default(hs_params* p) {
  if (!p) return fail(HS_ERR_INVALID, "null params");
  p->huberTH = 9;
  p->outlierTHSumComponent = 50 * 50;
  p->frameEnergyTHN = 0.7f;
  p->frameEnergyTHFacMedian = 1.5;
  p->frameEnergyTHConstWeight = 0.5;
  p->overallEnergyTHWeight = 1;
  p->idepthFixPrior = 50 * 50;
  p->initialCalibHessian = 5e9;
  p->affineOptModeA = 1e12;
  p->affineOptModeB = 1e8;
  p->initialRotPrior = 1e11;
  p->initialTransPrior = 1e10;
  p->initialAffAPrior = 1e14;
  p->initialAffBPrior = 1e14;
  p->solverModeDelta = 0.00001;
  p->thOptIterations = 1.2;
  p->coarseCutoffTH = 20;
  p->minOptIterations = 1;
  p->pad = 0;
  p->outlierTH = 12 * 12;
  p->maxPixSearch = 0.027f;
  p->trace_slackInterval = 1.5f;
  p->trace_stepsize = 1.0f;
  p->trace_minImprovementFactor = 2;
  p->trace_GNThreshold = 0.1f;
  p->trace_extraSlackOnTH = 1.2f;
  p->minTraceTestRadius = 2;
  p->trace_GNIterations = 3;
  p->idepthFixPriorMargFac = 600 * 600;
  p->margWeightFac = 0.5f * 0.5f;
  p->desiredPointDensity = 2000;
  p->minTraceQuality = 3;
  p->minIdepthH_act = 100;
  p->GNItsOnPointActivation = 3;
  p->minGradHistCut = 0.5f;
  p->minGradHistAdd = 7;
  p->gradDownweightPerLevel = 0.75f;
  p->selectDirectionDistribution = 1;
  return HS_OK;
}

const char* hs_last_error(void) { return g_err.c_str(); }

int hs_create(hs_ctx** out, const hs_params* params, int device_id) {
  if (!out) return fail(HS_ERR_INVALID, "null out");
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(HS_ERR_HIP, "no HIP device");
  if (device_id < 0 || device_id >= ndev) return fail(HS_ERR_INVALID, "bad device id");
  hs_ctx* c = new hs_ctx();
  if (params) c->P = *params;
  else hs_params_default(&c->P);
  c->device = device_id;
  const char* ev = std::getenv("HS_EVENT_TIMING");
  c->events = ev ? std::atoi(ev) : 0;
  if (hipSetDevice(device_id) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipHostMalloc((void**)&c->h_state, sizeof(HsDevState)) != hipSuccess ||
      hipHostMalloc((void**)&c->h_ctl, 8 * sizeof(int)) != hipSuccess ||
      hipHostMalloc((void**)&c->h_res, sizeof(double) * (kLogCap + 3), hipHostMallocMapped | hipHostMallocCoherent) !=
          hipSuccess ||
      hipHostGetDevicePointer((void**)&c->d_res, c->h_res, 0) != hipSuccess ||
      hipHostMalloc((void**)&c->h_fstage, fstage_bytes() + 256) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_upload, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_ready, hipEventDisableTiming) != hipSuccess) {
    delete c;
    return fail(HS_ERR_HIP, "stream / pinned allocation failed");
  }
  c->ev.assign(4 * kEventIters, nullptr);
  for (auto& e : c->ev) HS_HIP(hipEventCreate(&e));
  *out = c;
  return HS_OK;
}

void hs_destroy(hs_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->abort_thread.joinable()) c->abort_thread.join();  // an aborted communicator (comm_fail)
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  free_buffers(c);
  if (c->comm) ncclCommDestroy(c->comm);
  for (auto& e : c->ev)
    if (e) (void)hipEventDestroy(e);
  if (c->h_state) (void)hipHostFree(c->h_state);
  if (c->h_ctl) (void)hipHostFree(c->h_ctl);
  if (c->h_res) (void)hipHostFree(c->h_res);
  if (c->h_rb) (void)hipHostFree(c->h_rb);
  if (c->h_fstage) (void)hipHostFree(c->h_fstage);
  if (c->ev_upload) (void)hipEventDestroy(c->ev_upload);
  if (c->ev_ready) (void)hipEventDestroy(c->ev_ready);
  for (auto& e : c->ev_xch)
    if (e) (void)hipEventDestroy(e);
  for (hs_ctx* p : c->group)  // a destroyed member leaves its group (the others can no longer exchange)
    if (p != c) p->group.clear();
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

// every per-window device buffer back to the state of a fresh allocation (zero; candidates NaN) over the first nP
// points, so a reused context runs a new window exactly as a fresh one would
static int zero_window(hs_ctx* c, int nP) {
  hipStream_t s = c->stream;
  const size_t P = (size_t)std::max(nP, 1), P8 = P * 8;
  const int nmax = HS_MAXDIM, SLmax = nmax * nmax + nmax, ne = hs_ne(true), FF = HS_MAXF * HS_MAXF;
  auto z = [&](void* p, size_t bytes) { return hipMemsetAsync(p, 0, bytes, s); };
  for (auto& q : c->ps) {
    HS_HIP(z(q.u, P * 4)); HS_HIP(z(q.v, P * 4)); HS_HIP(z(q.idepth, P * 4)); HS_HIP(z(q.idepth_zero, P * 4));
    HS_HIP(z(q.priorF, P * 4)); HS_HIP(z(q.color, P8 * 4)); HS_HIP(z(q.weight, P8 * 4));
    HS_HIP(z(q.relBL, P * 4)); HS_HIP(z(q.nGood, P * 4)); HS_HIP(z(q.r_state, P8)); HS_HIP(z(q.r_center, P8 * 12));
  }
  HS_HIP(z(c->d_res_of_slot, P8 * 4)); HS_HIP(z(c->d_res_order, P8)); HS_HIP(z(c->d_pt_host, P * 4));
  HS_HIP(z(c->d_r_active, P8)); HS_HIP(z(c->d_r_energy, P8 * 4)); HS_HIP(z(c->d_r_newEnergy, P8 * 4));
  HS_HIP(z(c->d_r_ewo, P8 * 4)); HS_HIP(z(c->d_p_actmask, P)); HS_HIP(z(c->d_p_HdiF, P * 4));
  HS_HIP(z(c->d_p_HdiF_alt, P * 4)); HS_HIP(z(c->d_p_bdSumF, P * 4)); HS_HIP(z(c->d_p_Hcd, P * 16));
  HS_HIP(z(c->d_p_JpJdF, P8 * 32)); HS_HIP(z(c->d_p_step, P * 4)); HS_HIP(z(c->d_marg, P));
  HS_HIP(z(c->d_part, (size_t)c->cap_blk * ne * 64 * 4)); HS_HIP(z(c->d_part_e, (size_t)c->cap_blk * 32));
  HS_HIP(z(c->d_hostsum, (size_t)HS_MAXF * ne * 64 * 8));
  HS_HIP(z(c->d_sys, ((size_t)SLmax + 3 + HS_MAXF * 64) * 8));
  HS_HIP(z(c->d_sep_aux, (size_t)HS_MAXF * 64 * 8));
  HS_HIP(z(c->d_sep, (size_t)2 * SLmax * 8)); HS_HIP(z(c->d_HM, (size_t)nmax * nmax * 8)); HS_HIP(z(c->d_bM, nmax * 8));
  HS_HIP(z(c->d_xAd, FF * 32)); HS_HIP(z(c->d_x, nmax * 8)); HS_HIP(z(c->d_elog, kLogCap * 8));
  HS_HIP(z(c->d_adHTdelta, FF * 32)); HS_HIP(z(c->d_frameTH, HS_MAXF * 4));
  HS_HIP(hipMemsetAsync(c->d_cand, 0xff, sizeof(float) * (size_t)c->cap_stride * c->nranks, s));
  c->hdif_solved = c->d_p_HdiF;
  return HS_OK;
}

int hs_ba_set_window(hs_ctx* c, const hs_camera* cam, int nF, const hs_frame* fr, const float* const* images,
                     const hs_points* pts, const hs_residuals* rs) {
  if (!c || !cam || !fr || !images || !pts || !rs) return fail(HS_ERR_INVALID, "null argument");
  if (nF < 2 || nF > HS_MAXF) return fail(HS_ERR_INVALID, "nF must be in [2, 8]");
  if (cam->width < 8 || cam->height < 8) return fail(HS_ERR_INVALID, "bad camera size");
  if (pts->n < 0 || rs->n < 0) return fail(HS_ERR_INVALID, "negative counts");
  HS_HIP(hipSetDevice(c->device));
  HS_TRY(wait_stream(c));
  drop_graph(c);
  const int nP = pts->n, nR = rs->n;
  // ---- validate and index the residual graph (host)
  std::vector<int> pt_host(pts->host, pts->host + nP);
  for (int i = 0; i < nP; i++)
    if (pt_host[i] < 0 || pt_host[i] >= nF) return fail(HS_ERR_INVALID, "bad point host");
  for (int i = 1; i < nP; i++)
    if (pt_host[i] < pt_host[i - 1]) return fail(HS_ERR_INVALID, "points must be sorted by host");
  std::vector<int> res_of_slot((size_t)nP * 8, -1), res_point(nR), res_target(nR);
  std::vector<int8_t> res_order((size_t)nP * 8, (int8_t)-1);
  std::vector<int> nres(nP, 0);
  int lastp = -1;
  for (int r = 0; r < nR; r++) {
    const int p = rs->point[r], t = rs->target[r];
    if (p < 0 || p >= nP || t < 0 || t >= nF) return fail(HS_ERR_INVALID, "bad residual index");
    if (p < lastp) return fail(HS_ERR_INVALID, "residuals must be grouped by point in point order");
    if (t == pt_host[p]) return fail(HS_ERR_INVALID, "residual target == host");
    if (res_of_slot[(size_t)p * 8 + t] >= 0) return fail(HS_ERR_INVALID, "duplicate (point, target) residual");
    lastp = p;
    res_of_slot[(size_t)p * 8 + t] = r;
    res_order[(size_t)p * 8 + nres[p]] = (int8_t)t;
    res_point[r] = p;
    res_target[r] = t;
    nres[p]++;
  }
  // ---- capacity: reused while the window fits (no per-window allocation)
  int stride = nP;
  HS_TRY(cand_stride_for(c, nP, &stride));
  const int needP = std::max(nP, stride);
  HS_TRY(ensure_capacity(c, cam->width, cam->height, needP, max_blocks_for(needP)));
  c->cam = *cam;
  c->haveCam = true;
  c->incremental = false;
  c->dirty = false;
  c->wframes.clear();
  c->wpts.clear();
  c->staged.clear();
  c->nF = nF;
  c->nP = nP;
  c->nR = nR;
  c->pt_host.swap(pt_host);
  c->res_of_slot.swap(res_of_slot);
  c->res_order.swap(res_order);
  c->res_point.swap(res_point);
  c->res_target.swap(res_target);
  c->host_pt_begin.assign(nF + 1, nP);
  {
    int p = 0;
    for (int h = 0; h < nF; h++) {
      c->host_pt_begin[h] = p;
      while (p < nP && c->pt_host[p] == h) p++;
    }
    c->host_pt_begin[nF] = nP;
  }
  c->cand_stride = stride;
  HS_TRY(make_partition(c));
  for (int f = 0; f < HS_MAXF; f++) c->img_slot[f] = f;
  HS_TRY(zero_window(c, nP));

  // ---- window state: calib (CalibData ctor: setValueScaled, value_zero = value) and frames
  HsDevState& S = *c->h_state;
  std::memset((void*)&S, 0, sizeof(HsDevState));
  CalibH& cal = S.calib;
  cal.W = cam->width;
  cal.H = cam->height;
  double vs[4] = {cam->fx, cam->fy, cam->cx, cam->cy};
  cal.setValueScaled(vs);
  for (int i = 0; i < 4; i++) {
    cal.value_zero[i] = cal.value[i];
    cal.value_minus_value_zero[i] = 0;
    cal.step[i] = 0;
    cal.value_backup[i] = cal.value[i];
  }
  for (int i = 0; i < nF; i++) {
    FrameH& f = S.frames[i];
    f = FrameH();
    f.id = fr[i].id;
    f.idx = i;
    f.ab_exposure = fr[i].ab_exposure;
    f.frameEnergyTH = fr[i].frameEnergyTH;
    f.evalPT = SE3::fromData(fr[i].worldToCam_evalPT);
    f.setState(fr[i].state);
    f.setStateZero(fr[i].state_zero);
    f.takeData(c->P);
  }
  S.dcal = cal.device();
  S.nF = nF;
  const int n = c->dim();
  c->HM.assign((size_t)n * n, 0.0);
  c->bM.assign(n, 0.0);
  c->hm_zero = true;
  c->hm_host_stale = false;
  HS_TRY(upload_frames(c));

  // ---- uploads (the legacy whole-window path: pageable host arrays, synchronous)
  const size_t npx = (size_t)cam->width * cam->height;
  std::vector<float4> tex(npx);
  for (int f = 0; f < nF; f++) {
    const float* src = images[f];
    for (size_t i = 0; i < npx; i++) tex[i] = make_float4(src[3 * i], src[3 * i + 1], src[3 * i + 2], 0.f);
    HS_HIP(hipMemcpyAsync(c->d_img_all + (size_t)f * npx, tex.data(), npx * sizeof(float4), hipMemcpyHostToDevice,
                          c->stream));
    HS_TRY(wait_stream(c));  // tex is reused
    HS_TRY(pack_slot(c, f));
  }
  const size_t P8 = (size_t)nP * 8;
  std::vector<float> prior(nP, 0.f);
  for (int i = 0; i < nP; i++)
    prior[i] = (pts->has_depth_prior && pts->has_depth_prior[i]) ? c->P.idepthFixPrior * 1.0f * 1.0f : 0.f;
  std::vector<float> th(nF);
  for (int i = 0; i < nF; i++) th[i] = S.frames[i].frameEnergyTH;
  // stream-ordered copies from host vectors that live until the synchronize at the end
  std::vector<uint8_t> slot_state;
  HS_HIP(hipMemcpyAsync(c->d_frameTH, th.data(), sizeof(float) * nF, hipMemcpyHostToDevice, c->stream));
  if (nP > 0) {
    HS_HIP(hipMemcpyAsync(c->d_u, pts->u, sizeof(float) * nP, hipMemcpyHostToDevice, c->stream));
    HS_HIP(hipMemcpyAsync(c->d_v, pts->v, sizeof(float) * nP, hipMemcpyHostToDevice, c->stream));
    HS_HIP(hipMemcpyAsync(c->d_idepth, pts->idepth, sizeof(float) * nP, hipMemcpyHostToDevice, c->stream));
    HS_HIP(hipMemcpyAsync(c->d_idepth_zero, pts->idepth_zero, sizeof(float) * nP, hipMemcpyHostToDevice, c->stream));
    HS_HIP(hipMemcpyAsync(c->d_priorF, prior.data(), sizeof(float) * nP, hipMemcpyHostToDevice, c->stream));
    HS_HIP(hipMemcpyAsync(c->d_color, pts->color, sizeof(float) * P8, hipMemcpyHostToDevice, c->stream));
    HS_HIP(hipMemcpyAsync(c->d_weight, pts->weights, sizeof(float) * P8, hipMemcpyHostToDevice, c->stream));
    HS_HIP(hipMemcpyAsync(c->d_res_of_slot, c->res_of_slot.data(), sizeof(int) * P8, hipMemcpyHostToDevice, c->stream));
    HS_HIP(hipMemcpyAsync(c->d_res_order, c->res_order.data(), P8, hipMemcpyHostToDevice, c->stream));
    HS_HIP(hipMemcpyAsync(c->d_pt_host, c->pt_host.data(), sizeof(int) * nP, hipMemcpyHostToDevice, c->stream));
  }
  HS_HIP(hipMemcpyAsync(c->d_host_pt_begin, c->host_pt_begin.data(), sizeof(int) * (nF + 1), hipMemcpyHostToDevice, c->stream));
  if (nR > 0) {
    if (rs->state) {
      slot_state.assign(P8, HS_RES_OOB);
      for (int r = 0; r < nR; r++) slot_state[(size_t)c->res_point[r] * 8 + c->res_target[r]] = rs->state[r];
      HS_HIP(hipMemcpyAsync(c->d_r_state, slot_state.data(), P8, hipMemcpyHostToDevice, c->stream));
    } else {
      HS_TRY(reset_states(c));
    }
  }
  c->pt_handle.resize(nP);
  for (int i = 0; i < nP; i++) c->pt_handle[i] = i;
  HS_TRY(wait_stream(c));
  return HS_OK;
}

int hs_ba_linearize(hs_ctx* c, int reset, double* energy_out) {
  HS_TRY(begin_call(c));
  HS_HIP(hipSetDevice(c->device));
  HS_TRY(linearize_pass(c, reset != 0));
  double e = 0.0;
  HS_HIP(hipMemcpyAsync(&c->h_ctl[4], c->sysE(), sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HS_HIP(hipMemcpyAsync(&c->h_ctl[1], (char*)c->d_state + offsetof(HsDevState, status), sizeof(int),
                        hipMemcpyDeviceToHost, c->stream));
  HS_TRY(wait_stream(c));
  c->rb_pending = false;
  std::memcpy(&e, &c->h_ctl[4], sizeof(double));
  if (energy_out) *energy_out = e;
  if (c->h_ctl[1] & HS_STATUS_STALE) return status_error(c->h_ctl[1]);
  if (!std::isfinite(e)) return fail(HS_ERR_NONFINITE, "non-finite energy (isLost)");
  return HS_OK;
}

int hs_ba_solve_system(hs_ctx* c, int iteration, double* x_out) {
  HS_TRY(begin_call(c));
  if (!c->haveSystem) return fail(HS_ERR_STATE, "hs_ba_linearize must run first");
  HS_HIP(hipSetDevice(c->device));
  HS_HIP(hipMemsetAsync((char*)c->d_state + offsetof(HsDevState, status), 0, sizeof(int), c->stream));
  HS_TRY(launch_solve(c, HS_SOLVE, iteration < 0 ? 0 : iteration, false));
  c->haveSystem = false;
  HsResubArgs ra;
  ra.n = c->nP; ra.nF = c->nF; ra.apply = 0; ra.st = c->d_state;
  ra.host = c->d_pt_host; ra.xAd = c->d_xAd; ra.actmask = c->d_p_actmask; ra.bdSumF = c->d_p_bdSumF;
  ra.HdiF = c->d_p_HdiF; ra.Hcd = c->d_p_Hcd; ra.JpJdF = c->d_p_JpJdF; ra.res_order = c->d_res_order;
  ra.idepth = c->d_idepth; ra.idepth_zero = c->d_idepth_zero; ra.step = c->d_p_step;
  c->hdif_solved = c->d_p_HdiF;
  if (c->nP > 0) hipLaunchKernelGGL(hs_k_resub, dim3((c->nP + 255) / 256), dim3(256), 0, c->stream, ra);
  HS_HIP(hipGetLastError());
  std::vector<double> x(c->dim());
  HS_HIP(hipMemcpyAsync(x.data(), c->d_x, sizeof(double) * x.size(), hipMemcpyDeviceToHost, c->stream));
  HS_HIP(hipMemcpyAsync(&c->h_ctl[1], (char*)c->d_state + offsetof(HsDevState, status), sizeof(int),
                        hipMemcpyDeviceToHost, c->stream));
  HS_TRY(wait_stream(c));
  if (x_out) std::memcpy(x_out, x.data(), sizeof(double) * x.size());
  HS_TRY(status_error(c->h_ctl[1]));
  return HS_OK;
}

int hs_ba_do_step(hs_ctx* c, int* canbreak_out) {
  HS_TRY(begin_call(c));
  HS_HIP(hipSetDevice(c->device));
  if (c->nP > 0)
    hipLaunchKernelGGL(hs_k_apply_step, dim3((c->nP + 255) / 256), dim3(256), 0, c->stream, c->nP, c->d_p_step,
                       c->d_idepth, c->d_idepth_zero);
  HS_HIP(hipGetLastError());
  HS_TRY(launch_solve(c, HS_APPLY, -1, false));
  HS_HIP(hipMemcpyAsync(&c->h_ctl[3], (char*)c->d_state + offsetof(HsDevState, canbreak), sizeof(int),
                        hipMemcpyDeviceToHost, c->stream));
  HS_TRY(wait_stream(c));
  if (canbreak_out) *canbreak_out = c->h_ctl[3] ? 1 : 0;
  return HS_OK;
}

int hs_ba_optimize(hs_ctx* c, int max_iters, int allow_break, double* energies_out, int* iters_done) {
  HS_TRY(begin_call(c));
  if (max_iters < 0) return fail(HS_ERR_INVALID, "max_iters < 0");
  HS_HIP(hipSetDevice(c->device));
  // energies_out holds max_iters + 1 entries (hs_ba.h) whatever the override below runs
  const int cap = max_iters + 1;
  // System::optimize: two sequential overrides, so a 2- or 3-frame window runs 15 iterations
  if (c->nF < 3) max_iters = 20;
  if (c->nF < 4) max_iters = 15;
  auto t0 = std::chrono::steady_clock::now();
  HS_TRY(linearize_pass(c, true));
  int done = 0;
  std::vector<double> e(max_iters + 1, 0.0);
  // e[0]: the energy of the initial linearization (the first logged energy; with no iteration, the current one)
  HS_TRY(gn_iterations(c, 0, max_iters, allow_break != 0, e.data() + 1, &done, &e[0]));
  c->t_wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (energies_out) std::memcpy(energies_out, e.data(), sizeof(double) * std::min(done + 1, cap));
  if (iters_done) *iters_done = done;
  return HS_OK;
}

int hs_ba_iterate(hs_ctx* c, int first_iteration, int n_iters, double* energies_out) {
  HS_TRY(begin_call(c));
  if (!c->haveSystem) return fail(HS_ERR_STATE, "hs_ba_linearize must run first");
  if (n_iters < 0) return fail(HS_ERR_INVALID, "n_iters < 0");
  HS_HIP(hipSetDevice(c->device));
  auto t0 = std::chrono::steady_clock::now();
  int done = 0;
  HS_TRY(gn_iterations(c, first_iteration, n_iters, false, energies_out, &done));
  c->t_wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return HS_OK;
}

// System::optimize's tail (Src/FullSystemOptimize.cpp:498-516): the newest frame's setEvalPT(PRE_worldToCam,
// state with only a / b kept) (Include/Frame.h:213-218), setAdjointsF + setPrecalcValues (host, fp64: the same
// code as hs_ba_set_window), then linearizeAll(true) as one hs_k_lin_fix pass (linearize + applyRes + the per-point
// maxRelBaseline / numGoodResiduals bookkeeping) followed by the usual reduce / stitch (setNewFrameEnergyTH; the
// stitched system is that of the fixed linearization).
int hs_ba_fix_linearization(hs_ctx* c, double* energy_out, uint8_t* drop_out, float* maxRelBaseline,
                            int* numGoodResiduals, float* HdiF_out) {
  HS_TRY(begin_call(c));
  if ((maxRelBaseline == nullptr) != (numGoodResiduals == nullptr))
    return fail(HS_ERR_INVALID, "maxRelBaseline and numGoodResiduals go together");
  HS_HIP(hipSetDevice(c->device));
  const int nP = c->nP;
  // pinned staging of the read-backs: HdiF [nP] floats, then the active flags [nP][8]; one sync for all of them
  HS_HIP(c->rb_stage(sizeof(float) * (size_t)nP + (size_t)nP * 8));
  c->rb_pending = true;  // cleared after the stream sync below; an early return leaves it for the next rb_stage
  float* h_hdif = reinterpret_cast<float*>(c->h_rb);
  unsigned char* h_act = c->h_rb + sizeof(float) * (size_t)nP;
  // HdiF of the last solve, before this pass relinearizes
  if (HdiF_out && nP > 0)
    HS_HIP(hipMemcpyAsync(h_hdif, c->hdif_solved, sizeof(float) * nP, hipMemcpyDeviceToHost, c->stream));
  // the newest frame's setEvalPT + EnergyFunctional::setAdjointsF + setPrecalcValues, on the device (the nullspaces
  // and projector follow on the host when the state is next fetched)
  hipLaunchKernelGGL(hs_k_fix_frames, dim3(1), dim3(64), 0, c->stream, c->d_state, c->d_pre, c->d_adHost,
                     c->d_adTarget, c->d_adHostF, c->d_adTargetF, c->P, 1, next_adj_seq(c), c->d_ticket + 1);
  HS_HIP(hipGetLastError());
  c->h_state_valid = false;
  c->tail_pending = true;
  if (nP > 0) {
    if (maxRelBaseline) {
      HS_HIP(hipMemcpyAsync(c->d_fix_relBL, maxRelBaseline, sizeof(float) * nP, hipMemcpyHostToDevice, c->stream));
      HS_HIP(hipMemcpyAsync(c->d_fix_nGood, numGoodResiduals, sizeof(int) * nP, hipMemcpyHostToDevice, c->stream));
    }  // else: the context's own per-point values (hs_ba_set_window: 0; hs_ba_insert_points: the given seeds)
  }
  // linearizeAll(true): no resetOOB (OOB stays sticky from the GN loop), no point step
  HS_TRY(launch_linearize(c, 0, false, true, true));
  HS_TRY(launch_reduce(c, false, true));
  c->haveSystem = true;
  double e = 0.0;
  HS_HIP(hipMemcpyAsync(&c->h_ctl[4], c->sysE(), sizeof(double), hipMemcpyDeviceToHost, c->stream));
  if (nP > 0 && maxRelBaseline) {
    HS_HIP(hipMemcpyAsync(maxRelBaseline, c->d_fix_relBL, sizeof(float) * nP, hipMemcpyDeviceToHost, c->stream));
    HS_HIP(hipMemcpyAsync(numGoodResiduals, c->d_fix_nGood, sizeof(int) * nP, hipMemcpyDeviceToHost, c->stream));
  }
  const bool want_drop = drop_out && c->nR > 0;
  if (want_drop)
    HS_HIP(hipMemcpyAsync(h_act, c->d_r_active, (size_t)nP * 8, hipMemcpyDeviceToHost, c->stream));
  HS_HIP(hipMemcpyAsync(&c->h_ctl[1], (char*)c->d_state + offsetof(HsDevState, status), sizeof(int),
                        hipMemcpyDeviceToHost, c->stream));
  HS_TRY(wait_stream(c));
  c->rb_pending = false;
  if (c->h_ctl[1] & HS_STATUS_STALE) return status_error(c->h_ctl[1]);
  std::memcpy(&e, &c->h_ctl[4], sizeof(double));
  if (energy_out) *energy_out = e;
  if (HdiF_out && nP > 0) std::memcpy(HdiF_out, h_hdif, sizeof(float) * nP);
  if (want_drop)  // toRemove: every residual not active after applyRes(true)
    for (int r = 0; r < c->nR; r++) drop_out[r] = h_act[(size_t)c->res_point[r] * 8 + c->res_target[r]] ? 0 : 1;
  if (!std::isfinite(e)) return fail(HS_ERR_NONFINITE, "non-finite energy (isLost)");
  return HS_OK;
}

int hs_ba_get_system(hs_ctx* c, int which, double* H, double* b) {
  HS_TRY(begin_call(c));
  if (which < 0 || which > 2) return fail(HS_ERR_INVALID, "which must be 0, 1 or 2");
  if (!c->haveSystem) return fail(HS_ERR_STATE, "no stitched system (linearize first)");
  HS_HIP(hipSetDevice(c->device));
  const int n = c->dim(), nF = c->nF;
  std::vector<double> HH((size_t)n * n, 0.0), bb(n, 0.0);
  if (which == 1) {
    // accumulateLF_MT with no linearized residuals = the priors of stitchDoubleInternal(usePrior)
    HS_TRY(fetch_state(c));
    const HsDevState& S = *c->h_state;
    for (int i = 0; i < 4; i++) {
      HH[i * n + i] += c->P.initialCalibHessian;
      bb[i] += (double)c->P.initialCalibHessian * (double)(float)S.calib.value_minus_value_zero[i];
    }
    for (int h = 0; h < nF; h++)
      for (int i = 0; i < 8; i++) {
        const int j = 4 + 8 * h + i;
        HH[j * n + j] += S.frames[h].prior[i];
        bb[j] += S.frames[h].prior[i] * S.frames[h].delta_prior[i];
      }
  } else {
    // HA | bA (which 0) or HSC | bSC (which 2) of the last linearization, mirrored (the stitch writes the upper
    // triangles: stitchDoubleMT's symmetrization and calib-row copy); this rank's share on a multi-rank window.
    // If the last stitch ran without the separate output (the GN loop), it is re-run on that linearization's
    // host sums (deterministic: the same sums).
    if (!c->sepValid) HS_TRY(launch_reduce(c, true, true, true));
    const int SL = c->SL();
    std::vector<double> sep((size_t)2 * SL);
    HS_HIP(hipMemcpyAsync(sep.data(), c->d_sep, sizeof(double) * sep.size(), hipMemcpyDeviceToHost, c->stream));
    HS_TRY(wait_stream(c));
    if (which == 2) {  // HSC: the diagonal blocks' host-f Schur terms, formed in blocks of their own
      std::vector<double> aux((size_t)64 * nF);
      HS_HIP(hipMemcpy(aux.data(), c->d_sep_aux, sizeof(double) * aux.size(), hipMemcpyDeviceToHost));
      for (int f = 0; f < nF; f++)
        for (int i = 0; i < 8; i++)
          for (int k = i; k < 8; k++) sep[SL + (size_t)(4 + 8 * f + i) * n + 4 + 8 * f + k] += aux[f * 64 + i * 8 + k];
    }
    const double* src = sep.data() + (which == 0 ? 0 : SL);
    for (int r = 0; r < n; r++) {
      for (int q = r; q < n; q++) HH[(size_t)r * n + q] = HH[(size_t)q * n + r] = src[(size_t)r * n + q];
      bb[r] = src[(size_t)n * n + r];
    }
  }
  if (H) std::memcpy(H, HH.data(), sizeof(double) * n * n);
  if (b) std::memcpy(b, bb.data(), sizeof(double) * n);
  return HS_OK;
}

int hs_ba_get_residuals(hs_ctx* c, uint8_t* state, uint8_t* active, float* energy, float* energy_wo, float* JpJdF,
                        float* center) {
  HS_TRY(begin_call(c));
  HS_HIP(hipSetDevice(c->device));
  HS_TRY(wait_stream(c));
  const size_t m = c->nR;
  if (m == 0) return HS_OK;
  // slot layout [point][target] -> residual order
  const size_t P8 = (size_t)c->nP * 8;
  auto slot_of = [&](size_t r) { return (size_t)c->res_point[r] * 8 + c->res_target[r]; };
  std::vector<uint8_t> act(P8);
  HS_HIP(hipMemcpy(act.data(), c->d_r_active, P8, hipMemcpyDeviceToHost));
  if (state) {
    std::vector<uint8_t> v(P8);
    HS_HIP(hipMemcpy(v.data(), c->d_r_state, P8, hipMemcpyDeviceToHost));
    for (size_t r = 0; r < m; r++) state[r] = v[slot_of(r)];
  }
  if (active)
    for (size_t r = 0; r < m; r++) active[r] = act[slot_of(r)];
  for (auto pr : {std::make_pair(energy, c->d_r_energy), std::make_pair(energy_wo, c->d_r_ewo)}) {
    if (!pr.first) continue;
    std::vector<float> v(P8);
    HS_HIP(hipMemcpy(v.data(), pr.second, P8 * 4, hipMemcpyDeviceToHost));
    for (size_t r = 0; r < m; r++) pr.first[r] = v[slot_of(r)];
  }
  if (center) {
    std::vector<float> v(P8 * 3);
    HS_HIP(hipMemcpy(v.data(), c->d_r_center, P8 * 12, hipMemcpyDeviceToHost));
    for (size_t r = 0; r < m; r++)
      for (int i = 0; i < 3; i++) center[r * 3 + i] = v[slot_of(r) * 3 + i];
  }
  if (JpJdF) {
    // slot layout [point][target][8] -> residual order; zero for inactive residuals
    std::vector<float> slot(P8 * 8);
    if (c->nP > 0) HS_HIP(hipMemcpy(slot.data(), c->d_p_JpJdF, slot.size() * 4, hipMemcpyDeviceToHost));
    for (size_t r = 0; r < m; r++)
      for (int i = 0; i < 8; i++) JpJdF[r * 8 + i] = act[slot_of(r)] ? slot[slot_of(r) * 8 + i] : 0.f;
  }
  return HS_OK;
}

int hs_ba_get_points(hs_ctx* c, float* idepth, float* step, float* HdiF, float* bdSumF) {
  HS_TRY(begin_call(c));
  HS_HIP(hipSetDevice(c->device));
  HS_TRY(wait_stream(c));
  const size_t n = c->nP;
  if (n == 0) return HS_OK;
  if (idepth) HS_HIP(hipMemcpy(idepth, c->d_idepth, n * 4, hipMemcpyDeviceToHost));
  if (step) HS_HIP(hipMemcpy(step, c->d_p_step, n * 4, hipMemcpyDeviceToHost));
  if (HdiF) HS_HIP(hipMemcpy(HdiF, c->d_p_HdiF, n * 4, hipMemcpyDeviceToHost));
  if (bdSumF) HS_HIP(hipMemcpy(bdSumF, c->d_p_bdSumF, n * 4, hipMemcpyDeviceToHost));
  return HS_OK;
}

// EnergyFunctional::calcLEnergyF_MT / calcMEnergyF (Src/EnergyFunctional.cpp:277-368), the energies System::optimize
// only evaluates without setting_forceAceptStep (Src/FullSystemOptimize.cpp:337-345,565-572): the frame and calib
// prior terms and calcMEnergyF on the host in fp64 (the deltas of the current state), the points' prior term on
// the device (hs_k_lenergy).
int hs_ba_calc_energies(hs_ctx* c, double* energyL, double* energyM) {
  HS_TRY(begin_call(c));
  HS_HIP(hipSetDevice(c->device));
  HS_TRY(fetch_state(c));
  const HsDevState& S = *c->h_state;
  const int nF = c->nF, n = c->dim();
  double EL = 0.0;
  for (int f = 0; f < nF; f++) {  // delta_prior .* prior . delta_prior
    double s = 0.0;
    for (int i = 0; i < 8; i++) s += S.frames[f].delta_prior[i] * S.frames[f].prior[i] * S.frames[f].delta_prior[i];
    EL += s;
  }
  float cd[4];
  for (int i = 0; i < 4; i++) cd[i] = (float)S.calib.value_minus_value_zero[i];  // cDeltaF
  {
    const float cp = (float)c->P.initialCalibHessian;  // cPriorF
    float s = 0.f;
    for (int i = 0; i < 4; i++) s += cd[i] * cp * cd[i];
    EL += s;
  }
  if (c->nP > 0) {
    // the window holds no linearized residuals (PointFrameResidual::isLinearized is never set on this path), so
    // calcLEnergyPt's residual terms vanish and only the depth priors remain
    hipLaunchKernelGGL(hs_k_lenergy, dim3(1), dim3(256), 0, c->stream, c->nP, c->d_idepth, c->d_idepth_zero,
                       c->d_priorF, c->d_le_chunk, c->d_le_out);
    HS_HIP(hipGetLastError());
    HS_HIP(hipMemcpyAsync(&c->h_ctl[4], c->d_le_out, sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HS_TRY(wait_stream(c));
    double ep = 0.0;
    std::memcpy(&ep, &c->h_ctl[4], sizeof(double));
    EL += ep;
  }
  // calcMEnergyF: delta . (2 bM + HM delta), delta = getStitchedDeltaF (Src/EnergyFunctional.cpp:842-846)
  HS_TRY(sync_hm(c));
  std::vector<double> d(n);
  for (int i = 0; i < 4; i++) d[i] = (double)cd[i];
  for (int f = 0; f < nF; f++)
    for (int i = 0; i < 8; i++) d[4 + 8 * f + i] = S.frames[f].delta[i];
  double EM = 0.0;
  for (int r = 0; r < n; r++) {
    double hd = 0.0;
    for (int k = 0; k < n; k++) hd += c->HM[(size_t)r * n + k] * d[k];
    EM += d[r] * (2 * c->bM[r] + hd);
  }
  if (energyL) *energyL = EL;
  if (energyM) *energyM = EM;
  return HS_OK;
}

int hs_ba_get_frames(hs_ctx* c, double* state, float* energyTH, double* pose7, double* calib4) {
  HS_TRY(begin_call(c));
  HS_HIP(hipSetDevice(c->device));
  HS_TRY(fetch_state(c));
  const HsDevState& S = *c->h_state;
  if (energyTH) HS_HIP(hipMemcpy(energyTH, c->d_frameTH, sizeof(float) * c->nF, hipMemcpyDeviceToHost));
  for (int i = 0; i < c->nF; i++) {
    if (state)
      for (int k = 0; k < 10; k++) state[i * 10 + k] = S.frames[i].state[k];
    if (pose7) S.frames[i].PRE_worldToCam.toData(pose7 + 7 * i);
  }
  if (calib4)
    for (int k = 0; k < 4; k++) calib4[k] = S.calib.value[k];
  return HS_OK;
}

int hs_ba_get_frame_eval(hs_ctx* c, double* evalPT7, double* state_zero) {
  HS_TRY(begin_call(c));
  HS_HIP(hipSetDevice(c->device));
  HS_TRY(fetch_state(c));
  const HsDevState& S = *c->h_state;
  for (int i = 0; i < c->nF; i++) {
    if (evalPT7) S.frames[i].evalPT.toData(evalPT7 + 7 * i);
    if (state_zero)
      for (int k = 0; k < 10; k++) state_zero[i * 10 + k] = S.frames[i].state_zero[k];
  }
  return HS_OK;
}

int hs_ba_set_marginal_prior(hs_ctx* c, const double* HM, const double* bM) {
  HS_TRY(begin_call(c));
  if (!HM || !bM) return fail(HS_ERR_INVALID, "null HM / bM");
  HS_HIP(hipSetDevice(c->device));
  const int n = c->dim();
  c->HM.assign(HM, HM + n * n);
  c->bM.assign(bM, bM + n);
  c->hm_host_stale = false;
  c->hm_zero = std::all_of(c->HM.begin(), c->HM.end(), [](double v) { return v == 0.0; });
  drop_graph(c);  // the solve's arguments depend on hm_zero
  HS_HIP(hipMemcpyAsync(c->d_HM, c->HM.data(), sizeof(double) * n * n, hipMemcpyHostToDevice, c->stream));
  HS_HIP(hipMemcpyAsync(c->d_bM, c->bM.data(), sizeof(double) * n, hipMemcpyHostToDevice, c->stream));
  HS_TRY(wait_stream(c));
  return HS_OK;
}

// System::flagPointsForRemoval's per-point part (Src/Mapping.cpp:280-293) + EnergyFunctional::marginalizePointsF
// (Src/EnergyFunctional.cpp:545-609) for n window points: one marginalization pass of the linearize / accumulate
// kernels over the flagged points (resetOOB, linearize, applyRes, fixLinearizationF, addPoint<2>, SC addPoint(p,
// false)), stitched into M and Msc; HM += margWeightFac (M - Msc), bM likewise.
int hs_ba_marginalize_points(hs_ctx* c, int n, const int* points, double* HM_out, double* bM_out) {
  HS_TRY(begin_call(c));
  if (n < 0 || (n > 0 && !points)) return fail(HS_ERR_INVALID, "bad point list");
  HS_HIP(hipSetDevice(c->device));
  const int nF = c->nF, dim = c->dim();
  std::vector<uint8_t> flag((size_t)std::max(c->nP, 1), 0);
  for (int i = 0; i < n; i++) {
    if (points[i] < 0 || points[i] >= c->nP) return fail(HS_ERR_INVALID, "point index out of range");
    if (flag[points[i]]) return fail(HS_ERR_INVALID, "duplicate point in the marginalization list");
    flag[points[i]] = 1;
  }
  // EnergyFunctional::setDeltaF (Src/EnergyFunctional.cpp:128-152) from the device state, in fp32 (hs_k_marg_delta);
  // the flags through the pinned staging, asynchronous (rb_pending: the next rb_stage waits for the copy)
  HS_HIP(c->rb_stage((size_t)c->nP + 1));
  c->rb_pending = true;
  std::memcpy(c->h_rb, flag.data(), (size_t)c->nP);
  if (c->nP > 0) HS_HIP(hipMemcpyAsync(c->d_marg, c->h_rb, c->nP, hipMemcpyHostToDevice, c->stream));
  const int nd = nF * nF * 8 + 4;
  hipLaunchKernelGGL(hs_k_marg_delta, dim3((nd + 255) / 256), dim3(256), 0, c->stream, c->d_state, c->d_adHostF,
                     c->d_adTargetF, c->d_adHTdelta);
  HS_HIP(hipGetLastError());
  // the pass; setNewFrameEnergyTH is not part of it.  Then HM += w (M - Msc) on the device
  HS_TRY(launch_linearize(c, 0, true));
  HS_TRY(launch_reduce(c, true, true));
  const int nm = dim * dim + dim;
  hipLaunchKernelGGL(hs_k_marg_update, dim3((nm + 255) / 256), dim3(256), 0, c->stream, c->d_sep, c->d_sep_aux,
                     c->d_HM, c->d_bM, nF, c->SL(), (double)c->P.margWeightFac);
  HS_HIP(hipGetLastError());
  // the window's linearization is consumed: the caller drops the points (hs_ba_set_window) and relinearizes
  c->haveSystem = false;
  c->hm_host_stale = true;
  if (c->hm_zero && n > 0) {
    c->hm_zero = false;
    drop_graph(c);  // the solve's arguments depend on hm_zero
  }
  if (HM_out || bM_out) {
    HS_TRY(sync_hm(c));
    c->rb_pending = false;
    if (HM_out) std::memcpy(HM_out, c->HM.data(), sizeof(double) * dim * dim);
    if (bM_out) std::memcpy(bM_out, c->bM.data(), sizeof(double) * dim);
  }
  return HS_OK;
}

// 8x8 inverse: LU with partial pivoting (row swaps recorded), then solve for the identity columns
static bool inverse8(const double* A, double* Ainv) {
  double lu[64];
  int piv[8];
  std::memcpy(lu, A, sizeof(lu));
  for (int k = 0; k < 8; k++) {
    int p = k;
    for (int r = k + 1; r < 8; r++)
      if (std::fabs(lu[r * 8 + k]) > std::fabs(lu[p * 8 + k])) p = r;
    piv[k] = p;
    if (p != k)
      for (int j = 0; j < 8; j++) std::swap(lu[k * 8 + j], lu[p * 8 + j]);
    if (lu[k * 8 + k] == 0.0) return false;
    for (int r = k + 1; r < 8; r++) {
      lu[r * 8 + k] /= lu[k * 8 + k];
      for (int j = k + 1; j < 8; j++) lu[r * 8 + j] -= lu[r * 8 + k] * lu[k * 8 + j];
    }
  }
  for (int col = 0; col < 8; col++) {
    double x[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    x[col] = 1.0;
    for (int k = 0; k < 8; k++) std::swap(x[k], x[piv[k]]);
    for (int r = 1; r < 8; r++)
      for (int j = 0; j < r; j++) x[r] -= lu[r * 8 + j] * x[j];
    for (int r = 7; r >= 0; r--) {
      for (int j = r + 1; j < 8; j++) x[r] -= lu[r * 8 + j] * x[j];
      x[r] /= lu[r * 8 + r];
    }
    for (int r = 0; r < 8; r++) Ainv[r * 8 + col] = x[r];
  }
  return true;
}

}  // extern "C"

// EnergyFunctional::marginalizeFrame (Src/EnergyFunctional.cpp:456-543) on the context's HM / bM: a dense 68x68
// host operation once per marginalized keyframe (not on the GN path).  HMn / bMn: the (dim-8) prior.
int hs::marginalize_frame_prior(hs_ctx* c, int frame, std::vector<double>& HMn, std::vector<double>& bMn) {
  if (!c->h_state_valid) HS_TRY(fetch_state(c));  // (brings a device-updated HM / bM along)
  HS_TRY(sync_hm(c));
  const int od = c->dim(), nd = od - 8, f0 = 4 + 8 * frame;
  std::vector<double> HMc = c->HM, bMc = c->bM;
  if (HMc.size() != (size_t)od * od) HMc.assign((size_t)od * od, 0.0);
  if (bMc.size() != (size_t)od) bMc.assign(od, 0.0);
  // order: every row except the frame's, then the frame's 8 (the reference's move-to-end)
  std::vector<int> ord;
  for (int i = 0; i < od; i++)
    if (i < f0 || i >= f0 + 8) ord.push_back(i);
  for (int i = 0; i < 8; i++) ord.push_back(f0 + i);
  std::vector<double> H((size_t)od * od), b(od);
  for (int r = 0; r < od; r++) {
    b[r] = bMc[ord[r]];
    for (int q = 0; q < od; q++) H[(size_t)r * od + q] = HMc[(size_t)ord[r] * od + ord[q]];
  }
  const hs::FrameH& F = c->h_state->frames[frame];
  for (int i = 0; i < 8; i++) {  // the frame's prior, added here instead of to the active system
    H[(size_t)(nd + i) * od + nd + i] += F.prior[i];
    b[nd + i] += F.prior[i] * F.delta_prior[i];
  }
  std::vector<double> sv(od);
  for (int i = 0; i < od; i++) sv[i] = std::sqrt(std::fabs(H[(size_t)i * od + i]) + 10.0);
  for (int r = 0; r < od; r++) {
    for (int q = 0; q < od; q++) H[(size_t)r * od + q] = (1.0 / sv[r]) * H[(size_t)r * od + q] * (1.0 / sv[q]);
    b[r] = (1.0 / sv[r]) * b[r];
  }
  double hpi[64], hinv[64];
  for (int r = 0; r < 8; r++)
    for (int q = 0; q < 8; q++) hpi[r * 8 + q] = 0.5f * (H[(size_t)(nd + r) * od + nd + q] * 2.0);
  if (!inverse8(hpi, hinv)) return fail(HS_ERR_NONFINITE, "singular frame block in marginalizeFrame");
  for (int i = 0; i < 64; i++) hinv[i] = 0.5f * (hinv[i] * 2.0);
  for (int r = 0; r < nd; r++) {
    double bl[8];  // row r of (bottom-left)^T * hpi
    for (int q = 0; q < 8; q++) {
      double t = 0;
      for (int k = 0; k < 8; k++) t += H[(size_t)(nd + k) * od + r] * hinv[k * 8 + q];
      bl[q] = t;
    }
    for (int q = 0; q < nd; q++) {
      double t = 0;
      for (int k = 0; k < 8; k++) t += bl[k] * H[(size_t)(nd + k) * od + q];
      H[(size_t)r * od + q] -= t;
    }
    double t = 0;
    for (int k = 0; k < 8; k++) t += bl[k] * b[nd + k];
    b[r] -= t;
  }
  HMn.assign((size_t)nd * nd, 0.0);
  bMn.assign(nd, 0.0);
  for (int r = 0; r < nd; r++) {
    bMn[r] = sv[r] * b[r];
    for (int q = 0; q < nd; q++)
      HMn[(size_t)r * nd + q] = 0.5 * (sv[r] * H[(size_t)r * od + q] * sv[q] + sv[q] * H[(size_t)q * od + r] * sv[r]);
  }
  return HS_OK;
}

extern "C" {

int hs_ba_marginalize_frame(hs_ctx* c, int frame, double* HM_out, double* bM_out) {
  if (!c || (c->nF == 0 && !c->dirty)) return fail(HS_ERR_STATE, "no window");
  HS_HIP(hipSetDevice(c->device));
  HS_TRY(commit_if_dirty(c));
  if (frame < 0 || frame >= c->nF) return fail(HS_ERR_INVALID, "frame index out of range");
  if (c->nF < 2) return fail(HS_ERR_INVALID, "cannot marginalize the only frame");
  std::vector<double> HMn, bMn;
  HS_TRY(marginalize_frame_prior(c, frame, HMn, bMn));
  if (HM_out) std::memcpy(HM_out, HMn.data(), sizeof(double) * HMn.size());
  if (bM_out) std::memcpy(bM_out, bMn.data(), sizeof(double) * bMn.size());
  return HS_OK;
}

int hs_ba_get_timings(hs_ctx* c, double* out6) {
  if (!c || !out6) return fail(HS_ERR_INVALID, "null");
  out6[0] = c->t_lin; out6[1] = c->t_acc; out6[2] = c->t_solve; out6[3] = c->t_timed; out6[4] = c->t_wall;
  out6[5] = c->t_iters;
  return HS_OK;
}

int hs_ba_set_event_timing(hs_ctx* c, int mode) {
  if (!c || mode < 0 || mode > 2) return fail(HS_ERR_INVALID, "bad event-timing mode");
  c->events = mode;
  return HS_OK;
}

int hs_ba_get_partition(hs_ctx* c, int* out4) {
  if (!c || !out4) return fail(HS_ERR_INVALID, "null");
  out4[0] = c->lin8 ? 1 : 0;
  out4[1] = c->nblk;
  out4[2] = c->W;
  out4[3] = c->exact ? 1 : 0;
  return HS_OK;
}

int hs_ba_time_linearize(hs_ctx* c, int reps, double* avg_ms) {
  if (!c || !avg_ms || reps < 1) return fail(HS_ERR_INVALID, "bad args");
  HS_TRY(begin_call(c));
  HS_HIP(hipSetDevice(c->device));
  HS_HIP(hipEventRecord(c->ev[0], c->stream));
  for (int k = 0; k < reps; k++) HS_TRY(launch_linearize(c, 0));
  HS_HIP(hipEventRecord(c->ev[1], c->stream));
  if (c->hist_in_lin) {  // no reduce consumes these passes' pass-1 counts: the next select must find it zero
    HS_HIP(hipMemsetAsync(c->d_th_hist, 0, sizeof(unsigned int) * HS_TH_BINS, c->stream));
    c->hist_in_lin = false;
  }
  HS_HIP(hipEventSynchronize(c->ev[1]));
  float ms = 0;
  HS_HIP(hipEventElapsedTime(&ms, c->ev[0], c->ev[1]));
  *avg_ms = ms / reps;
  return HS_OK;
}

// ---- test hook: an in-process rank group on one device (the multi-rank path's exchange without RCCL)
int hs_ba_debug_group(hs_ctx** ctxs, int n, int cand_stride) {
  if (!ctxs || n < 1 || cand_stride < 1) return fail(HS_ERR_INVALID, "bad group args");
  for (int r = 0; r < n; r++) {
    hs_ctx* c = ctxs[r];
    if (!c) return fail(HS_ERR_INVALID, "null group member");
    if (c->nF != 0 || c->d_state) return fail(HS_ERR_STATE, "hs_ba_debug_group must precede the window");
    if (c->comm || !c->group.empty()) return fail(HS_ERR_STATE, "context already has ranks");
    if (c->device != ctxs[0]->device) return fail(HS_ERR_INVALID, "group members on different devices");
  }
  for (int r = 0; r < n; r++) {
    hs_ctx* c = ctxs[r];
    HS_HIP(hipSetDevice(c->device));
    for (auto& e : c->ev_xch) HS_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    c->group.assign(ctxs, ctxs + n);
    c->rank = r;
    c->nranks = n;
    c->group_stride = cand_stride;
  }
  return HS_OK;
}

static int group_members(hs_ctx** ctxs, int n, std::vector<hs_ctx*>& g) {
  if (!ctxs || n < 1 || !ctxs[0] || (int)ctxs[0]->group.size() != n) return fail(HS_ERR_INVALID, "not a rank group");
  g = ctxs[0]->group;
  for (int r = 0; r < n; r++)
    if (ctxs[r] != g[r]) return fail(HS_ERR_INVALID, "contexts out of rank order");
  for (hs_ctx* c : g) HS_TRY(begin_call(c));
  return HS_OK;
}

// hs_ba_linearize over the group (energy_out: the summed energy, every member's)
int hs_ba_group_linearize(hs_ctx** ctxs, int n, int reset, double* energy_out) {
  std::vector<hs_ctx*> g;
  HS_TRY(group_members(ctxs, n, g));
  for (hs_ctx* c : g) {
    HS_HIP(hipSetDevice(c->device));
    if (reset) HS_TRY(reset_states(c));
    HS_TRY(launch_linearize(c, 0));
    HS_TRY(launch_reduce(c, false, true));
    c->haveSystem = true;
  }
  HS_TRY(group_exchange(g));
  double e = 0.0;
  HS_HIP(hipMemcpyAsync(&e, g[0]->sysE(), sizeof(double), hipMemcpyDeviceToHost, g[0]->stream));
  for (hs_ctx* c : g) HS_TRY(wait_stream(c));
  if (energy_out) *energy_out = e;
  return HS_OK;
}

// hs_ba_iterate over the group: the fused GN loop of every member, the exchange once per iteration
int hs_ba_group_iterate(hs_ctx** ctxs, int n, int first_iteration, int n_iters, double* energies_out) {
  std::vector<hs_ctx*> g;
  HS_TRY(group_members(ctxs, n, g));
  if (n_iters < 0 || n_iters > kLogCap - 1) return fail(HS_ERR_INVALID, "bad n_iters");
  for (hs_ctx* c : g) {
    if (!c->haveSystem) return fail(HS_ERR_STATE, "hs_ba_group_linearize must run first");
    HS_TRY(set_loop_counters(c, first_iteration));
  }
  for (int k = 0; k < n_iters; k++) {
    for (hs_ctx* c : g) {
      HS_TRY(launch_solve(c, HS_SOLVE | HS_APPLY, -1, true));
      HS_TRY(launch_linearize(c, 1));
      HS_TRY(launch_reduce(c, false, false, false, k + 1 < n_iters));
    }
    HS_TRY(group_exchange(g));
  }
  std::vector<double> elog(n_iters + 1, 0.0);
  if (n_iters > 0)
    HS_HIP(hipMemcpyAsync(elog.data(), g[0]->d_elog, sizeof(double) * n_iters, hipMemcpyDeviceToHost, g[0]->stream));
  HS_HIP(hipMemcpyAsync(&elog[n_iters], g[0]->sysE(), sizeof(double), hipMemcpyDeviceToHost, g[0]->stream));
  for (hs_ctx* c : g) HS_TRY(wait_stream(c));
  if (energies_out)
    for (int q = 0; q < n_iters; q++) energies_out[q] = elog[q + 1];
  return HS_OK;
}

int hs_comm_get_unique_id(char* id128) {
  if (!id128) return fail(HS_ERR_INVALID, "null");
  ncclUniqueId id;
  HS_NCCL(ncclGetUniqueId(&id));
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  std::memcpy(id128, &id, 128);
  return HS_OK;
}

int hs_comm_init(hs_ctx* c, const char* id128, int rank, int nranks) {
  if (!c || !id128 || nranks < 1 || rank < 0 || rank >= nranks) return fail(HS_ERR_INVALID, "bad comm args");
  if (c->nF != 0) return fail(HS_ERR_STATE, "hs_comm_init must precede hs_ba_set_window");
  if (c->comm) return fail(HS_ERR_STATE, "communicator already initialised");
  HS_HIP(hipSetDevice(c->device));
  ncclUniqueId id;
  std::memcpy(&id, id128, 128);
  HS_NCCL(ncclCommInitRank(&c->comm, nranks, id, rank));
  c->rank = rank;
  c->nranks = nranks;
  return HS_OK;
}

int hs_comm_set_timeout(hs_ctx* c, int timeout_ms) {
  if (!c || timeout_ms < 1) return fail(HS_ERR_INVALID, "bad timeout");
  c->comm_timeout_ms = timeout_ms;
  return HS_OK;
}

int hs_comm_size(hs_ctx* c, int* nranks, int* rank) {
  if (!c || !nranks || !rank) return fail(HS_ERR_INVALID, "null");
  if (!c->comm) {
    *nranks = 1;
    *rank = 0;
    return HS_OK;
  }
  HS_NCCL(ncclCommCount(c->comm, nranks));
  HS_NCCL(ncclCommUserRank(c->comm, rank));
  return HS_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- test hook (not part of include/hs_ba.h)
// Runs hs_k_stitch alone on host-provided per-host sums and adjoints: tests/test_gpu_stitch.py checks it against a
// numpy restatement of the reference's pair-wise stitchDoubleInternal.  hostsum [nF][hs_ne(exact)][64], adH / adT
// [nF*nF][64] (index h + nF t), out [n*n + n], sep [2][n*n + n] (nullable).
// test hook (not in the header): setNewFrameEnergyTH's select on n candidates (hs_k_reduce's histogram blocks +
// the stitch launch's select block; multi > 0: the multi-block pass 2; multi < 0: the multi-rank path's one-block
// select of the solve / combine launches, pass 1 in LDS); th_out = the newest frame's threshold
extern "C" int hs_debug_threshold(const float* cand, int n, float thn, float facMedian, float constWeight,
                                  float overallWeight, int multi, float* th_out) {
  if (n < 1 || !cand || !th_out) return fail(HS_ERR_INVALID, "bad arguments");
  float *d_c = nullptr, *d_th = nullptr;
  unsigned int *d_h = nullptr, *d_h2 = nullptr, *d_surv = nullptr, *d_ns = nullptr;
  double* d_e = nullptr;
  HS_TRY(dalloc(&d_c, n, nullptr)); HS_TRY(dalloc(&d_th, 1, nullptr)); HS_TRY(dalloc(&d_h, HS_TH_BINS, nullptr)); HS_TRY(dalloc(&d_e, 4, nullptr));
  HS_TRY(dalloc(&d_h2, 1024, nullptr)); HS_TRY(dalloc(&d_surv, HS_TH_SURV, nullptr)); HS_TRY(dalloc(&d_ns, 2, nullptr));
  HS_HIP(hipMemcpy(d_c, cand, sizeof(float) * n, hipMemcpyHostToDevice));
  HsRedArgs a;
  std::memset(&a, 0, sizeof(a));
  a.sysE = d_e; a.cand = d_c; a.nranks = 1; a.stride = n; a.frameTH = d_th; a.newest = 0;
  a.frameEnergyTHN = thn; a.facMedian = facMedian; a.constWeight = constWeight; a.overallWeight = overallWeight;
  a.th_hist = d_h;
  a.nhist = std::min(64, std::max(1, (n + 4095) / 4096));
  if (multi < 0) {
    HsSolveArgs sa;
    std::memset(&sa, 0, sizeof(sa));
    sa.th_local = 1;
    sa.th = a;
    hipLaunchKernelGGL(hs_k_combine, dim3(2), dim3(HS_SOLVE_NT), 0, 0, sa);
  } else {
    hipLaunchKernelGGL(hs_k_reduce, dim3(1 + a.nhist), dim3(256), 0, 0, a);
  }
  if (multi > 0) {  // the large-window path: pass 2 over np2 blocks, then pass 3 on their survivor list
    a.th_hist2 = d_h2;
    a.th_surv = d_surv;
    a.th_nsurv = d_ns;
    a.np2 = multi > 1 ? std::min(multi, 64) : std::min(64, std::max(1, (n + 4095) / 4096));
    hipLaunchKernelGGL(hs_k_th_pass2, dim3(a.np2), dim3(HS_STITCH_NT), 0, 0, a);
  }
  if (multi >= 0) hipLaunchKernelGGL(hs_k_th_select, dim3(1), dim3(HS_STITCH_NT), 0, 0, a);
  HS_HIP(hipGetLastError());
  std::vector<unsigned int> hz(HS_TH_BINS), h2(1024), ns(2);
  HS_HIP(hipMemcpy(th_out, d_th, sizeof(float), hipMemcpyDeviceToHost));
  HS_HIP(hipMemcpy(hz.data(), d_h, sizeof(unsigned int) * HS_TH_BINS, hipMemcpyDeviceToHost));
  HS_HIP(hipMemcpy(h2.data(), d_h2, sizeof(unsigned int) * 1024, hipMemcpyDeviceToHost));
  HS_HIP(hipMemcpy(ns.data(), d_ns, sizeof(unsigned int) * 2, hipMemcpyDeviceToHost));
  for (void* p : {(void*)d_c, (void*)d_th, (void*)d_h, (void*)d_e, (void*)d_h2, (void*)d_surv, (void*)d_ns})
    (void)hipFree(p);
  for (unsigned int v : hz)
    if (v) return fail(HS_ERR_STATE, "threshold histogram not re-zeroed");
  for (unsigned int v : h2)
    if (v) return fail(HS_ERR_STATE, "pass-2 histogram not re-zeroed");
  if (ns[0] || ns[1]) return fail(HS_ERR_STATE, "survivor count / overflow word not re-zeroed");
  return HS_OK;
}

// test hook (not in the header): the product SE3 (hs_se3.h) evaluated on the device (on_device = 1, hs_k_debug_se3,
// including the doStep's series exp / product, ops 1 and 6) or by the same header compiled for the host (0: the
// host algebra of setAdjointsF / setPrecalcValues); op and layouts as hs_k_debug_se3.
extern "C" int hs_debug_se3(int on_device, int op, int n, const double* in14, double* out36) {
  if (n < 1 || !in14 || !out36 || op < 0 || op > 7) return fail(HS_ERR_INVALID, "bad arguments");
  if (!on_device) {
    if (op == 1 || op == 6) return fail(HS_ERR_INVALID, "device-only op");
    for (int i = 0; i < n; i++) {
      const double* x = in14 + 14 * i;
      double* o = out36 + 36 * i;
      hs::SE3 r;
      switch (op) {
        case 0: r = hs::SE3::exp(x); r.toData(o); break;
        case 2: hs::SE3::fromData(x).log(o); break;
        case 3: hs::SE3::fromData(x).Adj(o); break;
        case 4: r = hs::SE3::fromData(x) * hs::SE3::fromData(x + 7); r.toData(o); break;
        case 5: r = hs::SE3::fromData(x).inverse(); r.toData(o); break;
        default: hs::SE3::fromData(x).rotationMatrix(o); break;
      }
    }
    return HS_OK;
  }
  double *d_in = nullptr, *d_out = nullptr;
  HS_TRY(dalloc(&d_in, (size_t)14 * n, nullptr));
  HS_TRY(dalloc(&d_out, (size_t)36 * n, nullptr));
  HS_HIP(hipMemcpy(d_in, in14, sizeof(double) * 14 * n, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(hs_k_debug_se3, dim3((n + 63) / 64), dim3(64), 0, 0, op, n, d_in, d_out);
  HS_HIP(hipGetLastError());
  HS_HIP(hipMemcpy(out36, d_out, sizeof(double) * 36 * n, hipMemcpyDeviceToHost));
  (void)hipFree(d_in);
  (void)hipFree(d_out);
  return HS_OK;
}

// test hook (not in the header): hs_k_lin8's range-step-free quotient / square root beside the IEEE ones, out [n][4]
extern "C" int hs_debug_fastmath(int n, const float* a, const float* b, float* out4) {
  if (n < 1 || !a || !b || !out4) return fail(HS_ERR_INVALID, "bad arguments");
  float *d_a = nullptr, *d_b = nullptr, *d_o = nullptr;
  HS_TRY(dalloc(&d_a, (size_t)n, nullptr));
  HS_TRY(dalloc(&d_b, (size_t)n, nullptr));
  HS_TRY(dalloc(&d_o, (size_t)4 * n, nullptr));
  HS_HIP(hipMemcpy(d_a, a, sizeof(float) * n, hipMemcpyHostToDevice));
  HS_HIP(hipMemcpy(d_b, b, sizeof(float) * n, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(hs_k_debug_fastmath, dim3((n + 255) / 256), dim3(256), 0, 0, n, d_a, d_b, d_o);
  HS_HIP(hipGetLastError());
  HS_HIP(hipMemcpy(out4, d_o, sizeof(float) * 4 * n, hipMemcpyDeviceToHost));
  (void)hipFree(d_a);
  (void)hipFree(d_b);
  (void)hipFree(d_o);
  return HS_OK;
}

// test hooks (not in the header): the system vector the ranks all-reduce (SL + 3 doubles: upper triangle of
// HA (1+lambda on the diagonal) - HSC / (1+lambda) in the n x n layout, bA - bSC, energy, sum |idepth|, #points) and
// this rank's newest-frame candidates (cand_stride floats, NaN = none) of the last linearization
// the system vector [SL + 3] as the solve consumes it: the diagonal blocks' host-f Schur terms folded in
// (out(f, f) -= sc aux[f], the solve prefetch's operation); raw = 1: the unfolded [SX] vector as the stitch wrote it
// (what a multi-rank exchange moves)
extern "C" int hs_debug_get_sysvec(hs_ctx* c, double* out, int raw) {
  if (!c || !out || c->nF == 0) return fail(HS_ERR_INVALID, "null / no window");
  const int SL = c->SL(), n = c->dim();
  std::vector<double> v((size_t)c->SX());
  HS_HIP(hipMemcpyAsync(v.data(), c->d_sys, sizeof(double) * v.size(), hipMemcpyDeviceToHost, c->stream));
  HS_TRY(wait_stream(c));
  if (!raw) {
    const double sc = (double)(1.0f / (1 + 1e-5));
    const double* aux = v.data() + SL + 3;
    for (int f = 0; f < c->nF; f++)
      for (int i = 0; i < 8; i++)
        for (int k = i; k < 8; k++) v[(size_t)(4 + 8 * f + i) * n + 4 + 8 * f + k] -= sc * aux[f * 64 + i * 8 + k];
  }
  std::memcpy(out, v.data(), sizeof(double) * (raw ? v.size() : (size_t)SL + 3));
  return HS_OK;
}
extern "C" int hs_debug_get_candidates(hs_ctx* c, float* out, int* stride) {
  if (!c || !stride || c->nF == 0) return fail(HS_ERR_INVALID, "null / no window");
  *stride = c->cand_stride;
  if (out)
    HS_HIP(hipMemcpyAsync(out, c->d_cand + (size_t)c->rank * c->cand_stride, sizeof(float) * c->cand_stride,
                          hipMemcpyDeviceToHost, c->stream));
  HS_TRY(wait_stream(c));
  return HS_OK;
}

extern "C" int hs_debug_stitch(int nF, int exact, const double* hostsum, const double* adH, const double* adT,
                               double* out, double* sep) {
  if (nF < 1 || nF > HS_MAXF || !hostsum || !adH || !adT || !out) return fail(HS_ERR_INVALID, "bad args");
  const int n = 4 + 8 * nF, SL = n * n + n, ne = hs_ne(exact != 0);
  double *dh = nullptr, *da = nullptr, *dt = nullptr, *dout = nullptr, *dsep = nullptr, *dax = nullptr, *dax2 = nullptr;
  HS_TRY(dalloc(&dax, (size_t)nF * 64, nullptr));
  HS_TRY(dalloc(&dax2, (size_t)nF * 64, nullptr));
  HS_TRY(dalloc(&dh, (size_t)nF * ne * 64, nullptr));
  HS_TRY(dalloc(&da, (size_t)nF * nF * 64, nullptr));
  HS_TRY(dalloc(&dt, (size_t)nF * nF * 64, nullptr));
  HS_TRY(dalloc(&dout, (size_t)SL, nullptr));
  HS_TRY(dalloc(&dsep, (size_t)2 * SL, nullptr));
  HS_HIP(hipMemcpy(dh, hostsum, sizeof(double) * nF * ne * 64, hipMemcpyHostToDevice));
  HS_HIP(hipMemcpy(da, adH, sizeof(double) * nF * nF * 64, hipMemcpyHostToDevice));
  HS_HIP(hipMemcpy(dt, adT, sizeof(double) * nF * nF * 64, hipMemcpyHostToDevice));
  HsStitchArgs st;
  std::memset(&st, 0, sizeof(st));
  st.nF = nF; st.exact = exact ? 1 : 0; st.ne = ne;
  st.hostsum = dh; st.adHost = da; st.adTarget = dt; st.out = dout; st.sep = dsep;
  st.aux_out = dax; st.aux_sep = dax2;
  st.lambda1 = 1 + 1e-5;
  st.sc = 1.0f / (1 + 1e-5);
  st.red.skip_threshold = 1;
  hipLaunchKernelGGL(hs_k_stitch, dim3(nF + nF * (nF + 1) / 2 + nF + 2), dim3(HS_STITCH_NT), 0, 0, st);
  HS_HIP(hipGetLastError());
  HS_HIP(hipDeviceSynchronize());
  HS_HIP(hipMemcpy(out, dout, sizeof(double) * SL, hipMemcpyDeviceToHost));
  if (sep) HS_HIP(hipMemcpy(sep, dsep, sizeof(double) * 2 * SL, hipMemcpyDeviceToHost));
  std::vector<double> ax((size_t)nF * 64), ax2((size_t)nF * 64);
  HS_HIP(hipMemcpy(ax.data(), dax, sizeof(double) * ax.size(), hipMemcpyDeviceToHost));
  HS_HIP(hipMemcpy(ax2.data(), dax2, sizeof(double) * ax2.size(), hipMemcpyDeviceToHost));
  for (double* p : {dh, da, dt, dout, dsep, dax, dax2}) (void)hipFree(p);
  // the consumers' fold of the diagonal blocks' host-f Schur terms
  for (int f = 0; f < nF; f++)
    for (int i = 0; i < 8; i++)
      for (int k = i; k < 8; k++) {
        const size_t e = (size_t)(4 + 8 * f + i) * n + 4 + 8 * f + k;
        out[e] -= st.sc * ax[f * 64 + i * 8 + k];
        if (sep) sep[SL + e] += ax2[f * 64 + i * 8 + k];
      }
  return HS_OK;
}

// test hook (not in the header): the failure the adjoint stamp guards against -- a zero fill of the fp64 (which 0) or
// fp32 (which 1) adjoint buffers, stamp included, enqueued on the context's stream after the last upload
extern "C" int hs_debug_stale_adjoints(hs_ctx* c, int which) {
  if (!c || c->nF == 0 || which < 0 || which > 1) return fail(HS_ERR_INVALID, "bad arguments / no window");
  HS_HIP(hipSetDevice(c->device));
  const size_t n = (size_t)HS_ADJ_STAMP + 1;
  if (which == 0) HS_HIP(hipMemsetAsync(c->d_adHost, 0, n * sizeof(double), c->stream));
  else HS_HIP(hipMemsetAsync(c->d_adHostF, 0, n * sizeof(float), c->stream));
  return HS_OK;
}

// test hook (not in the header): the next GN loop call withholds its done word for ms milliseconds -- a kernel that
// spins that long (bounded: it exits by itself) is enqueued after the call's last collective and before its results,
// so the call's wait finds the stream stalled as behind a collective whose peer stopped
extern "C" int hs_debug_stall(hs_ctx* c, int ms) {
  if (!c || ms < 0 || ms > 10000) return fail(HS_ERR_INVALID, "bad arguments");
  c->dbg_stall_ms = ms;
  return HS_OK;
}

// test hook (not in the header, no device work): whether a W x H window may run hs_k_lin8 (lin8_supported)
extern "C" int hs_debug_lin8_supported(int W, int H) { return hs::lin8_supported(W, H) ? 1 : 0; }
