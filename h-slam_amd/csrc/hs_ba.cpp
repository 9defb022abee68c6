// hs_ba.cpp — C-ABI implementation (include/hs_ba.h): context, device memory, the
// GN loop of System::optimize with the hot point/residual work on the GPU and
// the small fp64 68x68 solve on the host (as the reference does with Eigen).
// Compiled by hipcc as HIP (-x hip) together with hs_ba_kernels.hip into
// libhslam_amd.so; no torch, no Eigen.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/hs_ba.h"
#include "hs_host_math.h"
#include "hs_kernels.h"

using namespace hs;

namespace {
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
}  // namespace

#define HS_HIP(x)                                                                              \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) return fail(HS_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

#define HS_NCCL(x)                                                                              \
  do {                                                                                          \
    ncclResult_t r_ = (x);                                                                      \
    if (r_ != ncclSuccess) return fail(HS_ERR_RCCL, std::string(#x) + ": " + ncclGetErrorString(r_)); \
  } while (0)

template <typename T>
static int dalloc(T** p, size_t n) {
  if (n == 0) n = 1;
  HS_HIP(hipMalloc((void**)p, n * sizeof(T)));
  return HS_OK;
}

struct hs_ctx {
  hs_params P;
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev[8];

  // window (host mirror)
  int nF = 0, nP = 0, nR = 0;
  CalibH calib;
  std::vector<FrameH> frames;
  std::vector<int> pt_host;
  std::vector<int> res_of_slot;    // [nP*8]
  std::vector<int8_t> res_order;   // [nP*8]
  std::vector<int> chunk_begin, chunk_host, host_chunk_begin;
  std::vector<double> adHost, adTarget;  // [nF*nF][64]
  std::vector<float> adHostF, adTargetF;
  std::vector<double> HM, bM, Porth;     // marginal prior, nullspace projector
  std::vector<double> HA, bA, HL, bL, HSC, bSC;
  double lastEnergy = 0;
  bool haveSystem = false;
  int chunk_size = 8;

  // device
  float4* d_img[HS_MAXF] = {nullptr};
  HsPrecalc* d_pre = nullptr;
  float* d_frameTH = nullptr;
  float *d_u = nullptr, *d_v = nullptr, *d_idepth = nullptr, *d_idepth_zero = nullptr, *d_priorF = nullptr;
  float *d_color = nullptr, *d_weight = nullptr;
  int* d_res_of_slot = nullptr;
  int8_t* d_res_order = nullptr;
  int *d_chunk_begin = nullptr, *d_chunk_host = nullptr, *d_host_chunk_begin = nullptr, *d_pt_host = nullptr;
  uint8_t *d_r_state = nullptr, *d_r_active = nullptr;
  float *d_r_energy = nullptr, *d_r_newEnergy = nullptr, *d_r_ewo = nullptr, *d_r_JpJdF = nullptr,
        *d_r_center = nullptr;
  float *d_p_HdiF = nullptr, *d_p_bdSumF = nullptr, *d_p_Hcd = nullptr, *d_p_step = nullptr;
  uint8_t* d_p_ngood = nullptr;
  HsWavePartial* d_partials = nullptr;
  HsHostSlab* d_slabs = nullptr;
  double *d_adHost = nullptr, *d_adTarget = nullptr;
  double* d_sys = nullptr;  // HA | bA | HSC | bSC | energy
  double* h_sys = nullptr;  // pinned mirror
  float* d_xAd = nullptr;
  float* h_xAd = nullptr;   // pinned
  HsPrecalc* h_pre = nullptr;  // pinned
  float* d_cand = nullptr;     // [nranks][cand_stride]; this rank writes slot `rank`
  int* d_cnt = nullptr;        // [nranks]
  int cand_stride = 0;
  double* d_stat = nullptr;
  int n_stat_blocks = 0;

  // RCCL
  ncclComm_t comm = nullptr;
  int rank = 0, nranks = 1;

  // timings of the last optimize
  double t_lin = 0, t_stitch = 0, t_resub = 0, t_th = 0, t_wall = 0, t_iters = 0;

  int dim() const { return 4 + 8 * nF; }
  size_t sys_len() const { return (size_t)2 * dim() * dim() + 2 * dim() + 2; }
};

static void free_window(hs_ctx* c) {
  for (int i = 0; i < HS_MAXF; i++) { if (c->d_img[i]) (void)hipFree(c->d_img[i]); c->d_img[i] = nullptr; }
  void* ptrs[] = {c->d_pre, c->d_frameTH, c->d_u, c->d_v, c->d_idepth, c->d_idepth_zero, c->d_priorF, c->d_color,
                  c->d_weight, c->d_res_of_slot, c->d_res_order, c->d_chunk_begin, c->d_chunk_host,
                  c->d_host_chunk_begin, c->d_pt_host, c->d_r_state, c->d_r_active, c->d_r_energy,
                  c->d_r_newEnergy, c->d_r_ewo, c->d_r_JpJdF, c->d_r_center, c->d_p_HdiF, c->d_p_bdSumF,
                  c->d_p_Hcd, c->d_p_step, c->d_p_ngood, c->d_partials, c->d_slabs, c->d_adHost, c->d_adTarget,
                  c->d_sys, c->d_xAd, c->d_cand, c->d_cnt, c->d_stat};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (c->h_sys) (void)hipHostFree(c->h_sys);
  if (c->h_xAd) (void)hipHostFree(c->h_xAd);
  if (c->h_pre) (void)hipHostFree(c->h_pre);
  c->d_pre = nullptr; c->d_frameTH = nullptr; c->d_u = c->d_v = c->d_idepth = c->d_idepth_zero = c->d_priorF = nullptr;
  c->d_color = c->d_weight = nullptr; c->d_res_of_slot = nullptr; c->d_res_order = nullptr;
  c->d_chunk_begin = c->d_chunk_host = c->d_host_chunk_begin = c->d_pt_host = nullptr;
  c->d_r_state = c->d_r_active = nullptr;
  c->d_r_energy = c->d_r_newEnergy = c->d_r_ewo = c->d_r_JpJdF = c->d_r_center = nullptr;
  c->d_p_HdiF = c->d_p_bdSumF = c->d_p_Hcd = c->d_p_step = nullptr; c->d_p_ngood = nullptr;
  c->d_partials = nullptr; c->d_slabs = nullptr; c->d_adHost = c->d_adTarget = nullptr; c->d_sys = nullptr;
  c->h_sys = nullptr; c->d_xAd = nullptr; c->h_xAd = nullptr; c->h_pre = nullptr; c->d_cand = nullptr;
  c->d_cnt = nullptr; c->d_stat = nullptr;
  c->nF = c->nP = c->nR = 0;
  c->haveSystem = false;
}

// ---------------------------------------------------------------- host pieces of the GN loop
static void compute_priors(hs_ctx* c) {
  // accumulateLF_MT with no linearized residuals = the priors of stitchDoubleInternal(usePrior)
  const int n = c->dim();
  c->HL.assign(n * n, 0.0);
  c->bL.assign(n, 0.0);
  for (int i = 0; i < 4; i++) {
    c->HL[i * n + i] += c->P.initialCalibHessian;
    c->bL[i] += (double)c->P.initialCalibHessian * (double)(float)c->calib.value_minus_value_zero[i];
  }
  for (int h = 0; h < c->nF; h++)
    for (int i = 0; i < 8; i++) {
      const int j = 4 + 8 * h + i;
      c->HL[j * n + j] += c->frames[h].prior[i];
      c->bL[j] += c->frames[h].prior[i] * c->frames[h].delta_prior[i];
    }
}

static void set_delta(hs_ctx* c) {  // the frame part of setDeltaF (points: idepth_zero reset keeps deltaF = 0)
  for (auto& f : c->frames)
    for (int i = 0; i < 8; i++) {
      f.delta[i] = f.state[i] - f.state_zero[i];
      f.delta_prior[i] = f.state[i] - 0.0;
    }
}

static int upload_precalc(hs_ctx* c) {
  for (int h = 0; h < c->nF; h++)
    for (int t = 0; t < c->nF; t++) c->h_pre[h * c->nF + t] = make_precalc(c->frames[h], c->frames[t], c->calib);
  HS_HIP(hipMemcpyAsync(c->d_pre, c->h_pre, sizeof(HsPrecalc) * c->nF * c->nF, hipMemcpyHostToDevice, c->stream));
  set_delta(c);
  return HS_OK;
}

static void compute_projector(hs_ctx* c) {
  const int n = c->dim();
  std::vector<std::vector<double>> ns;
  for (int i = 0; i < 6; i++) {
    std::vector<double> v(n, 0.0);
    for (auto& f : c->frames) {
      for (int k = 0; k < 6; k++) v[4 + f.idx * 8 + k] = f.nullspaces_pose[i][k];
      for (int k = 0; k < 3; k++) v[4 + f.idx * 8 + k] *= SCALE_XI_TRANS_INVERSE;
      for (int k = 3; k < 6; k++) v[4 + f.idx * 8 + k] *= SCALE_XI_ROT_INVERSE;
    }
    ns.push_back(v);
  }
  std::vector<double> v(n, 0.0);
  for (auto& f : c->frames) {
    for (int k = 0; k < 6; k++) v[4 + f.idx * 8 + k] = f.nullspaces_scale[k];
    for (int k = 0; k < 3; k++) v[4 + f.idx * 8 + k] *= SCALE_XI_TRANS_INVERSE;
    for (int k = 3; k < 6; k++) v[4 + f.idx * 8 + k] *= SCALE_XI_ROT_INVERSE;
  }
  ns.push_back(v);
  nullspace_projector(ns, n, c->P.solverModeDelta, c->Porth);
}

// stitchDoubleMT post-processing: copy calib column blocks, symmetrize the top frame blocks
static void finish_systems(hs_ctx* c) {
  const int n = c->dim(), nF = c->nF;
  const double* s = c->h_sys;
  c->HA.assign(s, s + n * n);
  c->bA.assign(s + n * n, s + n * n + n);
  c->HSC.assign(s + n * n + n, s + 2 * n * n + n);
  c->bSC.assign(s + 2 * n * n + n, s + 2 * n * n + 2 * n);
  c->lastEnergy = s[2 * n * n + 2 * n];
  std::vector<double>& H = c->HA;
  for (int h = 0; h < nF; h++) {
    const int hIdx = 4 + h * 8;
    for (int r = 0; r < 8; r++)
      for (int cc = 0; cc < 4; cc++) H[cc * n + hIdx + r] = H[(hIdx + r) * n + cc];
    for (int t = h + 1; t < nF; t++) {
      const int tIdx = 4 + t * 8;
      for (int r = 0; r < 8; r++)
        for (int cc = 0; cc < 8; cc++) H[(hIdx + r) * n + tIdx + cc] += H[(tIdx + cc) * n + hIdx + r];
      for (int r = 0; r < 8; r++)
        for (int cc = 0; cc < 8; cc++) H[(tIdx + r) * n + hIdx + cc] = H[(hIdx + cc) * n + tIdx + r];
    }
  }
  for (int h = 0; h < nF; h++) {
    const int hIdx = 4 + h * 8;
    for (int r = 0; r < 8; r++)
      for (int cc = 0; cc < 4; cc++) c->HSC[cc * n + hIdx + r] = c->HSC[(hIdx + r) * n + cc];
  }
  compute_priors(c);
  c->haveSystem = true;
}

// launch linearize + reduce + energy threshold (no sync)
static int launch_linearize(hs_ctx* c, bool timed) {
  const int n_chunks = (int)c->chunk_host.size();
  HsLinArgs a;
  std::memset(&a, 0, sizeof(a));
  for (int i = 0; i < c->nF; i++) a.img[i] = c->d_img[i];
  a.calib = c->calib.device();
  a.lp.huberTH = c->P.huberTH;
  a.lp.outlierTHSumComponent = c->P.outlierTHSumComponent;
  a.lp.affineOptModeA = c->P.affineOptModeA;
  a.lp.affineOptModeB = c->P.affineOptModeB;
  a.nF = c->nF;
  a.write_center = 1;
  a.pre = c->d_pre;
  a.frameTH = c->d_frameTH;
  a.u = c->d_u; a.v = c->d_v; a.idepth = c->d_idepth; a.idepth_zero = c->d_idepth_zero; a.priorF = c->d_priorF;
  a.color = c->d_color; a.weight = c->d_weight;
  a.res_of_slot = c->d_res_of_slot; a.res_order = c->d_res_order;
  a.chunk_begin = c->d_chunk_begin; a.chunk_host = c->d_chunk_host;
  a.r_state = c->d_r_state; a.r_active = c->d_r_active; a.r_energy = c->d_r_energy; a.r_newEnergy = c->d_r_newEnergy;
  a.r_ewo = c->d_r_ewo; a.r_JpJdF = c->d_r_JpJdF; a.r_center = c->d_r_center;
  a.p_HdiF = c->d_p_HdiF; a.p_bdSumF = c->d_p_bdSumF; a.p_Hcd = c->d_p_Hcd; a.p_ngood = c->d_p_ngood;
  a.partials = c->d_partials;
  a.newest_cand = c->d_cand + (size_t)c->rank * c->cand_stride;
  a.newest_cnt = c->d_cnt + c->rank;
  HS_HIP(hipMemsetAsync(c->d_cnt + c->rank, 0, sizeof(int), c->stream));
  if (timed) HS_HIP(hipEventRecord(c->ev[0], c->stream));
  if (n_chunks > 0) hipLaunchKernelGGL(hs_k_linearize, dim3(n_chunks), dim3(64), 0, c->stream, a);
  HS_HIP(hipGetLastError());
  if (timed) HS_HIP(hipEventRecord(c->ev[1], c->stream));
  HsReduceArgs ra;
  ra.partials = c->d_partials;
  ra.host_chunk_begin = c->d_host_chunk_begin;
  ra.n_chunks = n_chunks;
  ra.slabs = c->d_slabs;
  const int n = c->dim();
  ra.energy = c->d_sys + 2 * n * n + 2 * n;
  hipLaunchKernelGGL(hs_k_reduce, dim3(8, c->nF), dim3(256), 0, c->stream, ra);
  HS_HIP(hipGetLastError());
  if (c->comm && c->nranks > 1) {
    // setNewFrameEnergyTH needs the union of all ranks' energies into the newest frame
    HS_NCCL(ncclAllGather(c->d_cnt + c->rank, c->d_cnt, 1, ncclInt, c->comm, c->stream));
    HS_NCCL(ncclAllGather(c->d_cand + (size_t)c->rank * c->cand_stride, c->d_cand, c->cand_stride, ncclFloat,
                          c->comm, c->stream));
  }
  HsEnergyThArgs ea;
  ea.cand = c->d_cand;
  ea.cnt = c->d_cnt;
  ea.nranks = c->nranks;
  ea.stride = c->cand_stride;
  ea.frameTH = c->d_frameTH;
  ea.newest = c->nF - 1;
  ea.frameEnergyTHN = c->P.frameEnergyTHN;
  ea.facMedian = c->P.frameEnergyTHFacMedian;
  ea.constWeight = c->P.frameEnergyTHConstWeight;
  ea.overallWeight = c->P.overallEnergyTHWeight;
  if (timed) HS_HIP(hipEventRecord(c->ev[2], c->stream));
  hipLaunchKernelGGL(hs_k_energy_th, dim3(1), dim3(1024), 0, c->stream, ea);
  HS_HIP(hipGetLastError());
  if (timed) HS_HIP(hipEventRecord(c->ev[3], c->stream));
  return HS_OK;
}

// stitch (+ all-reduce) + D2H of the systems, then sync
static int stitch_and_fetch(hs_ctx* c, bool timed) {
  const int n = c->dim();
  // zero H/b (keep the energy slot written by hs_k_reduce)
  HS_HIP(hipMemsetAsync(c->d_sys, 0, sizeof(double) * (2 * n * n + 2 * n), c->stream));
  HsStitchArgs sa;
  sa.nF = c->nF;
  sa.slabs = c->d_slabs;
  sa.adHost = c->d_adHost;
  sa.adTarget = c->d_adTarget;
  sa.HA = c->d_sys;
  sa.bA = c->d_sys + n * n;
  sa.HSC = c->d_sys + n * n + n;
  sa.bSC = c->d_sys + 2 * n * n + n;
  hipLaunchKernelGGL(hs_k_stitch, dim3(c->nF * c->nF), dim3(64), 0, c->stream, sa);
  HS_HIP(hipGetLastError());
  if (timed) HS_HIP(hipEventRecord(c->ev[4], c->stream));
  if (c->comm && c->nranks > 1)
    HS_NCCL(ncclAllReduce(c->d_sys, c->d_sys, c->sys_len(), ncclDouble, ncclSum, c->comm, c->stream));
  HS_HIP(hipMemcpyAsync(c->h_sys, c->d_sys, sizeof(double) * c->sys_len(), hipMemcpyDeviceToHost, c->stream));
  HS_HIP(hipStreamSynchronize(c->stream));
  finish_systems(c);
  return HS_OK;
}

// solveSystemF on the fetched systems; writes frame/calib steps, uploads xAd
static int host_solve(hs_ctx* c, int iteration, std::vector<double>& x) {
  const int n = c->dim();
  const double lambda = 1e-5;  // SOLVER_FIX_LAMBDA
  std::vector<double> delta(n);
  for (int i = 0; i < 4; i++) delta[i] = (double)(float)c->calib.value_minus_value_zero[i];
  for (int h = 0; h < c->nF; h++)
    for (int i = 0; i < 8; i++) delta[4 + 8 * h + i] = c->frames[h].delta[i];
  std::vector<double> Hf(n * n), bf(n);
  for (int i = 0; i < n; i++) {
    double s = 0;
    for (int j = 0; j < n; j++) s += c->HM[i * n + j] * delta[j];
    bf[i] = c->bL[i] + (c->bM[i] + s) + c->bA[i] - c->bSC[i];
  }
  for (int i = 0; i < n * n; i++) Hf[i] = c->HL[i] + c->HM[i] + c->HA[i];
  for (int i = 0; i < n; i++) Hf[i * n + i] *= (1 + lambda);
  const double sc = (double)(1.0f / (1 + lambda));
  for (int i = 0; i < n * n; i++) Hf[i] -= c->HSC[i] * sc;
  std::vector<double> S(n);
  for (int i = 0; i < n; i++) S[i] = 1.0 / std::sqrt(Hf[i * n + i] + 10);
  std::vector<double> Hs(n * n), bs(n);
  for (int i = 0; i < n; i++)
    for (int j = 0; j < n; j++) Hs[i * n + j] = S[i] * Hf[i * n + j] * S[j];
  for (int i = 0; i < n; i++) bs[i] = S[i] * bf[i];
  std::vector<double> y;
  ldlt_solve(Hs, n, bs, y);
  x.assign(n, 0.0);
  for (int i = 0; i < n; i++) x[i] = S[i] * y[i];
  if (iteration >= 2) {
    std::vector<double> px(n, 0.0);
    for (int i = 0; i < n; i++) {
      double s = 0;
      for (int j = 0; j < n; j++) s += c->Porth[i * n + j] * x[j];
      px[i] = s;
    }
    for (int i = 0; i < n; i++) x[i] -= px[i];
  }
  for (double v : x)
    if (!std::isfinite(v)) return fail(HS_ERR_NONFINITE, "non-finite GN step");
  // resubstituteF_MT host part
  std::vector<float> xF(n);
  for (int i = 0; i < n; i++) xF[i] = (float)x[i];
  for (int i = 0; i < 4; i++) c->calib.step[i] = -x[i];
  const int nF = c->nF;
  for (int h = 0; h < nF; h++) {
    for (int i = 0; i < 8; i++) c->frames[h].step[i] = -x[4 + 8 * h + i];
    c->frames[h].step[8] = c->frames[h].step[9] = 0;
    for (int t = 0; t < nF; t++) {
      const float* aH = &c->adHostF[(h + nF * t) * 64];
      const float* aT = &c->adTargetF[(h + nF * t) * 64];
      for (int cc = 0; cc < 8; cc++) {
        float s1 = 0, s2 = 0;
        for (int r = 0; r < 8; r++) s1 += xF[4 + 8 * h + r] * aH[r * 8 + cc];
        for (int r = 0; r < 8; r++) s2 += xF[4 + 8 * t + r] * aT[r * 8 + cc];
        c->h_xAd[(nF * h + t) * 8 + cc] = s1 + s2;
      }
    }
  }
  HS_HIP(hipMemcpyAsync(c->d_xAd, c->h_xAd, sizeof(float) * nF * nF * 8, hipMemcpyHostToDevice, c->stream));
  return HS_OK;
}

static int launch_resub(hs_ctx* c, const std::vector<double>& x, int apply) {
  HsResubArgs ra;
  ra.n = c->nP;
  ra.nF = c->nF;
  ra.apply = apply;
  for (int i = 0; i < 4; i++) ra.cstep[i] = (float)x[i];
  ra.host = c->d_pt_host;
  ra.xAd = c->d_xAd;
  ra.bdSumF = c->d_p_bdSumF;
  ra.HdiF = c->d_p_HdiF;
  ra.Hcd = c->d_p_Hcd;
  ra.ngood = c->d_p_ngood;
  ra.res_of_slot = c->d_res_of_slot;
  ra.res_order = c->d_res_order;
  ra.r_active = c->d_r_active;
  ra.JpJdF = c->d_r_JpJdF;
  ra.idepth = c->d_idepth;
  ra.idepth_zero = c->d_idepth_zero;
  ra.step = c->d_p_step;
  ra.stat_partial = c->d_stat;
  if (c->nP > 0) hipLaunchKernelGGL(hs_k_resub, dim3(c->n_stat_blocks), dim3(256), 0, c->stream, ra);
  HS_HIP(hipGetLastError());
  return HS_OK;
}

static void backup_state(hs_ctx* c) {
  for (int i = 0; i < 4; i++) c->calib.value_backup[i] = c->calib.value[i];
  for (auto& f : c->frames)
    for (int i = 0; i < 10; i++) f.state_backup[i] = f.state[i];
}

// frame/calib half of doStepFromBackup + setPrecalcValues (points were stepped on the device)
static int host_step(hs_ctx* c, bool* canbreak) {
  double nv[4];
  for (int i = 0; i < 4; i++) nv[i] = c->calib.value_backup[i] + 1.0f * c->calib.step[i];
  c->calib.setValue(nv);
  float sumA = 0, sumB = 0, sumT = 0, sumR = 0;
  for (auto& f : c->frames) {
    double s[10];
    for (int i = 0; i < 10; i++) s[i] = f.state_backup[i] + 1.0 * f.step[i];
    f.setState(s);
    sumA += f.step[6] * f.step[6];
    sumB += f.step[7] * f.step[7];
    sumT += f.step[0] * f.step[0] + f.step[1] * f.step[1] + f.step[2] * f.step[2];
    sumR += f.step[3] * f.step[3] + f.step[4] * f.step[4] + f.step[5] * f.step[5];
  }
  int rc = upload_precalc(c);
  if (rc) return rc;
  if (canbreak) {
    std::vector<double> st(2 * c->n_stat_blocks);
    HS_HIP(hipMemcpyAsync(st.data(), c->d_stat, sizeof(double) * st.size(), hipMemcpyDeviceToHost, c->stream));
    HS_HIP(hipStreamSynchronize(c->stream));
    double sID = 0, sNID = 0;
    for (int b = 0; b < c->n_stat_blocks; b++) { sID += st[2 * b]; sNID += st[2 * b + 1]; }
    const float nfr = (float)c->frames.size();
    sumA /= nfr; sumB /= nfr; sumR /= nfr; sumT /= nfr;
    const float sumID = (float)(sID / c->nP), sumNID = (float)(sNID / c->nP);
    (void)sumID;
    const float th = c->P.thOptIterations;
    *canbreak = sqrtf(sumA) < 0.0005 * th && sqrtf(sumB) < 0.00005 * th && sqrtf(sumR) < 0.00005 * th &&
                sqrtf(sumT) * sumNID < 0.00005 * th;
  }
  return HS_OK;
}

static int reset_states(hs_ctx* c) {  // PointFrameResidual::resetOOB on every active residual
  HS_HIP(hipMemsetAsync(c->d_r_state, HS_RES_IN, c->nR, c->stream));
  HS_HIP(hipMemsetAsync(c->d_r_active, 0, c->nR, c->stream));
  HS_HIP(hipMemsetAsync(c->d_r_energy, 0, sizeof(float) * c->nR, c->stream));
  HS_HIP(hipMemsetAsync(c->d_r_newEnergy, 0, sizeof(float) * c->nR, c->stream));
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
  return HS_OK;
}

const char* hs_last_error(void) { return g_err.c_str(); }

int hs_create(hs_ctx** out, const hs_params* params, int device_id) {
  if (!out) return fail(HS_ERR_INVALID, "null out");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(HS_ERR_HIP, "no HIP device");
  if (device_id < 0 || device_id >= ndev) return fail(HS_ERR_INVALID, "bad device id");
  hs_ctx* c = new hs_ctx();
  if (params) c->P = *params;
  else hs_params_default(&c->P);
  c->device = device_id;
  HS_HIP(hipSetDevice(device_id));
  HS_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  for (auto& e : c->ev) HS_HIP(hipEventCreate(&e));
  *out = c;
  return HS_OK;
}

void hs_destroy(hs_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  free_window(c);
  if (c->comm) ncclCommDestroy(c->comm);
  for (auto& e : c->ev) (void)hipEventDestroy(e);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

int hs_ba_set_window(hs_ctx* c, const hs_camera* cam, int nF, const hs_frame* fr, const float* const* images,
                     const hs_points* pts, const hs_residuals* rs) {
  if (!c || !cam || !fr || !images || !pts || !rs) return fail(HS_ERR_INVALID, "null argument");
  if (nF < 2 || nF > HS_MAXF) return fail(HS_ERR_INVALID, "nF must be in [2, 8]");
  if (cam->width < 8 || cam->height < 8) return fail(HS_ERR_INVALID, "bad camera size");
  HS_HIP(hipSetDevice(c->device));
  free_window(c);
  c->nF = nF;
  c->nP = pts->n;
  c->nR = rs->n;
  const int W = cam->width, H = cam->height;
  // calib (CalibData constructor: setValueScaled, value_zero = value)
  c->calib.W = W;
  c->calib.H = H;
  double vs[4] = {cam->fx, cam->fy, cam->cx, cam->cy};
  for (int i = 0; i < 4; i++) c->calib.value_zero[i] = 0;
  c->calib.setValueScaled(vs);
  for (int i = 0; i < 4; i++) {
    c->calib.value_zero[i] = c->calib.value[i];
    c->calib.value_minus_value_zero[i] = 0;
    c->calib.step[i] = 0;
  }
  // frames
  c->frames.assign(nF, FrameH());
  for (int i = 0; i < nF; i++) {
    FrameH& f = c->frames[i];
    f.id = fr[i].id;
    f.idx = i;
    f.ab_exposure = fr[i].ab_exposure;
    f.frameEnergyTH = fr[i].frameEnergyTH;
    f.evalPT = SE3::fromData(fr[i].worldToCam_evalPT);
    f.setState(fr[i].state);
    f.setStateZero(fr[i].state_zero);
    f.takeData(c->P);
  }
  // points / residual CSR
  c->pt_host.assign(pts->host, pts->host + c->nP);
  for (int i = 1; i < c->nP; i++)
    if (c->pt_host[i] < c->pt_host[i - 1]) return fail(HS_ERR_INVALID, "points must be sorted by host");
  for (int i = 0; i < c->nP; i++)
    if (c->pt_host[i] < 0 || c->pt_host[i] >= nF) return fail(HS_ERR_INVALID, "bad point host");
  c->res_of_slot.assign((size_t)c->nP * 8, -1);
  c->res_order.assign((size_t)c->nP * 8, (int8_t)-1);
  std::vector<int> nres(c->nP, 0);
  int lastp = -1;
  for (int r = 0; r < c->nR; r++) {
    const int p = rs->point[r], t = rs->target[r];
    if (p < 0 || p >= c->nP || t < 0 || t >= nF) return fail(HS_ERR_INVALID, "bad residual index");
    if (p < lastp) return fail(HS_ERR_INVALID, "residuals must be grouped by point in point order");
    if (t == c->pt_host[p]) return fail(HS_ERR_INVALID, "residual target == host");
    if (c->res_of_slot[p * 8 + t] >= 0) return fail(HS_ERR_INVALID, "duplicate (point, target) residual");
    lastp = p;
    c->res_of_slot[p * 8 + t] = r;
    c->res_order[p * 8 + nres[p]] = (int8_t)t;
    nres[p]++;
  }
  // chunks of <= chunk_size points of one host
  c->chunk_begin.clear();
  c->chunk_host.clear();
  c->host_chunk_begin.assign(nF + 1, 0);
  {
    int p = 0;
    for (int h = 0; h < nF; h++) {
      c->host_chunk_begin[h] = (int)c->chunk_host.size();
      while (p < c->nP && c->pt_host[p] == h) {
        int e = p;
        while (e < c->nP && c->pt_host[e] == h && e - p < c->chunk_size) e++;
        c->chunk_begin.push_back(p);
        c->chunk_host.push_back(h);
        p = e;
      }
    }
    c->host_chunk_begin[nF] = (int)c->chunk_host.size();
    c->chunk_begin.push_back(c->nP);
  }
  const int n_chunks = (int)c->chunk_host.size();
  // adjoints (constant while evalPT is fixed)
  c->adHost.assign(nF * nF * 64, 0.0);
  c->adTarget.assign(nF * nF * 64, 0.0);
  c->adHostF.assign(nF * nF * 64, 0.f);
  c->adTargetF.assign(nF * nF * 64, 0.f);
  for (int h = 0; h < nF; h++)
    for (int t = 0; t < nF; t++) {
      const int idx = h + t * nF;
      make_adjoints(c->frames[h], c->frames[t], &c->adHost[idx * 64], &c->adTarget[idx * 64]);
      for (int i = 0; i < 64; i++) {
        c->adHostF[idx * 64 + i] = (float)c->adHost[idx * 64 + i];
        c->adTargetF[idx * 64 + i] = (float)c->adTarget[idx * 64 + i];
      }
    }
  const int n = c->dim();
  if (c->HM.size() != (size_t)n * n) { c->HM.assign(n * n, 0.0); c->bM.assign(n, 0.0); }
  compute_projector(c);

  // ---- device allocations + uploads
  const size_t npx = (size_t)W * H;
  std::vector<float4> tex(npx);
  for (int f = 0; f < nF; f++) {
    if (dalloc(&c->d_img[f], npx)) return HS_ERR_HIP;
    const float* src = images[f];
    for (size_t i = 0; i < npx; i++) tex[i] = make_float4(src[3 * i], src[3 * i + 1], src[3 * i + 2], 0.f);
    HS_HIP(hipMemcpy(c->d_img[f], tex.data(), npx * sizeof(float4), hipMemcpyHostToDevice));
  }
  int rc = 0;
  rc |= dalloc(&c->d_pre, nF * nF);
  rc |= dalloc(&c->d_frameTH, nF);
  rc |= dalloc(&c->d_u, c->nP); rc |= dalloc(&c->d_v, c->nP);
  rc |= dalloc(&c->d_idepth, c->nP); rc |= dalloc(&c->d_idepth_zero, c->nP); rc |= dalloc(&c->d_priorF, c->nP);
  rc |= dalloc(&c->d_color, (size_t)c->nP * 8); rc |= dalloc(&c->d_weight, (size_t)c->nP * 8);
  rc |= dalloc(&c->d_res_of_slot, (size_t)c->nP * 8); rc |= dalloc(&c->d_res_order, (size_t)c->nP * 8);
  rc |= dalloc(&c->d_chunk_begin, n_chunks + 1); rc |= dalloc(&c->d_chunk_host, n_chunks);
  rc |= dalloc(&c->d_host_chunk_begin, nF + 1); rc |= dalloc(&c->d_pt_host, c->nP);
  rc |= dalloc(&c->d_r_state, c->nR); rc |= dalloc(&c->d_r_active, c->nR);
  rc |= dalloc(&c->d_r_energy, c->nR); rc |= dalloc(&c->d_r_newEnergy, c->nR); rc |= dalloc(&c->d_r_ewo, c->nR);
  rc |= dalloc(&c->d_r_JpJdF, (size_t)c->nR * 8); rc |= dalloc(&c->d_r_center, (size_t)c->nR * 3);
  rc |= dalloc(&c->d_p_HdiF, c->nP); rc |= dalloc(&c->d_p_bdSumF, c->nP); rc |= dalloc(&c->d_p_Hcd, (size_t)c->nP * 4);
  rc |= dalloc(&c->d_p_step, c->nP); rc |= dalloc(&c->d_p_ngood, c->nP);
  rc |= dalloc(&c->d_partials, n_chunks); rc |= dalloc(&c->d_slabs, nF);
  rc |= dalloc(&c->d_adHost, nF * nF * 64); rc |= dalloc(&c->d_adTarget, nF * nF * 64);
  rc |= dalloc(&c->d_sys, c->sys_len());
  rc |= dalloc(&c->d_xAd, nF * nF * 8);
  // candidate buffer: every rank uses the same stride (max residual count over ranks)
  c->cand_stride = c->nR > 0 ? c->nR : 1;
  if (c->comm && c->nranks > 1) {
    int* d_tmp = nullptr;
    if (dalloc(&d_tmp, 1)) return HS_ERR_HIP;
    HS_HIP(hipMemcpy(d_tmp, &c->cand_stride, sizeof(int), hipMemcpyHostToDevice));
    HS_NCCL(ncclAllReduce(d_tmp, d_tmp, 1, ncclInt, ncclMax, c->comm, c->stream));
    HS_HIP(hipStreamSynchronize(c->stream));
    HS_HIP(hipMemcpy(&c->cand_stride, d_tmp, sizeof(int), hipMemcpyDeviceToHost));
    (void)hipFree(d_tmp);
  }
  rc |= dalloc(&c->d_cand, (size_t)c->cand_stride * c->nranks);
  rc |= dalloc(&c->d_cnt, c->nranks);
  c->n_stat_blocks = (c->nP + 255) / 256;
  rc |= dalloc(&c->d_stat, 2 * (c->n_stat_blocks > 0 ? c->n_stat_blocks : 1));
  if (rc) return HS_ERR_HIP;
  HS_HIP(hipHostMalloc((void**)&c->h_sys, sizeof(double) * c->sys_len()));
  HS_HIP(hipHostMalloc((void**)&c->h_xAd, sizeof(float) * nF * nF * 8));
  HS_HIP(hipHostMalloc((void**)&c->h_pre, sizeof(HsPrecalc) * nF * nF));
  std::vector<float> prior(c->nP, 0.f);
  for (int i = 0; i < c->nP; i++)
    prior[i] = (pts->has_depth_prior && pts->has_depth_prior[i]) ? c->P.idepthFixPrior * 1.0f * 1.0f : 0.f;
  std::vector<float> th(nF);
  for (int i = 0; i < nF; i++) th[i] = c->frames[i].frameEnergyTH;
  HS_HIP(hipMemcpy(c->d_frameTH, th.data(), sizeof(float) * nF, hipMemcpyHostToDevice));
  HS_HIP(hipMemcpy(c->d_u, pts->u, sizeof(float) * c->nP, hipMemcpyHostToDevice));
  HS_HIP(hipMemcpy(c->d_v, pts->v, sizeof(float) * c->nP, hipMemcpyHostToDevice));
  HS_HIP(hipMemcpy(c->d_idepth, pts->idepth, sizeof(float) * c->nP, hipMemcpyHostToDevice));
  HS_HIP(hipMemcpy(c->d_idepth_zero, pts->idepth_zero, sizeof(float) * c->nP, hipMemcpyHostToDevice));
  HS_HIP(hipMemcpy(c->d_priorF, prior.data(), sizeof(float) * c->nP, hipMemcpyHostToDevice));
  HS_HIP(hipMemcpy(c->d_color, pts->color, sizeof(float) * 8 * c->nP, hipMemcpyHostToDevice));
  HS_HIP(hipMemcpy(c->d_weight, pts->weights, sizeof(float) * 8 * c->nP, hipMemcpyHostToDevice));
  HS_HIP(hipMemcpy(c->d_res_of_slot, c->res_of_slot.data(), sizeof(int) * 8 * c->nP, hipMemcpyHostToDevice));
  HS_HIP(hipMemcpy(c->d_res_order, c->res_order.data(), 8 * c->nP, hipMemcpyHostToDevice));
  HS_HIP(hipMemcpy(c->d_chunk_begin, c->chunk_begin.data(), sizeof(int) * (n_chunks + 1), hipMemcpyHostToDevice));
  HS_HIP(hipMemcpy(c->d_chunk_host, c->chunk_host.data(), sizeof(int) * n_chunks, hipMemcpyHostToDevice));
  HS_HIP(hipMemcpy(c->d_host_chunk_begin, c->host_chunk_begin.data(), sizeof(int) * (nF + 1), hipMemcpyHostToDevice));
  HS_HIP(hipMemcpy(c->d_pt_host, c->pt_host.data(), sizeof(int) * c->nP, hipMemcpyHostToDevice));
  HS_HIP(hipMemcpy(c->d_adHost, c->adHost.data(), sizeof(double) * nF * nF * 64, hipMemcpyHostToDevice));
  HS_HIP(hipMemcpy(c->d_adTarget, c->adTarget.data(), sizeof(double) * nF * nF * 64, hipMemcpyHostToDevice));
  HS_HIP(hipMemset(c->d_partials, 0, sizeof(HsWavePartial) * (n_chunks > 0 ? n_chunks : 1)));
  HS_HIP(hipMemset(c->d_r_JpJdF, 0, sizeof(float) * 8 * (c->nR > 0 ? c->nR : 1)));
  HS_HIP(hipMemset(c->d_r_center, 0, sizeof(float) * 3 * (c->nR > 0 ? c->nR : 1)));
  HS_HIP(hipMemset(c->d_r_ewo, 0, sizeof(float) * (c->nR > 0 ? c->nR : 1)));
  HS_HIP(hipMemset(c->d_p_step, 0, sizeof(float) * (c->nP > 0 ? c->nP : 1)));
  if (rs->state) {
    HS_HIP(hipMemcpy(c->d_r_state, rs->state, c->nR, hipMemcpyHostToDevice));
    HS_HIP(hipMemset(c->d_r_active, 0, c->nR));
    HS_HIP(hipMemset(c->d_r_energy, 0, sizeof(float) * c->nR));
    HS_HIP(hipMemset(c->d_r_newEnergy, 0, sizeof(float) * c->nR));
  } else {
    if (reset_states(c)) return HS_ERR_HIP;
  }
  rc = upload_precalc(c);
  if (rc) return rc;
  compute_priors(c);
  HS_HIP(hipStreamSynchronize(c->stream));
  return HS_OK;
}

int hs_ba_linearize(hs_ctx* c, int reset, double* energy_out) {
  if (!c || c->nF == 0) return fail(HS_ERR_STATE, "no window");
  HS_HIP(hipSetDevice(c->device));
  if (reset && reset_states(c)) return HS_ERR_HIP;
  int rc = launch_linearize(c, false);
  if (rc) return rc;
  rc = stitch_and_fetch(c, false);
  if (rc) return rc;
  if (energy_out) *energy_out = c->lastEnergy;
  if (!std::isfinite(c->lastEnergy)) return fail(HS_ERR_NONFINITE, "non-finite energy (isLost)");
  return HS_OK;
}

int hs_ba_solve_system(hs_ctx* c, int iteration, double* x_out) {
  if (!c || c->nF == 0) return fail(HS_ERR_STATE, "no window");
  if (!c->haveSystem) return fail(HS_ERR_STATE, "hs_ba_linearize must run first");
  HS_HIP(hipSetDevice(c->device));
  std::vector<double> x;
  int rc = host_solve(c, iteration, x);
  if (rc) return rc;
  rc = launch_resub(c, x, 0);
  if (rc) return rc;
  HS_HIP(hipStreamSynchronize(c->stream));
  if (x_out) std::memcpy(x_out, x.data(), sizeof(double) * x.size());
  return HS_OK;
}

int hs_ba_do_step(hs_ctx* c, int* canbreak_out) {
  if (!c || c->nF == 0) return fail(HS_ERR_STATE, "no window");
  HS_HIP(hipSetDevice(c->device));
  backup_state(c);
  if (c->nP > 0) hipLaunchKernelGGL(hs_k_apply_step, dim3((c->nP + 255) / 256), dim3(256), 0, c->stream, c->nP,
                                    c->d_p_step, c->d_idepth, c->d_idepth_zero);
  HS_HIP(hipGetLastError());
  bool cb = false;
  int rc = host_step(c, canbreak_out ? &cb : nullptr);
  if (rc) return rc;
  HS_HIP(hipStreamSynchronize(c->stream));
  if (canbreak_out) *canbreak_out = cb ? 1 : 0;
  return HS_OK;
}

// K GN iterations continuing from the current linearization (System::optimize loop body)
static int gn_iterations(hs_ctx* c, int it0, int K, bool allow_break, double* energies_out, int* done) {
  double tl = 0, ts = 0, tr = 0, tt = 0;
  int it = it0, k = 0;
  int rc;
  for (; k < K; k++, it++) {
    backup_state(c);
    std::vector<double> x;
    rc = host_solve(c, it, x);
    if (rc) return rc;
    HS_HIP(hipEventRecord(c->ev[6], c->stream));
    rc = launch_resub(c, x, 1);
    if (rc) return rc;
    HS_HIP(hipEventRecord(c->ev[7], c->stream));
    bool cb = false;
    rc = host_step(c, allow_break ? &cb : nullptr);
    if (rc) return rc;
    rc = launch_linearize(c, true);
    if (rc) return rc;
    rc = stitch_and_fetch(c, true);
    if (rc) return rc;
    float ms;
    (void)hipEventElapsedTime(&ms, c->ev[0], c->ev[1]); tl += ms;
    (void)hipEventElapsedTime(&ms, c->ev[1], c->ev[2]); ts += ms;
    (void)hipEventElapsedTime(&ms, c->ev[3], c->ev[4]); ts += ms;
    (void)hipEventElapsedTime(&ms, c->ev[2], c->ev[3]); tt += ms;
    (void)hipEventElapsedTime(&ms, c->ev[6], c->ev[7]); tr += ms;
    if (energies_out) energies_out[k] = c->lastEnergy;
    if (!std::isfinite(c->lastEnergy)) return fail(HS_ERR_NONFINITE, "non-finite energy (isLost)");
    if (allow_break && cb && it >= c->P.minOptIterations) { k++; break; }
  }
  c->t_lin = tl; c->t_stitch = ts; c->t_resub = tr; c->t_th = tt;
  c->t_iters = k;
  if (done) *done = k;
  return HS_OK;
}

int hs_ba_optimize(hs_ctx* c, int max_iters, int allow_break, double* energies_out, int* iters_done) {
  if (!c || c->nF == 0) return fail(HS_ERR_STATE, "no window");
  HS_HIP(hipSetDevice(c->device));
  if (c->nF < 3) max_iters = 20;
  else if (c->nF < 4) max_iters = 15;
  auto t0 = std::chrono::steady_clock::now();
  if (reset_states(c)) return HS_ERR_HIP;
  int rc = launch_linearize(c, false);
  if (rc) return rc;
  rc = stitch_and_fetch(c, false);
  if (rc) return rc;
  if (energies_out) energies_out[0] = c->lastEnergy;
  int done = 0;
  rc = gn_iterations(c, 0, max_iters, allow_break != 0, energies_out ? energies_out + 1 : nullptr, &done);
  if (rc) return rc;
  c->t_wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (iters_done) *iters_done = done;
  return HS_OK;
}

int hs_ba_iterate(hs_ctx* c, int first_iteration, int n_iters, double* energies_out) {
  if (!c || c->nF == 0) return fail(HS_ERR_STATE, "no window");
  if (!c->haveSystem) return fail(HS_ERR_STATE, "hs_ba_linearize must run first");
  HS_HIP(hipSetDevice(c->device));
  auto t0 = std::chrono::steady_clock::now();
  int done = 0;
  int rc = gn_iterations(c, first_iteration, n_iters, false, energies_out, &done);
  if (rc) return rc;
  c->t_wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return HS_OK;
}

int hs_ba_get_system(hs_ctx* c, int which, double* H, double* b) {
  if (!c || !c->haveSystem) return fail(HS_ERR_STATE, "no system");
  const int n = c->dim();
  const std::vector<double>* HH = which == 0 ? &c->HA : which == 1 ? &c->HL : &c->HSC;
  const std::vector<double>* bb = which == 0 ? &c->bA : which == 1 ? &c->bL : &c->bSC;
  if (which < 0 || which > 2) return fail(HS_ERR_INVALID, "which must be 0, 1 or 2");
  if (H) std::memcpy(H, HH->data(), sizeof(double) * n * n);
  if (b) std::memcpy(b, bb->data(), sizeof(double) * n);
  return HS_OK;
}

int hs_ba_get_residuals(hs_ctx* c, uint8_t* state, uint8_t* active, float* energy, float* energy_wo, float* JpJdF,
                        float* center) {
  if (!c || c->nF == 0) return fail(HS_ERR_STATE, "no window");
  HS_HIP(hipSetDevice(c->device));
  const size_t m = c->nR;
  if (state) HS_HIP(hipMemcpy(state, c->d_r_state, m, hipMemcpyDeviceToHost));
  if (active) HS_HIP(hipMemcpy(active, c->d_r_active, m, hipMemcpyDeviceToHost));
  if (energy) HS_HIP(hipMemcpy(energy, c->d_r_energy, m * 4, hipMemcpyDeviceToHost));
  if (energy_wo) HS_HIP(hipMemcpy(energy_wo, c->d_r_ewo, m * 4, hipMemcpyDeviceToHost));
  if (JpJdF) HS_HIP(hipMemcpy(JpJdF, c->d_r_JpJdF, m * 32, hipMemcpyDeviceToHost));
  if (center) HS_HIP(hipMemcpy(center, c->d_r_center, m * 12, hipMemcpyDeviceToHost));
  return HS_OK;
}

int hs_ba_get_points(hs_ctx* c, float* idepth, float* step, float* HdiF, float* bdSumF) {
  if (!c || c->nF == 0) return fail(HS_ERR_STATE, "no window");
  HS_HIP(hipSetDevice(c->device));
  const size_t n = c->nP;
  if (idepth) HS_HIP(hipMemcpy(idepth, c->d_idepth, n * 4, hipMemcpyDeviceToHost));
  if (step) HS_HIP(hipMemcpy(step, c->d_p_step, n * 4, hipMemcpyDeviceToHost));
  if (HdiF) HS_HIP(hipMemcpy(HdiF, c->d_p_HdiF, n * 4, hipMemcpyDeviceToHost));
  if (bdSumF) HS_HIP(hipMemcpy(bdSumF, c->d_p_bdSumF, n * 4, hipMemcpyDeviceToHost));
  return HS_OK;
}

int hs_ba_get_frames(hs_ctx* c, double* state, float* energyTH, double* pose7, double* calib4) {
  if (!c || c->nF == 0) return fail(HS_ERR_STATE, "no window");
  HS_HIP(hipSetDevice(c->device));
  if (energyTH) HS_HIP(hipMemcpy(energyTH, c->d_frameTH, sizeof(float) * c->nF, hipMemcpyDeviceToHost));
  for (int i = 0; i < c->nF; i++) {
    if (state) for (int k = 0; k < 10; k++) state[i * 10 + k] = c->frames[i].state[k];
    if (pose7) c->frames[i].PRE_worldToCam.toData(pose7 + 7 * i);
  }
  if (calib4) for (int k = 0; k < 4; k++) calib4[k] = c->calib.value[k];
  return HS_OK;
}

int hs_ba_set_marginal_prior(hs_ctx* c, const double* HM, const double* bM) {
  if (!c || c->nF == 0) return fail(HS_ERR_STATE, "no window");
  const int n = c->dim();
  c->HM.assign(HM, HM + n * n);
  c->bM.assign(bM, bM + n);
  return HS_OK;
}

int hs_ba_get_timings(hs_ctx* c, double* out6) {
  if (!c || !out6) return fail(HS_ERR_INVALID, "null");
  out6[0] = c->t_lin; out6[1] = c->t_stitch; out6[2] = c->t_resub; out6[3] = c->t_th; out6[4] = c->t_wall;
  out6[5] = c->t_iters;
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
  HS_HIP(hipSetDevice(c->device));
  ncclUniqueId id;
  std::memcpy(&id, id128, 128);
  HS_NCCL(ncclCommInitRank(&c->comm, nranks, id, rank));
  c->rank = rank;
  c->nranks = nranks;
  return HS_OK;
}

}  // extern "C"
