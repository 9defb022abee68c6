// hs_trace.cpp — C-ABI implementation of the immature-point tracing boundary (include/hs_trace.h):
// tracer context, device SoA of ImmaturePoint state, ctor / traceOn / tally launches.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/hs_ba.h"
#include "../../include/hs_trace.h"
#include "hs_trace_kernels.h"
#include "hs_pyr_kernels.h"

#define HS_MAXF_ACT 8                        // activation window (nF <= 8 keyframes)
#define HS_ACT_LDS_MAP_MAX (156 * 1024)     // level-1 distance map in LDS up to this size

namespace hs {
extern thread_local std::string g_err;
}

namespace {
int cfail(int code, const std::string& msg) {
  hs::g_err = msg;
  return code;
}
}  // namespace

#define TR_TRY(x)        \
  do {                   \
    int rc_ = (x);       \
    if (rc_) return rc_; \
  } while (0)
#define TR_HIP(x)                                                                                   \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) return cfail(HS_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

struct hs_tracer {
  hs_params P;
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  int W = 0, H = 0, cap = 0, n = 0;
  float4* d_host_img[HS_TRC_MAXHOST] = {nullptr};
  const float4** d_host_tab = nullptr;
  float4* d_new = nullptr;
  float* d_raw = nullptr;  // staging of a raw level-0 frame (hs_tracer_set_frame_raw)
  bool have_frame = false;
  hs_trace_host* d_hosts = nullptr;
  int* d_host = nullptr;
  float *d_u = nullptr, *d_v = nullptr, *d_color = nullptr, *d_weights = nullptr, *d_gradH = nullptr;
  float *d_energyTH = nullptr, *d_quality = nullptr, *d_idmin = nullptr, *d_idmax = nullptr;
  float *d_uv = nullptr, *d_interval = nullptr;
  uint8_t* d_status = nullptr;
  int* d_steps = nullptr;
  int* d_counts = nullptr;
  int* h_counts = nullptr;
  float last_ms = 0;
  long long last_steps = 0;
  bool stats_pending = false;
  int max_host = -1;  // largest host slot of the stored points
  float* d_type = nullptr;  // ImmaturePoint::my_type
  // point activation scratch (allocated by the first hs_tracer_activate)
  bool act_ready = false;
  int w1 = 0, h1 = 0, act_cap = 0;
  uint8_t* d_dist = nullptr;
  int *d_list_a = nullptr, *d_list_b = nullptr, *d_act_cnt = nullptr;
  hs_act_frame* d_act_frames = nullptr;
  hs_act_pair* d_act_pairs = nullptr;
  int* d_frame_of_slot = nullptr;
  int *d_order = nullptr, *d_cell = nullptr, *d_toopt = nullptr, *d_act_seeds = nullptr;
  uint8_t *d_cand = nullptr, *d_action = nullptr, *d_res_in = nullptr;
  float *d_frac = nullptr, *d_thr = nullptr, *d_act_idepth = nullptr;
  int* d_ap_frame = nullptr;
  float *d_ap_u = nullptr, *d_ap_v = nullptr, *d_ap_id = nullptr;
};

static int upload_img(hs_tracer* t, float4* dst, const float* src) {
  const size_t n = (size_t)t->W * t->H;
  std::vector<float4> tex(n);
  for (size_t i = 0; i < n; i++) tex[i] = make_float4(src[3 * i], src[3 * i + 1], src[3 * i + 2], 0.f);
  TR_HIP(hipMemcpyAsync(dst, tex.data(), n * sizeof(float4), hipMemcpyHostToDevice, t->stream));
  TR_HIP(hipStreamSynchronize(t->stream));
  return HS_OK;
}

static int sync_stats(hs_tracer* t) {
  if (!t->stats_pending) return HS_OK;
  TR_HIP(hipStreamSynchronize(t->stream));
  TR_HIP(hipEventElapsedTime(&t->last_ms, t->e0, t->e1));
  long long st = 0;
  memcpy(&st, t->h_counts + 6, sizeof(st));
  t->last_steps = st;
  t->stats_pending = false;
  return HS_OK;
}

static int launch_ctor(hs_tracer* t, int first, int n) {
  HsImmCtorArgs a;
  a.n = n;
  a.first = first;
  a.W = t->W;
  a.H = t->H;
  a.host_img = t->d_host_tab;
  a.host = t->d_host;
  a.u = t->d_u;
  a.v = t->d_v;
  a.outlierTHSumComponent = t->P.outlierTHSumComponent;
  a.outlierTH = t->P.outlierTH;
  a.overallEnergyTHWeight = t->P.overallEnergyTHWeight;
  a.color = t->d_color;
  a.weights = t->d_weights;
  a.gradH = t->d_gradH;
  a.energyTH = t->d_energyTH;
  a.quality = t->d_quality;
  a.idepth_min = t->d_idmin;
  a.idepth_max = t->d_idmax;
  a.status = t->d_status;
  a.uv = t->d_uv;
  a.interval = t->d_interval;
  hipLaunchKernelGGL(hs_k_imm_ctor, dim3((n + 255) / 256), dim3(256), 0, t->stream, a);
  TR_HIP(hipGetLastError());
  return HS_OK;
}

extern "C" {

int hs_tracer_create(hs_tracer** out, const hs_params* params, int device_id, int width, int height, int capacity) {
  if (!out) return cfail(HS_ERR_INVALID, "null out");
  *out = nullptr;
  if (width < 16 || height < 16 || capacity < 1) return cfail(HS_ERR_INVALID, "bad size / capacity");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return cfail(HS_ERR_HIP, "no HIP device");
  if (device_id < 0 || device_id >= ndev) return cfail(HS_ERR_INVALID, "bad device id");
  hs_tracer* t = new hs_tracer();
  if (params) t->P = *params;
  else hs_params_default(&t->P);
  t->device = device_id;
  t->W = width;
  t->H = height;
  t->cap = capacity;
  if (hipSetDevice(device_id) != hipSuccess || hipStreamCreateWithFlags(&t->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&t->e0) != hipSuccess || hipEventCreate(&t->e1) != hipSuccess) {
    delete t;
    return cfail(HS_ERR_HIP, "stream / event creation failed");
  }
  const size_t c = capacity;
  TR_HIP(hipMalloc((void**)&t->d_new, (size_t)width * height * sizeof(float4)));
  TR_HIP(hipMalloc((void**)&t->d_host_tab, sizeof(float4*) * HS_TRC_MAXHOST));
  TR_HIP(hipMemsetAsync(t->d_host_tab, 0, sizeof(float4*) * HS_TRC_MAXHOST, t->stream));  // the kernels' stream
  TR_HIP(hipMalloc((void**)&t->d_hosts, sizeof(hs_trace_host) * HS_TRC_MAXHOST));
  TR_HIP(hipMalloc((void**)&t->d_host, sizeof(int) * c));
  TR_HIP(hipMalloc((void**)&t->d_u, sizeof(float) * c));
  TR_HIP(hipMalloc((void**)&t->d_v, sizeof(float) * c));
  TR_HIP(hipMalloc((void**)&t->d_color, sizeof(float) * 8 * c));
  TR_HIP(hipMalloc((void**)&t->d_weights, sizeof(float) * 8 * c));
  TR_HIP(hipMalloc((void**)&t->d_gradH, sizeof(float) * 4 * c));
  TR_HIP(hipMalloc((void**)&t->d_energyTH, sizeof(float) * c));
  TR_HIP(hipMalloc((void**)&t->d_quality, sizeof(float) * c));
  TR_HIP(hipMalloc((void**)&t->d_idmin, sizeof(float) * c));
  TR_HIP(hipMalloc((void**)&t->d_idmax, sizeof(float) * c));
  TR_HIP(hipMalloc((void**)&t->d_uv, sizeof(float) * 2 * c));
  TR_HIP(hipMalloc((void**)&t->d_interval, sizeof(float) * c));
  TR_HIP(hipMalloc((void**)&t->d_status, c));
  TR_HIP(hipMalloc((void**)&t->d_steps, sizeof(int) * c));
  TR_HIP(hipMalloc((void**)&t->d_type, sizeof(float) * c));
  TR_HIP(hipMalloc((void**)&t->d_counts, sizeof(int) * 8));
  TR_HIP(hipHostMalloc((void**)&t->h_counts, sizeof(int) * 8));
  *out = t;
  return HS_OK;
}

void hs_tracer_destroy(hs_tracer* t) {
  if (!t) return;
  (void)hipSetDevice(t->device);
  if (t->stream) (void)hipStreamSynchronize(t->stream);
  for (auto* p : t->d_host_img) (void)hipFree(p);
  void* bufs[] = {t->d_host_tab, t->d_new, t->d_hosts, t->d_host, t->d_u, t->d_v, t->d_color, t->d_weights,
                  t->d_gradH, t->d_energyTH, t->d_quality, t->d_idmin, t->d_idmax, t->d_uv, t->d_interval,
                  t->d_status, t->d_steps, t->d_counts, t->d_raw, t->d_type, t->d_dist, t->d_list_a,
                  t->d_list_b, t->d_act_cnt, t->d_act_frames, t->d_act_pairs, t->d_frame_of_slot, t->d_order,
                  t->d_cell, t->d_toopt, t->d_act_seeds, t->d_cand, t->d_action, t->d_res_in, t->d_frac, t->d_thr,
                  t->d_act_idepth, t->d_ap_frame, t->d_ap_u, t->d_ap_v, t->d_ap_id};
  for (void* b : bufs) (void)hipFree(b);
  (void)hipHostFree(t->h_counts);
  if (t->e0) (void)hipEventDestroy(t->e0);
  if (t->e1) (void)hipEventDestroy(t->e1);
  if (t->stream) (void)hipStreamDestroy(t->stream);
  delete t;
}

int hs_tracer_set_host_image(hs_tracer* t, int slot, const float* img) {
  if (!t || !img) return cfail(HS_ERR_INVALID, "null argument");
  if (slot < 0 || slot >= HS_TRC_MAXHOST) return cfail(HS_ERR_INVALID, "host slot out of range");
  TR_HIP(hipSetDevice(t->device));
  if (!t->d_host_img[slot]) {
    TR_HIP(hipMalloc((void**)&t->d_host_img[slot], (size_t)t->W * t->H * sizeof(float4)));
    TR_HIP(hipMemcpyAsync(t->d_host_tab + slot, &t->d_host_img[slot], sizeof(float4*), hipMemcpyHostToDevice,
                          t->stream));
  }
  return upload_img(t, t->d_host_img[slot], img);
}

int hs_tracer_clear(hs_tracer* t) {
  if (!t) return cfail(HS_ERR_INVALID, "null tracer");
  t->n = 0;
  t->max_host = -1;
  return HS_OK;
}

int hs_tracer_add_points(hs_tracer* t, int n, const int* host, const float* u, const float* v) {
  if (!t || (n > 0 && (!host || !u || !v))) return cfail(HS_ERR_INVALID, "null argument");
  if (n < 0 || t->n + n > t->cap) return cfail(HS_ERR_INVALID, "point capacity exceeded");
  if (n == 0) return HS_OK;
  for (int i = 0; i < n; i++) {
    // the ctor's BiLin taps reach 2 px around (u, v) plus one texel: reject points whose pattern leaves the image
    if (host[i] < 0 || host[i] >= HS_TRC_MAXHOST || !t->d_host_img[host[i]])
      return cfail(HS_ERR_INVALID, "point on a host slot without an image");
    if (!(u[i] >= 2 && v[i] >= 2 && u[i] < t->W - 3 && v[i] < t->H - 3))
      return cfail(HS_ERR_INVALID, "immature point too close to the image border");
  }
  TR_HIP(hipSetDevice(t->device));
  const int f = t->n;
  TR_HIP(hipMemcpyAsync(t->d_host + f, host, sizeof(int) * n, hipMemcpyHostToDevice, t->stream));
  TR_HIP(hipMemcpyAsync(t->d_u + f, u, sizeof(float) * n, hipMemcpyHostToDevice, t->stream));
  TR_HIP(hipMemcpyAsync(t->d_v + f, v, sizeof(float) * n, hipMemcpyHostToDevice, t->stream));
  const std::vector<float> ones(n, 1.f);
  TR_HIP(hipMemcpyAsync(t->d_type + f, ones.data(), sizeof(float) * n, hipMemcpyHostToDevice, t->stream));
  for (int i = 0; i < n; i++) t->max_host = std::max(t->max_host, host[i]);
  TR_TRY(launch_ctor(t, f, n));
  TR_HIP(hipStreamSynchronize(t->stream));  // host arrays may go away after return
  t->n += n;
  return HS_OK;
}

int hs_tracer_set_state(hs_tracer* t, const float* idepth_min, const float* idepth_max, const float* quality,
                        const uint8_t* status, const float* interval) {
  if (!t) return cfail(HS_ERR_INVALID, "null tracer");
  if (status)
    for (int i = 0; i < t->n; i++)
      if (status[i] > HS_IPS_UNINITIALIZED) return cfail(HS_ERR_INVALID, "bad ImmaturePointStatus");
  TR_HIP(hipSetDevice(t->device));
  const size_t n = t->n;
  if (idepth_min) TR_HIP(hipMemcpyAsync(t->d_idmin, idepth_min, 4 * n, hipMemcpyHostToDevice, t->stream));
  if (idepth_max) TR_HIP(hipMemcpyAsync(t->d_idmax, idepth_max, 4 * n, hipMemcpyHostToDevice, t->stream));
  if (quality) TR_HIP(hipMemcpyAsync(t->d_quality, quality, 4 * n, hipMemcpyHostToDevice, t->stream));
  if (status) TR_HIP(hipMemcpyAsync(t->d_status, status, n, hipMemcpyHostToDevice, t->stream));
  if (interval) TR_HIP(hipMemcpyAsync(t->d_interval, interval, 4 * n, hipMemcpyHostToDevice, t->stream));
  TR_HIP(hipStreamSynchronize(t->stream));
  return HS_OK;
}

int hs_tracer_set_frame(hs_tracer* t, const float* img) {
  if (!t || !img) return cfail(HS_ERR_INVALID, "null argument");
  TR_HIP(hipSetDevice(t->device));
  int rc = upload_img(t, t->d_new, img);
  if (rc) return rc;
  t->have_frame = true;
  return HS_OK;
}

int hs_tracer_set_frame_raw(hs_tracer* t, const float* img) {
  if (!t || !img) return cfail(HS_ERR_INVALID, "null argument");
  TR_HIP(hipSetDevice(t->device));
  if (!t->d_raw) TR_HIP(hipMalloc((void**)&t->d_raw, sizeof(float) * t->W * t->H));
  TR_HIP(hipMemcpyAsync(t->d_raw, img, sizeof(float) * t->W * t->H, hipMemcpyHostToDevice, t->stream));
  float4* lv[1] = {t->d_new};
  TR_HIP(hs_build_dir_pyramid(t->stream, t->d_raw, t->W, t->H, 1, lv, nullptr));
  TR_HIP(hipStreamSynchronize(t->stream));
  t->have_frame = true;
  return HS_OK;
}

int hs_tracer_trace(hs_tracer* t, int n_hosts, const hs_trace_host* hosts, int counts6[6]) {
  if (!t || (n_hosts > 0 && !hosts)) return cfail(HS_ERR_INVALID, "null argument");
  if (n_hosts < 0 || n_hosts > HS_TRC_MAXHOST) return cfail(HS_ERR_INVALID, "n_hosts out of range");
  if (!t->have_frame) return cfail(HS_ERR_STATE, "no frame to trace on (hs_tracer_set_frame)");
  TR_HIP(hipSetDevice(t->device));
  if (t->n > 0) {
    // every point's host slot must have its (KRKi, Kt, aff)
    if (t->max_host >= n_hosts) return cfail(HS_ERR_INVALID, "a point's host slot has no hs_trace_host entry");
    TR_HIP(hipMemcpyAsync(t->d_hosts, hosts, sizeof(hs_trace_host) * n_hosts, hipMemcpyHostToDevice, t->stream));
  }
  HsTraceArgs a;
  a.n = t->n;
  a.W = t->W;
  a.H = t->H;
  a.img = t->d_new;
  a.hosts = t->d_hosts;
  a.host = t->d_host;
  a.u = t->d_u;
  a.v = t->d_v;
  a.color = t->d_color;
  a.weights = t->d_weights;
  a.gradH = t->d_gradH;
  a.energyTH = t->d_energyTH;
  a.quality = t->d_quality;
  a.idepth_min = t->d_idmin;
  a.idepth_max = t->d_idmax;
  a.status = t->d_status;
  a.uv = t->d_uv;
  a.interval = t->d_interval;
  a.steps = t->d_steps;
  a.huberTH = t->P.huberTH;
  a.maxPixSearch = t->P.maxPixSearch;
  a.slackInterval = t->P.trace_slackInterval;
  a.stepsize = t->P.trace_stepsize;
  a.minImprovementFactor = t->P.trace_minImprovementFactor;
  a.GNThreshold = t->P.trace_GNThreshold;
  a.extraSlackOnTH = t->P.trace_extraSlackOnTH;
  a.minTraceTestRadius = t->P.minTraceTestRadius;
  a.GNIterations = t->P.trace_GNIterations;
  TR_HIP(hipEventRecord(t->e0, t->stream));
  if (t->n > 0) {
    hipLaunchKernelGGL(hs_k_trace_on, dim3((t->n + 3) / 4), dim3(256), 0, t->stream, a);
    TR_HIP(hipGetLastError());
  }
  TR_HIP(hipEventRecord(t->e1, t->stream));
  hipLaunchKernelGGL(hs_k_trace_count, dim3(1), dim3(1024), 0, t->stream, t->n, t->d_status, t->d_steps,
                     t->d_counts);
  TR_HIP(hipGetLastError());
  TR_HIP(hipMemcpyAsync(t->h_counts, t->d_counts, sizeof(int) * 8, hipMemcpyDeviceToHost, t->stream));
  t->stats_pending = true;
  if (!counts6) return HS_OK;  // asynchronous: hs_tracer_last_stats / get_points synchronise
  TR_TRY(sync_stats(t));
  for (int k = 0; k < 6; k++) counts6[k] = t->h_counts[k];
  return HS_OK;
}

int hs_tracer_get_points(hs_tracer* t, int* n, uint8_t* status, float* idepth_min, float* idepth_max, float* quality,
                         float* uv, float* interval, float* energyTH, float* color, float* weights, float* gradH) {
  if (!t) return cfail(HS_ERR_INVALID, "null tracer");
  TR_HIP(hipSetDevice(t->device));
  TR_HIP(hipStreamSynchronize(t->stream));
  const size_t m = t->n;
  if (n) *n = t->n;
  if (status) TR_HIP(hipMemcpy(status, t->d_status, m, hipMemcpyDeviceToHost));
  if (idepth_min) TR_HIP(hipMemcpy(idepth_min, t->d_idmin, 4 * m, hipMemcpyDeviceToHost));
  if (idepth_max) TR_HIP(hipMemcpy(idepth_max, t->d_idmax, 4 * m, hipMemcpyDeviceToHost));
  if (quality) TR_HIP(hipMemcpy(quality, t->d_quality, 4 * m, hipMemcpyDeviceToHost));
  if (uv) TR_HIP(hipMemcpy(uv, t->d_uv, 8 * m, hipMemcpyDeviceToHost));
  if (interval) TR_HIP(hipMemcpy(interval, t->d_interval, 4 * m, hipMemcpyDeviceToHost));
  if (energyTH) TR_HIP(hipMemcpy(energyTH, t->d_energyTH, 4 * m, hipMemcpyDeviceToHost));
  if (color) TR_HIP(hipMemcpy(color, t->d_color, 32 * m, hipMemcpyDeviceToHost));
  if (weights) TR_HIP(hipMemcpy(weights, t->d_weights, 32 * m, hipMemcpyDeviceToHost));
  if (gradH) TR_HIP(hipMemcpy(gradH, t->d_gradH, 16 * m, hipMemcpyDeviceToHost));
  return HS_OK;
}

int hs_tracer_last_stats(hs_tracer* t, double* ms, long long* search_steps) {
  if (!t) return cfail(HS_ERR_INVALID, "null tracer");
  TR_HIP(hipSetDevice(t->device));
  TR_TRY(sync_stats(t));
  if (ms) *ms = t->last_ms;
  if (search_steps) *search_steps = t->last_steps;
  return HS_OK;
}

int hs_tracer_reinit(hs_tracer* t) {
  if (!t) return cfail(HS_ERR_INVALID, "null tracer");
  if (t->n == 0) return HS_OK;
  TR_HIP(hipSetDevice(t->device));
  return launch_ctor(t, 0, t->n);
}

int hs_tracer_set_types(hs_tracer* t, const float* my_type) {
  if (!t || (t->n > 0 && !my_type)) return cfail(HS_ERR_INVALID, "null argument");
  TR_HIP(hipSetDevice(t->device));
  TR_HIP(hipMemcpyAsync(t->d_type, my_type, sizeof(float) * t->n, hipMemcpyHostToDevice, t->stream));
  TR_HIP(hipStreamSynchronize(t->stream));
  return HS_OK;
}

static int act_alloc(hs_tracer* t) {
  if (t->act_ready) return HS_OK;
  t->w1 = t->W >> 1;
  t->h1 = t->H >> 1;
  const size_t wh1 = (size_t)t->w1 * t->h1, c = t->cap;
  TR_HIP(hipMalloc((void**)&t->d_dist, (wh1 + 3) & ~(size_t)3));
  TR_HIP(hipMalloc((void**)&t->d_list_a, sizeof(int) * wh1));
  TR_HIP(hipMalloc((void**)&t->d_list_b, sizeof(int) * wh1));
  TR_HIP(hipMalloc((void**)&t->d_act_cnt, sizeof(int) * 2));
  TR_HIP(hipMalloc((void**)&t->d_act_frames, sizeof(hs_act_frame) * HS_MAXF_ACT));
  TR_HIP(hipMalloc((void**)&t->d_act_pairs, sizeof(hs_act_pair) * HS_MAXF_ACT * HS_MAXF_ACT));
  TR_HIP(hipMalloc((void**)&t->d_frame_of_slot, sizeof(int) * HS_TRC_MAXHOST));
  TR_HIP(hipMalloc((void**)&t->d_order, sizeof(int) * c));
  TR_HIP(hipMalloc((void**)&t->d_cell, sizeof(int) * c));
  TR_HIP(hipMalloc((void**)&t->d_toopt, sizeof(int) * (c + 64)));  // + the greedy loop's 64 scratch slots
  TR_HIP(hipMalloc((void**)&t->d_act_seeds, sizeof(int) * 2 * (size_t)c));  // seeds | the select's pending list
  TR_HIP(hipMalloc((void**)&t->d_cand, c));
  TR_HIP(hipMalloc((void**)&t->d_action, c));
  TR_HIP(hipMalloc((void**)&t->d_res_in, c));
  TR_HIP(hipMalloc((void**)&t->d_frac, sizeof(float) * c));
  TR_HIP(hipMalloc((void**)&t->d_thr, sizeof(float) * c));
  TR_HIP(hipMalloc((void**)&t->d_act_idepth, sizeof(float) * c));
  t->act_ready = true;
  return HS_OK;
}

static int act_points_alloc(hs_tracer* t, int n) {
  if (n <= t->act_cap) return HS_OK;
  void* old[] = {t->d_ap_frame, t->d_ap_u, t->d_ap_v, t->d_ap_id};
  for (void* b : old) TR_HIP(hipFree(b));
  t->d_ap_frame = nullptr;
  t->d_ap_u = t->d_ap_v = t->d_ap_id = nullptr;
  t->act_cap = 0;
  TR_HIP(hipMalloc((void**)&t->d_ap_frame, sizeof(int) * n));
  TR_HIP(hipMalloc((void**)&t->d_ap_u, sizeof(float) * n));
  TR_HIP(hipMalloc((void**)&t->d_ap_v, sizeof(float) * n));
  TR_HIP(hipMalloc((void**)&t->d_ap_id, sizeof(float) * n));
  t->act_cap = n;
  return HS_OK;
}

// System::activatePointsMT :332-352 (float currentMinActDist, double constants as in the reference)
static void update_min_act_dist(const hs_params& P, int nPoints, float& d) {
  if (nPoints < P.desiredPointDensity * 0.66) d -= 0.8;
  if (nPoints < P.desiredPointDensity * 0.8) d -= 0.5;
  else if (nPoints < P.desiredPointDensity * 0.9) d -= 0.2;
  else if (nPoints < P.desiredPointDensity) d -= 0.1;
  if (nPoints > P.desiredPointDensity * 1.5) d += 0.8;
  if (nPoints > P.desiredPointDensity * 1.3) d += 0.5;
  if (nPoints > P.desiredPointDensity * 1.15) d += 0.2;
  if (nPoints > P.desiredPointDensity) d += 0.1;
  if (d < 0) d = 0;
  if (d > 4) d = 4;
}

int hs_tracer_activate(hs_tracer* t, const float K4[4], int nF, const hs_act_frame* frames, const hs_act_pair* pairs,
                       int n_active, const int* act_frame, const float* act_u, const float* act_v,
                       const float* act_idepth, int ef_nPoints, float* currentMinActDist, int n_order,
                       const int* order, uint8_t* action, float* idepth, uint8_t* res_in, int* activated,
                       int* n_activated) {
  if (!t || !K4 || !frames || !pairs || !currentMinActDist) return cfail(HS_ERR_INVALID, "null argument");
  if (nF < 2 || nF > HS_MAXF_ACT) return cfail(HS_ERR_INVALID, "window size out of range (2..8 keyframes)");
  if (n_active < 0 || (n_active > 0 && (!act_frame || !act_u || !act_v || !act_idepth)))
    return cfail(HS_ERR_INVALID, "bad active point arrays");
  if (!(K4[0] > 0) || !(K4[1] > 0)) return cfail(HS_ERR_INVALID, "bad intrinsics");
  std::vector<int> fos(HS_TRC_MAXHOST, -1);
  for (int f = 0; f < nF; f++) {
    const int sl = frames[f].slot;
    if (sl < 0 || sl >= HS_TRC_MAXHOST || !t->d_host_img[sl]) return cfail(HS_ERR_INVALID, "window frame without an image slot");
    if (fos[sl] >= 0) return cfail(HS_ERR_INVALID, "two window frames on one slot");
    fos[sl] = f;
  }
  for (int i = 0; i < n_active; i++)
    if (act_frame[i] < 0 || act_frame[i] >= nF) return cfail(HS_ERR_INVALID, "active point on no window frame");
  const int m = order ? n_order : t->n;
  if (order) {
    if (n_order < 0 || n_order > t->n) return cfail(HS_ERR_INVALID, "bad n_order");
    std::vector<char> seen(t->n, 0);
    for (int j = 0; j < n_order; j++) {
      if (order[j] < 0 || order[j] >= t->n || seen[order[j]]) return cfail(HS_ERR_INVALID, "order is not a subset permutation");
      seen[order[j]] = 1;
    }
  }
  TR_HIP(hipSetDevice(t->device));
  TR_TRY(sync_stats(t));
  TR_TRY(act_alloc(t));
  TR_TRY(act_points_alloc(t, std::max(1, n_active)));
  update_min_act_dist(t->P, ef_nPoints, *currentMinActDist);
  hipStream_t s = t->stream;
  const int wh1 = t->w1 * t->h1;
  TR_HIP(hipMemcpyAsync(t->d_act_frames, frames, sizeof(hs_act_frame) * nF, hipMemcpyHostToDevice, s));
  TR_HIP(hipMemcpyAsync(t->d_act_pairs, pairs, sizeof(hs_act_pair) * nF * nF, hipMemcpyHostToDevice, s));
  TR_HIP(hipMemcpyAsync(t->d_frame_of_slot, fos.data(), sizeof(int) * HS_TRC_MAXHOST, hipMemcpyHostToDevice, s));
  if (order && m > 0) TR_HIP(hipMemcpyAsync(t->d_order, order, sizeof(int) * m, hipMemcpyHostToDevice, s));
  if (n_active > 0) {
    TR_HIP(hipMemcpyAsync(t->d_ap_frame, act_frame, sizeof(int) * n_active, hipMemcpyHostToDevice, s));
    TR_HIP(hipMemcpyAsync(t->d_ap_u, act_u, sizeof(float) * n_active, hipMemcpyHostToDevice, s));
    TR_HIP(hipMemcpyAsync(t->d_ap_v, act_v, sizeof(float) * n_active, hipMemcpyHostToDevice, s));
    TR_HIP(hipMemcpyAsync(t->d_ap_id, act_idepth, sizeof(float) * n_active, hipMemcpyHostToDevice, s));
  }
  TR_HIP(hipMemsetAsync(t->d_dist, 0xff, (wh1 + 3) & ~3, s));
  TR_HIP(hipMemsetAsync(t->d_act_cnt, 0, sizeof(int) * 2, s));
  TR_HIP(hipMemsetAsync(t->d_action, HS_ACT_KEEP, std::max(1, t->n), s));
  TR_HIP(hipMemsetAsync(t->d_res_in, 0, std::max(1, t->n), s));

  HsActSeedArgs sa;
  sa.n = n_active;
  sa.newest = nF - 1;
  sa.w1 = t->w1;
  sa.h1 = t->h1;
  sa.frames = t->d_act_frames;
  sa.frame = t->d_ap_frame;
  sa.u = t->d_ap_u;
  sa.v = t->d_ap_v;
  sa.idepth = t->d_ap_id;
  sa.dist = t->d_dist;
  sa.list = t->d_list_a;
  sa.count = t->d_act_cnt;
  if (n_active > 0) {
    hipLaunchKernelGGL(hs_k_act_seed, dim3((n_active + 255) / 256), dim3(256), 0, s, sa);
    TR_HIP(hipGetLastError());
  }
  HsActCandArgs ca;
  ca.m = m;
  ca.newest = nF - 1;
  ca.w1 = t->w1;
  ca.h1 = t->h1;
  ca.minTraceQuality = t->P.minTraceQuality;
  ca.currentMinActDist = *currentMinActDist;
  ca.order = order ? t->d_order : nullptr;
  ca.frame_of_slot = t->d_frame_of_slot;
  ca.frames = t->d_act_frames;
  ca.host = t->d_host;
  ca.u = t->d_u;
  ca.v = t->d_v;
  ca.idepth_min = t->d_idmin;
  ca.idepth_max = t->d_idmax;
  ca.quality = t->d_quality;
  ca.interval = t->d_interval;
  ca.my_type = t->d_type;
  ca.status = t->d_status;
  ca.cand = t->d_cand;
  ca.cell = t->d_cell;
  ca.frac = t->d_frac;
  ca.thr = t->d_thr;
  ca.action = t->d_action;
  if (m > 0) {
    hipLaunchKernelGGL(hs_k_act_cand, dim3((m + 255) / 256), dim3(256), 0, s, ca);
    TR_HIP(hipGetLastError());
  }
  // makeDistanceMap's growDistBFS over the seeds
  HsActDistArgs ma;
  ma.w1 = t->w1;
  ma.h1 = t->h1;
  ma.mode = 0;
  static const int act_dbg = getenv("HS_ACT_DBG") ? atoi(getenv("HS_ACT_DBG")) : 0;
  ma.dbg = act_dbg;
  ma.n_tiles_x = (t->w1 - 2 + 15) / 16;
  ma.n_tiles = ma.n_tiles_x * ((t->h1 - 2 + 15) / 16);
  const int border_waves = 2 * ((t->w1 + 63) / 64) + 2 * ((t->h1 - 2 + 63) / 64);
  const int dist_blocks = ma.n_tiles + (border_waves + 3) / 4;
  ma.seeds = t->d_list_a;
  ma.n_seeds = t->d_act_cnt;
  ma.init = t->d_dist;
  ma.out = reinterpret_cast<uint8_t*>(t->d_list_b);
  hipLaunchKernelGGL(hs_k_act_dist, dim3(dist_blocks), dim3(256), 0, s, ma);
  TR_HIP(hipGetLastError());
  HsActSelectArgs se;
  se.m = m;
  se.w1 = t->w1;
  se.h1 = t->h1;
  const size_t map_bytes = (size_t)((wh1 + 3) & ~3);
  se.lds_map = map_bytes <= HS_ACT_LDS_MAP_MAX ? 1 : 0;
  se.order = order ? t->d_order : nullptr;
  se.cand = t->d_cand;
  se.cell = t->d_cell;
  se.frac = t->d_frac;
  se.thr = t->d_thr;
  se.dist = t->d_dist;
  se.map0 = reinterpret_cast<uint8_t*>(t->d_list_b);
  se.seeds = t->d_act_seeds;
  se.plist = t->d_act_seeds + t->cap;
  se.toopt = t->d_toopt;
  se.n_toopt = t->d_act_cnt + 1;
  static const bool prof_on = getenv("HS_ACT_PROF") != nullptr;
  long long* d_prof = nullptr;
  if (prof_on) TR_HIP(hipMalloc((void**)&d_prof, sizeof(long long) * 11));
  se.prof = d_prof;
  const size_t lds = se.lds_map ? map_bytes : 0;
  if (lds > 65536)
    TR_HIP(hipFuncSetAttribute((const void*)hs_k_act_select, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(hs_k_act_select, dim3(1), dim3(1024), lds, s, se);
  TR_HIP(hipGetLastError());
  HsActDistArgs fa = ma;  // the map the greedy loop leaves
  fa.mode = 1;
  fa.seeds = se.seeds;
  fa.n_seeds = se.n_toopt;
  fa.init = ma.out;
  fa.out = t->d_dist;
  hipLaunchKernelGGL(hs_k_act_dist, dim3(dist_blocks), dim3(256), 0, s, fa);
  TR_HIP(hipGetLastError());
  int cnt[2] = {0, 0};
  TR_HIP(hipMemcpyAsync(cnt, t->d_act_cnt, sizeof(cnt), hipMemcpyDeviceToHost, s));
  TR_HIP(hipStreamSynchronize(s));
  const int n_toopt = cnt[1];
  if (d_prof) {
    long long pr[11];
    TR_HIP(hipMemcpy(pr, d_prof, sizeof(pr), hipMemcpyDeviceToHost));
    TR_HIP(hipFree(d_prof));
    fprintf(stderr, "hs act prof: prologue %.1f us, greedy %.1f us (decisions %.1f, folds %.1f of which border %.1f; "
            "wall_clock64 @100 MHz), %d selected; %lld batches, %lld seed patches of radius %lld; core clock %.0f MHz\n",
            (pr[1] - pr[0]) * 1e-2, (pr[2] - pr[1]) * 1e-2, pr[8] * 1e-2, pr[9] * 1e-2, pr[10] * 1e-2, n_toopt, pr[3],
            pr[4], pr[5],
            (double)(pr[7] - pr[6]) / ((pr[2] - pr[1]) * 1e-2));
  }
  if (n_toopt > 0) {
    HsActOptArgs oa;
    oa.n = n_toopt;
    oa.nF = nF;
    oa.W = t->W;
    oa.H = t->H;
    oa.fxl = K4[0];
    oa.fyl = K4[1];
    oa.cxl = K4[2];
    oa.cyl = K4[3];
    oa.fxli = 1.0f / K4[0];
    oa.fyli = 1.0f / K4[1];
    oa.huberTH = t->P.huberTH;
    oa.minIdepthH_act = t->P.minIdepthH_act;
    oa.GNIts = t->P.GNItsOnPointActivation;
    oa.toopt = t->d_toopt;
    oa.frame_of_slot = t->d_frame_of_slot;
    oa.frames = t->d_act_frames;
    oa.pairs = t->d_act_pairs;
    oa.img = t->d_host_tab;
    oa.host = t->d_host;
    oa.u = t->d_u;
    oa.v = t->d_v;
    oa.idepth_min = t->d_idmin;
    oa.idepth_max = t->d_idmax;
    oa.color = t->d_color;
    oa.weights = t->d_weights;
    oa.energyTH = t->d_energyTH;
    oa.action = t->d_action;
    oa.idepth_out = t->d_act_idepth;
    oa.res_in = t->d_res_in;
    hipLaunchKernelGGL(hs_k_act_optimize, dim3((n_toopt + 3) / 4), dim3(256), 0, s, oa);
    TR_HIP(hipGetLastError());
  }
  const size_t n = t->n;
  std::vector<uint8_t> act(std::max<size_t>(1, n));
  std::vector<int> toopt(std::max(1, n_toopt));
  TR_HIP(hipMemcpyAsync(act.data(), t->d_action, n, hipMemcpyDeviceToHost, s));
  if (n_toopt > 0) TR_HIP(hipMemcpyAsync(toopt.data(), t->d_toopt, sizeof(int) * n_toopt, hipMemcpyDeviceToHost, s));
  if (idepth && n) TR_HIP(hipMemcpyAsync(idepth, t->d_act_idepth, sizeof(float) * n, hipMemcpyDeviceToHost, s));
  if (res_in && n) TR_HIP(hipMemcpyAsync(res_in, t->d_res_in, n, hipMemcpyDeviceToHost, s));
  TR_HIP(hipStreamSynchronize(s));
  if (action && n) memcpy(action, act.data(), n);
  int na = 0;
  for (int k = 0; k < n_toopt; k++)
    if (act[toopt[k]] == HS_ACT_ACTIVATED) {
      if (activated) activated[na] = toopt[k];
      na++;
    }
  if (idepth)  // the idepth output is defined for activated points only
    for (size_t i = 0; i < n; i++)
      if (act[i] != HS_ACT_ACTIVATED) idepth[i] = 0.f;
  if (n_activated) *n_activated = na;
  return HS_OK;
}

int hs_tracer_get_distance_map(hs_tracer* t, float* dist) {
  if (!t || !dist) return cfail(HS_ERR_INVALID, "null argument");
  if (!t->act_ready) return cfail(HS_ERR_STATE, "no activation has run");
  TR_HIP(hipSetDevice(t->device));
  const size_t wh1 = (size_t)t->w1 * t->h1;
  std::vector<uint8_t> b(wh1);
  TR_HIP(hipStreamSynchronize(t->stream));
  TR_HIP(hipMemcpy(b.data(), t->d_dist, wh1, hipMemcpyDeviceToHost));
  for (size_t i = 0; i < wh1; i++) dist[i] = b[i] == 255 ? 1000.f : (float)b[i];
  return HS_OK;
}

// stable compaction of every per-point array (a host round trip: once per keyframe)
extern "C++" template <typename T>
static int compact_array(hs_tracer* t, T* d, int per, const std::vector<int>& keep_idx) {
  const size_t n = t->n;
  std::vector<T> h(n * per), o(keep_idx.size() * per);
  if (n) TR_HIP(hipMemcpy(h.data(), d, sizeof(T) * n * per, hipMemcpyDeviceToHost));
  for (size_t k = 0; k < keep_idx.size(); k++)
    for (int c = 0; c < per; c++) o[k * per + c] = h[(size_t)keep_idx[k] * per + c];
  if (!o.empty()) {  // on the kernels' stream; o lives until the copy has landed
    TR_HIP(hipMemcpyAsync(d, o.data(), sizeof(T) * o.size(), hipMemcpyHostToDevice, t->stream));
    TR_HIP(hipStreamSynchronize(t->stream));
  }
  return HS_OK;
}

int hs_tracer_compact(hs_tracer* t, const uint8_t* keep) {
  if (!t || (t->n > 0 && !keep)) return cfail(HS_ERR_INVALID, "null argument");
  TR_HIP(hipSetDevice(t->device));
  TR_TRY(sync_stats(t));
  TR_HIP(hipStreamSynchronize(t->stream));
  std::vector<int> idx;
  for (int i = 0; i < t->n; i++)
    if (keep[i]) idx.push_back(i);
  TR_TRY(compact_array(t, t->d_host, 1, idx));
  TR_TRY(compact_array(t, t->d_u, 1, idx));
  TR_TRY(compact_array(t, t->d_v, 1, idx));
  TR_TRY(compact_array(t, t->d_color, 8, idx));
  TR_TRY(compact_array(t, t->d_weights, 8, idx));
  TR_TRY(compact_array(t, t->d_gradH, 4, idx));
  TR_TRY(compact_array(t, t->d_energyTH, 1, idx));
  TR_TRY(compact_array(t, t->d_quality, 1, idx));
  TR_TRY(compact_array(t, t->d_idmin, 1, idx));
  TR_TRY(compact_array(t, t->d_idmax, 1, idx));
  TR_TRY(compact_array(t, t->d_uv, 2, idx));
  TR_TRY(compact_array(t, t->d_interval, 1, idx));
  TR_TRY(compact_array(t, t->d_status, 1, idx));
  TR_TRY(compact_array(t, t->d_steps, 1, idx));
  TR_TRY(compact_array(t, t->d_type, 1, idx));
  std::vector<int> hosts(idx.size());
  if (!idx.empty()) TR_HIP(hipMemcpy(hosts.data(), t->d_host, sizeof(int) * idx.size(), hipMemcpyDeviceToHost));
  t->max_host = -1;
  for (int h : hosts) t->max_host = std::max(t->max_host, h);
  t->n = (int)idx.size();
  return HS_OK;
}

}  // extern "C"
