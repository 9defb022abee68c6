// hs_trace.cpp — C-ABI implementation of the immature-point tracing boundary (include/hs_trace.h):
// tracer context, device SoA of ImmaturePoint state, ctor / traceOn / tally launches.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/hs_ba.h"
#include "../../include/hs_trace.h"
#include "hs_trace_kernels.h"
#include "hs_pyr_kernels.h"

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
  TR_HIP(hipMemset(t->d_host_tab, 0, sizeof(float4*) * HS_TRC_MAXHOST));
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
                  t->d_status, t->d_steps, t->d_counts, t->d_raw};
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
    TR_HIP(hipMemcpy(t->d_host_tab + slot, &t->d_host_img[slot], sizeof(float4*), hipMemcpyHostToDevice));
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
  for (int i = 0; i < n; i++) t->max_host = std::max(t->max_host, host[i]);
  TR_TRY(launch_ctor(t, f, n));
  TR_HIP(hipStreamSynchronize(t->stream));  // host arrays may go away after return
  t->n += n;
  return HS_OK;
}

int hs_tracer_set_state(hs_tracer* t, const float* idepth_min, const float* idepth_max, const float* quality,
                        const uint8_t* status) {
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

}  // extern "C"
