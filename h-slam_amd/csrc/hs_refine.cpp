// hs_refine.cpp — C-ABI implementation of the DirectRefinement boundary (include/hs_refine.h): refiner
// context, device frames and point state (structure of arrays), and the LM step launches (one kernel per
// iteration, enqueued in batches; the device-side control block decides and stops).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/hs_refine.h"
#include "hs_refine_kernels.h"

namespace hs {
extern thread_local std::string g_err;
}

namespace {
int rfail(int code, const std::string& msg) {
  hs::g_err = msg;
  return code;
}

// Eigen compute_inverse_size3 in double (CalibData: pyrKi[0] = pyrK[0].inverse(), Include/CalibData.h:150)
void inv3d(const double m[9], double r[9]) {
  auto M = [&](int i, int j) { return m[i * 3 + j]; };
  auto cof = [&](int i, int j) {
    int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
    return M(i1, j1) * M(i2, j2) - M(i1, j2) * M(i2, j1);
  };
  const double c00 = cof(0, 0), c10 = cof(1, 0), c20 = cof(2, 0);
  const double invdet = 1.0 / (c00 * M(0, 0) + c10 * M(1, 0) + c20 * M(2, 0));
  r[0] = c00 * invdet; r[1] = c10 * invdet; r[2] = c20 * invdet;
  r[3] = cof(0, 1) * invdet; r[4] = cof(1, 1) * invdet; r[5] = cof(2, 1) * invdet;
  r[6] = cof(0, 2) * invdet; r[7] = cof(1, 2) * invdet; r[8] = cof(2, 2) * invdet;
}
}  // namespace

#define RF_HIP(x)                                                                                   \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) return rfail(HS_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)
#define RF_TRY(x)        \
  do {                   \
    int rc_ = (x);       \
    if (rc_) return rc_; \
  } while (0)

// per-point planes of the device state block (floats unless noted)
enum { PF_U, PF_V, PF_INVZ, PF_ID, PF_IDN, PF_IR, PF_E0, PF_E1, PF_EN0, PF_EN1, PF_LH, PF_LHN, PF_MS, PF_JB0 = PF_MS + 1,
       PF_COUNT = PF_JB0 + 20 };

struct hs_refiner {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  int W = 0, H = 0;
  double K4[4] = {0, 0, 0, 0};
  double Ki[9];
  float4* d_img1 = nullptr;
  float4* d_img2 = nullptr;
  float expo1 = 0, expo2 = 0;
  bool haveFrames = false;
  int n = 0, cap = 0;
  float* d_pf = nullptr;     // PF_COUNT planes of cap floats
  uint8_t* d_pb = nullptr;   // tri | good | good_new, cap bytes each
  int jb_sel = 0;
  HsRefCtl* d_ctl = nullptr;
  HsRefCtl* h_ctl = nullptr;
  int* h_flags = nullptr;
  double* d_part = nullptr;  // [nblocks][HS_REF_NRED]
  int* d_ticket = nullptr;
  float* d_log = nullptr;
  int last_iters = 0;
  long long* d_trace = nullptr;  // HS_REF_TRACE=1: per-block stamps of each step launch, dumped to stderr
  double last_ms = 0;
};

static HsRefPoints points_of(hs_refiner* r) {
  HsRefPoints p;
  const size_t c = (size_t)r->cap;
  float* f = r->d_pf;
  p.u = f + PF_U * c; p.v = f + PF_V * c; p.invz = f + PF_INVZ * c;
  p.idepth = f + PF_ID * c; p.idepth_new = f + PF_IDN * c; p.iR = f + PF_IR * c;
  p.energy = f + PF_E0 * c;        // [2][n]: planes E0 | E1 are contiguous only when n == cap, so n = cap below
  p.energy_new = f + PF_EN0 * c;
  p.lastH = f + PF_LH * c; p.lastH_new = f + PF_LHN * c; p.maxstep = f + PF_MS * c;
  p.jb[0] = f + PF_JB0 * c; p.jb[1] = f + (PF_JB0 + 10) * c;
  p.tri = r->d_pb; p.good = r->d_pb + c; p.good_new = r->d_pb + 2 * c;
  return p;
}

static HsRefArgs make_args(hs_refiner* r, int mode) {
  HsRefArgs a;
  std::memset(&a, 0, sizeof(a));
  a.p = points_of(r);
  a.n = r->n;
  a.W = r->W; a.H = r->H;
  a.mode = mode;
  a.nblocks = (r->n + HS_REF_PPB - 1) / HS_REF_PPB;
  a.fx = (float)r->K4[0]; a.fy = (float)r->K4[1]; a.cx = (float)r->K4[2]; a.cy = (float)r->K4[3];
  for (int q = 0; q < 9; q++) a.Ki[q] = r->Ki[q];
  a.img1 = r->d_img1;
  a.img2 = r->d_img2;
  a.huberTH = 9.f;                  // setting_huberTH (Src/Settings.cpp:68)
  a.outlierTH = 12 * 12;            // setting_outlierTH (Src/Settings.cpp:65)
  a.jb_sel0 = r->jb_sel;
  a.ctl = r->d_ctl;
  a.part = r->d_part;
  a.ticket = r->d_ticket;
  a.log = r->d_log;
  a.trace = r->d_trace;
  return a;
}

static int enqueue(hs_refiner* r, const HsRefArgs& a) {
  hipLaunchKernelGGL(hs_k_refine_step, dim3(a.nblocks), dim3(256), 0, r->stream, a);
  RF_HIP(hipGetLastError());
  return HS_OK;
}

static int dump_trace(hs_refiner* r, int nb, int launch_no) {
  std::vector<long long> t((size_t)nb * 16);
  RF_HIP(hipMemcpyAsync(t.data(), r->d_trace, t.size() * sizeof(long long), hipMemcpyDeviceToHost, r->stream));
  RF_HIP(hipStreamSynchronize(r->stream));
  int khz = 0;
  RF_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, r->device));
  const double us = khz > 0 ? 1e3 / khz : 0.01;
  long long t0 = t[0];
  for (int b = 0; b < nb; b++) t0 = std::min(t0, t[(size_t)b * 16]);
  for (int k = 0; k < 16; k++) {
    std::vector<double> v;
    for (int b = 0; b < nb; b++) {
      const long long x = t[(size_t)b * 16 + k];
      if (x >= t0) v.push_back((x - t0) * us);
    }
    if (v.empty()) continue;
    std::sort(v.begin(), v.end());
    std::fprintf(stderr, "[hs refine trace] launch %d cp%d n %3zu min %7.2f med %7.2f max %7.2f us\n", launch_no, k,
                 v.size(), v.front(), v[v.size() / 2], v.back());
  }
  RF_HIP(hipMemsetAsync(r->d_trace, 0, t.size() * sizeof(long long), r->stream));
  return HS_OK;
}

static int read_ctl(hs_refiner* r) {
  RF_HIP(hipMemcpyAsync(r->h_ctl, r->d_ctl, sizeof(HsRefCtl), hipMemcpyDeviceToHost, r->stream));
  RF_HIP(hipStreamSynchronize(r->stream));
  return HS_OK;
}

static int check_ready(hs_refiner* r) {
  if (!r->haveFrames) return rfail(HS_ERR_STATE, "hs_refiner_set_frames first");
  if (r->n <= 0) return rfail(HS_ERR_STATE, "hs_refiner_set_points first");
  RF_HIP(hipSetDevice(r->device));
  return HS_OK;
}

// resetPoints + one calcResAndGS at (T, aff)
static int run_calc(hs_refiner* r, const double T7[7], const double aff[2]) {
  RF_TRY(check_ready(r));
  HsRefArgs a = make_args(r, HS_REF_CALC);
  hs_ref_pass_consts(T7, aff, r->Ki, r->n, &a.pc0);
  RF_HIP(hipEventRecord(r->e0, r->stream));
  RF_TRY(enqueue(r, a));
  RF_HIP(hipEventRecord(r->e1, r->stream));
  RF_TRY(read_ctl(r));
  float ms = 0;
  RF_HIP(hipEventElapsedTime(&ms, r->e0, r->e1));
  r->last_ms = ms;
  return HS_OK;
}

// Refine: the first pass, then LM steps enqueued in batches until the device sets done, then the final applyStep
static int run_refine(hs_refiner* r, const double T7[7], const double aff[2]) {
  RF_TRY(check_ready(r));
  HsRefArgs a = make_args(r, HS_REF_INIT);
  hs_ref_pass_consts(T7, aff, r->Ki, r->n, &a.pc0);
  for (int q = 0; q < 7; q++) a.T0[q] = T7[q];
  a.aff0[0] = aff[0];
  a.aff0[1] = aff[1];
  RF_HIP(hipEventRecord(r->e0, r->stream));
  RF_TRY(enqueue(r, a));
  HsRefArgs it = make_args(r, HS_REF_ITER);
  int launched = 0, batch = 4;
  if (r->d_trace) batch = 1;
  for (;;) {
    for (int k = 0; k < batch; k++) RF_TRY(enqueue(r, it));
    if (r->d_trace && launched < 3) RF_TRY(dump_trace(r, it.nblocks, launched));
    launched += batch;
    RF_HIP(hipMemcpyAsync(&r->h_flags[0], &r->d_ctl->done, sizeof(int), hipMemcpyDeviceToHost, r->stream));
    RF_HIP(hipStreamSynchronize(r->stream));
    if (r->h_flags[0]) break;
    if (launched > HS_REF_MAXLOG + 8) return rfail(HS_ERR_STATE, "refine did not stop within the iteration cap");
    if (!r->d_trace) batch = std::min(2 * batch, 32);
  }
  RF_TRY(enqueue(r, make_args(r, HS_REF_FINAL)));  // the pending applyStep + optReg of the last accepted pass
  RF_HIP(hipEventRecord(r->e1, r->stream));
  RF_TRY(read_ctl(r));
  float ms = 0;
  RF_HIP(hipEventElapsedTime(&ms, r->e0, r->e1));
  r->last_ms = ms;
  r->jb_sel = r->h_ctl->jb_sel ^ r->h_ctl->apply_prev;
  r->last_iters = r->h_ctl->iteration + 1;
  return HS_OK;
}

extern "C" {

int hs_refiner_create(hs_refiner** out, int device_id, int width, int height, const double K4[4]) {
  if (!out || !K4 || width < 8 || height < 8) return rfail(HS_ERR_INVALID, "bad refiner arguments");
  hs_refiner* r = new hs_refiner();
  r->device = device_id;
  r->W = width;
  r->H = height;
  for (int q = 0; q < 4; q++) r->K4[q] = K4[q];
  const double K[9] = {K4[0], 0, K4[2], 0, K4[1], K4[3], 0, 0, 1};
  inv3d(K, r->Ki);
  const size_t np = (size_t)width * height;
  if (hipSetDevice(device_id) != hipSuccess || hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&r->e0) != hipSuccess || hipEventCreate(&r->e1) != hipSuccess ||
      hipMalloc(&r->d_img1, np * sizeof(float4)) != hipSuccess || hipMalloc(&r->d_img2, np * sizeof(float4)) != hipSuccess ||
      hipMalloc(&r->d_ctl, sizeof(HsRefCtl)) != hipSuccess || hipHostMalloc(&r->h_ctl, sizeof(HsRefCtl)) != hipSuccess ||
      hipHostMalloc(&r->h_flags, 4 * sizeof(int)) != hipSuccess || hipMalloc(&r->d_ticket, sizeof(int)) != hipSuccess ||
      hipMemsetAsync(r->d_ticket, 0, sizeof(int), r->stream) != hipSuccess ||
      hipMemsetAsync(r->d_ctl, 0, sizeof(HsRefCtl), r->stream) != hipSuccess ||
      hipMalloc(&r->d_log, sizeof(float) * HS_REF_MAXLOG * HS_REF_LOGW) != hipSuccess) {
    hs_refiner_destroy(r);
    return rfail(HS_ERR_HIP, "refiner allocation failed");
  }
  *out = r;
  return HS_OK;
}

void hs_refiner_destroy(hs_refiner* r) {
  if (!r) return;
  (void)hipSetDevice(r->device);
  if (r->stream) (void)hipStreamSynchronize(r->stream);
  (void)hipFree(r->d_img1);
  (void)hipFree(r->d_img2);
  (void)hipFree(r->d_pf);
  (void)hipFree(r->d_pb);
  (void)hipFree(r->d_ctl);
  (void)hipFree(r->d_part);
  (void)hipFree(r->d_ticket);
  (void)hipFree(r->d_trace);
  (void)hipFree(r->d_log);
  if (r->h_ctl) (void)hipHostFree(r->h_ctl);
  if (r->h_flags) (void)hipHostFree(r->h_flags);
  if (r->e0) (void)hipEventDestroy(r->e0);
  if (r->e1) (void)hipEventDestroy(r->e1);
  if (r->stream) (void)hipStreamDestroy(r->stream);
  delete r;
}

int hs_refiner_set_frames(hs_refiner* r, const float* first, const float* second, float e1, float e2) {
  if (!r || !first || !second) return rfail(HS_ERR_INVALID, "null frame");
  RF_HIP(hipSetDevice(r->device));
  const size_t np = (size_t)r->W * r->H;
  std::vector<float4> tex(np);
  float4* dst[2] = {r->d_img1, r->d_img2};
  const float* src[2] = {first, second};
  for (int f = 0; f < 2; f++) {
    for (size_t i = 0; i < np; i++) tex[i] = make_float4(src[f][3 * i], src[f][3 * i + 1], src[f][3 * i + 2], 0.f);
    RF_HIP(hipMemcpyAsync(dst[f], tex.data(), np * sizeof(float4), hipMemcpyHostToDevice, r->stream));
    RF_HIP(hipStreamSynchronize(r->stream));  // tex is reused
  }
  r->expo1 = e1;
  r->expo2 = e2;
  r->haveFrames = true;
  return HS_OK;
}

int hs_refiner_set_points(hs_refiner* r, int n, const float* u, const float* v, const uint8_t* tri, const float* z) {
  if (!r || n <= 0 || !u || !v || !tri || !z) return rfail(HS_ERR_INVALID, "bad points");
  for (int i = 0; i < n; i++)
    if (!std::isfinite(u[i]) || !std::isfinite(v[i]) || u[i] < 0 || v[i] < 0 || u[i] > r->W - 1 || v[i] > r->H - 1)
      return rfail(HS_ERR_INVALID, "keypoint outside the image");
  RF_HIP(hipSetDevice(r->device));
  (void)hipFree(r->d_pf);
  (void)hipFree(r->d_pb);
  (void)hipFree(r->d_part);
  r->d_pf = nullptr;
  r->d_pb = nullptr;
  r->d_part = nullptr;
  r->n = 0;
  r->cap = n;  // planes of exactly n: the [2][n] energy blocks are two adjacent planes
  RF_HIP(hipMalloc(&r->d_pf, sizeof(float) * PF_COUNT * (size_t)n));
  RF_HIP(hipMalloc(&r->d_pb, 3 * (size_t)n));
  RF_HIP(hipMalloc(&r->d_part, sizeof(double) * HS_REF_NRED * (size_t)((n + HS_REF_PPB - 1) / HS_REF_PPB)));
  (void)hipFree(r->d_trace);
  r->d_trace = nullptr;
  if (const char* e = std::getenv("HS_REF_TRACE"); e && std::atoi(e) > 0) {
    RF_HIP(hipMalloc(&r->d_trace, sizeof(long long) * 16 * (size_t)((n + HS_REF_PPB - 1) / HS_REF_PPB)));
    RF_HIP(hipMemsetAsync(r->d_trace, 0, sizeof(long long) * 16 * (size_t)((n + HS_REF_PPB - 1) / HS_REF_PPB),
                          r->stream));
  }
  // the ctor's Pnt set-up (Src/Initializer.cpp:1362-1382)
  std::vector<float> pf((size_t)PF_COUNT * n, 0.f);
  std::vector<uint8_t> pb(3 * (size_t)n, 0);
  for (int i = 0; i < n; i++) {
    const float invz = tri[i] ? (float)(1.0 / z[i]) : 1.0f;
    pf[PF_U * (size_t)n + i] = u[i];
    pf[PF_V * (size_t)n + i] = v[i];
    pf[PF_INVZ * (size_t)n + i] = invz;
    pf[PF_ID * (size_t)n + i] = invz;
    pf[PF_IDN * (size_t)n + i] = invz;
    pf[PF_IR * (size_t)n + i] = invz;
    pb[i] = tri[i] ? 1 : 0;
    pb[n + i] = 1;  // isGood
  }
  RF_HIP(hipMemcpyAsync(r->d_pf, pf.data(), pf.size() * sizeof(float), hipMemcpyHostToDevice, r->stream));
  RF_HIP(hipMemcpyAsync(r->d_pb, pb.data(), pb.size(), hipMemcpyHostToDevice, r->stream));
  RF_HIP(hipStreamSynchronize(r->stream));
  r->n = n;
  r->jb_sel = 0;
  r->last_iters = 0;
  return HS_OK;
}

int hs_refiner_refine(hs_refiner* r, double pose[7], float* idepth_out, uint8_t* good_out, int* iterations,
                      int* snapped) {
  if (!r || !pose) return rfail(HS_ERR_INVALID, "null");
  double aff[2] = {0, 0};  // thisToNext_aff = AffLight(0, 0)
  if (r->expo1 > 0 && r->expo2 > 0) aff[0] = (double)logf(r->expo2 / r->expo1);
  RF_TRY(run_refine(r, pose, aff));
  const HsRefCtl& o = *r->h_ctl;
  for (int q = 0; q < 7; q++) pose[q] = o.T[q];
  if (iterations) *iterations = r->last_iters;
  if (snapped) *snapped = o.snapped;
  if (idepth_out || good_out) {
    const size_t n = r->n;
    std::vector<float> id(n);
    std::vector<uint8_t> tri(n), good(n);
    const HsRefPoints p = points_of(r);
    RF_HIP(hipMemcpyAsync(id.data(), p.idepth, n * sizeof(float), hipMemcpyDeviceToHost, r->stream));
    RF_HIP(hipMemcpyAsync(tri.data(), p.tri, n, hipMemcpyDeviceToHost, r->stream));
    RF_HIP(hipMemcpyAsync(good.data(), p.good, n, hipMemcpyDeviceToHost, r->stream));
    RF_HIP(hipStreamSynchronize(r->stream));
    for (size_t i = 0; i < n; i++) {
      if (good_out) good_out[i] = good[i];
      if (idepth_out && good[i] && tri[i]) idepth_out[i] = id[i];  // _videpth write-back (:1389-1395)
    }
  }
  if (!std::isfinite(o.resOld[0])) return rfail(HS_ERR_NONFINITE, "non-finite refinement energy");
  return HS_OK;
}

int hs_refiner_calc_res(hs_refiner* r, const double T7[7], const double aff[2], float* H64, float* b8, float* Hsc64,
                        float* bsc8, float res3[3]) {
  if (!r || !T7 || !aff) return rfail(HS_ERR_INVALID, "null");
  RF_TRY(run_calc(r, T7, aff));
  const HsRefCtl& o = *r->h_ctl;
  if (H64) std::memcpy(H64, o.H, sizeof(o.H));
  if (b8) std::memcpy(b8, o.b, sizeof(o.b));
  if (Hsc64) std::memcpy(Hsc64, o.Hsc, sizeof(o.Hsc));
  if (bsc8) std::memcpy(bsc8, o.bsc, sizeof(o.bsc));
  if (res3) std::memcpy(res3, o.res, sizeof(o.res));
  return HS_OK;
}

int hs_refiner_get_points(hs_refiner* r, float* f7, uint8_t* g2, float* jb_new) {
  if (!r || !f7 || !g2) return rfail(HS_ERR_INVALID, "null");
  if (r->n <= 0) return rfail(HS_ERR_STATE, "no points");
  RF_HIP(hipSetDevice(r->device));
  const size_t n = r->n;
  std::vector<float> pf((size_t)PF_COUNT * n);
  std::vector<uint8_t> pb(3 * n);
  RF_HIP(hipMemcpyAsync(pf.data(), r->d_pf, pf.size() * sizeof(float), hipMemcpyDeviceToHost, r->stream));
  RF_HIP(hipMemcpyAsync(pb.data(), r->d_pb, pb.size(), hipMemcpyDeviceToHost, r->stream));
  RF_HIP(hipStreamSynchronize(r->stream));
  const int planes[7] = {PF_ID, PF_IDN, PF_IR, PF_EN0, PF_EN1, PF_MS, PF_LHN};
  for (size_t i = 0; i < n; i++) {
    for (int k = 0; k < 7; k++) f7[7 * i + k] = pf[planes[k] * n + i];
    g2[2 * i] = pb[n + i];
    g2[2 * i + 1] = pb[2 * n + i];
  }
  if (jb_new) {  // JbBuffer_new = the plane the next calcResAndGS writes
    const int base = PF_JB0 + 10 * (r->jb_sel ^ 1);
    for (size_t i = 0; i < n; i++)
      for (int k = 0; k < 10; k++) jb_new[10 * i + k] = pf[(base + k) * n + i];
  }
  return HS_OK;
}

int hs_refiner_get_log(hs_refiner* r, int cap, float* out) {
  if (!r || (cap > 0 && !out)) return rfail(HS_ERR_INVALID, "null");
  const int n = std::min(r->last_iters, HS_REF_MAXLOG);
  const int m = std::min(n, cap);
  if (m > 0) {
    RF_HIP(hipSetDevice(r->device));
    RF_HIP(hipStreamSynchronize(r->stream));
    RF_HIP(hipMemcpy(out, r->d_log, sizeof(float) * HS_REF_LOGW * m, hipMemcpyDeviceToHost));
  }
  return n;
}

int hs_refiner_last_ms(hs_refiner* r, double* ms) {
  if (!r || !ms) return rfail(HS_ERR_INVALID, "null");
  *ms = r->last_ms;
  return HS_OK;
}

}  // extern "C"
