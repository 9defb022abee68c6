// hs_select.cpp — C-ABI of the pixel selector (include/hs_select.h): PixelSelector's state on the device,
// makeMaps' recursion / sub-sampling decisions on the host from the device counts (Src/PixelSelector.cpp:118-262).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/hs_ba.h"
#include "../../include/hs_select.h"
#include "hs_pyr_kernels.h"
#include "hs_sel_kernels.h"

namespace hs {
extern thread_local std::string g_err;
}

namespace {
int sfail(int code, const std::string& msg) {
  hs::g_err = msg;
  return code;
}
}  // namespace

#define SL_TRY(x)        \
  do {                   \
    int rc_ = (x);       \
    if (rc_) return rc_; \
  } while (0)
#define SL_HIP(x)                                                                                   \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) return sfail(HS_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

struct hs_selector {
  hs_params P;
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  int W = 0, H = 0, w1 = 0, w2 = 0, w32 = 0, h32 = 0;
  int currentPotential = 3;
  int gradHistFrame = -1;
  bool hists_valid = false;
  size_t nths = 0;
  int max_slots = 0, max_tiles = 0;
  uint8_t* d_pattern = nullptr;
  float *d_ths = nullptr, *d_thsS = nullptr;
  unsigned int* d_ticket = nullptr;
  float* d_dI = nullptr;      // DirPyr[0] as uploaded triplets (stride 3)
  float4* d_lvl[3] = {nullptr, nullptr, nullptr};  // device pyramid (raw entry, stride 4)
  float* d_g[3] = {nullptr, nullptr, nullptr};
  float* d_raw = nullptr;
  float* d_map = nullptr;
  uint16_t* d_mask = nullptr;
  int* d_n2b = nullptr;
  uint8_t* d_has2 = nullptr;
  int* d_counts = nullptr;  // n2, n3, n4, removed
  int* h_counts = nullptr;  // pinned
  int* d_tiles = nullptr;
  float last_ms = 0;
  int last_passes = 0;
};

static int n4(int n, int pot) { return (n + 4 * pot - 1) / (4 * pot); }

extern "C" int hs_selector_create(hs_selector** out, const hs_params* params, int device_id, int width, int height) {
  if (!out) return sfail(HS_ERR_INVALID, "null out");
  *out = nullptr;
  if (width < 32 || height < 32) return sfail(HS_ERR_INVALID, "image smaller than one 32x32 histogram cell");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return sfail(HS_ERR_HIP, "no HIP device");
  if (device_id < 0 || device_id >= ndev) return sfail(HS_ERR_INVALID, "bad device id");
  hs_selector* s = new hs_selector();
  *out = s;
  if (params) s->P = *params;
  else hs_params_default(&s->P);
  s->device = device_id;
  s->W = width;
  s->H = height;
  s->w1 = width >> 1;
  s->w2 = width >> 2;
  s->w32 = width / 32;
  s->h32 = height / 32;
  // the reference's ths table is (W/32)*(H/32)+100 floats; select indexes past w32 x h32 for the last partial
  // cell column / row (oracle/sel_oracle.cpp): zeroed slack covering every index formed
  s->nths = std::max((size_t)s->w32 * s->h32 + 100, (size_t)s->w32 * (s->h32 + 1) + 1);
  const size_t area = (size_t)width * height;
  s->max_slots = n4(width, 1) * n4(height, 1) * 16;
  s->max_tiles = (int)((area + kSelSubTile - 1) / kSelSubTile);
  // randomPattern (:18-20): the C library generator, seeded as the reference
  std::vector<uint8_t> pat(area);
  std::srand(3141592);
  for (size_t i = 0; i < area; ++i) pat[i] = rand() & 0xFF;
  int rc = [&]() -> int {
    SL_HIP(hipSetDevice(device_id));
    SL_HIP(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
    SL_HIP(hipEventCreate(&s->e0));
    SL_HIP(hipEventCreate(&s->e1));
    SL_HIP(hipMalloc((void**)&s->d_pattern, area));
    SL_HIP(hipMalloc((void**)&s->d_ths, s->nths * sizeof(float)));
    SL_HIP(hipMalloc((void**)&s->d_thsS, s->nths * sizeof(float)));
    SL_HIP(hipMalloc((void**)&s->d_ticket, sizeof(unsigned int)));
    SL_HIP(hipMalloc((void**)&s->d_dI, area * 3 * sizeof(float)));
    for (int l = 0; l < 3; l++) {
      const size_t n = (size_t)(width >> l) * (height >> l);
      SL_HIP(hipMalloc((void**)&s->d_lvl[l], n * sizeof(float4)));
      SL_HIP(hipMalloc((void**)&s->d_g[l], n * sizeof(float)));
    }
    SL_HIP(hipMalloc((void**)&s->d_raw, area * sizeof(float)));
    SL_HIP(hipMalloc((void**)&s->d_map, area * sizeof(float)));
    SL_HIP(hipMalloc((void**)&s->d_mask, (size_t)s->max_slots * sizeof(uint16_t)));
    SL_HIP(hipMalloc((void**)&s->d_n2b, (size_t)s->max_slots * sizeof(int)));
    SL_HIP(hipMalloc((void**)&s->d_has2, (size_t)s->max_slots));
    SL_HIP(hipMalloc((void**)&s->d_counts, 4 * sizeof(int)));
    SL_HIP(hipHostMalloc((void**)&s->h_counts, 4 * sizeof(int), hipHostMallocDefault));
    SL_HIP(hipMalloc((void**)&s->d_tiles, (size_t)s->max_tiles * sizeof(int)));
    SL_HIP(hipMemcpyAsync(s->d_pattern, pat.data(), area, hipMemcpyHostToDevice, s->stream));
    SL_HIP(hipMemsetAsync(s->d_ths, 0, s->nths * sizeof(float), s->stream));
    SL_HIP(hipMemsetAsync(s->d_thsS, 0, s->nths * sizeof(float), s->stream));
    SL_HIP(hipMemsetAsync(s->d_ticket, 0, sizeof(unsigned int), s->stream));
    SL_HIP(hipStreamSynchronize(s->stream));
    return HS_OK;
  }();
  if (rc) {
    hs_selector_destroy(s);
    *out = nullptr;
  }
  return rc;
}

extern "C" void hs_selector_destroy(hs_selector* s) {
  if (!s) return;
  (void)hipSetDevice(s->device);
  if (s->stream) (void)hipStreamSynchronize(s->stream);
  void* dev[] = {s->d_pattern, s->d_ths, s->d_thsS, s->d_ticket, s->d_dI, s->d_lvl[0], s->d_lvl[1], s->d_lvl[2],
                 s->d_g[0], s->d_g[1], s->d_g[2], s->d_raw, s->d_map, s->d_mask, s->d_n2b, s->d_has2, s->d_counts,
                 s->d_tiles};
  for (void* p : dev)
    if (p) (void)hipFree(p);
  if (s->h_counts) (void)hipHostFree(s->h_counts);
  if (s->e0) (void)hipEventDestroy(s->e0);
  if (s->e1) (void)hipEventDestroy(s->e1);
  if (s->stream) (void)hipStreamDestroy(s->stream);
  delete s;
}

namespace {

// select (:265-415) at potential `pot` on the device; returns n2 + n3 + n4 through h_counts[0..2]
int run_select(hs_selector* s, const float* dI, int dstride, int pot, float thFactor) {
  HsSelArgs a;
  a.W = s->W;
  a.H = s->H;
  a.pot = pot;
  a.n4x = n4(s->W, pot);
  a.n4y = n4(s->H, pot);
  a.nslots = a.n4x * a.n4y * 16;
  if (a.nslots > s->max_slots) return sfail(HS_ERR_INVALID, "slot table overflow");
  a.dI = dI;
  a.dstride = dstride;
  a.g0 = s->d_g[0];
  a.g1 = s->d_g[1];
  a.g2 = s->d_g[2];
  a.w1 = s->w1;
  a.w2 = s->w2;
  a.thsSmoothed = s->d_thsS;
  a.thsStep = s->w32;
  a.dw1 = s->P.gradDownweightPerLevel;
  a.dw2 = a.dw1 * a.dw1;
  a.thFactor = thFactor;
  a.dirDist = s->P.selectDirectionDistribution;
  a.pattern = s->d_pattern;
  a.mask = s->d_mask;
  a.n2b = s->d_n2b;
  a.has2 = s->d_has2;
  a.map = s->d_map;
  a.counts = s->d_counts;
  SL_HIP(hipMemsetAsync(s->d_map, 0, (size_t)s->W * s->H * sizeof(float), s->stream));
  SL_HIP(hipMemsetAsync(s->d_counts, 0, 4 * sizeof(int), s->stream));
  hipLaunchKernelGGL(hs_k_sel_mask, dim3((a.nslots * 16 + 255) / 256), dim3(256), 0, s->stream, a);  // 16 lanes / slot
  SL_HIP(hipGetLastError());
  hipLaunchKernelGGL(hs_k_sel_scan, dim3(1), dim3(1024), 0, s->stream, a);
  SL_HIP(hipGetLastError());
  hipLaunchKernelGGL(hs_k_sel_pick, dim3((a.nslots * 4 + 255) / 256), dim3(256), 0, s->stream, a);  // 4 lanes / slot
  SL_HIP(hipGetLastError());
  SL_HIP(hipMemcpyAsync(s->h_counts, s->d_counts, 4 * sizeof(int), hipMemcpyDeviceToHost, s->stream));
  SL_HIP(hipStreamSynchronize(s->stream));
  s->last_passes++;
  return HS_OK;
}

int run_hists(hs_selector* s) {
  HsSelHistArgs h;
  h.W = s->W;
  h.H = s->H;
  h.w32 = s->w32;
  h.h32 = s->h32;
  h.absg0 = s->d_g[0];
  h.minGradHistCut = s->P.minGradHistCut;
  h.minGradHistAdd = s->P.minGradHistAdd;
  h.ths = s->d_ths;
  h.thsSmoothed = s->d_thsS;
  h.ticket = s->d_ticket;
  hipLaunchKernelGGL(hs_k_sel_hist, dim3(s->w32 * s->h32), dim3(256), 0, s->stream, h);
  SL_HIP(hipGetLastError());
  return HS_OK;
}

// makeMaps (:118-262) with the inputs resident on the device
int make_maps(hs_selector* s, const float* dI, int dstride, int id, float density, int recursionsLeft,
              float thFactor, int* n_out) {
  float numHave = 0;
  const float numWant = density;
  float quotia;
  int idealPotential = s->currentPotential;
  if (id != s->gradHistFrame || !s->hists_valid) {
    SL_TRY(run_hists(s));
    s->gradHistFrame = id;
    s->hists_valid = true;
  }
  SL_TRY(run_select(s, dI, dstride, s->currentPotential, thFactor));
  numHave = s->h_counts[0] + s->h_counts[1] + s->h_counts[2];
  quotia = numWant / numHave;
  const float K = numHave * (s->currentPotential + 1) * (s->currentPotential + 1);
  idealPotential = sqrtf(K / numWant) - 1;
  if (idealPotential < 1) idealPotential = 1;
  if (recursionsLeft > 0 && quotia > 1.25 && s->currentPotential > 1) {
    if (idealPotential >= s->currentPotential) idealPotential = s->currentPotential - 1;
    s->currentPotential = idealPotential;
    return make_maps(s, dI, dstride, id, density, recursionsLeft - 1, thFactor, n_out);
  } else if (recursionsLeft > 0 && quotia < 0.25) {
    if (idealPotential <= s->currentPotential) idealPotential = s->currentPotential + 1;
    s->currentPotential = idealPotential;
    return make_maps(s, dI, dstride, id, density, recursionsLeft - 1, thFactor, n_out);
  }
  int numHaveSub = numHave;
  if (quotia < 0.95) {
    HsSelSubArgs b;
    b.n = s->W * s->H;
    b.map = s->d_map;
    b.pattern = s->d_pattern;
    b.tile_cnt = s->d_tiles;
    b.ntiles = (b.n + kSelSubTile - 1) / kSelSubTile;
    b.charTH = (unsigned char)(255 * quotia);
    b.removed = s->d_counts + 3;
    hipLaunchKernelGGL(hs_k_sel_subcount, dim3(b.ntiles), dim3(256), 0, s->stream, b);
    SL_HIP(hipGetLastError());
    hipLaunchKernelGGL(hs_k_sel_subscan, dim3(1), dim3(1024), 0, s->stream, b);
    SL_HIP(hipGetLastError());
    hipLaunchKernelGGL(hs_k_sel_subapply, dim3(b.ntiles), dim3(256), 0, s->stream, b);
    SL_HIP(hipGetLastError());
    SL_HIP(hipMemcpyAsync(s->h_counts + 3, s->d_counts + 3, sizeof(int), hipMemcpyDeviceToHost, s->stream));
    SL_HIP(hipStreamSynchronize(s->stream));
    numHaveSub -= s->h_counts[3];
  }
  s->currentPotential = idealPotential;
  *n_out = numHaveSub;
  return HS_OK;
}

int check_args(hs_selector* s, float density, float th_factor) {
  if (!s) return sfail(HS_ERR_INVALID, "null selector");
  if (!(density > 0.f) || !std::isfinite(density)) return sfail(HS_ERR_INVALID, "density must be > 0");
  if (!(th_factor > 0.f) || !std::isfinite(th_factor)) return sfail(HS_ERR_INVALID, "thFactor must be > 0");
  if (s->currentPotential < 1 || s->currentPotential > std::max(s->W, s->H))
    return sfail(HS_ERR_STATE, "potential out of range");
  return HS_OK;
}

int finish(hs_selector* s, float* map_out, int* n_selected, int n) {
  SL_HIP(hipEventRecord(s->e1, s->stream));
  if (map_out)
    SL_HIP(hipMemcpyAsync(map_out, s->d_map, (size_t)s->W * s->H * sizeof(float), hipMemcpyDeviceToHost, s->stream));
  SL_HIP(hipStreamSynchronize(s->stream));
  SL_HIP(hipEventElapsedTime(&s->last_ms, s->e0, s->e1));
  if (n_selected) *n_selected = n;
  return HS_OK;
}

}  // namespace

extern "C" int hs_selector_make_maps(hs_selector* s, int frame_id, const float* dirpyr0, const float* absg0,
                                     const float* absg1, const float* absg2, float density, int recursions_left,
                                     float th_factor, float* map_out, int* n_selected) {
  SL_TRY(check_args(s, density, th_factor));
  if (!dirpyr0 || !absg0 || !absg1 || !absg2) return sfail(HS_ERR_INVALID, "null input level");
  SL_HIP(hipSetDevice(s->device));
  const size_t area = (size_t)s->W * s->H;
  const size_t n1 = (size_t)(s->W >> 1) * (s->H >> 1), n2 = (size_t)(s->W >> 2) * (s->H >> 2);
  SL_HIP(hipMemcpyAsync(s->d_dI, dirpyr0, area * 3 * sizeof(float), hipMemcpyHostToDevice, s->stream));
  // absSquaredGrad[0] feeds makeHists: a new upload invalidates the cached histograms of this frame id only if
  // the caller changes the frame id, as the reference (gradHistFrame)
  SL_HIP(hipMemcpyAsync(s->d_g[0], absg0, area * sizeof(float), hipMemcpyHostToDevice, s->stream));
  SL_HIP(hipMemcpyAsync(s->d_g[1], absg1, n1 * sizeof(float), hipMemcpyHostToDevice, s->stream));
  SL_HIP(hipMemcpyAsync(s->d_g[2], absg2, n2 * sizeof(float), hipMemcpyHostToDevice, s->stream));
  SL_HIP(hipEventRecord(s->e0, s->stream));
  s->last_passes = 0;
  int n = 0;
  SL_TRY(make_maps(s, s->d_dI, 3, frame_id, density, recursions_left, th_factor, &n));
  return finish(s, map_out, n_selected, n);
}

extern "C" int hs_selector_make_maps_raw(hs_selector* s, int frame_id, const float* img, float density,
                                         int recursions_left, float th_factor, float* map_out, int* n_selected) {
  SL_TRY(check_args(s, density, th_factor));
  if (!img) return sfail(HS_ERR_INVALID, "null image");
  SL_HIP(hipSetDevice(s->device));
  const size_t area = (size_t)s->W * s->H;
  SL_HIP(hipMemcpyAsync(s->d_raw, img, area * sizeof(float), hipMemcpyHostToDevice, s->stream));
  SL_HIP(hipEventRecord(s->e0, s->stream));
  SL_HIP(hs_build_dir_pyramid(s->stream, s->d_raw, s->W, s->H, 3, s->d_lvl, s->d_g));
  s->last_passes = 0;
  int n = 0;
  SL_TRY(make_maps(s, reinterpret_cast<const float*>(s->d_lvl[0]), 4, frame_id, density, recursions_left, th_factor,
                   &n));
  return finish(s, map_out, n_selected, n);
}

extern "C" int hs_selector_get_potential(hs_selector* s, int* potential) {
  if (!s || !potential) return sfail(HS_ERR_INVALID, "null argument");
  *potential = s->currentPotential;
  return HS_OK;
}

extern "C" int hs_selector_set_potential(hs_selector* s, int potential) {
  if (!s) return sfail(HS_ERR_INVALID, "null selector");
  if (potential < 1) return sfail(HS_ERR_INVALID, "potential must be >= 1");
  s->currentPotential = potential;
  return HS_OK;
}

extern "C" int hs_selector_last_stats(hs_selector* s, double* ms, int* passes) {
  if (!s) return sfail(HS_ERR_INVALID, "null selector");
  if (ms) *ms = s->last_ms;
  if (passes) *passes = s->last_passes;
  return HS_OK;
}
