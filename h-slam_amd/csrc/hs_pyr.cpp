// hs_pyr.cpp — host launcher of the device image pyramid and the standalone C-ABI entry (include/hs_pyr.h).
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "../../include/hs_ba.h"
#include "../../include/hs_pyr.h"
#include "hs_pyr_kernels.h"

namespace hs {
extern thread_local std::string g_err;
}

hipError_t hs_build_dir_pyramid(hipStream_t stream, const float* d_img, int W, int H, int nlev, float4* const* d_lvl,
                                float* const* d_absg) {
  const int n0 = W * H;
  hipLaunchKernelGGL(hs_k_pyr_load, dim3((n0 + 255) / 256), dim3(256), 0, stream, n0, d_img, d_lvl[0]);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  for (int l = 0; l < nlev; l++) {
    const int wl = W >> l, hl = H >> l, n = wl * hl;
    if (l > 0) {
      hipLaunchKernelGGL(hs_k_pyr_down, dim3((n + 255) / 256), dim3(256), 0, stream, wl, hl, W >> (l - 1), d_lvl[l - 1],
                         d_lvl[l]);
      if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    hipLaunchKernelGGL(hs_k_pyr_grad, dim3((n + 255) / 256), dim3(256), 0, stream, wl, hl, d_lvl[l],
                       d_absg ? d_absg[l] : nullptr);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t hs_build_dir_pyramid_upper(hipStream_t stream, int W, int H, int nlev, float4* const* d_lvl) {
  hipError_t e = hipSuccess;
  for (int l = 1; l < nlev; l++) {
    const int wl = W >> l, hl = H >> l, n = wl * hl;
    hipLaunchKernelGGL(hs_k_pyr_down, dim3((n + 255) / 256), dim3(256), 0, stream, wl, hl, W >> (l - 1), d_lvl[l - 1],
                       d_lvl[l]);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(hs_k_pyr_grad, dim3((n + 255) / 256), dim3(256), 0, stream, wl, hl, d_lvl[l], nullptr);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  return e;
}

namespace {
int pfail(int code, const std::string& msg) {
  hs::g_err = msg;
  return code;
}
}  // namespace

#define PY_HIP(x)                                                                                   \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) { rc = pfail(HS_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); goto done; } \
  } while (0)

extern "C" int hs_dir_pyramid(int device_id, int width, int height, int n_levels, const float* img, float* dirpyr_out,
                              float* abs_squared_grad_out) {
  if (!img) return pfail(HS_ERR_INVALID, "null image");
  if (n_levels < 1 || n_levels > HS_MAX_LEVELS || width < 4 || height < 4 || (width >> (n_levels - 1)) < 2 ||
      (height >> (n_levels - 1)) < 2)
    return pfail(HS_ERR_INVALID, "bad pyramid size");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return pfail(HS_ERR_HIP, "no HIP device");
  if (device_id < 0 || device_id >= ndev) return pfail(HS_ERR_INVALID, "bad device id");
  int rc = HS_OK;
  hipStream_t s = nullptr;
  float* d_img = nullptr;
  float4* lv[HS_MAX_LEVELS] = {nullptr};
  float* ag[HS_MAX_LEVELS] = {nullptr};
  size_t off3 = 0, off1 = 0;
  std::vector<float4> tex;
  PY_HIP(hipSetDevice(device_id));
  PY_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  PY_HIP(hipMalloc((void**)&d_img, sizeof(float) * width * height));
  for (int l = 0; l < n_levels; l++) {
    const size_t n = (size_t)(width >> l) * (height >> l);
    PY_HIP(hipMalloc((void**)&lv[l], n * sizeof(float4)));
    PY_HIP(hipMalloc((void**)&ag[l], n * sizeof(float)));
  }
  PY_HIP(hipMemcpyAsync(d_img, img, sizeof(float) * width * height, hipMemcpyHostToDevice, s));
  PY_HIP(hs_build_dir_pyramid(s, d_img, width, height, n_levels, lv, ag));
  for (int l = 0; l < n_levels; l++) {
    const size_t n = (size_t)(width >> l) * (height >> l);
    tex.resize(n);
    PY_HIP(hipMemcpyAsync(tex.data(), lv[l], n * sizeof(float4), hipMemcpyDeviceToHost, s));
    if (abs_squared_grad_out)
      PY_HIP(hipMemcpyAsync(abs_squared_grad_out + off1, ag[l], n * sizeof(float), hipMemcpyDeviceToHost, s));
    PY_HIP(hipStreamSynchronize(s));
    if (dirpyr_out)
      for (size_t i = 0; i < n; i++) {
        dirpyr_out[off3 + 3 * i] = tex[i].x;
        dirpyr_out[off3 + 3 * i + 1] = tex[i].y;
        dirpyr_out[off3 + 3 * i + 2] = tex[i].z;
      }
    off3 += 3 * n;
    off1 += n;
  }
done:
  if (s) (void)hipStreamSynchronize(s);
  for (int l = 0; l < HS_MAX_LEVELS; l++) {
    if (lv[l]) (void)hipFree(lv[l]);
    if (ag[l]) (void)hipFree(ag[l]);
  }
  if (d_img) (void)hipFree(d_img);
  if (s) (void)hipStreamDestroy(s);
  return rc;
}
