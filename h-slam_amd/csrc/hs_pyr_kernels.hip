// hs_pyr_kernels.hip — Frame::CreateDirPyrs (Src/Frame.cpp:104-181) on the device: the direct-image pyramid
// (I, dI/dx, dI/dy) of a frame built from its photometrically undistorted level-0 image (ImageData::fImgL,
// Include/DatasetLoader.h:436-506), so a frame crosses PCIe as W*H floats instead of levels x 12 B per pixel.
//   hs_k_pyr_load  level 0 intensities (texel w = 0; the gradients follow in hs_k_pyr_grad)
//   hs_k_pyr_down  level l from l-1: 0.25f * (((tl + tr) + bl) + br), the reference's operation order
//   hs_k_pyr_grad  central differences over the interior index range [w, w*(h-1)) of a level (row-wrapped at the
//                  left / right columns exactly as the reference's linear index loop), non-finite -> 0, and
//                  absSquaredGrad = dx*dx + dy*dy (the gamma weighting is skipped: Calib->PhotoUnDistL is null,
//                  SURVEY.md Appendix B quirk 4).  The first and last rows keep dI = 0 (the reference leaves
//                  them uninitialised).
#include <hip/hip_runtime.h>

#include "hs_pyr_kernels.h"

#pragma clang fp contract(off)

__global__ __launch_bounds__(256) void hs_k_pyr_load(int n, const float* __restrict__ img, float4* __restrict__ lvl0) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) lvl0[i] = make_float4(img[i], 0.f, 0.f, 0.f);
}

__global__ __launch_bounds__(256) void hs_k_pyr_down(int wl, int hl, int wlm1, const float4* __restrict__ src,
                                                     float4* __restrict__ dst) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= wl * hl) return;
  const int y = i / wl, x = i - y * wl;
  const float* s = reinterpret_cast<const float*>(src);
  const int b = 2 * x + 2 * y * wlm1;
  const float v = 0.25f * (((s[4 * b] + s[4 * (b + 1)]) + s[4 * (b + wlm1)]) + s[4 * (b + 1 + wlm1)]);
  dst[i] = make_float4(v, 0.f, 0.f, 0.f);
}

__global__ __launch_bounds__(256) void hs_k_pyr_grad(int wl, int hl, float4* __restrict__ lvl, float* __restrict__ absg) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= wl * hl) return;
  const float* s = reinterpret_cast<const float*>(lvl);
  const float I = s[4 * i];  // (the texel's own intensity: unchanged)
  float dx = 0.f, dy = 0.f, g = 0.f;
  const bool interior = i >= wl && i < wl * (hl - 1);
  if (interior) {
    dx = 0.5f * (s[4 * (i + 1)] - s[4 * (i - 1)]);
    dy = 0.5f * (s[4 * (i + wl)] - s[4 * (i - wl)]);
    if (!isfinite(dx)) dx = 0.f;
    if (!isfinite(dy)) dy = 0.f;
    g = dx * dx + dy * dy;
  }
  // threads read the neighbours' intensity lanes and write only their own gradient lanes (no overlap)
  (void)I;
  reinterpret_cast<float*>(lvl + i)[1] = dx;
  reinterpret_cast<float*>(lvl + i)[2] = dy;
  if (absg) absg[i] = g;
}
