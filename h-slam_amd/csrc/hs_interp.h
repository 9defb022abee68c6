// hs_interp.h — the reference's image interpolators (Include/GlobalTypes.h:355-401) on float4 level-0 images
// (I, dI/dx, dI/dy, 0), shared by the immature-point kernels.  Include inside a file compiled with
// `#pragma clang fp contract(off)`: the operation order is the reference's.
#pragma once
#include <hip/hip_runtime.h>

#pragma clang fp contract(off)

namespace hs_img {

// texel base ix + iy*W clamped to [0, W*H - W - 2]: identical to the reference for every in-buffer read
// (row-wrapped ones included); the reference's out-of-buffer reads (UB) land on the nearest valid base.
__device__ __forceinline__ int clamp_base(int ix, int iy, int W, int H) {
  const long b = (long)ix + (long)iy * W;
  const long hi = (long)W * H - W - 2;
  return (int)(b < 0 ? 0 : (b > hi ? hi : b));
}

// getInterpolatedElement31 (Include/GlobalTypes.h:390-401): intensity channel only
__device__ __forceinline__ float interp31(const float4* __restrict__ img, float x, float y, int W, int H) {
  const int ix = (int)x, iy = (int)y;
  const float dx = x - ix, dy = y - iy, dxdy = dx * dy;
  const float* bp = reinterpret_cast<const float*>(img + clamp_base(ix, iy, W, H));
  const float p00 = bp[0], p10 = bp[4], p01 = bp[4 * W], p11 = bp[4 * W + 4];
  return dxdy * p11 + (dy - dxdy) * p01 + (dx - dxdy) * p10 + (1 - dx - dy + dxdy) * p00;
}

// getInterpolatedElement33 (Include/GlobalTypes.h:377-388)
__device__ __forceinline__ float3 interp33(const float4* __restrict__ img, float x, float y, int W, int H) {
  const int ix = (int)x, iy = (int)y;
  const float dx = x - ix, dy = y - iy, dxdy = dx * dy;
  const float4* bp = img + clamp_base(ix, iy, W, H);
  const float4 p00 = bp[0], p10 = bp[1], p01 = bp[W], p11 = bp[W + 1];
  const float w11 = dxdy, w01 = dy - dxdy, w10 = dx - dxdy, w00 = 1 - dx - dy + dxdy;
  float3 r;
  r.x = w11 * p11.x + w01 * p01.x + w10 * p10.x + w00 * p00.x;
  r.y = w11 * p11.y + w01 * p01.y + w10 * p10.y + w00 * p00.y;
  r.z = w11 * p11.z + w01 * p01.z + w10 * p10.z + w00 * p00.z;
  return r;
}

// getInterpolatedElement33BiLin (Include/GlobalTypes.h:355-375)
__device__ __forceinline__ float3 interp33BiLin(const float4* __restrict__ img, float x, float y, int W, int H) {
  const int ix = (int)x, iy = (int)y;
  const float4* bp = img + clamp_base(ix, iy, W, H);
  const float tl = bp[0].x, tr = bp[1].x, bl = bp[W].x, br = bp[W + 1].x;
  const float dx = x - ix, dy = y - iy;
  const float topInt = dx * tr + (1 - dx) * tl;
  const float botInt = dx * br + (1 - dx) * bl;
  const float leftInt = dy * bl + (1 - dy) * tl;
  const float rightInt = dy * br + (1 - dy) * tr;
  float3 r;
  r.x = dx * rightInt + (1 - dx) * leftInt;
  r.y = rightInt - leftInt;
  r.z = botInt - topInt;
  return r;
}

}  // namespace hs_img
