// hs_pyr_kernels.h — device image pyramid (Frame::CreateDirPyrs) kernels and the shared host launcher.
#pragma once
#include <hip/hip_runtime.h>

__global__ void hs_k_pyr_load(int n, const float* img, float4* lvl0);
__global__ void hs_k_pyr_down(int wl, int hl, int wlm1, const float4* src, float4* dst);
__global__ void hs_k_pyr_grad(int wl, int hl, float4* lvl, float* absg);

// Builds levels 0 .. nlev-1 (sizes w >> l, h >> l: CalibData's wpyr / hpyr rule) of the direct pyramid from the
// device fp32 image d_img (W*H) into d_lvl[l] (float4 texels), absSquaredGrad into d_absg[l] when non-null.
// Enqueued on `stream`; returns the first launch error.
hipError_t hs_build_dir_pyramid(hipStream_t stream, const float* d_img, int W, int H, int nlev, float4* const* d_lvl,
                                float* const* d_absg);

// levels 1 .. nlev-1 from a level 0 already in d_lvl[0] (its intensities; the texels' gradients are not read)
hipError_t hs_build_dir_pyramid_upper(hipStream_t stream, int W, int H, int nlev, float4* const* d_lvl);
