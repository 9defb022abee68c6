// micro-benchmark (gfx950): latency of a wave-to-wave hand-off through LDS inside one workgroup (writer stamps
// s_memtime, stores a double; a reader polls it and stamps when it sees it), vs an s_barrier hand-off.
// build: hipcc --offload-arch=gfx950 -O3 -o handoff handoff.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#define HS_LDS __attribute__((address_space(3)))
constexpr unsigned long long kSent = 0x7FF4DEADBEEF0000ull;
__device__ __forceinline__ bool uni_sent(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readfirstlane((int)(b & 0xffffffffll));
  const int hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
  return ((((unsigned long long)(unsigned int)hi) << 32) | (unsigned int)lo) == kSent;
}
__device__ __forceinline__ void fence() { asm volatile("" ::: "memory"); }

template <int MODE>  // 0: others idle at the final barrier, 1: others sleep-poll, 2: others tight-poll, 3: s_barrier
__global__ __launch_bounds__(512) void k(long long* out, int reps) {
  __shared__ double flag[64];
  __shared__ double dummy[64];
  const int tid = threadIdx.x, w = __builtin_amdgcn_readfirstlane(tid >> 6), i = tid & 63;
  const double s = __longlong_as_double((long long)kSent);
  if (tid < 64) { flag[tid] = s; dummy[tid] = s; }
  __syncthreads();
  const HS_LDS double* F = (const HS_LDS double*)flag;
  const HS_LDS double* Dm = (const HS_LDS double*)dummy;
  long long tw = 0, tr = 0, acc = 0;
  double x = 1.0 + i;
  for (int r = 0; r < reps; r++) {
    if (MODE == 3) {
      if (w == 0) {
        for (int q = 0; q < 50; q++) x = __builtin_fma(x, 1.0000001, 1e-9);
        tw = clock64();
      }
      __syncthreads();
      if (w == 1) { tr = clock64(); acc += tr - __builtin_amdgcn_readfirstlane((int)0) * 0; }
      if (w == 0 && i == 0) out[r * 2] = tw;
      if (w == 1 && i == 0) out[r * 2 + 1] = tr;
      __syncthreads();
      continue;
    }
    if (w == 0) {
      for (int q = 0; q < 50; q++) x = __builtin_fma(x, 1.0000001, 1e-9);
      tw = clock64();
      ((HS_LDS double*)flag)[r] = x;
      fence();
      if (i == 0) out[r * 2] = tw;
    } else if (w == 1) {
      for (int spin = 0; spin < (1 << 22); spin++) {
        fence();
        if (!uni_sent(F[r])) break;
      }
      tr = clock64();
      if (i == 0) out[r * 2 + 1] = tr;
    } else if (MODE == 1 || MODE == 2) {
      for (int spin = 0; spin < (1 << 22); spin++) {
        fence();
        if (!uni_sent(F[r])) break;
        if (MODE == 1) __builtin_amdgcn_s_sleep(1);
        else x += Dm[(spin + i) & 63] * 0.0;
      }
    }
  }
  __syncthreads();
  if (tid == 0) out[2 * reps] = (long long)x;
}
int main() {
  long long* d;
  (void)hipMalloc(&d, 8 * 256);
  const char* names[] = {"LDS flag, others idle", "LDS flag, 6 others sleep-poll", "LDS flag, 6 others tight-poll",
                         "s_barrier"};
  for (int mode = 0; mode < 4; mode++) {
    long long h[129];
    for (int rep = 0; rep < 3; rep++) {
      switch (mode) {
        case 0: hipLaunchKernelGGL(k<0>, dim3(1), dim3(512), 0, 0, d, 32); break;
        case 1: hipLaunchKernelGGL(k<1>, dim3(1), dim3(512), 0, 0, d, 32); break;
        case 2: hipLaunchKernelGGL(k<2>, dim3(1), dim3(512), 0, 0, d, 32); break;
        default: hipLaunchKernelGGL(k<3>, dim3(1), dim3(512), 0, 0, d, 32); break;
      }
      (void)hipDeviceSynchronize();
    }
    (void)hipMemcpy(h, d, 8 * 65, hipMemcpyDeviceToHost);
    long long s = 0, mn = 1 << 30, mx = 0;
    for (int r = 1; r < 32; r++) {
      const long long v = h[2 * r + 1] - h[2 * r];
      s += v; mn = v < mn ? v : mn; mx = v > mx ? v : mx;
    }
    printf("%-32s hand-off cycles: mean %lld  min %lld  max %lld\n", names[mode], s / 31, mn, mx);
  }
  return 0;
}
