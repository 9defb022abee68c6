// micro-benchmark (gfx950): what instruction fetch costs a single-workgroup kernel with long straight-line code.
// `big` is one wave executing NI independent-ish v_add_f32 (4 B each, NI * 4 B of straight-line code, no loop);
// `other` is a different straight-line kernel of the same size (evicts `big` from the instruction cache / L2 it ran
// on).  Printed: shader cycles (s_memtime) per launch of `big` in these orders:
//   warm  : big(1 WG) right after big(1 WG)        -- the dispatcher may still pick another CU / XCD
//   wide  : big(1 WG) right after big on every CU  -- every CU's instruction cache holds the code
//   cold  : big(1 WG) right after `other` on every CU
// Ideal (cache hits): NI x 4 cycles (one wave alone issues a v_add_f32 every 4 cycles).
// build: hipcc --offload-arch=gfx950 -O3 -o icache icache.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define A1(op) asm volatile(op " %0, %0, %1" : "+v"(x) : "v"(y));
#define A4(op) A1(op) A1(op) A1(op) A1(op)
#define A16(op) A4(op) A4(op) A4(op) A4(op)
#define A64(op) A16(op) A16(op) A16(op) A16(op)
#define A256(op) A64(op) A64(op) A64(op) A64(op)
#define A1K(op) A256(op) A256(op) A256(op) A256(op)
#define A4K(op) A1K(op) A1K(op) A1K(op) A1K(op)

__global__ void big(float* out, long long* cyc) {
  float x = threadIdx.x, y = 1.0f;
  const long long t0 = __builtin_amdgcn_s_memtime();
  A4K("v_add_f32")
  A4K("v_add_f32")
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0 && blockIdx.x == 0) cyc[0] = t1 - t0;
  if (x == -1.f) out[threadIdx.x] = x;
}
__global__ void other(float* out, long long* cyc) {
  float x = threadIdx.x, y = 1.0f;
  const long long t0 = __builtin_amdgcn_s_memtime();
  A4K("v_mul_f32")
  A4K("v_mul_f32")
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0 && blockIdx.x == 0) cyc[1] = t1 - t0;
  if (x == -1.f) out[threadIdx.x] = x;
}

int main() {
  float* out;
  long long* cyc;
  hipMalloc(&out, 4096);
  hipMalloc(&cyc, 64);
  long long h[2];
  auto run = [&](const char* name, int pre, int pre_blocks) {
    std::vector<long long> v;
    for (int r = 0; r < 20; r++) {
      if (pre == 1) hipLaunchKernelGGL(big, dim3(pre_blocks), dim3(64), 0, 0, out, cyc + 2);
      if (pre == 2) hipLaunchKernelGGL(other, dim3(pre_blocks), dim3(64), 0, 0, out, cyc + 2);
      hipLaunchKernelGGL(big, dim3(1), dim3(64), 0, 0, out, cyc);
      hipMemcpy(h, cyc, 16, hipMemcpyDeviceToHost);
      v.push_back(h[0]);
    }
    long long mn = v[0], mx = v[0], s = 0;
    for (auto c : v) { mn = c < mn ? c : mn; mx = c > mx ? c : mx; s += c; }
    std::printf("%-6s cycles per big launch: min %lld  mean %lld  max %lld  (ideal ~%d)\n", name, mn, s / (long long)v.size(),
                mx, 8192 * 4);
  };
  run("warm", 1, 1);
  run("wide", 1, 2048);
  run("cold", 2, 2048);
  run("none", 0, 0);
  return 0;
}
