// micro-benchmark (gfx950, one workgroup): dependent-latency and issue costs of the instruction kinds on the
// solve kernel's critical path.  cycles = s_memtime ticks per op, loop overhead amortised over 32 unrolled ops
#include <hip/hip_runtime.h>
#include <cstdio>
#define U32(x) x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x
__device__ __forceinline__ double rl(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), lane);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__global__ void k(double* out, long long* cyc, int n, int mode) {
  __shared__ double lds[1024];
  const int t = threadIdx.x;
  double a = out[t], b = 1.0000001, c0 = a, c1 = a + 1, c2 = a + 2, c3 = a + 3;
  float f = (float)a;
  lds[t] = a;
  int idx = t;
  __shared__ int ilds[1024];
  ilds[t] = (t * 7 + 1) & 1023;
  __syncthreads();
  long long t0 = clock64();
  for (int i = 0; i < n; i++) {
    switch (mode) {
      case 0: U32(c0 = __builtin_fma(c0, b, 1e-9);) break;                                   // f64 fma dep
      case 1: U32(c0 = __builtin_fma(c0, b, 1e-9); c1 = __builtin_fma(c1, b, 1e-9);
                  c2 = __builtin_fma(c2, b, 1e-9); c3 = __builtin_fma(c3, b, 1e-9);) break;  // 4 indep
      case 2: U32(f = __builtin_fmaf(f, 1.0000001f, 1e-9f);) break;                          // f32 fma dep
      case 3: U32(c0 = c0 * b;) break;                                                        // f64 mul dep
      case 4: U32(c0 = __builtin_amdgcn_rcp(c0);) break;                                      // rcp_f64 dep
      case 5: U32(idx = ilds[idx];) break;                                                    // LDS b32 dep
      case 6: U32(c0 = lds[(int)c0 & 1023] + 1.0;) break;                                     // LDS b64 + add
      case 7: U32(c0 = rl(c0, 5) + 1.0;) break;                                               // readlane f64 + add
      case 8: U32(c0 = 1.0 / c0;) break;                                                      // IEEE f64 div
      case 9: U32(c0 = __shfl_xor(c0, 1) + 1.0;) break;                                       // shfl f64 + add
    }
  }
  long long t1 = clock64();
  out[t] = c0 + c1 + c2 + c3 + f + idx;
  if (t == 0) cyc[0] = t1 - t0;
}
int main() {
  double* d; long long* c;
  (void)hipMalloc(&d, 1024 * 8); (void)hipMalloc(&c, 8); (void)hipMemset(d, 0, 1024 * 8);
  const char* names[] = {"f64 fma dependent", "f64 fma 4 independent (per fma)", "f32 fma dependent", "f64 mul dependent",
                         "v_rcp_f64 dependent", "ds_read_b32 dependent", "ds_read_b64 + f64 add dependent",
                         "readlane f64 + f64 add dependent", "IEEE f64 1/x dependent", "shfl_xor f64 + add dependent"};
  const int per[] = {32, 128, 32, 32, 32, 32, 32, 32, 32, 32};
  for (int mode = 0; mode < 10; mode++)
    for (int thr : {64, 256}) {
      const int n = 200;
      long long cy = 0;
      for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(k, dim3(1), dim3(thr), 0, 0, d, c, n, mode);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(&cy, c, 8, hipMemcpyDeviceToHost);
      }
      printf("%-36s threads %3d: %6.1f cycles/op\n", names[mode], thr, (double)cy / (n * per[mode]));
    }
  return 0;
}
