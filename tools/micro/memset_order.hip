// memset_order.hip — does a null-stream hipMemset order against a kernel on a hipStreamNonBlocking stream?
//
// The BA context allocated every device buffer with dalloc (hipMalloc + hipMemset on the null stream) and then ran
// hs_k_fix_frames on its own non-blocking stream.  This measures the mechanism directly instead of re-running the
// flaky test: a large zero fill and then a small one go to the null stream (dalloc's order: d_img_all first, the
// adjoints late), a one-lane kernel on a non-blocking stream stores a marker into the small buffer, and after a
// device sync the host reads the marker back.  A zero there means the null-stream fill landed after the kernel's
// store: the "adjoints zero, precalc right" failure.
//   variant 0: hipMemset (null stream) then kernel on the non-blocking stream           (the round-5 code)
//   variant 1: hipMemsetAsync on the kernel's own stream                                (the fix)
//   variant 2: hipMemset then hipStreamSynchronize(nullptr) before the kernel           (the alternative fix)
// Also reports whether hipMemset returned before the fill completed (hipStreamQuery(nullptr) right after it).
// build: hipcc --offload-arch=gfx950 -O2 memset_order.hip -o memset_order
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

__global__ void mark(int* p, int v) {
  if (threadIdx.x == 0) p[0] = v;
}

int main(int argc, char** argv) {
  const size_t big = (argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 512) << 20;  // MiB of the large fill
  const int trials = argc > 2 ? std::atoi(argv[2]) : 20;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (int variant = 0; variant < 3; variant++) {
    int zeros = 0, pending = 0;
    for (int t = 0; t < trials; t++) {
      void* a = nullptr;
      int* b = nullptr;
      CK(hipMalloc(&a, big));
      CK(hipMalloc((void**)&b, 256));
      CK(hipDeviceSynchronize());
      if (variant == 1) {
        CK(hipMemsetAsync(a, 0, big, s));
        CK(hipMemsetAsync(b, 0, 256, s));
      } else {
        CK(hipMemset(a, 0, big));
        CK(hipMemset(b, 0, 256));
        if (hipStreamQuery(nullptr) == hipErrorNotReady) pending++;
        if (variant == 2) CK(hipStreamSynchronize(nullptr));
      }
      hipLaunchKernelGGL(mark, dim3(1), dim3(64), 0, s, b, 42);
      CK(hipGetLastError());
      CK(hipDeviceSynchronize());
      int h = -1;
      CK(hipMemcpy(&h, b, sizeof(int), hipMemcpyDeviceToHost));
      if (h != 42) zeros++;
      CK(hipFree(a));
      CK(hipFree(b));
    }
    std::printf("{\"variant\": %d, \"what\": \"%s\", \"fill_MiB\": %zu, \"trials\": %d, "
                "\"marker_overwritten\": %d, \"memset_returned_before_done\": %d}\n",
                variant,
                variant == 0 ? "hipMemset null stream, kernel on non-blocking stream"
                : variant == 1 ? "hipMemsetAsync on the kernel's stream"
                               : "hipMemset + hipStreamSynchronize(nullptr)",
                big >> 20, trials, zeros, pending);
  }
  CK(hipStreamDestroy(s));
  return 0;
}
