// Streaming bandwidth by working-set size (development tool):
// ping-pong copies A -> B -> A of S bytes each, repeated, so that for small S
// both buffers stay in the 256 MiB Infinity Cache (MALL) or in the L2s.
// Reports read + write bytes per second for S = 8 MiB ... 4 GiB.
//
//   hipcc -O3 --offload-arch=gfx950 tools/kbench/mallbw.hip -o tools/kbench/mallbw && tools/kbench/mallbw
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void k_copy(const u64x2* __restrict__ in, u64x2* __restrict__ out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    out[i] = in[i];
}

int main() {
  const int64_t max_bytes = (int64_t)4 << 30;
  u64x2 *a, *b;
  CK(hipMalloc(&a, max_bytes));
  CK(hipMalloc(&b, max_bytes));
  CK(hipMemset(a, 1, max_bytes));
  CK(hipMemset(b, 2, max_bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int64_t s = (int64_t)8 << 20; s <= max_bytes; s *= 2) {
    const int64_t n = s / 16;
    const int reps = (int)(((int64_t)64 << 30) / s) + 2;  // ~64 GiB moved per size
    const unsigned grid = (unsigned)(n / 256 < 8192 ? (n + 255) / 256 : 8192);
    for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, a, b, n);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int r = 0; r < reps; ++r) {
      if (r & 1) hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, b, a, n);
      else hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, a, b, n);
    }
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double per = ms / reps;
    printf("S = %7.1f MiB  %8.4f ms per copy  %7.0f GB/s (read + write)\n", s / 1048576.0, per,
           2.0 * s / (per * 1e-3) / 1e9);
    fflush(stdout);
  }
  return 0;
}
