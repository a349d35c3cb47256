// Misaligned synthetic radix pattern: like runs.hip but every run is shifted by
// SHIFT records, so run boundaries split 128-B lines between consecutive tiles.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)
struct alignas(16) E { uint64_t k, v; };
template <bool ORDERED>
__global__ __launch_bounds__(256) void k_runs(const E* __restrict__ in, E* __restrict__ out, int64_t m,
                                              int run_log2, int64_t tiles_per_block, int shift) {
  const int64_t region = m >> 8;
  const int64_t T = (int64_t)256 << run_log2;
  const int64_t ntiles = m / T;
  for (int64_t j = 0; j < tiles_per_block; ++j) {
    const int64_t tile = ORDERED ? blockIdx.x + j * gridDim.x : blockIdx.x * tiles_per_block + j;
    if (tile >= ntiles) break;
    for (int64_t p0 = 0; p0 < T; p0 += 1024) {
      E e[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) e[i] = in[tile * T + p0 + i * 256 + threadIdx.x];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t p = p0 + i * 256 + threadIdx.x;
        const int64_t bucket = p >> run_log2;
        const int64_t idx = p & ((1 << run_log2) - 1);
        int64_t g = bucket * region + (tile << run_log2) + idx + shift;
        if (g >= m) g -= m;
        out[g] = e[i];
      }
    }
  }
}
template <typename F> float time_ms(F&& f, int reps) {
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f(); CK(hipDeviceSynchronize()); CK(hipEventRecord(a, 0));
  for (int r = 0; r < reps; ++r) f();
  CK(hipEventRecord(b, 0)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b)); return ms / reps;
}
int main(int argc, char** argv) {
  const int64_t m = (int64_t)1 << 30;
  E *in, *out; CK(hipMalloc(&in, m * sizeof(E))); CK(hipMalloc(&out, m * sizeof(E)));
  CK(hipMemset(in, 1, m * sizeof(E)));
  const double gb = 32.0 * m / 1e9;
  for (int rl : {4, 5, 6}) for (int shift : {0, 1, 2, 4, 7, 8}) {
    const int64_t T = (int64_t)256 << rl, ntiles = m / T;
    const int grid = 512;
    const int64_t tpb = (ntiles + grid - 1) / grid;
    float o = time_ms([&] { hipLaunchKernelGGL(k_runs<true>, dim3(grid), dim3(256), 0, 0, in, out, m, rl, tpb, shift); }, 3);
    float c = time_ms([&] { hipLaunchKernelGGL(k_runs<false>, dim3(grid), dim3(256), 0, 0, in, out, m, rl, tpb, shift); }, 3);
    printf("run=%4d elems shift=%d (%3d B)  ordered %7.3f ms %6.0f GB/s | chunked %7.3f ms %6.0f GB/s\n",
           1 << rl, shift, shift * 16, o, gb / o * 1e3, c, gb / c * 1e3);
    fflush(stdout);
  }
  return 0;
}
