// Misaligned synthetic LSD write pattern, tiles processed in global order by
// concurrent blocks: (a) consecutive tiles on consecutive blocks (different
// XCDs under round-robin dispatch) vs (b) XCD-striped: consecutive tiles on
// blocks with equal blockIdx % 8 (same XCD), as a onesweep with per-XCD tile
// queues would run them.  (development tool)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)
struct alignas(16) E { uint64_t k, v; };
template <int MODE>  // 0 = round-robin order, 1 = XCD-striped
__global__ __launch_bounds__(256) void k_runs(const E* __restrict__ in, E* __restrict__ out, int64_t m,
                                              int run_log2, int64_t steps, int shift) {
  const int64_t region = m >> 8;
  const int64_t T = (int64_t)256 << run_log2;
  const int64_t ntiles = m / T;
  const int G = gridDim.x;
  for (int64_t j = 0; j < steps; ++j) {
    int64_t tile;
    if (MODE == 0) tile = blockIdx.x + j * G;
    else { const int x = blockIdx.x % 8, i = blockIdx.x / 8; tile = j * G + (int64_t)x * (G / 8) + i; }
    if (tile >= ntiles) break;
    for (int64_t p0 = 0; p0 < T; p0 += 1024) {
      E e[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) e[i] = in[tile * T + p0 + i * 256 + threadIdx.x];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t p = p0 + i * 256 + threadIdx.x;
        const int64_t bucket = p >> run_log2, idx = p & ((1 << run_log2) - 1);
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
int main() {
  const int64_t m = (int64_t)1 << 30;
  E *in, *out; CK(hipMalloc(&in, m * sizeof(E))); CK(hipMalloc(&out, m * sizeof(E)));
  CK(hipMemset(in, 1, m * sizeof(E)));
  const double gb = 32.0 * m / 1e9;
  for (int rl : {4, 5}) for (int G : {512, 1024}) for (int shift : {0, 3}) {
    const int64_t T = (int64_t)256 << rl, ntiles = m / T, steps = (ntiles + G - 1) / G;
    float a = time_ms([&] { hipLaunchKernelGGL(k_runs<0>, dim3(G), dim3(256), 0, 0, in, out, m, rl, steps, shift); }, 3);
    float b = time_ms([&] { hipLaunchKernelGGL(k_runs<1>, dim3(G), dim3(256), 0, 0, in, out, m, rl, steps, shift); }, 3);
    printf("run=%2d G=%4d shift=%d  round-robin %7.3f ms %5.0f GB/s | xcd-striped %7.3f ms %5.0f GB/s\n",
           1 << rl, G, shift, a, gb / a * 1e3, b, gb / b * 1e3);
    fflush(stdout);
  }
  return 0;
}
