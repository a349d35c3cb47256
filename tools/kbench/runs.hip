// Synthetic radix-scatter pattern: how does HBM throughput depend on the run
// length each tile writes per bucket?  (development tool)
// Reads 16-B records sequentially; tile t (T = 256 * RUN records) sends its
// i-th run of RUN records to bucket region i at offset t * RUN — the write
// pattern of an LSD pass over uniform digits, with no ranking work.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

struct alignas(16) E { uint64_t k, v; };

// ORDERED: tile index = blockIdx.x + j * gridDim.x (all blocks sweep together).
template <int IPT, bool ORDERED, bool NT>
__global__ __launch_bounds__(256) void k_runs(const E* __restrict__ in, E* __restrict__ out, int64_t m,
                                              int run_log2, int64_t tiles_per_block) {
  const int64_t region = m >> 8;  // 256 buckets
  const int64_t T = (int64_t)256 << run_log2;
  const int64_t ntiles = m / T;
  for (int64_t j = 0; j < tiles_per_block; ++j) {
    const int64_t tile = ORDERED ? blockIdx.x + j * gridDim.x : blockIdx.x * tiles_per_block + j;
    if (tile >= ntiles) break;
    for (int64_t p0 = 0; p0 < T; p0 += 256 * IPT) {
      E e[IPT];
#pragma unroll
      for (int i = 0; i < IPT; ++i) e[i] = in[tile * T + p0 + i * 256 + threadIdx.x];
#pragma unroll
      for (int i = 0; i < IPT; ++i) {
        const int64_t p = p0 + i * 256 + threadIdx.x;
        const int64_t bucket = p >> run_log2;
        const int64_t idx = p & ((1 << run_log2) - 1);
        E* dst = out + bucket * region + (tile << run_log2) + idx;
        if (NT) {
          __builtin_nontemporal_store(e[i].k, &dst->k);
          __builtin_nontemporal_store(e[i].v, &dst->v);
        } else {
          *dst = e[i];
        }
      }
    }
  }
}

template <typename F>
float time_ms(F&& f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f(); CK(hipDeviceSynchronize());
  CK(hipEventRecord(a, 0));
  for (int r = 0; r < reps; ++r) f();
  CK(hipEventRecord(b, 0)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char** argv) {
  const int lg = argc > 1 ? atoi(argv[1]) : 30;
  const int64_t m = (int64_t)1 << lg;
  E *in, *out;
  CK(hipMalloc(&in, m * sizeof(E)));
  CK(hipMalloc(&out, m * sizeof(E)));
  CK(hipMemset(in, 1, m * sizeof(E)));
  const double gb = 32.0 * m / 1e9;
  for (int rl : {2, 3, 4, 5, 6, 7, 8, 10, 12}) {
    const int64_t T = (int64_t)256 << rl;
    const int64_t ntiles = m / T;
    for (int grid : {512, 2048}) {
      const int64_t tpb = (ntiles + grid - 1) / grid;
      float o = time_ms([&] { hipLaunchKernelGGL((k_runs<4, true, false>), dim3(grid), dim3(256), 0, 0, in, out, m, rl, tpb); }, 3);
      float c = time_ms([&] { hipLaunchKernelGGL((k_runs<4, false, false>), dim3(grid), dim3(256), 0, 0, in, out, m, rl, tpb); }, 3);
      float n = time_ms([&] { hipLaunchKernelGGL((k_runs<4, true, true>), dim3(grid), dim3(256), 0, 0, in, out, m, rl, tpb); }, 3);
      printf("run=%5d elems (%6d B) grid=%4d  ordered %7.3f ms %6.0f GB/s | chunked %7.3f ms %6.0f GB/s | ordered+nt %7.3f ms %6.0f GB/s\n",
             1 << rl, 16 << rl, grid, o, gb / o * 1e3, c, gb / c * 1e3, n, gb / n * 1e3);
      fflush(stdout);
    }
  }
  return 0;
}
