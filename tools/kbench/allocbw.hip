// Does where a 16 GiB record buffer lands change how fast it streams?
// (development tool for the k_onesweep spread; VERDICT r03
// item 2).  NB buffers of 2^LG 16-byte records are allocated one after
// another in this fresh process; for each buffer a pure streaming read and
// a pure streaming write are timed, and for every ordered pair (X, Y) a copy
// X -> Y with k_onesweep's write pattern: each 4096-record tile of X sends a
// 16-record (256 B) run to each of 256 bucket frontiers of Y, so 256 write
// streams advance together as in an LSD pass (sequential reads).  A layout
// effect shows as a buffer or a pair that is consistently slower.
//
//   hipcc -O3 --offload-arch=gfx950 tools/kbench/allocbw.hip -o tools/kbench/allocbw
//   tools/kbench/allocbw [NB=4] [LG=30] [REPS=5] [POOL=0]
// POOL=1: one hipMalloc of NB buffers, cut into NB slices (+ POOL_PAD bytes
// between them, env, default 0) instead of NB hipMallocs.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                        \
  do {                                                               \
    hipError_t e = (x);                                              \
    if (e != hipSuccess) {                                           \
      printf("%s: %s\n", #x, hipGetErrorString(e));                  \
      exit(1);                                                       \
    }                                                                \
  } while (0)

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void k_read(const u64x2* __restrict__ in, int64_t n,
                                              unsigned long long* __restrict__ sink) {
  unsigned long long x = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const u64x2 v = __builtin_nontemporal_load(in + i);
    x ^= v.x ^ v.y;
  }
  if (x == 0x1234567ull) sink[0] = x;  // keeps the loads
}

__global__ __launch_bounds__(256) void k_write(u64x2* __restrict__ out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    out[i] = u64x2{(unsigned long long)i, 1ull};
}

// Record i = (tile t, slot j) of X goes to bucket b = j / 16 of Y at
// frontier b * (n / 256) + t * 16 + j % 16: 256 B runs, 256 frontiers.
__global__ __launch_bounds__(256) void k_runs(const u64x2* __restrict__ in, u64x2* __restrict__ out,
                                              int64_t n) {
  const int64_t per_bucket = n / 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t t = i >> 12;
    const int j = (int)(i & 4095);
    out[(int64_t)(j >> 4) * per_bucket + t * 16 + (j & 15)] = __builtin_nontemporal_load(in + i);
  }
}

int main(int argc, char** argv) {
  const int NB = argc > 1 ? atoi(argv[1]) : 4;
  const int LG = argc > 2 ? atoi(argv[2]) : 30;
  const int REPS = argc > 3 ? atoi(argv[3]) : 5;
  const int POOL = argc > 4 ? atoi(argv[4]) : 0;
  const int64_t pad = getenv("POOL_PAD") ? atoll(getenv("POOL_PAD")) : 0;
  const int64_t n = (int64_t)1 << LG;
  const size_t bytes = (size_t)n * 16;
  std::vector<u64x2*> buf(NB);
  if (POOL) {
    char* p = nullptr;
    CK(hipMalloc(&p, (bytes + pad) * NB));
    for (int i = 0; i < NB; ++i) buf[i] = reinterpret_cast<u64x2*>(p + (bytes + pad) * i);
  } else {
    for (int i = 0; i < NB; ++i) CK(hipMalloc(&buf[i], bytes));
  }
  unsigned long long* sink;
  CK(hipMalloc(&sink, 8));
  for (int i = 0; i < NB; ++i) {
    CK(hipMemset(buf[i], i + 1, bytes));
    printf("buffer %d at %p (va mod 1 GiB = %llu MiB, mod 2 MiB = %llu KiB)\n", i, (void*)buf[i],
           (unsigned long long)(((uintptr_t)buf[i] & ((1ull << 30) - 1)) >> 20),
           (unsigned long long)(((uintptr_t)buf[i] & ((1ull << 21) - 1)) >> 10));
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const unsigned grid = 8192;
  auto timed = [&](auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    float best = 1e30f, sum = 0.f;
    for (int r = 0; r < REPS; ++r) {
      CK(hipEventRecord(e0, 0));
      launch();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
      sum += ms;
    }
    return std::make_pair(best, sum / REPS);
  };
  for (int i = 0; i < NB; ++i) {
    auto rd = timed([&] { hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, buf[i], n, sink); });
    auto wr = timed([&] { hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, buf[i], n); });
    printf("buffer %d: read %.3f ms (%.0f GB/s)  write %.3f ms (%.0f GB/s)  [mean %.3f / %.3f]\n", i,
           rd.first, bytes / (rd.first * 1e-3) / 1e9, wr.first, bytes / (wr.first * 1e-3) / 1e9, rd.second,
           wr.second);
    fflush(stdout);
  }
  for (int x = 0; x < NB; ++x)
    for (int y = 0; y < NB; ++y) {
      if (x == y) continue;
      auto cp = timed([&] { hipLaunchKernelGGL(k_runs, dim3(grid), dim3(256), 0, 0, buf[x], buf[y], n); });
      printf("runs %d -> %d: %.3f ms (%.0f GB/s read + write) [mean %.3f]\n", x, y, cp.first,
             2.0 * bytes / (cp.first * 1e-3) / 1e9, cp.second);
      fflush(stdout);
    }
  return 0;
}
