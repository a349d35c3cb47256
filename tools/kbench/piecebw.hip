// Is a record buffer's write speed a property of its 1 GiB physical pieces?
// (DESIGN.md §4 "Record buffers": with 1 GiB VMM pieces one pass direction
// can still run ~4 % slow on some boxes, r05/v10.)  NP pieces are created
// (hipMemCreate) and each is mapped on its own; every piece's streaming
// write and read are timed REPS times, rounds interleaved, to see whether a
// piece's speed is stable.  Then two buffers of K pieces are built from the
// fastest writers and two from the slowest, and the LSD-pattern copy
// (tools/kbench/vmmbw.hip's k_runs) is timed both ways within each pair.
//
//   hipcc -O3 --offload-arch=gfx950 tools/kbench/piecebw.hip -o tools/kbench/piecebw
//   tools/kbench/piecebw [NP=48] [K=16] [REPS=4]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <numeric>
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
  if (x == 0x1234567ull) sink[0] = x;
}

__global__ __launch_bounds__(256) void k_write(u64x2* __restrict__ out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    out[i] = u64x2{(unsigned long long)i, 1ull};
}

// Each 4096-record tile of `in` sends a 256-B run to each of 256 bucket
// frontiers of `out` (an LSD pass's write pattern without the sort).
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
  const int NP = argc > 1 ? atoi(argv[1]) : 48;
  const int K = argc > 2 ? atoi(argv[2]) : 16;
  const int REPS = argc > 3 ? atoi(argv[3]) : 4;
  const size_t piece = (size_t)1 << 30;
  const int64_t pn = (int64_t)(piece / 16);
  int dev = 0;
  CK(hipGetDevice(&dev));
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = dev;
  hipMemAccessDesc acc = {};
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  std::vector<hipMemGenericAllocationHandle_t> h(NP);
  std::vector<u64x2*> va(NP);
  for (int p = 0; p < NP; ++p) {
    CK(hipMemCreate(&h[p], piece, &prop, 0));
    void* v = nullptr;
    CK(hipMemAddressReserve(&v, piece, piece, nullptr, 0));
    CK(hipMemMap(v, piece, 0, h[p], 0));
    CK(hipMemSetAccess(v, piece, &acc, 1));
    va[p] = reinterpret_cast<u64x2*>(v);
  }
  unsigned long long* sink;
  CK(hipMalloc(&sink, 8));
  hipEvent_t a0, a1;
  CK(hipEventCreate(&a0));
  CK(hipEventCreate(&a1));
  const unsigned grid = 8192;
  auto time = [&](auto launch) {
    CK(hipEventRecord(a0, 0));
    launch();
    CK(hipEventRecord(a1, 0));
    CK(hipEventSynchronize(a1));
    float ms;
    CK(hipEventElapsedTime(&ms, a0, a1));
    return ms;
  };
  for (int p = 0; p < NP; ++p) hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, va[p], pn);
  CK(hipDeviceSynchronize());
  std::vector<std::vector<float>> wr(NP), rd(NP);
  for (int r = 0; r < REPS; ++r)
    for (int p = 0; p < NP; ++p) {
      wr[p].push_back(time([&] { hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, va[p], pn); }));
      rd[p].push_back(time([&] { hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, va[p], pn, sink); }));
    }
  std::vector<double> wmean(NP);
  for (int p = 0; p < NP; ++p) {
    wmean[p] = std::accumulate(wr[p].begin(), wr[p].end(), 0.0) / REPS;
    printf("piece %2d: write", p);
    for (float x : wr[p]) printf(" %.4f", x);
    printf("  read");
    for (float x : rd[p]) printf(" %.4f", x);
    printf("  ms\n");
  }
  std::vector<int> ord(NP);
  std::iota(ord.begin(), ord.end(), 0);
  std::sort(ord.begin(), ord.end(), [&](int x, int y) { return wmean[x] < wmean[y]; });
  // Buffers: F0, F1 from the 2K fastest writers (alternating), S0, S1 from the 2K slowest.
  auto build = [&](std::vector<int> ids) {
    void* v = nullptr;
    CK(hipMemAddressReserve(&v, piece * ids.size(), piece, nullptr, 0));
    for (size_t j = 0; j < ids.size(); ++j)
      CK(hipMemMap(static_cast<char*>(v) + j * piece, piece, 0, h[ids[j]], 0));
    CK(hipMemSetAccess(v, piece * ids.size(), &acc, 1));
    return reinterpret_cast<u64x2*>(v);
  };
  if (NP < 4 * K) {
    printf("need NP >= 4K for the pair test\n");
    return 0;
  }
  std::vector<int> f0, f1, s0, s1;
  for (int j = 0; j < 2 * K; ++j) (j % 2 ? f1 : f0).push_back(ord[j]);
  for (int j = 0; j < 2 * K; ++j) (j % 2 ? s1 : s0).push_back(ord[NP - 1 - j]);
  u64x2* F0 = build(f0);
  u64x2* F1 = build(f1);
  u64x2* S0 = build(s0);
  u64x2* S1 = build(s1);
  const int64_t n = pn * K;
  double fw = 0, sw = 0;
  for (int j = 0; j < 2 * K; ++j) {
    fw += wmean[ord[j]];
    sw += wmean[ord[NP - 1 - j]];
  }
  printf("fastest %d pieces: mean write %.4f ms; slowest %d: %.4f ms\n", 2 * K, fw / (2 * K), 2 * K, sw / (2 * K));
  for (int r = 0; r < REPS; ++r) {
    const float ff = time([&] { hipLaunchKernelGGL(k_runs, dim3(grid), dim3(256), 0, 0, F0, F1, n); });
    const float fb = time([&] { hipLaunchKernelGGL(k_runs, dim3(grid), dim3(256), 0, 0, F1, F0, n); });
    const float sf = time([&] { hipLaunchKernelGGL(k_runs, dim3(grid), dim3(256), 0, 0, S0, S1, n); });
    const float sb = time([&] { hipLaunchKernelGGL(k_runs, dim3(grid), dim3(256), 0, 0, S1, S0, n); });
    printf("runs copy of %d GiB: fast pair %.3f / %.3f ms, slow pair %.3f / %.3f ms\n", K, ff, fb, sf, sb);
  }
  printf("SUMMARY piecebw NP %d K %d\n", NP, K);
  return 0;
}
