// Does a deterministic physical layout (HIP virtual memory management) remove
// the pair-dependent speed of 16 GiB record buffers?  (VERDICT r04 item 1;
// DESIGN.md §4 "Spread".)  tools/kbench/allocbw.hip showed that an LSD-pass
// write pattern between two hipMalloc'd buffers runs at 6.86 ms for most
// ordered pairs but 7.2-7.3 ms for some pairs, in both directions.  Here the
// NB buffers come from one of several allocators and every ordered pair is
// timed with the same copy (k_runs: each 4096-record tile of X sends a
// 256-B run to each of 256 bucket frontiers of Y).
//
//   hipcc -O3 --offload-arch=gfx950 tools/kbench/vmmbw.hip -o tools/kbench/vmmbw
//   tools/kbench/vmmbw MODE [NB=4] [LG=30] [REPS=5] [CHUNK_MIB=0: recommended]
// MODE 0  hipMalloc per buffer
//      1  VMM: one physical handle per buffer, mapped whole
//      2  VMM: CHUNK handles per buffer, created buffer by buffer, mapped in order
//      3  VMM: CHUNK handles created round-robin across the buffers (A0 B0 .. A1 B1 ..)
//      4  VMM: as 2, each buffer's chunks mapped in a shuffled order
//      5  VMM: all buffers' chunks created first, then dealt at random to (buffer, slot)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
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
  const int MODE = argc > 1 ? atoi(argv[1]) : 0;
  const int NB = argc > 2 ? atoi(argv[2]) : 4;
  const int LG = argc > 3 ? atoi(argv[3]) : 30;
  const int REPS = argc > 4 ? atoi(argv[4]) : 5;
  const size_t chunk_mib = argc > 5 ? (size_t)atoll(argv[5]) : 0;
  const int64_t n = (int64_t)1 << LG;
  const size_t bytes = (size_t)n * 16;
  int dev = 0;
  CK(hipGetDevice(&dev));
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = dev;
  size_t gmin = 0, grec = 0;
  CK(hipMemGetAllocationGranularity(&gmin, &prop, hipMemAllocationGranularityMinimum));
  CK(hipMemGetAllocationGranularity(&grec, &prop, hipMemAllocationGranularityRecommended));
  size_t chunk = chunk_mib ? chunk_mib << 20 : grec;
  if (MODE == 1) chunk = bytes;
  if (chunk % gmin || bytes % chunk) {
    printf("chunk %zu not a multiple of the granularity %zu or not dividing %zu\n", chunk, gmin, bytes);
    return 1;
  }
  const size_t per_buf = bytes / chunk;
  printf("mode %d nb %d lg %d granularity min %zu KiB recommended %zu KiB chunk %zu MiB (%zu per buffer)\n",
         MODE, NB, LG, gmin >> 10, grec >> 10, chunk >> 20, per_buf);
  std::vector<u64x2*> buf(NB);
  std::vector<hipMemGenericAllocationHandle_t> handles;
  std::mt19937_64 rng(12345);
  hipEvent_t a0, a1;
  CK(hipEventCreate(&a0));
  CK(hipEventCreate(&a1));
  auto t0 = std::chrono::steady_clock::now();
  if (MODE == 0) {
    for (int i = 0; i < NB; ++i) CK(hipMalloc(&buf[i], bytes));
  } else {
    for (int i = 0; i < NB; ++i) {
      void* va = nullptr;
      CK(hipMemAddressReserve(&va, bytes, std::max(grec, (size_t)1 << 21), nullptr, 0));
      buf[i] = reinterpret_cast<u64x2*>(va);
    }
    // (buffer, slot) of each handle in creation order
    std::vector<std::pair<int, size_t>> dst;
    if (MODE == 1 || MODE == 2 || MODE == 4) {
      for (int i = 0; i < NB; ++i) {
        std::vector<size_t> slots(per_buf);
        for (size_t s = 0; s < per_buf; ++s) slots[s] = s;
        if (MODE == 4) std::shuffle(slots.begin(), slots.end(), rng);
        for (size_t s = 0; s < per_buf; ++s) dst.push_back({i, slots[s]});
      }
    } else if (MODE == 3) {
      for (size_t s = 0; s < per_buf; ++s)
        for (int i = 0; i < NB; ++i) dst.push_back({i, s});
    } else {
      for (int i = 0; i < NB; ++i)
        for (size_t s = 0; s < per_buf; ++s) dst.push_back({i, s});
      std::shuffle(dst.begin(), dst.end(), rng);
    }
    for (auto& d : dst) {
      hipMemGenericAllocationHandle_t h;
      CK(hipMemCreate(&h, chunk, &prop, 0));
      handles.push_back(h);
      CK(hipMemMap(reinterpret_cast<char*>(buf[d.first]) + d.second * chunk, chunk, 0, h, 0));
    }
    hipMemAccessDesc acc = {};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    for (int i = 0; i < NB; ++i) CK(hipMemSetAccess(buf[i], bytes, &acc, 1));
  }
  const double alloc_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  printf("allocated %d buffers in %.3f s\n", NB, alloc_s);
  unsigned long long* sink;
  CK(hipMalloc(&sink, 8));
  for (int i = 0; i < NB; ++i) {
    CK(hipMemset(buf[i], i + 1, bytes));
    printf("buffer %d at %p\n", i, (void*)buf[i]);
  }
  CK(hipDeviceSynchronize());
  const unsigned grid = 8192;
  auto timed = [&](auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    float best = 1e30f, sum = 0.f;
    for (int r = 0; r < REPS; ++r) {
      CK(hipEventRecord(a0, 0));
      launch();
      CK(hipEventRecord(a1, 0));
      CK(hipEventSynchronize(a1));
      float ms;
      CK(hipEventElapsedTime(&ms, a0, a1));
      best = ms < best ? ms : best;
      sum += ms;
    }
    return std::make_pair(best, sum / REPS);
  };
  for (int i = 0; i < NB; ++i) {
    auto rd = timed([&] { hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, buf[i], n, sink); });
    auto wr = timed([&] { hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, buf[i], n); });
    printf("buffer %d: read %.3f ms  write %.3f ms  [mean %.3f / %.3f]\n", i, rd.first, wr.first, rd.second,
           wr.second);
  }
  float lo = 1e30f, hi = 0.f;
  for (int x = 0; x < NB; ++x)
    for (int y = 0; y < NB; ++y) {
      if (x == y) continue;
      auto cp = timed([&] { hipLaunchKernelGGL(k_runs, dim3(grid), dim3(256), 0, 0, buf[x], buf[y], n); });
      printf("runs %d -> %d: %.3f ms [mean %.3f]\n", x, y, cp.first, cp.second);
      lo = std::min(lo, cp.second);
      hi = std::max(hi, cp.second);
    }
  printf("SUMMARY mode %d chunk %zu MiB alloc %.3f s pair means %.3f .. %.3f ms\n", MODE, chunk >> 20, alloc_s,
         lo, hi);
  fflush(stdout);
  if (MODE == 0) {
    for (int i = 0; i < NB; ++i) CK(hipFree(buf[i]));
  } else {
    for (int i = 0; i < NB; ++i) CK(hipMemUnmap(buf[i], bytes));
    for (auto h : handles) CK(hipMemRelease(h));
    for (int i = 0; i < NB; ++i) CK(hipMemAddressFree(buf[i], bytes));
  }
  return 0;
}
