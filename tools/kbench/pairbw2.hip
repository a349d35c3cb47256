// Where does the slow LSD pass direction come from?  (tools/kbench/pairbw.hip
// found it depends on which pieces two buffers hold, not on their order.)
// With NB buffers of K 1 GiB VMM pieces each, plus SPARE pieces:
//   1. the LSD-pattern copy for every ordered pair (Ui -> Uj): a slow column
//      means a destination property, a slow row a source property;
//   2. for the slowest pair, each destination piece in turn swapped for a
//      spare: does one piece carry it?
//   3. every pair again with 15/16 of the records and the bucket starts
//      (a) packed (spacing not a power of two), (b) at the power-of-two
//      spacing with gaps, (c) at (b) plus a random offset below the gap:
//      is it the spacing of the 256 write frontiers?
//
//   hipcc -O3 --offload-arch=gfx950 tools/kbench/pairbw2.hip -o tools/kbench/pairbw2
//   tools/kbench/pairbw2 [NB=6] [K=8] [SPARE=8] [REPS=3]
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

__global__ __launch_bounds__(256) void k_write(u64x2* __restrict__ out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    out[i] = u64x2{(unsigned long long)i, 1ull};
}

// k_runs with bucket b's run starting at start[b] (n / 256 records each).
__global__ __launch_bounds__(256) void k_runs_at(const u64x2* __restrict__ in, u64x2* __restrict__ out,
                                                 int64_t n, const int64_t* __restrict__ start) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t t = i >> 12;
    const int j = (int)(i & 4095);
    out[start[j >> 4] + t * 16 + (j & 15)] = __builtin_nontemporal_load(in + i);
  }
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
  const int NB = argc > 1 ? atoi(argv[1]) : 6;
  const int K = argc > 2 ? atoi(argv[2]) : 8;
  const int SPARE = argc > 3 ? atoi(argv[3]) : 8;
  const int REPS = argc > 4 ? atoi(argv[4]) : 3;
  if (NB < 2 || K < 1 || SPARE < 1) return 1;
  const int NP = NB * K + SPARE;
  const size_t piece = (size_t)1 << 30;
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
  for (int p = 0; p < NP; ++p) CK(hipMemCreate(&h[p], piece, &prop, 0));
  auto build = [&](const std::vector<int>& ids) {
    void* v = nullptr;
    CK(hipMemAddressReserve(&v, piece * ids.size(), piece, nullptr, 0));
    for (size_t j = 0; j < ids.size(); ++j) {
      char* base = static_cast<char*>(v) + j * piece;
      CK(hipMemMap(base, piece, 0, h[ids[j]], 0));
    }
    CK(hipMemSetAccess(v, piece * ids.size(), &acc, 1));
    return reinterpret_cast<u64x2*>(v);
  };
  hipEvent_t a0, a1;
  CK(hipEventCreate(&a0));
  CK(hipEventCreate(&a1));
  const unsigned grid = 8192;
  const int64_t n = (int64_t)(piece / 16) * K;
  auto runs = [&](const u64x2* in, u64x2* out) {
    double s = 0;
    for (int r = 0; r < REPS; ++r) {
      CK(hipEventRecord(a0, 0));
      hipLaunchKernelGGL(k_runs, dim3(grid), dim3(256), 0, 0, in, out, n);
      CK(hipEventRecord(a1, 0));
      CK(hipEventSynchronize(a1));
      float ms;
      CK(hipEventElapsedTime(&ms, a0, a1));
      s += ms / REPS;
    }
    return s;
  };
  std::vector<std::vector<int>> sets(NB);
  std::vector<u64x2*> U(NB);
  for (int i = 0; i < NB; ++i) {
    for (int j = 0; j < K; ++j) sets[i].push_back(i * K + j);
    U[i] = build(sets[i]);
    hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, U[i], n);
  }
  CK(hipDeviceSynchronize());

  // 1. every ordered pair.
  std::vector<std::vector<double>> m(NB, std::vector<double>(NB, 0));
  int si = 0, sj = 1;
  printf("LSD-pattern copy of %d GiB, ms (row = source, column = destination)\n      ", K);
  for (int j = 0; j < NB; ++j) printf("   U%d  ", j);
  printf("\n");
  for (int i = 0; i < NB; ++i) {
    printf("U%d   ", i);
    for (int j = 0; j < NB; ++j) {
      if (i == j) {
        printf("   -   ");
        continue;
      }
      m[i][j] = runs(U[i], U[j]);
      printf(" %.3f ", m[i][j]);
      if (m[i][j] > m[si][sj]) si = i, sj = j;
    }
    printf("\n");
  }
  printf("slowest: U%d -> U%d %.3f ms (back %.3f)\n", si, sj, m[si][sj], m[sj][si]);

  // 2. each destination piece swapped for a spare.
  for (int q = 0; q < K; ++q) {
    std::vector<int> d = sets[sj];
    d[q] = NB * K + (q % SPARE);
    u64x2* D = build(d);
    printf("dest piece %d (id %d) -> spare %d: %.3f ms\n", q, sets[sj][q], d[q], runs(U[si], D));
  }
  // 2b. the source's pieces swapped for spares, all at once (is it the pair?).
  {
    std::vector<int> s2;
    for (int q = 0; q < K; ++q) s2.push_back(NB * K + (q % SPARE));
    u64x2* S2 = build(s2);
    hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, S2, n);
    CK(hipDeviceSynchronize());
    printf("spare source -> U%d: %.3f ms;  U%d -> U%d again: %.3f ms\n", sj, runs(S2, U[sj]), si, sj,
           runs(U[si], U[sj]));
  }
  // 3. 15/16 of the records; bucket starts packed / power-of-two / jittered.
  const int64_t full = n, n15 = n / 16 * 15, per = n15 / 256, slot = full / 256;
  int64_t* st;
  CK(hipMalloc(&st, 3 * 256 * sizeof(int64_t)));
  std::vector<int64_t> hs(3 * 256);
  unsigned long long rs = 0x9e3779b97f4a7c15ull;
  for (int b = 0; b < 256; ++b) {
    hs[b] = b * per;
    hs[256 + b] = b * slot;
    rs = rs * 6364136223846793005ull + 1442695040888963407ull;
    hs[512 + b] = b * slot + (int64_t)((rs >> 33) % (uint64_t)((slot - per) / 16)) * 16;
  }
  CK(hipMemcpy(st, hs.data(), hs.size() * sizeof(int64_t), hipMemcpyHostToDevice));
  auto runs_at = [&](const u64x2* in, u64x2* out, int v) {
    double s = 0;
    for (int r = 0; r < REPS; ++r) {
      CK(hipEventRecord(a0, 0));
      hipLaunchKernelGGL(k_runs_at, dim3(grid), dim3(256), 0, 0, in, out, n15, st + 256 * v);
      CK(hipEventRecord(a1, 0));
      CK(hipEventSynchronize(a1));
      float ms;
      CK(hipEventElapsedTime(&ms, a0, a1));
      s += ms / REPS;
    }
    return s;
  };
  const char* vn[3] = {"packed", "pow2", "jitter"};
  for (int v = 0; v < 3; ++v) {
    printf("15/16 of the records, starts %s (row = source, column = destination)\n", vn[v]);
    for (int i = 0; i < NB; ++i) {
      printf("U%d   ", i);
      for (int j = 0; j < NB; ++j) {
        if (i == j) {
          printf("   -   ");
          continue;
        }
        printf(" %.3f ", runs_at(U[i], U[j], v));
      }
      printf("\n");
    }
  }
  printf("SUMMARY pairbw2 NB %d K %d\n", NB, K);
  return 0;
}
