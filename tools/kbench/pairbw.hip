// Which property of a record buffer's physical pieces makes one LSD pass
// direction slow?  tools/kbench/piecebw.hip (r05_piece2) found that a pair of
// buffers built from the fastest streaming writers can still run the LSD write
// pattern 20 % slower one way than the other, so streaming speed is not it.
// Here, with NP 1 GiB pieces (hipMemCreate):
//   A. every piece's LSD-pattern speed as a destination (source: the next piece)
//      and as a source (destination: the next piece), REPS rounds interleaved;
//   B. TRIALS pairs of K-piece buffers drawn at random, the LSD-pattern copy
//      timed both ways, beside the sums of A's per-piece figures;
//   C. for the most asymmetric pair, its slow destination remapped with its
//      pieces in PERMS other orders, to see whether order alone changes it.
//
//   hipcc -O3 --offload-arch=gfx950 tools/kbench/pairbw.hip -o tools/kbench/pairbw
//   tools/kbench/pairbw [NP=48] [K=8] [REPS=3] [TRIALS=8] [PERMS=4]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <numeric>
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
  const int K = argc > 2 ? atoi(argv[2]) : 8;
  const int REPS = argc > 3 ? atoi(argv[3]) : 3;
  const int TRIALS = argc > 4 ? atoi(argv[4]) : 8;
  const int PERMS = argc > 5 ? atoi(argv[5]) : 4;
  if (NP < 2 * K || K < 1) {
    printf("need NP >= 2K\n");
    return 1;
  }
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
  auto build = [&](const std::vector<int>& ids) {
    void* v = nullptr;
    CK(hipMemAddressReserve(&v, piece * ids.size(), piece, nullptr, 0));
    for (size_t j = 0; j < ids.size(); ++j)
      CK(hipMemMap(static_cast<char*>(v) + j * piece, piece, 0, h[ids[j]], 0));
    CK(hipMemSetAccess(v, piece * ids.size(), &acc, 1));
    return reinterpret_cast<u64x2*>(v);
  };
  std::vector<u64x2*> va(NP);
  for (int p = 0; p < NP; ++p) {
    CK(hipMemCreate(&h[p], piece, &prop, 0));
    va[p] = build({p});
  }
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
  auto runs = [&](const u64x2* in, u64x2* out, int64_t n) {
    return time([&] { hipLaunchKernelGGL(k_runs, dim3(grid), dim3(256), 0, 0, in, out, n); });
  };
  for (int p = 0; p < NP; ++p) hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, va[p], pn);
  CK(hipDeviceSynchronize());

  // A. per-piece LSD-pattern speed as destination and as source.
  std::vector<double> as_dst(NP, 0), as_src(NP, 0);
  for (int r = 0; r < REPS; ++r)
    for (int p = 0; p < NP; ++p) {
      const int q = (p + 1) % NP;
      as_dst[p] += runs(va[q], va[p], pn) / REPS;
      as_src[p] += runs(va[p], va[q], pn) / REPS;
    }
  for (int p = 0; p < NP; ++p) printf("piece %2d: as dst %.4f  as src %.4f ms\n", p, as_dst[p], as_src[p]);

  // B. random pairs of K-piece buffers.
  std::mt19937 rng(12345);
  std::vector<int> all(NP);
  std::iota(all.begin(), all.end(), 0);
  const int64_t n = pn * K;
  double worst = 0;
  std::vector<int> wx, wy;
  bool worst_fwd = true;
  for (int t = 0; t < TRIALS; ++t) {
    std::shuffle(all.begin(), all.end(), rng);
    std::vector<int> x(all.begin(), all.begin() + K), y(all.begin() + K, all.begin() + 2 * K);
    u64x2* X = build(x);
    u64x2* Y = build(y);
    double fwd = 0, bwd = 0;
    for (int r = 0; r < REPS; ++r) {
      fwd += runs(X, Y, n) / REPS;
      bwd += runs(Y, X, n) / REPS;
    }
    double dx = 0, dy = 0, sx = 0, sy = 0;
    for (int j = 0; j < K; ++j) {
      dx += as_dst[x[j]] / K;
      dy += as_dst[y[j]] / K;
      sx += as_src[x[j]] / K;
      sy += as_src[y[j]] / K;
    }
    printf("trial %d: X->Y %.3f  Y->X %.3f ms | piece means: X dst %.4f src %.4f, Y dst %.4f src %.4f\n", t,
           fwd, bwd, dx, sx, dy, sy);
    const double asym = std::max(fwd, bwd) / std::min(fwd, bwd);
    if (asym > worst) {
      worst = asym;
      wx = x;
      wy = y;
      worst_fwd = fwd > bwd;
    }
  }

  // C. the most asymmetric pair: the slow direction's destination in other orders.
  printf("worst asymmetry %.3f (%s)\n", worst, worst_fwd ? "X->Y slow" : "Y->X slow");
  std::vector<int> src = worst_fwd ? wx : wy, dst = worst_fwd ? wy : wx;
  u64x2* S = build(src);
  for (int k = 0; k <= PERMS; ++k) {
    if (k) std::shuffle(dst.begin(), dst.end(), rng);
    u64x2* D = build(dst);
    double sd = 0, ds = 0;
    for (int r = 0; r < REPS; ++r) {
      sd += runs(S, D, n) / REPS;
      ds += runs(D, S, n) / REPS;
    }
    printf("order %d: src->dst %.3f  dst->src %.3f ms  [", k, sd, ds);
    for (int j : dst) printf(" %d", j);
    printf(" ]\n");
  }
  printf("SUMMARY pairbw NP %d K %d\n", NP, K);
  return 0;
}
