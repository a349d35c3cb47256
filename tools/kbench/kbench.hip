// Kernel micro-benchmark for the scatter pass (development tool, not the product).
// Includes the product kernels and adds experimental variants; every variant
// is checked bit-exact against the product k_scatter before it is timed.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/kbench/kbench.hip -o kbench
//   ./kbench [log2_n]
#include "../../distributed-lsb_amd/csrc/lsb_kernels.hip"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace lsb;

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

namespace lsb {
namespace {

__global__ void k_diff(const Elem* __restrict__ a, const Elem* __restrict__ b, int64_t m,
                       unsigned long long* bad) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += stride)
    if (a[i].key != b[i].key || a[i].val != b[i].val) atomicAdd(bad, 1ull);
}

template <int BLOCK, int IPT>
__global__ __launch_bounds__(BLOCK) void k_copy8(const Elem* __restrict__ in, Elem* __restrict__ out,
                                                 int64_t m) {
  const int64_t base = (int64_t)blockIdx.x * BLOCK * IPT + threadIdx.x;
  Elem e[IPT];
#pragma unroll
  for (int i = 0; i < IPT; ++i) e[i] = load_elem(in + base + i * BLOCK);
#pragma unroll
  for (int i = 0; i < IPT; ++i) store_elem(out + base + i * BLOCK, e[i]);
}

__global__ void k_copy(const Elem* __restrict__ in, Elem* __restrict__ out, int64_t m) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += stride)
    store_elem(out + i, load_elem(in + i));
}

// Variant scatter: BLOCK threads, IPT items/thread, optional register
// prefetch of the next tile, optional sequential output (diagnostic only).
template <int BLOCK, int IPT, bool PREFETCH, bool SEQ_OUT, int MINW>
__global__ __launch_bounds__(BLOCK, MINW) void k_scatter_v(const Elem* __restrict__ in,
                                                        Elem* __restrict__ out, int64_t m,
                                                        int shift, int64_t chunk_elems, int G,
                                                        const uint64_t* __restrict__ chunk_off,
                                                        const uint64_t* __restrict__ totals) {
  constexpr int W = BLOCK / 64;
  constexpr int T = BLOCK * IPT;
  __shared__ Elem stage[T];
  __shared__ uint32_t wcnt[W][kBuckets];
  __shared__ int64_t delta[kBuckets];
  __shared__ uint64_t scan64[W];
  __shared__ uint32_t scan32[W];

  const int t = threadIdx.x;
  const int w = t >> 6;
  const uint32_t lane = lane_id();
  const int c = blockIdx.x;
  const int64_t beg = (int64_t)c * chunk_elems;
  const int64_t end = beg + chunk_elems < m ? beg + chunk_elems : m;

  uint64_t run = 0;
  {
    const uint64_t tot = t < kBuckets ? totals[t] : 0ull;
    uint64_t all;
    const uint64_t bstart = block_exclusive_scan<BLOCK>(tot, scan64, &all);
    if (t < kBuckets) run = bstart + chunk_off[(int64_t)t * G + c];
  }
  const int wbase = w * 64 * IPT + (int)lane;

  Elem nx[IPT];
  if (PREFETCH && beg < end) {
    const int nv = (int)((end - beg) < T ? (end - beg) : T);
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      const int li = wbase + i * 64;
      nx[i] = li < nv ? load_elem(in + beg + li) : Elem{0ull, 0ull};
    }
  }

  for (int64_t tb = beg; tb < end; tb += T) {
    const int nvalid = (int)((end - tb) < T ? (end - tb) : T);
#pragma unroll
    for (int j = 0; j < kBuckets / 64; ++j) wcnt[w][lane + 64 * j] = 0;

    Elem e[IPT];
    if (PREFETCH) {
#pragma unroll
      for (int i = 0; i < IPT; ++i) e[i] = nx[i];
      const int64_t nb = tb + T;
      if (nb < end) {
        const int nv = (int)((end - nb) < T ? (end - nb) : T);
#pragma unroll
        for (int i = 0; i < IPT; ++i) {
          const int li = wbase + i * 64;
          nx[i] = li < nv ? load_elem(in + nb + li) : Elem{0ull, 0ull};
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < IPT; ++i) {
        const int li = wbase + i * 64;
        e[i] = li < nvalid ? load_elem(in + tb + li) : Elem{0ull, 0ull};
      }
    }

    uint32_t rk[IPT];
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      const bool valid = wbase + i * 64 < nvalid;
      const uint32_t d = (uint32_t)(e[i].key >> shift) & (kBuckets - 1);
      const uint64_t mt = match_digit8(d, __ballot(valid));
      const uint32_t below = mbcnt(mt);
      const uint32_t pre = wcnt[w][d];
      rk[i] = pre + below;
      if (valid && below == 0) wcnt[w][d] = pre + (uint32_t)__popcll(mt);
    }
    __syncthreads();

    uint32_t cnt = 0;
    if (t < kBuckets) {
#pragma unroll
      for (int ww = 0; ww < W; ++ww) {
        const uint32_t x = wcnt[ww][t];
        wcnt[ww][t] = cnt;
        cnt += x;
      }
    }
    uint32_t tile_total;
    const uint32_t lstart = block_exclusive_scan<BLOCK>(cnt, scan32, &tile_total);
    if (t < kBuckets) {
#pragma unroll
      for (int ww = 0; ww < W; ++ww) wcnt[ww][t] += lstart;
      delta[t] = (int64_t)run - (int64_t)lstart;
      run += cnt;
    }
    __syncthreads();

#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      if (wbase + i * 64 < nvalid) {
        const uint32_t d = (uint32_t)(e[i].key >> shift) & (kBuckets - 1);
        stage[wcnt[w][d] + rk[i]] = e[i];
      }
    }
    __syncthreads();

#pragma unroll
    for (int k = 0; k < IPT; ++k) {
      const int j = t + k * BLOCK;
      if (j < nvalid) {
        const Elem x = stage[j];
        const uint32_t d = (uint32_t)(x.key >> shift) & (kBuckets - 1);
        store_elem(out + (SEQ_OUT ? tb + j : delta[d] + j), x);
      }
    }
    __syncthreads();
  }
}

}  // namespace
}  // namespace lsb

struct Buf {
  Elem *in = nullptr, *out = nullptr, *ref = nullptr;
  uint32_t* hist = nullptr;
  uint64_t *off = nullptr, *tot = nullptr;
};

template <typename F>
float time_ms(F&& launch, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  launch();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a, 0));
  for (int r = 0; r < reps; ++r) launch();
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char** argv) {
  const int lg = argc > 1 ? atoi(argv[1]) : 30;
  const int64_t m = (int64_t)1 << lg;
  const int shift = argc > 2 ? atoi(argv[2]) : 0;
  Buf b;
  CK(hipMalloc(&b.in, m * sizeof(Elem)));
  CK(hipMalloc(&b.out, m * sizeof(Elem)));
  CK(hipMalloc(&b.ref, m * sizeof(Elem)));
  CK(hipMalloc(&b.hist, sizeof(uint32_t) * kBuckets * kMaxChunks));
  CK(hipMalloc(&b.off, sizeof(uint64_t) * kBuckets * kMaxChunks));
  CK(hipMalloc(&b.tot, sizeof(uint64_t) * kBuckets));
  KeyGen gen;
  if (argc > 3 && atoi(argv[3]) == 1) gen.dist = kDistZipf;
  CK(launch_pcg_fill(b.in, m, 0, 0, gen, 0));
  CK(hipDeviceSynchronize());
  const int reps = 5;
  const double gb = 32.0 * m / 1e9;

  float ms = time_ms([&] { hipLaunchKernelGGL(k_copy, dim3(4096), dim3(256), 0, 0, b.in, b.out, m); }, reps);
  printf("copy                      %8.3f ms  %7.1f GB/s\n", ms, gb / ms * 1e3);

  unsigned long long* bad;
  CK(hipMalloc(&bad, sizeof(unsigned long long)));
  typedef void (*KFn)(const Elem*, Elem*, int64_t, int, int64_t, int, const uint64_t*, const uint64_t*);
  // reference result: the no-carry variant (the round-1 product kernel)
  {
    Chunking ch = make_chunking(m, 512);
    CK(launch_upsweep(b.in, m, shift, ch, b.hist, nullptr, 0));
    CK(launch_scan(b.hist, ch.num_chunks, b.off, b.tot, 0));
    KFn k0 = k_scatter_v<256, 16, false, false, 2>;
    float t = time_ms([&] { hipLaunchKernelGGL(k0, dim3(ch.num_chunks), dim3(256), 0, 0, b.in, b.ref, m, shift, ch.chunk_elems, ch.num_chunks, b.off, b.tot); }, reps);
    printf("no-carry k_scatter_v       %8.3f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    float tp = time_ms([&] { CK(launch_scatter(b.in, b.out, m, shift, ch, b.off, b.tot, nullptr, 0)); }, reps);
    CK(hipMemset(bad, 0, sizeof(unsigned long long)));
    hipLaunchKernelGGL(k_diff, dim3(4096), dim3(256), 0, 0, b.out, b.ref, m, bad);
    unsigned long long h = 0;
    CK(hipMemcpy(&h, bad, sizeof h, hipMemcpyDeviceToHost));
    printf("product k_scatter (carry)  %8.3f ms  %7.1f GB/s  %s\n", tp, gb / tp * 1e3, h == 0 ? "OK" : "MISMATCH");
    float tu = time_ms([&] { CK(launch_upsweep(b.in, m, shift, ch, b.hist, nullptr, 0)); }, reps);
    printf("product k_upsweep          %8.3f ms  %7.1f GB/s (16 B/elt)\n", tu, 16.0 * m / 1e9 / tu * 1e3);
  }

  auto run_variant = [&](const char* name, int max_chunks, KFn kern, int block, int tile, bool check) {
    Chunking ch;
    const int64_t tiles = (m + tile - 1) / tile;
    const int64_t tpc = (tiles + max_chunks - 1) / max_chunks;
    ch.chunk_elems = tpc * tile;
    ch.num_chunks = (int)((m + ch.chunk_elems - 1) / ch.chunk_elems);
    CK(launch_upsweep(b.in, m, shift, ch, b.hist, nullptr, 0));
    CK(launch_scan(b.hist, ch.num_chunks, b.off, b.tot, 0));
    float t = time_ms([&] {
      hipLaunchKernelGGL(kern, dim3(ch.num_chunks), dim3(block), 0, 0, b.in, b.out, m, shift,
                         ch.chunk_elems, ch.num_chunks, b.off, b.tot);
    }, reps);
    CK(hipGetLastError());
    CK(hipMemset(bad, 0, sizeof(unsigned long long)));
    hipLaunchKernelGGL(k_diff, dim3(4096), dim3(256), 0, 0, b.out, b.ref, m, bad);
    unsigned long long h = 0;
    CK(hipMemcpy(&h, bad, sizeof h, hipMemcpyDeviceToHost));
    printf("%-26s %8.3f ms  %7.1f GB/s  chunks=%d %s\n", name, t, gb / t * 1e3, ch.num_chunks,
           !check ? "(unchecked)" : (h == 0 ? "OK" : "MISMATCH"));
    fflush(stdout);
  };

  run_variant("v256x16 pf SEQ", 512, k_scatter_v<256, 16, true, true, 2>, 256, 4096, false);
  {
    float ms = time_ms([&] { hipLaunchKernelGGL((k_copy8<256, 8>), dim3((unsigned)(m / 2048)), dim3(256), 0, 0, b.in, b.out, m); }, reps);
    printf("copy8 (8 loads in flight)  %8.3f ms  %7.1f GB/s\n", ms, gb / ms * 1e3);
  }
  return 0;
}
