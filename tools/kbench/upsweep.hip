// Upsweep (per-chunk digit histogram) variants vs a pure-read ceiling (dev tool).
#include "../../distributed-lsb_amd/csrc/lsb_kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace lsb;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

namespace lsb {
namespace {

// Plain LDS atomics into per-wave histograms (no match aggregation).
template <int BLOCK, int IPT, bool WIDE>
__global__ __launch_bounds__(BLOCK) void k_up_plain(const Elem* __restrict__ A, int64_t m, int shift,
                                                    int64_t chunk_elems, int G,
                                                    uint32_t* __restrict__ chunk_hist) {
  constexpr int W = BLOCK / 64;
  __shared__ uint32_t hist[W][kBuckets];
  for (int i = threadIdx.x; i < W * kBuckets; i += BLOCK) (&hist[0][0])[i] = 0;
  __syncthreads();
  const int w = threadIdx.x >> 6;
  const int c = blockIdx.x;
  const int64_t beg = (int64_t)c * chunk_elems;
  const int64_t end = beg + chunk_elems < m ? beg + chunk_elems : m;
  const uint64_t* __restrict__ keys = reinterpret_cast<const uint64_t*>(A);
  for (int64_t tb = beg; tb < end; tb += (int64_t)BLOCK * IPT) {
    uint64_t k[IPT];
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      const int64_t idx = tb + (int64_t)i * BLOCK + threadIdx.x;
      if (WIDE) k[i] = idx < end ? load_elem(A + idx).key : 0ull;
      else k[i] = idx < end ? keys[2 * idx] : 0ull;
    }
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      const int64_t idx = tb + (int64_t)i * BLOCK + threadIdx.x;
      if (idx < end) atomicAdd(&hist[w][(uint32_t)(k[i] >> shift) & (kBuckets - 1)], 1u);
    }
  }
  __syncthreads();
  for (int b = threadIdx.x; b < kBuckets; b += BLOCK) {
    uint32_t s = 0;
#pragma unroll
    for (int ww = 0; ww < W; ++ww) s += hist[ww][b];
    chunk_hist[(int64_t)b * G + c] = s;
  }
}

template <int BLOCK, int IPT>
__global__ __launch_bounds__(BLOCK) void k_read(const Elem* __restrict__ A, int64_t m, int64_t chunk_elems,
                                                uint64_t* sink) {
  const int c = blockIdx.x;
  const int64_t beg = (int64_t)c * chunk_elems;
  const int64_t end = beg + chunk_elems < m ? beg + chunk_elems : m;
  uint64_t acc = 0;
  for (int64_t tb = beg; tb < end; tb += (int64_t)BLOCK * IPT) {
    Elem e[IPT];
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      const int64_t idx = tb + (int64_t)i * BLOCK + threadIdx.x;
      e[i] = idx < end ? load_elem(A + idx) : Elem{0, 0};
    }
#pragma unroll
    for (int i = 0; i < IPT; ++i) acc ^= e[i].key + e[i].val;
  }
  if (acc == 0x123456789ull) sink[0] = acc;
}

}  // namespace
}  // namespace lsb

template <typename F> float time_ms(F&& f, int reps) {
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f(); CK(hipDeviceSynchronize()); CK(hipEventRecord(a, 0));
  for (int r = 0; r < reps; ++r) f();
  CK(hipEventRecord(b, 0)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b)); return ms / reps;
}

int main() {
  const int64_t m = (int64_t)1 << 30;
  Elem* A; uint32_t *h0, *h1; uint64_t* sink;
  CK(hipMalloc(&A, m * sizeof(Elem)));
  CK(hipMalloc(&h0, 4 << 20)); CK(hipMalloc(&h1, 4 << 20)); CK(hipMalloc(&sink, 8));
  CK(launch_pcg_fill(A, m, 0, 0, KeyGen{}, 0));
  const double gb = 16.0 * m / 1e9;
  std::vector<uint32_t> a(256 * 4096), b(256 * 4096);
  for (int G : {512, 1024, 2048}) {
    Chunking ch = make_chunking(m, G);
    float t0 = time_ms([&] { CK(launch_upsweep(A, m, 8, ch, h0, nullptr, 0)); }, 5);
    printf("G=%4d product (match)       %6.3f ms %6.0f GB/s\n", ch.num_chunks, t0, gb / t0 * 1e3);
    auto check = [&](const char* name, auto fn) {
      float t = time_ms(fn, 5);
      CK(hipMemcpy(a.data(), h0, 256 * ch.num_chunks * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(b.data(), h1, 256 * ch.num_chunks * 4, hipMemcpyDeviceToHost));
      bool ok = true;
      for (int i = 0; i < 256 * ch.num_chunks; ++i) ok &= a[i] == b[i];
      printf("G=%4d %-22s %6.3f ms %6.0f GB/s %s\n", ch.num_chunks, name, t, gb / t * 1e3, ok ? "OK" : "MISMATCH");
    };
    check("plain 256x16", [&] { hipLaunchKernelGGL((k_up_plain<256, 16, false>), dim3(ch.num_chunks), dim3(256), 0, 0, A, m, 8, ch.chunk_elems, ch.num_chunks, h1); });
    check("plain 512x16", [&] { hipLaunchKernelGGL((k_up_plain<512, 16, false>), dim3(ch.num_chunks), dim3(512), 0, 0, A, m, 8, ch.chunk_elems, ch.num_chunks, h1); });
    check("plain 1024x8", [&] { hipLaunchKernelGGL((k_up_plain<1024, 8, false>), dim3(ch.num_chunks), dim3(1024), 0, 0, A, m, 8, ch.chunk_elems, ch.num_chunks, h1); });
    check("plain 1024x16", [&] { hipLaunchKernelGGL((k_up_plain<1024, 16, false>), dim3(ch.num_chunks), dim3(1024), 0, 0, A, m, 8, ch.chunk_elems, ch.num_chunks, h1); });
    check("plain wide 512x16", [&] { hipLaunchKernelGGL((k_up_plain<512, 16, true>), dim3(ch.num_chunks), dim3(512), 0, 0, A, m, 8, ch.chunk_elems, ch.num_chunks, h1); });
    float tr = time_ms([&] { hipLaunchKernelGGL((k_read<512, 16>), dim3(ch.num_chunks), dim3(512), 0, 0, A, m, ch.chunk_elems, sink); }, 5);
    printf("G=%4d read ceiling 512x16      %6.3f ms %6.0f GB/s\n", ch.num_chunks, tr, gb / tr * 1e3);
    float tr2 = time_ms([&] { hipLaunchKernelGGL((k_read<1024, 16>), dim3(ch.num_chunks), dim3(1024), 0, 0, A, m, ch.chunk_elems, sink); }, 5);
    printf("G=%4d read ceiling 1024x16     %6.3f ms %6.0f GB/s\n", ch.num_chunks, tr2, gb / tr2 * 1e3);
    fflush(stdout);
  }
  return 0;
}
