// Does a pass run cheaper when processed in super-chunks that fit the 256 MiB
// Infinity Cache (upsweep reads from HBM, the scatter's re-read hits MALL)?
// (development tool; output is the exact pass result, checked vs one-shot)
#include "../../distributed-lsb_amd/csrc/lsb_kernels.hip"

#include <cstdio>
#include <cstdlib>

using namespace lsb;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

namespace lsb {
namespace {
// chunk_off[b][*] += base[b]; base[b] += totals[b]   (one thread per bucket row)
__global__ void k_add_base(uint64_t* chunk_off, int G, uint64_t* base, const uint64_t* totals) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= kBuckets) return;
  const uint64_t x = base[b];
  for (int c = 0; c < G; ++c) chunk_off[(int64_t)b * G + c] += x;
  base[b] = x + totals[b];
}
__global__ void k_excl(const uint64_t* tot, uint64_t* base) {  // one thread
  uint64_t s = 0;
  for (int b = 0; b < kBuckets; ++b) { base[b] = s; s += tot[b]; }
}
__global__ void k_diff(const Elem* a, const Elem* b, int64_t m, unsigned long long* bad) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x)
    if (a[i].key != b[i].key || a[i].val != b[i].val) atomicAdd(bad, 1ull);
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
  const int shift = 8;
  Elem *in, *out, *ref;
  uint32_t* hist; uint64_t *off, *tot, *zero, *base, *gtot;
  CK(hipMalloc(&in, m * 16)); CK(hipMalloc(&out, m * 16)); CK(hipMalloc(&ref, m * 16));
  CK(hipMalloc(&hist, 4 << 20)); CK(hipMalloc(&off, 8 << 20)); CK(hipMalloc(&tot, 2048));
  CK(hipMalloc(&zero, 2048)); CK(hipMalloc(&base, 2048)); CK(hipMalloc(&gtot, 2048));
  CK(hipMemset(zero, 0, 2048));
  CK(launch_pcg_fill(in, m, 0, 0, KeyGen{}, 0));
  unsigned long long* bad; CK(hipMalloc(&bad, 8));
  // one-shot pass (the product)
  Chunking ch = make_chunking(m, 512);
  auto one = [&] {
    CK(launch_upsweep(in, m, shift, ch, hist, nullptr, 0));
    CK(launch_scan(hist, ch.num_chunks, off, tot, 0));
    CK(launch_scatter(in, ref, m, shift, ch, off, tot, nullptr, 0));
  };
  float t1 = time_ms(one, 5);
  printf("one-shot pass                 %7.3f ms\n", t1);
  CK(hipMemcpy(gtot, tot, 2048, hipMemcpyDeviceToDevice));  // global digit totals
  for (int64_t sc : {(int64_t)4 << 20, (int64_t)8 << 20, (int64_t)16 << 20}) {
    for (int g : {256, 512}) {
      Chunking cs = make_chunking(sc, g);
      auto pass = [&] {
        hipLaunchKernelGGL(k_excl, dim3(1), dim3(1), 0, 0, gtot, base);
        for (int64_t s0 = 0; s0 < m; s0 += sc) {
          CK(launch_upsweep(in + s0, sc, shift, cs, hist, nullptr, 0));
          CK(launch_scan(hist, cs.num_chunks, off, tot, 0));
          hipLaunchKernelGGL(k_add_base, dim3(1), dim3(256), 0, 0, off, cs.num_chunks, base, tot);
          CK(launch_scatter(in + s0, out, sc, shift, cs, off, zero, nullptr, 0));
        }
      };
      float t = time_ms(pass, 3);
      CK(hipMemset(bad, 0, 8));
      hipLaunchKernelGGL(k_diff, dim3(4096), dim3(256), 0, 0, out, ref, m, bad);
      unsigned long long h; CK(hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost));
      printf("super-chunk %4lld MiB G=%d     %7.3f ms  %s\n", (long long)(sc * 16 >> 20), g, t,
             h ? "MISMATCH" : "OK");
      fflush(stdout);
    }
  }
  return 0;
}
