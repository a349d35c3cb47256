// Write ceiling of a direct 65536-bucket LSD pass (BASELINE configs[4], C5)
// against the 256-bucket pass (development tool).
//
// A stable LSD pass leaves workgroup c's records of bucket b as one run at a
// per-(chunk, bucket) frontier.  With NB buckets and C records per chunk the
// run holds C / NB records, and with uniform digits it is filled one record
// every ~NB input records.  This kernel writes exactly that geometry with no
// ranking work: record p of chunk c (read coalesced) goes to
//     out[(p mod NB) * region + c * (C / NB) + p / NB],   region = m / NB,
// so each output line of 8 records gathers records that are NB apart in the
// chunk.  At NB = 256 a line is complete after 2 K input records (in L2
// microseconds later); at NB = 65536 after 512 K, so up to 65536 half-written
// lines per workgroup are live at once, far more than L2 and the Infinity
// Cache hold.  A staged tile cannot help: a 4096-record tile holds 0.06
// records per bucket.
//
//   hipcc -O3 --offload-arch=gfx950 tools/kbench/scatter16.hip -o /tmp/scatter16 && /tmp/scatter16 30
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

struct alignas(16) E { uint64_t k, v; };

__global__ __launch_bounds__(256) void k_transpose_runs(const E* __restrict__ in, E* __restrict__ out,
                                                        int64_t m, int nb_log2, int64_t chunk) {
  const int64_t c = blockIdx.x;
  const int64_t region = m >> nb_log2;
  const int64_t per_run = chunk >> nb_log2;
  const int64_t nbm = ((int64_t)1 << nb_log2) - 1;
  const E* src = in + c * chunk;
  for (int64_t p0 = 0; p0 < chunk; p0 += 256 * 8) {
    E e[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) e[i] = src[p0 + i * 256 + threadIdx.x];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int64_t p = p0 + i * 256 + threadIdx.x;
      out[(p & nbm) * region + c * per_run + (p >> nb_log2)] = e[i];
    }
  }
}

__global__ __launch_bounds__(256) void k_copy(const E* __restrict__ in, E* __restrict__ out, int64_t m) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < m; i += (int64_t)gridDim.x * 256)
    out[i] = in[i];
}

template <typename F>
float time_ms(F&& f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a, 0));
  for (int r = 0; r < reps; ++r) f();
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
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
  const float tc = time_ms([&] { hipLaunchKernelGGL(k_copy, dim3(8192), dim3(256), 0, 0, in, out, m); }, 3);
  printf("copy (reference)                   %8.3f ms %6.0f GB/s\n", tc, gb / tc * 1e3);
  for (int nbl : {8, 11, 16}) {
    for (int g : {512, 1024}) {
      const int64_t chunk = m / g;
      if (chunk % (256 * 8) || (chunk >> nbl) == 0) continue;
      const float t = time_ms([&] {
        hipLaunchKernelGGL(k_transpose_runs, dim3(g), dim3(256), 0, 0, in, out, m, nbl, chunk);
      }, 3);
      printf("buckets %6d  chunks %5d  run %6lld  %8.3f ms %6.0f GB/s\n", 1 << nbl, g,
             (long long)(chunk >> nbl), t, gb / t * 1e3);
      fflush(stdout);
    }
  }
  return 0;
}
