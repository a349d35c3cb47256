// Synthetic scatter patterns for the layout / digit-width decision
// (development tool).  Each workgroup walks a contiguous chunk of tiles; tile
// t sends its i-th run of R records to bucket region i (NB buckets), at the
// workgroup's own frontier in that region — the write pattern of a chunked
// LSD pass whose runs are whole 128-B lines, with no ranking work.
//   AoS: 16-B {key,val} records in and out
//   SoA: key[] and val[] arrays in and out (8 B + 8 B per record)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

struct alignas(16) E { uint64_t k, v; };

// m records, G workgroups, NB buckets, runs of R records.  Workgroup w owns
// tiles [w*tpb, (w+1)*tpb) of T = NB*R records; in bucket region i its
// frontier starts at w*tpb*R.
template <bool SOA>
__global__ __launch_bounds__(256) void k_runs(const E* __restrict__ in, E* __restrict__ out,
                                              const uint64_t* __restrict__ ik, const uint64_t* __restrict__ iv,
                                              uint64_t* __restrict__ ok, uint64_t* __restrict__ ov,
                                              int64_t m, int nb_log2, int r_log2, int64_t tpb) {
  const int64_t region = m >> nb_log2;
  const int64_t T = (int64_t)1 << (nb_log2 + r_log2);
  const int64_t ntiles = m / T;
  for (int64_t j = 0; j < tpb; ++j) {
    const int64_t tile = blockIdx.x * tpb + j;
    if (tile >= ntiles) break;
    for (int64_t p0 = 0; p0 < T; p0 += 256 * 4) {
      const int64_t base = tile * T + p0;
      if (SOA) {
        uint64_t k[4], v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) { k[i] = ik[base + i * 256 + threadIdx.x]; v[i] = iv[base + i * 256 + threadIdx.x]; }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int64_t p = p0 + i * 256 + threadIdx.x;
          const int64_t d = (p >> r_log2) * region + (tile << r_log2) + (p & ((1 << r_log2) - 1));
          ok[d] = k[i];
          ov[d] = v[i];
        }
      } else {
        E e[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) e[i] = in[base + i * 256 + threadIdx.x];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int64_t p = p0 + i * 256 + threadIdx.x;
          out[(p >> r_log2) * region + (tile << r_log2) + (p & ((1 << r_log2) - 1))] = e[i];
        }
      }
    }
  }
}

// Key-only streaming read (the SoA count pass) vs the AoS record read.
__global__ __launch_bounds__(256) void k_read(const uint64_t* __restrict__ a, int64_t words, int stride,
                                              uint64_t* sink) {
  uint64_t acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < words; i += (int64_t)gridDim.x * 256)
    acc += a[i * stride];
  if (acc == 0x1234567) *sink = acc;
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
  uint64_t* ik = (uint64_t*)in;
  uint64_t* iv = ik + m;
  uint64_t* ok = (uint64_t*)out;
  uint64_t* ov = ok + m;
  uint64_t* sink;
  CK(hipMalloc(&sink, 8));
  const double gb = 32.0 * m / 1e9;
  for (int grid : {512, 1024}) {
    float t16 = time_ms([&] { hipLaunchKernelGGL(k_read, dim3(grid * 4), dim3(256), 0, 0, ik, m, 2, sink); }, 3);
    float t8 = time_ms([&] { hipLaunchKernelGGL(k_read, dim3(grid * 4), dim3(256), 0, 0, ik, m, 1, sink); }, 3);
    printf("read keys: AoS stride %7.3f ms | SoA %7.3f ms\n", t16, t8);
  }
  for (int nbl : {8, 9, 10, 11, 12}) {
    for (int rl : {3, 4}) {
      const int64_t T = (int64_t)1 << (nbl + rl);
      const int64_t ntiles = m / T;
      for (int grid : {256, 512, 1024}) {
        const int64_t tpb = (ntiles + grid - 1) / grid;
        float a = time_ms([&] { hipLaunchKernelGGL((k_runs<false>), dim3(grid), dim3(256), 0, 0, in, out, ik, iv, ok, ov, m, nbl, rl, tpb); }, 3);
        float s = time_ms([&] { hipLaunchKernelGGL((k_runs<true>), dim3(grid), dim3(256), 0, 0, in, out, ik, iv, ok, ov, m, nbl, rl, tpb); }, 3);
        printf("NB=%5d run=%3d grid=%5d  AoS %7.3f ms %6.0f GB/s | SoA %7.3f ms %6.0f GB/s\n",
               1 << nbl, 1 << rl, grid, a, gb / a * 1e3, s, gb / s * 1e3);
        fflush(stdout);
      }
    }
  }
  return 0;
}
