// Streaming ceilings of this box (development tool): copy / read / write of
// 16-byte records, several launch shapes.  Reference point for the merge and
// scatter kernels' TB/s.
//
//   ./copybw [log2 records = 30]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

// One record per thread, one-shot grid.
__global__ void k_copy1(const ulonglong2* __restrict__ a, ulonglong2* __restrict__ o, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) o[i] = a[i];
}

// U records per thread (block-strided), one-shot grid.
template <int U>
__global__ void k_copyU(const ulonglong2* __restrict__ a, ulonglong2* __restrict__ o, int64_t n) {
  const int64_t base = (int64_t)blockIdx.x * blockDim.x * U + threadIdx.x;
  ulonglong2 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + (int64_t)u * blockDim.x;
    if (i < n) v[u] = a[i];
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + (int64_t)u * blockDim.x;
    if (i < n) o[i] = v[u];
  }
}

// Persistent grid-stride, U records per thread per step.
template <int U>
__global__ void k_copyP(const ulonglong2* __restrict__ a, ulonglong2* __restrict__ o, int64_t n) {
  const int64_t step = (int64_t)gridDim.x * blockDim.x * U;
  for (int64_t base = (int64_t)blockIdx.x * blockDim.x * U + threadIdx.x; base < n; base += step) {
    ulonglong2 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + (int64_t)u * blockDim.x;
      if (i < n) v[u] = a[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + (int64_t)u * blockDim.x;
      if (i < n) o[i] = v[u];
    }
  }
}

// One record per thread with a dynamic LDS allocation that caps the
// workgroups per CU (occupancy probe).
__global__ void k_copy1_lds(const ulonglong2* __restrict__ a, ulonglong2* __restrict__ o, int64_t n) {
  extern __shared__ int dyn[];
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) o[i] = a[i];
  if (i == n + 1) dyn[0] = 0;  // keep the allocation
}

// Wave-contiguous U records per thread: the wave covers U KiB in order
// (onesweep's tile layout), loads then stores.
template <int U>
__global__ void k_copyW(const ulonglong2* __restrict__ a, ulonglong2* __restrict__ o, int64_t n) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t base = (int64_t)blockIdx.x * blockDim.x * U + (int64_t)w * 64 * U + lane;
  ulonglong2 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + (int64_t)u * 64;
    if (i < n) v[u] = a[i];
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + (int64_t)u * 64;
    if (i < n) o[i] = v[u];
  }
}

// Persistent tiles of 4096 records staged through LDS with barriers (the
// shape of k_onesweep / k_merge2 without the ranking): G workgroups, LDS
// sized to 2 or 4 workgroups per CU.
template <int IPT>
__global__ void k_copyT(const ulonglong2* __restrict__ a, ulonglong2* __restrict__ o, int64_t n) {
  constexpr int T = 256 * IPT;
  __shared__ ulonglong2 st[T];
  const int64_t tiles = n / T;
  for (int64_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
    ulonglong2 v[IPT];
#pragma unroll
    for (int u = 0; u < IPT; ++u) v[u] = a[tile * T + u * 256 + threadIdx.x];
#pragma unroll
    for (int u = 0; u < IPT; ++u) st[u * 256 + threadIdx.x] = v[u];
    __syncthreads();
#pragma unroll
    for (int u = 0; u < IPT; ++u) o[tile * T + u * 256 + threadIdx.x] = st[u * 256 + threadIdx.x];
    __syncthreads();
  }
}

// The same tile copy with BLOCK threads per workgroup (tile = BLOCK * IPT
// records), optional streaming (nontemporal) loads, and PF = 1: the next
// tile's loads are issued before this tile's stores (software pipeline,
// twice the registers).
template <int BLOCK, int IPT, bool NT, bool PF>
__global__ __launch_bounds__(BLOCK) void k_copyTB(const ulonglong2* __restrict__ a, ulonglong2* __restrict__ o,
                                                  int64_t n) {
  constexpr int T = BLOCK * IPT;
  __shared__ ulonglong2 st[T];
  const int64_t tiles = n / T;
  typedef unsigned long long v2u64 __attribute__((ext_vector_type(2)));
  auto ld = [&](int64_t i) -> ulonglong2 {
    if (NT) {
      const v2u64 x = __builtin_nontemporal_load(reinterpret_cast<const v2u64*>(a + i));
      return make_ulonglong2(x.x, x.y);
    }
    return a[i];
  };
  ulonglong2 v[IPT];
  int64_t tile = blockIdx.x;
  if (PF && tile < tiles) {
#pragma unroll
    for (int u = 0; u < IPT; ++u) v[u] = ld(tile * T + u * BLOCK + threadIdx.x);
  }
  for (; tile < tiles; tile += gridDim.x) {
    if (!PF) {
#pragma unroll
      for (int u = 0; u < IPT; ++u) v[u] = ld(tile * T + u * BLOCK + threadIdx.x);
    }
#pragma unroll
    for (int u = 0; u < IPT; ++u) st[u * BLOCK + threadIdx.x] = v[u];
    __syncthreads();
    if (PF && tile + gridDim.x < tiles) {
#pragma unroll
      for (int u = 0; u < IPT; ++u) v[u] = ld((tile + gridDim.x) * T + u * BLOCK + threadIdx.x);
    }
#pragma unroll
    for (int u = 0; u < IPT; ++u) o[tile * T + u * BLOCK + threadIdx.x] = st[u * BLOCK + threadIdx.x];
    __syncthreads();
  }
}

__global__ void k_read(const ulonglong2* __restrict__ a, int64_t n, unsigned long long* sink) {
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x * 4 + threadIdx.x;
  uint64_t s = 0;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int64_t i = i0 + (int64_t)u * blockDim.x;
    if (i < n) { const ulonglong2 v = a[i]; s ^= v.x ^ v.y; }
  }
  if (s == 0x123456789ull) atomicAdd(sink, 1ull);
}

__global__ void k_write(ulonglong2* __restrict__ o, int64_t n) {
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x * 4 + threadIdx.x;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int64_t i = i0 + (int64_t)u * blockDim.x;
    if (i < n) o[i] = make_ulonglong2((uint64_t)i, (uint64_t)i);
  }
}

template <typename F>
float time_ms(F&& f, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  f(); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0));
  for (int r = 0; r < reps; ++r) f();
  CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

int main(int argc, char** argv) {
  const int lg = argc > 1 ? atoi(argv[1]) : 30;
  const int64_t n = (int64_t)1 << lg;
  ulonglong2 *a, *o;
  unsigned long long* sink;
  CK(hipMalloc(&a, n * 16)); CK(hipMalloc(&o, n * 16)); CK(hipMalloc(&sink, 8));
  CK(hipMemset(a, 1, n * 16)); CK(hipMemset(o, 0, n * 16));
  const double cp = n * 32.0 / 1e9, one = n * 16.0 / 1e9;
  const int reps = 10;
  auto rep = [&](const char* name, float ms, double gb) { printf("%-14s %8.3f ms  %6.2f TB/s\n", name, ms, gb / ms); };
  rep("copy1 b256", time_ms([&] { k_copy1<<<(n + 255) / 256, 256>>>(a, o, n); }, reps), cp);
  rep("copy1 b1024", time_ms([&] { k_copy1<<<(n + 1023) / 1024, 1024>>>(a, o, n); }, reps), cp);
  rep("copy4 b256", time_ms([&] { k_copyU<4><<<(n + 1023) / 1024, 256>>>(a, o, n); }, reps), cp);
  rep("copy8 b256", time_ms([&] { k_copyU<8><<<(n + 2047) / 2048, 256>>>(a, o, n); }, reps), cp);
  rep("copy16 b256", time_ms([&] { k_copyU<16><<<(n + 4095) / 4096, 256>>>(a, o, n); }, reps), cp);
  for (int g : {1024, 2048, 4096, 8192})
    for (int u : {4, 8}) {
      char nm[32];
      snprintf(nm, sizeof nm, "copyP%d g%d", u, g);
      if (u == 4) rep(nm, time_ms([&] { k_copyP<4><<<g, 256>>>(a, o, n); }, reps), cp);
      else rep(nm, time_ms([&] { k_copyP<8><<<g, 256>>>(a, o, n); }, reps), cp);
    }
  for (int kb : {20, 40, 80}) {
    char nm[32];
    snprintf(nm, sizeof nm, "copy1 lds%dK", kb);
    rep(nm, time_ms([&] { k_copy1_lds<<<(n + 255) / 256, 256, kb * 1024>>>(a, o, n); }, reps), cp);
  }
  rep("copyW4", time_ms([&] { k_copyW<4><<<(n + 1023) / 1024, 256>>>(a, o, n); }, reps), cp);
  rep("copyW16", time_ms([&] { k_copyW<16><<<(n + 4095) / 4096, 256>>>(a, o, n); }, reps), cp);
  for (int g : {512, 1024, 2048}) {
    char nm[32];
    snprintf(nm, sizeof nm, "copyT16 g%d", g);
    rep(nm, time_ms([&] { k_copyT<16><<<g, 256>>>(a, o, n); }, reps), cp);
    snprintf(nm, sizeof nm, "copyT8 g%d", g);
    rep(nm, time_ms([&] { k_copyT<8><<<g, 256>>>(a, o, n); }, reps), cp);
  }
  // Shape study for k_onesweep (4096-record tiles, 64 KiB of LDS, 2 per CU):
  // waves per workgroup, streaming loads, next-tile prefetch.
  rep("TB256x16 g512", time_ms([&] { k_copyTB<256, 16, false, false><<<512, 256>>>(a, o, n); }, reps), cp);
  rep("TB256x16nt g512", time_ms([&] { k_copyTB<256, 16, true, false><<<512, 256>>>(a, o, n); }, reps), cp);
  rep("TB512x8 g512", time_ms([&] { k_copyTB<512, 8, false, false><<<512, 512>>>(a, o, n); }, reps), cp);
  rep("TB512x8nt g512", time_ms([&] { k_copyTB<512, 8, true, false><<<512, 512>>>(a, o, n); }, reps), cp);
  rep("TB1024x4 g512", time_ms([&] { k_copyTB<1024, 4, false, false><<<512, 1024>>>(a, o, n); }, reps), cp);
  rep("TB256x16pf g512", time_ms([&] { k_copyTB<256, 16, false, true><<<512, 256>>>(a, o, n); }, reps), cp);
  rep("TB512x8pf g512", time_ms([&] { k_copyTB<512, 8, false, true><<<512, 512>>>(a, o, n); }, reps), cp);
  rep("TB256x12 g512", time_ms([&] { k_copyTB<256, 12, false, false><<<512, 256>>>(a, o, n); }, reps), cp);
  rep("read4", time_ms([&] { k_read<<<(n + 1023) / 1024, 256>>>(a, n, sink); }, reps), one);
  rep("write4", time_ms([&] { k_write<<<(n + 1023) / 1024, 256>>>(o, n); }, reps), one);
  rep("hipMemcpyD2D", time_ms([&] { CK(hipMemcpyAsync(o, a, n * 16, hipMemcpyDeviceToDevice, 0)); }, reps), cp);
  return 0;
}
