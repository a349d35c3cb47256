// Stable two-way merge of 16-byte records: which tile design streams?
// (development tool for k_merge2 in csrc/lsb_merge.hip)
//
//   ./merge [log2 records per run = 29]
//
// Two key-sorted runs with randomly interleaving keys are merged into one
// output of 2 * 2^lg records.  Variants (all merge-path partitioned into
// 4096-output tiles staged in LDS, 256 threads, 16 outputs per thread):
//   copy     plain 16-byte copy of the same bytes (the streaming ceiling)
//   idx      unpadded tile, per-thread sequential merge writes a u16 source
//            index per output, then a coalesced copy-out from LDS
//   idxpad   the same with one pad slot per 8 records (conflict-free reads)
//   direct   padded tile, each thread stores its 16 outputs itself
//   rank     padded tile, every record finds its output slot by a binary
//            search in the other run (no sequential chain), u16 index
//            scatter, coalesced copy-out
// Each output is checked (sorted by key, stable, a permutation of the input).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

constexpr int T = 4096, BLK = 256, IPT = 16;  // defaults (copy, direct, rank)

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// key = i * stride + jitter < stride: sorted, interleaving randomly with the
// other run; val = global input index (a first, then b).
__global__ void k_fill(ulonglong2* r, int64_t n, uint64_t stride, uint64_t salt, uint64_t val0) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  r[i] = make_ulonglong2((uint64_t)i * stride + mix(i ^ salt) % stride, val0 + i);
}

__global__ void k_path(const ulonglong2* a, int64_t na, const ulonglong2* b, int64_t nb, int64_t tiles,
                       int64_t* path) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t > tiles) return;
  const int64_t n = na + nb, d = t * T < n ? t * T : n;
  int64_t lo = d > nb ? d - nb : 0, hi = d < na ? d : na;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid].x <= b[d - 1 - mid].x) lo = mid + 1;
    else hi = mid;
  }
  path[t] = lo;
}

__global__ __launch_bounds__(256) void k_copy(const ulonglong2* a, ulonglong2* o, int64_t n) {
  const int64_t base = (int64_t)blockIdx.x * T;
  ulonglong2 v[IPT];
#pragma unroll
  for (int k = 0; k < IPT; ++k) v[k] = a[base + threadIdx.x + k * BLK];
#pragma unroll
  for (int k = 0; k < IPT; ++k) o[base + threadIdx.x + k * BLK] = v[k];
}

template <bool PAD>
__device__ __forceinline__ int slot(int x) {
  x = x < T - 1 ? x : T - 1;  // a run's end is read but never used
  return PAD ? x + (x >> 3) : x;
}

struct Tile {
  int64_t d0, i0, j0;
  int ta, tb, nt;
};

__device__ __forceinline__ Tile tile_of(int64_t na, int64_t nb, const int64_t* path) {
  Tile t;
  const int64_t n = na + nb;
  t.d0 = (int64_t)blockIdx.x * T;
  const int64_t d1 = t.d0 + T < n ? t.d0 + T : n;
  t.i0 = path[blockIdx.x];
  t.j0 = t.d0 - t.i0;
  t.ta = (int)(path[blockIdx.x + 1] - t.i0);
  t.nt = (int)(d1 - t.d0);
  t.tb = t.nt - t.ta;
  return t;
}

template <bool PAD>
__device__ __forceinline__ void stage(ulonglong2* tile, const ulonglong2* a, const ulonglong2* b,
                                      const Tile& t) {
  ulonglong2 v[IPT];
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    const int x = threadIdx.x + k * BLK;
    if (x < t.nt) v[k] = x < t.ta ? a[t.i0 + x] : b[t.j0 + (x - t.ta)];
  }
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    const int x = threadIdx.x + k * BLK;
    if (x < t.nt) tile[slot<PAD>(x)] = v[k];
  }
}

template <bool PAD>
__device__ __forceinline__ int tile_corank(const ulonglong2* tile, const Tile& t, int dl) {
  int lo = dl > t.tb ? dl - t.tb : 0, hi = dl < t.ta ? dl : t.ta;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (tile[slot<PAD>(mid)].x <= tile[slot<PAD>(t.ta + dl - 1 - mid)].x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

template <bool PAD>
__global__ __launch_bounds__(256, 2) void k_idx(const ulonglong2* a, int64_t na, const ulonglong2* b,
                                                int64_t nb, const int64_t* path, ulonglong2* out) {
  __shared__ ulonglong2 tile[T + T / 8];
  __shared__ uint16_t idx[T];
  const Tile t = tile_of(na, nb, path);
  stage<PAD>(tile, a, b, t);
  __syncthreads();
  const int dl = threadIdx.x * IPT;
  if (dl < t.nt) {
    int ia = tile_corank<PAD>(tile, t, dl), ib = dl - ia;
    uint64_t ka = tile[slot<PAD>(ia)].x, kb = tile[slot<PAD>(t.ta + ib)].x;
    const int end = dl + IPT < t.nt ? dl + IPT : t.nt;
    for (int k = dl; k < end; ++k) {
      const bool ta_ = ib >= t.tb || (ia < t.ta && ka <= kb);
      const int src = ta_ ? ia : t.ta + ib;
      idx[k] = (uint16_t)slot<PAD>(src);
      if (ta_) ++ia;
      else ++ib;
      const uint64_t nk = tile[slot<PAD>(ta_ ? ia : t.ta + ib)].x;
      if (ta_) ka = nk;
      else kb = nk;
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    const int x = threadIdx.x + k * BLK;
    if (x < t.nt) out[t.d0 + x] = tile[idx[x]];
  }
}

__global__ __launch_bounds__(256, 2) void k_direct(const ulonglong2* a, int64_t na, const ulonglong2* b,
                                                   int64_t nb, const int64_t* path, ulonglong2* out) {
  __shared__ ulonglong2 tile[T + T / 8];
  const Tile t = tile_of(na, nb, path);
  stage<true>(tile, a, b, t);
  __syncthreads();
  const int dl = threadIdx.x * IPT;
  if (dl >= t.nt) return;
  int ia = tile_corank<true>(tile, t, dl), ib = dl - ia;
  ulonglong2 ra = tile[slot<true>(ia)], rb = tile[slot<true>(t.ta + ib)];
  const int end = dl + IPT < t.nt ? dl + IPT : t.nt;
  for (int k = dl; k < end; ++k) {
    const bool ta_ = ib >= t.tb || (ia < t.ta && ra.x <= rb.x);
    out[t.d0 + k] = ta_ ? ra : rb;
    if (ta_) ++ia;
    else ++ib;
    const ulonglong2 r = tile[slot<true>(ta_ ? ia : t.ta + ib)];
    if (ta_) ra = r;
    else rb = r;
  }
}

// Every tile record x finds its output slot: x's index in its run plus its
// rank in the other run (a: count of b keys < k; b: count of a keys <= k).
__global__ __launch_bounds__(256, 2) void k_rank(const ulonglong2* a, int64_t na, const ulonglong2* b,
                                                 int64_t nb, const int64_t* path, ulonglong2* out) {
  __shared__ ulonglong2 tile[T + T / 8];
  __shared__ uint16_t idx[T];
  const Tile t = tile_of(na, nb, path);
  stage<true>(tile, a, b, t);
  __syncthreads();
#pragma unroll 4
  for (int k = 0; k < IPT; ++k) {
    const int x = threadIdx.x + k * BLK;
    if (x >= t.nt) break;
    const uint64_t key = tile[slot<true>(x)].x;
    const bool in_a = x < t.ta;
    // search the other run: [base, base + len)
    const int base = in_a ? t.ta : 0, len = in_a ? t.tb : t.ta;
    int lo = 0, hi = len;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      const uint64_t m = tile[slot<true>(base + mid)].x;
      if (in_a ? m < key : m <= key) lo = mid + 1;
      else hi = mid;
    }
    const int pos = (in_a ? x : x - t.ta) + lo;
    idx[pos] = (uint16_t)slot<true>(x);
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    const int x = threadIdx.x + k * BLK;
    if (x < t.nt) out[t.d0 + x] = tile[idx[x]];
  }
}


// Path at any tile size TT.
template <int TT>
__global__ void k_pathg(const ulonglong2* a, int64_t na, const ulonglong2* b, int64_t nb, int64_t tiles,
                        int64_t* path) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t > tiles) return;
  const int64_t n = na + nb, d = t * TT < n ? t * TT : n;
  int64_t lo = d > nb ? d - nb : 0, hi = d < na ? d : na;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid].x <= b[d - 1 - mid].x) lo = mid + 1;
    else hi = mid;
  }
  path[t] = lo;
}

// Persistent grid-stride copy, I records in flight per thread.
template <int I>
__global__ __launch_bounds__(256) void k_copy2(const ulonglong2* a, ulonglong2* o, int64_t n) {
  const int64_t step = (int64_t)gridDim.x * 256 * I;
  for (int64_t base = (int64_t)blockIdx.x * 256 * I + threadIdx.x; base < n; base += step) {
    ulonglong2 v[I];
#pragma unroll
    for (int k = 0; k < I; ++k) if (base + k * 256 < n) v[k] = a[base + k * 256];
#pragma unroll
    for (int k = 0; k < I; ++k) if (base + k * 256 < n) o[base + k * 256] = v[k];
  }
}

// Persistent merge: tiles blockIdx.x, + gridDim.x, ...; tile TT = B * I
// outputs; PF: the next tile's records are loaded into registers while the
// current one merges; NT: nontemporal output stores.
template <int B, int I, bool PF, bool NT>
__global__ __launch_bounds__(B) void k_pm(const ulonglong2* a, int64_t na, const ulonglong2* b,
                                          int64_t nb, const int64_t* path, int64_t tiles,
                                          ulonglong2* out) {
  constexpr int TT = B * I;
  __shared__ ulonglong2 tile[TT + TT / 8];
  __shared__ uint16_t idx[TT];
  const int64_t n = na + nb;
  auto sl = [](int x) { x = x < TT - 1 ? x : TT - 1; return x + (x >> 3); };
  ulonglong2 v[I];
  auto load = [&](int64_t tt) {
    const int64_t d0 = tt * TT, d1 = d0 + TT < n ? d0 + TT : n;
    const int64_t i0 = path[tt], ta = path[tt + 1] - i0, j0 = d0 - i0;
    const int nt = (int)(d1 - d0);
#pragma unroll
    for (int k = 0; k < I; ++k) {
      const int x = threadIdx.x + k * B;
      if (x < nt) v[k] = x < ta ? a[i0 + x] : b[j0 + (x - ta)];
    }
  };
  int64_t tt = blockIdx.x;
  if (tt >= tiles) return;
  load(tt);
  for (; tt < tiles; tt += gridDim.x) {
    const int64_t d0 = tt * TT, d1 = d0 + TT < n ? d0 + TT : n;
    const int64_t i0 = path[tt];
    const int ta = (int)(path[tt + 1] - i0), nt = (int)(d1 - d0), tb = nt - ta;
#pragma unroll
    for (int k = 0; k < I; ++k) {
      const int x = threadIdx.x + k * B;
      if (x < nt) tile[sl(x)] = v[k];
    }
    __syncthreads();
    if (PF && tt + gridDim.x < tiles) load(tt + gridDim.x);
    const int dl = threadIdx.x * I;
    if (dl < nt) {
      int lo = dl > tb ? dl - tb : 0, hi = dl < ta ? dl : ta;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (tile[sl(mid)].x <= tile[sl(ta + dl - 1 - mid)].x) lo = mid + 1;
        else hi = mid;
      }
      int ia = lo, ib = dl - lo;
      uint64_t ka = tile[sl(ia)].x, kb = tile[sl(ta + ib)].x;
      const int end = dl + I < nt ? dl + I : nt;
      for (int k = dl; k < end; ++k) {
        const bool ta_ = ib >= tb || (ia < ta && ka <= kb);
        idx[k] = (uint16_t)sl(ta_ ? ia : ta + ib);
        if (ta_) ++ia;
        else ++ib;
        const uint64_t nk = tile[sl(ta_ ? ia : ta + ib)].x;
        if (ta_) ka = nk;
        else kb = nk;
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < I; ++k) {
      const int x = threadIdx.x + k * B;
      if (x < nt) {
        const ulonglong2 r = tile[idx[x]];
        if (NT) {
          __builtin_nontemporal_store(r.x, &out[d0 + x].x);
          __builtin_nontemporal_store(r.y, &out[d0 + x].y);
        } else {
          out[d0 + x] = r;
        }
      }
    }
    __syncthreads();
    if (!PF && tt + gridDim.x < tiles) load(tt + gridDim.x);
  }
}

__global__ void k_check(const ulonglong2* o, int64_t n, unsigned long long* bad, unsigned long long* sum) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  atomicAdd(sum, (unsigned long long)o[i].y);
  if (i + 1 < n) {
    const ulonglong2 x = o[i], y = o[i + 1];
    if (x.x > y.x || (x.x == y.x && x.y > y.y)) atomicAdd(bad, 1ull);
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
  const int lg = argc > 1 ? atoi(argv[1]) : 29;
  const int64_t na = (int64_t)1 << lg, nb = na, n = na + nb;
  ulonglong2 *a, *b, *o;
  int64_t* path;
  unsigned long long* chk;
  CK(hipMalloc(&a, na * 16)); CK(hipMalloc(&b, nb * 16)); CK(hipMalloc(&o, n * 16));
  const int64_t tiles = (n + T - 1) / T;
  CK(hipMalloc(&path, (tiles + 1) * 8)); CK(hipMalloc(&chk, 16));
  const uint64_t sa = ~0ull / (uint64_t)na, sb = ~0ull / (uint64_t)nb;
  k_fill<<<(na + 255) / 256, 256>>>(a, na, sa, 1, 0);
  k_fill<<<(nb + 255) / 256, 256>>>(b, nb, sb, 2, na);
  k_path<<<(tiles + 256) / 256, 256>>>(a, na, b, nb, tiles, path);
  CK(hipDeviceSynchronize());
  const double gb = n * 32.0 / 1e9;
  auto report = [&](const char* name, float ms, bool check) {
    unsigned long long h[2] = {0, 0};
    if (check) {
      CK(hipMemset(chk, 0, 16));
      k_check<<<(n + 255) / 256, 256>>>(o, n, chk, chk + 1);
      CK(hipMemcpy(h, chk, 16, hipMemcpyDeviceToHost));
    }
    const unsigned long long want = (unsigned long long)((__int128)n * (n - 1) / 2);
    printf("%-8s %8.3f ms  %6.2f TB/s  %s\n", name, ms, gb / ms, !check ? "" : (h[0] == 0 && h[1] == want) ? "ok" : "BAD");
  };
  const int reps = 5;
  const unsigned g = (unsigned)tiles;
  report("path", time_ms([&] { k_path<<<(tiles + 256) / 256, 256>>>(a, na, b, nb, tiles, path); }, reps), false);
  report("copy", time_ms([&] { k_copy<<<g / 2, 256>>>(a, o, n); k_copy<<<g / 2, 256>>>(b, o + na, n); }, reps), false);
  report("idx", time_ms([&] { k_idx<false><<<g, 256>>>(a, na, b, nb, path, o); }, reps), true);
  report("idxpad", time_ms([&] { k_idx<true><<<g, 256>>>(a, na, b, nb, path, o); }, reps), true);
  report("direct", time_ms([&] { k_direct<<<g, 256>>>(a, na, b, nb, path, o); }, reps), true);
  report("rank", time_ms([&] { k_rank<<<g, 256>>>(a, na, b, nb, path, o); }, reps), true);
  for (int cg : {256, 512, 1024, 2048})
    report(cg == 256 ? "copy2/256" : cg == 512 ? "copy2/512" : cg == 1024 ? "copy2/1k" : "copy2/2k",
           time_ms([&] { k_copy2<8><<<cg, 256>>>(a, o, na); k_copy2<8><<<cg, 256>>>(b, o + na, nb); }, reps), false);
  int64_t* path2;
  CK(hipMalloc(&path2, (n / 512 + 2) * 8));
  auto run_pm = [&](const char* name, auto kern, int tt_size, int blk, int wg_per_cu) {
    const int64_t tl = (n + tt_size - 1) / tt_size;
    if (tt_size == 1024) k_pathg<1024><<<(tl + 256) / 256, 256>>>(a, na, b, nb, tl, path2);
    if (tt_size == 2048) k_pathg<2048><<<(tl + 256) / 256, 256>>>(a, na, b, nb, tl, path2);
    if (tt_size == 4096) k_pathg<4096><<<(tl + 256) / 256, 256>>>(a, na, b, nb, tl, path2);
    CK(hipDeviceSynchronize());
    const int grid = 256 * wg_per_cu;
    report(name, time_ms([&] { kern<<<grid, blk>>>(a, na, b, nb, path2, tl, o); }, reps), true);
  };
  run_pm("pm256x8", k_pm<256, 8, false, false>, 2048, 256, 4);
  run_pm("pm256x8PF", k_pm<256, 8, true, false>, 2048, 256, 4);
  run_pm("pm256x8PFNT", k_pm<256, 8, true, true>, 2048, 256, 4);
  run_pm("pm256x4PF", k_pm<256, 4, true, false>, 1024, 256, 8);
  run_pm("pm256x16PF", k_pm<256, 16, true, false>, 4096, 256, 2);
  run_pm("pm512x8PF", k_pm<512, 8, true, false>, 4096, 512, 2);
  run_pm("pm256x8PFx2", k_pm<256, 8, true, false>, 2048, 256, 2);
  run_pm("pm256x8PFx3", k_pm<256, 8, true, false>, 2048, 256, 3);
  return 0;
}
