// Stable two-way merge of 16-byte records, round 2: which persistent shape
// streams when the merge must leave room on every CU for RCCL's kernel
// (ncclDevKernel_Generic: 37,888 B of LDS, 256 threads; tools/rccl_kernels.sh)?
// (development tool for k_merge2 in csrc/lsb_merge.hip)
//
//   ./merge2 [log2 records per run = 29]
//
// Variants: tile of TT = B * I outputs merge-path partitioned (path per tile
// precomputed, as k_merge_path does), persistent grid of G workgroups:
//   S  static tile striding (tile = blockIdx.x + k * G), the shipped form
//   D  dynamic: tile ids from an atomic counter, fetched one tile ahead
//   K  keys-only LDS: the tile's keys are staged (8 B per record), the merge
//      writes a source index per output, and the write-out gathers each
//      record from global memory (L2) by that index: half the LDS
// Each output is checked (sorted by key, stable, a permutation).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <type_traits>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void k_fill(ulonglong2* r, int64_t n, uint64_t stride, uint64_t salt, uint64_t val0) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  r[i] = make_ulonglong2((uint64_t)i * stride + mix(i ^ salt) % stride, val0 + i);
}

template <int TT>
__global__ void k_path(const ulonglong2* a, int64_t na, const ulonglong2* b, int64_t nb, int64_t tiles,
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

// MODE 0: static striding; 1: dynamic counter.  KO: keys-only LDS.
// W16: the keys-only stage loads whole 16-byte records (key kept).
// NT: nontemporal output stores (leave L2 to the gather's re-reads).
template <int B, int I, int MODE, bool KO, bool W16 = false, bool NT = false>
__global__ __launch_bounds__(B) void k_pm(const ulonglong2* __restrict__ a, int64_t na,
                                          const ulonglong2* __restrict__ b, int64_t nb,
                                          const int64_t* __restrict__ path, int64_t tiles,
                                          ulonglong2* __restrict__ out, unsigned* ctr) {
  constexpr int TT = B * I;
  constexpr int SLOTS = TT + TT / 8;
  __shared__ typename std::conditional<KO, uint64_t, ulonglong2>::type tile[KO ? TT + 1 : SLOTS];
  __shared__ uint16_t idx[TT];
  __shared__ int64_t s_next;
  const int64_t n = na + nb;
  auto sl = [](int x) { x = x < TT - 1 ? x : TT - 1; return KO ? x : x + (x >> 3); };
  auto key_of = [&](int s) -> uint64_t {
    if constexpr (KO) return tile[s];
    else return tile[s].x;
  };
  int64_t tt;
  if (MODE == 0) {
    tt = blockIdx.x;
  } else {
    if (threadIdx.x == 0) s_next = atomicAdd(ctr, 1u);
    __syncthreads();
    tt = s_next;
    __syncthreads();
  }
  while (tt < tiles) {
    if (MODE == 1 && threadIdx.x == 0) s_next = atomicAdd(ctr, 1u);  // read after the next barrier
    const int64_t d0 = tt * TT, d1 = d0 + TT < n ? d0 + TT : n;
    const int64_t i0 = path[tt];
    const int ta = (int)(path[tt + 1] - i0), nt = (int)(d1 - d0), tb = nt - ta;
    const int64_t j0 = d0 - i0;
    {
      ulonglong2 v[I];
#pragma unroll
      for (int k = 0; k < I; ++k) {
        const int x = threadIdx.x + k * B;
        if (x < nt) {
          if (KO && !W16) v[k].x = x < ta ? a[i0 + x].x : b[j0 + (x - ta)].x;
          else v[k] = x < ta ? a[i0 + x] : b[j0 + (x - ta)];
        }
      }
#pragma unroll
      for (int k = 0; k < I; ++k) {
        const int x = threadIdx.x + k * B;
        if (x < nt) {
          if constexpr (KO) tile[x] = v[k].x;
          else tile[sl(x)] = v[k];
        }
      }
    }
    __syncthreads();
    const int dl = threadIdx.x * I;
    if (dl < nt) {
      int lo = dl > tb ? dl - tb : 0, hi = dl < ta ? dl : ta;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (key_of(sl(mid)) <= key_of(sl(ta + dl - 1 - mid))) lo = mid + 1;
        else hi = mid;
      }
      int ia = lo, ib = dl - lo;
      uint64_t ka = key_of(sl(ia)), kb = key_of(sl(ta + ib));
      const int end = dl + I < nt ? dl + I : nt;
      for (int k = dl; k < end; ++k) {
        const bool ta_ = ib >= tb || (ia < ta && ka <= kb);
        idx[k] = (uint16_t)(KO ? (ta_ ? ia : ta + ib) : sl(ta_ ? ia : ta + ib));
        if (ta_) ++ia;
        else ++ib;
        const uint64_t nk = key_of(sl(ta_ ? ia : ta + ib));
        if (ta_) ka = nk;
        else kb = nk;
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < I; ++k) {
      const int x = threadIdx.x + k * B;
      if (x < nt) {
        if constexpr (KO) {
          const int s = idx[x];
          const ulonglong2 r = s < ta ? a[i0 + s] : b[j0 + (s - ta)];
          if (NT) {
            __builtin_nontemporal_store(r.x, &out[d0 + x].x);
            __builtin_nontemporal_store(r.y, &out[d0 + x].y);
          } else {
            out[d0 + x] = r;
          }
        } else {
          out[d0 + x] = tile[idx[x]];
        }
      }
    }
    if (MODE == 0) {
      tt += gridDim.x;
      __syncthreads();
    } else {
      __syncthreads();
      tt = s_next;
    }
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
  unsigned* ctr;
  CK(hipMalloc(&a, na * 16)); CK(hipMalloc(&b, nb * 16)); CK(hipMalloc(&o, n * 16));
  CK(hipMalloc(&path, (n / 512 + 2) * 8)); CK(hipMalloc(&chk, 16)); CK(hipMalloc(&ctr, 4));
  const uint64_t sa = ~0ull / (uint64_t)na, sb = ~0ull / (uint64_t)nb;
  k_fill<<<(na + 255) / 256, 256>>>(a, na, sa, 1, 0);
  k_fill<<<(nb + 255) / 256, 256>>>(b, nb, sb, 2, na);
  CK(hipDeviceSynchronize());
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const double gb = n * 32.0 / 1e9;
  const int reps = 5;
  auto check = [&]() {
    unsigned long long h[2] = {0, 0};
    CK(hipMemset(chk, 0, 16));
    k_check<<<(n + 255) / 256, 256>>>(o, n, chk, chk + 1);
    CK(hipMemcpy(h, chk, 16, hipMemcpyDeviceToHost));
    const unsigned long long want = (unsigned long long)((__int128)n * (n - 1) / 2);
    return h[0] == 0 && h[1] == want;
  };
  auto run = [&](const char* name, auto kern, int TT, int B, double per_cu) {
    const int64_t tiles = (n + TT - 1) / TT;
    if (TT == 1024) k_path<1024><<<(tiles + 256) / 256, 256>>>(a, na, b, nb, tiles, path);
    if (TT == 2048) k_path<2048><<<(tiles + 256) / 256, 256>>>(a, na, b, nb, tiles, path);
    if (TT == 4096) k_path<4096><<<(tiles + 256) / 256, 256>>>(a, na, b, nb, tiles, path);
    CK(hipDeviceSynchronize());
    const int grid = (int)(cus * per_cu);
    CK(hipMemset(o, 0, n * 16));
    const float ms = time_ms([&] {
      CK(hipMemsetAsync(ctr, 0, 4, 0));
      kern<<<grid, B>>>(a, na, b, nb, path, tiles, o, ctr);
    }, reps);
    printf("%-22s grid %5d  %8.3f ms  %6.2f TB/s  %s\n", name, grid, ms, gb / ms, check() ? "ok" : "BAD");
  };
  const bool pmc = argc > 2;  // short list for counter passes
  for (double g : {2.0, 3.0}) {
    run("S 256x8 (old)", k_pm<256, 8, 0, false>, 2048, 256, g);
    run("K 256x8 (shipped)", k_pm<256, 8, 0, true>, 2048, 256, g);
    run("K 256x8 w16", k_pm<256, 8, 0, true, true>, 2048, 256, g);
    run("K 256x8 nt", k_pm<256, 8, 0, true, false, true>, 2048, 256, g);
    run("K 256x8 w16 nt", k_pm<256, 8, 0, true, true, true>, 2048, 256, g);
    if (pmc) continue;
    run("K 256x16", k_pm<256, 16, 0, true>, 4096, 256, g);
    run("K 256x16 nt", k_pm<256, 16, 0, true, false, true>, 4096, 256, g);
  }
  return 0;
}
