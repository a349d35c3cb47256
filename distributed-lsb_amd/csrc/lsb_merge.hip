// Whole-key exchange (radix_bits = 64): the kernels of the one-exchange form
// of the multi-GPU sort.
//
// With an exchange digit of 64 bits, globalShuffle (mpi/mpi_lsbsort.cpp:481-577)
// has one pass: every rank sorts its block locally on the whole key (the
// 8 stable 8-bit passes of localShuffle, :213-247), then the records move
// once to the ranks owning their final global positions.  The order is the
// reference's: key, then input position (rank, then local index), because the
// local passes are stable and ranks are merged in rank order.
//
//   k_split_cands / k_split_update / k_split_final
//       global position T_q = q * per (q = 1 .. P-1) -> the key k* found there
//       and each rank's count of keys < k* and <= k*, by a 256-ary search of
//       the key space (8 rounds for 64 bits; the per-candidate counts are
//       binary searches in the rank's sorted block, summed over ranks from an
//       all-gather).  This replaces copyCountsToGlobalCounts + exclusiveScan +
//       copyStartsFromGlobalStarts (:327-479) for a digit with 2^64 buckets.
//   k_merge_path / k_merge2
//       the receiver's placement (:568-575): P sorted runs (one per source, in
//       rank order) -> one sorted block, by a tree of stable two-way merges
//       (ties: the left run, i.e. the lower source ranks, first).  One launch
//       pair per tree level merges all of the level's pairs; each merge is
//       merge-path partitioned into 2048-output tiles staged in LDS and written
//       back as whole, coalesced lines.
#include "lsb_kernels.h"

#ifdef LSB_DEBUG
#include <cassert>
#define LSB_MERGE_ASSERT(c) assert(c)
#else
#define LSB_MERGE_ASSERT(c) ((void)0)
#endif

namespace lsb {
namespace {

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint64_t key_at(const Elem* p, int64_t i) {
  return reinterpret_cast<const uint64_t*>(p)[2 * i];
}

// #{i < m : A[i].key < k} (strict) or <= k, A sorted by key.
template <bool kUpper>
__device__ int64_t count_keys(const Elem* __restrict__ A, int64_t m, uint64_t k) {
  int64_t lo = 0, hi = m;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    const uint64_t x = key_at(A, mid);
    if (kUpper ? x <= k : x < k) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// Candidate j of the interval [lo, hi]: lo + j * step while inside, else hi.
// step = width / 256 + 1, so the next interval is < step wide: 8 rounds take a
// 64-bit interval to one key.  Nondecreasing in j.
__device__ __forceinline__ uint64_t split_cand(uint64_t lo, uint64_t hi, int j) {
  const uint64_t width = hi - lo;
  const uint64_t step = (width >> 8) + 1;
  const uint64_t off = (uint64_t)j * step;  // < 2^64: j < 256, step <= 2^56
  return off <= width ? lo + off : hi;
}

// Thread (t, j): cnt[t * K + j] = #{keys < candidate j of target t}.
__global__ __launch_bounds__(256) void k_split_cands(const Elem* __restrict__ A, int64_t m,
                                                     const uint64_t* __restrict__ state, int Q,
                                                     uint64_t* __restrict__ cnt) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= Q * kSplitCands) return;
  const int t = i / kSplitCands, j = i % kSplitCands;
  const uint64_t c = split_cand(state[2 * t], state[2 * t + 1], j);
  cnt[i] = (uint64_t)count_keys<false>(A, m, c);
}

// One workgroup per target t: sum the P ranks' counts of every candidate,
// keep the largest candidate with at most T_t keys below it (the key at
// global position T_t is >= it) and cut the interval below the next one.
__global__ __launch_bounds__(kSplitCands) void k_split_update(const uint64_t* __restrict__ gathered,
                                                              int P, int Q,
                                                              const int64_t* __restrict__ targets,
                                                              uint64_t* __restrict__ state) {
  __shared__ int best;
  const int t = blockIdx.x, j = threadIdx.x;
  const uint64_t lo = state[2 * t], hi = state[2 * t + 1];
  uint64_t below = 0;
  for (int s = 0; s < P; ++s) below += gathered[((size_t)s * Q + t) * kSplitCands + j];
  if (j == 0) best = 0;
  __syncthreads();
  if (below <= (uint64_t)targets[t]) atomicMax(&best, j);
  __syncthreads();
  if (j == 0) {
    const int b = best;
    const uint64_t c = split_cand(lo, hi, b);
    uint64_t nhi = hi;
    if (b + 1 < kSplitCands) {
      const uint64_t c1 = split_cand(lo, hi, b + 1);
      if (c1 > c) nhi = c1 - 1;  // candidate b + 1 has more than T_t keys below it
    }
    state[2 * t] = c;
    state[2 * t + 1] = nhi;
  }
}

// out[2t] = #{keys < k*_t}, out[2t + 1] = #{keys <= k*_t} (k*_t = state lo).
__global__ __launch_bounds__(64) void k_split_final(const Elem* __restrict__ A, int64_t m,
                                                    const uint64_t* __restrict__ state, int Q,
                                                    uint64_t* __restrict__ out) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= 2 * Q) return;
  const uint64_t k = state[2 * (i >> 1)];
  out[i] = (uint64_t)((i & 1) ? count_keys<true>(A, m, k) : count_keys<false>(A, m, k));
}

__global__ void k_split_init(uint64_t* __restrict__ state, int Q) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= Q) return;
  state[2 * t] = 0;
  state[2 * t + 1] = ~0ull;
}

// ------------------------------------------------------------------ merge
// Stable merge of a (na) and b (nb): an a-record goes before an equal b-record.
// Merge path: out[0, d) takes i records of a and d - i of b, with i the first
// index where a[i] > b[d - 1 - i].
__device__ __forceinline__ int64_t merge_path_global(const Elem* __restrict__ a, int64_t na,
                                                     const Elem* __restrict__ b, int64_t nb,
                                                     int64_t d) {
  int64_t lo = d > nb ? d - nb : 0, hi = d < na ? d : na;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (key_at(a, mid) <= key_at(b, d - 1 - mid)) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// Pair of a merge level that holds global tile x (kPathEntries: path entry
// x, k_merge_path): the last p with first[p] <= x, where pair p's tiles start
// at tile0[p] and its path entries at tile0[p] + p (one more entry than
// tiles).  The descriptors stay kernel arguments, indexed in place.
template <bool kPathEntries>
__device__ __forceinline__ int level_pair(const MergeLevel& L, int64_t x) {
  int p = 0;
  for (int q = 1; q < L.npairs; ++q)
    if ((kPathEntries ? L.p[q].tile0 + q : L.p[q].tile0) <= x) p = q;
  return p;
}

// Every path entry of the level: co-rank (records of a) of output position
// min(t * kMergeTile, na + nb) of its pair's tile t.
__global__ __launch_bounds__(256) void k_merge_path(MergeLevel L, int64_t* __restrict__ path) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= L.tiles + L.npairs) return;
  const int p = level_pair<true>(L, e);
  const MergePair& q = L.p[p];
  const int64_t t = e - q.tile0 - p;
  const int64_t n = q.na + q.nb;
  const int64_t d = t * kMergeTile < n ? t * kMergeTile : n;
  path[e] = merge_path_global(q.a, q.na, q.b, q.nb, d);
}

constexpr int kMergeBlock = 256;
constexpr int kMergeIpt = kMergeTile / kMergeBlock;  // 8 outputs per thread

// Step 3 of k_merge2: output x of the tile = input record idx[x] (a-range
// first, then the b-range), gathered and stored by consecutive lanes.  Every
// lane issues all its loads before its first store, so the loads stay in
// flight together instead of waiting one by one.  Nontemporal
// stores: the output is read again only by the next level, milliseconds
// later; L2 is left to the gather's re-reads.
__device__ __forceinline__ void write_out(const Elem* __restrict__ a, const Elem* __restrict__ b,
                                          Elem* __restrict__ out, int64_t i0, int64_t j0, int ta,
                                          int nt, int64_t d0, const uint16_t* idx, int t) {
  u64x2 r[kMergeIpt];
#pragma unroll
  for (int k = 0; k < kMergeIpt; ++k) {
    const int x = t + k * kMergeBlock;
    const int s = idx[x < nt ? x : nt - 1];
    r[k] = *reinterpret_cast<const u64x2*>(s < ta ? a + (i0 + s) : b + (j0 + (s - ta)));
  }
  // No branch around the stores (a masked store cost k_onesweep 6 %): a lane
  // past the end of a partial tile holds output nt - 1 and stores that same
  // value again, to the same place.
#pragma unroll
  for (int k = 0; k < kMergeIpt; ++k) {
    const int x = t + k * kMergeBlock;
    __builtin_nontemporal_store(r[k], reinterpret_cast<u64x2*>(out + (d0 + (x < nt ? x : nt - 1))));
  }
}

// Persistent: workgroup w merges tiles w, w + grid, ... of the whole level
// (every pair; 3 workgroups per CU, 20 KiB of LDS each, so RCCL's kernel,
// 37 KiB of LDS, still fits on every CU while a level runs beside an
// all-to-all).  Per tile of kMergeTile outputs:
//   1. the KEYS of its a- and b-ranges (from the tile path) -> LDS, from
//      16-byte loads of consecutive lanes (a-range first, then the b-range);
//   2. each thread owns kMergeIpt consecutive outputs: merge path inside the
//      tile, then a sequential merge that writes the source index of every
//      output;
//   3. output x of the tile = record idx[x] of the tile's input, loaded
//      again (its line was fetched by step 1, mostly still in L2) and
//      stored nontemporally by consecutive lanes: whole 128-byte lines.
// tools/kbench/merge2.hip: keys-only staging streams at 5.2 TB/s (a plain
// tile copy through LDS: 5.1), the full 16-byte records staged in LDS at
// 2.5 TB/s (2 WG/CU) to 3.7 TB/s (4 WG/CU).  A pair with nb = 0 is a copy
// through the same path.
__global__ __launch_bounds__(kMergeBlock) void k_merge2(MergeLevel L, const int64_t* __restrict__ path) {
  __shared__ uint64_t keys[kMergeTile];  // 16 KiB
  __shared__ uint16_t idx[kMergeTile];   // 4 KiB
  const int t = threadIdx.x;
  auto key = [&](int x) { return keys[x < kMergeTile - 1 ? x : kMergeTile - 1]; };  // run ends: never used
  for (int64_t gt = blockIdx.x; gt < L.tiles; gt += gridDim.x) {
    const int p = level_pair<false>(L, gt);
    const MergePair& q = L.p[p];
    const Elem* __restrict__ a = q.a;
    const Elem* __restrict__ b = q.b;
    Elem* __restrict__ out = q.out;
    const int64_t n = q.na + q.nb;
    const int64_t lt = gt - q.tile0;
    const int64_t* pp = path + q.tile0 + p + lt;
    const int64_t d0 = lt * kMergeTile;
    const int64_t d1 = d0 + kMergeTile < n ? d0 + kMergeTile : n;
    const int64_t i0 = pp[0];
    const int64_t j0 = d0 - i0;
    const int ta = (int)(pp[1] - i0);        // records of a in this tile
    const int nt = (int)(d1 - d0);            // ta + tb
    const int tb = nt - ta;

    // 1. stage the keys
    {
      uint64_t v[kMergeIpt];
#pragma unroll
      for (int k = 0; k < kMergeIpt; ++k) {
        const int x = t + k * kMergeBlock;
        if (x < nt) v[k] = (x < ta ? a + (i0 + x) : b + (j0 + (x - ta)))->key;
      }
#pragma unroll
      for (int k = 0; k < kMergeIpt; ++k) {
        const int x = t + k * kMergeBlock;
        if (x < nt) keys[x] = v[k];
      }
    }
    __syncthreads();

    // 2. merge kMergeIpt outputs per thread
    const int dl = t * kMergeIpt;
    if (dl < nt) {
      int lo = dl > tb ? dl - tb : 0, hi = dl < ta ? dl : ta;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (key(mid) <= key(ta + dl - 1 - mid)) lo = mid + 1;
        else hi = mid;
      }
      int ia = lo, ib = dl - lo;
      uint64_t ka = key(ia), kb = key(ta + ib);
      const int end = dl + kMergeIpt < nt ? dl + kMergeIpt : nt;
      for (int k = dl; k < end; ++k) {
        const bool take_a = ib >= tb || (ia < ta && ka <= kb);
        idx[k] = (uint16_t)(take_a ? ia : ta + ib);
        if (take_a) ++ia;
        else ++ib;
        const uint64_t nk = key(take_a ? ia : ta + ib);
        if (take_a) ka = nk;
        else kb = nk;
      }
    }
    __syncthreads();

    // 3. gather the records in output order and write them out
    write_out(a, b, out, i0, j0, ta, nt, d0, idx, t);
    __syncthreads();  // the tile's LDS is reused
  }
}

}  // namespace

hipError_t launch_split_init(uint64_t* state, int Q, hipStream_t s) {
  if (Q <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_split_init, dim3((Q + 63) / 64), dim3(64), 0, s, state, Q);
  return hipGetLastError();
}

hipError_t launch_split_cands(const Elem* A, int64_t m, const uint64_t* state, int Q, uint64_t* cnt,
                              hipStream_t s) {
  if (Q <= 0) return hipSuccess;
  const int threads = Q * kSplitCands;
  hipLaunchKernelGGL(k_split_cands, dim3((threads + 255) / 256), dim3(256), 0, s, A, m, state, Q,
                     cnt);
  return hipGetLastError();
}

hipError_t launch_split_update(const uint64_t* gathered, int P, int Q, const int64_t* targets,
                               uint64_t* state, hipStream_t s) {
  if (Q <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_split_update, dim3(Q), dim3(kSplitCands), 0, s, gathered, P, Q, targets,
                     state);
  return hipGetLastError();
}

hipError_t launch_split_final(const Elem* A, int64_t m, const uint64_t* state, int Q, uint64_t* out,
                              hipStream_t s) {
  if (Q <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_split_final, dim3((2 * Q + 63) / 64), dim3(64), 0, s, A, m, state, Q, out);
  return hipGetLastError();
}

hipError_t launch_merge_level(const MergeLevel& level, int64_t* path, int grid, hipStream_t s) {
  if (level.npairs <= 0 || level.npairs > kMergeMaxPairs) return hipErrorInvalidValue;
  if (level.tiles == 0) return hipSuccess;
  const int64_t entries = level.tiles + level.npairs;
  hipLaunchKernelGGL(k_merge_path, dim3((unsigned)((entries + 255) / 256)), dim3(256), 0, s, level,
                     path);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int64_t g = level.tiles < grid ? level.tiles : grid;
  hipLaunchKernelGGL(k_merge2, dim3((unsigned)g), dim3(kMergeBlock), 0, s, level, path);
  return hipGetLastError();
}

}  // namespace lsb
