// Segmented local sort: the last pass of the hybrid local sort
// (LSB_OPT_HYBRID; lsb_runtime.cpp sort_hybrid_rank).
//
// The reference sorts a rank's block by 64 / RADIX stable passes of
// localShuffle (mpi/mpi_lsbsort.cpp:213-247, 580-585), least significant
// digit first; every pass streams the whole block through HBM.  The hybrid
// gets the same stable order from fewer passes over HBM:
//   1. k stable 8-bit k_onesweep passes on the k most significant varying
//      bytes (least significant of them first).  The block is then stably
//      sorted by those bytes: it is a sequence of segments, maximal runs of
//      records whose key agrees on them (key & pmask), each in input order.
//      k is chosen so a segment holds about one record on average (2^30
//      records: k = 4, 2^32 possible prefixes, 0.25 records each).
//   2. k_segsort (this file): every segment stably sorted by the whole key,
//      in one read and one write of the block.
// Records of different segments are ordered by their pmask bits, the top
// varying bits of the key, and equal keys share a segment, so the result is
// the stable sort of the block by key: bit-exact the reference's output.
//
// k_segsort: workgroup g takes tiles g, g + grid, ... of kSegTile records.
// It owns the segments that START in its tile; the last of them may run past
// the tile end, by up to kSegMax records (the "tail", read by wave 0 in
// 64-record steps until the prefix changes).  Records of the tile before its
// first start belong to the previous tile's owner.  A record's rank within
// its segment is counted by walking the segment's keys in LDS in both
// directions: rank = #(keys < mine) + #(equal keys before me), which is the
// stable order.  The walk costs ~segment length per record (about 2 LDS
// reads at the runtime's k); a segment longer than kSegMax sets *err and the runtime falls back to the
// LSD passes (it kept the input).  Records go straight from registers to
// their slot: a wave's 64 records lie in one or two segments, so its stores
// permute within a few contiguous lines, which the memory pipeline merges.
#include "lsb_kernels.h"

namespace lsb {
namespace {

constexpr int kSegBlock = 512;
constexpr int kSegIpt = 8;
constexpr int kSegTile = kSegBlock * kSegIpt;  // 4096 records
static_assert(kSegMax % 64 == 0 && kSegMax <= kSegTile, "tail in 64-record steps");
constexpr int kSegUnroll = 2;  // keys a walk has in flight

__device__ __forceinline__ Elem seg_load_nt(const Elem* p) {
  typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
  const u64x2 v = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(p));
  return Elem{v.x, v.y};
}

#ifndef LSB_SEG_WAVES
#define LSB_SEG_WAVES 6  // waves per SIMD: 3 workgroups of 8 waves per CU
#endif
__global__ __launch_bounds__(kSegBlock) __attribute__((amdgpu_waves_per_eu(LSB_SEG_WAVES))) void k_segsort(const Elem* __restrict__ in,
                                                       Elem* __restrict__ out, int64_t m,
                                                       uint64_t pmask, uint32_t* __restrict__ err) {
  constexpr int T = kSegTile;
  constexpr int KB = T + kSegMax;
  __shared__ uint64_t kbuf[KB];      // keys of the tile, then of its tail
  __shared__ uint64_t tval[kSegMax];  // vals of the tail
  __shared__ int s_w0, s_w1;          // owned records: tile positions [w0, w1)
  const int t = threadIdx.x;
  const int w = t >> 6;
  const int lane = t & 63;
  const int64_t TT = (m + T - 1) / T;
  bool bad = false;

  for (int64_t tile = blockIdx.x; tile < TT; tile += gridDim.x) {
    const int64_t tb = tile * T;
    const int nvalid = (int)((m - tb) < T ? (m - tb) : T);
    const bool last = tb + T >= m;
    if (t == 0) {
      s_w0 = nvalid;
      s_w1 = nvalid;
    }
    Elem e[kSegIpt];
    const int wbase = w * 64 * kSegIpt + lane;
#pragma unroll
    for (int i = 0; i < kSegIpt; ++i) {
      const int li = wbase + i * 64;
      e[i] = li < nvalid ? seg_load_nt(in + tb + li) : Elem{0ull, 0ull};
    }
    const uint64_t prevk = tb > 0 ? in[tb - 1].key : 0ull;
#pragma unroll
    for (int i = 0; i < kSegIpt; ++i) {
      const int li = wbase + i * 64;
      if (li < nvalid) kbuf[li] = e[i].key;
    }
    __syncthreads();
    // The tile's first segment start (position 0 of the block is one).
    {
      int my0 = nvalid;
#pragma unroll
      for (int i = kSegIpt - 1; i >= 0; --i) {
        const int li = wbase + i * 64;
        if (li < nvalid) {
          const uint64_t pk = li == 0 ? prevk : kbuf[li - 1];
          if ((li == 0 && tb == 0) || ((e[i].key ^ pk) & pmask) != 0) my0 = li;
        }
      }
      if (my0 < nvalid) atomicMin(&s_w0, my0);
    }
    // The end of the tile's last segment: the first start at or after the
    // tile's end, found in 64-record steps by wave 0; the records up to it
    // (the tail) go to LDS.
    if (!last && w == 0) {
      const uint64_t lk = kbuf[T - 1];
      int end = -1;
      for (int c = 0; c < kSegMax / 64 && end < 0; ++c) {
        const int64_t p = tb + T + c * 64 + lane;
        const Elem x = p < m ? in[p] : Elem{0ull, 0ull};
        const bool start = p >= m || ((x.key ^ lk) & pmask) != 0;
        const uint64_t b = __ballot(start);
        const int first = b ? (int)__builtin_ctzll(b) : 64;
        if (lane < first) {
          kbuf[T + c * 64 + lane] = x.key;
          tval[c * 64 + lane] = x.val;
        }
        if (b) end = T + c * 64 + first;
      }
      if (end < 0) {  // a segment longer than kSegMax runs on
        bad = true;
        end = T + kSegMax;
      }
      if (lane == 0) s_w1 = end;
    }
    __syncthreads();
    const int w0 = s_w0;
    const int w1 = s_w1 < KB ? s_w1 : KB;
    // Stable rank of one owned record (tile position li) within its segment:
    // walk the segment's keys in LDS both ways, kSegUnroll keys per step.
    auto place = [&](int li, uint64_t key, uint64_t val) {
      const uint64_t pk = key & pmask;
      uint32_t less = 0, eqb = 0;
      const int jlo = li - kSegMax > w0 ? li - kSegMax : w0;
      int j = li - 1;
      bool go = true;
      while (go && j >= jlo) {
        uint64_t k[kSegUnroll];
#pragma unroll
        for (int u = 0; u < kSegUnroll; ++u) k[u] = kbuf[j - u >= 0 ? j - u : 0];
#pragma unroll
        for (int u = 0; u < kSegUnroll; ++u) {
          if (go && j >= jlo) {
            if ((k[u] & pmask) != pk) {
              go = false;
            } else {
              less += k[u] < key ? 1u : 0u;
              eqb += k[u] == key ? 1u : 0u;
              --j;
            }
          }
        }
      }
      if (go && jlo > w0) bad = true;  // still inside the segment kSegMax back
      const int first = j + 1;         // the segment's first tile position
      const int jhi = li + 1 + kSegMax < w1 ? li + 1 + kSegMax : w1;
      j = li + 1;
      go = true;
      while (go && j < jhi) {
        uint64_t k[kSegUnroll];
#pragma unroll
        for (int u = 0; u < kSegUnroll; ++u) k[u] = kbuf[j + u < KB ? j + u : KB - 1];
#pragma unroll
        for (int u = 0; u < kSegUnroll; ++u) {
          if (go && j < jhi) {
            if ((k[u] & pmask) != pk) {
              go = false;
            } else {
              less += k[u] < key ? 1u : 0u;
              ++j;
            }
          }
        }
      }
      if (go && jhi < w1) bad = true;
      int64_t g = tb + first + (int64_t)(less + eqb);
      // In range by construction; the clamp keeps a record of an over-long
      // segment (output invalid, *err set) inside `out`.
      g = g < m ? g : m - 1;
#ifdef LSB_SEG_NT_STORE
      typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
      __builtin_nontemporal_store(u64x2{key, val}, reinterpret_cast<u64x2*>(out + g));
#else
      *reinterpret_cast<ulonglong2*>(out + g) = make_ulonglong2(key, val);
#endif
    };
    if (w0 < nvalid) {
#pragma unroll
      for (int i = 0; i < kSegIpt; ++i) {
        const int li = wbase + i * 64;
        if (li >= w0 && li < nvalid) place(li, e[i].key, e[i].val);
      }
      for (int q = t; q < w1 - T; q += kSegBlock) place(T + q, kbuf[T + q], tval[q]);
    }
    __syncthreads();  // kbuf, s_w0 and s_w1 are rewritten by the next tile
  }
  if (bad) atomicOr(err, 1u);
}

// k_segfix: after the hybrid's last pass with SegPass, the only segments
// out of order are those split between two tiles: a segment lies inside
// one rmask run, and only the run crossing the boundary between tiles t and
// t + 1 has records on both sides.  Each side sorted its part in the stage
// (k_onesweep SEG), and both parts sit in adjacent slots: the end of tile
// t's bucket run, then the start of tile t + 1's.  One wave per boundary
// reads both tiles' lists of the crossing run (slot, key, val), and for
// every bucket present on both sides merges the two sorted parts, stably
// (tile t's records first on equal keys), back into the same slots.  A
// record's new slot: its bucket's first slot on tile t's side + its rank on
// its own side (slot order, which is key order) + the other side's records
// before it.  ~64 records per boundary: loops over LDS broadcasts.
constexpr int kFixWaves = 4;  // boundaries per workgroup (one per wave)
constexpr int kFixLds = 128;  // list entries a wave stages in LDS (more: read from L2)

__global__ __launch_bounds__(64 * kFixWaves) void k_segfix(Elem* __restrict__ out, int64_t m, int shift,
                                                           int64_t TT, SegPass seg) {
  __shared__ SegEntry buf[kFixWaves][kFixLds];  // left part, then right part
  const int w = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  SegEntry* e = buf[w];
  for (int64_t b = (int64_t)blockIdx.x * kFixWaves + w; b + 1 < TT; b += (int64_t)gridDim.x * kFixWaves) {
    const int nl = (int)seg.meta[2 * b];
    const int nr = (int)seg.meta[2 * (b + 1) + 1];
    if (nl == 0 || nr == 0) continue;  // the same for the whole wave
    const SegEntry* L = seg.list + (2 * b) * kSegCap;
    const SegEntry* R = seg.list + (2 * (b + 1) + 1) * kSegCap;
    const int n = nl + nr;
    auto merge = [&](auto get) {
      for (int x = lane; x < n; x += 64) {
        const bool left = x < nl;
        const SegEntry me = get(x);
        const uint32_t c = (uint32_t)(me.key >> shift) & (kBuckets - 1);
        int64_t start = INT64_MAX;
        int own = 0, other = 0, in_l = 0, in_r = 0;
        for (int y = 0; y < n; ++y) {
          const SegEntry o = get(y);
          if (((uint32_t)(o.key >> shift) & (kBuckets - 1)) != c) continue;
          if (y < nl) {
            ++in_l;
            start = o.slot < start ? o.slot : start;
            if (left) own += o.slot < me.slot ? 1 : 0;
            else other += o.key <= me.key ? 1 : 0;
          } else {
            ++in_r;
            if (left) other += o.key < me.key ? 1 : 0;
            else own += o.slot < me.slot ? 1 : 0;
          }
        }
        if (in_l > 0 && in_r > 0) {
          const int64_t g = start + own + other;
          if (g >= 0 && g < m) out[g] = Elem{me.key, me.val};
        }
      }
    };
    if (n <= kFixLds) {
      for (int i = lane; i < n; i += 64) e[i] = i < nl ? L[i] : R[i - nl];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      merge([&](int y) { return e[y]; });
      __builtin_amdgcn_wave_barrier();  // e[] is rewritten for the next boundary
    } else {  // a long crossing run: the lists straight from L2
      merge([&](int y) { return y < nl ? L[y] : R[y - nl]; });
    }
  }
}

}  // namespace

hipError_t launch_segfix(Elem* out, int64_t m, int shift, const SegPass& seg, int grid, hipStream_t s) {
  if (m <= 0) return hipSuccess;
  const int64_t TT = (m + kTile - 1) / kTile;
  if (TT < 2) return hipSuccess;
  int64_t g = grid < 1 ? 1 : grid;
  if (g > TT - 1) g = TT - 1;
  g = (g + kFixWaves - 1) / kFixWaves;
  hipLaunchKernelGGL(k_segfix, dim3((unsigned)g), dim3(64 * kFixWaves), 0, s, out, m, shift, TT, seg);
  return hipGetLastError();
}

hipError_t launch_segsort(const Elem* in, Elem* out, int64_t m, uint64_t pmask, uint32_t* err,
                          int grid, hipStream_t s) {
  if (m <= 0) return hipSuccess;
  const int64_t TT = (m + kSegTile - 1) / kSegTile;
#ifdef LSB_SEG_GRID_PER_CU  // A/B: workgroups per CU (the runtime passes 3)
  grid = grid / 3 * LSB_SEG_GRID_PER_CU;
#endif
  int64_t g = grid < 1 ? 1 : grid;
  if (g > TT) g = TT;
  hipLaunchKernelGGL(k_segsort, dim3((unsigned)g), dim3(kSegBlock), 0, s, in, out, m, pmask, err);
  return hipGetLastError();
}

}  // namespace lsb
