// Segmented local sort: the last pass of the hybrid local sort
// (LSB_OPT_HYBRID; lsb_passes.cpp LocalSort).
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
#include "lsb_device.h"

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
// t's bucket-d block, then the start of tile t + 1's, both at
// P = base[sub-array of t][d] + tile t's inclusive look-back value for d.
// The pass itself records nothing: one wave per boundary finds the crossing
// run in the pass's input (records [b - a, b + c) around the boundary b,
// the pass's input being sorted by rmask), counts both sides per bucket in
// LDS, and re-places only the records of buckets present on both sides:
// slot = P - (left count) + #(keys < mine) + #(equal keys before me in the
// input), over the few such records (~4 buckets of ~64 run records at
// 2^30).  A run longer than CAP on one side, one spanning a whole tile (its
// segments then touch three tiles), or more than CAP records to re-place
// sets *err: the runtime sorts the segments with k_segsort instead.  The
// records to re-place are grouped by bucket in LDS, so each ranks itself
// against its own bucket's few.  Two shapes: CAP = kSegCap (256), one
// 64-record chunk per side loaded up front, 20 KiB of LDS per 4 waves (32
// waves per CU), when runs hold <= 64 records (m <= 2^30 at k = 4); and
// CAP = 1024, four chunks per side, 28 KiB per 2 waves, for longer runs
// (2^32 records: ~256 per run).
__device__ __forceinline__ uint64_t lane0_u64(uint64_t x) {
  return ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(x >> 32)) << 32) |
         (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)x);
}

// QW: 64-record chunks per side a boundary loads at once.
template <int CAP, int WAVES, int QW>
__global__ __launch_bounds__(64 * WAVES) void k_segfix(const Elem* __restrict__ in, Elem* __restrict__ out,
                                                       int64_t m, int shift, int64_t TT,
                                                       const uint32_t* __restrict__ status, SegPass seg) {
  static_assert(CAP < 0x8000, "16-bit side counts");
  __shared__ uint32_t cnt[WAVES][kBuckets];   // left count | right count << 16
  __shared__ uint32_t moff[WAVES][kBuckets];  // a bucket's slice of mkey / mpos
  __shared__ uint64_t mkey[WAVES][CAP];       // the records to re-place (at most
  __shared__ uint32_t mpos[WAVES][CAP];       // CAP), by bucket: key, position in the run
  const int w = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const uint64_t* __restrict__ K = reinterpret_cast<const uint64_t*>(in);
  auto wave_sync = []() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  };
  bool bad = false;
  for (int64_t t = (int64_t)blockIdx.x * WAVES + w; t + 1 < TT; t += (int64_t)gridDim.x * WAVES) {
    const int64_t b = (t + 1) * kTile;  // tile t + 1's first record
    const int64_t lo = t * kTile, hi = b + kTile < m ? b + kTile : m;
    // The QW 64-record chunks on each side of b in one round trip: the
    // boundary test, the run's extent and its keys (runs longer than that
    // are scanned on and re-read from L2).
    uint64_t kl[QW], kr[QW];
#pragma unroll
    for (int q = 0; q < QW; ++q) {
      const int64_t il = b - 1 - 64 * q - lane, ir = b + 64 * q + lane;
      kl[q] = il >= lo ? K[2 * il] : 0ull;
      kr[q] = ir < hi ? K[2 * ir] : 0ull;
    }
    const uint64_t v = lane0_u64(kl[0]) & seg.rmask;  // K[b - 1]
    if ((lane0_u64(kr[0]) & seg.rmask) != v) continue;  // the same for the whole wave
    int a = -1, c = -1;  // the run's records before / from b, up to the two tiles' ends
#pragma unroll
    for (int q = 0; q < QW; ++q) {
      const int64_t il = b - 1 - 64 * q - lane, ir = b + 64 * q + lane;
      const uint64_t sl = __ballot(!(il >= lo && (kl[q] & seg.rmask) == v));
      const uint64_t sr = __ballot(!(ir < hi && (kr[q] & seg.rmask) == v));
      if (a < 0 && sl) a = 64 * q + __builtin_ctzll(sl);
      if (c < 0 && sr) c = 64 * q + __builtin_ctzll(sr);
    }
    const bool fast = a >= 0 && c >= 0;
    if (a < 0) {
      a = 64 * QW;
      for (;;) {
        const int64_t i = b - 1 - a - lane;
        const uint64_t stop = __ballot(!(i >= lo && (K[2 * i] & seg.rmask) == v));
        a += stop ? __builtin_ctzll(stop) : 64;
        if (stop || a > CAP) break;
      }
    }
    if (c < 0) {
      c = 64 * QW;
      for (;;) {
        const int64_t i = b + c + lane;
        const uint64_t stop = __ballot(!(i < hi && (K[2 * i] & seg.rmask) == v));
        c += stop ? __builtin_ctzll(stop) : 64;
        if (stop || c > CAP) break;
      }
    }
    if (a > CAP || c > CAP || (b - a == lo && lo > 0 && (K[2 * (lo - 1)] & seg.rmask) == v) ||
        (b + c == hi && hi < m && (K[2 * hi] & seg.rmask) == v)) {
      bad = true;
      continue;
    }
    const int n = a + c;
    const int64_t r0 = b - a;
    // f(key, position in the run, valid) for every record of the run, 64 at
    // a time (wave-uniform calls): from the registers, or from L2.
    auto for_each = [&](auto&& f) {
      if (fast) {
#pragma unroll
        for (int q = 0; q < QW; ++q) {
          const int dist = 64 * q + lane;
          f(kl[q], a - 1 - dist, dist < a);
        }
#pragma unroll
        for (int q = 0; q < QW; ++q) {
          const int p = 64 * q + lane;
          f(kr[q], a + p, p < c);
        }
      } else {
        for (int x0 = 0; x0 < n; x0 += 64) {
          const int x = x0 + lane;
          f(x < n ? K[2 * (r0 + x)] : 0ull, x, x < n);
        }
      }
    };
    for (int d = lane; d < kBuckets; d += 64) cnt[w][d] = 0;
    wave_sync();
    for_each([&](uint64_t k, int x, bool ok) {
      if (ok) atomicAdd(&cnt[w][(uint32_t)(k >> shift) & (kBuckets - 1)], x < a ? 1u : 0x10000u);
    });
    wave_sync();
    // The records to re-place (buckets with both sides), grouped by bucket:
    // lane l owns buckets 4l..4l+3 and their slices' starts.
    auto both = [](uint32_t cc) { return (cc & 0xFFFFu) && (cc >> 16) ? (cc & 0xFFFFu) + (cc >> 16) : 0u; };
    uint32_t own = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) own += both(cnt[w][4 * lane + j]);
    uint32_t incl = own;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t o = __shfl_up(incl, off, 64);
      if (lane >= off) incl += o;
    }
    const int nm = (int)__shfl(incl, 63, 64);
    if (nm > CAP) {  // the same for the whole wave
      bad = true;
      wave_sync();
      continue;
    }
    uint32_t start = incl - own;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      moff[w][4 * lane + j] = start;
      start += both(cnt[w][4 * lane + j]);
    }
    wave_sync();
    for_each([&](uint64_t k, int x, bool ok) {
      if (!ok) return;
      const uint32_t d = (uint32_t)(k >> shift) & (kBuckets - 1);
      if (!both(cnt[w][d])) return;
      const uint32_t q = atomicAdd(&moff[w][d], 1u);  // any order: x breaks ties
      mkey[w][q] = k;
      mpos[w][q] = (uint32_t)x;
    });
    wave_sync();
    const int x_t = sub_of_tile(t, TT);
    for (int y = lane; y < nm; y += 64) {
      const uint64_t k = mkey[w][y];
      const uint32_t x = mpos[w][y];
      const uint32_t d = (uint32_t)(k >> shift) & (kBuckets - 1);
      uint32_t before = 0;
      const uint32_t z1 = moff[w][d];  // the end of bucket d's slice
      for (uint32_t z = z1 - both(cnt[w][d]); z < z1; ++z) {
        const uint64_t kz = mkey[w][z];
        before += (kz < k || (kz == k && mpos[w][z] < x)) ? 1u : 0u;
      }
      const int64_t P = seg.base[x_t * kBuckets + d] + (int64_t)(status[t * kBuckets + d] & kStatusValMask);
      const int64_t g = P - (int64_t)(cnt[w][d] & 0xFFFFu) + (int64_t)before;
      if (g >= 0 && g < m) out[g] = Elem{k, in[r0 + x].val};
    }
    wave_sync();  // cnt, mkey and mpos are rewritten for the next boundary
  }
  if (bad) atomicOr(seg.err, 1u);
}

}  // namespace

hipError_t launch_segfix(const Elem* in, Elem* out, int64_t m, int shift, const uint32_t* status,
                         const SegPass& seg, int grid, hipStream_t s) {
  if (m <= 0) return hipSuccess;
  const int64_t TT = (m + kTile - 1) / kTile;
  if (TT < 2) return hipSuccess;
  int64_t g = grid < 1 ? 1 : grid;
  if (g > TT - 1) g = TT - 1;
  // Records per run value: m over the run key's 2^bits values.
  const int rbits = __builtin_popcountll(seg.rmask);
  const int64_t rlen = rbits >= 62 ? 0 : m >> rbits;
  if (rlen <= 64) {
    g = (g + 3) / 4;
    hipLaunchKernelGGL((k_segfix<kSegCap, 4, 1>), dim3((unsigned)g), dim3(256), 0, s, in, out, m, shift, TT,
                       status, seg);
  } else {
    g = (g + 1) / 2;
    hipLaunchKernelGGL((k_segfix<4 * kSegCap, 2, 4>), dim3((unsigned)g), dim3(128), 0, s, in, out, m, shift, TT,
                       status, seg);
  }
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
