// HIP kernels of the MI355X-native LSD radix sort (gfx950 / CDNA4).
//
// A sort's local passes (localShuffle, mpi/mpi_lsbsort.cpp:213-247) read
// each record once per pass:
//   k_subhist  the first digit's histogram per sub-array, once per sort
//              (count loop :226-229), plus the key span
//   k_onesweep count + scan + stable scatter of one 8-bit digit in one read
//              (:226-246): offsets by decoupled look-back, and the next
//              digit's histogram counted as the records are written
// The reduce-then-scan form of the same pass (lsb_pass, LSB_OPT_ONESWEEP = 0):
//   k_upsweep  per-chunk digit histogram         (count loop, :226-229)
//   k_scan     chunk x bucket exclusive scan      (starts, :232-238 / exclusiveScan :385-414)
//   k_scatter  stable scatter through LDS         (shuffle loop, :241-246)
// and, when P > 1, after the RCCL exchange,
//   k_place    received runs -> final local slots (placement loop, :568-575),
//              counting the next local digit's histogram as it writes
//
// Everything is integer indexing, so the bound is HBM, not MFMA.  Design
// points for CDNA4:
//   * 16-byte records move as one dwordx4 per lane; tiles are read with
//     consecutive lanes on consecutive records (1 KiB per wave-instruction).
//   * Stable in-tile ranking uses 64-lane __ballot match masks (8 ballots
//     for 8 bits): rank = popc(match & lanemask_lt) + a per-wave LDS counter,
//     so equal digits never contend on an LDS atomic.
//   * The ranked tile is staged in LDS (64 KiB) and written back in
//     tile-sorted order, so each bucket's run leaves the CU as contiguous
//     16-byte stores from consecutive lanes.
#include "lsb_device.h"
#include <type_traits>

// Debug build (make debug, -DLSB_DEBUG): device-side bounds asserts on every
// scattered store.  A failing assert prints and traps the kernel.
#ifdef LSB_DEBUG
#include <cassert>
#define LSB_DASSERT(c) assert(c)
#else
#define LSB_DASSERT(c) ((void)0)
#endif

namespace lsb {
namespace {

typedef unsigned __int128 u128;

constexpr u128 kPcgMult = ((u128)0x2360ED051FC65DA4ULL << 64) | (u128)0x4385DF649FCCF645ULL;
constexpr u128 kPcgInc = ((u128)0x5851F42D4C957F2DULL << 64) | (u128)0x14057B7EF767814FULL;

// LCG jump table: stepping 2^k times is s -> mul[k]*s + add[k].
struct JumpTable {
  uint64_t mul_lo[64], mul_hi[64], add_lo[64], add_hi[64];
};

constexpr JumpTable make_jump_table() {
  JumpTable t{};
  u128 m = kPcgMult, a = kPcgInc;
  for (int k = 0; k < 64; ++k) {
    t.mul_lo[k] = (uint64_t)m;
    t.mul_hi[k] = (uint64_t)(m >> 64);
    t.add_lo[k] = (uint64_t)a;
    t.add_hi[k] = (uint64_t)(a >> 64);
    a = a * (m + 1);
    m = m * m;
  }
  return t;
}

__constant__ JumpTable kJump = make_jump_table();

__device__ __forceinline__ uint64_t pcg_output(u128 s) {
  const uint64_t x = (uint64_t)(s >> 64) ^ (uint64_t)s;
  const unsigned rot = (unsigned)(s >> 122);
  return (x >> rot) | (x << ((64u - rot) & 63u));
}

__device__ __forceinline__ u128 pcg_seed(uint64_t seed) {
  return ((u128)seed + kPcgInc) * kPcgMult + kPcgInc;
}

// Advance by `delta` steps; the 2^k maps commute, so bit order is free.
__device__ __forceinline__ u128 pcg_jump(u128 s, uint64_t delta) {
  while (delta) {
    const int k = __builtin_ctzll(delta);
    const u128 m = ((u128)kJump.mul_hi[k] << 64) | kJump.mul_lo[k];
    const u128 a = ((u128)kJump.add_hi[k] << 64) | kJump.add_lo[k];
    s = s * m + a;
    delta &= delta - 1;
  }
  return s;
}

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// popc(mask & lanemask_lt) in two instructions.
__device__ __forceinline__ uint32_t mbcnt(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                   __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// Lanes of `active` whose 8-bit digit equals mine.  Per bit: t = my bit
// sign-extended (0 or ~0), bal = lanes with the bit set, and the lanes whose
// bit equals mine are ~(bal ^ t); one gfx950 v_bitop3 per 32-bit half folds
// that into the running mask (truth table 0x90 = a & ~(b ^ c), index
// a*4 + b*2 + c).  4 VALU per bit: v_bfe_i32, v_cmp_ne (the ballot, taken
// on t itself through the compare intrinsic; __ballot(t != 0) let the
// compiler re-derive the bit with a shift, 5 per bit), two v_bitop3.  The
// select form (set ? bal : ~bal) compiles to 9.
__device__ __forceinline__ uint64_t match_digit8(uint32_t d, uint64_t active) {
  uint32_t lo = (uint32_t)active, hi = (uint32_t)(active >> 32);
#pragma unroll
  for (int bit = 0; bit < 8; ++bit) {
    const uint32_t t = (uint32_t)__builtin_amdgcn_sbfe((int)d, bit, 1);
    const uint64_t bal = __builtin_amdgcn_uicmp(t, 0u, 33);  // ICMP_NE: lanes whose bit is set
    lo = __builtin_amdgcn_bitop3_b32(lo, (uint32_t)bal, t, 0x90);
    hi = __builtin_amdgcn_bitop3_b32(hi, (uint32_t)(bal >> 32), t, 0x90);
  }
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ Elem load_elem(const Elem* p) {
  const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(p);
  return Elem{v.x, v.y};
}

// Streaming load: the record is read once per pass, so its line is marked
// for early eviction and L2 keeps room for the run-boundary lines the next
// tile completes (k_onesweep: -1...-5 % per sort, tools/ab.sh).
__device__ __forceinline__ Elem load_elem_nt(const Elem* p) {
  typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
  const u64x2 v = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(p));
  return Elem{v.x, v.y};
}

__device__ __forceinline__ void store_elem(Elem* p, const Elem& e) {
  *reinterpret_cast<ulonglong2*>(p) = make_ulonglong2(e.key, e.val);
}

// Inclusive wave scan (64 lanes).
template <typename T>
__device__ __forceinline__ T wave_inclusive_scan(T v) {
  const uint32_t lane = lane_id();
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const T u = __shfl_up(v, off, 64);
    if (lane >= (uint32_t)off) v += u;
  }
  return v;
}

// 32-bit form on DPP row shifts and row broadcasts (the generic form's
// __shfl_up is one ds_bpermute round trip per step).  Every lane active.
template <>
__device__ __forceinline__ uint32_t wave_inclusive_scan<uint32_t>(uint32_t v) {
  const uint32_t lane = lane_id(), rl = lane & 15u;
  uint32_t t;
  t = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
  if (rl >= 1) v += t;
  t = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
  if (rl >= 2) v += t;
  t = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
  if (rl >= 4) v += t;
  t = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
  if (rl >= 8) v += t;
  t = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x142, 0xf, 0xf, false);  // row_bcast:15
  if ((lane & 31u) >= 16) v += t;
  t = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x143, 0xf, 0xf, false);  // row_bcast:31
  if (lane >= 32) v += t;
  return v;
}

// The value of the neighbouring lane t ^ 1 (DPP quad_perm [1,0,3,2]).
__device__ __forceinline__ uint32_t pair_swap(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xf, 0xf, false);
}

// Exclusive scan over the whole workgroup (every thread must call it).
// `tmp` needs BLOCK/64 entries.  *total receives the block sum.
template <int BLOCK, typename T>
__device__ __forceinline__ T block_exclusive_scan(T v, T* tmp, T* total) {
  constexpr int W = BLOCK / 64;
  const int w = threadIdx.x >> 6;
  const T inc = wave_inclusive_scan(v);
  if (lane_id() == 63) tmp[w] = inc;
  __syncthreads();
  T pre = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < W; ++i) {
    const T x = tmp[i];
    pre += (i < w) ? x : T(0);
    tot += x;
  }
  __syncthreads();
  *total = tot;
  return pre + inc - v;
}

// ---------------------------------------------------------------- PCG fill
constexpr int kFillPerThread = 16;

// splitmix64 finalizer: a bijection on 64-bit words.
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Key of a record from its PCG draw.  Uniform: the draw itself (the
// reference's input).  Zipf (build-defined): rank
// k = floor(x) of a continuous power law on [1, N+1) with exponent s, by
// inverse CDF from u = top 53 bits of the draw; key = mix64(k), so every
// digit is skewed and duplicate keys are heavy.
__device__ __forceinline__ uint64_t make_key(uint64_t draw, const KeyGen& g) {
  if (g.dist == kDistUniform) return draw;
  const double u = (double)(draw >> 11) * 0x1.0p-53;  // [0, 1)
  const double n1 = (double)g.zipf_n + 1.0;
  double x;
  if (g.zipf_s == 1.0) {
    x = exp(u * log(n1));
  } else {
    const double e = 1.0 - g.zipf_s;
    x = pow(1.0 - u * (1.0 - pow(n1, e)), 1.0 / e);
  }
  uint64_t k = (uint64_t)x;
  if (k < 1) k = 1;
  if (k > g.zipf_n) k = g.zipf_n;
  return mix64(k);
}

__global__ __launch_bounds__(256) void k_pcg_fill(Elem* __restrict__ A, int64_t count,
                                                  uint64_t seed, uint64_t val0, KeyGen g) {
  const int64_t first = ((int64_t)blockIdx.x * 256 + threadIdx.x) * kFillPerThread;
  if (first >= count) return;
  u128 s = pcg_jump(pcg_seed(seed), (uint64_t)first);
  const int64_t last = first + kFillPerThread < count ? first + kFillPerThread : count;
  for (int64_t i = first; i < last; ++i) {
    s = s * kPcgMult + kPcgInc;  // operator(): bump, then output the new state
    store_elem(A + i, Elem{make_key(pcg_output(s), g), val0 + (uint64_t)i});
  }
}

// ----------------------------------------------------------------- upsweep
// Per-wave LDS histograms with plain ds_add: on uniform digits this runs at
// the pure-read rate (2.80 ms for 2^30 records = 6.1 TB/s, vs 3.57 ms with
// ballot-match aggregation; tools/kbench/upsweep.hip).  A wave whose 64
// digits are all equal (sorted or skewed input) adds once instead of
// serialising 64 same-address atomics.
//
// SPAN (first pass of lsb_sort only): also OR-reduce the keys and their
// complements into span[0], span[1]; bit i of span[0] & span[1] is set iff
// keys differ in bit i.  Digits with no such bit are skipped.
template <int BLOCK, int IPT, bool SPAN>
__global__ __launch_bounds__(BLOCK) void k_upsweep(const Elem* __restrict__ A, int64_t m,
                                                   int shift, int64_t chunk_elems, int G,
                                                   uint32_t* __restrict__ chunk_hist,
                                                   unsigned long long* __restrict__ span) {
  constexpr int W = BLOCK / 64;
  __shared__ uint32_t hist[W][kBuckets];
  __shared__ uint64_t span_or[W], span_nor[W];
  uint64_t kor = 0, knor = 0;
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
      k[i] = idx < end ? __builtin_nontemporal_load(keys + 2 * idx) : 0ull;  // streaming
    }
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      const int64_t idx = tb + (int64_t)i * BLOCK + threadIdx.x;
      const bool valid = idx < end;
      if (SPAN && valid) {
        kor |= k[i];
        knor |= ~k[i];
      }
      const uint32_t d = (uint32_t)(k[i] >> shift) & (kBuckets - 1);
      const uint32_t d0 = __builtin_amdgcn_readfirstlane(d);
      if (__all(valid && d == d0)) {
        if (lane_id() == 0) atomicAdd(&hist[w][d0], 64u);
      } else if (valid) {
        atomicAdd(&hist[w][d], 1u);
      }
    }
  }
  __syncthreads();
  for (int b = threadIdx.x; b < kBuckets; b += BLOCK) {
    uint32_t s = 0;
#pragma unroll
    for (int ww = 0; ww < W; ++ww) s += hist[ww][b];
    chunk_hist[(int64_t)b * G + c] = s;
  }
  if (SPAN) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      kor |= __shfl_xor(kor, off, 64);
      knor |= __shfl_xor(knor, off, 64);
    }
    if (lane_id() == 0) {
      span_or[w] = kor;
      span_nor[w] = knor;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      uint64_t o = 0, no = 0;
#pragma unroll
      for (int ww = 0; ww < W; ++ww) {
        o |= span_or[ww];
        no |= span_nor[ww];
      }
      atomicOr(&span[0], (unsigned long long)o);
      atomicOr(&span[1], (unsigned long long)no);
    }
  }
}

// -------------------------------------------------------------------- scan
constexpr int kScanBlock = 256;
constexpr int kScanPer = 4;  // one segment = 1024 chunks

// One workgroup per bucket row; the row is scanned in segments of
// kScanBlock * kScanPer chunks with a running carry.
__global__ __launch_bounds__(kScanBlock) void k_scan(const uint32_t* __restrict__ chunk_hist,
                                                     int G, uint64_t* __restrict__ chunk_off,
                                                     uint64_t* __restrict__ totals) {
  __shared__ uint64_t tmp[kScanBlock / 64];
  const int b = blockIdx.x;
  const uint32_t* row = chunk_hist + (int64_t)b * G;
  uint64_t carry = 0;
  for (int seg = 0; seg < G; seg += kScanBlock * kScanPer) {
    uint32_t v[kScanPer];
    uint64_t sum = 0;
#pragma unroll
    for (int j = 0; j < kScanPer; ++j) {
      const int c = seg + threadIdx.x * kScanPer + j;
      v[j] = c < G ? row[c] : 0u;
      sum += v[j];
    }
    uint64_t total;
    uint64_t pre = carry + block_exclusive_scan<kScanBlock>(sum, tmp, &total);
#pragma unroll
    for (int j = 0; j < kScanPer; ++j) {
      const int c = seg + threadIdx.x * kScanPer + j;
      if (c < G) chunk_off[(int64_t)b * G + c] = pre;
      pre += v[j];
    }
    carry += total;
  }
  if (threadIdx.x == 0) totals[b] = carry;
}

// ----------------------------------------------------------------- scatter
// One workgroup walks its chunk tile by tile.  A tile is split wave-major:
// wave w owns tile elements [w*64*IPT, (w+1)*64*IPT) and its item i is the
// 64 consecutive elements starting at w*64*IPT + i*64, so tile order is
// (wave, item, lane) and every load is a coalesced 1 KiB wave-instruction.
//
// Whole-line writes.  A tile's run of bucket b starts at an arbitrary record,
// so its first and last 128-B lines are shared with the previous and next
// tile's runs.  Written ~20 us apart, such a line is usually evicted from L2
// half-written and HBM pays for a partial-line write (measured: 256-B runs
// misaligned by 16 B drop from 4.6 to 3.6 TB/s; tools/kbench/runs2.hip).
// So a tile writes only [A_b, E_b) with E_b on a line boundary and keeps the
// <= 7 records of its last, incomplete line in registers of thread b (the
// "carry"); the next tile writes them in the same phase as the rest of that
// line, and L2 merges the line before it leaves.  Only a chunk's first and
// last line per bucket can still be partial.
constexpr int kLineElems = 8;  // 128-B line / 16-B record

// STARTS (P > 1, high byte of a 16-bit exchange digit): the output is then
// sorted by the 16-bit digit at shift16 = shift - 8, and the exchange needs
// its 65536 counts.  Instead of re-reading the output (k_digit_starts), the
// scatter marks where a 16-bit digit may begin: a record whose predecessor
// in the output has a different low byte, or is unknown.  A workgroup's
// bucket-b records land contiguously in stream order, so the predecessor is
// the previous record of the tile's run, the last record of this
// workgroup's previous run in b (prevlo[b]), or another workgroup's
// (unknown: the chunk's first record in b).  atomicMin over the marks is the
// first position of every digit: every true start is marked, and every other
// mark lies after it.  The input is sorted by the low byte, so a tile whose
// first and last records share it has one low byte throughout: only each
// run's first record needs a look (by its bucket's thread, once per tile).
// The rare tile across a low-byte boundary walks its runs.
template <int BLOCK, int IPT, bool STARTS>
__global__ __launch_bounds__(BLOCK, BLOCK / 128) void k_scatter(const Elem* __restrict__ in,
                                                      Elem* __restrict__ out, int64_t m,
                                                      int shift, int64_t chunk_elems, int G,
                                                      const uint64_t* __restrict__ chunk_off,
                                                      const uint64_t* __restrict__ totals,
                                                      long long* __restrict__ first16) {
  constexpr int W = BLOCK / 64;
  constexpr int T = BLOCK * IPT;
  constexpr int CY = kLineElems - 1;
  static_assert(BLOCK >= kBuckets, "one thread per bucket in the offset phase");

  __shared__ Elem stage[T];                 // the ranked tile (64 KiB)
  __shared__ uint32_t wcnt[W][kBuckets];    // per-wave digit counters -> positions
  __shared__ int64_t delta[kBuckets];       // global dest = delta[digit] + tile position
  __shared__ int64_t lim[kBuckets];         // write only dest < lim[digit] (E_b)
  __shared__ uint64_t scan64[W];
  __shared__ uint32_t scan32[W];
  __shared__ int32_t prevlo[STARTS ? kBuckets : 1];  // low byte of b's last record, -1 = none
  __shared__ uint32_t tile_lo[2];                     // low byte of the tile's first, last record

  const int t = threadIdx.x;
  const int w = t >> 6;
  const uint32_t lane = lane_id();
  const int c = blockIdx.x;
  const int64_t beg = (int64_t)c * chunk_elems;
  const int64_t end = beg + chunk_elems < m ? beg + chunk_elems : m;
  const int shift16 = shift - 8;
  if (STARTS && t < kBuckets) prevlo[t] = -1;

  // Global start of this chunk's run of each bucket.
  uint64_t run = 0;
  {
    const uint64_t tot = t < kBuckets ? totals[t] : 0ull;
    uint64_t all;
    const uint64_t bstart = block_exclusive_scan<BLOCK>(tot, scan64, &all);
    if (t < kBuckets) run = bstart + chunk_off[(int64_t)t * G + c];
  }
  // Carry of bucket t (thread t < 256): records for dest [run - cy_len, run).
  Elem cy[CY];
  uint32_t cy_len = 0;
#pragma unroll
  for (int i = 0; i < CY; ++i) cy[i] = Elem{0ull, 0ull};

  for (int64_t tb = beg; tb < end; tb += T) {
    const int nvalid = (int)((end - tb) < T ? (end - tb) : T);
    const bool last_tile = tb + T >= end;

#pragma unroll
    for (int j = 0; j < kBuckets / 64; ++j) wcnt[w][lane + 64 * j] = 0;

    Elem e[IPT];
    const int wbase = w * 64 * IPT + (int)lane;
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      const int li = wbase + i * 64;
      e[i] = li < nvalid ? load_elem(in + tb + li) : Elem{0ull, 0ull};
    }

    // Stable rank of every element among the wave's elements of its digit.
    uint32_t rk[IPT];
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      const bool valid = wbase + i * 64 < nvalid;
      const uint32_t d = (uint32_t)(e[i].key >> shift) & (kBuckets - 1);
      const uint64_t mt = match_digit8(d, __ballot(valid));
      const uint32_t below = mbcnt(mt);
      const uint32_t pre = wcnt[w][d];
      rk[i] = pre + below;
      if (STARTS && (wbase + i * 64 == 0 || wbase + i * 64 == nvalid - 1))
        tile_lo[wbase + i * 64 == 0 ? 0 : 1] = (uint32_t)(e[i].key >> shift16) & 0xFFu;
      if (valid && below == 0) wcnt[w][d] = pre + (uint32_t)__popcll(mt);
    }
    __syncthreads();

    // Per digit: wave-exclusive prefix, tile-local start, global delta.
    uint32_t cnt = 0;
    if (t < kBuckets) {
#pragma unroll
      for (int ww = 0; ww < W; ++ww) {
        const uint32_t x = wcnt[ww][t];
        wcnt[ww][t] = cnt;
        cnt += x;
      }
    }
    uint32_t tile_total;
    const uint32_t lstart = block_exclusive_scan<BLOCK>(cnt, scan32, &tile_total);
    // Read now: the next tile rewrites tile_lo before its first barrier.
    const uint32_t tlo0 = STARTS ? tile_lo[0] : 0u;
    const bool tmixed = STARTS && tile_lo[0] != tile_lo[1];
    // Run of bucket t in this tile: dest [R, R + cnt); carried [A, R).
    // Write [A, E): E = end of the last whole line, or everything at the
    // chunk's last tile; E == A means the line is still incomplete.
    int64_t R = 0, A = 0, E = 0, run_end = 0;
    bool flush_carry = false;
    if (t < kBuckets) {
#pragma unroll
      for (int ww = 0; ww < W; ++ww) wcnt[ww][t] += lstart;
      R = (int64_t)run;
      A = R - (int64_t)cy_len;
      run_end = R + cnt;
      const int64_t aligned = run_end & ~(int64_t)(kLineElems - 1);
      E = last_tile ? run_end : (aligned > A ? aligned : A);
      flush_carry = E > A;
      delta[t] = R - (int64_t)lstart;
      lim[t] = E;
      run = (uint64_t)run_end;
    }
    __syncthreads();

#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      if (wbase + i * 64 < nvalid) {
        const uint32_t d = (uint32_t)(e[i].key >> shift) & (kBuckets - 1);
        stage[wcnt[w][d] + rk[i]] = e[i];
      }
    }
    __syncthreads();

    for (int j = t; j < nvalid; j += BLOCK) {
      const Elem x = stage[j];
      const uint32_t d = (uint32_t)(x.key >> shift) & (kBuckets - 1);
      const int64_t g = delta[d] + j;
      if (g < lim[d]) {
        LSB_DASSERT(g >= 0 && g < m);
        store_elem(out + g, x);
      }
    }
    // The carried head of each line goes out in the same phase as its rest.
    if (flush_carry) {
#pragma unroll
      for (int i = 0; i < CY; ++i)
        if ((uint32_t)i < cy_len) {
          LSB_DASSERT(A + i >= 0 && A + i < m);
          store_elem(out + A + i, cy[i]);
        }
    }
    __syncthreads();

    // New carry: records for dest [E, run_end).  If nothing was written the
    // old carry stays in front and this tile's records are appended.
    if (t < kBuckets) {
      const uint32_t keep = flush_carry ? 0u : cy_len;
      const int64_t src0 = flush_carry ? (int64_t)lstart + (E - R) : (int64_t)lstart;
      const uint32_t new_len = (uint32_t)(run_end - E);
#pragma unroll
      for (int i = 0; i < CY; ++i) {
        if ((uint32_t)i >= keep && (uint32_t)i < new_len) cy[i] = stage[src0 + (i - (int)keep)];
      }
      cy_len = new_len;
      if (STARTS && cnt > 0) {
        // Run of bucket t in this tile: stage [lstart, lstart + cnt) -> out [R, ...).
        uint32_t lo = (uint32_t)(stage[lstart].key >> shift16) & 0xFFu;
        if (prevlo[t] != (int32_t)lo)
          atomicMin(&first16[(stage[lstart].key >> shift16) & 0xFFFFu], (long long)R);
        if (tmixed) {  // the tile straddles a low-byte boundary
          for (uint32_t k = 1; k < cnt; ++k) {
            const uint64_t key = stage[lstart + k].key;
            const uint32_t l = (uint32_t)(key >> shift16) & 0xFFu;
            if (l != lo) atomicMin(&first16[(key >> shift16) & 0xFFFFu], (long long)(R + k));
            lo = l;
          }
        } else {
          lo = tlo0;
        }
        prevlo[t] = (int32_t)lo;
      }
    }
  }
}

// ---------------------------------------------------------------- onesweep
// Single-read passes for P == 1 (the same stable counting pass,
// mpi/mpi_lsbsort.cpp:213-247, without the count re-read).  Reduce-then-scan
// reads every record twice per pass (k_upsweep, k_scatter) only to learn
// each chunk's bucket offsets.  Here those come from a decoupled look-back
// and from a histogram the previous pass produced as it wrote:
//
//   * The m records are kTile-record tiles, grouped into kSub = 8 contiguous
//     sub-arrays: sub-array x = tiles [x*TT/8, (x+1)*TT/8) (floor), so tile
//     t lies in sub-array (8t + 7) / TT.  Workgroups with the same
//     blockIdx % 8 share an XCD; that group takes sub-array blockIdx % 8's
//     tiles in order from its own counter, then helps the next sub-array
//     (the tail balances itself).  Consecutive tiles of a run boundary thus
//     mostly complete their shared 128-B lines in one XCD's L2.
//   * Record (tile t, bucket b) goes to bucket_start[b] + sub_pre[x][b] +
//     excl[t][b] + rank in tile, where sub_pre = exclusive prefix of the
//     sub-array histogram over x (known before the pass) and excl = the
//     sum of b-counts of earlier tiles of the same sub-array, found by a
//     look-back over status granules: status[t][b] = one self-tagged u32,
//     bits 0-29 the value, bit 30 set for an inclusive prefix (clear: the
//     tile's own count, its "aggregate"), bit 31 the launch's epoch parity.
//     Every launch writes every tile's row (a context's m never changes), so
//     a row holds either this launch's value or the previous launch's, whose
//     parity differs: status needs no reset (zeroed once at allocation; the
//     first launch has parity 1), and a granule is half the bytes of a
//     {value, tag} word pair (the status traffic was 6 % of the pass's HBM
//     bytes).  Buckets b, b+1 travel as one 8-byte write-through (sc1) buffer
//     store, polled with 8-byte sc1 loads (the guide's R2 form: the data is
//     the flag, no fences); each half carries its own tag and a pair is used
//     only when both agree.  The tile publishes its aggregate right after ranking and
//     reads its predecessor while it scans and stages; one predecessor per
//     round trip measured fastest (wider windows: +6 % at 2, +11 % at 4),
//     and the next tile's id is fetched while this one's records are written.
//   * NEXT: the pass also accumulates the sub-array histogram of the next
//     digit over its OUTPUT positions (the next pass's sub-arrays), in LDS,
//     one add per record, flushed with global atomics at the end.
//   * Workgroup shape: the 64 KiB stage holds a CU to 2 workgroups, so the
//     whole-stage form runs 8 waves x 8 records (kOsBlock = 512; threads
//     t < 256 own bucket t, the rest only load, rank, stage and write): the
//     rank chains are half as long and twice the waves hide them, -2.8 % per
//     sort against 4 waves x 16 (profiles/ab/r02_ab27_*).  The split stage
//     keeps 4 waves x 16: at 3 workgroups per CU, 8 waves spill.
// The first pass of a sort takes its sub-array histogram (and the key span)
// from k_subhist: one read per sort instead of one per pass.
constexpr int kSub = kOnesweepSubs;
constexpr uint32_t kSpinLimit = 1u << 22;  // look-back polls before giving up (seconds)
constexpr int kPollSleep = 1;              // s_sleep between look-back polls (4, 16: no change)
// Look-back rows in flight per round trip.  Wider windows lose: 2 / 4 / 8
// rows +3.8 / +7.3 / +12.8 % per sort (profiles/ab/r02_ab8_uniform.log; a
// tile then sums more rows, 6.7 instead of 5.0 at 4, as the extra loads
// slow every poll).
constexpr int kLookW = 1;
// Status stores write through (sc1): plain stores stay dirty in the
// writer's L2 and a poller on another XCD never sees them (look-back timed
// out).  Keeping every chain on its own XCD (tiles by XCC_ID, no helping)
// made plain stores work but not faster: a poll's round trip is queueing in
// the polling CU's memory pipeline, not the L2 miss
// (profiles/ab/r02_ab15_uniform.log).
constexpr int kStPol = 16;

typedef __attribute__((address_space(1))) uint32_t gu32;
typedef uint32_t v2u __attribute__((ext_vector_type(2)));

// Piece table of a gathered pass (GatherSrc): the last piece e in [e0, e1]
// with gstart[e] <= p (the one holding placed position p), and its record.
__device__ __forceinline__ int gather_piece(const GatherSrc& g, int e0, int e1, int64_t p) {
  int lo = e0, hi = e1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (g.gstart[mid] <= p) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}
// gadj[e] = 2 * (pointer adjustment of piece e) + (1: the piece is in A).
__device__ __forceinline__ int64_t gather_adj(const GatherSrc& g, int e) {
  const int src = e % g.P, b = e / g.P;
  const bool in_a = src == g.me && g.self_in_a;
  return 2 * ((in_a ? g.self_adj[(b & (kBuckets - 1)) >> g.chunk_shift] : 0) - g.place[(int64_t)src * g.nb + b]) +
         (in_a ? 1 : 0);
}
__device__ __forceinline__ const Elem* gather_search(const GatherSrc& g, int e0, int e1, int64_t p) {
  const int64_t v = g.gadj[gather_piece(g, e0, e1, p)];
  return ((v & 1) ? g.A : g.R) + (p + (v >> 1));
}
#ifdef LSB_DEBUG
// A gathered read lies inside A or R (LSB_DASSERT: debug builds only).
__device__ __forceinline__ bool gather_in(const GatherSrc& g, const Elem* p) {
  return (p >= g.A && p < g.A + g.a_len) || (p >= g.R && p < g.R + g.r_len);
}
#endif

// sub_first_tile, sub_of_tile: lsb_device.h

// sub_hist[x * 256 + b] += number of records of sub-array x with digit b;
// SPAN as in k_upsweep.  Workgroup c walks tiles [c*tpw, (c+1)*tpw).
template <int BLOCK, int IPT, bool SPAN>
__global__ __launch_bounds__(BLOCK) void k_subhist(const Elem* __restrict__ A, int64_t m,
                                                   int shift, int64_t tiles_per_wg,
                                                   uint32_t* __restrict__ sub_hist,
                                                   unsigned long long* __restrict__ span) {
  constexpr int W = BLOCK / 64;
  constexpr int T = BLOCK * IPT;
  __shared__ uint32_t hist[W][kBuckets];
  __shared__ uint64_t span_or[W], span_nor[W];
  uint64_t kor = 0, knor = 0;
  for (int i = threadIdx.x; i < W * kBuckets; i += BLOCK) (&hist[0][0])[i] = 0;
  const int w = threadIdx.x >> 6;
  const int64_t TT = (m + T - 1) / T;
  const int64_t t0 = (int64_t)blockIdx.x * tiles_per_wg;
  const int64_t t1 = t0 + tiles_per_wg < TT ? t0 + tiles_per_wg : TT;
  const uint64_t* __restrict__ keys = reinterpret_cast<const uint64_t*>(A);
  int cur = t0 < t1 ? sub_of_tile(t0, TT) : 0;
  __syncthreads();

  auto flush = [&](int x) {
    __syncthreads();
    for (int b = threadIdx.x; b < kBuckets; b += BLOCK) {
      uint32_t s = 0;
#pragma unroll
      for (int ww = 0; ww < W; ++ww) {
        s += hist[ww][b];
        hist[ww][b] = 0;
      }
      if (s) atomicAdd(&sub_hist[x * kBuckets + b], s);
    }
    __syncthreads();
  };

  for (int64_t tile = t0; tile < t1; ++tile) {
    const int x = sub_of_tile(tile, TT);
    if (x != cur) {
      flush(cur);
      cur = x;
    }
    const int64_t tb = tile * T;
    const int64_t end = tb + T < m ? tb + T : m;
    uint64_t k[IPT];
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      const int64_t idx = tb + (int64_t)i * BLOCK + threadIdx.x;
      k[i] = idx < end ? __builtin_nontemporal_load(keys + 2 * idx) : 0ull;  // streaming
    }
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      const int64_t idx = tb + (int64_t)i * BLOCK + threadIdx.x;
      const bool valid = idx < end;
      if (SPAN && valid) {
        kor |= k[i];
        knor |= ~k[i];
      }
      const uint32_t d = (uint32_t)(k[i] >> shift) & (kBuckets - 1);
      const uint32_t d0 = __builtin_amdgcn_readfirstlane(d);
      if (__all(valid && d == d0)) {
        if (lane_id() == 0) atomicAdd(&hist[w][d0], 64u);
      } else if (valid) {
        atomicAdd(&hist[w][d], 1u);
      }
    }
  }
  if (t0 < t1) flush(cur);
  if (SPAN) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      kor |= __shfl_xor(kor, off, 64);
      knor |= __shfl_xor(knor, off, 64);
    }
    if (lane_id() == 0) {
      span_or[w] = kor;
      span_nor[w] = knor;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      uint64_t o = 0, no = 0;
#pragma unroll
      for (int ww = 0; ww < W; ++ww) {
        o |= span_or[ww];
        no |= span_nor[ww];
      }
      atomicOr(&span[0], (unsigned long long)o);
      atomicOr(&span[1], (unsigned long long)no);
    }
  }
}

// k_count16c (launch_count16_chunks, the chunked per-digit exchange): B is
// sorted by the low byte l, so a tile holds one l and one (chunk, sub-array)
// except at the ~256 + 8 C tiles across a boundary.  The tile's high-byte
// counts (per-wave LDS rows) are added to a running row per target -- count16
// of l, chunk_hist of (k, x) -- flushed to global memory when the target
// changes; a tile across a boundary adds record by record to global memory.
// Workgroup c walks tiles [c * tpw, (c + 1) * tpw).
template <int BLOCK, int IPT>
__global__ __launch_bounds__(BLOCK) void k_count16c(const Elem* __restrict__ B, int64_t m, int shift16,
                                                    const uint32_t* __restrict__ lo_hist, int cshift,
                                                    int64_t tiles_per_wg, unsigned long long* __restrict__ count16,
                                                    uint32_t* __restrict__ chunk_hist) {
  constexpr int W = BLOCK / 64;
  constexpr int T = BLOCK * IPT;
  static_assert(BLOCK == kBuckets, "thread t owns high byte t");
  __shared__ uint32_t th[W][kBuckets];
  __shared__ int64_t tot[kBuckets];
  __shared__ int64_t cstart[kMaxExchangeChunks + 1];
  const int t = threadIdx.x, w = t >> 6;
  const int C = kBuckets >> cshift;
  {
    int64_t v = 0;
#pragma unroll
    for (int x = 0; x < kSub; ++x) v += lo_hist[x * kBuckets + t];
    tot[t] = v;
    for (int ww = 0; ww < W; ++ww) th[ww][t] = 0;
  }
  __syncthreads();
  if (t <= C) {
    int64_t a = 0;
    for (int l = 0; l < (t << cshift) && l < kBuckets; ++l) a += tot[l];
    cstart[t] = a;
  }
  __syncthreads();
  const uint64_t* __restrict__ keys = reinterpret_cast<const uint64_t*>(B);
  const int64_t TT = (m + T - 1) / T;
  const int64_t t0 = (int64_t)blockIdx.x * tiles_per_wg;
  const int64_t t1 = t0 + tiles_per_wg < TT ? t0 + tiles_per_wg : TT;
  // (chunk, sub-array) of position p whose low byte is l
  auto target = [&](int64_t p, uint32_t l) -> uint32_t {
    const uint32_t k = l >> cshift;
    const int64_t len = cstart[k + 1] - cstart[k];
    const int64_t TTk = (len + T - 1) / T;
    return k * kSub + (uint32_t)sub_of_tile((p - cstart[k]) / T, TTk);
  };
  uint32_t cur_l = 0xFFFFFFFFu, cur_s = 0xFFFFFFFFu;  // the running rows' targets
  uint32_t acc_l = 0, acc_s = 0;                      // thread t: bin t of each row
  auto flush_l = [&]() {
    if (cur_l != 0xFFFFFFFFu && acc_l) atomicAdd(&count16[((uint32_t)t << 8) | cur_l], (unsigned long long)acc_l);
    acc_l = 0;
  };
  auto flush_s = [&]() {
    if (cur_s != 0xFFFFFFFFu && acc_s) atomicAdd(&chunk_hist[cur_s * kBuckets + t], acc_s);
    acc_s = 0;
  };
  for (int64_t tile = t0; tile < t1; ++tile) {
    const int64_t tb = tile * T;
    const int64_t end = tb + T < m ? tb + T : m;
    const uint32_t lf = (uint32_t)(keys[2 * tb] >> shift16) & 0xFFu;
    const uint32_t ll = (uint32_t)(keys[2 * (end - 1)] >> shift16) & 0xFFu;
    const uint32_t sf = target(tb, lf), sl = target(end - 1, ll);
    const bool uniform = lf == ll && sf == sl;  // the same for the whole workgroup
    uint64_t k[IPT];
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      const int64_t idx = tb + (int64_t)i * BLOCK + t;
      k[i] = idx < end ? __builtin_nontemporal_load(keys + 2 * idx) : 0ull;  // streaming
    }
    if (uniform) {
#pragma unroll
      for (int i = 0; i < IPT; ++i) {
        const int64_t idx = tb + (int64_t)i * BLOCK + t;
        if (idx < end) atomicAdd(&th[w][(uint32_t)(k[i] >> (shift16 + 8)) & 0xFFu], 1u);
      }
      __syncthreads();
      uint32_t v = 0;
#pragma unroll
      for (int ww = 0; ww < W; ++ww) {
        v += th[ww][t];
        th[ww][t] = 0;
      }
      if (lf != cur_l) {
        flush_l();
        cur_l = lf;
      }
      if (sf != cur_s) {
        flush_s();
        cur_s = sf;
      }
      acc_l += v;
      acc_s += v;
      __syncthreads();
    } else {
#pragma unroll
      for (int i = 0; i < IPT; ++i) {
        const int64_t idx = tb + (int64_t)i * BLOCK + t;
        if (idx >= end) continue;
        const uint32_t l = (uint32_t)(k[i] >> shift16) & 0xFFu, h = (uint32_t)(k[i] >> (shift16 + 8)) & 0xFFu;
        atomicAdd(&count16[(h << 8) | l], 1ull);
        atomicAdd(&chunk_hist[target(idx, l) * kBuckets + h], 1u);
      }
    }
  }
  flush_l();
  flush_s();
}

// The regional first pass's sample (launch_sample): workgroup g reads tile
// floor(g * TT / G) of A, 16 records per thread.
constexpr int kSampleBlock = 256;
constexpr int kSampleTiles = 256;
__global__ __launch_bounds__(kSampleBlock) void k_sample(const Elem* __restrict__ A, int64_t m, int shift,
                                                         uint32_t* __restrict__ hist,
                                                         unsigned long long* __restrict__ span) {
  constexpr int IPT = kTile / kSampleBlock;
  __shared__ uint32_t h[kBuckets];
  h[threadIdx.x] = 0;
  __syncthreads();
  const int64_t TT = (m + kTile - 1) / kTile;
  const int64_t tb = (int64_t)blockIdx.x * TT / gridDim.x * kTile;
  const uint64_t* __restrict__ keys = reinterpret_cast<const uint64_t*>(A);
  uint64_t kor = 0, knor = 0;
#pragma unroll
  for (int i = 0; i < IPT; ++i) {
    const int64_t idx = tb + (int64_t)i * kSampleBlock + threadIdx.x;
    if (idx < m) {
      const uint64_t k = __builtin_nontemporal_load(keys + 2 * idx);
      kor |= k;
      knor |= ~k;
      atomicAdd(&h[(uint32_t)(k >> shift) & (kBuckets - 1)], 1u);
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    kor |= __shfl_xor(kor, off, 64);
    knor |= __shfl_xor(knor, off, 64);
  }
  if (lane_id() == 0) {
    atomicOr(&span[0], (unsigned long long)kor);
    atomicOr(&span[1], (unsigned long long)knor);
  }
  __syncthreads();
  if (h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], h[threadIdx.x]);
}

// Phase timing (profiling build, -DLSB_OS_PROFILE): thread 0 of every
// workgroup adds s_memtime deltas between the barriers of a tile into
// g_os_prof[phase]; the runtime prints them at lsb_destroy.
#ifdef LSB_OS_PROFILE
__device__ unsigned long long g_os_prof[10];
#define OS_MARK(k)                                                       \
  do {                                                                   \
    if (t == 0) {                                                        \
      const uint64_t now = __builtin_amdgcn_s_memtime();                 \
      prof[k] += now - prof_last;                                        \
      prof_last = now;                                                   \
    }                                                                    \
  } while (0)
#else
#define OS_MARK(k) ((void)0)
#endif

//
// For the per-digit exchange forms (P > 1) a pass also hands the exchange its
// counts: `totals` (workgroup 0 writes the 256 digit totals), and with C16
// (the high byte of a 16-bit exchange digit) the 65536 counts of the 16-bit
// digit at shift16 = shift - 8.  The input is then sorted by that low byte,
// so a tile whose first and last records share it has one low byte
// throughout, and its bucket-b run adds cnt_b to count16[b][lo]; thread b
// keeps a running count per (b, lo) in registers and adds it to memory when
// its tile's low byte changes (a workgroup's tiles are taken in order, so
// that is a few times per launch).  A tile across a low-byte boundary adds
// its counts in the write-out instead: each wave-instruction's run of equal
// (digit, low byte) slots adds once, from its head lane (run-length atomics,
// so a hot key's run costs one add per instruction, not one per record).
//
// HALVES = 2 (skewed keys, chosen per sort by the runtime): the ranked tile
// is staged and written in two halves of the tile's output order, so the
// stage is 32 KiB and 3 workgroups fit a CU instead of 2.  The records stay
// in registers until their half is staged.  Zipf keys sort 5.7 % faster
// this way (their serialised next-digit adds hide behind a third
// workgroup); uniform keys 4.7 % slower (two more barriers per tile, half-
// length write phases): profiles/ab/r02_ab12_*.
//
// Neighbours each way a SEG walk loads together before walking on (LSB_SEG_WIN;
// 0: the plain one-read-at-a-time walk).
#ifndef LSB_SEG_WIN
#define LSB_SEG_WIN 2
#endif
constexpr int kSegWin = LSB_SEG_WIN;
// The SEG instance's stage neighbours from LDS instead of DPP (experiment).
#ifndef LSB_SEG_LDSNB
#define LSB_SEG_LDSNB 0
#endif
// The SEG instance's whole tiles through the batched write-out (records, then
// their delta entries, read LSB_SEG_BATCH at a time first; 0: one by one).
#ifndef LSB_SEG_BATCH
#define LSB_SEG_BATCH 4
#endif
// GATHER: one lane loads the descriptor LSB_GATHER_PF tiles ahead in the
// sub-array into L2, so wave 0's descriptor fetch for the workgroup that
// takes that tile finds it there (0: none).  Wave 0 fetches the next tile's
// descriptor after its write-out, so the loop top's wait for it also waits
// for its stores (vmcnt(0)); from L2 that wait is shorter: gathered pass
// 7.63-7.67 -> 7.45-7.48 ms at 2^30 (profiles/r06/gather/).
#ifndef LSB_GATHER_PF
#define LSB_GATHER_PF 64
#endif

// SEG (the hybrid's last pass, SegPass in lsb_kernels.h): the write-out also
// orders each segment (records equal on seg.pmask; inside the tile they are
// adjacent in the stage, in one bucket run) by the whole key: a record's slot
// in its run is its segment's first slot + #(segment keys < mine) + #(equal
// keys staged before me).  Segments hold ~0.25 records on average at the
// runtime's choice of bytes, so a record first compares its two stage
// neighbours, which are its neighbouring lanes (DPP), and walks the stage in
// LDS only when one of them shares its segment.  Segments split between
// tiles are merged afterwards by launch_segfix, from this pass's input and
// look-back rows and the bucket bases workgroup 0 writes to seg.base: the
// pass records nothing per tile (crossing-run lists appended here cost it
// ~1 ms at 2^30, profiles/r03_ab_seg.log).
//
// GATHER (the pass after a per-digit exchange, LSB_OPT_EXCHANGE_GATHER): the
// tile's records are read where the exchange left them (GatherSrc: the
// receive buffer, and the rank's own segment in A) instead of from a placed
// copy.  Wave 0 fetches the next tile's TileDesc while this tile is written,
// so the loads at the loop top wait on nothing new; a tile of more than
// kDescPieces pieces searches the piece table per record.
//
// RG (the regional first pass, RegionPass in lsb_kernels.h): RG = 1 is a
// sort's first pass without a histogram: bucket b's run of a tile of
// sub-array x starts at region (b, x)'s first slot plus the look-back sum,
// and the next digit is counted over the regional layout's tiles.  RG = 2
// reads that layout: tile t takes the valid prefix of its region's slots.
template <int BLOCK, int IPT, bool NEXT, bool C16, int HALVES, bool SEG, bool GATHER, int RG>
__device__ __forceinline__ void onesweep_body(
    const Elem* __restrict__ in, Elem* __restrict__ out, int64_t m, int shift, int next_shift,
    const uint32_t* __restrict__ sub_hist, uint32_t* __restrict__ next_hist,
    uint32_t* __restrict__ status, uint32_t* __restrict__ tile_ctr, uint32_t epoch,
    uint32_t* __restrict__ err, uint64_t* __restrict__ totals,
    unsigned long long* __restrict__ count16, SegPass seg, GatherSrc gs, RegionPass rg) {
  constexpr int W = BLOCK / 64;
  constexpr int T = BLOCK * IPT;
  static_assert(!SEG || (!NEXT && !C16 && HALVES == 1), "the segment pass: last pass, whole stage");
  static_assert(RG == 0 || (!C16 && HALVES == 1 && !SEG && !GATHER), "regional passes: plain whole stage");
  static_assert(RG != 1 || NEXT, "the regional first pass counts the next digit");
  // Thread t < 256 owns bucket t (counts, scan, look-back, offsets); with
  // BLOCK = 512 the other threads only load, rank, stage and write.
  static_assert(BLOCK % kBuckets == 0, "bucket threads");
  // Per-wave digit counters -> tile positions (< 4096): 16-bit at 8 waves,
  // so the counters of two workgroups still fit a CU beside their stages.
  using WC = typename std::conditional<(W > 4), uint16_t, uint32_t>::type;

  constexpr int HT = T / HALVES;                // staged records per half
  __shared__ Elem stage[HT];                    // the ranked tile (64 KiB, or one half)
  __shared__ WC wcnt[W][kBuckets];              // per-wave digit counters -> positions
  __shared__ int64_t delta[kBuckets];           // global dest = delta[digit] + tile position
  __shared__ uint32_t cut[NEXT ? kBuckets : 1];  // next-pass sub-array of a run: see below
  __shared__ uint32_t nh[NEXT ? kSub * kBuckets : 1];  // next digit's sub-array histogram
  __shared__ uint64_t scan64[W];
  __shared__ uint32_t scan32[W];
  __shared__ int32_t s_tile, s_sub;
  __shared__ uint32_t tile_lo[2];  // C16: low byte of the tile's first, last record
  __shared__ TileDesc s_desc;      // GATHER: where this tile's records are

  const int t = threadIdx.x;
  const bool bkt = BLOCK == kBuckets || t < kBuckets;  // a bucket thread
  const int w = t >> 6;
  const uint32_t lane = lane_id();
  // Tiles of this pass's input (TT) and of the next pass's (TTn: its
  // sub-arrays are what the next digit is counted by); output slots (mcap).
  const int64_t TT = RG == 2 ? rg.cap / T * kRegions : (m + T - 1) / T;
  const int64_t TTn = RG == 1 ? rg.cap / T * kRegions : (m + T - 1) / T;
  const int64_t mcap = RG == 1 ? region_stride(rg.cap) * kRegions : m;
  uint32_t racc = 0;                     // RG = 1: thread t's count of region (t, cur_sub)
  // Granule tags (bits 30-31): this launch's parity, and the prefix bit.
  constexpr uint32_t kValMask = kStatusValMask, kPreBit = 1u << 30;
  const uint32_t tag_agg = (epoch & 1u) << 31, tag_pre = tag_agg | kPreBit;
  const int shift16 = shift - 8;
  uint32_t acc_lo = 0xFFFFFFFFu;  // C16: thread t's running count of digit (t, acc_lo)
  uint64_t acc = 0;
  auto c16_flush = [&]() {
    if (acc) atomicAdd(count16 + (((uint32_t)t << 8) | acc_lo), (unsigned long long)acc);
    acc = 0;
  };

  // Bucket starts (exclusive scan of the digit totals) and this thread's
  // bucket column of the sub-array histogram.
  // (The split-stage form re-reads the column when it changes sub-array,
  // a few times per launch: its records need the registers.)
  uint32_t col[HALVES == 1 ? kSub : 1];
  uint64_t tot = 0;
#pragma unroll
  for (int x = 0; x < kSub; ++x) {
    const uint32_t v = bkt && RG != 1 ? sub_hist[x * kBuckets + t] : 0u;
    if (HALVES == 1) col[x] = v;
    tot += v;
  }
  uint64_t all;
  const uint64_t bstart = block_exclusive_scan<BLOCK>(tot, scan64, &all);
  if (totals != nullptr && blockIdx.x == 0 && bkt) totals[t] = tot;
  if (SEG && blockIdx.x == 0 && bkt) {  // k_segfix's bucket bases per sub-array
    uint64_t pre = bstart;
#pragma unroll
    for (int x = 0; x < kSub; ++x) {
      seg.base[x * kBuckets + t] = (int64_t)pre;
      pre += col[x];
    }
  }
  // Skewed digit (one bucket holds more than 1/32 of the records, e.g. Zipf
  // keys): runs of equal next digits are then long, and 64 lanes adding to
  // one LDS counter serialise.  Such launches add once per run of equal
  // slots within a wave-instruction; uniform keys keep the plain add (a
  // per-instruction check costs them 5.7 %, tools/ab.sh).  Launch-uniform.
  const bool skewed = NEXT && __syncthreads_or(tot > (uint64_t)(m >> 5)) != 0;
  if (NEXT)
    for (int i = t; i < kSub * kBuckets; i += BLOCK) nh[i] = 0;

#ifdef LSB_OS_PROFILE
  uint64_t prof[10] = {};  // phases 0-6; 7: rows summed in look-backs, 8: tiles
  uint64_t prof_last = __builtin_amdgcn_s_memtime();
#endif
  int sub = (int)(blockIdx.x % kSub);  // thread 0's dequeue cursor
  int tries = 0;
  int cur_sub = -1;
  uint64_t base = 0;  // bstart + sub_pre[cur_sub][t]
  // Thread 0: the next tile of sub-array `sub` in order, else of the next
  // sub-array (-1 when all are taken).
  auto grab = [&](int& tile_out, int& sub_out) {
    int tile = -1;
    while (tries < kSub) {
      const int64_t f0 = sub_first_tile(sub, TT), f1 = sub_first_tile(sub + 1, TT);
      if (f1 > f0) {
        const uint32_t jj = atomicAdd(&tile_ctr[sub], 1u);
        if ((int64_t)jj < f1 - f0) {
          tile = (int)(f0 + jj);
          break;
        }
      }
      sub = sub + 1 == kSub ? 0 : sub + 1;
      ++tries;
    }
    tile_out = tile;
    sub_out = sub;
  };
  // The next tile's id is fetched while this tile's records are written
  // (a device-scope atomic is ~1 us under load; 3 % of the sort, measured).
  int nxt_tile = -1, nxt_sub = 0;
  // RG = 2: thread 0 also reads the next tile's region count (tile k of
  // region r holds that region's slots [k * T, (k + 1) * T)) while this tile
  // is written, so the loads at the loop top wait on nothing new.
  // The count is only consumed at the loop top, so the load's latency hides
  // behind this tile's write-out (computing the valid count right away made
  // wave 0, and with it the workgroup's closing barrier, wait for it).
  if (t == 0) grab(nxt_tile, nxt_sub);
  // GATHER: lanes 0-3 of wave 0 hold the next tile's descriptor.
  uint4 dreg = make_uint4(0u, 0u, 0u, 0u);
  auto fetch_desc = [&]() {
    if (GATHER && w == 0) {
      const int nt = __builtin_amdgcn_readfirstlane(nxt_tile);
      if (nt >= 0 && lane < 4) dreg = reinterpret_cast<const uint4*>(gs.desc + nt)[lane];
    }
  };
  fetch_desc();

  for (;;) {
    if (t == 0) {
      s_tile = nxt_tile;
      s_sub = nxt_sub;
    }
    if (GATHER && w == 0 && lane < 4) {
      // The lane's slot recomputed here, opaque to the compiler: hoisted out
      // of the loop, it was spilled, and the spill's reload from scratch is
      // one more memory round trip before this barrier.
      uint32_t l;
      asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0" : "=v"(l));
      *reinterpret_cast<uint4*>(reinterpret_cast<char*>(&s_desc) + l * 16u) = dreg;
    }
#pragma unroll
    for (int j = 0; j < kBuckets / 64; ++j) wcnt[w][lane + 64 * j] = 0;
    __syncthreads();
    OS_MARK(0);  // dequeue
    const int tile = s_tile;
    if (tile < 0) break;
    const int x = s_sub;
    if (x != cur_sub) {
      if (RG == 1) {
        if (bkt && cur_sub >= 0 && racc) atomicAdd(&rg.counts[t * kSub + cur_sub], racc);
        racc = 0;
        base = (uint64_t)region_base((bkt ? t : 0) * kSub + x, rg.cap);  // region (t, x)
      } else {
        uint64_t pre = 0;
#pragma unroll
        for (int xx = 0; xx < kSub; ++xx)
          pre += xx < x ? (HALVES == 1 ? col[xx] : (bkt ? sub_hist[xx * kBuckets + t] : 0u)) : 0u;
        base = bstart + pre;
      }
      cur_sub = x;
    }
    int64_t tb = (int64_t)tile * T;
    int nvalid = (int)((m - tb) < T ? (m - tb) : T);
    uint32_t rg_reg = 0, rg_k = 0;
    if (RG == 2) {
      // Tile k of region r: that region's slots [k * T, (k + 1) * T), all
      // inside the buffer, so the record loads need no count: the count is
      // loaded after them (below).  (Thread 0 fetching it with the next
      // tile's id made the loop top wait for wave 0's write-out stores as
      // well, vmcnt(0); loaded before the records, it held back half of
      // their loads.)
      const uint32_t tu = (uint32_t)__builtin_amdgcn_readfirstlane(tile);
      const uint32_t ct = (uint32_t)(rg.cap / T);
      rg_reg = tu / ct;
      rg_k = tu - rg_reg * ct;
      tb = region_base(rg_reg, rg.cap) + (int64_t)rg_k * T;
    }

    Elem e[IPT];
    const int wbase = w * 64 * IPT + (int)lane;
    if (GATHER) {
      const int dn = __builtin_amdgcn_readfirstlane(s_desc.n);
      if (dn != kDescOverflow) {
        // The pieces' base pointers and first tile positions are uniform
        // (scalar registers); a record picks its piece by compares.
        const uint32_t sel = (uint32_t)__builtin_amdgcn_readfirstlane(s_desc.sel);
        const Elem* pb[kDescPieces];
        int st[kDescPieces];
#pragma unroll
        for (int k = 0; k < kDescPieces; ++k) {
          st[k] = __builtin_amdgcn_readfirstlane(s_desc.start[k]);
          const uint64_t a = s_desc.adj[k];
          const int64_t adj = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(a >> 32)) << 32) |
                                        (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a));
          pb[k] = ((sel >> k) & 1u ? gs.A : gs.R) + (tb + adj);
        }
        // A wave's load i covers tile positions [g0, g0 + 64): when one piece
        // holds them all (every load but the <= 3 that straddle a piece
        // start), its base is picked by scalar compares, not per lane
        // (forced 16-bit exchange: -0.3 % uniform, -0.7 % Zipf per sort,
        // profiles/r04/ab_gu/).
        const int wu = __builtin_amdgcn_readfirstlane(w);
#pragma unroll
        for (int i = 0; i < IPT; ++i) {
          const int li = wbase + i * 64;
          const int g0 = wu * 64 * IPT + i * 64;
          int ka = 0, kb = 0;
#pragma unroll
          for (int k = 1; k < kDescPieces; ++k) {
            ka += g0 >= st[k] ? 1 : 0;
            kb += g0 + 63 >= st[k] ? 1 : 0;
          }
          const Elem* src = pb[0];
          if (ka == kb) {
#pragma unroll
            for (int k = 1; k < kDescPieces; ++k) src = ka >= k ? pb[k] : src;
          } else {
#pragma unroll
            for (int k = 1; k < kDescPieces; ++k) src = li >= st[k] ? pb[k] : src;
          }
          LSB_DASSERT(li >= nvalid || gather_in(gs, src + li));
          e[i] = li < nvalid ? load_elem_nt(src + li) : Elem{0ull, 0ull};
        }
      } else {
        // One record's search at a time (the scheduling barrier keeps the
        // compiler from interleaving 8 searches, which would spill).
        const int e0 = s_desc.e0, e1 = s_desc.e1;
#pragma unroll
        for (int i = 0; i < IPT; ++i) {
          const int li = wbase + i * 64;
          LSB_DASSERT(li >= nvalid || gather_in(gs, gather_search(gs, e0, e1, tb + li)));
          e[i] = li < nvalid ? load_elem_nt(gather_search(gs, e0, e1, tb + li)) : Elem{0ull, 0ull};
          __builtin_amdgcn_sched_barrier(0);
        }
      }
#if LSB_GATHER_PF
      // Bring the descriptor of the tile LSB_GATHER_PF ahead in this
      // sub-array into L2 (this XCD's workgroups take its tiles in order).
      if (w == 1 && lane == 0) {
        const int pf = tile + LSB_GATHER_PF;
        if (pf < sub_first_tile(x + 1, TT))
          (void)__hip_atomic_load(const_cast<int32_t*>(&gs.desc[pf].n), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
#endif
    } else {
#pragma unroll
      for (int i = 0; i < IPT; ++i) {
        const int li = wbase + i * 64;
        e[i] = RG == 2 || li < nvalid ? load_elem_nt(in + tb + li) : Elem{0ull, 0ull};
      }
      if (RG == 2) {
        __builtin_amdgcn_sched_barrier(0);
        const int64_t v = (int64_t)rg.counts[rg_reg] - (int64_t)rg_k * T;
        nvalid = (int)(v < 0 ? 0 : (v < T ? v : T));
      }
    }
#ifdef LSB_OS_PROFILE
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    OS_MARK(6);  // tile loads in flight
#endif
    // Status rows of this sub-array through one buffer descriptor (byte
    // offsets < 2^31); the even lane of a pair publishes and polls buckets
    // t, t + 1 as one 8-byte sc1 access: two self-tagged 4-byte halves,
    // written by one store, so a pair is consumed only when both tags agree.
    const int64_t first = sub_first_tile(x, TT);
    const int64_t last = sub_first_tile(x + 1, TT);
    const bool head = tile == first;
    const bool even = (lane & 1u) == 0;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        status + first * kBuckets, 0, (int)((last - first) * kBuckets * 4), 0x00020000);
    constexpr uint32_t kRowBytes = kBuckets * 4;
    const uint32_t my_off = (uint32_t)(tile - first) * kRowBytes + (uint32_t)t * 4u;
    uint32_t prow = (uint32_t)(tile - first) - 1u;  // newest predecessor row not yet summed
    // Look-back window: rows prow, prow - 1, ... in flight together.  Rows
    // before the sub-array's first read as 0 (buffer range check) and are
    // never consumed: the first row always carries its prefix.
    v2u g[kLookW];
    auto load_window = [&]() {
#pragma unroll
      for (int r = 0; r < kLookW; ++r)
        g[r] = __builtin_amdgcn_raw_buffer_load_b64(rs, (prow - (uint32_t)r) * kRowBytes + (uint32_t)t * 4u, 0, 16);
    };
    uint32_t cnt = 0, lstart;
    // Stable rank of every element among the wave's elements of its digit
    // (per-wave counters), then the tile's counts: publish the aggregate,
    // put the first look-back window in flight, and scan and stage the tile
    // in LDS (neither needs the global offset) while it travels.
    uint32_t rk[IPT];
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      const bool valid = wbase + i * 64 < nvalid;
      const uint32_t d = (uint32_t)(e[i].key >> shift) & (kBuckets - 1);
      const uint64_t mt = match_digit8(d, __ballot(valid));
      const uint32_t below = mbcnt(mt);
      const uint32_t pre = wcnt[w][d];
      rk[i] = pre + below;
      if (valid && below == 0) wcnt[w][d] = (WC)(pre + (uint32_t)__popcll(mt));
      if (C16) {
        const int li = wbase + i * 64;
        if (li == 0) tile_lo[0] = (uint32_t)(e[i].key >> shift16) & 0xFFu;
        if (li == nvalid - 1) tile_lo[1] = (uint32_t)(e[i].key >> shift16) & 0xFFu;
      }
    }
    __syncthreads();
    OS_MARK(1);  // load + rank
    if (bkt) {
#pragma unroll
      for (int ww = 0; ww < W; ++ww) {
        const uint32_t v = wcnt[ww][t];
        wcnt[ww][t] = (WC)cnt;
        cnt += v;
      }
      if (RG == 1) racc += cnt;
    }
    bool mixed16 = false;
    if (C16) {
      const uint32_t l0 = tile_lo[0];
      mixed16 = l0 != tile_lo[1];
      if (!mixed16 && cnt > 0) {
        if (l0 != acc_lo) {
          c16_flush();
          acc_lo = l0;
        }
        acc += cnt;
      }
    }
    const uint32_t cnt_b = pair_swap(cnt);  // even lanes: lane t + 1's count
    if (even && bkt) {
      const uint32_t tg = head ? tag_pre : tag_agg;
      __builtin_amdgcn_raw_buffer_store_b64(v2u{cnt | tg, cnt_b | tg}, rs, my_off, 0, kStPol);
      if (!head) load_window();
    }
    {
      uint32_t tile_total;
      lstart = block_exclusive_scan<BLOCK>(cnt, scan32, &tile_total);
      if (bkt) {
#pragma unroll
        for (int ww = 0; ww < W; ++ww) wcnt[ww][t] = (WC)(wcnt[ww][t] + lstart);
      }
    }
    __syncthreads();
    OS_MARK(2);  // publish + scan
    // Split stage: half 0 turns rk[i] into the record's tile position and
    // the later half reuses it.
    auto stage_half = [&](int h) {
#pragma unroll
      for (int i = 0; i < IPT; ++i) {
        if (wbase + i * 64 < nvalid) {
          const uint32_t d = (uint32_t)(e[i].key >> shift) & (kBuckets - 1);
          if (HALVES == 1) {
            stage[wcnt[w][d] + rk[i]] = e[i];
          } else {
            if (h == 0) rk[i] += wcnt[w][d];
            if ((int)(rk[i] / HT) == h) stage[rk[i] - h * HT] = e[i];
          }
        }
      }
    };
    stage_half(0);

    OS_MARK(3);  // stage
    uint32_t ea = 0, eb = 0;
    if (even && bkt && !head) {
      uint32_t spins = 0;
      for (;;) {
        // Rows in order, while they are ready: both halves of this launch
        // (parity) and of one kind (prefix bit); stop at a prefix.
        uint32_t used = 0;
        bool done = false;
#pragma unroll
        for (int r = 0; r < kLookW; ++r) {
          if (done || used != (uint32_t)r) continue;
          if (((g[r].x ^ g[r].y) >> 30) == 0 && (g[r].x & ~kValMask & ~kPreBit) == tag_agg) {
            ea += g[r].x & kValMask;
            eb += g[r].y & kValMask;
            ++used;
            done = (g[r].x & kPreBit) != 0;
          }
        }
#ifdef LSB_OS_PROFILE
        if (t == 0) prof[7] += used;
#endif
        if (done) break;
        if (used == 0) {
          __builtin_amdgcn_s_sleep(kPollSleep);
          if ((++spins & 1023u) == 0 &&
              (spins > kSpinLimit ||
               __hip_atomic_load((gu32*)err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0)) {
            atomicOr(err, 1u);
            break;
          }
        }
        prow -= used;
        load_window();
      }
      __builtin_amdgcn_raw_buffer_store_b64(v2u{(ea + cnt) | tag_pre, (eb + cnt_b) | tag_pre}, rs,
                                            my_off, 0, kStPol);
    }
    const uint32_t eb_left = pair_swap(eb);  // odd lanes: lane t - 1's sum
    const uint64_t excl = even ? ea : eb_left;
    int64_t R = (int64_t)(base + excl);  // first output slot of the run
    if (RG == 1 && bkt && excl + cnt > (uint64_t)rg.cap) {
      // Region (t, x) overflows: the output is invalid (the runtime redoes
      // the sort from the kept input); keep the run inside the buffer.
      atomicOr(rg.ovf, 1u);
      R = R < mcap - (int64_t)cnt ? R : mcap - (int64_t)cnt;
    }
    if (bkt) delta[t] = R - (int64_t)lstart;
    if (NEXT && bkt) {
      // The run [R, R + cnt) lies in next-pass sub-array x0, except from
      // stage position jb on (x1) when it crosses a sub-array boundary (at
      // most one: a non-empty sub-array holds >= kTile records).
      uint32_t c = 0xFFFFu;  // jb = 0xFFFF: never
      if (RG == 1) {
        // Region (t, x) lies in the next pass's sub-array t / 32 (its
        // sub-arrays are 256 whole regions): no run crosses one.
        c = 0xFFFFu | ((uint32_t)(t >> 5) << 16) | ((uint32_t)(t >> 5) << 24);
      } else if (cnt > 0) {
        const int x0 = sub_of_tile(R / T, TTn);
        const int64_t bnd = x0 + 1 < kSub ? sub_first_tile(x0 + 1, TTn) * T : mcap;
        if (R + cnt > bnd) {
          const int x1 = sub_of_tile(bnd / T, TTn);
          c = (uint32_t)(lstart + (bnd - R)) | ((uint32_t)x0 << 16) | ((uint32_t)x1 << 24);
        } else {
          c = 0xFFFFu | ((uint32_t)x0 << 16) | ((uint32_t)x0 << 24);
        }
      }
      cut[t] = c;
    }
    __syncthreads();
    OS_MARK(5);  // look-back (+ run cuts, barrier)
#ifdef LSB_OS_PROFILE
    if (t == 0) ++prof[8];
#endif
    if (t == 0) {  // in flight during the writes
      grab(nxt_tile, nxt_sub);
    }

    // emit: one staged record (tile position j, output slot delta + pos) to
    // memory, and its next digit to the sub-array histogram.
    // g = delta[digit] + the record's slot in its run, c = cut[digit].
    auto emit = [&](auto skew_tag, const Elem& v, int j, int64_t g, uint32_t c) {
      constexpr bool kSkew = decltype(skew_tag)::value;
      LSB_DASSERT(g >= 0 && g < mcap);
      // In range by construction.  The clamp keeps a look-back that gave up
      // (err set, output reported invalid) from storing outside `out`; a
      // clamp, not a branch: the conditional store cost 6 % of the sort.
      const uint64_t gs = (uint64_t)g < (uint64_t)(mcap - 1) ? (uint64_t)g : (uint64_t)(mcap - 1);
      store_elem(out + gs, v);
      if (NEXT) {
        const uint32_t xs = (uint32_t)j >= (c & 0xFFFFu) ? (c >> 24) : ((c >> 16) & 0xFFu);
        const uint32_t dn = (uint32_t)(v.key >> next_shift) & (kBuckets - 1);
        const uint32_t slot = xs * kBuckets + dn;
        if (kSkew) {
          // One add per run of equal slots within the wave-instruction: the
          // head lane of each run adds the run's length.  Hot keys come in
          // long runs in the staged (bucket-ordered) tile, so the 64-way
          // same-address LDS atomics that serialise become one or two adds.
          // Active lanes are a prefix (j < nvalid), so a run ends at the
          // next head or at the active count.
          // The previous lane's slot by DPP wave_shr:1 (lane 0 keeps ~slot,
          // so it is always a head); __shfl_up is a ds_bpermute round trip
          // (-1.5 % Zipf, uniform unchanged: profiles/ab/r02_ab7_*).
          const uint64_t act = __ballot(1);
          const uint32_t prev =
              (uint32_t)__builtin_amdgcn_update_dpp((int)~slot, (int)slot, 0x138, 0xf, 0xf, false);
          const bool head = prev != slot;
          const uint64_t heads = __ballot(head);
          if (head) {
            const uint64_t above = heads & ~((2ull << lane) - 1ull);
            const uint32_t end = above ? (uint32_t)__builtin_ctzll(above) : (uint32_t)__popcll(act);
            atomicAdd(&nh[slot], end - lane);
          }
        } else {
          atomicAdd(&nh[slot], 1u);
        }
      }
    };
    // The write-out is instantiated twice (the launch-uniform `skewed` picks
    // one outside it): a per-record branch on it cost uniform keys 2.4 %.
    // SEG: record v's slot in its tile stage (pos = j unless a stage
    // neighbour shares its segment): its segment's first stage slot +
    // #(segment keys < v) + #(equal keys staged before v).  Lanes of a wave
    // hold consecutive j, so the neighbours are the next lanes (DPP).
    auto seg_pos = [&](const Elem& v, int j, int jend) -> int {
      int pos = j;
#if LSB_SEG_LDSNB
      // Stage neighbours j - 1 and j + 1 read from LDS by every lane (two
      // independent reads; no DPP, no edge-lane branches).
      const uint64_t pv = j > 0 ? stage[j - 1].key : ~v.key;
      const uint64_t nx = j + 1 < nvalid ? stage[j + 1].key : ~v.key;
#else
      // Stage neighbours j - 1 and j + 1 are the neighbouring lanes'
      // records (the wave's j are consecutive; lanes 0 and 63 read LDS).
      const uint32_t kl = (uint32_t)v.key, kh = (uint32_t)(v.key >> 32);
      uint64_t pv = ((uint64_t)(uint32_t)__builtin_amdgcn_update_dpp(0, (int)kh, 0x138, 0xf, 0xf, false) << 32) |
                    (uint32_t)__builtin_amdgcn_update_dpp(0, (int)kl, 0x138, 0xf, 0xf, false);
      uint64_t nx = ((uint64_t)(uint32_t)__builtin_amdgcn_update_dpp(0, (int)kh, 0x130, 0xf, 0xf, false) << 32) |
                    (uint32_t)__builtin_amdgcn_update_dpp(0, (int)kl, 0x130, 0xf, 0xf, false);
      if (lane == 0 && j > 0) pv = stage[j - 1].key;
      if ((lane == 63 || j + 1 == jend) && j + 1 < nvalid) nx = stage[j + 1].key;
#endif
      const uint64_t pk = v.key & seg.pmask;
      const bool sp = j > 0 && (pv & seg.pmask) == pk;
      const bool sn = j + 1 < nvalid && (nx & seg.pmask) == pk;
      if (sp || sn) {
        // Walk the segment in LDS (bounded: kSegMax each way).  The first
        // kSegWin neighbours each way are loaded together (independent
        // LDS reads; segments hold ~2 records at the runtime's bytes), and
        // the walk goes on one read at a time only past them.  Out of
        // range, a neighbour reads as ~v.key, outside the segment.
        uint32_t less = 0, eqb = 0;
        const int klo = j - kSegMax > 0 ? j - kSegMax : 0;
        const int khi = j + 1 + kSegMax < nvalid ? j + 1 + kSegMax : nvalid;
        uint64_t wb[kSegWin > 0 ? kSegWin : 1], wf[kSegWin > 0 ? kSegWin : 1];
#pragma unroll
        for (int q = 0; q < kSegWin; ++q) {
          // (the first of each: pv / nx, already read)
          wb[q] = q == 0 && j - 1 >= klo ? pv : j - 1 - q >= klo ? stage[j - 1 - q].key : ~v.key;
          wf[q] = q == 0 && j + 1 < khi ? nx : j + 1 + q < khi ? stage[j + 1 + q].key : ~v.key;
        }
        int k = j - 1;
        bool on = true;
#pragma unroll
        for (int q = 0; q < kSegWin; ++q) {
          on = on && (wb[q] & seg.pmask) == pk;
          if (on) {
            less += wb[q] < v.key ? 1u : 0u;
            eqb += wb[q] == v.key ? 1u : 0u;
            --k;
          }
        }
        while (on && k >= klo) {
          const uint64_t kk = stage[k].key;
          if ((kk & seg.pmask) != pk) break;
          less += kk < v.key ? 1u : 0u;
          eqb += kk == v.key ? 1u : 0u;
          --k;
        }
        const int sfirst = k + 1;  // the segment's first stage slot
        // kSegMax records walked without leaving the segment: too long
        bool too_long = k < klo && klo > 0;
        k = j + 1;
        on = true;
#pragma unroll
        for (int q = 0; q < kSegWin; ++q) {
          on = on && (wf[q] & seg.pmask) == pk;
          if (on) {
            less += wf[q] < v.key ? 1u : 0u;
            ++k;
          }
        }
        while (on && k < khi) {
          const uint64_t kk = stage[k].key;
          if ((kk & seg.pmask) != pk) break;
          less += kk < v.key ? 1u : 0u;
          ++k;
        }
        too_long |= k == khi && khi < nvalid;
        // 2: this tile's slots may collide (not a permutation, SegPass).
        if (too_long) atomicOr(seg.err, 2u);
        pos = sfirst + (int)(less + eqb);
      }
      return pos;
    };
    auto write_out = [&](auto skew_tag, int h) {
      const int jend = HALVES == 1 || (h + 1) * HT >= nvalid ? nvalid : (h + 1) * HT;
      // A whole tile: every thread's T / BLOCK records read from the stage
      // together, then their delta and cut entries, so the LDS round trips
      // overlap instead of serialising twice per record (-0.6...-0.9 % per
      // sort, profiles/r04/ab_wo/).  Only the LSD passes' whole-stage
      // instances: the exchange's and the split stage's would spill.
      if ((!SEG || LSB_SEG_BATCH) && HALVES == 1 && !C16 && !GATHER && jend == HT) {
        // G records per batch (the SEG instance: LSB_SEG_BATCH at a time, so
        // its walk registers fit beside them).
        constexpr int G = SEG && LSB_SEG_BATCH > 0 && LSB_SEG_BATCH < HT / BLOCK ? LSB_SEG_BATCH : HT / BLOCK;
#pragma unroll
        for (int k0 = 0; k0 < HT / BLOCK; k0 += G) {
          Elem v[G];
          int64_t dl[G];
          uint32_t ct[G];
#pragma unroll
          for (int k = 0; k < G; ++k) v[k] = stage[(k0 + k) * BLOCK + t];
#pragma unroll
          for (int k = 0; k < G; ++k) {
            const uint32_t d = (uint32_t)(v[k].key >> shift) & (kBuckets - 1);
            dl[k] = delta[d];
            ct[k] = NEXT ? cut[d] : 0u;
          }
#pragma unroll
          for (int k = 0; k < G; ++k) {
            const int j = (k0 + k) * BLOCK + t;
            emit(skew_tag, v[k], j, dl[k] + (SEG ? seg_pos(v[k], j, jend) : j), ct[k]);
          }
        }
        return;
      }
      for (int j = h * HT + t; j < jend; j += BLOCK) {
        const Elem v = stage[j - h * HT];
        int pos = j;
        if (SEG) pos = seg_pos(v, j, jend);
        const uint32_t d = (uint32_t)(v.key >> shift) & (kBuckets - 1);
        emit(skew_tag, v, j, delta[d] + pos, NEXT ? cut[d] : 0u);
        if (C16 && mixed16) {
          // The tile crosses a low-byte boundary: its 16-bit digit counts by
          // runs of equal (digit, low byte) slots within each wave-instruction
          // (the stage is in that order), one add per run by its head lane,
          // instead of thread t walking its whole bucket run alone (a hot
          // key's run kept its workgroup, and the tile it had already
          // reserved, for the length of the walk).  Active lanes are a
          // prefix, as in emit's skewed count.
          const uint32_t s16 = (d << 8) | ((uint32_t)(v.key >> shift16) & 0xFFu);
          const uint64_t act = __ballot(1);
          const uint32_t prev = (uint32_t)__builtin_amdgcn_update_dpp((int)~s16, (int)s16, 0x138, 0xf, 0xf, false);
          const bool head = prev != s16;
          const uint64_t heads = __ballot(head);
          if (head) {
            const uint64_t above = heads & ~((2ull << lane) - 1ull);
            const uint32_t end = above ? (uint32_t)__builtin_ctzll(above) : (uint32_t)__popcll(act);
            atomicAdd(count16 + s16, (unsigned long long)(end - lane));
          }
        }
      }
    };
    for (int h = 0; h < HALVES; ++h) {
      if (h > 0) {
        stage_half(h);
        __syncthreads();
      }
      if (skewed) write_out(std::true_type{}, h);
      else write_out(std::false_type{}, h);
      // After wave 0's writes: the grab has returned by then.
      if (h == HALVES - 1) fetch_desc();
      __syncthreads();
    }
    OS_MARK(4);  // write
  }
  if (C16) c16_flush();
#ifdef LSB_OS_PROFILE
  if (t == 0)
    for (int k = 0; k < 10; ++k) atomicAdd(&g_os_prof[k], (unsigned long long)prof[k]);
#endif
  if (NEXT) {
    for (int i = t; i < kSub * kBuckets; i += BLOCK)
      if (nh[i]) atomicAdd(&next_hist[i], nh[i]);
  }
  if (RG == 1 && bkt && cur_sub >= 0 && racc) atomicAdd(&rg.counts[t * kSub + cur_sub], racc);
}

template <int BLOCK, int IPT, bool NEXT, bool C16, int HALVES, bool SEG = false, bool GATHER = false, int RG = 0>
__global__ __launch_bounds__(BLOCK, (HALVES == 1 ? 2 : 3) * BLOCK / 256) void k_onesweep(
    const Elem* __restrict__ in, Elem* __restrict__ out, int64_t m, int shift, int next_shift,
    const uint32_t* __restrict__ sub_hist, uint32_t* __restrict__ next_hist,
    uint32_t* __restrict__ status, uint32_t* __restrict__ tile_ctr, uint32_t epoch,
    uint32_t* __restrict__ err, uint64_t* __restrict__ totals,
    unsigned long long* __restrict__ count16, SegPass seg, GatherSrc gs, RegionPass rg) {
  onesweep_body<BLOCK, IPT, NEXT, C16, HALVES, SEG, GATHER, RG>(in, out, m, shift, next_shift, sub_hist,
                                                                next_hist, status, tile_ctr, epoch, err, totals,
                                                                count16, seg, gs, rg);
}

// The placement probe's pass (lsb_context.cpp alloc_records): the same code
// as k_onesweep's next-counting instance under its own name, so that profiles
// and the bench's PMC passes keep the probe launches at context creation
// apart from the sort's.
__global__ __launch_bounds__(kOsBlock, 2 * kOsBlock / 256) void k_onesweep_probe(
    const Elem* __restrict__ in, Elem* __restrict__ out, int64_t m, int shift, int next_shift,
    const uint32_t* __restrict__ sub_hist, uint32_t* __restrict__ next_hist,
    uint32_t* __restrict__ status, uint32_t* __restrict__ tile_ctr, uint32_t epoch,
    uint32_t* __restrict__ err, uint64_t* __restrict__ totals,
    unsigned long long* __restrict__ count16, SegPass seg, GatherSrc gs) {
  onesweep_body<kOsBlock, kOsIpt, true, false, 1, false, false, 0>(in, out, m, shift, next_shift, sub_hist,
                                                                   next_hist, status, tile_ctr, epoch, err,
                                                                   totals, count16, seg, gs, RegionPass());
}

// ------------------------------------------------------------------- place
constexpr int kPlaceBlock = 256;
constexpr int kPlaceIpt = 8;
constexpr int kPlaceLdsBuckets = 4096;  // offset rows up to here (32 KiB) are staged in LDS
constexpr int kPlaceNextGrid = 1024;    // k_place<., kNext> grid cap (one flush per workgroup)

// One source's received range: record k in [k0, k0 + count) of the receive
// order (src[k - k0]) goes to out[off[digit] + k], off = that source's row of
// the placement table.  The exchange launches it per source and per slice,
// so a slice is placed while the next one is still in flight.
//
// kNext (per-digit exchange with single-read local passes): the placement
// also counts the next local digit (at next_shift) of every record by the
// onesweep sub-array of its output position over out_len records, in LDS,
// added to next_hist at the end: the next pass's sub_hist, so that pass
// needs no count read (k_subhist).  The exchange launches one k_place per
// (source, slice); they all add into one next_hist.
//
// kStore = false (LSB_OPT_EXCHANGE_GATHER): the count alone; the next pass
// gathers its tiles from where the records arrived (GatherSrc), so the
// placement's 16 B per record of writes go.
template <bool kLds, bool kNext, bool kStore = true>
__global__ __launch_bounds__(kPlaceBlock) void k_place(const Elem* __restrict__ src,
                                                       Elem* __restrict__ out, int64_t k0,
                                                       int64_t count, int shift, uint32_t mask,
                                                       const int64_t* __restrict__ off_row,
                                                       int64_t out_len, int next_shift,
                                                       uint32_t* __restrict__ next_hist, uint32_t skew) {
  __shared__ int64_t lds_off[kLds ? kPlaceLdsBuckets : 1];
  __shared__ uint32_t nh[kNext ? kSub * kBuckets : 1];
  const int nb = (int)mask + 1;
  const int64_t* off = off_row;
  const int64_t TT = (out_len + kTile - 1) / kTile;
  if (kNext)
    for (int i = threadIdx.x; i < kSub * kBuckets; i += kPlaceBlock) nh[i] = 0;
  if (kLds) {
    for (int i = threadIdx.x; i < nb; i += kPlaceBlock) lds_off[i] = off_row[i];
    off = lds_off;
  }
  if (kLds || kNext) __syncthreads();
  // kPlaceIpt records in flight per thread (a 1-record grid-stride loop
  // reached 4.4 TB/s; streaming copies need several loads outstanding).
  const int64_t step = (int64_t)gridDim.x * kPlaceBlock * kPlaceIpt;
  for (int64_t base = (int64_t)blockIdx.x * kPlaceBlock * kPlaceIpt + threadIdx.x; base < count;
       base += step) {
    Elem x[kPlaceIpt];
#pragma unroll
    for (int i = 0; i < kPlaceIpt; ++i) {
      const int64_t k = base + (int64_t)i * kPlaceBlock;
      x[i] = k < count ? load_elem(src + k) : Elem{0ull, 0ull};
    }
#pragma unroll
    for (int i = 0; i < kPlaceIpt; ++i) {
      const int64_t k = base + (int64_t)i * kPlaceBlock;
      if (k < count) {
        const uint32_t d = (uint32_t)(x[i].key >> shift) & mask;
        const int64_t g = off[d] + k0 + k;
        LSB_DASSERT(g >= 0 && g < out_len);
        if (kStore) store_elem(out + g, x[i]);
        if (kNext) {
          const uint32_t xs = (uint32_t)sub_of_tile(g / kTile, TT);
          const uint32_t slot = xs * kBuckets + ((uint32_t)(x[i].key >> next_shift) & (kBuckets - 1));
          if (skew) {
            // Skewed keys (the sort's stage split): one add per run of equal
            // slots within the wave-instruction, as k_onesweep's skewed count
            // (a source's records arrive in digit order, so hot keys come in
            // runs; active lanes are a prefix).  64 lanes adding to one LDS
            // counter cost 50 conflict cycles per instruction (Zipf, forced
            // 16-bit exchange: the count 3.43 vs 3.07 ms uniform).
            const uint64_t act = __ballot(1);
            const uint32_t lane = lane_id();
            const uint32_t prev =
                (uint32_t)__builtin_amdgcn_update_dpp((int)~slot, (int)slot, 0x138, 0xf, 0xf, false);
            const bool head = prev != slot;
            const uint64_t heads = __ballot(head);
            if (head) {
              const uint64_t above = heads & ~((2ull << lane) - 1ull);
              const uint32_t end = above ? (uint32_t)__builtin_ctzll(above) : (uint32_t)__popcll(act);
              atomicAdd(&nh[slot], end - lane);
            }
          } else {
            atomicAdd(&nh[slot], 1u);
          }
        }
      }
    }
  }
  if (kNext) {
    __syncthreads();
    for (int i = threadIdx.x; i < kSub * kBuckets; i += kPlaceBlock)
      if (nh[i]) atomicAdd(&next_hist[i], nh[i]);
  }
}

// ------------------------------------------ peer-store exchange (opt-in)
// The SHMEM / MPI-RMA form of the exchange (shmem/shmem_lsbsort.cpp:441-456
// shmem_putmem, mpi/mpi_lsbsort_onesided.cpp:487-509 MPI_Put): the sender
// writes each record straight into its owner's next A.  Record i of my
// bucket-ordered buffer, in bucket b, has global position g = base[b] + i,
// base[b] = (global start of (b, me) in digit-major, rank-minor order) -
// (local start of b); owner q = g / per, slot g - q * per.
struct PeerDests {
  Elem* dst[64];  // rank q's receiving buffer (this process's view of it)
};

constexpr int kPeerBaseBlock = 1024;
// s_waitcnt operand: vmcnt(0) (bits 3:0 and 15:14), expcnt(7) and lgkmcnt(15)
// left at their maxima, i.e. wait for this wave's vector memory operations only.
constexpr int kWaitVmcnt0 = 0x0F70;

// One workgroup: base[b] for b < nb from the all-gathered counts hist[s * nb + b].
__global__ __launch_bounds__(kPeerBaseBlock) void k_peer_base(const uint64_t* __restrict__ hist,
                                                              int P, int nb, int me,
                                                              int64_t* __restrict__ base) {
  __shared__ uint64_t tmp_t[kPeerBaseBlock / 64], tmp_m[kPeerBaseBlock / 64];
  const int t = threadIdx.x;
  const int per_t = (nb + kPeerBaseBlock - 1) / kPeerBaseBlock;
  const int b0 = t * per_t, b1 = min(nb, b0 + per_t);
  uint64_t tot = 0, mine = 0;
  for (int b = b0; b < b1; ++b) {
    for (int s = 0; s < P; ++s) tot += hist[(int64_t)s * nb + b];
    mine += hist[(int64_t)me * nb + b];
  }
  uint64_t all_t, all_m;
  uint64_t gt = block_exclusive_scan<kPeerBaseBlock>(tot, tmp_t, &all_t);
  uint64_t gm = block_exclusive_scan<kPeerBaseBlock>(mine, tmp_m, &all_m);
  for (int b = b0; b < b1; ++b) {
    uint64_t before = 0, tb = 0;
    for (int s = 0; s < P; ++s) {
      const uint64_t h = hist[(int64_t)s * nb + b];
      if (s < me) before += h;
      tb += h;
    }
    base[b] = (int64_t)(gt + before) - (int64_t)gm;
    gt += tb;
    gm += hist[(int64_t)me * nb + b];
  }
}

template <bool kLds>
__global__ __launch_bounds__(kPlaceBlock) void k_peer_scatter(const Elem* __restrict__ src,
                                                              int64_t m, int shift, uint32_t mask,
                                                              const int64_t* __restrict__ base_g,
                                                              int64_t per, int P, PeerDests d) {
  __shared__ int64_t lds_base[kLds ? kPlaceLdsBuckets : 1];
  const int nb = (int)mask + 1;
  const int64_t* base = base_g;
  if (kLds) {
    for (int i = threadIdx.x; i < nb; i += kPlaceBlock) lds_base[i] = base_g[i];
    __syncthreads();
    base = lds_base;
  }
  const double inv_per = 1.0 / (double)per;
  const int64_t step = (int64_t)gridDim.x * kPlaceBlock * kPlaceIpt;
  for (int64_t i0 = (int64_t)blockIdx.x * kPlaceBlock * kPlaceIpt + threadIdx.x; i0 < m;
       i0 += step) {
    Elem x[kPlaceIpt];
#pragma unroll
    for (int j = 0; j < kPlaceIpt; ++j) {
      const int64_t i = i0 + (int64_t)j * kPlaceBlock;
      x[j] = i < m ? load_elem(src + i) : Elem{0ull, 0ull};
    }
#pragma unroll
    for (int j = 0; j < kPlaceIpt; ++j) {
      const int64_t i = i0 + (int64_t)j * kPlaceBlock;
      if (i < m) {
        const uint32_t b = (uint32_t)(x[j].key >> shift) & mask;
        const int64_t g = base[b] + i;
        int q = (int)((double)g * inv_per);  // then exact: q * per <= g < (q + 1) * per
        if ((int64_t)q * per > g) --q;
        if ((int64_t)(q + 1) * per <= g) ++q;
        LSB_DASSERT(q >= 0 && q < P);
        store_elem(d.dst[q] + (g - (int64_t)q * per), x[j]);
      }
    }
  }
  // Release at system scope (shmem_putmem's completion before
  // shmem_barrier_all, shmem/shmem_lsbsort.cpp:455-456).  Every wave first
  // waits for its own stores to complete (s_waitcnt vmcnt(0); a store
  // completes once the L2 has taken it).  __syncthreads alone does not emit
  // that wait: the compiler's workgroup-scope barrier relies on the CU's
  // in-order path to the L2, which says nothing about what another wave's
  // stores have reached when wave 0 writes the L2 back.  After the barrier
  // the workgroup's stores are all in this XCD's L2, and one system-scope
  // release writes it back (buffer_wbl2 sc0 sc1, then its own wait), so
  // stores to a peer's memory that the L2 holds reach it before the kernel
  // ends.  tests/test_peer_fence.py checks this order in the code object.
  // The owner acquires (k_system_acquire) after the barrier collective,
  // before its next pass reads the buffer.
  __builtin_amdgcn_s_waitcnt(kWaitVmcnt0);
  __syncthreads();
  if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
}

// Acquire at system scope on every XCD (workgroup w runs on XCD w % 8):
// invalidates the L2 lines a peer's stores may have made stale, before the
// owner reads what the peers wrote into its buffer.
__global__ __launch_bounds__(64) void k_system_acquire() {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

// --------------------------------------------- 16-bit digit counts (P > 1)
// After the two 8-bit local sub-passes of a 16-bit digit the rank's records
// are sorted by that digit, so its 65536-bin histogram is the run lengths:
// k_digit_starts marks the first index of every present digit, k_starts_to_counts
// turns starts into counts (an absent digit counts 0).
__global__ __launch_bounds__(256) void k_digit_starts(const Elem* __restrict__ A, int64_t m,
                                                      int shift, int64_t* __restrict__ first) {
  constexpr int IPT = 8;
  const uint64_t* __restrict__ keys = reinterpret_cast<const uint64_t*>(A);
  const int64_t step = (int64_t)gridDim.x * 256 * IPT;
  for (int64_t base = (int64_t)blockIdx.x * 256 * IPT + threadIdx.x; base < m; base += step) {
    uint64_t k[IPT], kp[IPT];
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
      const int64_t i = base + (int64_t)j * 256;
      k[j] = i < m ? keys[2 * i] : 0ull;
      kp[j] = (i > 0 && i < m) ? keys[2 * (i - 1)] : 0ull;  // L1/L2 hit: the neighbour lane's line
    }
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
      const int64_t i = base + (int64_t)j * 256;
      const uint32_t d = (uint32_t)(k[j] >> shift) & 0xFFFFu;
      if (i < m && (i == 0 || ((uint32_t)(kp[j] >> shift) & 0xFFFFu) != d)) first[d] = i;
    }
  }
}

constexpr int kStartsBlock = 1024;
constexpr int kStartsPer = 65536 / kStartsBlock;  // 64 digits per thread

// One workgroup.  first[d] = -1 for absent digits.
__global__ __launch_bounds__(kStartsBlock) void k_starts_to_counts(const int64_t* __restrict__ first,
                                                                   int64_t m,
                                                                   uint64_t* __restrict__ counts) {
  __shared__ int64_t nxt[kStartsBlock / 64];
  const int t = threadIdx.x;
  const int d0 = t * kStartsPer;
  // first present start in my range (or m): the suffix-min seen by the thread before me
  int64_t mine = m;
  for (int j = kStartsPer - 1; j >= 0; --j) {
    const int64_t f = first[d0 + j];
    if (f >= 0 && f < m) mine = f;
  }
  // suffix min over threads t+1.. (starts increase with the digit, so the
  // next present start after my range is the first present start of the
  // nearest later thread that has one)
  int64_t after = m;
  {
    int64_t v = mine;
    const uint32_t lane = lane_id();
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int64_t u = __shfl_down(v, off, 64);
      if (lane + off < 64) v = u < v ? u : v;
    }
    // v = min over lanes >= lane in this wave; need strictly later threads
    const int64_t later_in_wave = __shfl_down(v, 1, 64);
    if (lane == 0) nxt[t >> 6] = v;
    __syncthreads();
    int64_t later_waves = m;
    for (int w = (t >> 6) + 1; w < kStartsBlock / 64; ++w) later_waves = nxt[w] < later_waves ? nxt[w] : later_waves;
    after = lane == 63 ? later_waves : (later_in_wave < later_waves ? later_in_wave : later_waves);
  }
  int64_t next = after;
  for (int j = kStartsPer - 1; j >= 0; --j) {
    const int64_t f = first[d0 + j];
    if (f >= 0 && f < m) {
      counts[d0 + j] = (uint64_t)(next - f);
      next = f;
    } else {
      counts[d0 + j] = 0;
    }
  }
}

// ------------------------------------------------------------ device plan
// The exchange plan of rank `me` from the all-gathered counts hist[s][b]
// (the same rule as the host planner lsb_plan_exchange):
//   gstart[b][s] = base[b] + colpre[s][b],  base = excl. scan of column sums,
//   colpre[s][b] = sum_{s'<s} hist[s'][b]   (digit-major, rank-minor order,
//   mpi/mpi_lsbsort.cpp:350,378,401)
// k_plan_cols:   colpre (into work) and column totals
// k_plan_base:   base = exclusive scan of the totals (one workgroup)
// k_plan_pieces: the piece of run (s, b) inside my range -> len (into work),
//                its first dest (into place); my own runs -> send counts
// k_plan_rows:   per source, exclusive scan of piece lengths over buckets
// k_plan_finish: place_off[s][b] = (piece start - lo) - (recv_displ[s] + k),
//                rend[s] = inclusive scan of recv counts
__global__ __launch_bounds__(256) void k_plan_cols(const uint64_t* __restrict__ hist, int P, int nb,
                                                   int64_t* __restrict__ work,
                                                   int64_t* __restrict__ total) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b >= nb) return;
  int64_t t = 0;
  for (int s = 0; s < P; ++s) {
    work[(int64_t)s * nb + b] = t;
    t += (int64_t)hist[(int64_t)s * nb + b];
  }
  total[b] = t;
}

constexpr int kPlanScanBlock = 1024;

// Exclusive scan of v[idx(0..len)) in place by one workgroup, in the order
// idx gives (the identity, or the chunked exchange's order), returns the sum.
// Segments of 4 * kPlanScanBlock entries; thread t owns 4 consecutive
// entries of a segment, so every load and store is coalesced (for the
// chunked order: runs of 2^cshift consecutive entries).
template <typename Idx>
__device__ int64_t block_scan_inplace(int64_t* v, int len, int64_t* tmp, Idx idx) {
  constexpr int V = 4;
  int64_t carry = 0;
  for (int seg = 0; seg < len; seg += V * kPlanScanBlock) {
    const int i0 = seg + V * (int)threadIdx.x;
    int64_t x[V];
    int64_t s = 0;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      x[j] = i0 + j < len ? v[idx(i0 + j)] : 0;
      s += x[j];
    }
    int64_t tot;
    int64_t pre = carry + block_exclusive_scan<kPlanScanBlock>(s, tmp, &tot);
#pragma unroll
    for (int j = 0; j < V; ++j) {
      if (i0 + j < len) v[idx(i0 + j)] = pre;
      pre += x[j];
    }
    carry += tot;
  }
  return carry;
}

__global__ __launch_bounds__(kPlanScanBlock) void k_plan_base(int64_t* __restrict__ total, int nb) {
  __shared__ int64_t tmp[kPlanScanBlock / 64];
  block_scan_inplace(total, nb, tmp, [](int i) { return i; });  // total -> base
}

// cshift < 8 (the chunked exchange): also the send counts per (owner q,
// chunk k of b) into chunk_send[q * C + k].
__global__ __launch_bounds__(256) void k_plan_pieces(const uint64_t* __restrict__ hist, int P, int nb,
                                                     int me, int64_t per, int64_t lo, int64_t hi,
                                                     const int64_t* __restrict__ base,
                                                     int64_t* __restrict__ work,
                                                     int64_t* __restrict__ place,
                                                     unsigned long long* __restrict__ send_counts,
                                                     int64_t* __restrict__ gstart, int cshift,
                                                     unsigned long long* __restrict__ chunk_send) {
  // Send counts are summed per workgroup in LDS first: every bucket of a
  // rank adds to the same few owners, and 65536 same-address global
  // atomics took 0.8 ms.
  __shared__ unsigned long long sc[64 * kMaxExchangeChunks];
  const int C = kBuckets >> cshift;  // 1 unchunked
  for (int i = threadIdx.x; i < 64 * kMaxExchangeChunks; i += 256) sc[i] = 0;
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < (int64_t)P * nb) {
    const int s = (int)(i / nb);
    const int b = (int)(i - (int64_t)s * nb);
    const int64_t h = (int64_t)hist[i];
    const int64_t g0 = base[b] + work[i];
    const int64_t g1 = g0 + h;
    const int64_t plo = g0 > lo ? g0 : lo;
    const int64_t phi = g1 < hi ? g1 : hi;
    work[i] = phi > plo ? phi - plo : 0;  // piece length
    place[i] = plo;                       // piece's first dest (if any)
    if (gstart) {  // (b, s) order: the placed order of my block
      const int64_t l = g0 < lo ? 0 : (g0 > hi ? hi - lo : g0 - lo);
      gstart[(int64_t)b * P + s] = l;
    }
    if (s == me && h > 0) {
      const int k = (b & (kBuckets - 1)) >> cshift;
      int64_t g = g0;
      while (g < g1) {  // split my run over its owners
        const int64_t q = g / per;
        const int64_t qend = g1 < (q + 1) * per ? g1 : (q + 1) * per;
        atomicAdd(&sc[q * C + k], (unsigned long long)(qend - g));
        g = qend;
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < P * C; i += 256) {
    if (!sc[i]) continue;
    atomicAdd(&send_counts[i / C], sc[i]);
    if (chunk_send) atomicAdd(&chunk_send[i], sc[i]);
  }
}

// cshift < 8 (the chunked exchange, nb = 65536): source s's pieces scanned
// in chunk order -- (chunk of the low byte, high byte, low byte), the order
// its records arrive in R -- and chunk_recv[s * C + k] = the records of chunk
// k it sends me.
__global__ __launch_bounds__(kPlanScanBlock) void k_plan_rows(int64_t* __restrict__ work, int nb,
                                                              int64_t* __restrict__ recv_counts, int cshift,
                                                              int64_t* __restrict__ chunk_recv) {
  __shared__ int64_t tmp[kPlanScanBlock / 64];
  const int s = blockIdx.x;
  int64_t* row = work + (int64_t)s * nb;
  int64_t tot;
  if (cshift >= 8) {
    tot = block_scan_inplace(row, nb, tmp, [](int i) { return i; });
  } else {
    const int lw = 1 << cshift;
    tot = block_scan_inplace(row, nb, tmp, [=](int i) {
      const int k = i >> (8 + cshift), h = (i >> cshift) & (kBuckets - 1), l = (k << cshift) | (i & (lw - 1));
      return (h << 8) | l;
    });
    __syncthreads();
    const int C = kBuckets >> cshift;
    if ((int)threadIdx.x < C) {
      const int k = threadIdx.x;
      const int64_t a = row[k << cshift];  // the first digit of chunk k in that order: (h 0, l = k << cshift)
      const int64_t e = k + 1 < C ? row[(k + 1) << cshift] : tot;
      chunk_recv[(int64_t)s * C + k] = e - a;
    }
  }
  if (threadIdx.x == 0) recv_counts[s] = tot;
}

__global__ __launch_bounds__(256) void k_plan_finish(int P, int nb, int64_t lo,
                                                     const int64_t* __restrict__ work,
                                                     const int64_t* __restrict__ recv_counts,
                                                     int64_t* __restrict__ place) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < P) {  // rend
    int64_t acc = 0;
    for (int s = 0; s <= (int)i; ++s) acc += recv_counts[s];
    place[(int64_t)P * nb + i] = acc;
  }
  if (i >= (int64_t)P * nb) return;
  const int s = (int)(i / nb);
  int64_t displ = 0;
  for (int q = 0; q < s; ++q) displ += recv_counts[q];
  place[i] = (place[i] - lo) - (displ + work[i]);
}

__global__ __launch_bounds__(256) void k_gather_adj(GatherSrc g, int64_t* __restrict__ gadj) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e < (int64_t)g.P * g.nb) gadj[e] = gather_adj(g, (int)e);
}

// Tile descriptors of a gathered pass: tile t's pieces (at most kDescPieces,
// else kDescOverflow and the per-record search over [e0, e1]).
__global__ __launch_bounds__(256) void k_gather_desc(GatherSrc g, int64_t m, int64_t TT,
                                                     TileDesc* __restrict__ desc) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= TT) return;
  const int cells = g.P * g.nb;
  const int64_t tb = t * kTile;
  const int64_t te = (tb + kTile < m ? tb + kTile : m) - 1;
  const int e0 = gather_piece(g, 0, cells - 1, tb);
  const int e1 = gather_piece(g, e0, cells - 1, te);
  TileDesc d;
  d.e0 = e0;
  d.e1 = e1;
  d.sel = 0;
  int n = 0;
#pragma unroll
  for (int k = 0; k < kDescPieces; ++k) {
    d.start[k] = 0x7FFFFFFF;
    d.adj[k] = 0;
  }
  if (e1 - e0 < 64) {
    for (int e = e0; e <= e1; ++e) {
      const int64_t st = g.gstart[e], en = e + 1 < cells ? g.gstart[e + 1] : m;
      if (en <= st) continue;  // empty piece
      if (n == kDescPieces) {
        n = kDescOverflow;
        break;
      }
      const int64_t v = gather_adj(g, e);
      d.start[n] = st > tb ? (int32_t)(st - tb) : 0;
      d.adj[n] = v >> 1;
      d.sel |= (int)(v & 1) << n;
      ++n;
    }
  } else {
    n = kDescOverflow;
  }
  d.n = n;
  desc[t] = d;
}

// ------------------------------------------------------------------ copy
// A loopback exchange's transfer between two record buffers of one device
// (copy_range): a plain streaming copy whose addresses go through the GPU's
// page tables only, not through the runtime's lookup of what a pointer
// belongs to (hipMemcpyAsync), which has to track VMM ranges as they are
// mapped, released and mapped again.
__global__ __launch_bounds__(256) void k_copy_records(Elem* __restrict__ dst, const Elem* __restrict__ src,
                                                      int64_t cnt) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < cnt; i += stride)
    store_elem(dst + i, load_elem_nt(src + i));
}

// ------------------------------------------------------------------ checks
__global__ __launch_bounds__(256) void k_verify(const Elem* __restrict__ A, int64_t here,
                                                int64_t gbase, int64_t n, int64_t per, KeyGen gen,
                                                unsigned long long* first_bad) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < here; i += stride) {
    const Elem x = load_elem(A + i);
    bool bad = x.val >= (uint64_t)n;
    if (!bad) {
      const uint64_t r = x.val / (uint64_t)per;
      const uint64_t idx = x.val - r * (uint64_t)per;
      bad = make_key(pcg_output(pcg_jump(pcg_seed(r), idx + 1)), gen) != x.key;
    }
    if (i + 1 < here) {
      const Elem y = load_elem(A + i + 1);
      bad |= !(x.key < y.key || (x.key == y.key && x.val < y.val));
    }
    if (bad) atomicMin(first_bad, (unsigned long long)(gbase + i));
  }
}

__global__ __launch_bounds__(256) void k_check_sorted(const Elem* __restrict__ A, int64_t here,
                                                      unsigned int* unsorted) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i + 1 < here; i += stride) {
    if (A[i + 1].key < A[i].key) *unsorted = 1u;
  }
}

int grid_for(int64_t work, int block, int cap) {
  const int64_t g = (work + block - 1) / block;
  return (int)(g < 1 ? 1 : (g > cap ? cap : g));
}

}  // namespace

Chunking make_chunking(int64_t m, int max_chunks) {
  Chunking ch;
  if (m <= 0) return ch;
  if (max_chunks > kMaxChunks) max_chunks = kMaxChunks;
  if (max_chunks < 1) max_chunks = 1;
  const int64_t tiles = (m + kTile - 1) / kTile;
  const int64_t tiles_per_chunk = (tiles + max_chunks - 1) / max_chunks;
  ch.chunk_elems = tiles_per_chunk * kTile;
  ch.num_chunks = (int)((m + ch.chunk_elems - 1) / ch.chunk_elems);
  return ch;
}

hipError_t launch_pcg_fill(Elem* A, int64_t count, uint64_t seed, uint64_t val0, KeyGen gen,
                           hipStream_t s) {
  if (count <= 0) return hipSuccess;
  const int64_t threads = (count + kFillPerThread - 1) / kFillPerThread;
  const int64_t blocks = (threads + 255) / 256;
  hipLaunchKernelGGL(k_pcg_fill, dim3((unsigned)blocks), dim3(256), 0, s, A, count, seed, val0,
                     gen);
  return hipGetLastError();
}

hipError_t launch_digit16_counts(const Elem* A, int64_t m, int shift, int64_t* first,
                                 uint64_t* counts, hipStream_t s) {
  hipError_t e = hipMemsetAsync(first, 0xff, sizeof(int64_t) * 65536, s);
  if (e != hipSuccess) return e;
  if (m > 0)
    hipLaunchKernelGGL(k_digit_starts, dim3(grid_for(m, 256, 8192)), dim3(256), 0, s, A, m, shift,
                       first);
  hipLaunchKernelGGL(k_starts_to_counts, dim3(1), dim3(kStartsBlock), 0, s, first, m, counts);
  return hipGetLastError();
}

hipError_t launch_starts_reset(int64_t* first, hipStream_t s) {
  // 0x7f7f... > any record index: "absent" for atomicMin and for the counts.
  return hipMemsetAsync(first, 0x7f, sizeof(int64_t) * 65536, s);
}

hipError_t launch_starts_to_counts(const int64_t* first, int64_t m, uint64_t* counts,
                                   hipStream_t s) {
  hipLaunchKernelGGL(k_starts_to_counts, dim3(1), dim3(kStartsBlock), 0, s, first, m, counts);
  return hipGetLastError();
}

hipError_t launch_upsweep(const Elem* A, int64_t m, int shift, Chunking ch, uint32_t* chunk_hist,
                          uint64_t* span, hipStream_t s) {
  if (m <= 0) return hipSuccess;
  if (span)
    hipLaunchKernelGGL((k_upsweep<256, 16, true>), dim3(ch.num_chunks), dim3(256), 0, s, A, m,
                       shift, ch.chunk_elems, ch.num_chunks, chunk_hist,
                       reinterpret_cast<unsigned long long*>(span));
  else
    hipLaunchKernelGGL((k_upsweep<256, 16, false>), dim3(ch.num_chunks), dim3(256), 0, s, A, m,
                       shift, ch.chunk_elems, ch.num_chunks, chunk_hist, nullptr);
  return hipGetLastError();
}

hipError_t launch_scan(const uint32_t* chunk_hist, int G, uint64_t* chunk_off, uint64_t* totals,
                       hipStream_t s) {
  if (G <= 0) return hipSuccess;
  if (G > kMaxChunks) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_scan, dim3(kBuckets), dim3(kScanBlock), 0, s, chunk_hist, G, chunk_off,
                     totals);
  return hipGetLastError();
}

hipError_t launch_scatter(const Elem* in, Elem* out, int64_t m, int shift, Chunking ch,
                          const uint64_t* chunk_off, const uint64_t* totals, int64_t* first16,
                          hipStream_t s) {
  if (m <= 0) return hipSuccess;
  if (first16) {
    if (shift < 8) return hipErrorInvalidValue;
    hipLaunchKernelGGL((k_scatter<kScatterBlock, kScatterIpt, true>), dim3(ch.num_chunks),
                       dim3(kScatterBlock), 0, s, in, out, m, shift, ch.chunk_elems, ch.num_chunks,
                       chunk_off, totals, reinterpret_cast<long long*>(first16));
  } else {
    hipLaunchKernelGGL((k_scatter<kScatterBlock, kScatterIpt, false>), dim3(ch.num_chunks),
                       dim3(kScatterBlock), 0, s, in, out, m, shift, ch.chunk_elems, ch.num_chunks,
                       chunk_off, totals, nullptr);
  }
  return hipGetLastError();
}

hipError_t onesweep_profile(unsigned long long* out10, bool reset) {
#ifdef LSB_OS_PROFILE
  hipError_t e = hipMemcpyFromSymbol(out10, HIP_SYMBOL(g_os_prof), 10 * sizeof(unsigned long long));
  if (e != hipSuccess || !reset) return e;
  const unsigned long long z[10] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_os_prof), z, sizeof z);
#else
  for (int k = 0; k < 10; ++k) out10[k] = 0;
  (void)reset;
  return hipErrorNotSupported;
#endif
}

hipError_t launch_subhist(const Elem* A, int64_t m, int shift, int grid, uint32_t* sub_hist,
                          uint64_t* span, hipStream_t s) {
  hipError_t e = hipMemsetAsync(sub_hist, 0, sizeof(uint32_t) * kSub * kBuckets, s);
  if (e != hipSuccess || m <= 0) return e;
  const int64_t TT = (m + kTile - 1) / kTile;
  if (grid < 1) grid = 1;
  const int64_t tpw = (TT + grid - 1) / grid;
  const dim3 g((unsigned)((TT + tpw - 1) / tpw));
  if (span)
    hipLaunchKernelGGL((k_subhist<kScatterBlock, kScatterIpt, true>), g, dim3(kScatterBlock), 0, s,
                       A, m, shift, tpw, sub_hist, reinterpret_cast<unsigned long long*>(span));
  else
    hipLaunchKernelGGL((k_subhist<kScatterBlock, kScatterIpt, false>), g, dim3(kScatterBlock), 0, s,
                       A, m, shift, tpw, sub_hist, nullptr);
  return hipGetLastError();
}

hipError_t launch_count16_chunks(const Elem* B, int64_t m, int shift16, const uint32_t* lo_hist, int cshift,
                                 int grid, uint64_t* count16, uint32_t* chunk_hist, hipStream_t s) {
  if (shift16 < 0 || shift16 > 48 || cshift < 5 || cshift > 7 || !lo_hist) return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(count16, 0, sizeof(uint64_t) * 65536, s);
  if (e == hipSuccess)
    e = hipMemsetAsync(chunk_hist, 0, sizeof(uint32_t) * (kBuckets >> cshift) * kSub * kBuckets, s);
  if (e != hipSuccess || m <= 0) return e;
  const int64_t TT = (m + kTile - 1) / kTile;
  if (grid < 1) grid = 1;
  const int64_t tpw = (TT + grid - 1) / grid;
  hipLaunchKernelGGL((k_count16c<kScatterBlock, kScatterIpt>), dim3((unsigned)((TT + tpw - 1) / tpw)),
                     dim3(kScatterBlock), 0, s, B, m, shift16, lo_hist, cshift, tpw,
                     reinterpret_cast<unsigned long long*>(count16), chunk_hist);
  return hipGetLastError();
}

hipError_t launch_sample(const Elem* A, int64_t m, int shift, uint32_t* hist, uint64_t* span, hipStream_t s) {
  if (shift < 0 || shift > 56) return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(hist, 0, sizeof(uint32_t) * kBuckets, s);
  if (e == hipSuccess) e = hipMemsetAsync(span, 0, 2 * sizeof(uint64_t), s);
  if (e != hipSuccess || m <= 0) return e;
  const int64_t TT = (m + kTile - 1) / kTile;
  const unsigned g = (unsigned)(TT < kSampleTiles ? TT : kSampleTiles);
  hipLaunchKernelGGL(k_sample, dim3(g), dim3(kSampleBlock), 0, s, A, m, shift, hist,
                     reinterpret_cast<unsigned long long*>(span));
  return hipGetLastError();
}

int onesweep_halves_for(const uint32_t* h, int64_t m) {
  for (int b = 0; b < kBuckets; ++b) {
    uint64_t tot = 0;
    for (int x = 0; x < kSub; ++x) tot += h[x * kBuckets + b];
    // The kernel's own `skewed` test; a bucket holding every record is a
    // constant byte of this rank (its pass is the identity), not skew.
    if (tot > (uint64_t)(m >> 5) && tot < (uint64_t)m) return 2;
  }
  return 1;
}

hipError_t launch_onesweep(const Elem* in, Elem* out, int64_t m, int shift, int next_shift,
                           const uint32_t* sub_hist, uint32_t* next_hist, uint32_t* status,
                           uint32_t* tile_ctr, uint32_t epoch, uint32_t* err, int grid,
                           hipStream_t s, OnesweepExtra extra) {
  if (m <= 0) return hipSuccess;
  if (m > kOnesweepMaxElems || epoch == 0 || epoch >= (1u << 31) || shift < 0 || shift > 56 ||
      next_shift > 56 || (extra.halves != 1 && extra.halves != 2))
    return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(tile_ctr, 0, sizeof(uint32_t) * kSub, s);
  if (e != hipSuccess) return e;
  const int rm = extra.region_mode;
  const RegionPass rp = extra.region ? *extra.region : RegionPass();
  if (rm < 0 || rm > 2 || (rm != 0 && (!extra.region || rp.cap <= 0 || rp.cap % kTile != 0 ||
                                       rp.cap * kRegions < m || !rp.counts)))
    return hipErrorInvalidValue;
  // Tiles of the input: the regional layout's slots for its reading pass.
  const int64_t TT = rm == 2 ? rp.cap / kTile * kRegions : (m + kTile - 1) / kTile;
  auto* c16 = reinterpret_cast<unsigned long long*>(extra.count16);
  const bool gat = extra.gather != nullptr;
  // The split stage only for the plain and next-digit forms, never gathered
  // (its gathered instances spill: 160-236 B per lane at 168 VGPRs; a
  // gathered pass takes the whole stage, lsb_exchange.cpp local_pass_os).
  if (extra.halves == 2 && gat) return hipErrorInvalidValue;
  const bool split = extra.halves == 2 && c16 == nullptr;
  // Persistent grid (`grid` = 2 workgroups per CU; 3 with the split stage),
  // a multiple of the XCD count; no more than the tiles.
  int64_t g = split ? (int64_t)grid * 3 / 2 : grid;
  if (g < kSub) g = kSub;
  if (g > (TT + kSub - 1) / kSub * kSub) g = (TT + kSub - 1) / kSub * kSub;
  const dim3 gd((unsigned)g), bd(split ? kOsSplitBlock : kOsBlock);
  uint32_t* st = status;
  const GatherSrc gsrc = extra.gather ? *extra.gather : GatherSrc();
  // One launch of the instance, gathered or not.
  auto go = [&](auto kplain, auto kgather, int nshift, uint32_t* nhist, unsigned long long* cnt16,
                SegPass sp) {
    hipLaunchKernelGGL(gat ? kgather : kplain, gd, bd, 0, s, in, out, m, shift, nshift, sub_hist, nhist,
                       st, tile_ctr, epoch, err, extra.totals, cnt16, sp, gsrc, RegionPass());
  };
  if (rm != 0) {
    // The regional first pass (rm = 1) and the pass that reads its layout
    // (rm = 2): whole stage, no 16-bit counts, totals, segments or gathering.
    if (c16 || extra.halves != 1 || extra.seg || gat || extra.probe || extra.totals) return hipErrorInvalidValue;
    if (rm == 1 && (next_shift < 0 || !rp.ovf)) return hipErrorInvalidValue;
    if (next_shift >= 0) {
      e = hipMemsetAsync(next_hist, 0, sizeof(uint32_t) * kSub * kBuckets, s);
      if (e != hipSuccess) return e;
    }
    if (rm == 1) {
      e = hipMemsetAsync(rp.counts, 0, sizeof(uint32_t) * kRegions, s);
      if (e == hipSuccess) e = hipMemsetAsync(rp.ovf, 0, sizeof(uint32_t), s);
      if (e != hipSuccess) return e;
      hipLaunchKernelGGL((k_onesweep<kOsBlock, kOsIpt, true, false, 1, false, false, 1>), gd, bd, 0, s, in, out,
                         m, shift, next_shift, sub_hist, next_hist, st, tile_ctr, epoch, err, nullptr, nullptr,
                         SegPass(), gsrc, rp);
    } else if (next_shift >= 0) {
      hipLaunchKernelGGL((k_onesweep<kOsBlock, kOsIpt, true, false, 1, false, false, 2>), gd, bd, 0, s, in, out,
                         m, shift, next_shift, sub_hist, next_hist, st, tile_ctr, epoch, err, nullptr, nullptr,
                         SegPass(), gsrc, rp);
    } else {
      hipLaunchKernelGGL((k_onesweep<kOsBlock, kOsIpt, false, false, 1, false, false, 2>), gd, bd, 0, s, in, out,
                         m, shift, 0, sub_hist, nullptr, st, tile_ctr, epoch, err, nullptr, nullptr, SegPass(),
                         gsrc, rp);
    }
  } else if (extra.probe) {
    // The placement probe: a pass counting the next digit (the sort's usual
    // instance), whole stage, under its own name.
    if (next_shift < 0 || !next_hist || c16 || extra.halves != 1 || extra.seg || gat) return hipErrorInvalidValue;
    e = hipMemsetAsync(next_hist, 0, sizeof(uint32_t) * kSub * kBuckets, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_onesweep_probe, gd, bd, 0, s, in, out, m, shift, next_shift, sub_hist, next_hist, st,
                       tile_ctr, epoch, err, nullptr, nullptr, SegPass(), gsrc);
  } else if (extra.seg) {
    // The hybrid's last pass: no next digit, no 16-bit counts, whole stage.
    if (next_shift >= 0 || c16 || extra.halves != 1 || !extra.seg->base ||
        !extra.seg->err || gat)
      return hipErrorInvalidValue;
    hipLaunchKernelGGL((k_onesweep<kOsBlock, kOsIpt, false, false, 1, true>), gd, bd, 0, s, in, out, m,
                       shift, 0, sub_hist, nullptr, st, tile_ctr, epoch, err, extra.totals, nullptr,
                       *extra.seg, gsrc, RegionPass());
  } else if (c16) {
    // The 16-bit counts need the low byte below this digit, and no next
    // digit: the exchange follows this pass.
    if (shift < 8 || next_shift >= 0) return hipErrorInvalidValue;
    e = hipMemsetAsync(c16, 0, sizeof(uint64_t) * 65536, s);
    if (e != hipSuccess) return e;
    go(k_onesweep<kOsBlock, kOsIpt, false, true, 1>, k_onesweep<kOsBlock, kOsIpt, false, true, 1, false, true>,
       0, nullptr, c16, SegPass());
  } else if (next_shift >= 0) {
    e = hipMemsetAsync(next_hist, 0, sizeof(uint32_t) * kSub * kBuckets, s);
    if (e != hipSuccess) return e;
    if (split)  // never gathered (checked above)
      go(k_onesweep<kOsSplitBlock, kOsSplitIpt, true, false, 2>,
         k_onesweep<kOsSplitBlock, kOsSplitIpt, true, false, 2>, next_shift, next_hist, nullptr, SegPass());
    else
      go(k_onesweep<kOsBlock, kOsIpt, true, false, 1>, k_onesweep<kOsBlock, kOsIpt, true, false, 1, false, true>,
         next_shift, next_hist, nullptr, SegPass());
  } else if (split) {  // never gathered (checked above)
    go(k_onesweep<kOsSplitBlock, kOsSplitIpt, false, false, 2>,
       k_onesweep<kOsSplitBlock, kOsSplitIpt, false, false, 2>, 0, nullptr, nullptr, SegPass());
  } else {
    go(k_onesweep<kOsBlock, kOsIpt, false, false, 1>, k_onesweep<kOsBlock, kOsIpt, false, false, 1, false, true>,
       0, nullptr, nullptr, SegPass());
  }
  return hipGetLastError();
}

hipError_t launch_place(const Elem* src, Elem* out, int64_t out_len, int64_t k0, int64_t count,
                        int shift, int nbuckets, const int64_t* off_row, hipStream_t s,
                        int next_shift, uint32_t* next_hist, bool store, bool skew) {
  if (count <= 0) return hipSuccess;
  if (nbuckets != 256 && nbuckets != 65536) return hipErrorInvalidValue;
  if (k0 < 0 || k0 + count > out_len) return hipErrorInvalidValue;
  const uint32_t mask = (uint32_t)nbuckets - 1;
  const bool lds = nbuckets <= kPlaceLdsBuckets;
  if (next_shift >= 0) {
    if (next_shift > 56 || !next_hist || out_len > kOnesweepMaxElems) return hipErrorInvalidValue;
    // Fewer, longer-lived workgroups: each flushes its 8 x 256 counters once.
    const dim3 grid(grid_for(count, kPlaceBlock * kPlaceIpt, kPlaceNextGrid));
    if (!store) {
      if (lds)
        hipLaunchKernelGGL((k_place<true, true, false>), grid, dim3(kPlaceBlock), 0, s, src, out, k0,
                           count, shift, mask, off_row, out_len, next_shift, next_hist, skew ? 1u : 0u);
      else
        hipLaunchKernelGGL((k_place<false, true, false>), grid, dim3(kPlaceBlock), 0, s, src, out, k0,
                           count, shift, mask, off_row, out_len, next_shift, next_hist, skew ? 1u : 0u);
      return hipGetLastError();
    }
    if (lds)
      hipLaunchKernelGGL((k_place<true, true>), grid, dim3(kPlaceBlock), 0, s, src, out, k0, count,
                         shift, mask, off_row, out_len, next_shift, next_hist, skew ? 1u : 0u);
    else
      hipLaunchKernelGGL((k_place<false, true>), grid, dim3(kPlaceBlock), 0, s, src, out, k0, count,
                         shift, mask, off_row, out_len, next_shift, next_hist, skew ? 1u : 0u);
    return hipGetLastError();
  }
  if (!store) return hipErrorInvalidValue;  // nothing to count
  const dim3 grid(grid_for(count, kPlaceBlock * kPlaceIpt, 4096));
  if (lds)
    hipLaunchKernelGGL((k_place<true, false>), grid, dim3(kPlaceBlock), 0, s, src, out, k0, count,
                       shift, mask, off_row, out_len, 0, nullptr, 0u);
  else
    hipLaunchKernelGGL((k_place<false, false>), grid, dim3(kPlaceBlock), 0, s, src, out, k0, count,
                       shift, mask, off_row, out_len, 0, nullptr, 0u);
  return hipGetLastError();
}

hipError_t launch_peer_exchange(const Elem* src, int64_t m, int shift, int nbuckets,
                                const uint64_t* hist, int P, int me, int64_t per,
                                Elem* const* dst, int64_t* base, hipStream_t s) {
  if (P < 1 || P > 64 || me < 0 || me >= P || (nbuckets != 256 && nbuckets != 65536))
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_peer_base, dim3(1), dim3(kPeerBaseBlock), 0, s, hist, P, nbuckets, me, base);
  if (m <= 0) return hipGetLastError();
  PeerDests d{};
  for (int q = 0; q < P; ++q) d.dst[q] = dst[q];
  const dim3 grid(grid_for(m, kPlaceBlock * kPlaceIpt, 4096));
  const uint32_t mask = (uint32_t)nbuckets - 1;
  if (nbuckets <= kPlaceLdsBuckets)
    hipLaunchKernelGGL(k_peer_scatter<true>, grid, dim3(kPlaceBlock), 0, s, src, m, shift, mask,
                       base, per, P, d);
  else
    hipLaunchKernelGGL(k_peer_scatter<false>, grid, dim3(kPlaceBlock), 0, s, src, m, shift, mask,
                       base, per, P, d);
  return hipGetLastError();
}

hipError_t launch_system_acquire(hipStream_t s) {
  hipLaunchKernelGGL(k_system_acquire, dim3(64), dim3(64), 0, s);
  return hipGetLastError();
}

hipError_t launch_plan(const uint64_t* hist, int P, int nb, int me, int64_t n, int64_t* work,
                       int64_t* total, int64_t* place, int64_t* counts, hipStream_t s,
                       int64_t* gstart, int cshift, int64_t* chunk_counts) {
  if (P < 1 || me < 0 || me >= P || nb < 1 || n < 0) return hipErrorInvalidValue;
  if (cshift < 8 && (nb != 65536 || cshift < 5 || !chunk_counts || P > 64)) return hipErrorInvalidValue;
  const int C = cshift < 8 ? kBuckets >> cshift : 1;
  if (cshift < 8) {
    hipError_t e = hipMemsetAsync(chunk_counts, 0, sizeof(int64_t) * 2 * P * C, s);
    if (e != hipSuccess) return e;
  }
  const int64_t per = (n + P - 1) / P;
  const int64_t lo = (int64_t)me * per;
  int64_t here = n - lo;
  if (here > per) here = per;
  if (here < 0) here = 0;
  const int64_t hi = lo + here;
  hipError_t e = hipMemsetAsync(counts, 0, sizeof(int64_t) * 2 * P, s);
  if (e != hipSuccess) return e;
  const int64_t cells = (int64_t)P * nb;
  hipLaunchKernelGGL(k_plan_cols, dim3((nb + 255) / 256), dim3(256), 0, s, hist, P, nb, work, total);
  hipLaunchKernelGGL(k_plan_base, dim3(1), dim3(kPlanScanBlock), 0, s, total, nb);
  hipLaunchKernelGGL(k_plan_pieces, dim3((unsigned)((cells + 255) / 256)), dim3(256), 0, s, hist, P,
                     nb, me, per, lo, hi, total, work, place,
                     reinterpret_cast<unsigned long long*>(counts), gstart, cshift < 8 ? cshift : 8,
                     cshift < 8 ? reinterpret_cast<unsigned long long*>(chunk_counts) : nullptr);
  hipLaunchKernelGGL(k_plan_rows, dim3(P), dim3(kPlanScanBlock), 0, s, work, nb, counts + P, cshift < 8 ? cshift : 8,
                     cshift < 8 ? chunk_counts + (size_t)P * C : nullptr);
  hipLaunchKernelGGL(k_plan_finish, dim3((unsigned)((cells + 255) / 256)), dim3(256), 0, s, P, nb,
                     lo, work, counts + P, place);
  return hipGetLastError();
}

hipError_t launch_gather_desc(const GatherSrc& g, int64_t m, TileDesc* desc, hipStream_t s) {
  if (m <= 0) return hipSuccess;
  if (!g.R || !g.A || !g.place || !g.gstart || !g.gadj || !desc || g.P < 1 || g.me < 0 || g.me >= g.P ||
      (g.nb != 256 && g.nb != 65536) || (int64_t)g.P * g.nb > (int64_t(1) << 30))
    return hipErrorInvalidValue;
  const int64_t TT = (m + kTile - 1) / kTile;
  const int64_t cells = (int64_t)g.P * g.nb;
  hipLaunchKernelGGL(k_gather_adj, dim3((unsigned)((cells + 255) / 256)), dim3(256), 0, s, g,
                     const_cast<int64_t*>(g.gadj));
  hipLaunchKernelGGL(k_gather_desc, dim3((unsigned)((TT + 255) / 256)), dim3(256), 0, s, g, m, TT, desc);
  return hipGetLastError();
}

hipError_t launch_copy_records(Elem* dst, const Elem* src, int64_t cnt, hipStream_t s) {
  if (cnt <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_copy_records, dim3(grid_for(cnt, 256, 8192)), dim3(256), 0, s, dst, src, cnt);
  return hipGetLastError();
}

hipError_t launch_verify(const Elem* A, int64_t here, int64_t gbase, int64_t n, int64_t per,
                         KeyGen gen, unsigned long long* first_bad, hipStream_t s) {
  if (here <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_verify, dim3(grid_for(here, 256, 8192)), dim3(256), 0, s, A, here, gbase, n,
                     per, gen, first_bad);
  return hipGetLastError();
}

hipError_t launch_check_sorted(const Elem* A, int64_t here, unsigned int* unsorted, hipStream_t s) {
  if (here <= 1) return hipSuccess;
  hipLaunchKernelGGL(k_check_sorted, dim3(grid_for(here, 256, 8192)), dim3(256), 0, s, A, here,
                     unsorted);
  return hipGetLastError();
}

}  // namespace lsb
