// Internal interface between the runtime (lsb_context.cpp, lsb_passes.cpp,
// lsb_exchange.cpp, lsb_wholekey.cpp) and the HIP kernels (lsb_kernels.hip).  Not part of the C ABI (that is include/lsb.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lsb {

// == SortElement (mpi/mpi_lsbsort.cpp:29-32); lsb_elem_t in the ABI.
struct alignas(16) Elem {
  uint64_t key;
  uint64_t val;
};
static_assert(sizeof(Elem) == 16, "16-byte records");

constexpr int kDigitBits = 8;                 // one local pass = one 8-bit digit
constexpr int kBuckets = 1 << kDigitBits;     // 256
#ifndef LSB_SCATTER_BLOCK
#define LSB_SCATTER_BLOCK 256
#define LSB_SCATTER_IPT 16
#endif
constexpr int kScatterBlock = LSB_SCATTER_BLOCK;  // 4 waves
constexpr int kScatterIpt = LSB_SCATTER_IPT;      // items per thread
constexpr int kTile = kScatterBlock * kScatterIpt;  // 4096 elements = 64 KiB in LDS
#ifndef LSB_OS_BLOCK
#define LSB_OS_BLOCK 512
#endif
// k_onesweep workgroups: 8 waves x 8 records for the whole stage (2 per CU),
// 4 waves x 16 for the split stage (3 per CU; at 8 waves its registers spill).
constexpr int kOsBlock = LSB_OS_BLOCK;
constexpr int kOsIpt = kTile / kOsBlock;
#ifndef LSB_OS_SPLIT_BLOCK
#define LSB_OS_SPLIT_BLOCK 256
#endif
constexpr int kOsSplitBlock = LSB_OS_SPLIT_BLOCK;
constexpr int kOsSplitIpt = kTile / kOsSplitBlock;
static_assert(kOsBlock % kBuckets == 0 && kOsBlock * kOsIpt == kTile, "onesweep tile shape");
constexpr int kMaxChunks = 65536;             // upper bound on the chunk grid

// A rank's `m` elements are cut into `num_chunks` contiguous chunks of
// `chunk_elems` (a multiple of kTile; the last may be short).  The count
// (upsweep) and scatter kernels both run one workgroup per chunk, so the
// per-chunk bucket counts of the former are the exact run offsets of the
// latter.
struct Chunking {
  int64_t chunk_elems = 0;
  int num_chunks = 0;
};
Chunking make_chunking(int64_t m, int max_chunks);

// Input distribution of lsb_generate_ex: the key made from the PCG draw.
constexpr int kDistUniform = 0;  // key = draw (the reference's input)
constexpr int kDistZipf = 1;     // key = mix64(Zipf-like rank of the draw), SURVEY §8d C4
struct KeyGen {
  int dist = kDistUniform;
  double zipf_s = 1.1;
  uint64_t zipf_n = 1ull << 30;
};

// On-device PCG64 (pcg-cpp setseq_xsl_rr_128_64):
// A[i] = {make_key(pcg64(seed)[i]), val0 + i}.
hipError_t launch_pcg_fill(Elem* A, int64_t count, uint64_t seed, uint64_t val0, KeyGen gen,
                           hipStream_t s);

// 65536-bin histogram of the 16-bit digit at `shift` of records already
// sorted by that digit (first[] is 65536 int64 scratch).
hipError_t launch_digit16_counts(const Elem* A, int64_t m, int shift, int64_t* first,
                                 uint64_t* counts, hipStream_t s);

// chunk_hist[b * G + c] = number of elements of chunk c whose digit is b.
// span (optional, 2 words, OR-accumulated): span[0] |= OR of the keys,
// span[1] |= OR of their complements.
hipError_t launch_upsweep(const Elem* A, int64_t m, int shift, Chunking ch,
                          uint32_t* chunk_hist, uint64_t* span, hipStream_t s);

// chunk_off[b * G + c] = sum_{c' < c} chunk_hist[b * G + c'];  totals[b] = row sum.
hipError_t launch_scan(const uint32_t* chunk_hist, int G, uint64_t* chunk_off,
                       uint64_t* totals, hipStream_t s);

// Stable counting-sort scatter of one digit: out[pos] with
// pos = bucket_start[b] + chunk_off[b][c] + rank of the element among the
// chunk's digit-b elements (localShuffle, mpi/mpi_lsbsort.cpp:240-246).
// first16 (optional; the high byte of a 16-bit digit whose low byte the input
// is sorted by): atomicMin of candidate start positions of every 16-bit digit
// at shift - 8; reset it with launch_starts_reset, then launch_starts_to_counts.
hipError_t launch_scatter(const Elem* in, Elem* out, int64_t m, int shift, Chunking ch,
                          const uint64_t* chunk_off, const uint64_t* totals, int64_t* first16,
                          hipStream_t s);
hipError_t launch_starts_reset(int64_t* first16, hipStream_t s);
// counts[d] of a rank whose m records are sorted by the 16-bit digit, from the
// first index of every present digit (first[d] < 0 or >= m: absent).
hipError_t launch_starts_to_counts(const int64_t* first16, int64_t m, uint64_t* counts,
                                   hipStream_t s);

// Single-read passes (P == 1; k_onesweep in lsb_kernels.hip).  The m records
// are kTile-record tiles in kOnesweepSubs contiguous sub-arrays, sub-array x
// = tiles [x*TT/8, (x+1)*TT/8).  sub_hist[x * 256 + b] = count of digit b
// in sub-array x.
constexpr int kOnesweepSubs = 8;
// Look-back values are 30 bits (a bucket's count within one sub-array of
// m / 8 + kTile records): m < 2^33 - 2^16, i.e. 137 GB per record buffer.
constexpr int64_t kOnesweepMaxElems = (int64_t(1) << 33) - (int64_t(1) << 16);
inline int64_t onesweep_tiles(int64_t m) { return (m + kTile - 1) / kTile; }
// sub_hist (zeroed here) of the digit at `shift`; span as for launch_upsweep.
hipError_t launch_subhist(const Elem* A, int64_t m, int shift, int grid, uint32_t* sub_hist,
                          uint64_t* span, hipStream_t s);
// One stable pass in -> out on the digit at `shift`, offsets from sub_hist
// plus a look-back over status (onesweep_tiles(m) * 256 u32 granules, zeroed
// once at allocation; epoch >= 1, new for every launch over the same m, and
// the first launch after a zeroing odd: a granule's tag is the epoch's
// parity, so every launch must write every row).  next_shift >= 0: also
// next_hist (zeroed here) = sub_hist of the digit at next_shift over out.
// tile_ctr: kOnesweepSubs words of scratch; *err |= 1 if a look-back gave up.
// -DLSB_OS_PROFILE builds: summed s_memtime ticks of k_onesweep's phases
// (dequeue, load + rank, look-back + scan, stage, write, unused) over all
// workgroups' thread 0; hipErrorNotSupported otherwise.
hipError_t onesweep_profile(unsigned long long* out10, bool reset);
// What a pass also hands the exchange that follows it (per-digit exchange
// forms, P > 1): totals[b] = the pass's 256 digit counts; count16 (zeroed
// here) = the 65536 counts of the 16-bit digit at shift - 8, for the high
// byte of a 16-bit exchange digit whose input is sorted by the low byte.
// The hybrid's last byte pass (LSB_OPT_HYBRID, lsb_segsort.hip): the pass
// also orders every segment (records equal on pmask, the k top varying
// bytes) inside its tile by the whole key, so no separate k_segsort pass is
// needed.  A segment lies inside one run of records equal on rmask (pmask
// without this pass's byte), and the pass's input is sorted by rmask; only
// runs that cross a tile boundary can leave a segment split between two
// tiles, and launch_segfix merges those from the pass's input, its look-back
// rows and base (workgroup 0 writes base[x * 256 + b] = the first output slot
// of bucket b's sub-array x records).  *err |= 1 (launch_segfix) when a
// crossing run holds more than kSegCap records (4 * kSegCap when runs
// average over 64 records) on one side of its boundary or spans a whole
// tile: that boundary is left alone, the output is still a permutation sorted
// by pmask, and the runtime runs k_segsort on it.  *err |= 2 (this pass)
// when a segment inside a tile holds more than kSegMax records: its records'
// slots came from walks cut at kSegMax and may collide, so the output is not
// a permutation, and the runtime sorts the kept input with the LSD passes
// (stress seed 19: k_segsort over such an output, its holes holding stale
// records that split the long segments, found nothing too long and kept a
// wrong result).
constexpr int kSegCap = 256;
struct SegPass {
  uint64_t pmask = 0;
  uint64_t rmask = 0;
  int64_t* base = nullptr;  // kOnesweepSubs * 256
  uint32_t* err = nullptr;
};
// Gathered input (per-digit exchange, LSB_OPT_EXCHANGE_GATHER): the pass
// after an exchange reads its records where they arrived instead of from a
// placed copy.  Position p of the placed order (the rank's block in
// (digit, source) order) lies in piece e = b * P + s (bucket b's records from
// source s), the last e with gstart[e] <= p; its record is
//   R[p - place[s * nb + b]]                          (a peer's piece)
//   A[p - place[s * nb + b] + self_adj[chunk of b]]   (s == me, self_in_a)
// (chunk of b: (b & 255) >> chunk_shift; the per-digit exchange in chunks,
// launch_count16_chunks, keeps the rank's own records in C chunk ranges of A;
// unchunked, chunk_shift = 8: one chunk.)
// TileDesc caches that per onesweep tile: up to 4 pieces (first position
// relative to the tile, pointer adjustment, bit j of sel: piece j is in A);
// n = kDescOverflow sends the tile's records to the search over [e0, e1].
constexpr int kDescPieces = 4;
constexpr int kDescOverflow = 0xFF;
struct alignas(16) TileDesc {
  int32_t n, e0, e1, sel;
  int32_t start[kDescPieces];
  int64_t adj[kDescPieces];
};
constexpr int kMaxExchangeChunks = 8;
struct GatherSrc {
  const Elem* R = nullptr;
  const Elem* A = nullptr;
  int64_t self_adj[kMaxExchangeChunks] = {};
  int chunk_shift = 8;
  const int64_t* place = nullptr;  // P * nb place_off (launch_plan)
  const int64_t* gstart = nullptr;  // P * nb piece starts (launch_plan)
  const int64_t* gadj = nullptr;    // P * nb scratch: 2 * pointer adjustment + (1: in A)
  const TileDesc* desc = nullptr;   // onesweep_tiles(m)
  int P = 1, nb = 256, me = 0, self_in_a = 1;
  int64_t a_len = 0, r_len = 0;     // records in A and R (debug builds check every gathered read)
};
// gadj, then desc[t] for every onesweep tile of m records (after launch_plan
// with gstart).
hipError_t launch_gather_desc(const GatherSrc& g, int64_t m, TileDesc* desc, hipStream_t s);
// The per-digit exchange in chunks (LSB_OPT_EXCHANGE_CHUNKS, 16-bit digits;
// DESIGN.md §6): after the low-byte pass of digit d, B (m records) is sorted
// by the low byte l; chunk k = the records with l in [k << cshift,
// (k + 1) << cshift), a contiguous range of B (C = 256 >> cshift chunks).  One
// read of B gives count16[(h << 8) | l] (zeroed here: the digit's 65536
// counts, for the exchange plan) and chunk_hist[(k * 8 + x) * 256 + h]
// (zeroed here: the high byte's sub-array histogram over chunk k's own tiles,
// the sub_hist of chunk k's high-byte pass), so the plan and the sends can
// precede the high-byte pass, which then runs chunk by chunk while the
// previous chunk is on the wire.  lo_hist: the low byte's sub-array
// histogram (its totals give the chunk bounds).  shift16 = 16 * d.
hipError_t launch_count16_chunks(const Elem* B, int64_t m, int shift16, const uint32_t* lo_hist, int cshift,
                                 int grid, uint64_t* count16, uint32_t* chunk_hist, hipStream_t s);
// Regional first pass (P == 1 LSD sorts of at least kRegionMin records,
// LSB_OPT_REGION_FIRST): the sort's first pass needs no
// histogram read.  Its records of digit b from sub-array x go to region
// r = b * kOnesweepSubs + x of the output, a slot range of `cap` records
// (a multiple of kTile, with slack over the mean region_mean(m)): slot
// r * cap + (the record's rank among them, from the look-back alone).  The
// output then holds the records in the stable order of that digit, with a
// gap at the end of every region, and the second pass reads it tile by tile,
// taking counts[r] records of each region (its tiles of kTile slots:
// the valid prefix of each).  A region that would overflow sets *ovf (the
// output is invalid and the runtime sorts the kept input the usual way).
// Mode 1 (the first pass, next digit counted over the regional layout's
// tiles): counts[r] accumulated here (zeroed by the launcher).  Mode 2 (the
// second pass): reads that layout, writes a dense one.  No key span: the
// runtime takes the form only when a sample shows every byte varying.
constexpr int64_t kRegionMin = int64_t(1) << 27;
constexpr int kRegions = kBuckets * kOnesweepSubs;  // 2048
inline int64_t region_mean(int64_t m) { return (m + kRegions - 1) / kRegions; }
// Slots per region for m records (0: fewer than min_m records, too few for
// the form): the mean plus max(mean / 64, 6 standard deviations of a uniform
// region's count), rounded up to whole tiles.  2^27 records: +6.25 % slots;
// 2^30: +1.6 % (130 tiles per region).  (Tests lower min_m to cover small
// sorts, whose regions are then one mostly empty tile each.)  The two
// constants are build knobs for experiments (tools/r05/region_slack.sh).
#ifndef LSB_REGION_SIGMA
#define LSB_REGION_SIGMA 6
#endif
#ifndef LSB_REGION_DIV
#define LSB_REGION_DIV 64
#endif
inline int64_t region_cap(int64_t m, int64_t min_m = kRegionMin) {
  if (m < min_m || m <= 0) return 0;
  const int64_t mu = region_mean(m);
  int64_t sd = 1;
  while (sd * sd < mu) ++sd;
  const int64_t a = mu / LSB_REGION_DIV, b = LSB_REGION_SIGMA * sd;
  const int64_t slack = a > b ? a : b;
  return (mu + slack + kTile - 1) / kTile * kTile;
}
// Region r's first slot.  LSB_REGION_STAGGER (experiment): regions one tile
// apart more than `cap`, each shifted by (37 r mod 16) x 256 records, so that
// the first pass's 2048 write frontiers do not sit at one stride.
#ifndef LSB_REGION_STAGGER
#define LSB_REGION_STAGGER 0
#endif
__host__ __device__ inline int64_t region_stride(int64_t cap) { return cap + (LSB_REGION_STAGGER ? kTile : 0); }
__host__ __device__ inline int64_t region_base(int64_t r, int64_t cap) {
  return r * region_stride(cap) + (LSB_REGION_STAGGER ? ((r * 37) & 15) * 256 : 0);
}
// Records a buffer holding the regional layout needs.
inline int64_t region_slots(int64_t m, int64_t min_m = kRegionMin) {
  return region_stride(region_cap(m, min_m)) * kRegions;
}
struct RegionPass {
  int64_t cap = 0;                    // slots per region
  uint32_t* counts = nullptr;         // [kRegions] records per region
  uint32_t* ovf = nullptr;            // mode 1: set when a region overflows
};
// Sample of the sort's first digit (the regional first pass's go / no-go):
// 256 workgroups read one tile each, spread over the m records; hist[256]
// (zeroed here) gets the tiles' digit counts at `shift`, span[2] (zeroed
// here) the OR of their keys and complements.
hipError_t launch_sample(const Elem* A, int64_t m, int shift, uint32_t* hist, uint64_t* span,
                         hipStream_t s);
struct OnesweepExtra {
  uint64_t* totals = nullptr;
  uint64_t* count16 = nullptr;
  int halves = 1;  // 2: split stage, 3 workgroups per CU (skewed keys; not with count16)
  const SegPass* seg = nullptr;  // the hybrid's last pass (no next digit, whole stage)
  const GatherSrc* gather = nullptr;  // records gathered from an exchange (`in` unused)
  bool probe = false;  // the placement probe's pass (a last pass, launched as k_onesweep_probe)
  const RegionPass* region = nullptr;  // with region_mode 1 or 2: the regional layout
  int region_mode = 0;  // 1: write it (needs a next digit); 2: read it (sub_hist over its tiles)
};
// The runtime's choice of OnesweepExtra::halves for a rank, from a digit's
// sub-array histogram (kOnesweepSubs x 256 counts of m records): 2 when one
// bucket holds more than 1/32 of the records.
int onesweep_halves_for(const uint32_t* sub_hist_host, int64_t m);
hipError_t launch_onesweep(const Elem* in, Elem* out, int64_t m, int shift, int next_shift,
                           const uint32_t* sub_hist, uint32_t* next_hist, uint32_t* status,
                           uint32_t* tile_ctr, uint32_t epoch, uint32_t* err, int grid,
                           hipStream_t s, OnesweepExtra extra = OnesweepExtra());

// Hybrid local sort (LSB_OPT_HYBRID, lsb_segsort.hip): `in` is stably sorted
// by the bits of pmask (the top varying bytes of the key); k_segsort sorts
// every segment (maximal run of equal key & pmask) stably by the whole key,
// in -> out.  A segment longer than kSegMax records sets *err (output
// invalid: the runtime sorts the kept input by the LSD passes instead).
// grid: persistent workgroups (3 per CU).
// 64: past ~32 records per segment the walks cost more than the LSD passes
// the hybrid saves (64 per segment: k_segsort 69 ms against 7 for a byte
// pass), and each walk is bounded by kSegMax each way, so
// duplicate-heavy keys that do not look skewed (e.g. 2^20 distinct keys,
// ~1000 copies each, at 2^30 records) cost the hybrid at most a few ms of
// walks before the sort redoes the kept input by the LSD passes (advisor
// r03).  Uniform keys at the runtime's k hold ~0.25-2 records per segment
// (the longest of 2^33 records: ~17).
constexpr int kSegMax = 64;
hipError_t launch_segsort(const Elem* in, Elem* out, int64_t m, uint64_t pmask, uint32_t* err,
                          int grid, hipStream_t s);
// After a SegPass launch in -> out over m records on the byte at `shift`
// (status: that launch's look-back rows): merge every segment split between
// tiles t and t + 1, in place in `out`.
hipError_t launch_segfix(const Elem* in, Elem* out, int64_t m, int shift, const uint32_t* status,
                         const SegPass& seg, int grid, hipStream_t s);

// Receiver-side placement of one source's received range: src[i] (receive
// index k0 + i) goes to out[off_row[digit] + k0 + i], off_row = the source's
// row of the placement table (place_off[s * nbuckets ...]); out holds
// out_len records (the receive order [k0, k0 + count) lies inside it).
// next_shift >= 0: also add the placed records' digit at next_shift to
// next_hist[x * 256 + b] (x = the out position's onesweep sub-array over
// out_len records; zeroed by the caller): the next local pass's sub_hist.
// store = false (with next_shift >= 0): count only, out untouched (the next
// pass gathers, GatherSrc).  skew: the sort's keys are skewed (its stage
// split): the count adds once per run of equal counters.
hipError_t launch_place(const Elem* src, Elem* out, int64_t out_len, int64_t k0, int64_t count,
                        int shift, int nbuckets, const int64_t* off_row, hipStream_t s,
                        int next_shift = -1, uint32_t* next_hist = nullptr, bool store = true,
                        bool skew = false);

// Peer-store exchange (opt-in, LSB_OPT_EXCHANGE_PEER): from the all-gathered
// counts hist[s * nb + b], rank `me` writes each of its m bucket-ordered
// records straight into its owner's receiving buffer: record i of bucket b
// goes to global position g = base[b] + i, i.e. dst[g / per][g % per].
// dst[q] is rank q's buffer as this process sees it; base: nb int64 scratch.
// Each workgroup ends with a system-scope release; launch_system_acquire is
// the owner's matching acquire (every XCD's L2) after the barrier collective.
hipError_t launch_peer_exchange(const Elem* src, int64_t m, int shift, int nbuckets,
                                const uint64_t* hist, int P, int me, int64_t per,
                                Elem* const* dst, int64_t* base, hipStream_t s);
hipError_t launch_system_acquire(hipStream_t s);

// Exchange plan of rank `me` on device from the all-gathered counts
// hist[s * nb + b] (same rule as the host planner lsb_plan_exchange):
// place[s * nb + b] = place_off, place[P * nb + s] = rend (inclusive scan of
// recv counts), counts[0..P) = send counts, counts[P..2P) = recv counts.
// work: P * nb int64, total: nb int64 scratch.  gstart (optional, P * nb):
// gstart[b * P + s] = first position of piece (b, s) in my block, clamped to
// [0, here] (nondecreasing in b * P + s).  cshift < 8 (the chunked exchange,
// nb = 65536, C = 256 >> cshift chunks of the low byte): a source's pieces
// lie in R in chunk order (chunk of l, h, l) instead of digit order, which
// place_off follows, and chunk_counts[q * C + k] = my records of chunk k for
// owner q, chunk_counts[P * C + s * C + k] = source s's records of chunk k
// for me.
hipError_t launch_plan(const uint64_t* hist, int P, int nb, int me, int64_t n, int64_t* work,
                       int64_t* total, int64_t* place, int64_t* counts, hipStream_t s,
                       int64_t* gstart = nullptr, int cshift = 8, int64_t* chunk_counts = nullptr);

// ---- whole-key exchange (radix_bits = 64; lsb_merge.hip) ----
// Splitter search: for Q targets T_t, state[2t .. 2t+1] = key interval
// [lo, hi] holding the key found at global position T_t.  One round:
// launch_split_cands (cnt[t * kSplitCands + j] = this rank's count of keys
// below candidate j), all-gather cnt over the P ranks, launch_split_update.
// kSplitRounds rounds leave lo == hi; launch_split_final then writes this
// rank's {#keys < k*, #keys <= k*} per target.  A is sorted by key.
constexpr int kSplitCands = 256;
constexpr int kSplitRounds = 8;
constexpr int kMergeMaxCuts = 512;  // P * slices cap of the whole-key exchange
hipError_t launch_split_init(uint64_t* state, int Q, hipStream_t s);
hipError_t launch_split_cands(const Elem* A, int64_t m, const uint64_t* state, int Q, uint64_t* cnt,
                              hipStream_t s);
hipError_t launch_split_update(const uint64_t* gathered, int P, int Q, const int64_t* targets,
                               uint64_t* state, hipStream_t s);
hipError_t launch_split_final(const Elem* A, int64_t m, const uint64_t* state, int Q, uint64_t* out,
                              hipStream_t s);
// One level of a merge tree: npairs stable merges of two key-sorted runs (a
// before b on equal keys; nb = 0 copies a) into out (na + nb records,
// disjoint from a and b).  tile0[p] = first tile of pair p in the level's
// tile numbering (tiles of kMergeTile outputs), tiles = their total.
// path: tiles + npairs int64 scratch; grid: persistent workgroups (3 per CU).
constexpr int kMergeTile = 2048;
constexpr int kMergeMaxPairs = 32;
struct MergePair {
  const Elem* a;
  const Elem* b;
  Elem* out;
  int64_t na, nb, tile0;
};
struct MergeLevel {
  MergePair p[kMergeMaxPairs];
  int npairs;
  int64_t tiles;
};
inline int64_t merge_tiles(int64_t n) { return (n + kMergeTile - 1) / kMergeTile; }
hipError_t launch_merge_level(const MergeLevel& level, int64_t* path, int grid, hipStream_t s);

// O(n) bit-exact stable-sort check of a rank's here-part (see lsb_verify).
// first_bad must hold UINT64_MAX before the launch; receives min bad global index.
// cnt records src -> dst on one device (loopback exchange copies).
hipError_t launch_copy_records(Elem* dst, const Elem* src, int64_t cnt, hipStream_t s);
hipError_t launch_verify(const Elem* A, int64_t here, int64_t gbase, int64_t n, int64_t per,
                         KeyGen gen, unsigned long long* first_bad, hipStream_t s);

// Key-only local sortedness (checkSorted); *unsorted set to 1 on a descent.
hipError_t launch_check_sorted(const Elem* A, int64_t here, unsigned int* unsorted, hipStream_t s);

}  // namespace lsb
