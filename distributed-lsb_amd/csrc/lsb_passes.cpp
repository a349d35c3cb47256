// The local pass driver (mySort's localShuffle, mpi/mpi_lsbsort.cpp:213-247,
// and the pass loop of :580-585 when nothing is exchanged):
//   * reduce-then-scan passes (k_upsweep + k_scan + k_scatter; lsb_pass and
//     LSB_OPT_ONESWEEP = 0), and the digit loop do_pass that follows each
//     exchange digit's local passes with its exchange (lsb_exchange.cpp);
//   * single-read passes: one k_subhist read per sort, then one k_onesweep
//     per varying byte (decoupled look-back), histograms carried from pass to
//     pass;
//   * the hybrid local sort (LSB_OPT_HYBRID): k_onesweep on the top varying
//     bytes, segments ordered by k_segfix / k_segsort (lsb_segsort.hip).
#include "lsb_rt.h"

#include <cmath>

#include <deque>

namespace lsb_rt {

// ---- one local stable 8-bit pass A -> B, then swap (localShuffle) -------
// want_span: also reduce the key span (lsb_sort's first pass).  starts16:
// this is the high byte of a 16-bit exchange digit; the scatter also marks
// the digit's run starts, so digit_counts needs no extra read.
int local_pass(lsb_ctx* c, Rank& r, int shift, bool want_span, bool starts16) {
  HIP_TRY(hipSetDevice(r.dev));
  r.starts_fused = starts16;
  if (r.here == 0) {
    HIP_TRY(hipMemsetAsync(r.totals, 0, sizeof(uint64_t) * lsb::kBuckets, r.stream));
    return LSB_OK;
  }
  if (starts16) HIP_TRY(lsb::launch_starts_reset(r.first16, r.stream));
  const lsb::Chunking& ch = r.chunking;
  {
    Timer t(c, &r, LSB_K_UPSWEEP);
    HIP_TRY(lsb::launch_upsweep(r.A, r.here, shift, ch, r.chunk_hist,
                                want_span ? r.span : nullptr, r.stream));
  }
  {
    Timer t(c, &r, LSB_K_SCAN);
    HIP_TRY(lsb::launch_scan(r.chunk_hist, ch.num_chunks, r.chunk_off, r.totals, r.stream));
  }
  {
    Timer t(c, &r, LSB_K_SCATTER);
    HIP_TRY(lsb::launch_scatter(r.A, r.B, r.here, shift, ch, r.chunk_off, r.totals,
                                starts16 ? r.first16 : nullptr, r.stream));
    count_pass_elems(c, r.here);
  }
  std::swap(r.A, r.B);
  return LSB_OK;
}

// One exchange digit: its 8-bit local sub-passes, then (P > 1) the exchange.
// varying: key bits that differ somewhere; a sub-pass whose byte is constant
// is the identity and is skipped (all ~0 = run everything).  want_span: the
// first sub-pass also reduces the key span (lsb_sort, digit 0).

int do_pass(lsb_ctx* c, int digit, uint64_t varying, bool want_span) {
  if (c->bits == 64 && exchanging(c)) return merge_sort(c);  // the one 64-bit digit
  for (Rank& r : c->ranks) r.starts_fused = false;
  const int subs = c->bits / lsb::kDigitBits;
  for (int sub = 0; sub < subs; ++sub) {
    const int shift = digit * c->bits + sub * lsb::kDigitBits;
    if (!want_span && ((varying >> shift) & (lsb::kBuckets - 1)) == 0) continue;
    // The high byte of a 16-bit exchange digit also marks the digit's starts.
    const bool starts16 = exchanging(c) && subs == 2 && sub == 1;
    begin_pass(c, shift);
    for (Rank& r : c->ranks) LSB_TRY(local_pass(c, r, shift, want_span && sub == 0, starts16));
    ++c->last_local_passes;
  }
  if (!exchanging(c)) return LSB_OK;
  ++c->last_exchanges;
  return exchange_digit(c, digit);
}

// ---- single-read passes (P == 1) ------------------------------------------
bool onesweep_applies(const lsb_ctx* c) {
  return c->onesweep && !exchanging(c) && c->ranks.size() == 1 && c->ranks[0].here > 0 &&
         c->ranks[0].here <= lsb::kOnesweepMaxElems;
}

// The regional first pass's rg_buf words (region_sample, region_first): [kRgCounts, +2048) region counts, [kRgHist, +256) the
// sample's digit counts, kRgOvf the overflow word, [kRgSpan, +4) the
// sample's span (2 u64).
constexpr int kRgCounts = 0, kRgHist = lsb::kRegions, kRgOvf = kRgHist + lsb::kBuckets,
              kRgSpan = kRgOvf + 2, kRgWords = kRgSpan + 4;

int onesweep_ensure(Rank& r) {
  if (r.os_status) return LSB_OK;
  const size_t tiles = (size_t)lsb::onesweep_tiles(r.here);
  LSB_TRY(dev_alloc(&r.os_status, tiles * lsb::kBuckets));
  LSB_TRY(dev_alloc(&r.os_hist, 2 * lsb::kOnesweepSubs * lsb::kBuckets));
  LSB_TRY(dev_alloc(&r.os_ctr, 2 * lsb::kOnesweepSubs));
  LSB_TRY(host_alloc(&r.os_err_h, 2));  // [0] look-back gave up, [1] k_segsort error
  r.os_err_h[0] = r.os_err_h[1] = 0;
  LSB_TRY(host_alloc(&r.os_hist_h, (size_t)lsb::kOnesweepSubs * lsb::kBuckets));
  HIP_TRY(hipMemsetAsync(r.os_status, 0, tiles * lsb::kBuckets * sizeof(uint32_t), r.stream));
  HIP_TRY(hipMemsetAsync(r.os_ctr, 0, 2 * lsb::kOnesweepSubs * sizeof(uint32_t), r.stream));
  r.os_epoch = 0;
  r.os_grid = max_chunks_for_device(r.dev);
  if (r.rg_cap > 0) {  // the regional first pass's buffers (region_ensure)
    const size_t rows = (size_t)lsb::onesweep_tiles(r.rg_cap * lsb::kRegions) * lsb::kBuckets;
    LSB_TRY(dev_alloc(&r.rg_buf, (size_t)kRgWords));
    LSB_TRY(host_alloc(&r.rg_h, (size_t)kRgWords));
    LSB_TRY(dev_alloc(&r.os_status2, rows));
    HIP_TRY(hipMemsetAsync(r.os_status2, 0, rows * sizeof(uint32_t), r.stream));
    r.os_epoch2 = 0;
  }
  return LSB_OK;
}

// One k_onesweep launch of rank r, r.A -> r.B on the byte at `shift` (then
// the buffers swap), under a fresh look-back epoch.  Granules carry the
// epoch's parity, and every launch rewrites every row, so only the
// alternation matters (the counter runs on for the record).  The epoch
// advances only once the launch is queued: a launch that fails before its
// kernel runs writes no rows, and a later launch would then accept rows of
// two launches back as current.  So a failure marks the rows dirty; the next
// launch zeroes them first and restarts the epochs (the first is odd).
// The pass that reads the regional layout (region_mode 2) has more tiles
// than the others and keeps its rows on a track of its own (os_status2,
// os_epoch2).
void zero_status(Rank& r) {
  (void)hipMemsetAsync(r.os_status, 0, (size_t)lsb::onesweep_tiles(r.here) * lsb::kBuckets * sizeof(uint32_t),
                       r.stream);
  if (r.os_status2)
    (void)hipMemsetAsync(r.os_status2, 0,
                         (size_t)lsb::onesweep_tiles(r.rg_cap * lsb::kRegions) * lsb::kBuckets * sizeof(uint32_t),
                         r.stream);
  r.os_epoch = 0;
  r.os_epoch2 = 0;
}

int onesweep_launch(lsb_ctx* c, Rank& r, int shift, int next, const uint32_t* hist,
                    uint32_t* next_hist, lsb::OnesweepExtra x) {
  if (r.os_dirty) {
    zero_status(r);
    HIP_TRY(hipGetLastError());
    r.os_dirty = false;
  }
  const bool track2 = x.region_mode == 2;
  uint32_t* status = track2 ? r.os_status2 : r.os_status;
  uint32_t& last_epoch = track2 ? r.os_epoch2 : r.os_epoch;
  if (!status) return fail(LSB_ERR_INVALID, "onesweep_launch", "regional layout's look-back rows");
  uint32_t epoch = last_epoch + 1;
  if (epoch >= (1u << 30)) epoch = 2;  // 2^30 is even: keep the alternation
  hipError_t e;
  if (c->fail_onesweep > 0 && --c->fail_onesweep == 0) {  // LSB_OPT_FAIL_ONESWEEP (tests)
    r.os_dirty = true;
    return fail(LSB_ERR_HIP, "launch_onesweep", "injected launch failure (LSB_OPT_FAIL_ONESWEEP)");
  }
  {
    Timer t(c, &r, LSB_K_SCATTER);
    e = lsb::launch_onesweep(r.A, r.B, r.here, shift, next, hist, next_hist, status, r.os_ctr,
                             epoch, r.os_ctr + lsb::kOnesweepSubs, r.os_grid, r.stream, x);
  }
  if (e != hipSuccess) {
    (void)hipGetLastError();
    r.os_dirty = true;
    return fail(LSB_ERR_HIP, "launch_onesweep", hipGetErrorString(e));
  }
  last_epoch = epoch;
  count_pass_elems(c, r.here);
  std::swap(r.A, r.B);
  return LSB_OK;
}

// This sort's k_onesweep stage split for rank r (LSB_OPT_ONESWEEP_SPLIT).
// Auto decides from the first digit's sub-array histogram (`hist`, on
// r.stream): queue_halves queues its 8 KiB read-back, to share the span's
// stream sync; choose_halves decides after that sync.
int queue_halves(lsb_ctx* c, Rank& r, const uint32_t* hist) {
  if (c->os_split != 0 || r.here == 0) return LSB_OK;
  HIP_TRY(hipMemcpyAsync(r.os_hist_h, hist, sizeof(uint32_t) * lsb::kOnesweepSubs * lsb::kBuckets,
                         hipMemcpyDeviceToHost, r.stream));
  return LSB_OK;
}

int choose_halves(lsb_ctx* c, Rank& r, bool synced) {
  if (c->os_split != 0 || r.here == 0) {
    r.os_halves = c->os_split == 2 ? 2 : 1;
    return LSB_OK;
  }
  if (!synced) HIP_TRY(hipStreamSynchronize(r.stream));
  r.os_halves = lsb::onesweep_halves_for(r.os_hist_h, r.here);
  return LSB_OK;
}

// k_subhist of the byte `byte` of rank r's A into os_hist[0] (the sub-array
// histogram the first pass reads), with the key span when `span`.
int count_byte(lsb_ctx* c, Rank& r, int byte, bool span) {
  Timer t(c, &r, LSB_K_UPSWEEP);
  HIP_TRY(lsb::launch_subhist(r.A, r.here, byte * lsb::kDigitBits, r.os_grid, r.os_hist,
                              span ? r.span : nullptr, r.stream));
  return LSB_OK;
}

// The bytes of `varying` (ascending): the digits a sort must run.
std::vector<int> varying_bytes(uint64_t varying) {
  std::vector<int> d;
  for (int b = 0; b < 64 / lsb::kDigitBits; ++b)
    if (((varying >> (b * lsb::kDigitBits)) & (lsb::kBuckets - 1)) != 0) d.push_back(b);
  return d;
}

// One k_onesweep pass per byte of `digits` (ascending), r.A -> r.B ->
// ..., each also counting the next byte over its output; os_hist[0] holds
// the sub-array histogram of digits[0] over r.A.
// From digits[from] on; rp: digits[from]'s pass reads the regional layout
// (its input's histogram in os_hist[from & 1]).
// *disarm (when given) turns false once pass `from` is queued.
int onesweep_digits(lsb_ctx* c, Rank& r, const std::vector<int>& digits, int* passes, size_t from = 0,
                    const lsb::RegionPass* rp = nullptr, bool* disarm = nullptr) {
  uint32_t* hist[2] = {r.os_hist, r.os_hist + lsb::kOnesweepSubs * lsb::kBuckets};
  for (size_t i = from; i < digits.size(); ++i) {
    const int shift = digits[i] * lsb::kDigitBits;
    const int next = i + 1 < digits.size() ? digits[i + 1] * lsb::kDigitBits : -1;
    begin_pass(c, shift);
    lsb::OnesweepExtra x;
    x.halves = r.os_halves;
    if (rp && i == from) {
      x.region = rp;
      x.region_mode = 2;
    }
    LSB_TRY(onesweep_launch(c, r, shift, next, hist[i & 1], hist[(i + 1) & 1], x));
    ++*passes;
    if (disarm) *disarm = false;
  }
  return LSB_OK;
}

// ---- the regional first pass (LSB_OPT_REGION_FIRST) ------------
// A P == 1 LSD sort's first pass takes no histogram read (k_subhist, 16 B per
// record): k_onesweep writes digit 0's records into 2048 regions of slots
// (digit b, sub-array x), each as long as a uniform region could need with
// ample slack, so their offsets come from the look-back alone; the second
// pass reads that layout region by region (its valid prefix per tile) and
// writes the dense one.  The first pass also counts the regions and digit 1
// over the layout's tiles.  A sample of 2^20 records decides beforehand:
// every byte of the sampled keys must vary (then every digit varies, and no
// key span is needed: all passes run) and no bucket of digit 0 may hold over
// 1.1 / 256 of the sample (6 standard deviations over the mean in small
// samples); skewed or structured keys take the usual start,
// k_subhist's read with the exact span.  A region that still overflows sets
// a word the host reads after the first pass, and the sort then starts over
// from the input, which the first pass left in place.

// The hybrid's passes may start with it too (its first pass on the lowest of
// its top bytes; region_first's shift).
bool region_applies(const lsb_ctx* c, const Rank& r) {
  return c->region && !exchanging(c) && c->onesweep && c->os_split == 0 && r.rg_cap > 0 &&
         r.here == c->per && r.cap >= lsb::region_stride(r.rg_cap) * lsb::kRegions &&
         r.here <= lsb::kOnesweepMaxElems;
}

lsb::RegionPass region_pass(Rank& r) {
  lsb::RegionPass rp;
  rp.cap = r.rg_cap;
  rp.counts = r.rg_buf + kRgCounts;
  rp.ovf = r.rg_buf + kRgOvf;
  return rp;
}

// The sample (filed as the sort's count) of the byte the first pass sorts
// on: *go = take the regional pass; *seen = the key bits that vary in it.
int region_sample(lsb_ctx* c, Rank& r, int byte, bool* go, uint64_t* seen) {
  *go = false;
  if (!r.os_status2) return LSB_OK;  // allocated by onesweep_ensure
  {
    Timer t(c, &r, LSB_K_UPSWEEP);
    HIP_TRY(lsb::launch_sample(r.A, r.here, byte * lsb::kDigitBits, r.rg_buf + kRgHist,
                               reinterpret_cast<uint64_t*>(r.rg_buf + kRgSpan), r.stream));
  }
  HIP_TRY(hipMemcpyAsync(r.rg_h + kRgHist, r.rg_buf + kRgHist, (size_t)(kRgWords - kRgHist) * sizeof(uint32_t),
                         hipMemcpyDeviceToHost, r.stream));
  HIP_TRY(hipStreamSynchronize(r.stream));
  uint64_t S = 0, top = 0;
  for (int b = 0; b < lsb::kBuckets; ++b) {
    S += r.rg_h[kRgHist + b];
    top = std::max<uint64_t>(top, r.rg_h[kRgHist + b]);
  }
  uint64_t sp[2];
  memcpy(sp, r.rg_h + kRgSpan, sizeof sp);
  *seen = sp[0] & sp[1];
  bool every_byte = true;
  for (int b = 0; b < 64 / lsb::kDigitBits; ++b)
    every_byte = every_byte && ((*seen >> (b * lsb::kDigitBits)) & (lsb::kBuckets - 1)) != 0;
  // No bucket over the mean by more than max(10 %, 6 standard deviations of
  // a uniform bucket's count in a sample this size), nor by more than the
  // regions' own slack (region_cap over the uniform mean: +1.6 % at 2^30)
  // plus 4 standard deviations: at 2^30 a bucket 8-10 % over the mean would
  // pass the first bound and overflow its regions for certain (advisor r05).
  // Below ~5 % the sample cannot tell such a bucket from noise; the overflow
  // word catches it.
  const double mean = (double)S / lsb::kBuckets, sd = std::sqrt(mean);
  const double slack = (double)r.rg_cap / (double)lsb::region_mean(r.here);
  const double gate = std::min(mean + std::max(0.1 * mean, 6.0 * sd), mean * slack + 4.0 * sd);
  *go = every_byte && S > 0 && (double)top <= gate;
  return LSB_OK;
}

// The first pass into the regional layout (r.A -> r.B, then they swap) on
// the byte at `shift`, counting the byte at next_shift into os_hist[1]; the
// overflow word's read-back is queued.
int region_first(lsb_ctx* c, Rank& r, int shift, int next_shift, int* passes) {
  const lsb::RegionPass rp = region_pass(r);
  begin_pass(c, shift);
  lsb::OnesweepExtra x;
  x.region = &rp;
  x.region_mode = 1;
  LSB_TRY(onesweep_launch(c, r, shift, next_shift, nullptr, r.os_hist + lsb::kOnesweepSubs * lsb::kBuckets, x));
  ++*passes;
  HIP_TRY(hipMemcpyAsync(r.rg_h + kRgOvf, r.rg_buf + kRgOvf, sizeof(uint32_t), hipMemcpyDeviceToHost, r.stream));
  return LSB_OK;
}

// ---- a rank's local sort, in three steps -----------------------------------
// LocalSort is one rank's local sort as begin() (queue the first count read
// and its read-backs), queue() (wait for those, queue the passes) and
// finish() (the hybrid: read its error word; rarely, sort again).
// sort_local_rank runs the steps back to back; sort_local_ranks runs each step
// on every rank before the next one, so that the host's waits for one rank
// (the span, the first histogram, the hybrid's error word) do not hold back
// the other devices of a loopback context (advisor r03).  Each rank keeps
// its own pass cursor (begin_pass) from step to step.
//
// Single-read passes (nothing exchanged): one k_subhist read (digit 0's
// sub-array histogram and the key span), then one k_onesweep per digit that
// varies, each also counting the next such digit over its output.  Same
// output as the reduce-then-scan loop (do_pass).  A constant digit 0 is
// skipped like any other: its pass would be the identity, so the first
// digit that varies is counted by a second k_subhist read (a read, not a
// pass), and that digit's histogram also decides the stage split.
//
// The hybrid (LSB_OPT_HYBRID): the same stable order as the LSD passes from
// fewer passes over HBM (lsb_segsort.hip): k_onesweep passes on the k most
// significant varying bytes only, then k_segsort orders every segment (run
// of records equal on those bytes) by the whole key.  k: the fewest top
// varying bytes whose varying bits reach ceil(log2 m), so uniform keys leave
// segments of about one record (2^30 records: k = 4, 0.25 on average;
// k_segsort's walk then costs ~2 LDS reads per record and the pass streams
// at copy speed.  k = 3, 64 per segment, made k_segsort compute-bound: 69 ms
// against 7 for the fourth byte's pass, profiles/r03_h1_probe.log).  The k
// passes leave the input A untouched (A -> B, then B <-> R), so when
// k_segsort meets a segment longer than kSegMax the sort starts over from A
// with the LSD passes; skewed keys (the first pass's byte has a bucket over
// 1/32 of the records, as for the stage split: duplicate-heavy keys make
// long segments) take them directly.
std::vector<int> hybrid_bytes(uint64_t varying, int64_t m) {
  int need = 0;
  while ((int64_t(1) << need) < m) ++need;
  std::vector<int> top;
  int bits = 0;
  for (int b = 64 / lsb::kDigitBits - 1; b >= 0 && bits < need; --b) {
    const uint64_t v = (varying >> (b * lsb::kDigitBits)) & (lsb::kBuckets - 1);
    if (!v) continue;
    top.insert(top.begin(), b);
    bits += __builtin_popcountll(v);
  }
  return top;
}

namespace {

struct LocalSort {
  lsb_ctx* c;
  Rank& r;
  int passes = 0;        // local passes run
  uint64_t varying = 0;  // key bits that vary in the block
  enum Kind { kDone, kLsd, kHybrid } kind = kDone;
  int cursor = 0, cur = 0;  // this rank's pass cursor between the steps
  int counted = -1;         // the byte os_hist[0] counts
  bool hist_queued = false;  // its read-back into os_hist_h is queued
  std::vector<int> digits, msd;
  bool fuse = false;
  bool region = false;  // pass 0 ran into the regional layout (region_first)
  // {A, B, R} stays a permutation of {X0, X1, X2} at every step (the pass
  // loop swaps A and B; R holds X0, the kept input, from the first pass on).
  // While armed, an error return restores A = X0, B = X1, R = X2, so the
  // context keeps its input in A and three distinct buffers (advisor r03).
  Elem *X0 = nullptr, *X1 = nullptr, *X2 = nullptr;
  bool armed = false;
  uint64_t pmask = 0;
  lsb::SegPass sp;
  const Elem* seg_in = nullptr;  // the last pass's input, read by k_segfix
  uint32_t* err = nullptr;       // the segment sorts' error word

  LocalSort(lsb_ctx* c_, Rank& r_) : c(c_), r(r_) {}
  LocalSort(const LocalSort&) = delete;
  ~LocalSort() {
    if (armed) {
      r.A = X0;
      r.B = X1;
      r.R = X2;
    }
  }
  struct Step {  // resume and save the rank's pass cursor
    LocalSort& s;
    explicit Step(LocalSort& s_) : s(s_) {
      s.c->pass_cursor = s.cursor;
      s.c->cur_pass = s.cur;
    }
    ~Step() {
      s.cursor = s.c->pass_cursor;
      s.cur = s.c->cur_pass;
    }
  };

  int begin();
  int queue();
  int finish();
  int hybrid_passes(size_t from);
  int classic();
  int first_hist(int byte, bool* skewed, bool* constant);
  int queue_err_word() {
    // The look-back's give-up word, read by lsb_sync.
    HIP_TRY(hipMemcpyAsync(r.os_err_h, r.os_ctr + lsb::kOnesweepSubs, sizeof(uint32_t),
                           hipMemcpyDeviceToHost, r.stream));
    return LSB_OK;
  }
};

// Count + scan + scatter passes (the single-read ones do not apply), run whole.
int LocalSort::classic() {
  HIP_TRY(hipMemsetAsync(r.span, 0, 2 * sizeof(uint64_t), r.stream));
  c->pass_cursor = 0;
  begin_pass(c, 0);
  LSB_TRY(local_pass(c, r, 0, c->skip_constant));
  passes = 1;
  varying = ~0ull;
  if (c->skip_constant) {
    HIP_TRY(hipMemcpyAsync(r.span_h, r.span, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, r.stream));
    HIP_TRY(hipStreamSynchronize(r.stream));
    varying = r.span_h[0] & r.span_h[1];
  }
  for (int d = 1; d < 64 / lsb::kDigitBits; ++d) {
    if (((varying >> (d * lsb::kDigitBits)) & (lsb::kBuckets - 1)) == 0) continue;
    begin_pass(c, d * lsb::kDigitBits);
    LSB_TRY(local_pass(c, r, d * lsb::kDigitBits));
    ++passes;
  }
  return LSB_OK;
}

int LocalSort::begin() {
  Step step(*this);
  kind = kDone;
  if (r.here == 0) return LSB_OK;
  HIP_TRY(hipSetDevice(r.dev));
  if (!c->onesweep || r.here > lsb::kOnesweepMaxElems) return classic();
  LSB_TRY(onesweep_ensure(r));
  c->pass_cursor = 0;
  c->cur_pass = 0;  // the count reads are filed under the first pass
  varying = ~0ull;
  HIP_TRY(hipMemsetAsync(r.span, 0, 2 * sizeof(uint64_t), r.stream));
  if (c->hybrid) {
    kind = kHybrid;
    LSB_TRY(ensure_recv(c, r));
    // Count the byte the first pass most likely sorts on (full 64-bit keys)
    // in the same read as the span, and queue its read-back beside the span's.
    const std::vector<int> guess = hybrid_bytes(~0ull, r.here);
    region = false;
    // The regional first pass for the hybrid's first byte pass (k >= 3: the
    // pass that reads the layout must not be the segment pass).
    if (guess.size() >= 3 && region_applies(c, r)) LSB_TRY(region_sample(c, r, guess[0], &region, &varying));
    if (region) {  // every byte varies: the top bytes are the guess
      c->last_first = LSB_FIRST_REGIONAL;
      msd = guess;
      X0 = r.A;
      X1 = r.B;
      X2 = r.R;
      armed = true;
      LSB_TRY(region_first(c, r, guess[0] * lsb::kDigitBits, guess[1] * lsb::kDigitBits, &passes));
      r.B = X2;  // A is X1 now, B is X0: keep X0, write X2 next (hybrid_passes)
      r.R = X0;
      return LSB_OK;
    }
    varying = ~0ull;
    counted = guess.empty() ? 0 : guess[0];
    LSB_TRY(count_byte(c, r, counted, c->skip_constant));
    HIP_TRY(hipMemcpyAsync(r.os_hist_h, r.os_hist, sizeof(uint32_t) * lsb::kOnesweepSubs * lsb::kBuckets,
                           hipMemcpyDeviceToHost, r.stream));
    hist_queued = true;
  } else {
    kind = kLsd;
    region = false;
    if (region_applies(c, r)) LSB_TRY(region_sample(c, r, 0, &region, &varying));
    if (region) {  // every digit varies: no span read
      c->last_first = LSB_FIRST_REGIONAL;
      // Armed until the pass that reads the regional layout is queued: A then
      // holds the layout (gaps of stale slots, no permutation), so an error
      // return before that restores the input to A (advisor r05).
      X0 = r.A;
      X1 = r.B;
      X2 = r.R;
      armed = true;
      return region_first(c, r, 0, lsb::kDigitBits, &passes);
    }
    varying = ~0ull;
    LSB_TRY(count_byte(c, r, 0, c->skip_constant));
    LSB_TRY(queue_halves(c, r, r.os_hist));
  }
  if (c->skip_constant)
    HIP_TRY(hipMemcpyAsync(r.span_h, r.span, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, r.stream));
  return LSB_OK;
}

// The first byte sorted on decides the stage split and whether keys are
// skewed (*skewed: a bucket over 1/32 of the records).  *constant: one bucket
// holds every record (the byte is constant here; only possible for the
// guessed bytes, with LSB_OPT_SKIP_CONSTANT_DIGITS off).
int LocalSort::first_hist(int byte, bool* skewed, bool* constant) {
  if (byte != counted) {
    LSB_TRY(count_byte(c, r, byte, false));
    counted = byte;
    hist_queued = false;
  }
  if (!hist_queued)
    HIP_TRY(hipMemcpyAsync(r.os_hist_h, r.os_hist, sizeof(uint32_t) * lsb::kOnesweepSubs * lsb::kBuckets,
                           hipMemcpyDeviceToHost, r.stream));
  hist_queued = false;  // the passes overwrite os_hist
  HIP_TRY(hipStreamSynchronize(r.stream));
  const int64_t m = r.here;
  const int h = lsb::onesweep_halves_for(r.os_hist_h, m);
  r.os_halves = c->os_split == 0 ? h : (c->os_split == 2 ? 2 : 1);
  *skewed = h == 2;
  *constant = false;
  for (int b = 0; b < lsb::kBuckets && !*constant; ++b) {
    uint64_t tot = 0;
    for (int x = 0; x < lsb::kOnesweepSubs; ++x) tot += r.os_hist_h[x * lsb::kBuckets + b];
    *constant = tot == (uint64_t)m;
  }
  return LSB_OK;
}

int LocalSort::queue() {
  if (kind == kDone) return LSB_OK;
  Step step(*this);
  HIP_TRY(hipSetDevice(r.dev));
  const int64_t m = r.here;
  if (kind == kLsd && region) {
    // Every digit varies (region_sample).  The second pass reads the
    // regional layout (pass 0 counted digit 1 over its tiles into os_hist[1]).
    region = false;
    HIP_TRY(hipStreamSynchronize(r.stream));
    digits = varying_bytes(~0ull);
    if (r.rg_h[kRgOvf] == 0) {
      r.os_halves = 1;
      const lsb::RegionPass rp = region_pass(r);
      LSB_TRY(onesweep_digits(c, r, digits, &passes, 1, &rp, &armed));
      kind = kDone;
      return queue_err_word();
    }
    // A region overflowed: start over from the input, kept in place (pass 0
    // read it and wrote the other buffer), with the usual first read.
    c->last_first = LSB_FIRST_REGIONAL_REDONE;
    std::swap(r.A, r.B);
    armed = false;
    passes = 0;
    c->pass_cursor = 0;
    c->cur_pass = 0;
    HIP_TRY(hipMemsetAsync(r.span, 0, 2 * sizeof(uint64_t), r.stream));
    LSB_TRY(count_byte(c, r, 0, c->skip_constant));
    LSB_TRY(queue_halves(c, r, r.os_hist));
    HIP_TRY(hipMemcpyAsync(r.span_h, r.span, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, r.stream));
    HIP_TRY(hipStreamSynchronize(r.stream));
    varying = c->skip_constant ? r.span_h[0] & r.span_h[1] : ~0ull;
    digits = varying_bytes(varying);
    LSB_TRY(choose_halves(c, r, true));
    LSB_TRY(onesweep_digits(c, r, digits, &passes));
    kind = kDone;
    return queue_err_word();
  }
  if (kind == kHybrid && region) {
    region = false;
    HIP_TRY(hipStreamSynchronize(r.stream));
    if (r.rg_h[kRgOvf] == 0) {
      digits = varying_bytes(~0ull);
      r.os_halves = 1;
      return hybrid_passes(1);
    }
    // A region overflowed: the kept input X0 and the usual start.
    r.A = X0;
    r.B = X1;
    r.R = X2;
    armed = false;
    passes = 0;
    c->pass_cursor = 0;
    c->cur_pass = 0;
    c->last_first = LSB_FIRST_REGIONAL_REDONE;
    HIP_TRY(hipMemsetAsync(r.span, 0, 2 * sizeof(uint64_t), r.stream));
    counted = msd[0];
    LSB_TRY(count_byte(c, r, counted, c->skip_constant));
    HIP_TRY(hipMemcpyAsync(r.os_hist_h, r.os_hist, sizeof(uint32_t) * lsb::kOnesweepSubs * lsb::kBuckets,
                           hipMemcpyDeviceToHost, r.stream));
    hist_queued = true;
    if (c->skip_constant)
      HIP_TRY(hipMemcpyAsync(r.span_h, r.span, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, r.stream));
    varying = ~0ull;
  }
  if (c->skip_constant) HIP_TRY(hipStreamSynchronize(r.stream));
  if (c->skip_constant) varying = r.span_h[0] & r.span_h[1];
  digits = varying_bytes(varying);
  if (kind == kLsd) {
    if (!digits.empty() && digits[0] != 0) {
      LSB_TRY(count_byte(c, r, digits[0], false));
      LSB_TRY(queue_halves(c, r, r.os_hist));
      LSB_TRY(choose_halves(c, r, false));
    } else {
      LSB_TRY(choose_halves(c, r, c->skip_constant));
    }
    LSB_TRY(onesweep_digits(c, r, digits, &passes));
    kind = kDone;
    return queue_err_word();
  }
  msd = hybrid_bytes(c->skip_constant ? varying : ~0ull, m);
  bool hybrid = msd.size() < digits.size();
  bool skewed = false, constant = false;
  if (hybrid && !msd.empty()) {
    LSB_TRY(first_hist(msd[0], &skewed, &constant));
    // Skewed keys make long segments; a constant first byte means the guessed
    // top bytes are not where the keys vary (advisor r03): the LSD passes.
    if (skewed || constant) hybrid = false;
  }
  if (!hybrid) {
    if (!digits.empty()) LSB_TRY(first_hist(digits[0], &skewed, &constant));
    LSB_TRY(onesweep_digits(c, r, digits, &passes));
    kind = kDone;
    return queue_err_word();
  }
  return hybrid_passes(0);
}

// The k passes: A -> B, then B <-> R; the input X0 is kept.  The last one
// also orders every segment inside its tile (SegPass) and k_segfix merges
// the segments split between tiles; LSB_OPT_HYBRID = 2, or the split stage,
// leaves the segments to a k_segsort pass instead.  from = 1: the first pass
// ran into the regional layout (begin), the second reads it.
int LocalSort::hybrid_passes(size_t from) {
  const int64_t m = r.here;
  if (from == 0) {
    X0 = r.A;
    X1 = r.B;
    X2 = r.R;
    armed = true;
  }
  for (int b : msd) pmask |= (uint64_t)(lsb::kBuckets - 1) << (b * lsb::kDigitBits);
  err = r.os_ctr + lsb::kOnesweepSubs + 1;
  fuse = c->hybrid == 1 && r.os_halves == 1 && !msd.empty();
  if (fuse) {
    if (!r.seg_base) LSB_TRY(dev_alloc(&r.seg_base, (size_t)lsb::kOnesweepSubs * lsb::kBuckets));
    sp.pmask = pmask;
    sp.rmask = pmask & ~((uint64_t)(lsb::kBuckets - 1) << (msd.back() * lsb::kDigitBits));
    sp.base = r.seg_base;
    sp.err = err;
  }
  HIP_TRY(hipMemsetAsync(err, 0, sizeof(uint32_t), r.stream));
  uint32_t* hist[2] = {r.os_hist, r.os_hist + lsb::kOnesweepSubs * lsb::kBuckets};
  const lsb::RegionPass rp = from == 1 ? region_pass(r) : lsb::RegionPass();
  for (size_t i = from; i < msd.size(); ++i) {
    const int shift = msd[i] * lsb::kDigitBits;
    const int next = i + 1 < msd.size() ? msd[i + 1] * lsb::kDigitBits : -1;
    begin_pass(c, shift);
    lsb::OnesweepExtra x;
    x.halves = r.os_halves;
    if (from == 1 && i == 1) {
      x.region = &rp;
      x.region_mode = 2;
    }
    if (fuse && i + 1 == msd.size()) {
      x.seg = &sp;
      seg_in = r.A;
    }
    LSB_TRY(onesweep_launch(c, r, shift, next, hist[i & 1], hist[(i + 1) & 1], x));
    ++passes;
    if (i == 0) {  // A is X1 now, B is X0: keep X0, write X2 next
      r.B = X2;
      r.R = X0;
    }
  }
  if (msd.empty()) {
    r.B = X1;
    r.R = X2;
  }
  if (fuse) {
    {
      Timer t(c, &r, LSB_K_SEGSORT);
      // one wave per tile boundary, 32 waves per CU
      HIP_TRY(lsb::launch_segfix(seg_in, r.A, m, msd.back() * lsb::kDigitBits, r.os_status, sp,
                                 16 * r.os_grid, r.stream));
    }
    HIP_TRY(hipMemcpyAsync(r.os_err_h + 1, err, sizeof(uint32_t), hipMemcpyDeviceToHost, r.stream));
  }
  return LSB_OK;
}

int LocalSort::finish() {
  if (kind != kHybrid) return LSB_OK;
  Step step(*this);
  HIP_TRY(hipSetDevice(r.dev));
  auto sync_err = [&](uint32_t* v) -> int {
    HIP_TRY(hipStreamSynchronize(r.stream));
    *v = r.os_err_h[1];
    return LSB_OK;
  };
  bool sorted = false, a_valid = true;
  if (fuse) {  // its error word's read-back was queued after k_segfix
    uint32_t e = 0;
    LSB_TRY(sync_err(&e));
    sorted = e == 0;
    // Bit 2: a segment of the fused pass ran past kSegMax inside its tile,
    // so r.A is not a permutation (SegPass, lsb_kernels.h): straight to the
    // LSD passes over the kept input.  Bit 1 alone: k_segfix left a
    // boundary, and k_segsort finishes r.A.
    a_valid = (e & 2u) == 0;
  }
  if (!sorted && a_valid) {
    // k_segsort: r.A is stably sorted by pmask (the fused pass's segments
    // too, in or out of order).
    HIP_TRY(hipMemsetAsync(err, 0, sizeof(uint32_t), r.stream));
    begin_pass(c, 64);
    {
      Timer t(c, &r, LSB_K_SEGSORT);
      HIP_TRY(lsb::launch_segsort(r.A, r.B, r.here, pmask, err, 3 * r.os_grid / 2, r.stream));
    }
    count_pass_elems(c, r.here, false);
    ++passes;
    HIP_TRY(hipMemcpyAsync(r.os_err_h + 1, err, sizeof(uint32_t), hipMemcpyDeviceToHost, r.stream));
    uint32_t e = 0;
    LSB_TRY(sync_err(&e));
    if (e == 0) {
      std::swap(r.A, r.B);
      sorted = true;
    }
  }
  kind = kDone;
  if (sorted) {
    r.R = (X0 != r.A && X0 != r.B) ? X0 : (X1 != r.A && X1 != r.B) ? X1 : X2;
    armed = false;
  } else {  // a segment too long for the segment sorts: the LSD passes over the kept input
    r.A = X0;
    r.B = X1;
    r.R = X2;
    armed = false;
    counted = -1;
    bool skewed = false, constant = false;
    if (!digits.empty()) LSB_TRY(first_hist(digits[0], &skewed, &constant));
    LSB_TRY(onesweep_digits(c, r, digits, &passes));
  }
  return queue_err_word();
}

}  // namespace

// Rank r alone (its local block); *passes gets the passes it ran, *varying the
// key bits that vary in the block (0 for an empty block).
int sort_local_rank(lsb_ctx* c, Rank& r, int* passes, uint64_t* varying) {
  LocalSort s(c, r);
  LSB_TRY(s.begin());
  LSB_TRY(s.queue());
  LSB_TRY(s.finish());
  *passes = s.passes;
  *varying = s.varying;
  return LSB_OK;
}

// Every rank's local block, step by step across the ranks: c->last_local_passes
// gets the most passes a rank ran, c->last_varying the bits that vary anywhere.
int sort_local_ranks(lsb_ctx* c) {
  std::deque<LocalSort> jobs;
  for (Rank& r : c->ranks) jobs.emplace_back(c, r);
  for (LocalSort& j : jobs) LSB_TRY(j.begin());
  for (LocalSort& j : jobs) LSB_TRY(j.queue());
  for (LocalSort& j : jobs) LSB_TRY(j.finish());
  c->last_local_passes = 0;
  c->last_varying = 0;
  for (const LocalSort& j : jobs) {
    c->last_local_passes = std::max(c->last_local_passes, j.passes);
    c->last_varying |= j.varying;
  }
  return LSB_OK;
}

int sort_onesweep(lsb_ctx* c) {
  return sort_local_rank(c, c->ranks[0], &c->last_local_passes, &c->last_varying);
}

// After a stream sync: did a look-back give up?  (Never expected: every
// tile's predecessors belong to running workgroups.)
#ifdef LSB_OS_PROFILE
void os_profile_report() {
  unsigned long long p[10];
  if (lsb::onesweep_profile(p, true) != hipSuccess) return;
  const double tot = (double)(p[0] + p[1] + p[2] + p[3] + p[4] + p[5] + p[6]) + 1e-9;
  fprintf(stderr,
          "os_profile: dequeue %.4f load %.4f rank %.4f scan %.4f stage %.4f lookback %.4f write %.4f "
          "(ticks %.0f; rows summed per tile %.2f over %llu tiles)\n",
          p[0] / tot, p[6] / tot, p[1] / tot, p[2] / tot, p[3] / tot, p[5] / tot, p[4] / tot, tot,
          p[8] ? (double)p[7] / (double)p[8] : 0.0, p[8]);
}
#endif

int onesweep_check(Rank& r) {
  if (!r.os_err_h || *r.os_err_h == 0) return LSB_OK;
  *r.os_err_h = 0;
  HIP_TRY(hipMemset(r.os_ctr + lsb::kOnesweepSubs, 0, sizeof(uint32_t)));
  // A launch that gave up may have left rows of an older parity: start the
  // granules over (zeroed; the next launch is odd).
  zero_status(r);
  HIP_TRY(hipStreamSynchronize(r.stream));
  return fail(LSB_ERR_HIP, "k_onesweep", "look-back timed out; output invalid");
}

}  // namespace lsb_rt
