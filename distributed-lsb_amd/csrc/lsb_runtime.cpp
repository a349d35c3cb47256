// Runtime behind include/lsb.h: contexts, device buffers, the pass loop
// (mySort / globalShuffle) and the exchange (RCCL or in-process loopback).
//
// Per pass on digit d of `bits` bits (64 / bits passes, least significant
// first, mpi/mpi_lsbsort.cpp:580-585), for every rank r:
//   1. local stable pass(es) A -> B, then swap (localShuffle,
//      mpi/mpi_lsbsort.cpp:213-247): one 8-bit pass for bits = 8, two stable
//      8-bit sub-passes (low byte, high byte) for bits = 16.  A is then
//      ordered by digit d.
//   P == 1: done.
//   P  > 1:
//   2. the rank's bucket counts of digit d (k_scan totals for 8 bits,
//      run lengths of the sorted 16-bit digits for 16 bits), all-gathered
//      (replaces copyCountsToGlobalCounts + MPI_Exscan +
//      copyStartsFromGlobalStarts, mpi/mpi_lsbsort.cpp:327-479: every rank
//      scans the P x nbuckets matrix in digit-major, rank-minor order itself)
//   3. device plan (k_plan_*, same rule as lsb_plan_exchange): placement
//      table on the device, the 2P send/recv counts to the host
//   4. all-to-all-v of 16-byte records out of A into R (MPI_Alltoallv of
//      24-byte ShuffleBufSortElement at mpi/mpi_lsbsort.cpp:563; no
//      destination index travels: the receiver derives it from the counts),
//      cut into `slices` groups: slice j carries part j of every peer segment
//   5. k_place -> B on a second stream (mpi/mpi_lsbsort.cpp:568-575): the
//      self segment straight out of A at once, slice j of R as soon as it has
//      arrived, overlapping slice j+1 on the wire; then swap
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/lsb.h"
#include "lsb_kernels.h"

using lsb::Elem;

namespace {

// kLoopback: all ranks in this process (lsb_create); kRccl: this process is
// one rank, RCCL collectives (lsb_create_rank); kOps: one rank, the caller's
// host collectives (lsb_create_rank_ops).
enum class Mode { kLoopback, kRccl, kOps };

struct PendingEvent {
  int kid;
  int dev;
  int pass;  // local pass the launch is filed under (lsb_get_pass_stats), -1: none
  hipEvent_t start, stop;
};

struct Rank {
  int rank = 0;
  int dev = 0;
  hipStream_t stream = nullptr;
  hipStream_t pstream = nullptr;        // placement stream (overlaps the exchange)
  hipEvent_t pevent = nullptr;          // stream -> pstream handoff
  hipEvent_t pdone = nullptr;           // pstream -> stream: placement finished
  int64_t here = 0;
  Elem* A = nullptr;  // per slots: input / output (DistributedArray A)
  Elem* B = nullptr;  // per slots: ping-pong partner
  Elem* R = nullptr;  // per slots: receive buffer (P > 1 only)
  uint32_t* chunk_hist = nullptr;       // [256][num_chunks]
  uint64_t* chunk_off = nullptr;        // [256][num_chunks]
  uint64_t* totals = nullptr;           // [256] local counts of the current 8-bit digit
  uint64_t* totals16 = nullptr;         // [65536] local counts of a 16-bit digit (bits = 16, P > 1)
  int64_t* first16 = nullptr;           // [65536] scratch of the 16-bit count
  bool starts_fused = false;            // first16 holds this digit's starts (marked by k_scatter)
  uint64_t* gather = nullptr;           // [P][nb] all-gathered counts
  int64_t* place = nullptr;             // [P][nb] place_off, then [P] rend (device plan)
  int64_t* plan_work = nullptr;         // [P][nb] device-plan scratch
  int64_t* plan_total = nullptr;        // [nb]    device-plan scratch
  int64_t* plan_counts = nullptr;       // [2P] send counts, recv counts
  unsigned long long* check = nullptr;  // [4] verify / check_sorted scratch
  uint64_t* span = nullptr;             // [2] OR of keys, OR of ~keys (first pass of lsb_sort)
  uint64_t* span_gather = nullptr;      // [2P] all-gathered spans (RCCL)
  uint64_t* span_h = nullptr;           // [2P] pinned host mirror
  int64_t* counts_h = nullptr;          // pinned host mirror of plan_counts
  lsb::Chunking chunking;
  // Peer-store exchange (LSB_OPT_EXCHANGE_PEER): the two physical record
  // buffers (A and B swap between them), every rank's two buffers as this
  // process sees them (IPC-opened for other processes), and the base table.
  Elem* buf[2] = {nullptr, nullptr};
  std::vector<Elem*> peer0, peer1;
  std::vector<void*> ipc_opened;
  int64_t* peer_base = nullptr;         // [nb]
  // Single-read passes (LSB_OPT_ONESWEEP, P == 1), allocated on first use.
  uint32_t* os_status = nullptr;        // [tiles][256] look-back granules (self-tagged u32)
  uint32_t* os_hist = nullptr;          // [2][8][256] sub-array histograms (ping-pong)
  uint32_t* os_ctr = nullptr;           // [8] tile counters, [8] look-back error word
  uint32_t* os_err_h = nullptr;         // pinned mirror of the error word
  uint32_t* os_hist_h = nullptr;        // pinned mirror of a sub-array histogram
  int os_halves = 1;                    // this sort's k_onesweep stage split (1 or 2)
  uint32_t os_epoch = 0;                // last look-back epoch
  bool os_dirty = false;                // a launch failed: zero os_status before the next
  int64_t* seg_base = nullptr;          // [kOnesweepSubs][256] the hybrid's bucket bases (k_segfix)
  int os_grid = 0;                      // persistent grid (2 workgroups per CU)
  // Per-digit exchange with single-read local passes (sort_exchange_onesweep):
  // os_hist[os_cur] is A's sub-array histogram of the byte at os_valid (-1:
  // none; the next pass reads A once with k_subhist).  The exchange's
  // placements count the byte at place_next into place_hist as they write.
  int os_cur = 0;
  int os_valid = -1;
  int place_next = -1;
  uint32_t* place_hist = nullptr;
  bool counts_ready = false;            // totals16 = this exchange digit's counts (k_onesweep C16)
  // Gathered passes (LSB_OPT_EXCHANGE_GATHER): an exchange whose placement
  // only counts leaves the peers' records in R and the rank's own in A; the
  // next local pass reads them there through gsrc (piece starts in gstart,
  // one descriptor per onesweep tile in gdesc), allocated on first use.
  bool gather_next = false;             // this exchange counts only
  bool gather_pending = false;          // the next local pass gathers
  int64_t* gstart = nullptr;            // [nb][P] piece starts in the placed order
  lsb::TileDesc* gdesc = nullptr;       // [tiles]
  lsb::GatherSrc gsrc;
  // Whole-key exchange (radix_bits = 64), allocated on first use.
  uint64_t* split_state = nullptr;      // [Q][2] key interval per target
  int64_t* split_targets = nullptr;     // [Q] global positions q * per
  uint64_t* split_cnt = nullptr;        // [Q][kSplitCands] counts below the candidates
  uint64_t* split_gather = nullptr;     // [P][Q][kSplitCands] all-gathered
  uint64_t* split_fin = nullptr;        // [Q][2] #keys < k*, #keys <= k*
  uint64_t* split_fin_gather = nullptr; // [P][Q][2]
  uint64_t* split_h = nullptr;          // pinned mirror of split_fin_gather
  int64_t* merge_path = nullptr;        // merge-path tile boundaries
  int split_q = 0, split_S = 0;         // geometry the split buffers were sized for
  std::vector<int64_t> mcut;            // [P][P * S + 1] cuts of every source (host)
  std::vector<int64_t> send_counts, send_displs, recv_counts, recv_displs;
};

}  // namespace

struct lsb_ctx {
  Mode mode = Mode::kLoopback;
  int64_t n = 0;
  int64_t per = 0;
  int P = 1;
  int bits = 8;      // exchange digit width: 8, 16, or 64 (the whole key: one exchange)
  int nb = 256;      // 1 << bits (256 for bits = 64: the buckets of the local passes)
  int first_rank = 0;
  std::vector<Rank> ranks;  // local ranks
  ncclComm_t comm = nullptr;
  lsb_comm_ops_t ops = {};  // Mode::kOps
  bool timing = false;
  bool force_exchange = false;
  bool skip_constant = true;  // lsb_sort skips digits on which all keys agree
  int slices = 0;             // exchange slices (placement overlaps the next slice); 0 = default
  bool p2p = false;           // RCCL exchange as grouped ncclSend/ncclRecv, not ncclAllToAllv
  bool peer = false;          // exchange by direct stores into the owners' buffers
  bool peer_ready = false;    // peer tables set up
  bool onesweep = true;       // P == 1: single-read passes (k_subhist + k_onesweep)
  bool self_coll = false;     // the self segment also goes through the collective
  bool gather = true;         // LSB_OPT_EXCHANGE_GATHER: count-only placement + gathered pass
  int os_split = 0;           // LSB_OPT_ONESWEEP_SPLIT: 0 auto, 1 never, 2 always
  int hybrid = 0;             // LSB_OPT_HYBRID: 0 off, 1 k byte passes (the last one
                              // ordering segments, + k_segfix), 2 the same + a k_segsort pass
  int64_t coll_calls = 0, coll_bytes = 0, coll_max = 0;  // element payload handed to the collective
  // What the last lsb_sort ran (lsb_get_last_sort).
  int last_local_passes = 0;
  int last_exchanges = 0;
  uint64_t last_varying = 0;
  lsb::KeyGen keygen;
  std::vector<PendingEvent> pending;
  std::vector<hipEvent_t> event_pool;
  int64_t launches[LSB_K_COUNT] = {};
  double total_ms[LSB_K_COUNT] = {};
  int64_t scatter_elems = 0;
  // Per local pass (lsb_get_pass_stats): the pass the next timed launch is
  // filed under (pass_cursor counts the local passes of the current sort).
  int cur_pass = 0;
  int pass_cursor = 0;
  int pass_shift[LSB_MAX_PASSES] = {};
  int64_t pass_launches[LSB_MAX_PASSES][LSB_K_COUNT] = {};
  double pass_ms[LSB_MAX_PASSES][LSB_K_COUNT] = {};
  int64_t pass_elems[LSB_MAX_PASSES] = {};
};

namespace {

thread_local std::string g_last_error;

int fail(int code, const char* what, const char* detail) {
  char buf[512];
  snprintf(buf, sizeof buf, "%s: %s", what, detail ? detail : "");
  g_last_error = buf;
  if (getenv("LSB_DEBUG")) fprintf(stderr, "[lsb] %s\n", buf);
  return code;
}

#define HIP_TRY(expr)                                                    \
  do {                                                                   \
    hipError_t _e = (expr);                                              \
    if (_e != hipSuccess) return fail(LSB_ERR_HIP, #expr, hipGetErrorString(_e)); \
  } while (0)

#define RCCL_TRY(expr)                                                   \
  do {                                                                   \
    ncclResult_t _r = (expr);                                            \
    if (_r != ncclSuccess) return fail(LSB_ERR_RCCL, #expr, ncclGetErrorString(_r)); \
  } while (0)

#define LSB_TRY(expr)              \
  do {                             \
    int _c = (expr);               \
    if (_c != LSB_OK) return _c;   \
  } while (0)

int64_t div_ceil(int64_t x, int64_t y) { return (x + y - 1) / y; }

int64_t here_of(int64_t n, int P, int r) {
  const int64_t per = P > 0 ? div_ceil(n, P) : 0;
  int64_t h = per;
  if (per * r + h > n) h = n - per * r;
  return h < 0 ? 0 : h;
}

bool exchanging(const lsb_ctx* c) { return c->P > 1 || c->force_exchange; }

// ---- timing -------------------------------------------------------------
hipEvent_t take_event(lsb_ctx* c) {
  if (!c->event_pool.empty()) {
    hipEvent_t e = c->event_pool.back();
    c->event_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

struct Timer {
  lsb_ctx* c;
  Rank* r;
  int kid;
  int pass;
  hipStream_t stream;
  hipEvent_t start = nullptr;
  Timer(lsb_ctx* c_, Rank* r_, int kid_, hipStream_t s = nullptr)
      : c(c_), r(r_), kid(kid_), pass(kid_ == LSB_K_SORT ? -1 : c_->cur_pass),
        stream(s ? s : r_->stream) {
    if (!c->timing) return;
    start = take_event(c);
    if (start) (void)hipEventRecord(start, stream);
  }
  void stop() {
    if (!start) return;
    hipEvent_t e = take_event(c);
    if (!e) return;
    (void)hipEventRecord(e, stream);
    c->pending.push_back({kid, r->dev, pass, start, e});
    start = nullptr;
  }
  ~Timer() { stop(); }
};

// The local pass the following launches belong to: the pass_cursor-th local
// pass of this sort, on the byte at `shift` (lsb_get_pass_stats).
void begin_pass(lsb_ctx* c, int shift) {
  c->cur_pass = c->pass_cursor++;
  if (c->cur_pass < LSB_MAX_PASSES) c->pass_shift[c->cur_pass] = shift;
}

// Records one local pass of m records processed (lsb_get_pass_stats); a
// scatter kernel's records also go to lsb_get_scatter_elems.
void count_pass_elems(lsb_ctx* c, int64_t m, bool scatter = true) {
  if (!c->timing) return;
  if (scatter) c->scatter_elems += m;
  if (c->cur_pass >= 0 && c->cur_pass < LSB_MAX_PASSES) c->pass_elems[c->cur_pass] += m;
}

int resolve_timing(lsb_ctx* c) {
  for (auto& p : c->pending) {
    HIP_TRY(hipSetDevice(p.dev));
    HIP_TRY(hipEventSynchronize(p.stop));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, p.start, p.stop));
    c->launches[p.kid] += 1;
    c->total_ms[p.kid] += ms;
    if (p.pass >= 0 && p.pass < LSB_MAX_PASSES) {
      c->pass_launches[p.pass][p.kid] += 1;
      c->pass_ms[p.pass][p.kid] += ms;
    }
    c->event_pool.push_back(p.start);
    c->event_pool.push_back(p.stop);
  }
  c->pending.clear();
  return LSB_OK;
}

// ---- allocation -----------------------------------------------------------
template <typename T>
int dev_alloc(T** p, size_t count) {
  *p = nullptr;
  if (count == 0) count = 1;
  hipError_t e = hipMalloc(reinterpret_cast<void**>(p), count * sizeof(T));
  if (e != hipSuccess) return fail(LSB_ERR_NOMEM, "hipMalloc", hipGetErrorString(e));
  return LSB_OK;
}

template <typename T>
int host_alloc(T** p, size_t count) {
  *p = nullptr;
  if (count == 0) count = 1;
  hipError_t e = hipHostMalloc(reinterpret_cast<void**>(p), count * sizeof(T), 0);
  if (e != hipSuccess) return fail(LSB_ERR_NOMEM, "hipHostMalloc", hipGetErrorString(e));
  return LSB_OK;
}

int max_chunks_for_device(int dev) {
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess || prop.multiProcessorCount <= 0) return 512;
  // Two scatter workgroups fit one CU (72 KiB LDS each): one chunk per slot.
  return std::min(lsb::kMaxChunks, 2 * prop.multiProcessorCount);
}

int init_rank(lsb_ctx* c, Rank& r, int rank, int dev) {
  r.rank = rank;
  r.dev = dev;
  r.here = here_of(c->n, c->P, rank);
  HIP_TRY(hipSetDevice(dev));
  HIP_TRY(hipStreamCreateWithFlags(&r.stream, hipStreamNonBlocking));
  HIP_TRY(hipStreamCreateWithFlags(&r.pstream, hipStreamNonBlocking));
  HIP_TRY(hipEventCreateWithFlags(&r.pevent, hipEventDisableTiming));
  HIP_TRY(hipEventCreateWithFlags(&r.pdone, hipEventDisableTiming));
  const size_t per = (size_t)c->per;
  r.chunking = lsb::make_chunking(r.here, max_chunks_for_device(dev));
  const size_t hist_entries = (size_t)lsb::kBuckets * std::max(1, r.chunking.num_chunks);
  const size_t P = (size_t)c->P, nb = (size_t)c->nb;
  LSB_TRY(dev_alloc(&r.A, per));
  LSB_TRY(dev_alloc(&r.B, per));
  r.buf[0] = r.A;
  r.buf[1] = r.B;
  // R (the all-to-all receive buffer) is allocated on first use: a context
  // that never runs the all-to-all (P = 1, peer stores) keeps its HBM.
  LSB_TRY(dev_alloc(&r.chunk_hist, hist_entries));
  LSB_TRY(dev_alloc(&r.chunk_off, hist_entries));
  LSB_TRY(dev_alloc(&r.totals, lsb::kBuckets));
  if (c->bits == 16) {
    LSB_TRY(dev_alloc(&r.totals16, 65536));
    LSB_TRY(dev_alloc(&r.first16, 65536));
  }
  LSB_TRY(dev_alloc(&r.gather, std::max(P * nb, P * 4)));
  LSB_TRY(dev_alloc(&r.place, P * nb + P));
  LSB_TRY(dev_alloc(&r.plan_work, P * nb));
  LSB_TRY(dev_alloc(&r.plan_total, nb));
  LSB_TRY(dev_alloc(&r.plan_counts, 2 * P));
  LSB_TRY(dev_alloc(&r.check, 4));
  LSB_TRY(dev_alloc(&r.span, 2));
  LSB_TRY(dev_alloc(&r.span_gather, 2 * P));
  LSB_TRY(host_alloc(&r.span_h, 2 * P));
  LSB_TRY(host_alloc(&r.counts_h, 2 * P));
  r.send_counts.assign(c->P, 0);
  r.send_displs.assign(c->P, 0);
  r.recv_counts.assign(c->P, 0);
  r.recv_displs.assign(c->P, 0);
  return LSB_OK;
}

void free_rank(Rank& r) {
  if (r.stream) {
    (void)hipSetDevice(r.dev);
    (void)hipStreamSynchronize(r.stream);
  }
  for (void* p : r.ipc_opened) (void)hipIpcCloseMemHandle(p);
  (void)hipFree(r.peer_base);
  (void)hipFree(r.split_state);
  (void)hipFree(r.split_targets);
  (void)hipFree(r.split_cnt);
  (void)hipFree(r.split_gather);
  (void)hipFree(r.split_fin);
  (void)hipFree(r.split_fin_gather);
  (void)hipHostFree(r.split_h);
  (void)hipFree(r.merge_path);
  (void)hipFree(r.os_status);
  (void)hipFree(r.gstart);
  (void)hipFree(r.gdesc);
  (void)hipFree(r.seg_base);
  (void)hipFree(r.os_hist);
  (void)hipFree(r.os_ctr);
  (void)hipHostFree(r.os_err_h);
  (void)hipHostFree(r.os_hist_h);
  (void)hipFree(r.A);
  (void)hipFree(r.B);
  (void)hipFree(r.R);
  (void)hipFree(r.chunk_hist);
  (void)hipFree(r.chunk_off);
  (void)hipFree(r.totals);
  (void)hipFree(r.totals16);
  (void)hipFree(r.first16);
  (void)hipFree(r.gather);
  (void)hipFree(r.place);
  (void)hipFree(r.plan_work);
  (void)hipFree(r.plan_total);
  (void)hipFree(r.plan_counts);
  (void)hipFree(r.check);
  (void)hipFree(r.span);
  (void)hipFree(r.span_gather);
  (void)hipHostFree(r.span_h);
  (void)hipHostFree(r.counts_h);
  if (r.pstream) {
    (void)hipStreamSynchronize(r.pstream);
    (void)hipStreamDestroy(r.pstream);
  }
  if (r.pevent) (void)hipEventDestroy(r.pevent);
  if (r.pdone) (void)hipEventDestroy(r.pdone);
  if (r.stream) (void)hipStreamDestroy(r.stream);
  r = Rank();
}

Rank* local_rank(lsb_ctx* c, int rank) {
  const int i = rank - c->first_rank;
  if (i < 0 || i >= (int)c->ranks.size()) return nullptr;
  return &c->ranks[i];
}

// ---- one local stable 8-bit pass A -> B, then swap (localShuffle) -------
// want_span: also reduce the key span (lsb_sort's first pass).  starts16:
// this is the high byte of a 16-bit exchange digit; the scatter also marks
// the digit's run starts, so digit_counts needs no extra read.
int local_pass(lsb_ctx* c, Rank& r, int shift, bool want_span = false, bool starts16 = false) {
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

// Device counts of the exchange digit for rank r (A is ordered by it).
int digit_counts(lsb_ctx* c, Rank& r, int digit, const uint64_t** counts) {
  if (c->bits == 8) {
    *counts = r.totals;  // k_scan totals of the (only) sub-pass
    return LSB_OK;
  }
  if (r.counts_ready) {  // counted by the high-byte k_onesweep
    *counts = r.totals16;
    return LSB_OK;
  }
  HIP_TRY(hipSetDevice(r.dev));
  {
    Timer t(c, &r, LSB_K_UPSWEEP);
    if (r.starts_fused)  // the high-byte scatter marked the starts
      HIP_TRY(lsb::launch_starts_to_counts(r.first16, r.here, r.totals16, r.stream));
    else  // high byte constant (skipped) or lsb_pass: read A once more
      HIP_TRY(lsb::launch_digit16_counts(r.A, r.here, digit * 16, r.first16, r.totals16,
                                         r.stream));
  }
  *counts = r.totals16;
  return LSB_OK;
}

// Device plan of rank r from its gathered count matrix (r.gather): the
// placement table stays on the device; only the 2P send/recv counts come
// back (RCCL takes host counts).  Call plan_fetch after a stream sync.
int plan_launch(lsb_ctx* c, Rank& r) {
  HIP_TRY(hipSetDevice(r.dev));
  if (r.gather_next && !r.gstart) {
    LSB_TRY(dev_alloc(&r.gstart, (size_t)2 * c->P * c->nb));  // gstart, then gadj
    LSB_TRY(dev_alloc(&r.gdesc, (size_t)lsb::onesweep_tiles(r.here)));
  }
  {
    Timer t(c, &r, LSB_K_EXCHANGE);
    HIP_TRY(lsb::launch_plan(r.gather, c->P, c->nb, r.rank, c->n, r.plan_work, r.plan_total,
                             r.place, r.plan_counts, r.stream, r.gather_next ? r.gstart : nullptr));
  }
  HIP_TRY(hipMemcpyAsync(r.counts_h, r.plan_counts, sizeof(int64_t) * 2 * c->P,
                         hipMemcpyDeviceToHost, r.stream));
  return LSB_OK;
}

void plan_fetch(lsb_ctx* c, Rank& r) {
  int64_t sd = 0, rd = 0;
  for (int q = 0; q < c->P; ++q) {
    r.send_counts[q] = r.counts_h[q];
    r.recv_counts[q] = r.counts_h[c->P + q];
    r.send_displs[q] = sd;
    r.recv_displs[q] = rd;
    sd += r.send_counts[q];
    rd += r.recv_counts[q];
  }
}

// ---- placement, overlapped with the exchange ------------------------------
// Part j of n records cut into `slices` parts: [part(n, j), part(n, j + 1)).
// Sender and receiver cut a segment alike (send_counts[q] at s equals
// recv_counts[s] at q).
int64_t part(int64_t n, int j, int slices) { return n * j / slices; }

// Slices of an exchange: the option, else 4 per exchange digit, or 8 for the
// whole-key exchange, whose one all-to-all carries every record: its last
// slice's merge (ceil(log2 P) levels) is the tail after the wire goes quiet.
int slices_of(const lsb_ctx* c) { return c->slices > 0 ? c->slices : (c->bits == 64 ? 8 : 4); }

// After an exchange's placements: B holds the placed block and becomes A, or
// (count-only placement) the next pass gathers from R and A.
void end_placement(Rank& r) {
  if (r.gather_next) r.gather_pending = true;
  else std::swap(r.A, r.B);
}

// Everything after this on r.stream waits for r.pstream's work so far.
int join_place(Rank& r) {
  HIP_TRY(hipEventRecord(r.pdone, r.pstream));
  HIP_TRY(hipStreamWaitEvent(r.stream, r.pdone, 0));
  return LSB_OK;
}

// Place one source's received range [k0, k0 + cnt) (records at src) into B.
int place_range(lsb_ctx* c, Rank& r, int shift, int src_rank, const Elem* src, int64_t k0,
                int64_t cnt) {
  if (cnt <= 0) return LSB_OK;
  Timer t(c, &r, LSB_K_PLACE, r.pstream);
  HIP_TRY(lsb::launch_place(src, r.B, r.here, k0, cnt, shift, c->nb,
                            r.place + (size_t)src_rank * c->nb, r.pstream, r.place_next,
                            r.place_hist, !r.gather_next));
  return LSB_OK;
}

// The receive buffer, allocated at the first all-to-all of the context.
int ensure_recv(lsb_ctx* c, Rank& r) {
  if (r.R) return LSB_OK;
  HIP_TRY(hipSetDevice(r.dev));
  return dev_alloc(&r.R, (size_t)c->per);
}

// The self segment needs no transfer: place it straight out of A as soon as
// the plan is on the device (call after the host has the plan).  With
// LSB_OPT_EXCHANGE_SELF it travels through the collective instead and is
// placed from R by place_slice like every other source.
int place_self(lsb_ctx* c, Rank& r, int shift) {
  const int me = r.rank;
  if (r.send_counts[me] != r.recv_counts[me])
    return fail(LSB_ERR_STATE, "exchange", "self count mismatch");
  LSB_TRY(ensure_recv(c, r));
  if (r.gather_next) {  // where the next pass will find each tile's records
    lsb::GatherSrc& g = r.gsrc;
    g.R = r.R;
    g.A = r.A;
    g.self_adj = r.send_displs[me] - r.recv_displs[me];
    g.place = r.place;
    g.gstart = r.gstart;
    g.gadj = r.gstart + (size_t)c->P * c->nb;
    g.desc = r.gdesc;
    g.P = c->P;
    g.nb = c->nb;
    g.me = me;
    g.self_in_a = !(c->self_coll && c->mode != Mode::kLoopback);
    HIP_TRY(hipSetDevice(r.dev));
    Timer t(c, &r, LSB_K_EXCHANGE);
    HIP_TRY(lsb::launch_gather_desc(g, r.here, r.gdesc, r.stream));
  }
  if (c->self_coll && c->mode != Mode::kLoopback) return LSB_OK;
  HIP_TRY(hipSetDevice(r.dev));
  HIP_TRY(hipEventRecord(r.pevent, r.stream));  // plan kernels done
  HIP_TRY(hipStreamWaitEvent(r.pstream, r.pevent, 0));
  return place_range(c, r, shift, me, r.A + r.send_displs[me], r.recv_displs[me],
                     r.recv_counts[me]);
}

// Slice j of every peer segment has arrived in R (r.stream): place it on
// r.pstream while r.stream carries slice j + 1.
int place_slice(lsb_ctx* c, Rank& r, int shift, int j) {
  HIP_TRY(hipSetDevice(r.dev));
  HIP_TRY(hipEventRecord(r.pevent, r.stream));
  HIP_TRY(hipStreamWaitEvent(r.pstream, r.pevent, 0));
  const bool self_in_r = c->self_coll && c->mode != Mode::kLoopback;
  for (int s = 0; s < c->P; ++s) {
    if (s == r.rank && !self_in_r) continue;
    const int64_t lo = part(r.recv_counts[s], j, slices_of(c));
    const int64_t hi = part(r.recv_counts[s], j + 1, slices_of(c));
    LSB_TRY(place_range(c, r, shift, s, r.R + r.recv_displs[s] + lo, r.recv_displs[s] + lo, hi - lo));
  }
  return LSB_OK;
}

// ---- exchange: in-process loopback --------------------------------------
// The same slices and placement as the RCCL path; device copies stand in for
// ncclAllToAllv.
int exchange_loopback(lsb_ctx* c, int digit) {
  const int shift = digit * c->bits;
  const size_t nb = (size_t)c->nb;
  // counts of every rank into every rank's gather matrix (the device copies
  // stand in for ncclAllGather), then every rank's device plan.
  std::vector<const uint64_t*> counts(c->ranks.size(), nullptr);
  for (Rank& r : c->ranks) LSB_TRY(digit_counts(c, r, digit, &counts[r.rank]));
  for (Rank& r : c->ranks) {
    HIP_TRY(hipSetDevice(r.dev));
    HIP_TRY(hipStreamSynchronize(r.stream));
  }
  for (Rank& q : c->ranks) {
    HIP_TRY(hipSetDevice(q.dev));
    for (Rank& s : c->ranks)
      HIP_TRY(hipMemcpyAsync(q.gather + (size_t)s.rank * nb, counts[s.rank], sizeof(uint64_t) * nb,
                             hipMemcpyDefault, q.stream));
    LSB_TRY(plan_launch(c, q));
  }
  for (Rank& r : c->ranks) {
    HIP_TRY(hipSetDevice(r.dev));
    HIP_TRY(hipStreamSynchronize(r.stream));
    plan_fetch(c, r);
  }
  for (Rank& q : c->ranks)
    for (Rank& s : c->ranks)
      if (s.send_counts[q.rank] != q.recv_counts[s.rank])
        return fail(LSB_ERR_STATE, "exchange_loopback", "send/recv count mismatch");
  for (Rank& r : c->ranks) LSB_TRY(place_self(c, r, shift));
  // all-to-all-v, slice by slice: part j of segment q of rank s's
  // digit-ordered A -> rank q's R.
  for (int j = 0; j < slices_of(c); ++j) {
    for (Rank& q : c->ranks) {
      Timer t(c, &q, LSB_K_EXCHANGE);
      HIP_TRY(hipSetDevice(q.dev));
      for (Rank& s : c->ranks) {
        if (s.rank == q.rank) continue;
        const int64_t cnt = s.send_counts[q.rank];
        const int64_t lo = part(cnt, j, slices_of(c)), hi = part(cnt, j + 1, slices_of(c));
        if (hi <= lo) continue;
        HIP_TRY(hipMemcpyAsync(q.R + q.recv_displs[s.rank] + lo, s.A + s.send_displs[q.rank] + lo,
                               (size_t)(hi - lo) * sizeof(Elem), hipMemcpyDefault, q.stream));
      }
    }
    for (Rank& q : c->ranks) LSB_TRY(place_slice(c, q, shift, j));
  }
  // Every rank's copies out of A must be done before any rank's next pass
  // rewrites that A (it becomes B after the swap).
  for (Rank& r : c->ranks) {
    LSB_TRY(join_place(r));
    HIP_TRY(hipStreamSynchronize(r.stream));
    end_placement(r);
  }
  return LSB_OK;
}

// ---- collectives of a one-rank-per-process context -------------------------
// RCCL on the rank's stream (Mode::kRccl), or the caller's host callbacks
// (Mode::kOps: sync the stream, stage through host memory, call, copy back).
int ops_fail(const char* what) { return fail(LSB_ERR_RCCL, what, "comm callback failed"); }

// count u64 per rank into recv[P * count]; in place when send == recv + rank * count.
int coll_allgather_u64(lsb_ctx* c, Rank& r, const uint64_t* send, uint64_t* recv, size_t count) {
  if (c->mode == Mode::kRccl) {
    RCCL_TRY(ncclAllGather(send, recv, count, ncclUint64, c->comm, r.stream));
    return LSB_OK;
  }
  std::vector<uint64_t> hs(count), hr(count * c->P);
  HIP_TRY(hipMemcpyAsync(hs.data(), send, count * 8, hipMemcpyDeviceToHost, r.stream));
  HIP_TRY(hipStreamSynchronize(r.stream));
  if (c->ops.allgather(c->ops.user, hs.data(), hr.data(), count * 8) != 0) return ops_fail("allgather");
  HIP_TRY(hipMemcpyAsync(recv, hr.data(), count * 8 * c->P, hipMemcpyHostToDevice, r.stream));
  HIP_TRY(hipStreamSynchronize(r.stream));
  return LSB_OK;
}

// MPI_Alltoallv semantics in uint64 units (counts and displacements).
int coll_alltoallv_u64(lsb_ctx* c, Rank& r, const uint64_t* send, const size_t* sc,
                       const size_t* sd, uint64_t* recv, const size_t* rc, const size_t* rd) {
  const int P = c->P;
  int64_t call_bytes = 0;
  for (int q = 0; q < P; ++q) call_bytes += (int64_t)sc[q] * 8;
  c->coll_calls += 1;
  c->coll_bytes += call_bytes;
  c->coll_max = std::max(c->coll_max, call_bytes);
  if (c->mode == Mode::kRccl) {
    if (!c->p2p) {
      RCCL_TRY(ncclAllToAllv(send, sc, sd, recv, rc, rd, ncclUint64, c->comm, r.stream));
    } else {  // the same exchange as explicit grouped point-to-point calls
      RCCL_TRY(ncclGroupStart());
      for (int q = 0; q < P; ++q) {
        if (sc[q] > 0) RCCL_TRY(ncclSend(send + sd[q], sc[q], ncclUint64, q, c->comm, r.stream));
        if (rc[q] > 0) RCCL_TRY(ncclRecv(recv + rd[q], rc[q], ncclUint64, q, c->comm, r.stream));
      }
      RCCL_TRY(ncclGroupEnd());
    }
    return LSB_OK;
  }
  size_t send_end = 0, recv_end = 0;
  for (int q = 0; q < P; ++q) {
    if (sc[q]) send_end = std::max(send_end, sd[q] + sc[q]);
    if (rc[q]) recv_end = std::max(recv_end, rd[q] + rc[q]);
  }
  std::vector<uint64_t> hs(std::max<size_t>(send_end, 1)), hr(std::max<size_t>(recv_end, 1));
  std::vector<size_t> sb(P), sdb(P), rb(P), rdb(P);
  for (int q = 0; q < P; ++q) {
    if (sc[q])
      HIP_TRY(hipMemcpyAsync(hs.data() + sd[q], send + sd[q], sc[q] * 8, hipMemcpyDeviceToHost,
                             r.stream));
    sb[q] = sc[q] * 8;
    sdb[q] = sd[q] * 8;
    rb[q] = rc[q] * 8;
    rdb[q] = rd[q] * 8;
  }
  HIP_TRY(hipStreamSynchronize(r.stream));
  if (c->ops.alltoallv(c->ops.user, hs.data(), sb.data(), sdb.data(), hr.data(), rb.data(),
                       rdb.data()) != 0)
    return ops_fail("alltoallv");
  for (int q = 0; q < P; ++q)
    if (rc[q])
      HIP_TRY(hipMemcpyAsync(recv + rd[q], hr.data() + rd[q], rc[q] * 8, hipMemcpyHostToDevice,
                             r.stream));
  HIP_TRY(hipStreamSynchronize(r.stream));
  return LSB_OK;
}

// ---- exchange: peer stores (opt-in, LSB_OPT_EXCHANGE_PEER) ----------------
// Each rank writes its records straight into its owners' receiving buffers
// (shmem_putmem / MPI_Put in the reference, shmem/shmem_lsbsort.cpp:441-456,
// mpi/mpi_lsbsort_onesided.cpp:487-509): no R buffer, no all-to-all, no
// placement pass.  Ordering: the counts all-gather cannot complete before
// every rank's local pass has (stream order), so no store lands in a buffer
// still being read; a barrier after the stores orders them before any
// rank's next pass.  Visibility across GPUs is made explicit rather than left
// to kernel boundaries: k_peer_scatter ends every workgroup with a
// system-scope release (L2 write-back of the XCD), and after the barrier the
// owner runs a system-scope acquire on every XCD (L2 invalidate) before its
// next pass reads the buffer.

// Every rank's two physical buffers as this process sees them.
int peer_setup(lsb_ctx* c) {
  if (c->peer_ready) return LSB_OK;
  const int P = c->P;
  if (c->mode == Mode::kLoopback) {
    for (Rank& r : c->ranks) {
      r.peer0.assign(P, nullptr);
      r.peer1.assign(P, nullptr);
      HIP_TRY(hipSetDevice(r.dev));
      for (Rank& q : c->ranks) {
        r.peer0[q.rank] = q.buf[0];
        r.peer1[q.rank] = q.buf[1];
        if (q.dev != r.dev) {
          hipError_t e = hipDeviceEnablePeerAccess(q.dev, 0);
          if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
            return fail(LSB_ERR_HIP, "hipDeviceEnablePeerAccess", hipGetErrorString(e));
          (void)hipGetLastError();
        }
      }
    }
    c->peer_ready = true;
    return LSB_OK;
  }
  // One rank per process: IPC handles of both buffers, all-gathered.
  Rank& r = c->ranks[0];
  HIP_TRY(hipSetDevice(r.dev));
  static_assert(sizeof(hipIpcMemHandle_t) % 8 == 0, "handle in u64 words");
  constexpr size_t kW = sizeof(hipIpcMemHandle_t) / 8;  // words per handle
  std::vector<uint64_t> mine(2 * kW), all((size_t)P * 2 * kW);
  HIP_TRY(hipIpcGetMemHandle(reinterpret_cast<hipIpcMemHandle_t*>(mine.data()), r.buf[0]));
  HIP_TRY(hipIpcGetMemHandle(reinterpret_cast<hipIpcMemHandle_t*>(mine.data() + kW), r.buf[1]));
  uint64_t* d = r.gather;  // >= P * 2 * kW words (P * nb, nb >= 256)
  HIP_TRY(hipMemcpyAsync(d + (size_t)r.rank * 2 * kW, mine.data(), 2 * kW * 8,
                         hipMemcpyHostToDevice, r.stream));
  LSB_TRY(coll_allgather_u64(c, r, d + (size_t)r.rank * 2 * kW, d, 2 * kW));
  HIP_TRY(hipMemcpyAsync(all.data(), d, all.size() * 8, hipMemcpyDeviceToHost, r.stream));
  HIP_TRY(hipStreamSynchronize(r.stream));
  r.peer0.assign(P, nullptr);
  r.peer1.assign(P, nullptr);
  for (int q = 0; q < P; ++q) {
    if (q == r.rank) {
      r.peer0[q] = r.buf[0];
      r.peer1[q] = r.buf[1];
      continue;
    }
    for (int k = 0; k < 2; ++k) {
      hipIpcMemHandle_t h;
      memcpy(&h, all.data() + ((size_t)q * 2 + k) * kW, sizeof h);
      void* p = nullptr;
      HIP_TRY(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
      r.ipc_opened.push_back(p);
      (k == 0 ? r.peer0 : r.peer1)[q] = static_cast<Elem*>(p);
    }
  }
  c->peer_ready = true;
  return LSB_OK;
}

// All ranks' stores are done: loopback waits for every stream, one rank per
// process runs a barrier collective after its own stores.
int peer_barrier(lsb_ctx* c) {
  if (c->mode == Mode::kLoopback) {
    for (Rank& r : c->ranks) {
      HIP_TRY(hipSetDevice(r.dev));
      HIP_TRY(hipStreamSynchronize(r.stream));
    }
    return LSB_OK;
  }
  Rank& r = c->ranks[0];
  HIP_TRY(hipSetDevice(r.dev));
  if (c->mode == Mode::kRccl) {
    RCCL_TRY(ncclAllReduce(r.check, r.check, 1, ncclUint64, ncclSum, c->comm, r.stream));
    return LSB_OK;
  }
  HIP_TRY(hipStreamSynchronize(r.stream));
  return c->ops.barrier(c->ops.user) == 0 ? LSB_OK : ops_fail("barrier");
}

int exchange_peer(lsb_ctx* c, int digit) {
  const int shift = digit * c->bits;
  const size_t nb = (size_t)c->nb;
  LSB_TRY(peer_setup(c));
  // counts of every rank into every local rank's gather matrix
  if (c->mode == Mode::kLoopback) {
    std::vector<const uint64_t*> counts(c->ranks.size(), nullptr);
    for (Rank& r : c->ranks) LSB_TRY(digit_counts(c, r, digit, &counts[r.rank]));
    for (Rank& r : c->ranks) {
      HIP_TRY(hipSetDevice(r.dev));
      HIP_TRY(hipStreamSynchronize(r.stream));
    }
    for (Rank& q : c->ranks) {
      HIP_TRY(hipSetDevice(q.dev));
      for (Rank& s : c->ranks)
        HIP_TRY(hipMemcpyAsync(q.gather + (size_t)s.rank * nb, counts[s.rank],
                               sizeof(uint64_t) * nb, hipMemcpyDefault, q.stream));
    }
  } else {
    Rank& r = c->ranks[0];
    const uint64_t* counts = nullptr;
    LSB_TRY(digit_counts(c, r, digit, &counts));
    HIP_TRY(hipSetDevice(r.dev));
    Timer t(c, &r, LSB_K_EXCHANGE);
    LSB_TRY(coll_allgather_u64(c, r, counts, r.gather, nb));
  }
  for (Rank& r : c->ranks) {
    HIP_TRY(hipSetDevice(r.dev));
    if (!r.peer_base) {
      HIP_TRY(hipMalloc(reinterpret_cast<void**>(&r.peer_base), sizeof(int64_t) * nb));
    }
    // Every rank swaps alike, so B is the same physical buffer index everywhere.
    const bool free1 = r.B == r.buf[1];
    Timer t(c, &r, LSB_K_EXCHANGE);
    HIP_TRY(lsb::launch_peer_exchange(r.A, r.here, shift, c->nb, r.gather, c->P, r.rank, c->per,
                                      (free1 ? r.peer1 : r.peer0).data(), r.peer_base,
                                      r.stream));
  }
  LSB_TRY(peer_barrier(c));
  for (Rank& r : c->ranks) {
    // Acquire what the peers released (k_peer_scatter's system-scope fence).
    HIP_TRY(hipSetDevice(r.dev));
    HIP_TRY(lsb::launch_system_acquire(r.stream));
    std::swap(r.A, r.B);
  }
  return LSB_OK;
}

// ---- exchange: one rank per process (RCCL, or the caller's collectives) ----
int exchange_rccl(lsb_ctx* c, int digit) {
  const int shift = digit * c->bits;
  const int P = c->P;
  const size_t nb = (size_t)c->nb;
  Rank& r = c->ranks[0];
  const uint64_t* counts = nullptr;
  LSB_TRY(digit_counts(c, r, digit, &counts));
  HIP_TRY(hipSetDevice(r.dev));
  {
    Timer t(c, &r, LSB_K_EXCHANGE);
    LSB_TRY(coll_allgather_u64(c, r, counts, r.gather, nb));
  }
  LSB_TRY(plan_launch(c, r));
  HIP_TRY(hipStreamSynchronize(r.stream));
  plan_fetch(c, r);
  LSB_TRY(place_self(c, r, shift));
  const int me = r.rank;
  // ncclAllToAllv per slice (the reference's MPI_Alltoallv,
  // mpi/mpi_lsbsort.cpp:316-324), in uint64 units; the self entry is 0
  // because the self segment was placed straight out of A (unless
  // LSB_OPT_EXCHANGE_SELF sends it through the collective too).
  const bool skip_self = !c->self_coll;
  std::vector<size_t> sc(P), sd(P), rc(P), rdp(P);
  for (int j = 0; j < slices_of(c); ++j) {
    {
      Timer t(c, &r, LSB_K_EXCHANGE);
      for (int q = 0; q < P; ++q) {
        const int64_t slo = part(r.send_counts[q], j, slices_of(c));
        const int64_t shi = part(r.send_counts[q], j + 1, slices_of(c));
        const int64_t rlo = part(r.recv_counts[q], j, slices_of(c));
        const int64_t rhi = part(r.recv_counts[q], j + 1, slices_of(c));
        sc[q] = q == me && skip_self ? 0 : (size_t)(shi - slo) * 2;
        rc[q] = q == me && skip_self ? 0 : (size_t)(rhi - rlo) * 2;
        sd[q] = (size_t)(r.send_displs[q] + slo) * 2;
        rdp[q] = (size_t)(r.recv_displs[q] + rlo) * 2;
      }
      LSB_TRY(coll_alltoallv_u64(c, r, reinterpret_cast<const uint64_t*>(r.A), sc.data(),
                                 sd.data(), reinterpret_cast<uint64_t*>(r.R), rc.data(),
                                 rdp.data()));
    }
    LSB_TRY(place_slice(c, r, shift, j));
  }
  LSB_TRY(join_place(r));
  end_placement(r);
  return LSB_OK;
}

// One exchange digit: its 8-bit local sub-passes, then (P > 1) the exchange.
// varying: key bits that differ somewhere; a sub-pass whose byte is constant
// is the identity and is skipped (all ~0 = run everything).  want_span: the
// first sub-pass also reduces the key span (lsb_sort, digit 0).
int merge_sort(lsb_ctx* c);
int exchange_digit(lsb_ctx* c, int digit);

int do_pass(lsb_ctx* c, int digit, uint64_t varying = ~0ull, bool want_span = false) {
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

int exchange_digit(lsb_ctx* c, int digit) {
  if (c->peer) return exchange_peer(c, digit);
  if (c->mode != Mode::kLoopback) return exchange_rccl(c, digit);
  return exchange_loopback(c, digit);
}

// ---- single-read passes (P == 1) ------------------------------------------
bool onesweep_applies(const lsb_ctx* c) {
  return c->onesweep && !exchanging(c) && c->ranks.size() == 1 && c->ranks[0].here > 0 &&
         c->ranks[0].here <= lsb::kOnesweepMaxElems;
}

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
int onesweep_launch(lsb_ctx* c, Rank& r, int shift, int next, const uint32_t* hist,
                    uint32_t* next_hist, lsb::OnesweepExtra x) {
  const size_t status_bytes = (size_t)lsb::onesweep_tiles(r.here) * lsb::kBuckets * sizeof(uint32_t);
  if (r.os_dirty) {
    HIP_TRY(hipMemsetAsync(r.os_status, 0, status_bytes, r.stream));
    r.os_epoch = 0;
    r.os_dirty = false;
  }
  uint32_t epoch = r.os_epoch + 1;
  if (epoch >= (1u << 30)) epoch = 2;  // 2^30 is even: keep the alternation
  hipError_t e;
  {
    Timer t(c, &r, LSB_K_SCATTER);
    e = lsb::launch_onesweep(r.A, r.B, r.here, shift, next, hist, next_hist, r.os_status, r.os_ctr,
                             epoch, r.os_ctr + lsb::kOnesweepSubs, r.os_grid, r.stream, x);
  }
  if (e != hipSuccess) {
    (void)hipGetLastError();
    r.os_dirty = true;
    return fail(LSB_ERR_HIP, "launch_onesweep", hipGetErrorString(e));
  }
  r.os_epoch = epoch;
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
int onesweep_digits(lsb_ctx* c, Rank& r, const std::vector<int>& digits, int* passes) {
  uint32_t* hist[2] = {r.os_hist, r.os_hist + lsb::kOnesweepSubs * lsb::kBuckets};
  for (size_t i = 0; i < digits.size(); ++i) {
    const int shift = digits[i] * lsb::kDigitBits;
    const int next = i + 1 < digits.size() ? digits[i + 1] * lsb::kDigitBits : -1;
    begin_pass(c, shift);
    lsb::OnesweepExtra x;
    x.halves = r.os_halves;
    LSB_TRY(onesweep_launch(c, r, shift, next, hist[i & 1], hist[(i + 1) & 1], x));
    ++*passes;
  }
  return LSB_OK;
}

int sort_hybrid_rank(lsb_ctx* c, Rank& r, int* passes, uint64_t* varying);

// lsb_sort when nothing is exchanged: one k_subhist read (digit 0's
// sub-array histogram and the key span), then one k_onesweep per digit that
// varies, each also counting the next such digit over its output.  Same
// output as the reduce-then-scan loop (do_pass).  A constant digit 0 is
// skipped like any other: its pass would be the identity, so the first
// digit that varies is counted by a second k_subhist read (a read, not a
// pass), and that digit's histogram also decides the stage split.
// Rank r alone (its local block); *passes gets the passes it ran, *varying the
// key bits that vary in the block.  LSB_OPT_HYBRID: sort_hybrid_rank.
int sort_onesweep_rank(lsb_ctx* c, Rank& r, int* passes, uint64_t* varying) {
  if (c->hybrid) return sort_hybrid_rank(c, r, passes, varying);
  HIP_TRY(hipSetDevice(r.dev));
  LSB_TRY(onesweep_ensure(r));
  c->pass_cursor = 0;
  c->cur_pass = 0;  // the count reads are filed under the first pass
  HIP_TRY(hipMemsetAsync(r.span, 0, 2 * sizeof(uint64_t), r.stream));
  LSB_TRY(count_byte(c, r, 0, c->skip_constant));
  LSB_TRY(queue_halves(c, r, r.os_hist));
  *varying = ~0ull;
  *passes = 0;
  if (c->skip_constant) {
    HIP_TRY(hipMemcpyAsync(r.span_h, r.span, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, r.stream));
    HIP_TRY(hipStreamSynchronize(r.stream));
    *varying = r.span_h[0] & r.span_h[1];
  }
  const std::vector<int> digits = varying_bytes(*varying);
  if (!digits.empty() && digits[0] != 0) {
    LSB_TRY(count_byte(c, r, digits[0], false));
    LSB_TRY(queue_halves(c, r, r.os_hist));
    LSB_TRY(choose_halves(c, r, false));
  } else {
    LSB_TRY(choose_halves(c, r, c->skip_constant));
  }
  LSB_TRY(onesweep_digits(c, r, digits, passes));
  // The look-back's give-up word, read by lsb_sync.
  HIP_TRY(hipMemcpyAsync(r.os_err_h, r.os_ctr + lsb::kOnesweepSubs, sizeof(uint32_t),
                         hipMemcpyDeviceToHost, r.stream));
  return LSB_OK;
}

// ---- hybrid local sort (LSB_OPT_HYBRID) ------------------------------------
// The same stable order as the LSD passes from fewer passes over HBM
// (lsb_segsort.hip): k_onesweep passes on the k most significant varying
// bytes only, then k_segsort orders every segment (run of records equal on
// those bytes) by the whole key.  k: the fewest top varying bytes whose
// varying bits reach ceil(log2 m), so uniform keys leave segments of about
// one record (2^30 records: k = 4, 0.25 on average; k_segsort's walk then
// costs ~2 LDS reads per record and the pass streams at copy speed.  k = 3,
// 64 per segment, made k_segsort compute-bound: 69 ms against 7 for the
// fourth byte's pass, profiles/r03_h1_probe.log).
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

// The hybrid for rank r.  The k passes leave the input A untouched (A -> B,
// then B <-> R), so when k_segsort meets a segment longer than kSegMax the
// sort starts over from A with the LSD passes; skewed keys (the first
// pass's byte has a bucket over 1/32 of the records, as for the stage
// split: duplicate-heavy keys make long segments) take them directly.  One
// host sync, after k_segsort, reads its error word.
int sort_hybrid_rank(lsb_ctx* c, Rank& r, int* passes, uint64_t* varying) {
  HIP_TRY(hipSetDevice(r.dev));
  LSB_TRY(onesweep_ensure(r));
  LSB_TRY(ensure_recv(c, r));
  c->pass_cursor = 0;
  c->cur_pass = 0;
  const int64_t m = r.here;
  *passes = 0;
  *varying = ~0ull;
  // Count the byte the first pass most likely sorts on (full 64-bit keys)
  // in the same read as the span.
  const std::vector<int> guess = hybrid_bytes(~0ull, m);
  int counted = guess.empty() ? 0 : guess[0];
  HIP_TRY(hipMemsetAsync(r.span, 0, 2 * sizeof(uint64_t), r.stream));
  LSB_TRY(count_byte(c, r, counted, c->skip_constant));
  if (c->skip_constant) {
    HIP_TRY(hipMemcpyAsync(r.span_h, r.span, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, r.stream));
    HIP_TRY(hipStreamSynchronize(r.stream));
    *varying = r.span_h[0] & r.span_h[1];
  }
  const std::vector<int> digits = varying_bytes(*varying);
  const std::vector<int> msd = c->skip_constant ? hybrid_bytes(*varying, m) : guess;
  bool hybrid = msd.size() < digits.size();
  // The first byte sorted on decides the stage split and whether keys are
  // skewed (*skewed: a bucket over 1/32 of the records).
  auto first_hist = [&](int byte, bool* skewed) -> int {
    if (byte != counted) {
      LSB_TRY(count_byte(c, r, byte, false));
      counted = byte;
    }
    HIP_TRY(hipMemcpyAsync(r.os_hist_h, r.os_hist, sizeof(uint32_t) * lsb::kOnesweepSubs * lsb::kBuckets,
                           hipMemcpyDeviceToHost, r.stream));
    HIP_TRY(hipStreamSynchronize(r.stream));
    const int h = lsb::onesweep_halves_for(r.os_hist_h, m);
    r.os_halves = c->os_split == 0 ? h : (c->os_split == 2 ? 2 : 1);
    *skewed = h == 2;
    return LSB_OK;
  };
  bool skewed = false;
  if (hybrid && !msd.empty()) {
    LSB_TRY(first_hist(msd[0], &skewed));
    if (skewed) hybrid = false;
  }
  if (!hybrid) {
    if (!digits.empty()) LSB_TRY(first_hist(digits[0], &skewed));
    LSB_TRY(onesweep_digits(c, r, digits, passes));
  } else {
    // The k passes: A -> B, then B <-> R; the input X0 is kept.  The last
    // one also orders every segment inside its tile (SegPass) and k_segfix
    // merges the segments split between tiles; LSB_OPT_HYBRID = 2, or the
    // split stage, leaves the segments to a k_segsort pass instead.
    Elem* const X0 = r.A;
    Elem* const X1 = r.B;
    Elem* const X2 = r.R;
    uint64_t pmask = 0;
    for (int b : msd) pmask |= (uint64_t)(lsb::kBuckets - 1) << (b * lsb::kDigitBits);
    uint32_t* err = r.os_ctr + lsb::kOnesweepSubs + 1;
    const bool fuse = c->hybrid == 1 && r.os_halves == 1 && !msd.empty();
    lsb::SegPass sp;
    if (fuse) {
      if (!r.seg_base) LSB_TRY(dev_alloc(&r.seg_base, (size_t)lsb::kOnesweepSubs * lsb::kBuckets));
      sp.pmask = pmask;
      sp.rmask = pmask & ~((uint64_t)(lsb::kBuckets - 1) << (msd.back() * lsb::kDigitBits));
      sp.base = r.seg_base;
      sp.err = err;
    }
    HIP_TRY(hipMemsetAsync(err, 0, sizeof(uint32_t), r.stream));
    uint32_t* hist[2] = {r.os_hist, r.os_hist + lsb::kOnesweepSubs * lsb::kBuckets};
    const Elem* seg_in = nullptr;  // the last pass's input, read by k_segfix
    for (size_t i = 0; i < msd.size(); ++i) {
      const int shift = msd[i] * lsb::kDigitBits;
      const int next = i + 1 < msd.size() ? msd[i + 1] * lsb::kDigitBits : -1;
      begin_pass(c, shift);
      lsb::OnesweepExtra x;
      x.halves = r.os_halves;
      if (fuse && i + 1 == msd.size()) {
        x.seg = &sp;
        seg_in = r.A;
      }
      LSB_TRY(onesweep_launch(c, r, shift, next, hist[i & 1], hist[(i + 1) & 1], x));
      ++*passes;
      if (i == 0) r.B = X2;  // A is X1 now
    }
    if (msd.empty()) r.B = X1;
    auto sync_err = [&](uint32_t* v) -> int {
      HIP_TRY(hipMemcpyAsync(r.os_err_h + 1, err, sizeof(uint32_t), hipMemcpyDeviceToHost, r.stream));
      HIP_TRY(hipStreamSynchronize(r.stream));
      *v = r.os_err_h[1];
      return LSB_OK;
    };
    bool sorted = false;
    if (fuse) {
      {
        Timer t(c, &r, LSB_K_SEGSORT);
        // one wave per tile boundary, 32 waves per CU
        HIP_TRY(lsb::launch_segfix(seg_in, r.A, m, msd.back() * lsb::kDigitBits, r.os_status, sp,
                                   16 * r.os_grid, r.stream));
      }
      uint32_t e = 0;
      LSB_TRY(sync_err(&e));
      sorted = e == 0;
    }
    if (!sorted) {
      // k_segsort: r.A is stably sorted by pmask (the fused pass's segments
      // too, in or out of order).
      HIP_TRY(hipMemsetAsync(err, 0, sizeof(uint32_t), r.stream));
      begin_pass(c, 64);
      {
        Timer t(c, &r, LSB_K_SEGSORT);
        HIP_TRY(lsb::launch_segsort(r.A, r.B, m, pmask, err, 3 * r.os_grid / 2, r.stream));
      }
      count_pass_elems(c, m, false);
      ++*passes;
      uint32_t e = 0;
      LSB_TRY(sync_err(&e));
      if (e == 0) {
        std::swap(r.A, r.B);
        sorted = true;
      }
    }
    if (sorted) {
      r.R = (X0 != r.A && X0 != r.B) ? X0 : (X1 != r.A && X1 != r.B) ? X1 : X2;
    } else {  // a segment too long for the segment sorts: the LSD passes over the kept input
      r.A = X0;
      r.B = X1;
      r.R = X2;
      counted = -1;
      if (!digits.empty()) LSB_TRY(first_hist(digits[0], &skewed));
      LSB_TRY(onesweep_digits(c, r, digits, passes));
    }
  }
  // The look-back's give-up word, read by lsb_sync.
  HIP_TRY(hipMemcpyAsync(r.os_err_h, r.os_ctr + lsb::kOnesweepSubs, sizeof(uint32_t),
                         hipMemcpyDeviceToHost, r.stream));
  return LSB_OK;
}

int sort_onesweep(lsb_ctx* c) {
  return sort_onesweep_rank(c, c->ranks[0], &c->last_local_passes, &c->last_varying);
}

// ---- per-digit exchange with single-read local passes ----------------------
// lsb_sort of the per-digit exchange forms (radix_bits 8 / 16, P > 1): the
// reference's pass loop (mpi/mpi_lsbsort.cpp:580-585), each exchange digit's
// localShuffle (:213-247) as one or two k_onesweep passes instead of count +
// scan + scatter.  One k_subhist read per sort gives the first byte's
// sub-array histogram and the key span; after that every histogram is
// counted by whatever writes the records: the previous local pass, or the
// exchange's k_place launches (their output is the next pass's input).  The
// last local pass of an exchange digit hands the exchange its counts: the
// 256 totals, or (16-bit digits) the 65536 counts, from the high-byte pass.
bool exchange_onesweep_applies(const lsb_ctx* c) {
  if (!c->onesweep || !exchanging(c) || c->bits == 64) return false;
  for (const Rank& r : c->ranks)
    if (r.here > lsb::kOnesweepMaxElems) return false;
  return true;
}

// One local pass of rank r on the byte at `shift`; next >= 0: also count the
// byte at `next` over the output (the next local pass follows directly).
int local_pass_os(lsb_ctx* c, Rank& r, int shift, int next, lsb::OnesweepExtra extra) {
  HIP_TRY(hipSetDevice(r.dev));
  extra.halves = r.os_halves;
  r.starts_fused = false;
  const int64_t m = r.here;
  if (m == 0) {
    if (extra.totals) HIP_TRY(hipMemsetAsync(extra.totals, 0, sizeof(uint64_t) * lsb::kBuckets, r.stream));
    if (extra.count16) HIP_TRY(hipMemsetAsync(extra.count16, 0, sizeof(uint64_t) * 65536, r.stream));
    r.os_valid = -1;
    return LSB_OK;
  }
  uint32_t* hist[2] = {r.os_hist, r.os_hist + lsb::kOnesweepSubs * lsb::kBuckets};
  if (r.gather_pending) {  // the exchange's count-only placement counted this byte
    if (r.os_valid != shift) {
      r.gather_pending = false;
      return fail(LSB_ERR_STATE, "local_pass_os", "gathered pass without its count");
    }
    extra.gather = &r.gsrc;
  } else if (r.os_valid != shift) {  // nothing counted this byte over A: read it
    Timer t(c, &r, LSB_K_UPSWEEP);
    HIP_TRY(lsb::launch_subhist(r.A, m, shift, r.os_grid, hist[r.os_cur], nullptr, r.stream));
  }
  const int rc = onesweep_launch(c, r, shift, next, hist[r.os_cur], hist[r.os_cur ^ 1], extra);
  r.gather_pending = false;
  LSB_TRY(rc);
  if (next >= 0) {
    r.os_cur ^= 1;
    r.os_valid = next;
  } else {
    r.os_valid = -1;
  }
  return LSB_OK;
}

int gather_span(lsb_ctx* c, uint64_t* kor, uint64_t* knor);

int sort_exchange_onesweep(lsb_ctx* c) {
  const int D = 64 / c->bits, subs = c->bits / lsb::kDigitBits;
  c->pass_cursor = 0;
  c->cur_pass = 0;
  for (Rank& r : c->ranks) {
    HIP_TRY(hipSetDevice(r.dev));
    LSB_TRY(onesweep_ensure(r));
    HIP_TRY(hipMemsetAsync(r.span, 0, 2 * sizeof(uint64_t), r.stream));
    r.os_cur = 0;
    r.os_valid = -1;
    if (r.here > 0) {
      Timer t(c, &r, LSB_K_UPSWEEP);
      HIP_TRY(lsb::launch_subhist(r.A, r.here, 0, r.os_grid, r.os_hist,
                                  c->skip_constant ? r.span : nullptr, r.stream));
      r.os_valid = 0;
    }
    LSB_TRY(queue_halves(c, r, r.os_hist));
  }
  uint64_t varying = ~0ull;
  if (c->skip_constant) {
    uint64_t kor = 0, knor = 0;
    LSB_TRY(gather_span(c, &kor, &knor));
    varying = kor & knor;
  }
  c->last_varying = varying;
  // Local passes in order; an exchange follows the last one of each digit.
  // A digit on which every key agrees needs neither (its stable pass and its
  // (digit, rank) exchange order are the identity), nor does a constant byte
  // its local pass.
  struct Step {
    int shift, digit;
    bool exch;
  };
  std::vector<Step> steps;
  const uint64_t dmask = (1ull << c->bits) - 1;
  for (int d = 0; d < D; ++d) {
    if (((varying >> (d * c->bits)) & dmask) == 0) continue;
    for (int sub = 0; sub < subs; ++sub) {
      const int shift = d * c->bits + sub * lsb::kDigitBits;
      if (((varying >> shift) & (lsb::kBuckets - 1)) != 0) steps.push_back({shift, d, false});
    }
    steps.back().exch = true;
  }
  // The stage split is decided from the first byte that is sorted on: when
  // byte 0 is constant, that byte is counted now (its pass reads the
  // histogram instead of counting it again).  gather_span syncs only the
  // streams it reads from: each rank syncs in choose_halves.
  for (Rank& r : c->ranks) {
    HIP_TRY(hipSetDevice(r.dev));
    if (!steps.empty() && steps[0].shift != 0 && r.here > 0) {
      {
        Timer t(c, &r, LSB_K_UPSWEEP);
        HIP_TRY(lsb::launch_subhist(r.A, r.here, steps[0].shift, r.os_grid, r.os_hist, nullptr,
                                    r.stream));
      }
      r.os_cur = 0;
      r.os_valid = steps[0].shift;
      LSB_TRY(queue_halves(c, r, r.os_hist));
    }
    LSB_TRY(choose_halves(c, r, false));
  }
  for (size_t i = 0; i < steps.size(); ++i) {
    const Step& st = steps[i];
    const int after = i + 1 < steps.size() ? steps[i + 1].shift : -1;
    // 16-bit digit: its high-byte pass counts the 65536 digits (a constant
    // high byte leaves the count to digit_counts' read of A).
    const bool c16 = c->bits == 16 && st.exch && st.shift == st.digit * 16 + lsb::kDigitBits;
    begin_pass(c, st.shift);
    for (Rank& r : c->ranks) {
      lsb::OnesweepExtra x;
      if (st.exch && c->bits == 8) x.totals = r.totals;
      if (c16) x.count16 = r.totals16;
      r.counts_ready = c16;
      LSB_TRY(local_pass_os(c, r, st.shift, st.exch ? -1 : after, x));
    }
    ++c->last_local_passes;
    if (!st.exch) continue;
    for (Rank& r : c->ranks) {
      r.place_next = c->peer || r.here == 0 ? -1 : after;
      // Not with the split stage (skewed keys): its gathered instances spill.
      r.gather_next = c->gather && r.place_next >= 0 && r.os_halves == 1;
      r.place_hist = nullptr;
      if (r.place_next >= 0) {
        r.place_hist = r.os_hist + (size_t)(r.os_cur ^ 1) * lsb::kOnesweepSubs * lsb::kBuckets;
        HIP_TRY(hipSetDevice(r.dev));
        HIP_TRY(hipMemsetAsync(r.place_hist, 0, sizeof(uint32_t) * lsb::kOnesweepSubs * lsb::kBuckets,
                               r.stream));
      }
    }
    ++c->last_exchanges;
    const int rc = exchange_digit(c, st.digit);
    for (Rank& r : c->ranks) {
      if (rc == LSB_OK && r.place_next >= 0) {
        r.os_cur ^= 1;
        r.os_valid = r.place_next;
      } else {
        r.os_valid = -1;
      }
      r.place_next = -1;
      r.place_hist = nullptr;
      r.counts_ready = false;
      r.gather_next = false;
      if (rc != LSB_OK) r.gather_pending = false;
    }
    LSB_TRY(rc);
  }
  // The look-back's give-up word, read by lsb_sync.
  for (Rank& r : c->ranks) {
    if (r.here == 0) continue;
    HIP_TRY(hipSetDevice(r.dev));
    HIP_TRY(hipMemcpyAsync(r.os_err_h, r.os_ctr + lsb::kOnesweepSubs, sizeof(uint32_t),
                           hipMemcpyDeviceToHost, r.stream));
  }
  return LSB_OK;
}

// ---- whole-key exchange (radix_bits = 64) ----------------------------------
// globalShuffle with a 64-bit digit (mpi/mpi_lsbsort.cpp:481-577 with one
// pass): each rank sorts its block locally on the whole key, the ranks find
// where the global positions q * per fall (a splitter search over the sorted
// blocks, in place of the count transposes and scan of :327-479), every rank
// sends each owner one contiguous range (one all-to-all-v for the whole sort,
// :316-324), and each owner merges its P sorted runs in rank order (the
// placement of :568-575).  Same output as 64 / 8 or 64 / 16 exchanges: the
// stable order by key, ties by input position.

// Cut positions of the exchange: owner q's block [q * per, q * per + here_q)
// is cut into S slices (sub-blocks) at q * per + part(here_q, j, S); cut k =
// q * S + j, plus k = P * S at n.  Every cut strictly inside (0, n) is a
// target of the splitter search.  S = 1 gives the owner boundaries q * per.
// Slices let the owner merge slice j while slice j + 1 is on the wire.
struct MergeGeom {
  int S = 1;
  std::vector<int64_t> pos;   // [P * S + 1] global cut positions, nondecreasing
  std::vector<int> target;    // cut indices k with 0 < pos[k] < n (splitter targets)
};

MergeGeom merge_geometry(int64_t n, int P, int slices) {
  MergeGeom g;
  const int64_t per = div_ceil(n, P);
  g.S = std::max(1, std::min(slices, lsb::kMergeMaxCuts / P));
  g.pos.resize((size_t)P * g.S + 1);
  for (int q = 0; q < P; ++q) {
    const int64_t h = here_of(n, P, q);
    for (int j = 0; j < g.S; ++j)
      g.pos[(size_t)q * g.S + j] = std::min(n, (int64_t)q * per + part(h, j, g.S));
  }
  g.pos[(size_t)P * g.S] = n;
  for (size_t k = 0; k < g.pos.size(); ++k)
    if (g.pos[k] > 0 && g.pos[k] < n) g.target.push_back((int)k);
  return g;
}

// Host side of the plan: from every rank's {#keys < k*_t, #keys <= k*_t}
// (fin[(s * Q + t) * 2 + {0,1}], t over g.target) the cut of source s at
// position T is
//   below_s + min(equal_s, max(0, T - sum_s below_s - sum_{s' < s} equal_s'))
// (equal keys in rank order = input order).  cut[s * (K + 1) + k].
int merge_cuts(int64_t n, int P, const MergeGeom& g, const uint64_t* fin, std::vector<int64_t>& cut) {
  const size_t K1 = g.pos.size();
  const int Q = (int)g.target.size();
  cut.assign((size_t)P * K1, 0);
  for (int s = 0; s < P; ++s)
    for (size_t k = 0; k < K1; ++k) cut[s * K1 + k] = g.pos[k] >= n ? here_of(n, P, s) : 0;
  for (int t = 0; t < Q; ++t) {
    const int k = g.target[t];
    const int64_t T = g.pos[k];
    int64_t below = 0, all = 0;
    for (int s = 0; s < P; ++s) {
      const uint64_t b = fin[((size_t)s * Q + t) * 2], u = fin[((size_t)s * Q + t) * 2 + 1];
      if (b > u || (int64_t)u > here_of(n, P, s))
        return fail(LSB_ERR_INVALID, "plan_merge", "counts out of range");
      below += (int64_t)b;
      all += (int64_t)u;
    }
    if (!(below <= T && T < all)) return fail(LSB_ERR_INVALID, "plan_merge", "target not bracketed");
    int64_t rem = T - below;
    for (int s = 0; s < P; ++s) {
      const int64_t b = (int64_t)fin[((size_t)s * Q + t) * 2];
      const int64_t take = std::min((int64_t)fin[((size_t)s * Q + t) * 2 + 1] - b, rem);
      cut[s * K1 + k] = b + take;
      rem -= take;
    }
  }
  for (int s = 0; s < P; ++s)
    for (size_t k = 0; k + 1 < K1; ++k)
      if (cut[s * K1 + k + 1] < cut[s * K1 + k])
        return fail(LSB_ERR_INVALID, "plan_merge", "cuts not monotone");
  return LSB_OK;
}

// Owner-level counts of rank `me` (lsb_plan_merge): send [cut_q, cut_{q+1}) to
// q, receive [cut_me, cut_{me+1}) of every s.
int merge_owner_counts(int64_t n, int P, int me, const MergeGeom& g, const std::vector<int64_t>& cut,
                       int64_t* sc, int64_t* sd, int64_t* rc, int64_t* rd) {
  const size_t K1 = g.pos.size();
  const int S = g.S;
  int64_t a = 0, b = 0;
  for (int q = 0; q < P; ++q) {
    sc[q] = cut[(size_t)me * K1 + (size_t)(q + 1) * S] - cut[(size_t)me * K1 + (size_t)q * S];
    rc[q] = cut[(size_t)q * K1 + (size_t)(me + 1) * S] - cut[(size_t)q * K1 + (size_t)me * S];
    sd[q] = a;
    rd[q] = b;
    a += sc[q];
    b += rc[q];
  }
  if (b != here_of(n, P, me)) return fail(LSB_ERR_INVALID, "plan_merge", "receive total");
  return LSB_OK;
}

int merge_ensure(lsb_ctx* c, Rank& r, const MergeGeom& g) {
  HIP_TRY(hipSetDevice(r.dev));
  if (!r.R) LSB_TRY(dev_alloc(&r.R, (size_t)c->per));
  if (!r.merge_path)
    LSB_TRY(dev_alloc(&r.merge_path, (size_t)(lsb::merge_tiles(c->per) + 2 * lsb::kMergeMaxPairs + 1)));
  const int Q = (int)g.target.size();
  if (Q == 0 || (r.split_state && r.split_q == Q && r.split_S == g.S)) return LSB_OK;
  for (void* p : {(void*)r.split_state, (void*)r.split_targets, (void*)r.split_cnt,
                  (void*)r.split_gather, (void*)r.split_fin, (void*)r.split_fin_gather})
    (void)hipFree(p);
  (void)hipHostFree(r.split_h);
  const size_t P = (size_t)c->P, K = lsb::kSplitCands;
  LSB_TRY(dev_alloc(&r.split_state, 2 * (size_t)Q));
  LSB_TRY(dev_alloc(&r.split_targets, (size_t)Q));
  LSB_TRY(dev_alloc(&r.split_cnt, (size_t)Q * K));
  LSB_TRY(dev_alloc(&r.split_gather, P * Q * K));
  LSB_TRY(dev_alloc(&r.split_fin, 2 * (size_t)Q));
  LSB_TRY(dev_alloc(&r.split_fin_gather, P * 2 * Q));
  LSB_TRY(host_alloc(&r.split_h, P * 2 * Q));
  std::vector<int64_t> t(Q);
  for (int i = 0; i < Q; ++i) t[i] = g.pos[g.target[i]];
  HIP_TRY(hipMemcpy(r.split_targets, t.data(), sizeof(int64_t) * Q, hipMemcpyHostToDevice));
  r.split_q = Q;
  r.split_S = g.S;
  return LSB_OK;
}

// recv[s * count ..] = send of rank s, for every local rank (loopback: device
// copies once every rank's stream is done; otherwise the collective).
template <typename SendOf, typename RecvOf>
int gather_ranks(lsb_ctx* c, size_t count, SendOf send_of, RecvOf recv_of) {
  if (c->mode != Mode::kLoopback) {
    Rank& r = c->ranks[0];
    HIP_TRY(hipSetDevice(r.dev));
    return coll_allgather_u64(c, r, send_of(r), recv_of(r), count);
  }
  for (Rank& r : c->ranks) {
    HIP_TRY(hipSetDevice(r.dev));
    HIP_TRY(hipStreamSynchronize(r.stream));
  }
  for (Rank& q : c->ranks) {
    HIP_TRY(hipSetDevice(q.dev));
    for (Rank& s : c->ranks)
      HIP_TRY(hipMemcpyAsync(recv_of(q) + (size_t)s.rank * count, send_of(s), count * 8,
                             hipMemcpyDefault, q.stream));
  }
  return LSB_OK;
}

// Rank r's block sorted on the whole key: single-read passes, or count + scan
// + scatter when they do not apply.  Digits constant over the block are skipped.
int sort_local_rank(lsb_ctx* c, Rank& r, int* passes, uint64_t* varying) {
  *passes = 0;
  *varying = 0;
  if (r.here == 0) return LSB_OK;
  if (c->onesweep && r.here <= lsb::kOnesweepMaxElems) return sort_onesweep_rank(c, r, passes, varying);
  HIP_TRY(hipSetDevice(r.dev));
  HIP_TRY(hipMemsetAsync(r.span, 0, 2 * sizeof(uint64_t), r.stream));
  c->pass_cursor = 0;
  begin_pass(c, 0);
  LSB_TRY(local_pass(c, r, 0, c->skip_constant));
  *passes = 1;
  *varying = ~0ull;
  if (c->skip_constant) {
    HIP_TRY(hipMemcpyAsync(r.span_h, r.span, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, r.stream));
    HIP_TRY(hipStreamSynchronize(r.stream));
    *varying = r.span_h[0] & r.span_h[1];
  }
  for (int d = 1; d < 64 / lsb::kDigitBits; ++d) {
    if (((*varying >> (d * lsb::kDigitBits)) & (lsb::kBuckets - 1)) == 0) continue;
    begin_pass(c, d * lsb::kDigitBits);
    LSB_TRY(local_pass(c, r, d * lsb::kDigitBits));
    ++*passes;
  }
  return LSB_OK;
}

// Records of source s in owner r's slice j, where they sit in R, and the
// slice's output range [lo, hi) of r's block.
struct SliceRun {
  int64_t len, roff;
};

void slice_runs(const lsb_ctx* c, const Rank& r, const MergeGeom& g, int j, std::vector<SliceRun>& out,
                int64_t* lo, int64_t* hi) {
  const size_t K1 = g.pos.size();
  const int64_t base = (int64_t)r.rank * c->per;
  const size_t k = (size_t)r.rank * g.S + j;
  *lo = g.pos[k] - base;
  *hi = g.pos[k + 1] - base;
  if (*lo < 0) *lo = 0;
  if (*hi < *lo) *hi = *lo;
  out.resize(c->P);
  int64_t off = *lo;
  for (int s = 0; s < c->P; ++s) {
    out[s].len = r.mcut[s * K1 + k + 1] - r.mcut[s * K1 + k];
    out[s].roff = off;
    off += out[s].len;
  }
}

// Levels of the merge tree over `runs` runs (a single run is one copy level).
int merge_levels(size_t runs) {
  int L = 0;
  for (size_t m = runs; m > 1; m = (m + 1) / 2) ++L;
  return L > 0 ? L : 1;
}

// Merge slice j of owner r on r.pstream: its P runs (source order; my own
// straight out of A) -> F[lo, hi), F = B or R.  A tree of stable two-way
// merges, one launch per level, adjacent runs paired so the lower ranks stay
// on the left; level l writes B (l even) or R (l odd): the slice's own region
// of R is free once level 0 has read it, and A, still being sent from, is
// never written.  A result that ends in the other buffer is copied to F
// (only slices with fewer non-empty runs than the rest).
int merge_slice(lsb_ctx* c, Rank& r, const MergeGeom& g, int j, Elem* F) {
  struct Run {
    const Elem* p;
    int64_t n;
  };
  std::vector<SliceRun> sr;
  int64_t lo = 0, hi = 0;
  slice_runs(c, r, g, j, sr, &lo, &hi);
  if (hi == lo) return LSB_OK;
  const size_t K1 = g.pos.size();
  std::vector<Run> runs;
  for (int s = 0; s < c->P; ++s) {
    if (sr[s].len == 0) continue;
    const bool own = s == r.rank && !(c->self_coll && c->mode != Mode::kLoopback);
    const Elem* p = own ? r.A + r.mcut[s * K1 + (size_t)r.rank * g.S + j] : r.R + sr[s].roff;
    runs.push_back({p, sr[s].len});
  }
  Timer t(c, &r, LSB_K_PLACE, r.pstream);
  // 3 merge workgroups per CU (max_chunks = 2 per CU): 60 KiB of LDS, so
  // RCCL's kernel for the next slice (37 KiB) still finds room on every CU.
  const int grid = 3 * max_chunks_for_device(r.dev) / 2;
  const int L = merge_levels(runs.size());
  for (int level = 0; level < L; ++level) {
    Elem* dst = (level % 2 == 0 ? r.B : r.R) + lo;
    lsb::MergeLevel lv{};
    std::vector<Run> next;
    int64_t off = 0;
    for (size_t i = 0; i < runs.size(); i += 2) {
      const bool pair = i + 1 < runs.size();
      lsb::MergePair& m = lv.p[lv.npairs++];
      m.a = runs[i].p;
      m.na = runs[i].n;
      m.b = pair ? runs[i + 1].p : runs[i].p;
      m.nb = pair ? runs[i + 1].n : 0;
      m.out = dst + off;
      m.tile0 = lv.tiles;
      lv.tiles += lsb::merge_tiles(m.na + m.nb);
      next.push_back({dst + off, m.na + m.nb});
      off += m.na + m.nb;
    }
    HIP_TRY(lsb::launch_merge_level(lv, r.merge_path, grid, r.pstream));
    runs.swap(next);
  }
  Elem* fin = (L - 1) % 2 == 0 ? r.B : r.R;
  if (fin != F)
    HIP_TRY(hipMemcpyAsync(F + lo, fin + lo, (size_t)(hi - lo) * sizeof(Elem), hipMemcpyDeviceToDevice,
                           r.pstream));
  return LSB_OK;
}

// Slice j of the all-to-all has arrived on r.stream: merge it on r.pstream
// while the next slice is on the wire.
int merge_slice_async(lsb_ctx* c, Rank& r, const MergeGeom& g, int j, Elem* F) {
  HIP_TRY(hipSetDevice(r.dev));
  HIP_TRY(hipEventRecord(r.pevent, r.stream));
  HIP_TRY(hipStreamWaitEvent(r.pstream, r.pevent, 0));
  return merge_slice(c, r, g, j, F);
}

int exchange_merge(lsb_ctx* c) {
  const int P = c->P;
  const MergeGeom g = merge_geometry(c->n, P, slices_of(c));
  const int Q = (int)g.target.size();
  const size_t K = lsb::kSplitCands, K1 = g.pos.size();
  for (Rank& r : c->ranks) LSB_TRY(merge_ensure(c, r, g));
  // 1. splitter search: kSplitRounds rounds of candidate counts, all-gathered.
  if (Q > 0) {
    for (Rank& r : c->ranks) {
      HIP_TRY(hipSetDevice(r.dev));
      HIP_TRY(lsb::launch_split_init(r.split_state, Q, r.stream));
    }
    for (int round = 0; round < lsb::kSplitRounds; ++round) {
      for (Rank& r : c->ranks) {
        HIP_TRY(hipSetDevice(r.dev));
        Timer t(c, &r, LSB_K_EXCHANGE);
        HIP_TRY(lsb::launch_split_cands(r.A, r.here, r.split_state, Q, r.split_cnt, r.stream));
      }
      LSB_TRY(gather_ranks(c, (size_t)Q * K, [](Rank& r) { return r.split_cnt; },
                           [](Rank& r) { return r.split_gather; }));
      for (Rank& r : c->ranks) {
        HIP_TRY(hipSetDevice(r.dev));
        HIP_TRY(lsb::launch_split_update(r.split_gather, P, Q, r.split_targets, r.split_state,
                                         r.stream));
      }
    }
    for (Rank& r : c->ranks) {
      HIP_TRY(hipSetDevice(r.dev));
      HIP_TRY(lsb::launch_split_final(r.A, r.here, r.split_state, Q, r.split_fin, r.stream));
    }
    LSB_TRY(gather_ranks(c, 2 * (size_t)Q, [](Rank& r) { return r.split_fin; },
                         [](Rank& r) { return r.split_fin_gather; }));
    for (Rank& r : c->ranks) {
      HIP_TRY(hipSetDevice(r.dev));
      HIP_TRY(hipMemcpyAsync(r.split_h, r.split_fin_gather, sizeof(uint64_t) * P * 2 * Q,
                             hipMemcpyDeviceToHost, r.stream));
    }
  }
  // 2. the cuts, on the host (the all-to-all takes host counts)
  for (Rank& r : c->ranks) {
    HIP_TRY(hipSetDevice(r.dev));
    HIP_TRY(hipStreamSynchronize(r.stream));
    LSB_TRY(merge_cuts(c->n, P, g, r.split_h, r.mcut));
  }
  // 3. slice by slice: all-to-all-v of contiguous ranges (my own range stays
  //    in A), then the slice's merge on the placement stream.  The merged
  //    block lands in B or R, whichever the last level of a P-run tree writes.
  const bool final_b = (merge_levels((size_t)P) - 1) % 2 == 0;
  std::vector<SliceRun> sr;
  int64_t lo = 0, hi = 0;
  for (int j = 0; j < g.S; ++j) {
    if (c->mode == Mode::kLoopback) {
      for (Rank& q : c->ranks) {
        HIP_TRY(hipSetDevice(q.dev));
        Timer t(c, &q, LSB_K_EXCHANGE);
        slice_runs(c, q, g, j, sr, &lo, &hi);
        for (Rank& s : c->ranks) {
          if (s.rank == q.rank || sr[s.rank].len == 0) continue;
          HIP_TRY(hipMemcpyAsync(q.R + sr[s.rank].roff, s.A + q.mcut[s.rank * K1 + (size_t)q.rank * g.S + j],
                                 (size_t)sr[s.rank].len * sizeof(Elem), hipMemcpyDefault, q.stream));
        }
      }
      for (Rank& q : c->ranks) LSB_TRY(merge_slice_async(c, q, g, j, final_b ? q.B : q.R));
    } else {
      Rank& r = c->ranks[0];
      HIP_TRY(hipSetDevice(r.dev));
      slice_runs(c, r, g, j, sr, &lo, &hi);
      std::vector<size_t> sc(P), sd(P), rc(P), rdp(P);
      for (int q = 0; q < P; ++q) {
        const size_t kq = (size_t)q * g.S + j;
        const bool skip = q == r.rank && !c->self_coll;  // own range stays in A
        sc[q] = skip ? 0 : (size_t)(r.mcut[(size_t)r.rank * K1 + kq + 1] - r.mcut[(size_t)r.rank * K1 + kq]) * 2;
        sd[q] = (size_t)r.mcut[(size_t)r.rank * K1 + kq] * 2;
        rc[q] = skip ? 0 : (size_t)sr[q].len * 2;
        rdp[q] = (size_t)sr[q].roff * 2;
      }
      {
        Timer t(c, &r, LSB_K_EXCHANGE);
        LSB_TRY(coll_alltoallv_u64(c, r, reinterpret_cast<const uint64_t*>(r.A), sc.data(), sd.data(),
                                   reinterpret_cast<uint64_t*>(r.R), rc.data(), rdp.data()));
      }
      LSB_TRY(merge_slice_async(c, r, g, j, final_b ? r.B : r.R));
    }
  }
  // 4. the merged block (B or R) becomes A: every rank's sends out of A are done
  //    (loopback: all copies; RCCL / ops: my stream finished the collectives).
  if (c->mode == Mode::kLoopback)
    for (Rank& r : c->ranks) {
      HIP_TRY(hipSetDevice(r.dev));
      HIP_TRY(hipStreamSynchronize(r.stream));
    }
  for (Rank& r : c->ranks) {
    LSB_TRY(join_place(r));
    std::swap(r.A, final_b ? r.B : r.R);
  }
  return LSB_OK;
}

// lsb_sort / lsb_pass(0) with a 64-bit exchange digit on an exchanging context.
int merge_sort(lsb_ctx* c) {
  c->last_local_passes = 0;
  c->last_varying = 0;
  for (Rank& r : c->ranks) {
    int passes = 0;
    uint64_t varying = 0;
    LSB_TRY(sort_local_rank(c, r, &passes, &varying));
    c->last_local_passes = std::max(c->last_local_passes, passes);
    c->last_varying |= varying;
  }
  c->last_exchanges = 1;
  return exchange_merge(c);
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
  HIP_TRY(hipMemset(r.os_status, 0, (size_t)lsb::onesweep_tiles(r.here) * lsb::kBuckets * sizeof(uint32_t)));
  r.os_epoch = 0;
  return fail(LSB_ERR_HIP, "k_onesweep", "look-back timed out; output invalid");
}

int check_ctx(const lsb_ctx* c) {
  if (!c) return fail(LSB_ERR_INVALID, "lsb", "null context");
  return LSB_OK;
}

lsb_ctx* new_ctx(int64_t n_total, int num_ranks, int radix_bits) {
  lsb_ctx* c = new (std::nothrow) lsb_ctx();
  if (!c) return nullptr;
  c->n = n_total;
  c->P = num_ranks;
  c->per = div_ceil(n_total, num_ranks);
  c->bits = radix_bits;
  c->nb = radix_bits == 64 ? lsb::kBuckets : 1 << radix_bits;
  return c;
}

// Boundary records of every rank (first, last of its here-part), gathered on
// the host: [rank][0..3] = first.key, first.val, last.key, last.val.
int gather_boundaries(lsb_ctx* c, std::vector<uint64_t>& bnd) {
  const int P = c->P;
  bnd.assign((size_t)P * 4, 0);
  if (c->mode == Mode::kLoopback) {
    for (Rank& r : c->ranks) {
      if (r.here == 0) continue;
      HIP_TRY(hipSetDevice(r.dev));
      HIP_TRY(hipStreamSynchronize(r.stream));
      HIP_TRY(hipMemcpy(&bnd[(size_t)r.rank * 4], r.A, 16, hipMemcpyDeviceToHost));
      HIP_TRY(hipMemcpy(&bnd[(size_t)r.rank * 4 + 2], r.A + (r.here - 1), 16, hipMemcpyDeviceToHost));
    }
    return LSB_OK;
  }
  Rank& r = c->ranks[0];
  HIP_TRY(hipSetDevice(r.dev));
  uint64_t* d = r.gather;  // >= 4 * P entries
  HIP_TRY(hipMemsetAsync(d, 0, sizeof(uint64_t) * 4 * P, r.stream));
  if (r.here > 0) {
    HIP_TRY(hipMemcpyAsync(d + (size_t)r.rank * 4, r.A, 16, hipMemcpyDeviceToDevice, r.stream));
    HIP_TRY(hipMemcpyAsync(d + (size_t)r.rank * 4 + 2, r.A + (r.here - 1), 16,
                           hipMemcpyDeviceToDevice, r.stream));
  }
  // Each rank contributes its own 4 words (in-place all-gather).
  LSB_TRY(coll_allgather_u64(c, r, d + (size_t)r.rank * 4, d, 4));
  HIP_TRY(hipMemcpyAsync(bnd.data(), d, sizeof(uint64_t) * 4 * P, hipMemcpyDeviceToHost, r.stream));
  HIP_TRY(hipStreamSynchronize(r.stream));
  return LSB_OK;
}

int allreduce_min_i64(lsb_ctx* c, int64_t* v) {
  if (c->mode == Mode::kLoopback) return LSB_OK;
  if (c->mode == Mode::kOps)
    return c->ops.allreduce_min_i64(c->ops.user, v) == 0 ? LSB_OK : ops_fail("allreduce_min_i64");
  Rank& r = c->ranks[0];
  HIP_TRY(hipSetDevice(r.dev));
  int64_t* d = reinterpret_cast<int64_t*>(r.check);
  HIP_TRY(hipMemcpyAsync(d, v, sizeof(int64_t), hipMemcpyHostToDevice, r.stream));
  RCCL_TRY(ncclAllReduce(d, d, 1, ncclInt64, ncclMin, c->comm, r.stream));
  HIP_TRY(hipMemcpyAsync(v, d, sizeof(int64_t), hipMemcpyDeviceToHost, r.stream));
  HIP_TRY(hipStreamSynchronize(r.stream));
  return LSB_OK;
}

// Global key span after the first pass: OR of all keys and of their
// complements over every rank (RCCL: all-gather of the 2 words per rank).
int gather_span(lsb_ctx* c, uint64_t* kor, uint64_t* knor) {
  *kor = *knor = 0;
  if (c->mode != Mode::kLoopback) {
    Rank& r = c->ranks[0];
    HIP_TRY(hipSetDevice(r.dev));
    LSB_TRY(coll_allgather_u64(c, r, r.span, r.span_gather, 2));
    HIP_TRY(hipMemcpyAsync(r.span_h, r.span_gather, sizeof(uint64_t) * 2 * c->P,
                           hipMemcpyDeviceToHost, r.stream));
    HIP_TRY(hipStreamSynchronize(r.stream));
    for (int q = 0; q < c->P; ++q) {
      *kor |= r.span_h[2 * q];
      *knor |= r.span_h[2 * q + 1];
    }
    return LSB_OK;
  }
  for (Rank& r : c->ranks) {
    HIP_TRY(hipSetDevice(r.dev));
    HIP_TRY(hipMemcpyAsync(r.span_h, r.span, sizeof(uint64_t) * 2, hipMemcpyDeviceToHost, r.stream));
  }
  for (Rank& r : c->ranks) {
    HIP_TRY(hipSetDevice(r.dev));
    HIP_TRY(hipStreamSynchronize(r.stream));
    *kor |= r.span_h[0];
    *knor |= r.span_h[1];
  }
  return LSB_OK;
}

}  // namespace

// ======================================================================
extern "C" {

int64_t lsb_per_rank(int64_t n_total, int num_ranks) {
  return (num_ranks > 0 && n_total >= 0) ? div_ceil(n_total, num_ranks) : 0;
}

int64_t lsb_here(int64_t n_total, int num_ranks, int rank) {
  if (num_ranks <= 0 || n_total < 0 || rank < 0 || rank >= num_ranks) return 0;
  return here_of(n_total, num_ranks, rank);
}

const char* lsb_strerror(int code) {
  switch (code) {
    case LSB_OK: return "ok";
    case LSB_ERR_INVALID: return "invalid argument";
    case LSB_ERR_HIP: return g_last_error.empty() ? "HIP error" : g_last_error.c_str();
    case LSB_ERR_RCCL: return g_last_error.empty() ? "RCCL error" : g_last_error.c_str();
    case LSB_ERR_NOMEM: return "out of memory";
    case LSB_ERR_VERIFY: return "verification failed";
    case LSB_ERR_UNSUPPORTED: return "unsupported";
    case LSB_ERR_STATE: return g_last_error.empty() ? "invalid state" : g_last_error.c_str();
    default: return "unknown error";
  }
}

int lsb_create(lsb_ctx_t** out, int64_t n_total, int num_ranks, const int* dev_ids,
               int radix_bits) {
  if (!out) return fail(LSB_ERR_INVALID, "lsb_create", "null out");
  *out = nullptr;
  if (n_total < 0 || num_ranks < 1 || num_ranks > 64)
    return fail(LSB_ERR_INVALID, "lsb_create", "n or P");
  if (radix_bits != 8 && radix_bits != 16 && radix_bits != 64)
    return fail(LSB_ERR_UNSUPPORTED, "lsb_create", "radix_bits must be 8, 16 or 64");
  lsb_ctx* c = new_ctx(n_total, num_ranks, radix_bits);
  if (!c) return LSB_ERR_NOMEM;
  c->mode = Mode::kLoopback;
  c->first_rank = 0;
  c->ranks.resize(num_ranks);
  for (int r = 0; r < num_ranks; ++r) {
    int rc = init_rank(c, c->ranks[r], r, dev_ids ? dev_ids[r] : 0);
    if (rc != LSB_OK) {
      lsb_destroy(c);
      return rc;
    }
  }
  *out = c;
  return LSB_OK;
}

int lsb_get_unique_id(unsigned char id[LSB_UNIQUE_ID_BYTES]) {
  if (!id) return fail(LSB_ERR_INVALID, "lsb_get_unique_id", "null");
  ncclUniqueId uid;
  RCCL_TRY(ncclGetUniqueId(&uid));
  static_assert(sizeof(uid) == LSB_UNIQUE_ID_BYTES, "id size");
  memcpy(id, &uid, sizeof uid);
  return LSB_OK;
}

int lsb_create_rank(lsb_ctx_t** out, int64_t n_total, int num_ranks, int rank, int dev_id,
                    int radix_bits, const unsigned char id[LSB_UNIQUE_ID_BYTES]) {
  if (!out) return fail(LSB_ERR_INVALID, "lsb_create_rank", "null out");
  *out = nullptr;
  if (n_total < 0 || num_ranks < 1 || num_ranks > 64 || rank < 0 || rank >= num_ranks || !id)
    return fail(LSB_ERR_INVALID, "lsb_create_rank", "n, P, rank or id");
  if (radix_bits != 8 && radix_bits != 16 && radix_bits != 64)
    return fail(LSB_ERR_UNSUPPORTED, "lsb_create_rank", "radix_bits must be 8, 16 or 64");
  lsb_ctx* c = new_ctx(n_total, num_ranks, radix_bits);
  if (!c) return LSB_ERR_NOMEM;
  c->mode = Mode::kRccl;
  c->first_rank = rank;
  c->ranks.resize(1);
  int rc = init_rank(c, c->ranks[0], rank, dev_id);
  if (rc == LSB_OK) {
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof uid);
    if (hipSetDevice(dev_id) != hipSuccess) rc = fail(LSB_ERR_HIP, "hipSetDevice", "");
    else {
      ncclResult_t nr = ncclCommInitRank(&c->comm, num_ranks, uid, rank);
      if (nr != ncclSuccess) {
        c->comm = nullptr;
        rc = fail(LSB_ERR_RCCL, "ncclCommInitRank", ncclGetErrorString(nr));
      }
    }
  }
  if (rc != LSB_OK) {
    lsb_destroy(c);
    return rc;
  }
  *out = c;
  return LSB_OK;
}

int lsb_create_rank_ops(lsb_ctx_t** out, int64_t n_total, int num_ranks, int rank, int dev_id,
                        int radix_bits, const lsb_comm_ops_t* ops) {
  if (!out) return fail(LSB_ERR_INVALID, "lsb_create_rank_ops", "null out");
  *out = nullptr;
  if (n_total < 0 || num_ranks < 1 || num_ranks > 64 || rank < 0 || rank >= num_ranks || !ops ||
      !ops->allgather || !ops->alltoallv || !ops->allreduce_min_i64 || !ops->barrier)
    return fail(LSB_ERR_INVALID, "lsb_create_rank_ops", "n, P, rank or ops");
  if (radix_bits != 8 && radix_bits != 16 && radix_bits != 64)
    return fail(LSB_ERR_UNSUPPORTED, "lsb_create_rank_ops", "radix_bits must be 8, 16 or 64");
  lsb_ctx* c = new_ctx(n_total, num_ranks, radix_bits);
  if (!c) return LSB_ERR_NOMEM;
  c->mode = Mode::kOps;
  c->ops = *ops;
  c->first_rank = rank;
  c->ranks.resize(1);
  const int rc = init_rank(c, c->ranks[0], rank, dev_id);
  if (rc != LSB_OK) {
    lsb_destroy(c);
    return rc;
  }
  *out = c;
  return LSB_OK;
}

void lsb_destroy(lsb_ctx_t* c) {
  if (!c) return;
  (void)resolve_timing(c);
#ifdef LSB_OS_PROFILE
  (void)lsb_sync(c);
  os_profile_report();
#endif
  for (Rank& r : c->ranks) free_rank(r);
  for (hipEvent_t e : c->event_pool) (void)hipEventDestroy(e);
  if (c->comm) (void)ncclCommDestroy(c->comm);
  delete c;
}

int lsb_set_option(lsb_ctx_t* c, int option, int64_t value) {
  LSB_TRY(check_ctx(c));
  switch (option) {
    case LSB_OPT_TIMING:
      c->timing = value != 0;
      return LSB_OK;
    case LSB_OPT_FORCE_EXCHANGE:
      c->force_exchange = value != 0;
      return LSB_OK;
    case LSB_OPT_SKIP_CONSTANT_DIGITS:
      c->skip_constant = value != 0;
      return LSB_OK;
    case LSB_OPT_ONESWEEP:
      c->onesweep = value != 0;
      return LSB_OK;
    case LSB_OPT_EXCHANGE_PEER:
      c->peer = value != 0;
      return LSB_OK;
    case LSB_OPT_EXCHANGE_P2P:
      c->p2p = value != 0;
      return LSB_OK;
    case LSB_OPT_EXCHANGE_SELF:
      c->self_coll = value != 0;
      return LSB_OK;
    case LSB_OPT_EXCHANGE_GATHER:
      c->gather = value != 0;
      return LSB_OK;
    case LSB_OPT_HYBRID:
      if (value < 0 || value > 2) return fail(LSB_ERR_INVALID, "lsb_set_option", "hybrid must be 0, 1 or 2");
      c->hybrid = (int)value;
      return LSB_OK;
    case LSB_OPT_ONESWEEP_SPLIT:
      if (value < 0 || value > 2) return fail(LSB_ERR_INVALID, "lsb_set_option", "split must be 0..2");
      c->os_split = (int)value;
      return LSB_OK;
    case LSB_OPT_EXCHANGE_SLICES:
      if (value < 1 || value > 64)
        return fail(LSB_ERR_INVALID, "lsb_set_option", "exchange slices must be 1..64");
      c->slices = (int)value;
      return LSB_OK;
    default:
      return fail(LSB_ERR_INVALID, "lsb_set_option", "unknown option");
  }
}

int lsb_local_ranks(const lsb_ctx_t* c, int* first_rank, int* num_local) {
  LSB_TRY(check_ctx(c));
  if (first_rank) *first_rank = c->first_rank;
  if (num_local) *num_local = (int)c->ranks.size();
  return LSB_OK;
}

int lsb_generate_ex(lsb_ctx_t* c, int dist, double param) {
  LSB_TRY(check_ctx(c));
  lsb::KeyGen g;
  if (dist == LSB_DIST_UNIFORM) {
    g.dist = lsb::kDistUniform;
  } else if (dist == LSB_DIST_ZIPF) {
    if (!(param > 0.0) || param > 16.0) return fail(LSB_ERR_INVALID, "lsb_generate_ex", "zipf s");
    g.dist = lsb::kDistZipf;
    g.zipf_s = param;
    g.zipf_n = 1ull << 30;
  } else {
    return fail(LSB_ERR_INVALID, "lsb_generate_ex", "dist");
  }
  c->keygen = g;
  for (Rank& r : c->ranks) {
    HIP_TRY(hipSetDevice(r.dev));
    // Every one of the `per` slots, like mpi/mpi_lsbsort.cpp:650-656.
    HIP_TRY(lsb::launch_pcg_fill(r.A, c->per, (uint64_t)r.rank, (uint64_t)r.rank * c->per, g,
                                 r.stream));
  }
  return lsb_sync(c);
}

int lsb_generate(lsb_ctx_t* c) { return lsb_generate_ex(c, LSB_DIST_UNIFORM, 0.0); }

int lsb_copy_in(lsb_ctx_t* c, int rank, int64_t off, int64_t cnt, const lsb_elem_t* host) {
  LSB_TRY(check_ctx(c));
  Rank* r = local_rank(c, rank);
  if (!r || off < 0 || cnt < 0 || off + cnt > c->per || (cnt > 0 && !host))
    return fail(LSB_ERR_INVALID, "lsb_copy_in", "rank or range");
  if (cnt == 0) return LSB_OK;
  HIP_TRY(hipSetDevice(r->dev));
  HIP_TRY(hipStreamSynchronize(r->stream));
  HIP_TRY(hipMemcpy(r->A + off, host, (size_t)cnt * sizeof(Elem), hipMemcpyHostToDevice));
  return LSB_OK;
}

int lsb_copy_out(lsb_ctx_t* c, int rank, int64_t off, int64_t cnt, lsb_elem_t* host) {
  LSB_TRY(check_ctx(c));
  Rank* r = local_rank(c, rank);
  if (!r || off < 0 || cnt < 0 || off + cnt > c->per || (cnt > 0 && !host))
    return fail(LSB_ERR_INVALID, "lsb_copy_out", "rank or range");
  if (cnt == 0) return LSB_OK;
  HIP_TRY(hipSetDevice(r->dev));
  HIP_TRY(hipStreamSynchronize(r->stream));
  HIP_TRY(hipMemcpy(host, r->A + off, (size_t)cnt * sizeof(Elem), hipMemcpyDeviceToHost));
  return LSB_OK;
}

int lsb_pass(lsb_ctx_t* c, int digit) {
  LSB_TRY(check_ctx(c));
  if (digit < 0 || digit >= 64 / c->bits) return fail(LSB_ERR_INVALID, "lsb_pass", "digit");
  // Filed under the digit's own local passes (a 64-bit digit: the whole sort).
  c->pass_cursor = c->bits == 64 ? 0 : digit * (c->bits / lsb::kDigitBits);
  return do_pass(c, digit);
}

int lsb_sort(lsb_ctx_t* c) {
  LSB_TRY(check_ctx(c));
  std::vector<Timer> sort_timers;
  sort_timers.reserve(c->ranks.size());
  for (Rank& r : c->ranks) sort_timers.emplace_back(c, &r, LSB_K_SORT);
  const int passes = 64 / c->bits;
  c->last_local_passes = c->last_exchanges = 0;
  c->last_varying = ~0ull;
  c->pass_cursor = 0;
  c->cur_pass = 0;
  if (c->bits == 64 && exchanging(c)) {
    LSB_TRY(merge_sort(c));
  } else if (onesweep_applies(c)) {
    LSB_TRY(sort_onesweep(c));
  } else if (exchange_onesweep_applies(c)) {
    LSB_TRY(sort_exchange_onesweep(c));
  } else if (!c->skip_constant) {
    for (int d = 0; d < passes; ++d) LSB_TRY(do_pass(c, d));
  } else {
    for (Rank& r : c->ranks) {
      HIP_TRY(hipSetDevice(r.dev));
      HIP_TRY(hipMemsetAsync(r.span, 0, 2 * sizeof(uint64_t), r.stream));
    }
    LSB_TRY(do_pass(c, 0, ~0ull, true));
    uint64_t kor = 0, knor = 0;
    LSB_TRY(gather_span(c, &kor, &knor));
    c->last_varying = kor & knor;
    const uint64_t digit_mask = (1ull << c->bits) - 1;
    for (int d = 1; d < passes; ++d) {
      // A digit on which every key agrees: the stable pass and the exchange
      // (order (digit, rank) = rank order) are both the identity.
      if (((c->last_varying >> (d * c->bits)) & digit_mask) == 0) continue;
      LSB_TRY(do_pass(c, d, c->last_varying));
    }
  }
  for (Timer& t : sort_timers) t.stop();
  return LSB_OK;
}

int lsb_get_last_sort(lsb_ctx_t* c, int* local_passes, int* exchanges, uint64_t* varying_bits) {
  LSB_TRY(check_ctx(c));
  if (local_passes) *local_passes = c->last_local_passes;
  if (exchanges) *exchanges = c->last_exchanges;
  if (varying_bits) *varying_bits = c->last_varying;
  return LSB_OK;
}

int lsb_sync(lsb_ctx_t* c) {
  LSB_TRY(check_ctx(c));
  for (Rank& r : c->ranks) {
    HIP_TRY(hipSetDevice(r.dev));
    HIP_TRY(hipStreamSynchronize(r.stream));
    LSB_TRY(onesweep_check(r));
  }
  return LSB_OK;
}

int lsb_barrier(lsb_ctx_t* c) {
  LSB_TRY(lsb_sync(c));
  if (c->mode == Mode::kLoopback) return LSB_OK;
  if (c->mode == Mode::kOps)
    return c->ops.barrier(c->ops.user) == 0 ? LSB_OK : ops_fail("barrier");
  Rank& r = c->ranks[0];
  HIP_TRY(hipSetDevice(r.dev));
  RCCL_TRY(ncclAllReduce(r.check, r.check, 1, ncclUint64, ncclSum, c->comm, r.stream));
  HIP_TRY(hipStreamSynchronize(r.stream));
  return LSB_OK;
}

int lsb_verify(lsb_ctx_t* c, int64_t* first_bad) {
  LSB_TRY(check_ctx(c));
  int64_t bad = INT64_MAX;
  for (Rank& r : c->ranks) {
    HIP_TRY(hipSetDevice(r.dev));
    HIP_TRY(hipMemsetAsync(r.check, 0xff, sizeof(unsigned long long), r.stream));
    HIP_TRY(lsb::launch_verify(r.A, r.here, (int64_t)r.rank * c->per, c->n, c->per, c->keygen,
                               r.check, r.stream));
    unsigned long long h = ~0ull;
    HIP_TRY(hipMemcpyAsync(&h, r.check, sizeof h, hipMemcpyDeviceToHost, r.stream));
    HIP_TRY(hipStreamSynchronize(r.stream));
    if (h != ~0ull && (int64_t)h < bad) bad = (int64_t)h;
  }
  // Rank boundaries: last record of each non-empty rank < first of the next.
  std::vector<uint64_t> bnd;
  LSB_TRY(gather_boundaries(c, bnd));
  int prev = -1;
  for (int s = 0; s < c->P; ++s) {
    if (here_of(c->n, c->P, s) == 0) continue;
    if (prev >= 0) {
      const uint64_t lk = bnd[(size_t)prev * 4 + 2], lv = bnd[(size_t)prev * 4 + 3];
      const uint64_t fk = bnd[(size_t)s * 4 + 0], fv = bnd[(size_t)s * 4 + 1];
      if (!(lk < fk || (lk == fk && lv < fv))) {
        const int64_t idx = (int64_t)prev * c->per + here_of(c->n, c->P, prev) - 1;
        if (idx < bad) bad = idx;
      }
    }
    prev = s;
  }
  LSB_TRY(allreduce_min_i64(c, &bad));
  if (first_bad) *first_bad = bad == INT64_MAX ? -1 : bad;
  return bad == INT64_MAX ? LSB_OK : LSB_ERR_VERIFY;
}

int lsb_check_sorted(lsb_ctx_t* c, int* sorted) {
  LSB_TRY(check_ctx(c));
  int local_ok = 1;
  for (Rank& r : c->ranks) {
    HIP_TRY(hipSetDevice(r.dev));
    HIP_TRY(hipMemsetAsync(r.check, 0, sizeof(unsigned int), r.stream));
    HIP_TRY(lsb::launch_check_sorted(r.A, r.here, reinterpret_cast<unsigned int*>(r.check),
                                     r.stream));
    unsigned int h = 0;
    HIP_TRY(hipMemcpyAsync(&h, r.check, sizeof h, hipMemcpyDeviceToHost, r.stream));
    HIP_TRY(hipStreamSynchronize(r.stream));
    if (h) local_ok = 0;
  }
  std::vector<uint64_t> bnd;
  LSB_TRY(gather_boundaries(c, bnd));
  int prev = -1;
  int bounds_ok = 1;
  for (int s = 0; s < c->P; ++s) {
    if (here_of(c->n, c->P, s) == 0) continue;
    if (prev >= 0 && bnd[(size_t)s * 4 + 0] < bnd[(size_t)prev * 4 + 2]) bounds_ok = 0;
    prev = s;
  }
  int64_t ok = (local_ok && bounds_ok) ? 1 : 0;  // min-reduced over ranks
  LSB_TRY(allreduce_min_i64(c, &ok));
  if (sorted) *sorted = (int)ok;
  return LSB_OK;
}

int lsb_get_kernel_stats(lsb_ctx_t* c, int kid, int64_t* launches, double* total_ms) {
  LSB_TRY(check_ctx(c));
  if (kid < 0 || kid >= LSB_K_COUNT) return fail(LSB_ERR_INVALID, "lsb_get_kernel_stats", "id");
  LSB_TRY(resolve_timing(c));
  if (launches) *launches = c->launches[kid];
  if (total_ms) *total_ms = c->total_ms[kid];
  return LSB_OK;
}

int lsb_reset_kernel_stats(lsb_ctx_t* c) {
  LSB_TRY(check_ctx(c));
  LSB_TRY(resolve_timing(c));
  for (int k = 0; k < LSB_K_COUNT; ++k) {
    c->launches[k] = 0;
    c->total_ms[k] = 0.0;
  }
  c->scatter_elems = 0;
  for (int p = 0; p < LSB_MAX_PASSES; ++p) {
    for (int k = 0; k < LSB_K_COUNT; ++k) {
      c->pass_launches[p][k] = 0;
      c->pass_ms[p][k] = 0.0;
    }
    c->pass_elems[p] = 0;
  }
  return LSB_OK;
}

int lsb_get_pass_stats(lsb_ctx_t* c, int pass, int* shift, int64_t* launches, int64_t* elems,
                       double* ms_count, double* ms_scatter, double* ms_exchange, double* ms_place) {
  LSB_TRY(check_ctx(c));
  if (pass < 0 || pass >= LSB_MAX_PASSES) return fail(LSB_ERR_INVALID, "lsb_get_pass_stats", "pass");
  LSB_TRY(resolve_timing(c));
  // The pass's sorting kernel: k_onesweep / k_scatter, or k_segsort (shift 64).
  const int64_t sorts = c->pass_launches[pass][LSB_K_SCATTER] + c->pass_launches[pass][LSB_K_SEGSORT];
  if (shift) *shift = sorts > 0 ? c->pass_shift[pass] : -1;
  if (launches) *launches = sorts;
  if (elems) *elems = c->pass_elems[pass];
  // The count kernels: k_subhist / k_upsweep (read) and k_scan.
  if (ms_count) *ms_count = c->pass_ms[pass][LSB_K_UPSWEEP] + c->pass_ms[pass][LSB_K_SCAN];
  if (ms_scatter) *ms_scatter = c->pass_ms[pass][LSB_K_SCATTER] + c->pass_ms[pass][LSB_K_SEGSORT];
  if (ms_exchange) *ms_exchange = c->pass_ms[pass][LSB_K_EXCHANGE];
  if (ms_place) *ms_place = c->pass_ms[pass][LSB_K_PLACE];
  return LSB_OK;
}

int lsb_get_scatter_elems(lsb_ctx_t* c, int64_t* elems) {
  LSB_TRY(check_ctx(c));
  if (elems) *elems = c->scatter_elems;
  return LSB_OK;
}

int lsb_get_exchange_bytes(lsb_ctx_t* c, int64_t* calls, int64_t* bytes, int64_t* max_call_bytes) {
  LSB_TRY(check_ctx(c));
  if (calls) *calls = c->coll_calls;
  if (bytes) *bytes = c->coll_bytes;
  if (max_call_bytes) *max_call_bytes = c->coll_max;
  return LSB_OK;
}

#ifndef LSB_SOURCE_DIGEST
#define LSB_SOURCE_DIGEST "unknown"
#endif
#ifndef LSB_BUILD_HOST
#define LSB_BUILD_HOST "unknown"
#endif
const char* lsb_build_info(void) { return "sha256=" LSB_SOURCE_DIGEST " host=" LSB_BUILD_HOST; }

// Host planner: see include/lsb.h.  For rank `me`, the global destination of
// its j-th bucket-b record is gstart[b][me] + j with
//   gstart[b][s] = sum_{b'<b} total[b'] + sum_{s'<s} hist[s'][b]
// (GlobalCounts[digit*P + rank] scanned, mpi/mpi_lsbsort.cpp:350,378,401-412),
// and owner(g) = g / per (globalIdxToLocalIdx, mpi/mpi_lsbsort.cpp:113-120).
int lsb_plan_exchange_device(int dev, int64_t n_total, int P, int me, int nb, const int64_t* hist,
                             int64_t* send_counts, int64_t* send_displs, int64_t* recv_counts,
                             int64_t* recv_displs, int64_t* place_off) {
  if (P < 1 || P > 64 || me < 0 || me >= P || nb < 1 || n_total < 0 || !hist || !send_counts ||
      !send_displs || !recv_counts || !recv_displs || !place_off)
    return fail(LSB_ERR_INVALID, "lsb_plan_exchange_device", "arguments");
  const size_t PN = (size_t)P * nb;
  for (size_t i = 0; i < PN; ++i)
    if (hist[i] < 0) return fail(LSB_ERR_INVALID, "lsb_plan_exchange_device", "negative count");
  HIP_TRY(hipSetDevice(dev));
  uint64_t* d_hist = nullptr;
  int64_t *d_work = nullptr, *d_total = nullptr, *d_place = nullptr, *d_counts = nullptr;
  int rc = LSB_OK;
  if ((rc = dev_alloc(&d_hist, PN)) == LSB_OK && (rc = dev_alloc(&d_work, PN)) == LSB_OK &&
      (rc = dev_alloc(&d_total, (size_t)nb)) == LSB_OK && (rc = dev_alloc(&d_place, PN + P)) == LSB_OK &&
      (rc = dev_alloc(&d_counts, 2 * (size_t)P)) == LSB_OK) {
    std::vector<int64_t> counts(2 * (size_t)P);
    hipError_t e = hipMemcpy(d_hist, hist, sizeof(int64_t) * PN, hipMemcpyHostToDevice);
    if (e == hipSuccess)
      e = lsb::launch_plan(d_hist, P, nb, me, n_total, d_work, d_total, d_place, d_counts, nullptr);
    if (e == hipSuccess) e = hipMemcpy(place_off, d_place, sizeof(int64_t) * PN, hipMemcpyDeviceToHost);
    if (e == hipSuccess)
      e = hipMemcpy(counts.data(), d_counts, sizeof(int64_t) * 2 * P, hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
      rc = fail(LSB_ERR_HIP, "lsb_plan_exchange_device", hipGetErrorString(e));
    } else {
      int64_t sd = 0, rd = 0;
      for (int q = 0; q < P; ++q) {
        send_counts[q] = counts[q];
        recv_counts[q] = counts[P + q];
        send_displs[q] = sd;
        recv_displs[q] = rd;
        sd += counts[q];
        rd += counts[P + q];
      }
    }
  }
  (void)hipFree(d_hist);
  (void)hipFree(d_work);
  (void)hipFree(d_total);
  (void)hipFree(d_place);
  (void)hipFree(d_counts);
  return rc;
}

int lsb_plan_merge(int64_t n_total, int P, int me, const int64_t* below, const int64_t* upto,
                   int64_t* send_counts, int64_t* send_displs, int64_t* recv_counts,
                   int64_t* recv_displs) {
  if (P < 1 || P > 64 || me < 0 || me >= P || n_total < 0 || (P > 1 && (!below || !upto)) ||
      !send_counts || !send_displs || !recv_counts || !recv_displs)
    return fail(LSB_ERR_INVALID, "lsb_plan_merge", "arguments");
  const MergeGeom g = merge_geometry(n_total, P, 1);  // targets q * per, q = 1 .. P-1 below n
  const int Q = (int)g.target.size();
  std::vector<uint64_t> fin((size_t)P * 2 * Q);
  for (int s = 0; s < P; ++s)
    for (int t = 0; t < Q; ++t) {
      const int q = g.target[t];  // cut index == owner (S = 1)
      const int64_t b = below[(size_t)s * (P - 1) + q - 1], u = upto[(size_t)s * (P - 1) + q - 1];
      if (b < 0 || u < 0) return fail(LSB_ERR_INVALID, "lsb_plan_merge", "negative count");
      fin[((size_t)s * Q + t) * 2] = (uint64_t)b;
      fin[((size_t)s * Q + t) * 2 + 1] = (uint64_t)u;
    }
  std::vector<int64_t> cut;
  LSB_TRY(merge_cuts(n_total, P, g, fin.data(), cut));
  return merge_owner_counts(n_total, P, me, g, cut, send_counts, send_displs, recv_counts, recv_displs);
}

int lsb_plan_exchange(int64_t n_total, int P, int me, int nb, const int64_t* hist,
                      int64_t* send_counts, int64_t* send_displs, int64_t* recv_counts,
                      int64_t* recv_displs, int64_t* place_off) {
  if (P < 1 || me < 0 || me >= P || nb < 1 || n_total < 0 || !hist || !send_counts ||
      !send_displs || !recv_counts || !recv_displs || !place_off)
    return fail(LSB_ERR_INVALID, "lsb_plan_exchange", "arguments");
  const int64_t per = div_ceil(n_total, P);
  for (int q = 0; q < P; ++q) send_counts[q] = recv_counts[q] = 0;
  const int64_t lo_me = (int64_t)me * per;
  const int64_t hi_me = lo_me + here_of(n_total, P, me);
  // The stream from source s is ordered by bucket: collect each (s, b)
  // piece that lands in my range first, then lay the pieces out.
  std::vector<int64_t> piece_lo((size_t)P * nb, 0), piece_len((size_t)P * nb, 0);
  int64_t base = 0;  // global start of bucket b
  for (int b = 0; b < nb; ++b) {
    int64_t acc = base;
    for (int s = 0; s < P; ++s) {
      const int64_t h = hist[(size_t)s * nb + b];
      if (h < 0) return fail(LSB_ERR_INVALID, "lsb_plan_exchange", "negative count");
      const int64_t g0 = acc, g1 = acc + h;
      if (g1 > n_total) return fail(LSB_ERR_INVALID, "lsb_plan_exchange", "counts exceed n");
      if (s == me && h > 0) {
        // split my run [g0, g1) over the owners
        int64_t g = g0;
        while (g < g1) {
          const int64_t q = g / per;
          const int64_t qend = std::min(g1, (q + 1) * per);
          send_counts[q] += qend - g;
          g = qend;
        }
      }
      // part of source s's run that lands in my range
      const int64_t lo = std::max(g0, lo_me), hi = std::min(g1, hi_me);
      if (hi > lo) {
        piece_lo[(size_t)s * nb + b] = lo;
        piece_len[(size_t)s * nb + b] = hi - lo;
        recv_counts[s] += hi - lo;
      }
      acc = g1;
    }
    base = acc;
  }
  int64_t acc = 0;
  for (int q = 0; q < P; ++q) {
    send_displs[q] = acc;
    acc += send_counts[q];
  }
  acc = 0;
  for (int s = 0; s < P; ++s) {
    recv_displs[s] = acc;
    int64_t k = acc;  // recv index where source s's next piece starts
    for (int b = 0; b < nb; ++b) {
      const size_t i = (size_t)s * nb + b;
      place_off[i] = (piece_lo[i] - lo_me) - k;
      k += piece_len[i];
    }
    acc += recv_counts[s];
  }
  return LSB_OK;
}

}  // extern "C"
