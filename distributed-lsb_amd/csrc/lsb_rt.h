// Internal header of the runtime behind include/lsb.h: the context and rank
// state, error and timing helpers, and every function the runtime's
// translation units share.  Not part of the C ABI.
//
//   lsb_alloc.cpp     record buffers (VMM pieces) and the optional placement probe
//   lsb_context.cpp   context / rank buffers, timing, host collectives
//   lsb_passes.cpp    the local pass driver: reduce-then-scan passes,
//                     single-read passes (k_subhist + k_onesweep), the hybrid
//   lsb_exchange.cpp  the per-digit exchange (plan, all-to-all, placement,
//                     gathered passes; loopback, RCCL / host ops, peer stores)
//   lsb_wholekey.cpp  the whole-key exchange (splitter search, one all-to-all,
//                     merge of the P runs)
//   lsb_abi.cpp       the extern "C" entry points and the host planners
#pragma once
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

namespace lsb_rt {

using lsb::Elem;

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
  // A and B were chosen among placement_k candidate buffers (alloc_records;
  // 0: allocated as they came): ms of the probe copy, mean of both
  // directions, of the chosen pair, of the first two allocated, of the worst.
  int placement_k = 0;
  double placement_ms[3] = {0.0, 0.0, 0.0};
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
  // The regional first pass (LSB_OPT_REGION_FIRST), allocated on first use:
  // the look-back rows of the pass that reads the regional layout (a track
  // of their own: that pass has more tiles than the others, and a status
  // buffer must only ever see one tile count), its epoch,
  // and rg_buf: region counts, the sample's histogram and span, the overflow
  // word (kRg* offsets, lsb_passes.cpp), rg_h its pinned mirror.
  int64_t cap = 0;                      // records A and B hold (>= here)
  int64_t rg_cap = 0;                   // slots per region (0: no regional first pass)
  uint32_t* os_status2 = nullptr;
  uint32_t os_epoch2 = 0;
  uint32_t* rg_buf = nullptr;
  uint32_t* rg_h = nullptr;
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
  // The per-digit exchange in chunks (LSB_OPT_EXCHANGE_CHUNKS, lsb_exchange.cpp
  // exchange_chunked), allocated on first use: the wire stream, chunk k's
  // events (its high-byte pass done on `stream`, its records received on
  // xstream), the count kernel's per-chunk histograms and the plan's
  // per-chunk counts (device, pinned mirror), the low byte's histogram mirror.
  hipStream_t xstream = nullptr;
  hipEvent_t ck_hi[lsb::kMaxExchangeChunks] = {};
  hipEvent_t ck_wire[lsb::kMaxExchangeChunks] = {};
  hipEvent_t xdone = nullptr;
  uint32_t* ck_hist = nullptr;          // [C][8][256]
  int64_t* ck_counts = nullptr;         // [2][P][C]: send per (owner, chunk), recv per (source, chunk)
  int64_t* ck_counts_h = nullptr;
  uint32_t* lo_hist_h = nullptr;        // [8][256]
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

}  // namespace lsb_rt

struct lsb_ctx {
  lsb_rt::Mode mode = lsb_rt::Mode::kLoopback;
  int64_t n = 0;
  int64_t per = 0;
  int P = 1;
  int bits = 8;      // exchange digit width: 8, 16, or 64 (the whole key: one exchange)
  int nb = 256;      // 1 << bits (256 for bits = 64: the buckets of the local passes)
  int first_rank = 0;
  std::vector<lsb_rt::Rank> ranks;  // local ranks
  ncclComm_t comm = nullptr;
  lsb_comm_ops_t ops = {};  // Mode::kOps
  bool timing = false;
  bool shared_device = false;  // two local ranks on one device (no placement probe)
  std::vector<int> access_devs;  // loopback: every device of the ranks (VMM record buffers map on all)
  bool force_exchange = false;
  bool skip_constant = true;  // lsb_sort skips digits on which all keys agree
  int slices = 0;             // exchange slices (placement overlaps the next slice); 0 = default
  int xchunks = 0;            // LSB_OPT_EXCHANGE_CHUNKS: 16-bit exchange digits in C chunks (0: off)
  int xchunk_reserve = 0;     // LSB_XCHUNK_RESERVE: workgroups the chunk passes leave to the wire
  bool p2p = false;           // RCCL exchange as grouped ncclSend/ncclRecv, not ncclAllToAllv
  bool peer = false;          // exchange by direct stores into the owners' buffers
  bool peer_ready = false;    // peer tables set up
  bool onesweep = true;       // P == 1: single-read passes (k_subhist + k_onesweep)
  bool region = true;         // LSB_OPT_REGION_FIRST: P == 1 LSD sorts start with the regional pass
  bool self_coll = false;     // the self segment also goes through the collective
  bool gather = true;         // LSB_OPT_EXCHANGE_GATHER: count-only placement + gathered pass
  int os_split = 0;           // LSB_OPT_ONESWEEP_SPLIT: 0 auto, 1 never, 2 always
  int fail_onesweep = 0;      // LSB_OPT_FAIL_ONESWEEP: the n-th k_onesweep launch fails (tests)
  int hybrid = 0;             // LSB_OPT_HYBRID: 0 off, 1 k byte passes (the last one
                              // ordering segments, + k_segfix), 2 the same + a k_segsort pass
  int64_t coll_calls = 0, coll_bytes = 0, coll_max = 0;  // element payload handed to the collective
  // What the last lsb_sort ran (lsb_get_last_sort).
  int last_local_passes = 0;
  int last_exchanges = 0;
  uint64_t last_varying = 0;
  int last_first = 0;  // the first pass's form (lsb_get_first_pass)
  lsb::KeyGen keygen;
  std::vector<lsb_rt::PendingEvent> pending;
  std::vector<std::pair<int, hipEvent_t>> event_pool;  // (device, event) of finished timings
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
  // Exchange steps since the last reset (lsb_get_exchange_stats).
  int64_t xs_exchanges = 0, xs_calls = 0;
  int64_t xs_sent[LSB_MAX_RANKS] = {}, xs_recv[LSB_MAX_RANKS] = {};
  int64_t xs_place_bytes = 0, xs_placed = 0, xs_counted = 0;
  int64_t pass_xbytes[LSB_MAX_PASSES] = {};
};

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

namespace lsb_rt {

// ---- errors (lsb_context.cpp) ------------------------------------------------
// Records `what: detail` for lsb_strerror and returns `code`.
int fail(int code, const char* what, const char* detail);
const std::string& last_error();

inline int64_t div_ceil(int64_t x, int64_t y) { return (x + y - 1) / y; }

inline int64_t here_of(int64_t n, int P, int r) {
  const int64_t per = P > 0 ? div_ceil(n, P) : 0;
  int64_t h = per;
  if (per * r + h > n) h = n - per * r;
  return h < 0 ? 0 : h;
}

inline bool exchanging(const lsb_ctx* c) { return c->P > 1 || c->force_exchange; }

// ---- timing (lsb_context.cpp) ----------------------------------------------
hipEvent_t take_event(lsb_ctx* c);

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

void begin_pass(lsb_ctx* c, int shift);
void count_pass_elems(lsb_ctx* c, int64_t m, bool scatter = true);
int resolve_timing(lsb_ctx* c);

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

// ---- record buffers (lsb_alloc.cpp) and rank buffers (lsb_context.cpp) ---------
// Record buffers (A, B, R, candidates): VMM-backed in 1 GiB pieces when at
// least one piece long, else hipMalloc; rec_free frees either kind.
int rec_alloc(const lsb_ctx* c, Elem** p, size_t count);
int rec_alloc_group(const lsb_ctx* c, Elem** const* outs, int k, size_t count);
size_t rec_bytes(size_t count);  // device bytes rec_alloc takes for count records
void rec_free(void* p);
bool rec_is_vmm(const void* p);
// A VMM record buffer that RCCL has seen is being released (an RCCL
// context's A, B or R): later RCCL contexts of this process take hipMalloc'd
// record buffers (lsb_alloc.cpp, "RCCL and VMM address reuse").
void mark_rccl_vmm_released();
int max_chunks_for_device(int dev);
// Records A and B are allocated for: the block, or the regional first
// pass's slots when a P == 1 context's sorts may start with it (blocks of at
// least region_min() records: lsb::kRegionMin, or LSB_REGION_MIN >= 2^16).
int64_t region_min();
int64_t region_cap_for(int64_t per, int P);
int64_t record_capacity(int64_t per, int P);
// The placement probe's request for record buffers of `bytes`, before the
// free-memory cap: candidates K (<= 2: no probe) and the share of the free
// memory the K buffers may take.  LSB_PLACEMENT_CANDIDATES = K sets it (at
// most 8, 90 %); unset, buffers of at least kProbeMinBytes get
// kDefaultCandidates within half the free memory.
constexpr int kDefaultCandidates = 4;
constexpr double kProbeMinBytes = double(int64_t(4) << 30);
int placement_request(double bytes, double* free_share);
int alloc_records(lsb_ctx* c, Rank& r);  // A and B (placement-calibrated)
int alloc_third(lsb_ctx* c, Rank& r);    // R, placed against A and B
int init_rank(lsb_ctx* c, Rank& r, int rank, int dev);
// Frees r's buffers once r's streams are idle.  c (LSB_DEBUG builds): check
// first that every rank's streams of c are idle (teardown_check).
void free_rank(Rank& r, const lsb_ctx* c = nullptr);
// Debug builds: every rank's stream and placement stream must be idle before
// any record buffer of the context is unmapped (VMM unmapping does not wait
// for the device).  Reports each busy stream on stderr; returns how many.
int teardown_check(const lsb_ctx* c, const Rank& freeing);
Rank* local_rank(lsb_ctx* c, int rank);
int check_ctx(const lsb_ctx* c);
lsb_ctx* new_ctx(int64_t n_total, int num_ranks, int radix_bits);

// ---- collectives (lsb_context.cpp) ------------------------------------------
int ops_fail(const char* what);
int coll_allgather_u64(lsb_ctx* c, Rank& r, const uint64_t* send, uint64_t* recv, size_t count);
// RCCL calls carry at most this many u64 (1 GiB) per peer (coll_alltoallv_u64).
constexpr size_t kMaxCallU64 = (size_t)1 << 27;
// The bound in force: kMaxCallU64, or LSB_RCCL_CALL_U64 (tests: a small bound
// makes small multi-rank sorts take the cut path, advisor r05).
size_t max_call_u64();
int coll_alltoallv_u64(lsb_ctx* c, Rank& r, const uint64_t* send, const size_t* sc,
                       const size_t* sd, uint64_t* recv, const size_t* rc, const size_t* rd,
                       size_t bound, hipStream_t stream = nullptr);
int gather_boundaries(lsb_ctx* c, std::vector<uint64_t>& bnd);
int allreduce_min_i64(lsb_ctx* c, int64_t* v);
int gather_span(lsb_ctx* c, uint64_t* kor, uint64_t* knor);

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

// ---- local passes (lsb_passes.cpp) ------------------------------------------
int local_pass(lsb_ctx* c, Rank& r, int shift, bool want_span = false, bool starts16 = false);
int do_pass(lsb_ctx* c, int digit, uint64_t varying = ~0ull, bool want_span = false);
bool onesweep_applies(const lsb_ctx* c);
int onesweep_ensure(Rank& r);
int onesweep_launch(lsb_ctx* c, Rank& r, int shift, int next, const uint32_t* hist,
                    uint32_t* next_hist, lsb::OnesweepExtra x);
int queue_halves(lsb_ctx* c, Rank& r, const uint32_t* hist);
int choose_halves(lsb_ctx* c, Rank& r, bool synced);
int sort_onesweep(lsb_ctx* c);
int sort_local_rank(lsb_ctx* c, Rank& r, int* passes, uint64_t* varying);
int sort_local_ranks(lsb_ctx* c);  // every rank, step by step across ranks
int onesweep_check(Rank& r);
#ifdef LSB_OS_PROFILE
void os_profile_report();
#endif

// ---- per-digit exchange (lsb_exchange.cpp) ------------------------------------

// ---- placement, overlapped with the exchange ------------------------------
// Part j of n records cut into `slices` equal parts: [part(n, j), part(n, j + 1))
// (the whole-key exchange's owner slices).
inline int64_t part(int64_t n, int j, int slices) { return n * j / slices; }

// Part j of a per-digit exchange segment of n records cut into `slices`
// halving parts: n/2, n/4, ..., and the last two n / 2^(slices-1) each.  A
// slice is placed (or counted) while the next one is on the wire, so what
// runs after the wire goes quiet is the last slice's placement: 1/16 of the
// records at 5 slices where equal slices leave 1/4 at 4.
// Sender and receiver cut a segment alike (send_counts[q] at s equals
// recv_counts[s] at q).
inline int64_t slice_part(int64_t n, int j, int slices) {
  if (j >= slices) return n;
  return j >= 63 ? n : n - (n >> j);
}

// Slices of an exchange: the option, else 5 halving slices per exchange digit,
// or 8 equal slices for the whole-key exchange, whose one all-to-all carries
// every record: its last slice's merge (ceil(log2 P) levels) is the tail
// after the wire goes quiet.
inline int slices_of(const lsb_ctx* c) { return c->slices > 0 ? c->slices : (c->bits == 64 ? 8 : 5); }

// Records of slice j of any peer segment of a rank block of `per` records, at
// most: a slice of a segment of n records holds ceil(floor(n / 2^j) / 2) (the
// last: floor(n / 2^(S-1))), non-decreasing in n, and n <= per.
inline int64_t slice_bound(int64_t per, int j, int slices) {
  return slice_part(per, j + 1, slices) - slice_part(per, j, slices);
}
int ensure_recv(lsb_ctx* c, Rank& r);
int join_place(Rank& r);
int join_place_timed(lsb_ctx* c, Rank& r);
int exchange_digit(lsb_ctx* c, int digit);
// A loopback exchange's device copy of cnt records src (a record buffer of
// src_rank) -> dst (one of dst_rank's), checked against the buffers first.
bool in_buffers(const Rank& q, const Elem* p, int64_t cnt);
int copy_range(const lsb_ctx* c, Rank& dst_rank, Elem* dst, const Rank& src_rank, const Elem* src, int64_t cnt,
               hipStream_t s);
// The per-digit exchange in chunks: digit `digit` (16 bits) whose low-byte
// pass has run (A sorted by the low byte; lo_hist its input's sub-array
// histogram on each rank), high-byte passes chunk by chunk, each chunk's
// records on the wire while the next chunk's pass runs.
bool chunked_applies(const lsb_ctx* c, uint64_t varying, int digit);
int exchange_chunked(lsb_ctx* c, int digit, const std::vector<const uint32_t*>& lo_hist);
bool exchange_onesweep_applies(const lsb_ctx* c);
int sort_exchange_onesweep(lsb_ctx* c);

// ---- whole-key exchange (lsb_wholekey.cpp) ------------------------------------

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
MergeGeom merge_geometry(int64_t n, int P, int slices);
int merge_cuts(int64_t n, int P, const MergeGeom& g, const uint64_t* fin, std::vector<int64_t>& cut);
int merge_owner_counts(int64_t n, int P, int me, const MergeGeom& g, const std::vector<int64_t>& cut,
                       int64_t* sc, int64_t* sd, int64_t* rc, int64_t* rd);
int merge_sort(lsb_ctx* c);

}  // namespace lsb_rt
