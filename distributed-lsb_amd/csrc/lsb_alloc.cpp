// Record buffers of the runtime (A, B, R: DistributedArray::create's
// localPart_, mpi/mpi_lsbsort.cpp:137-161): built from 1 GiB physical pieces
// (HIP virtual memory management), freed by rec_free whichever way they were
// made, and the optional placement probe that chooses A, B and R among timed
// candidate buffers (LSB_PLACEMENT_CANDIDATES).  DESIGN.md §4.
#include "lsb_rt.h"

#include <atomic>
#include <mutex>

namespace lsb_rt {

// ---- record buffers: physical memory in 1 GiB pieces ---------------------------
// A record buffer of at least one piece (LSB_VMM_CHUNK_MIB, default 1024) is
// not a hipMalloc: its address range is reserved once and backed by
// separately created 1 GiB physical allocations (hipMemCreate + hipMemMap,
// HIP's virtual memory management).  The same LSD write pattern between two
// hipMalloc'd 16 GiB buffers runs at 6.85 ms for most pairs and 7.2 ms for
// some (the driver's choice of physical pages), while between buffers built
// from 1 GiB pieces it runs at 5.7-6.8 ms (tools/kbench/vmmbw.hip,
// profiles/r05/vmm_*; DESIGN.md §4 "Spread").  LSB_RECORD_ALLOC=malloc keeps
// hipMalloc.  Pieces are readable and writable by the owner and by the other
// devices of a loopback context's ranks (hipMemSetAccess), as hipMalloc
// memory is once peer access is enabled; IPC handles cannot name them, so the
// peer-store exchange between processes moves the records into hipMalloc
// buffers at its setup (peer_setup).
namespace {

struct VmmBuffer {
  void* base = nullptr;
  size_t bytes = 0;
  size_t piece = 0;
  std::vector<hipMemGenericAllocationHandle_t> pieces;
};
std::mutex g_vmm_mu;
std::vector<VmmBuffer> g_vmm;  // live VMM record buffers of this process

size_t vmm_piece_bytes() {
  const char* mode = getenv("LSB_RECORD_ALLOC");
  if (mode && strcmp(mode, "malloc") == 0) return 0;
  size_t mib = 1024;
  if (const char* e = getenv("LSB_VMM_CHUNK_MIB")) mib = (size_t)std::max(0ll, atoll(e));
  return mib << 20;
}

// Unmaps and releases the first pieces.size() pieces of `piece` bytes (mapped
// in order from the base) and frees the address range.
void vmm_release(VmmBuffer& b, size_t piece) {
  for (size_t k = 0; k < b.pieces.size(); ++k) (void)hipMemUnmap(static_cast<char*>(b.base) + k * piece, piece);
  for (auto h : b.pieces) (void)hipMemRelease(h);
  if (b.base) (void)hipMemAddressFree(b.base, b.bytes);
  (void)hipGetLastError();
  b = VmmBuffer();
}

// RCCL and VMM address reuse.  RCCL contexts (RCCL 2.27.7) over VMM record
// buffers mapped at addresses that an earlier RCCL context's (released) VMM
// buffers had used delivered garbage: a world-of-one context sorting 2^28 records with 8-bit
// digits through ncclAllToAllv failed lsb_verify from its process's third
// such context on (zeros at the head, records lost; 3 of 5 and 3 of 6 sorts),
// never with hipMalloc'd buffers (5 of 5), nor while released address ranges
// stayed reserved (6 of 6, but then their memory is not given back: 288 ->
// 147 GiB free after 4 contexts); the reservation's address hint is not
// honoured, so the runtime hands the same ranges out again.  It needs records
// through RCCL (loopback contexts with the same buffers, and RCCL contexts
// sending no record through RCCL, stay right), is no stream race (it stays
// with the device drained around every call, LSB_RCCL_SYNC=1) and no
// leftover-data artefact (other input per context: same picture).  It is
// reproduced without liblsb and without RCCL (tools/rccl_vmm_reuse.cpp
// late ... kernel): ranges written by the GPU, released, and a range then
// mapped onto their addresses read back wrong through a plain copy kernel
// (never-written ranges and hipMalloc stay right), so the fault is in
// HIP/ROCm's VMM, and the rule below is a workaround for where we met it.
// profiles/r06/large_call/, tests/test_gpu_sort.py
// test_world_of_one_large_calls.  So once a VMM buffer of an
// RCCL context has been released in this process, later RCCL contexts take
// hipMalloc'd record buffers.  A process's first RCCL context keeps VMM
// pieces: every address RCCL sees there is mapped once (the placement
// probe's candidates are released before any collective touches them), so
// the bench's ranks (one context per process) are unchanged.
// LSB_RCCL_VMM=1 keeps VMM pieces regardless (reproduction).
std::atomic<bool> g_rccl_vmm_released{false};

bool malloc_for(const lsb_ctx* c) {
  if (!c || c->mode != Mode::kRccl || !g_rccl_vmm_released.load()) return false;
  const char* e = getenv("LSB_RCCL_VMM");
  return !(e && atoi(e));
}

}  // namespace

void mark_rccl_vmm_released() { g_rccl_vmm_released.store(true); }


size_t rec_bytes(size_t count) {
  const size_t piece = vmm_piece_bytes();
  const size_t want = std::max<size_t>(count, 1) * sizeof(Elem);
  return piece == 0 || want < piece ? want : (want + piece - 1) / piece * piece;
}

bool rec_is_vmm(const void* p) {
  std::lock_guard<std::mutex> lock(g_vmm_mu);
  for (const VmmBuffer& b : g_vmm)
    if (b.base == p) return true;
  return false;
}

// k record buffers of `count` records each.  VMM pieces are created in the
// order LSB_VMM_ORDER names: buffer by buffer (default), or "interleave"
// (piece j of every buffer before piece j + 1 of any).
int rec_alloc_group(const lsb_ctx* c, Elem** const* outs, int k, size_t count) {
  for (int i = 0; i < k; ++i) *outs[i] = nullptr;
  const size_t piece = malloc_for(c) ? 0 : vmm_piece_bytes();
  const size_t want = std::max<size_t>(count, 1) * sizeof(Elem);
  if (piece == 0 || want < piece) {
    for (int i = 0; i < k; ++i) {
      const int rc = dev_alloc(outs[i], count);
      if (rc != LSB_OK) {
        for (int q = 0; q < i; ++q) (void)hipFree(*outs[q]);
        return rc;
      }
    }
    return LSB_OK;
  }
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = dev;
  size_t gran = 0;
  HIP_TRY(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum));
  if (gran == 0 || piece % gran) return fail(LSB_ERR_INVALID, "rec_alloc", "LSB_VMM_CHUNK_MIB is not a multiple of the granularity");
  const char* order = getenv("LSB_VMM_ORDER");
  const bool interleave = order && strcmp(order, "interleave") == 0;
  std::vector<VmmBuffer> b((size_t)k);
  const size_t bytes = (want + piece - 1) / piece * piece, np = bytes / piece;
  hipError_t e = hipSuccess;
  for (int i = 0; i < k && e == hipSuccess; ++i) {
    b[i].bytes = bytes;
    b[i].piece = piece;
    e = hipMemAddressReserve(&b[i].base, bytes, piece, nullptr, 0);
    if (e != hipSuccess) b[i].base = nullptr;
  }
  // piece j of buffer i, in creation order (pieces of a buffer map in order)
  for (size_t t = 0; t < np * (size_t)k && e == hipSuccess; ++t) {
    const int i = interleave ? (int)(t % (size_t)k) : (int)(t / np);
    const size_t j = b[i].pieces.size();
    hipMemGenericAllocationHandle_t h;
    e = hipMemCreate(&h, piece, &prop, 0);
    if (e != hipSuccess) break;
    e = hipMemMap(static_cast<char*>(b[i].base) + j * piece, piece, 0, h, 0);
    if (e != hipSuccess) {
      (void)hipMemRelease(h);
      break;
    }
    b[i].pieces.push_back(h);
  }
  // This device, and the other devices of the context's ranks (loopback
  // contexts over several GPUs copy between them; a one-rank-per-process
  // context maps its buffers for its own device only, so no process sets up
  // mappings on the other GPUs of a node).
  std::vector<hipMemAccessDesc> acc;
  for (int q = -1; q < (int)c->access_devs.size(); ++q) {  // the owner first
    const int d = q < 0 ? dev : c->access_devs[q];
    int can = q < 0;
    if (q >= 0 && (d == dev || hipDeviceCanAccessPeer(&can, d, dev) != hipSuccess)) can = 0;
    if (!can) continue;
    hipMemAccessDesc a = {};
    a.location.type = hipMemLocationTypeDevice;
    a.location.id = d;
    a.flags = hipMemAccessFlagsProtReadWrite;
    acc.push_back(a);
  }
  for (int i = 0; i < k && e == hipSuccess; ++i) e = hipMemSetAccess(b[i].base, bytes, acc.data(), acc.size());
  if (e != hipSuccess && acc.size() > 1) {
    // The other devices of a loopback context cannot map the pieces: an
    // owner-only mapping would fault at sort time on their copies and peer
    // stores, so these buffers are hipMalloc'd instead, which peer access
    // reaches (advisor r05).
    for (VmmBuffer& x : b) vmm_release(x, piece);
    (void)hipGetLastError();
    for (int i = 0; i < k; ++i) {
      const int rc = dev_alloc(outs[i], count);
      if (rc != LSB_OK) {
        for (int q = 0; q < i; ++q) (void)hipFree(*outs[q]);
        return rc;
      }
    }
    return LSB_OK;
  }
  if (e != hipSuccess) {
    const std::string why = hipGetErrorString(e);
    for (VmmBuffer& x : b) vmm_release(x, piece);
    return fail(LSB_ERR_NOMEM, "rec_alloc (hipMemCreate / hipMemMap / hipMemSetAccess)", why.c_str());
  }
  std::lock_guard<std::mutex> lock(g_vmm_mu);
  for (int i = 0; i < k; ++i) {
    *outs[i] = static_cast<Elem*>(b[i].base);
    g_vmm.push_back(std::move(b[i]));
  }
  return LSB_OK;
}

int rec_alloc(const lsb_ctx* c, Elem** out, size_t count) {
  Elem** const outs[1] = {out};
  return rec_alloc_group(c, outs, 1, count);
}

void rec_free(void* p) {
  if (!p) return;
  VmmBuffer b;
  {
    std::lock_guard<std::mutex> lock(g_vmm_mu);
    for (size_t i = 0; i < g_vmm.size(); ++i)
      if (g_vmm[i].base == p) {
        b = std::move(g_vmm[i]);
        g_vmm.erase(g_vmm.begin() + (long)i);
        break;
      }
  }
  if (!b.base) {
    (void)hipFree(p);
    return;
  }
  // hipFree waits for the device; unmapping does not: a kernel or copy still
  // using the pieces would fault.
  (void)hipDeviceSynchronize();
  vmm_release(b, b.piece);
}

// ---- record buffers A and B: the placement probe ---------------------------------
// Before round 5 the record buffers were hipMalloc'd, and how fast an LSD pass
// streamed between two of them depended on where the driver placed them: the
// pass ran at 6.7-7.3 ms between pairs allocated in one process
// (profiles/r04/v5_pick.log).  Round 4 therefore chose A and B among 8
// candidate buffers by timing one k_onesweep pass between every ordered pair
// (~0.7 s and 128 GiB at context creation at 2^30 records).  Buffers built
// from 1 GiB VMM pieces (rec_alloc) narrowed the spread, and round 5 first
// turned the probe off.  They did not remove it: a buffer of pieces can still
// be a slow destination as a whole (tools/kbench/pairbw2.hip: 8-piece buffers
// 3.7-3.9 against 2.9 ms, 16-piece 5.71-5.96 ms for the LSD write pattern;
// profiles/r05/region/pairbw2_*.log), which left one pass direction 2-5 % slow on about
// half the boxes.  Four candidates of VMM pieces take the sort from
// 53.96-56.26 ms to 53.68-54.08 (profiles/r05/probe/, 24 fresh processes on
// 3 boxes), so the probe is on again by default, smaller: 4 candidates, for
// buffers of at least 4 GiB, within half the free memory (~0.2 s and two
// buffers more at creation); LSB_PLACEMENT_CANDIDATES = K sets K (0: off; at
// most 8, within 90 %).  Never when another rank of this context shares the
// device (its timings would be the other rank's too, and the candidates its
// memory).
namespace {

// How many candidate buffers of `bytes` to try, at most `cap` (<= 2: no probing).
int placement_candidates(double bytes, int cap) {
  double share = 0.0;
  int K = std::min(placement_request(bytes, &share), cap);
  size_t free_b = 0, total_b = 0;
  if (K > 2 && bytes >= (double)(1ull << 30) && hipMemGetInfo(&free_b, &total_b) == hipSuccess) {
    // At most three candidates are live at once (alloc_records, alloc_third).
    if (3 * bytes > share * (double)free_b) K = 2;
  } else {
    (void)hipGetLastError();
    K = 2;
  }
  return K;
}

// Events of the placement probe on the rank's stream.
struct Prober {
  hipStream_t s;
  int64_t m;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  hipError_t err = hipSuccess;
  Prober(hipStream_t s_, int64_t m_) : s(s_), m(m_) {
    err = hipEventCreate(&e0);
    if (err == hipSuccess) err = hipEventCreate(&e1);
  }
  ~Prober() {
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
  }
};

// Up to K buffers of per records (at least `need`).
int alloc_candidates(const lsb_ctx* c, size_t per, int K, size_t need, std::vector<Elem*>& cand) {
  cand.clear();
  for (int k = 0; k < K; ++k) {
    Elem* p = nullptr;
    if (rec_alloc(c, &p, per) != LSB_OK) break;  // fewer candidates than hoped
    cand.push_back(p);
  }
  (void)hipGetLastError();
  if (cand.size() >= need) return LSB_OK;
  for (Elem* p : cand) rec_free(p);
  cand.clear();
  return fail(LSB_ERR_NOMEM, "alloc_candidates", "record buffers");
}

}  // namespace

// Times one k_onesweep pass x -> y over the rank's here records on the byte
// at `shift` (its sub-array histogram in hist_in), counting the byte at
// next_shift over y into hist_out for the next pass of a chain, with the
// rank's own look-back rows (onesweep_ensure).
double time_pass(Rank& r, Prober& pr, const Elem* x, Elem* y, int shift, int next_shift, const uint32_t* hist_in,
                 uint32_t* hist_out) {
  if (pr.err != hipSuccess) return 0.0;
  uint32_t epoch = r.os_epoch + 1;
  if (epoch >= (1u << 30)) epoch = 2;  // as onesweep_launch: keep the parity alternation
  pr.err = hipEventRecord(pr.e0, r.stream);
  lsb::OnesweepExtra probe;
  probe.probe = true;  // k_onesweep_probe: the same pass under its own name (profiles)
  if (pr.err == hipSuccess)
    pr.err = lsb::launch_onesweep(x, y, r.here, shift, next_shift, hist_in, hist_out, r.os_status, r.os_ctr, epoch,
                                  r.os_ctr + lsb::kOnesweepSubs, r.os_grid, r.stream, probe);
  if (pr.err == hipSuccess) r.os_epoch = epoch;
  if (pr.err == hipSuccess) pr.err = hipEventRecord(pr.e1, r.stream);
  if (pr.err == hipSuccess) pr.err = hipEventSynchronize(pr.e1);
  float t = 0.f;
  if (pr.err == hipSuccess) pr.err = hipEventElapsedTime(&t, pr.e0, pr.e1);
  return t;
}

namespace {

// A chain of timed passes: each moves the latest records from the buffer
// holding them into `dst`, on the next byte, with the histogram the pass
// before counted (one k_subhist read at the start only).
struct Chain {
  Rank& r;
  Prober& pr;
  uint32_t* h[2];
  int cur = 0, shift = 0;
  Elem* holder;
  Chain(Rank& r_, Prober& pr_, uint32_t* hist2, Elem* first) : r(r_), pr(pr_), h{hist2, hist2 + lsb::kOnesweepSubs * lsb::kBuckets}, holder(first) {
    if (pr.err == hipSuccess) pr.err = lsb::launch_subhist(first, r.here, 0, r.os_grid, h[0], nullptr, r.stream);
  }
  int next() const { return (shift + lsb::kDigitBits) & 63; }
  // Times holder -> dst and leaves the chain where it was: a pass does not
  // touch its input, so the holder still has the records (and h[cur] their
  // histogram), and a losing candidate is freed without a pass moving the
  // records back.
  double attempt(Elem* dst) { return time_pass(r, pr, holder, dst, shift, next(), h[cur], h[cur ^ 1]); }
  // Moves the chain on to dst, right after attempt(dst) (which counted dst's
  // histogram into h[cur ^ 1]).
  void advance(Elem* dst) {
    cur ^= 1;
    shift = next();
    holder = dst;
  }
  double pass(Elem* dst) {
    const double t = attempt(dst);
    advance(dst);
    return t;
  }
};

}  // namespace

// After a probe: a probe pass that gave up on its look-back leaves the sort's
// give-up word set and its status rows of an older parity.  Start them over
// (as onesweep_check does) and fail the creation rather than hand the next
// sort a false error.
int probe_check(Rank& r) {
  uint32_t w = 0;
  HIP_TRY(hipMemcpy(&w, r.os_ctr + lsb::kOnesweepSubs, sizeof w, hipMemcpyDeviceToHost));
  if (w == 0) return LSB_OK;
  HIP_TRY(hipMemset(r.os_ctr + lsb::kOnesweepSubs, 0, sizeof(uint32_t)));
  HIP_TRY(hipMemset(r.os_status, 0, (size_t)lsb::onesweep_tiles(r.here) * lsb::kBuckets * sizeof(uint32_t)));
  r.os_epoch = 0;
  return fail(LSB_ERR_HIP, "placement probe", "k_onesweep look-back timed out");
}

int placement_request(double bytes, double* free_share) {
  if (const char* e = getenv("LSB_PLACEMENT_CANDIDATES")) {
    *free_share = 0.9;
    return std::min(atoi(e), 8);
  }
  *free_share = 0.5;
  return bytes >= kProbeMinBytes ? kDefaultCandidates : 0;
}

int64_t region_min() {
  if (const char* e = getenv("LSB_REGION_MIN")) return std::max<int64_t>(atoll(e), int64_t(1) << 16);
  return lsb::kRegionMin;
}

int64_t region_cap_for(int64_t per, int P) { return P == 1 ? lsb::region_cap(per, region_min()) : 0; }

int64_t record_capacity(int64_t per, int P) {
  const int64_t cap = region_cap_for(per, P);
  return cap > 0 ? std::max(per, lsb::region_stride(cap) * lsb::kRegions) : per;
}

// The probe times each candidate once, as a destination: a buffer of pieces
// is slow or fast as the destination of the LSD write pattern as a whole,
// whatever the source (tools/kbench/pairbw2.hip), so round 5's
// matrix of a timed pass between every ordered pair of K candidates measured
// each destination K - 1 times and held all K buffers at once.  Here the
// passes form one chain (each pass's input histogram counted by the pass
// before it: one k_subhist read in all): X (PCG keys) and Y first, each once
// a destination; then every further candidate Z once (the holder of the
// records -> Z), and whichever of the two kept buffers is the slower
// destination is freed at once (the chain moves on to Z) -- or Z, and the
// chain stays where it was (Chain::attempt: a pass leaves its input as it
// was, so no pass moves the records back).  K + 1 passes (5 at K = 4, one of
// them the warm-up; round 5: 13 passes and 13 histogram reads) and three
// buffers live: the probe's transient memory is one buffer (round 5: K - 2
// at once).  Interleaved with round 5's form in fresh processes, 53.65-53.92
// ms per sort against 53.66-53.90 (profiles/r06/probe/); a form timing every
// candidate twice gave the same (53.66-53.86) for 0.05 s more creation time.
int alloc_records(lsb_ctx* c, Rank& r) {
  const size_t per = (size_t)record_capacity(c->per, c->P);
  r.cap = (int64_t)per;
  r.rg_cap = region_cap_for(c->per, c->P);
  int K = c->shared_device ? 0 : placement_candidates((double)per * sizeof(Elem), 8);
  r.placement_k = 0;
  if (K <= 2 || r.here < (int64_t)lsb::kTile * lsb::kOnesweepSubs || r.here > lsb::kOnesweepMaxElems) {
    // LSB_ALLOC_R_EARLY=1 (experiment): R with A and B, at creation
    const char* early = getenv("LSB_ALLOC_R_EARLY");
    Elem** const outs[3] = {&r.A, &r.B, &r.R};
    return rec_alloc_group(c, outs, early && atoi(early) ? 3 : 2, per);
  }
  std::vector<Elem*> cand;
  LSB_TRY(alloc_candidates(c, per, 2, 2, cand));
  Elem* keep[2] = {cand[0], cand[1]};
  Elem* z = nullptr;
  auto give_up = [&](int rc) {
    for (Elem* p : {keep[0], keep[1], z}) rec_free(p);
    return rc;
  };
  int rc = onesweep_ensure(r);
  if (rc != LSB_OK) return give_up(rc);
  // LSB_PLACEMENT_PICK=worst keeps the slowest destinations instead
  // (experiments: tools/alloc_probe.py checks that the probe predicts the passes).
  const char* pick = getenv("LSB_PLACEMENT_PICK");
  const bool pick_worst = pick && strcmp(pick, "worst") == 0;
  auto better = [&](double a, double b) { return pick_worst ? a > b : a < b; };
  Prober pr(r.stream, r.here);
  if (pr.err == hipSuccess) pr.err = lsb::launch_pcg_fill(keep[0], r.here, 0x5eed, 0, lsb::KeyGen(), r.stream);
  Chain ch(r, pr, r.os_hist, keep[0]);
  (void)ch.pass(keep[1]);  // warm-up
  double ms[2];
  ms[0] = ch.pass(keep[0]);
  ms[1] = ch.pass(keep[1]);  // the records are in keep[1]
  const double first_pair = 0.5 * (ms[0] + ms[1]);
  double worst = std::max(ms[0], ms[1]);
  int tried = 2;
  for (; tried < K && pr.err == hipSuccess; ++tried) {
    if (rec_alloc(c, &z, per) != LSB_OK) {  // fewer candidates than hoped
      (void)hipGetLastError();
      z = nullptr;
      break;
    }
    const double t = ch.attempt(z);
    worst = std::max(worst, t);
    const int slow = better(ms[0], ms[1]) ? 1 : 0;
    if (better(t, ms[slow])) {  // z replaces the slower kept buffer
      ch.advance(z);            // the records are in z
      rec_free(keep[slow]);
      keep[slow] = z;
      ms[slow] = t;
    } else {
      rec_free(z);  // the records are still where they were
    }
    z = nullptr;
  }
  if (pr.err != hipSuccess) return give_up(fail(LSB_ERR_HIP, "alloc_records: placement probe", hipGetErrorString(pr.err)));
  rc = probe_check(r);
  if (rc != LSB_OK) return give_up(rc);
  r.placement_k = tried;
  r.placement_ms[0] = 0.5 * (ms[0] + ms[1]);
  r.placement_ms[1] = first_pair;  // the first two buffers allocated
  r.placement_ms[2] = worst;       // the slowest destination timed
  r.A = keep[0];
  r.B = keep[1];
  return LSB_OK;
}

// The third record buffer R (receive buffer of the exchanges, the hybrid's
// third pass buffer), placed like A and B: among up to 3 candidates, the
// fastest destination (once each, a timed pass B -> candidate that leaves
// the records in B; B is scratch whenever R is first needed: before a hybrid sort,
// at an exchange before its placement), each loser freed at once (two
// buffers live at most).  A may hold records by then and is not touched; the
// chain counts into histograms of its own, since a sort may hold one in
// r.os_hist.
int alloc_third(lsb_ctx* c, Rank& r) {
  // As many records as A and B: the hybrid permutes the three buffers, and
  // the regional first pass writes into whichever one is B by then.
  const size_t per = (size_t)r.cap;
  int K = r.placement_k > 0 ? placement_candidates((double)per * sizeof(Elem), 3) : 1;  // probed A and B only
  if (K <= 2) K = 1;
  if (K == 1 || !r.os_status) return rec_alloc(c, &r.R, per);
  uint32_t* hist = nullptr;
  LSB_TRY(dev_alloc(&hist, (size_t)2 * lsb::kOnesweepSubs * lsb::kBuckets));
  Prober pr(r.stream, r.here);
  pr.err = lsb::launch_pcg_fill(r.B, r.here, 0x5eed + 16, 0, lsb::KeyGen(), r.stream);
  Chain ch(r, pr, hist, r.B);
  Elem* best = nullptr;
  double best_ms = 1e300;
  int rc = LSB_OK;
  for (int k = 0; k < K && pr.err == hipSuccess; ++k) {
    Elem* z = nullptr;
    if (rec_alloc(c, &z, per) != LSB_OK) {  // fewer candidates than hoped
      (void)hipGetLastError();
      break;
    }
    const double t = ch.attempt(z);  // the records stay in B
    if (t < best_ms) {
      rec_free(best);
      best = z;
      best_ms = t;
    } else {
      rec_free(z);
    }
  }
  (void)hipFree(hist);
  if (pr.err != hipSuccess) rc = fail(LSB_ERR_HIP, "alloc_third: placement probe", hipGetErrorString(pr.err));
  if (rc == LSB_OK && !best) rc = fail(LSB_ERR_NOMEM, "alloc_third", "record buffer");
  if (rc == LSB_OK) rc = probe_check(r);
  if (rc != LSB_OK) {
    rec_free(best);
    return rc;
  }
  r.R = best;
  return LSB_OK;
}

}  // namespace lsb_rt
