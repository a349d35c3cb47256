// The per-digit exchange (radix_bits 8 / 16, P > 1 or forced): the reference's
// globalShuffle after its localShuffle (mpi/mpi_lsbsort.cpp:481-577).
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
//
// Three transports behind one driver: in-process loopback (device copies
// standing in for the collectives), one rank per process (RCCL, or the
// caller's host callbacks), and the opt-in peer stores (shmem_putmem /
// MPI_Put form).  sort_exchange_onesweep is lsb_sort of these forms with
// single-read local passes and gathered passes after count-only placements.
#include "lsb_rt.h"

namespace lsb_rt {

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

// join_place after the last slice of an exchange, timed (LSB_K_PLACE_TAIL):
// from the moment the rank's stream has issued its last transfer to the end
// of the placement, i.e. the placement work not overlapped with the wire.
int join_place_timed(lsb_ctx* c, Rank& r) {
  Timer t(c, &r, LSB_K_PLACE_TAIL);
  return join_place(r);
}

// [p, p + cnt) lies inside one of rank q's record buffers.  Every device
// copy and placement of the exchange checks its ranges on the host first, so
// a plan gone wrong fails the sort instead of faulting the device.
bool in_buffers(const Rank& q, const Elem* p, int64_t cnt) {
  for (const Elem* b : {q.A, q.B, q.R})
    if (b && cnt >= 0 && p >= b && p + cnt <= b + q.cap) return true;
  return false;
}

int copy_range(const lsb_ctx*, Rank& dst_rank, Elem* dst, const Rank& src_rank, const Elem* src, int64_t cnt,
               hipStream_t s) {
  if (cnt <= 0) return LSB_OK;
  if (!in_buffers(dst_rank, dst, cnt) || !in_buffers(src_rank, src, cnt))
    return fail(LSB_ERR_STATE, "exchange copy", "range outside the record buffers");
  if (dst_rank.dev == src_rank.dev) {
    // One device: a copy kernel (addresses through the page tables only).
    HIP_TRY(lsb::launch_copy_records(dst, src, cnt, s));
  } else {
    HIP_TRY(hipMemcpyAsync(dst, src, (size_t)cnt * sizeof(Elem), hipMemcpyDefault, s));
  }
  return LSB_OK;
}

// Place one source's received range [k0, k0 + cnt) (records at src) into B.
int place_range(lsb_ctx* c, Rank& r, int shift, int src_rank, const Elem* src, int64_t k0,
                int64_t cnt) {
  if (cnt <= 0) return LSB_OK;
  if (!in_buffers(r, src, cnt) || k0 < 0 || k0 + cnt > r.cap)
    return fail(LSB_ERR_STATE, "exchange placement", "range outside the record buffers");
  // 32 algorithmic bytes per placed record, 16 per record only counted
  c->xs_place_bytes += cnt * (r.gather_next ? 16 : 32);
  (r.gather_next ? c->xs_counted : c->xs_placed) += cnt;
  Timer t(c, &r, LSB_K_PLACE, r.pstream);
  HIP_TRY(lsb::launch_place(src, r.B, r.here, k0, cnt, shift, c->nb,
                            r.place + (size_t)src_rank * c->nb, r.pstream, r.place_next,
                            r.place_hist, !r.gather_next, r.os_halves == 2));
  return LSB_OK;
}

// The receive buffer, allocated at the first all-to-all of the context.
int ensure_recv(lsb_ctx* c, Rank& r) {
  if (r.R) return LSB_OK;
  HIP_TRY(hipSetDevice(r.dev));
  return alloc_third(c, r);
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
    for (int64_t& a : g.self_adj) a = r.send_displs[me] - r.recv_displs[me];
    g.chunk_shift = 8;
    g.place = r.place;
    g.gstart = r.gstart;
    g.gadj = r.gstart + (size_t)c->P * c->nb;
    g.desc = r.gdesc;
    g.P = c->P;
    g.nb = c->nb;
    g.me = me;
    g.self_in_a = !(c->self_coll && c->mode != Mode::kLoopback);
    g.a_len = g.r_len = r.cap;
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
    const int64_t lo = slice_part(r.recv_counts[s], j, slices_of(c));
    const int64_t hi = slice_part(r.recv_counts[s], j + 1, slices_of(c));
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
      HIP_TRY(hipSetDevice(q.dev));
      Timer t(c, &q, LSB_K_WIRE);
      for (Rank& s : c->ranks) {
        if (s.rank == q.rank) continue;
        const int64_t cnt = s.send_counts[q.rank];
        const int64_t lo = slice_part(cnt, j, slices_of(c)), hi = slice_part(cnt, j + 1, slices_of(c));
        if (hi <= lo) continue;
        LSB_TRY(copy_range(c, q, q.R + q.recv_displs[s.rank] + lo, s, s.A + s.send_displs[q.rank] + lo, hi - lo,
                           q.stream));
      }
    }
    for (Rank& q : c->ranks) LSB_TRY(place_slice(c, q, shift, j));
  }
  // Every rank's copies out of A must be done before any rank's next pass
  // rewrites that A (it becomes B after the swap).
  for (Rank& r : c->ranks) {
    LSB_TRY(join_place_timed(c, r));
    HIP_TRY(hipStreamSynchronize(r.stream));
    end_placement(r);
  }
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
  // IPC handles name hipMalloc memory only: a record buffer built from VMM
  // pieces (rec_alloc) is replaced by a hipMalloc'd one holding its records,
  // of the same capacity: a later sort with the exchange off may start with
  // the regional first pass, which writes r.cap slots (advisor r05).
  for (int k = 0; k < 2; ++k) {
    Elem* old = r.buf[k];
    if (!rec_is_vmm(old)) continue;
    Elem* nu = nullptr;
    LSB_TRY(dev_alloc(&nu, (size_t)std::max(r.cap, c->per)));
    HIP_TRY(hipMemcpyAsync(nu, old, sizeof(Elem) * (size_t)c->per, hipMemcpyDeviceToDevice, r.stream));
    HIP_TRY(hipStreamSynchronize(r.stream));
    for (Elem** p : {&r.A, &r.B, &r.R})
      if (*p == old) *p = nu;
    r.buf[k] = nu;
    if (c->mode == Mode::kRccl) mark_rccl_vmm_released();
    rec_free(old);
  }
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
    Timer t(c, &r, LSB_K_WIRE);  // the stores are the transfer (no payload counted)
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
  // Calls of more than 1 GiB per peer are cut (coll_alltoallv_u64), alike on
  // every rank: by the largest peer segment of this exchange on any rank, one
  // all-reduce of one word, asked only when a block could exceed it at all.
  int64_t seg = c->per;
  if (c->mode == Mode::kRccl && (size_t)slice_bound(c->per, 0, slices_of(c)) * 2 > max_call_u64()) {
    int64_t m = 0;
    for (int q = 0; q < P; ++q)
      if (q != me || c->self_coll) m = std::max(m, std::max(r.send_counts[q], r.recv_counts[q]));
    int64_t neg = -m;
    LSB_TRY(allreduce_min_i64(c, &neg));
    seg = -neg;
  }
  // ncclAllToAllv per slice (the reference's MPI_Alltoallv,
  // mpi/mpi_lsbsort.cpp:316-324), in uint64 units; the self entry is 0
  // because the self segment was placed straight out of A (unless
  // LSB_OPT_EXCHANGE_SELF sends it through the collective too).
  const bool skip_self = !c->self_coll;
  std::vector<size_t> sc(P), sd(P), rc(P), rdp(P);
  for (int j = 0; j < slices_of(c); ++j) {
    {
      Timer t(c, &r, LSB_K_WIRE);
      for (int q = 0; q < P; ++q) {
        const int64_t slo = slice_part(r.send_counts[q], j, slices_of(c));
        const int64_t shi = slice_part(r.send_counts[q], j + 1, slices_of(c));
        const int64_t rlo = slice_part(r.recv_counts[q], j, slices_of(c));
        const int64_t rhi = slice_part(r.recv_counts[q], j + 1, slices_of(c));
        sc[q] = q == me && skip_self ? 0 : (size_t)(shi - slo) * 2;
        rc[q] = q == me && skip_self ? 0 : (size_t)(rhi - rlo) * 2;
        sd[q] = (size_t)(r.send_displs[q] + slo) * 2;
        rdp[q] = (size_t)(r.recv_displs[q] + rlo) * 2;
      }
      LSB_TRY(coll_alltoallv_u64(c, r, reinterpret_cast<const uint64_t*>(r.A), sc.data(),
                                 sd.data(), reinterpret_cast<uint64_t*>(r.R), rc.data(),
                                 rdp.data(), (size_t)slice_bound(seg, j, slices_of(c)) * 2));
    }
    LSB_TRY(place_slice(c, r, shift, j));
  }
  LSB_TRY(join_place_timed(c, r));
  end_placement(r);
  return LSB_OK;
}

int exchange_digit(lsb_ctx* c, int digit) {
  ++c->xs_exchanges;
  if (c->peer) return exchange_peer(c, digit);
  if (c->mode != Mode::kLoopback) return exchange_rccl(c, digit);
  return exchange_loopback(c, digit);
}

// ---- the per-digit exchange in chunks (LSB_OPT_EXCHANGE_CHUNKS) -------------
// the exchange of chunk k overlaps the local
// work of chunk k + 1.  The reference runs localShuffle to the end and only
// then the whole exchange (mpi/mpi_lsbsort.cpp:481-577), and so does
// exchange_digit: the high-byte pass, then the wire.  Here, for a 16-bit
// digit d whose low-byte pass has run (A sorted by the low byte l):
//   1. one read of A (launch_count16_chunks) counts the digit's 65536 values
//      and, per chunk k (the records with l in [k 256 / C, (k + 1) 256 / C):
//      a contiguous range of A), the high byte's sub-array histogram;
//   2. the counts are all-gathered and planned as before, except that a
//      source's pieces lie in R in chunk order (launch_plan with cshift);
//   3. chunk by chunk: chunk k's high-byte pass (one k_onesweep over its range
//      of A, into the same range of B) on the rank's stream, then chunk k's
//      all-to-all on the wire stream while chunk k + 1's pass runs, then its
//      count-only placement (or, the last exchange, its placement once every
//      pass is done) on the placement stream.
// Inside chunk k the records end up ordered by (h, l), so every owner's
// share is one contiguous range, and a digit's records all lie in one chunk:
// the placed order, (digit, source), is the reference's, and the output is
// the same bit for bit.  The price is step 1's read (16 B per record); what it
// buys is the high-byte pass under the wire.
constexpr int64_t kChunkMinPer = int64_t(1) << 16;

bool chunked_applies(const lsb_ctx* c, uint64_t varying, int digit) {
  if (c->xchunks < 2 || c->bits != 16 || c->peer || c->mode == Mode::kOps || !exchanging(c)) return false;
  const int lo = digit * 16;
  if (((varying >> lo) & 0xFF) == 0 || ((varying >> (lo + 8)) & 0xFF) == 0) return false;
  return c->per >= kChunkMinPer;
}

namespace {

int cshift_of(int C) { return C >= 8 ? 5 : C == 4 ? 6 : 7; }

// One rank's chunk geometry (host) after the plan.
struct ChunkGeom {
  std::vector<int64_t> lo;     // [C + 1] chunk bounds in A and B
  std::vector<int64_t> send;   // [q * C + k] my records of chunk k for owner q
  std::vector<int64_t> recv;   // [s * C + k] source s's records of chunk k for me
  std::vector<int64_t> sdisp;  // [q * C + k] where owner q's share starts inside chunk k
  std::vector<int64_t> rpre;   // [s * C + k] where chunk k starts inside source s's range of R
};

int chunk_ensure(lsb_ctx* c, Rank& r) {
  if (r.xstream) return LSB_OK;
  HIP_TRY(hipSetDevice(r.dev));
  if (!r.ck_hist) LSB_TRY(dev_alloc(&r.ck_hist, (size_t)lsb::kMaxExchangeChunks * lsb::kOnesweepSubs * lsb::kBuckets));
  if (!r.ck_counts) LSB_TRY(dev_alloc(&r.ck_counts, (size_t)2 * c->P * lsb::kMaxExchangeChunks));
  if (!r.ck_counts_h) LSB_TRY(host_alloc(&r.ck_counts_h, (size_t)2 * c->P * lsb::kMaxExchangeChunks));
  if (!r.lo_hist_h) LSB_TRY(host_alloc(&r.lo_hist_h, (size_t)lsb::kOnesweepSubs * lsb::kBuckets));
  for (hipEvent_t& e : r.ck_hi)
    if (!e) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (hipEvent_t& e : r.ck_wire)
    if (!e) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  if (!r.xdone) HIP_TRY(hipEventCreateWithFlags(&r.xdone, hipEventDisableTiming));
  HIP_TRY(hipStreamCreateWithFlags(&r.xstream, hipStreamNonBlocking));  // last: marks the set complete
  return LSB_OK;
}

// The plan in chunk order; the send / recv totals and the per-chunk counts
// come back to the host (after a stream sync: chunk_geom).
int chunk_plan(lsb_ctx* c, Rank& r, int cs) {
  HIP_TRY(hipSetDevice(r.dev));
  if (r.gather_next && !r.gstart) {
    LSB_TRY(dev_alloc(&r.gstart, (size_t)2 * c->P * c->nb));  // gstart, then gadj
    LSB_TRY(dev_alloc(&r.gdesc, (size_t)lsb::onesweep_tiles(r.here)));
  }
  const int C = lsb::kBuckets >> cs;
  {
    Timer t(c, &r, LSB_K_EXCHANGE);
    HIP_TRY(lsb::launch_plan(r.gather, c->P, c->nb, r.rank, c->n, r.plan_work, r.plan_total, r.place,
                             r.plan_counts, r.stream, r.gather_next ? r.gstart : nullptr, cs, r.ck_counts));
  }
  HIP_TRY(hipMemcpyAsync(r.counts_h, r.plan_counts, sizeof(int64_t) * 2 * c->P, hipMemcpyDeviceToHost, r.stream));
  HIP_TRY(hipMemcpyAsync(r.ck_counts_h, r.ck_counts, sizeof(int64_t) * 2 * c->P * C, hipMemcpyDeviceToHost,
                         r.stream));
  return LSB_OK;
}

int chunk_geom(lsb_ctx* c, Rank& r, int C, ChunkGeom& g) {
  const int P = c->P, lw = lsb::kBuckets / C;
  g.lo.assign(C + 1, 0);
  if (r.here > 0) {
    int64_t acc = 0;
    for (int l = 0; l < lsb::kBuckets; ++l) {
      if (l % lw == 0) g.lo[l / lw] = acc;
      for (int x = 0; x < lsb::kOnesweepSubs; ++x) acc += r.lo_hist_h[x * lsb::kBuckets + l];
    }
    g.lo[C] = acc;
    if (acc != r.here) return fail(LSB_ERR_STATE, "exchange_chunked", "chunk bounds do not cover the block");
  }
  g.send.assign((size_t)P * C, 0);
  g.recv.assign((size_t)P * C, 0);
  g.sdisp.assign((size_t)P * C, 0);
  g.rpre.assign((size_t)P * C, 0);
  for (int i = 0; i < P * C; ++i) {
    g.send[i] = r.ck_counts_h[i];
    g.recv[i] = r.ck_counts_h[(size_t)P * C + i];
  }
  for (int k = 0; k < C; ++k) {
    int64_t a = 0;
    for (int q = 0; q < P; ++q) {
      g.sdisp[(size_t)q * C + k] = a;
      a += g.send[(size_t)q * C + k];
    }
    if (a != g.lo[k + 1] - g.lo[k]) return fail(LSB_ERR_STATE, "exchange_chunked", "chunk send counts");
  }
  for (int q = 0; q < P; ++q) {
    int64_t a = 0, sa = 0;
    for (int k = 0; k < C; ++k) {
      g.rpre[(size_t)q * C + k] = a;
      a += g.recv[(size_t)q * C + k];
      sa += g.send[(size_t)q * C + k];
    }
    if (a != r.recv_counts[q] || sa != r.send_counts[q])
      return fail(LSB_ERR_STATE, "exchange_chunked", "chunk counts do not add up");
  }
  return LSB_OK;
}

}  // namespace

int exchange_chunked(lsb_ctx* c, int digit, const std::vector<const uint32_t*>& lo_hist) {
  ++c->xs_exchanges;
  const int C = std::min(c->xchunks, lsb::kMaxExchangeChunks), cs = cshift_of(C), P = c->P;
  const size_t nb = (size_t)c->nb;
  const int shift = digit * 16, hi_shift = shift + lsb::kDigitBits;
  const bool loop = c->mode == Mode::kLoopback;
  const size_t nr = c->ranks.size();
  std::vector<ChunkGeom> geo(nr);
  std::vector<Elem*> X(nr), Y(nr);  // the high-byte pass reads X (A, sorted by l) and writes Y (B)
  // 1. the count read
  for (size_t i = 0; i < nr; ++i) {
    Rank& r = c->ranks[i];
    LSB_TRY(chunk_ensure(c, r));
    LSB_TRY(ensure_recv(c, r));
    HIP_TRY(hipSetDevice(r.dev));
    X[i] = r.A;
    Y[i] = r.B;
    {
      Timer t(c, &r, LSB_K_UPSWEEP);
      HIP_TRY(lsb::launch_count16_chunks(r.A, r.here, shift, lo_hist[i], cs, r.os_grid, r.totals16, r.ck_hist,
                                         r.stream));
    }
    HIP_TRY(hipMemcpyAsync(r.lo_hist_h, lo_hist[i], sizeof(uint32_t) * lsb::kOnesweepSubs * lsb::kBuckets,
                           hipMemcpyDeviceToHost, r.stream));
  }
  // 2. the counts to every rank, the plan in chunk order
  if (loop) {
    for (Rank& r : c->ranks) {
      HIP_TRY(hipSetDevice(r.dev));
      HIP_TRY(hipStreamSynchronize(r.stream));
    }
    for (Rank& q : c->ranks) {
      HIP_TRY(hipSetDevice(q.dev));
      for (Rank& s : c->ranks)
        HIP_TRY(hipMemcpyAsync(q.gather + (size_t)s.rank * nb, s.totals16, sizeof(uint64_t) * nb, hipMemcpyDefault,
                               q.stream));
      LSB_TRY(chunk_plan(c, q, cs));
    }
  } else {
    Rank& r = c->ranks[0];
    {
      Timer t(c, &r, LSB_K_EXCHANGE);
      LSB_TRY(coll_allgather_u64(c, r, r.totals16, r.gather, nb));
    }
    LSB_TRY(chunk_plan(c, r, cs));
  }
  for (size_t i = 0; i < nr; ++i) {
    Rank& r = c->ranks[i];
    HIP_TRY(hipSetDevice(r.dev));
    HIP_TRY(hipStreamSynchronize(r.stream));
    plan_fetch(c, r);
    LSB_TRY(chunk_geom(c, r, C, geo[i]));
  }
  if (loop)
    for (size_t q = 0; q < nr; ++q)
      for (size_t s = 0; s < nr; ++s)
        for (int k = 0; k < C; ++k)
          if (geo[s].send[q * C + k] != geo[q].recv[s * C + k])
            return fail(LSB_ERR_STATE, "exchange_chunked", "send/recv count mismatch");
  const bool self_in_r = c->self_coll && !loop;
  // Where the next (gathered) pass finds each tile's records: peers' pieces
  // in R, my own in Y, chunk k's at its own offset.
  for (size_t i = 0; i < nr; ++i) {
    Rank& r = c->ranks[i];
    const int me = r.rank;
    if (!r.gather_next) continue;
    lsb::GatherSrc& g = r.gsrc;
    g.R = r.R;
    g.A = Y[i];
    for (int k = 0; k < lsb::kMaxExchangeChunks; ++k)
      g.self_adj[k] = k < C ? geo[i].lo[k] + geo[i].sdisp[(size_t)me * C + k] -
                                  (r.recv_displs[me] + geo[i].rpre[(size_t)me * C + k])
                            : 0;
    g.chunk_shift = cs;
    g.place = r.place;
    g.gstart = r.gstart;
    g.gadj = r.gstart + (size_t)P * nb;
    g.desc = r.gdesc;
    g.P = P;
    g.nb = c->nb;
    g.me = me;
    g.self_in_a = !self_in_r;
    g.a_len = g.r_len = r.cap;
    HIP_TRY(hipSetDevice(r.dev));
    Timer t(c, &r, LSB_K_EXCHANGE);
    HIP_TRY(lsb::launch_gather_desc(g, r.here, r.gdesc, r.stream));
  }
  // RCCL calls of more than 1 GiB per peer are cut alike on every rank
  // (coll_alltoallv_u64): the largest (peer, chunk) segment anywhere.
  int64_t seg = 0;
  if (!loop) {
    Rank& r = c->ranks[0];
    for (int q = 0; q < P; ++q)
      if (q != r.rank || c->self_coll)
        for (int k = 0; k < C; ++k)
          seg = std::max(seg, std::max(geo[0].send[(size_t)q * C + k], geo[0].recv[(size_t)q * C + k]));
    if (c->mode == Mode::kRccl && (size_t)c->per * 2 > max_call_u64()) {  // a chunk may hold the block
      int64_t neg = -seg;
      LSB_TRY(allreduce_min_i64(c, &neg));
      seg = -neg;
    } else {
      seg = c->per;
    }
  }
  // 3. chunk by chunk: the high-byte pass, then the wire
  for (int k = 0; k < C; ++k) {
    for (size_t i = 0; i < nr; ++i) {
      Rank& r = c->ranks[i];
      HIP_TRY(hipSetDevice(r.dev));
      const int64_t lo = geo[i].lo[k], m = geo[i].lo[k + 1] - lo;
      if (m > 0) {
        // Chunk passes differ in tile count: each starts from zeroed look-back
        // rows (epoch 1), and the next plain pass zeroes them all (os_dirty).
        r.os_dirty = true;
        HIP_TRY(hipMemsetAsync(r.os_status, 0, (size_t)lsb::onesweep_tiles(m) * lsb::kBuckets * sizeof(uint32_t),
                               r.stream));
        lsb::OnesweepExtra x;
        x.halves = r.os_halves;
        const int grid = std::max(lsb::kOnesweepSubs, (r.os_grid - c->xchunk_reserve) / 8 * 8);
        hipError_t e;
        if (c->fail_onesweep > 0 && --c->fail_onesweep == 0)  // LSB_OPT_FAIL_ONESWEEP (tests)
          return fail(LSB_ERR_HIP, "exchange_chunked: launch_onesweep", "injected launch failure (LSB_OPT_FAIL_ONESWEEP)");
        {
          Timer t(c, &r, LSB_K_SCATTER);
          e = lsb::launch_onesweep(X[i] + lo, Y[i] + lo, m, hi_shift, -1,
                                   r.ck_hist + (size_t)k * lsb::kOnesweepSubs * lsb::kBuckets, nullptr, r.os_status,
                                   r.os_ctr, 1, r.os_ctr + lsb::kOnesweepSubs, grid, r.stream, x);
        }
        if (e != hipSuccess) {
          (void)hipGetLastError();
          return fail(LSB_ERR_HIP, "exchange_chunked: launch_onesweep", hipGetErrorString(e));
        }
        count_pass_elems(c, m);
      }
      HIP_TRY(hipEventRecord(r.ck_hi[k], r.stream));
    }
    if (loop) {
      for (size_t q = 0; q < nr; ++q) {
        Rank& rq = c->ranks[q];
        HIP_TRY(hipSetDevice(rq.dev));
        for (size_t s = 0; s < nr; ++s) HIP_TRY(hipStreamWaitEvent(rq.xstream, c->ranks[s].ck_hi[k], 0));
        {
          Timer t(c, &rq, LSB_K_WIRE, rq.xstream);
          for (size_t s = 0; s < nr; ++s) {
            if (s == q) continue;
            const int64_t cnt = geo[q].recv[s * C + k];
            if (cnt <= 0) continue;
            const Elem* src = Y[s] + geo[s].lo[k] + geo[s].sdisp[q * C + k];
            LSB_TRY(copy_range(c, rq, rq.R + rq.recv_displs[s] + geo[q].rpre[s * C + k], c->ranks[s], src, cnt,
                               rq.xstream));
          }
        }
        HIP_TRY(hipEventRecord(rq.ck_wire[k], rq.xstream));
      }
    } else {
      Rank& r = c->ranks[0];
      const ChunkGeom& g = geo[0];
      const int me = r.rank;
      HIP_TRY(hipStreamWaitEvent(r.xstream, r.ck_hi[k], 0));
      std::vector<size_t> sc(P), sd(P), rc(P), rdp(P);
      for (int q = 0; q < P; ++q) {
        const bool skip = q == me && !c->self_coll;
        sc[q] = skip ? 0 : (size_t)g.send[(size_t)q * C + k] * 2;
        rc[q] = skip ? 0 : (size_t)g.recv[(size_t)q * C + k] * 2;
        sd[q] = (size_t)(g.lo[k] + g.sdisp[(size_t)q * C + k]) * 2;
        rdp[q] = (size_t)(r.recv_displs[q] + g.rpre[(size_t)q * C + k]) * 2;
      }
      {
        Timer t(c, &r, LSB_K_WIRE, r.xstream);
        LSB_TRY(coll_alltoallv_u64(c, r, reinterpret_cast<const uint64_t*>(Y[0]), sc.data(), sd.data(),
                                   reinterpret_cast<uint64_t*>(r.R), rc.data(), rdp.data(), (size_t)seg * 2,
                                   r.xstream));
      }
      HIP_TRY(hipEventRecord(r.ck_wire[k], r.xstream));
    }
  }
  // 4. placements, chunk k's once it has arrived (the last exchange's, which
  //    write X, also once every chunk pass has read X)
  for (size_t i = 0; i < nr; ++i) {
    Rank& r = c->ranks[i];
    const ChunkGeom& g = geo[i];
    const int me = r.rank;
    HIP_TRY(hipSetDevice(r.dev));
    r.A = Y[i];  // the records, ordered by the digit chunk by chunk (my own segment's source)
    r.B = X[i];  // the placement's destination
    if (!r.gather_next) HIP_TRY(hipStreamWaitEvent(r.pstream, r.ck_hi[C - 1], 0));
    for (int k = 0; k < C; ++k) {
      HIP_TRY(hipStreamWaitEvent(r.pstream, r.ck_wire[k], 0));
      for (int s = 0; s < P; ++s) {
        const int64_t cnt = g.recv[(size_t)s * C + k];
        const int64_t k0 = r.recv_displs[s] + g.rpre[(size_t)s * C + k];
        if (s == me && !self_in_r)
          LSB_TRY(place_range(c, r, shift, s, Y[i] + g.lo[k] + g.sdisp[(size_t)me * C + k], k0, cnt));
        else
          LSB_TRY(place_range(c, r, shift, s, r.R + k0, k0, cnt));
      }
    }
    HIP_TRY(hipEventRecord(r.xdone, r.xstream));
    HIP_TRY(hipStreamWaitEvent(r.stream, r.xdone, 0));
    LSB_TRY(join_place_timed(c, r));
    end_placement(r);
  }
  // Every rank's copies out of Y must be done before any rank's next pass
  // rewrites it (loopback; RCCL ranks wait for their own wire stream above).
  if (loop)
    for (Rank& r : c->ranks) {
      HIP_TRY(hipSetDevice(r.dev));
      HIP_TRY(hipStreamSynchronize(r.stream));
    }
  return LSB_OK;
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
  // A gathered pass always takes the whole stage: the split stage's gathered
  // instances spill (168 VGPRs at 3 workgroups per CU: 160-236 B per lane),
  // while the whole stage's fit (128 VGPRs, no or 12 B of spill) and cost
  // skewed keys ~1 % per pass against the split (58.53 vs 59.24 ms per Zipf
  // sort, profiles/ab/r02_ab28_zipf_stage.log) -- far less than the placement
  // the gathered pass saves (32 B per record).
  extra.halves = r.gather_pending ? 1 : r.os_halves;
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
  std::vector<const uint32_t*> lo_hist(c->ranks.size(), nullptr);
  for (size_t i = 0; i < steps.size(); ++i) {
    const Step& st = steps[i];
    const int after = i + 1 < steps.size() ? steps[i + 1].shift : -1;
    // LSB_OPT_EXCHANGE_CHUNKS: the low byte's pass counts nothing for the next
    // (exchange_chunked's read does), and the high byte's pass runs chunk by
    // chunk inside exchange_chunked.
    const bool chunked = chunked_applies(c, varying, st.digit);
    if (chunked && st.exch) {
      begin_pass(c, st.shift);
    } else {
      // 16-bit digit: its high-byte pass counts the 65536 digits (a constant
      // high byte leaves the count to digit_counts' read of A).
      const bool c16 = c->bits == 16 && st.exch && st.shift == st.digit * 16 + lsb::kDigitBits;
      begin_pass(c, st.shift);
      for (size_t k = 0; k < c->ranks.size(); ++k) {
        Rank& r = c->ranks[k];
        lsb::OnesweepExtra x;
        if (st.exch && c->bits == 8) x.totals = r.totals;
        if (c16) x.count16 = r.totals16;
        r.counts_ready = c16;
        LSB_TRY(local_pass_os(c, r, st.shift, st.exch || chunked ? -1 : after, x));
        // the pass's input histogram (os_cur stays: next = -1): the chunk bounds
        lo_hist[k] = r.os_hist + (size_t)r.os_cur * lsb::kOnesweepSubs * lsb::kBuckets;
      }
    }
    ++c->last_local_passes;
    if (!st.exch) continue;
    for (Rank& r : c->ranks) {
      r.place_next = c->peer || r.here == 0 ? -1 : after;
      // Skewed keys too: their gathered pass takes the whole stage (local_pass_os).
      r.gather_next = c->gather && r.place_next >= 0;
      r.place_hist = nullptr;
      if (r.place_next >= 0) {
        r.place_hist = r.os_hist + (size_t)(r.os_cur ^ 1) * lsb::kOnesweepSubs * lsb::kBuckets;
        HIP_TRY(hipSetDevice(r.dev));
        HIP_TRY(hipMemsetAsync(r.place_hist, 0, sizeof(uint32_t) * lsb::kOnesweepSubs * lsb::kBuckets,
                               r.stream));
      }
    }
    ++c->last_exchanges;
    const int rc = chunked ? exchange_chunked(c, st.digit, lo_hist) : exchange_digit(c, st.digit);
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

}  // namespace lsb_rt
