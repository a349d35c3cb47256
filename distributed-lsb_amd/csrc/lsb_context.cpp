// Context and rank state of the runtime behind include/lsb.h: errors, HIP-event
// timing of launches (filed per local pass, lsb_get_pass_stats), a rank's
// buffers (DistributedArray::create, mpi/mpi_lsbsort.cpp:137-161; the record
// buffers themselves come from lsb_alloc.cpp), and the collectives of a
// one-rank-per-process context (RCCL, or the caller's host callbacks) that
// the pass driver and both exchange forms use.
#include "lsb_rt.h"

namespace lsb_rt {

thread_local std::string g_last_error;

const std::string& last_error() { return g_last_error; }

int fail(int code, const char* what, const char* detail) {
  char buf[512];
  snprintf(buf, sizeof buf, "%s: %s", what, detail ? detail : "");
  g_last_error = buf;
  if (getenv("LSB_DEBUG")) fprintf(stderr, "[lsb] %s\n", buf);
  return code;
}
// ---- timing -------------------------------------------------------------
// An event of the current device: from the pool (events are filed under the
// device they were created on), else a new one.
hipEvent_t take_event(lsb_ctx* c) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  for (size_t i = c->event_pool.size(); i-- > 0;)
    if (c->event_pool[i].first == dev) {
      hipEvent_t e = c->event_pool[i].second;
      c->event_pool.erase(c->event_pool.begin() + (long)i);
      return e;
    }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}


// The local pass the following launches belong to: the pass_cursor-th local
// pass of this sort, on the byte at `shift` (lsb_get_pass_stats).
void begin_pass(lsb_ctx* c, int shift) {
  c->cur_pass = c->pass_cursor++;
  if (c->cur_pass < LSB_MAX_PASSES) c->pass_shift[c->cur_pass] = shift;
}

// Records one local pass of m records processed (lsb_get_pass_stats); a
// scatter kernel's records also go to lsb_get_scatter_elems.
void count_pass_elems(lsb_ctx* c, int64_t m, bool scatter) {
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
    c->event_pool.push_back({p.dev, p.start});
    c->event_pool.push_back({p.dev, p.stop});
  }
  c->pending.clear();
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
  r.chunking = lsb::make_chunking(r.here, max_chunks_for_device(dev));
  const size_t hist_entries = (size_t)lsb::kBuckets * std::max(1, r.chunking.num_chunks);
  const size_t P = (size_t)c->P, nb = (size_t)c->nb;
  LSB_TRY(alloc_records(c, r));
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

int teardown_check(const lsb_ctx* c, const Rank& freeing) {
  int busy = 0;
  for (const Rank& q : c->ranks) {
    (void)hipSetDevice(q.dev);
    const hipStream_t s[3] = {q.stream, q.pstream, q.xstream};
    const char* name[3] = {"stream", "placement stream", "wire stream"};
    for (int k = 0; k < 3; ++k) {
      if (!s[k]) continue;
      const hipError_t e = hipStreamQuery(s[k]);
      (void)hipGetLastError();
      if (e == hipSuccess) continue;
      ++busy;
      fprintf(stderr, "[lsb] teardown check: rank %d's %s not idle (%s) as rank %d's record buffers are freed\n",
              q.rank, name[k], hipGetErrorString(e), freeing.rank);
    }
  }
  (void)hipSetDevice(freeing.dev);
  return busy;
}

void free_rank(Rank& r, const lsb_ctx* c) {
  (void)hipSetDevice(r.dev);
  // LSB_TEARDOWN_LEGACY (debug builds only): the order before round 5's fix,
  // this rank's stream alone, so that teardown_check can be seen to fire.
#ifdef LSB_DEBUG
  const bool legacy = getenv("LSB_TEARDOWN_LEGACY") != nullptr;
#else
  const bool legacy = false;
#endif
  if (r.stream) (void)hipStreamSynchronize(r.stream);
  if (r.pstream && !legacy) (void)hipStreamSynchronize(r.pstream);  // placements read R and write B
  if (r.xstream && !legacy) (void)hipStreamSynchronize(r.xstream);  // the chunked exchange's wire
#ifdef LSB_DEBUG
  if (c) (void)teardown_check(c, r);
#else
  (void)c;
#endif
  // RCCL has seen this context's record buffers: VMM ones released here make
  // later RCCL contexts of the process take hipMalloc'd ones (lsb_alloc.cpp).
  if (c && c->mode == Mode::kRccl)
    for (const Elem* p : {r.A, r.B, r.R})
      if (p && rec_is_vmm(p)) mark_rccl_vmm_released();
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
  (void)hipFree(r.os_status2);
  (void)hipFree(r.rg_buf);
  (void)hipHostFree(r.rg_h);
  (void)hipFree(r.gstart);
  (void)hipFree(r.gdesc);
  (void)hipFree(r.ck_hist);
  (void)hipFree(r.ck_counts);
  (void)hipHostFree(r.ck_counts_h);
  (void)hipHostFree(r.lo_hist_h);
  if (r.xstream) {
    (void)hipStreamSynchronize(r.xstream);
    (void)hipStreamDestroy(r.xstream);
  }
  for (hipEvent_t e : r.ck_hi)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : r.ck_wire)
    if (e) (void)hipEventDestroy(e);
  if (r.xdone) (void)hipEventDestroy(r.xdone);
  (void)hipFree(r.seg_base);
  (void)hipFree(r.os_hist);
  (void)hipFree(r.os_ctr);
  (void)hipHostFree(r.os_err_h);
  (void)hipHostFree(r.os_hist_h);
  rec_free(r.A);
  rec_free(r.B);
  rec_free(r.R);
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
// `bound`: a count no rank sends to any peer in this call exceeds (the same on
// every rank: every rank must issue the same RCCL calls).  RCCL moves a
// per-peer range of 2 GiB or more wrongly in a world of one (the x16 exchange
// at 2^28 records per rank, 2 GiB in its first slice, verified false:
// profiles/r05/x16dbg_probe.log; and RCCL alone, tools/rccl_big_call.cpp, RCCL
// 2.27.7: of a 2 GiB or 4 GiB range the second half comes back wrong, with
// ncclAllToAllv and with grouped ncclSend / ncclRecv; 512 MiB and 1 GiB
// right: profiles/r06/rccl_big/world1.jsonl).  Two ranks over RCCL's socket
// transport moved 2 and 4 GiB per peer, self ranges included, correctly
// (world2.jsonl); xGMI is untested here, so the cut stays at N > 1 too (at
// N = 8 with 2^30 uniform records per GPU no call is cut).  An RCCL call whose
// bound exceeds max_call_u64() goes as ceil(bound / max_call_u64()) calls,
// call i carrying part i of every peer's range on both sides.  (The reference's
// MPI_Alltoallv takes int counts and cannot pass 2^31 records at all,
// mpi/mpi_lsbsort.cpp:292-313.)
size_t max_call_u64() {
  static const size_t v = [] {
    const char* e = getenv("LSB_RCCL_CALL_U64");
    const long long x = e ? atoll(e) : 0;
    return x > 0 ? (size_t)x : kMaxCallU64;
  }();
  return v;
}

int coll_alltoallv_u64(lsb_ctx* c, Rank& r, const uint64_t* send, const size_t* sc,
                       const size_t* sd, uint64_t* recv, const size_t* rc, const size_t* rd,
                       size_t bound, hipStream_t stream) {
  const int P = c->P;
  hipStream_t st = stream ? stream : r.stream;
  const size_t lim = max_call_u64();
  const size_t k = c->mode == Mode::kRccl ? std::max<size_t>(1, (bound + lim - 1) / lim) : 1;
  if (k > 1) {
    std::vector<size_t> sc1(P), sd1(P), rc1(P), rd1(P);
    auto cut = [&](size_t n, size_t i) { return (size_t)((unsigned __int128)n * i / k); };
    for (size_t i = 0; i < k; ++i) {
      for (int q = 0; q < P; ++q) {
        sd1[q] = sd[q] + cut(sc[q], i);
        sc1[q] = cut(sc[q], i + 1) - cut(sc[q], i);
        rd1[q] = rd[q] + cut(rc[q], i);
        rc1[q] = cut(rc[q], i + 1) - cut(rc[q], i);
      }
      LSB_TRY(coll_alltoallv_u64(c, r, send, sc1.data(), sd1.data(), recv, rc1.data(), rd1.data(), 0, st));
    }
    return LSB_OK;
  }
  int64_t call_bytes = 0;
  for (int q = 0; q < P; ++q) call_bytes += (int64_t)sc[q] * 8;
  c->coll_calls += 1;
  c->coll_bytes += call_bytes;
  c->coll_max = std::max(c->coll_max, call_bytes);
  c->xs_calls += 1;
  for (int q = 0; q < P && q < LSB_MAX_RANKS; ++q) {
    c->xs_sent[q] += (int64_t)sc[q] * 8;
    c->xs_recv[q] += (int64_t)rc[q] * 8;
  }
  if (c->cur_pass >= 0 && c->cur_pass < LSB_MAX_PASSES) c->pass_xbytes[c->cur_pass] += call_bytes;
  if (c->mode == Mode::kRccl) {
    // LSB_RCCL_SYNC=1 (diagnostic): the device drains before and after every
    // call, so no work of any stream overlaps it.
    static const bool dsync = [] { const char* e = getenv("LSB_RCCL_SYNC"); return e && atoi(e); }();
    if (dsync) HIP_TRY(hipDeviceSynchronize());
    if (!c->p2p) {
      RCCL_TRY(ncclAllToAllv(send, sc, sd, recv, rc, rd, ncclUint64, c->comm, st));
    } else {  // the same exchange as explicit grouped point-to-point calls
      RCCL_TRY(ncclGroupStart());
      for (int q = 0; q < P; ++q) {
        if (sc[q] > 0) RCCL_TRY(ncclSend(send + sd[q], sc[q], ncclUint64, q, c->comm, st));
        if (rc[q] > 0) RCCL_TRY(ncclRecv(recv + rd[q], rc[q], ncclUint64, q, c->comm, st));
      }
      RCCL_TRY(ncclGroupEnd());
    }
    if (dsync) HIP_TRY(hipDeviceSynchronize());
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
  // LSB_REGION_FIRST=0: contexts start with the option off (A/B runs of
  // programs that do not set options, e.g. bench.py).
  if (const char* e = getenv("LSB_REGION_FIRST")) c->region = atoi(e) != 0;
  // LSB_EXCHANGE_CHUNKS=C: contexts start with LSB_OPT_EXCHANGE_CHUNKS = C
  // (A/B runs of programs that do not set options); LSB_XCHUNK_RESERVE: the
  // chunk passes' grid leaves that many workgroups to the wire (experiments).
  if (const char* e = getenv("LSB_EXCHANGE_CHUNKS")) {
    const int v = atoi(e);
    c->xchunks = v == 2 || v == 4 || v == 8 ? v : 0;
  }
  if (const char* e = getenv("LSB_XCHUNK_RESERVE")) c->xchunk_reserve = std::max(0, atoi(e));
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

}  // namespace lsb_rt
