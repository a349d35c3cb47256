// Context and rank state of the runtime behind include/lsb.h: errors, HIP-event
// timing of launches (filed per local pass, lsb_get_pass_stats), device
// buffers of a rank (DistributedArray::create, mpi/mpi_lsbsort.cpp:137-161),
// and the collectives of a one-rank-per-process context (RCCL, or the
// caller's host callbacks) that the pass driver and both exchange forms use.
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
    c->event_pool.push_back(p.start);
    c->event_pool.push_back(p.stop);
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

// ---- record buffers A and B, placement-calibrated ----------------------------
// How fast an LSD pass streams between two 16 GiB record buffers depends on
// where the driver placed them: per buffer the write side runs
// at 5.6-6.9 TB/s (tools/kbench/allocbw.hip, profiles/r04/allocbw_*.log), and
// k_onesweep's passes at 6.7-7.3 ms between pairs allocated in one process
// (profiles/r04/v5_pick.log).  So a rank's A and B are chosen among K
// candidate buffers by timing one k_onesweep pass between every ordered pair;
// the pair with the smallest sum of both directions (the passes ping-pong) is
// kept and the rest are freed.  K = LSB_PLACEMENT_CANDIDATES (environment,
// default 8; 2 or less: A and B as allocated), for buffers of at least 1 GiB
// and only as many as fit in 90 % of the free memory.  Eight candidates found
// a pair at 6.71-6.72 ms in each of four fresh processes, where four found one
// only in two of four (profiles/r04/v6_kcand_c{4,8}.log).  Cost at 2^30
// records: ~0.7 s at context creation, 128 GiB held while it runs.
namespace {

// How many candidate buffers of `bytes` to try (<= 2: no probing).
int placement_candidates(double bytes, int want) {
  int K = want;
  if (const char* e = getenv("LSB_PLACEMENT_CANDIDATES")) K = atoi(e);
  K = std::min(K, 8);
  size_t free_b = 0, total_b = 0;
  if (K > 2 && bytes >= (double)(1ull << 30) && hipMemGetInfo(&free_b, &total_b) == hipSuccess) {
    while (K > 2 && K * bytes > 0.9 * (double)free_b) --K;
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
int alloc_candidates(size_t per, int K, size_t need, std::vector<Elem*>& cand) {
  cand.clear();
  for (int k = 0; k < K; ++k) {
    Elem* p = nullptr;
    if (dev_alloc(&p, per) != LSB_OK) break;  // fewer candidates than hoped
    cand.push_back(p);
  }
  (void)hipGetLastError();
  if (cand.size() >= need) return LSB_OK;
  for (Elem* p : cand) (void)hipFree(p);
  cand.clear();
  return fail(LSB_ERR_NOMEM, "alloc_candidates", "record buffers");
}

}  // namespace

// Times one k_onesweep pass x -> y over the rank's here records on the byte
// at `shift`, with the rank's own look-back rows and histograms
// (onesweep_ensure); the histogram read before it is not timed.
// hist: kOnesweepSubs * 256 u32 of scratch (r.os_hist at creation; a buffer
// of its own once a sort may hold a histogram in r.os_hist).
double time_pass(Rank& r, Prober& pr, const Elem* x, Elem* y, int shift, uint32_t* hist) {
  if (pr.err != hipSuccess) return 0.0;
  pr.err = lsb::launch_subhist(x, r.here, shift, r.os_grid, hist, nullptr, r.stream);
  uint32_t epoch = r.os_epoch + 1;
  if (epoch >= (1u << 30)) epoch = 2;  // as onesweep_launch: keep the parity alternation
  if (pr.err == hipSuccess) pr.err = hipEventRecord(pr.e0, r.stream);
  lsb::OnesweepExtra probe;
  probe.probe = true;  // k_onesweep_probe: the same pass under its own name (profiles)
  if (pr.err == hipSuccess)
    pr.err = lsb::launch_onesweep(x, y, r.here, shift, -1, hist, nullptr, r.os_status, r.os_ctr, epoch,
                                  r.os_ctr + lsb::kOnesweepSubs, r.os_grid, r.stream, probe);
  if (pr.err == hipSuccess) r.os_epoch = epoch;
  if (pr.err == hipSuccess) pr.err = hipEventRecord(pr.e1, r.stream);
  if (pr.err == hipSuccess) pr.err = hipEventSynchronize(pr.e1);
  float t = 0.f;
  if (pr.err == hipSuccess) pr.err = hipEventElapsedTime(&t, pr.e0, pr.e1);
  return t;
}

// A and B.  The probe is the pass itself: each candidate gets uniform PCG
// keys, and one k_onesweep pass is timed between every ordered pair (on a
// byte the source is not ordered by).  A copy with the same write pattern
// (tools/kbench/allocbw.hip) ranked the buffers by their streaming write speed, but
// that did not predict the pass, whose tile loads sit on its look-back chain
// (profiles/r04/placement_*.log, pick.log).
int alloc_records(lsb_ctx* c, Rank& r) {
  const size_t per = (size_t)c->per;
  int K = placement_candidates((double)per * sizeof(Elem), 8);
  r.placement_k = 0;
  if (K <= 2 || r.here < (int64_t)lsb::kTile * lsb::kOnesweepSubs || r.here > lsb::kOnesweepMaxElems) {
    LSB_TRY(dev_alloc(&r.A, per));
    return dev_alloc(&r.B, per);
  }
  std::vector<Elem*> cand;
  LSB_TRY(alloc_candidates(per, K, 2, cand));
  K = (int)cand.size();
  auto give_up = [&](int rc) {
    for (Elem* p : cand) (void)hipFree(p);
    return rc;
  };
  int rc = onesweep_ensure(r);
  if (rc != LSB_OK) return give_up(rc);
  std::vector<double> ms((size_t)K * K, 0.0);
  std::vector<int> sorted_by(K, -8);
  Prober pr(r.stream, r.here);
  for (int k = 0; k < K && pr.err == hipSuccess; ++k)
    pr.err = lsb::launch_pcg_fill(cand[k], r.here, 0x5eed + (uint64_t)k, 0, lsb::KeyGen(), r.stream);
  (void)time_pass(r, pr, cand[0], cand[1], 0, r.os_hist);  // warm-up
  sorted_by[1] = 0;
  for (int x = 0; x < K; ++x)
    for (int y = 0; y < K; ++y) {
      if (x == y) continue;
      const int shift = (sorted_by[x] + 8) & 63;
      ms[(size_t)x * K + y] = time_pass(r, pr, cand[x], cand[y], shift, r.os_hist);
      sorted_by[y] = shift;
    }
  if (pr.err != hipSuccess) return give_up(fail(LSB_ERR_HIP, "alloc_records: placement probe", hipGetErrorString(pr.err)));
  // LSB_PLACEMENT_PICK=worst keeps the slowest pair instead (experiments:
  // tools/alloc_probe.py checks that the probe predicts the passes).
  const char* pick = getenv("LSB_PLACEMENT_PICK");
  const bool pick_worst = pick && strcmp(pick, "worst") == 0;
  int bx = 0, by = 1, wx = 0, wy = 1;
  double best = 1e300, worst = 0.0;
  for (int x = 0; x < K; ++x)
    for (int y = x + 1; y < K; ++y) {
      const double pair = 0.5 * (ms[(size_t)x * K + y] + ms[(size_t)y * K + x]);
      if (pair < best) {
        best = pair;
        bx = x;
        by = y;
      }
      if (pair > worst) {
        worst = pair;
        wx = x;
        wy = y;
      }
    }
  if (pick_worst) {
    bx = wx;
    by = wy;
  }
  r.placement_k = K;
  r.placement_ms[0] = pick_worst ? worst : best;
  r.placement_ms[1] = 0.5 * (ms[1] + ms[(size_t)K]);  // the first two buffers allocated
  r.placement_ms[2] = worst;
  r.A = cand[bx];
  r.B = cand[by];
  for (Elem* p : cand)
    if (p != r.A && p != r.B) (void)hipFree(p);
  return LSB_OK;
}

// The third record buffer R (receive buffer of the exchanges, the hybrid's
// third pass buffer), placed like A and B: among up to 3 candidates, the one
// whose timed passes to and from B (scratch whenever R is first needed:
// before a hybrid sort, at an exchange before its placement) take least time.
// A may hold records by then and is not touched; the probe counts into a
// histogram of its own, since a sort may hold one in r.os_hist.
int alloc_third(lsb_ctx* c, Rank& r) {
  const size_t per = (size_t)c->per;
  int K = r.placement_k > 0 ? placement_candidates((double)per * sizeof(Elem), 3) : 1;
  if (K <= 2) K = 1;
  if (K == 1 || !r.os_status) return dev_alloc(&r.R, per);
  std::vector<Elem*> cand;
  LSB_TRY(alloc_candidates(per, K, 1, cand));
  K = (int)cand.size();
  uint32_t* hist = nullptr;
  int rc = K > 1 ? dev_alloc(&hist, (size_t)lsb::kOnesweepSubs * lsb::kBuckets) : LSB_OK;
  Prober pr(r.stream, r.here);
  int bk = 0;
  double best = 1e300;
  for (int k = 0; k < K && K > 1 && rc == LSB_OK; ++k) {
    if (pr.err == hipSuccess)
      pr.err = lsb::launch_pcg_fill(cand[k], r.here, 0x5eed + 16 + (uint64_t)k, 0, lsb::KeyGen(), r.stream);
    const double t = time_pass(r, pr, cand[k], r.B, 0, hist) + time_pass(r, pr, r.B, cand[k], 8, hist);
    if (t < best) {
      best = t;
      bk = k;
    }
  }
  (void)hipFree(hist);
  if (rc == LSB_OK && pr.err != hipSuccess) rc = fail(LSB_ERR_HIP, "alloc_third: placement probe", hipGetErrorString(pr.err));
  if (rc != LSB_OK) {
    for (Elem* p : cand) (void)hipFree(p);
    return rc;
  }
  r.R = cand[bk];
  for (Elem* p : cand)
    if (p != r.R) (void)hipFree(p);
  return LSB_OK;
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
  c->xs_calls += 1;
  for (int q = 0; q < P && q < LSB_MAX_RANKS; ++q) {
    c->xs_sent[q] += (int64_t)sc[q] * 8;
    c->xs_recv[q] += (int64_t)rc[q] * 8;
  }
  if (c->cur_pass >= 0 && c->cur_pass < LSB_MAX_PASSES) c->pass_xbytes[c->cur_pass] += call_bytes;
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

}  // namespace lsb_rt
