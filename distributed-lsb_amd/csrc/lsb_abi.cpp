// The C ABI (include/lsb.h): entry points over the runtime (lsb_rt.h) and the
// pure host planners.
#include "lsb_rt.h"

using namespace lsb_rt;


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
    case LSB_ERR_HIP: return last_error().empty() ? "HIP error" : last_error().c_str();
    case LSB_ERR_RCCL: return last_error().empty() ? "RCCL error" : last_error().c_str();
    case LSB_ERR_NOMEM: return "out of memory";
    case LSB_ERR_VERIFY: return "verification failed";
    case LSB_ERR_UNSUPPORTED: return "unsupported";
    case LSB_ERR_STATE: return last_error().empty() ? "invalid state" : last_error().c_str();
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
    const int d = dev_ids ? dev_ids[r] : 0;
    for (int q = 0; q < r; ++q)
      if (d == (dev_ids ? dev_ids[q] : 0)) c->shared_device = true;
    if (std::find(c->access_devs.begin(), c->access_devs.end(), d) == c->access_devs.end())
      c->access_devs.push_back(d);
  }
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

int lsb_rank_footprint(int64_t n_total, int num_ranks, int radix_bits, int with_recv, int64_t* bytes,
                       int64_t* probe_bytes) {
  if (!bytes || n_total < 0 || num_ranks < 1 || num_ranks > 64)
    return fail(LSB_ERR_INVALID, "lsb_rank_footprint", "n, P or null");
  if (radix_bits != 8 && radix_bits != 16 && radix_bits != 64)
    return fail(LSB_ERR_UNSUPPORTED, "lsb_rank_footprint", "radix_bits must be 8, 16 or 64");
  const int64_t P = num_ranks, per = div_ceil(n_total, num_ranks);
  const int64_t nb = radix_bits == 64 ? lsb::kBuckets : (int64_t)1 << radix_bits;
  const int64_t cap = record_capacity(per, (int)P);                // A and B (regional slots)
  const int64_t tiles = lsb::onesweep_tiles(per);
  const lsb::Chunking ch = lsb::make_chunking(per, 2 * 256);
  int64_t b = (with_recv ? 3 : 2) * (int64_t)rec_bytes((size_t)cap);  // A, B (and R) hold the same
  b += tiles * lsb::kBuckets * 4;                                   // os_status
  if (region_cap_for(per, (int)P) > 0)  // os_status2 and rg_buf of the regional first pass
    b += lsb::onesweep_tiles(region_cap_for(per, (int)P) * lsb::kRegions) * lsb::kBuckets * 4 +
         (lsb::kRegions + 512) * 4;
  if (P > 1 || with_recv) b += tiles * (int64_t)sizeof(lsb::TileDesc) + 2 * P * nb * 8;  // gdesc, gstart
  b += (int64_t)lsb::kBuckets * std::max(1, ch.num_chunks) * 12;    // chunk_hist, chunk_off
  b += (int64_t)lsb::kBuckets * 8 + (radix_bits == 16 ? 2 * 65536 * 8 : 0);  // totals, totals16, first16
  b += (std::max(P * nb, 4 * P) + (P * nb + P) + P * nb + nb + 2 * P) * 8;   // gather, place, plan_*
  b += (2 * lsb::kOnesweepSubs * lsb::kBuckets + 2 * lsb::kOnesweepSubs) * 4 +
       (int64_t)lsb::kOnesweepSubs * lsb::kBuckets * 8;             // os_hist, os_ctr, seg_base
  if (radix_bits == 64 && P > 1)
    b += (lsb::merge_tiles(per) + 2 * lsb::kMergeMaxPairs + 1) * 8 +
         (int64_t)(P * 8) * lsb::kSplitCands * 8 * (P + 1);         // merge_path, split_* (8 slices)
  *bytes = b;
  if (probe_bytes) {
    const int64_t cap_rec = rec_bytes((size_t)cap);  // a candidate holds as many records as A
    double share = 0.0;
    const int K = placement_request((double)cap_rec, &share);
    // One candidate beyond A and B is live at a time (alloc_records).
    *probe_bytes = K > 2 && cap_rec >= ((int64_t)1 << 30) ? cap_rec : 0;
  }
  return LSB_OK;
}

int lsb_device_memory(int dev, int64_t* free_bytes, int64_t* total_bytes) {
  if (!free_bytes || !total_bytes) return fail(LSB_ERR_INVALID, "lsb_device_memory", "null");
  HIP_TRY(hipSetDevice(dev));
  size_t f = 0, t = 0;
  HIP_TRY(hipMemGetInfo(&f, &t));
  *free_bytes = (int64_t)f;
  *total_bytes = (int64_t)t;
  return LSB_OK;
}

int lsb_device_count(int* count) {
  if (!count) return fail(LSB_ERR_INVALID, "lsb_device_count", "null");
  *count = 0;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e == hipErrorNoDevice) {
    (void)hipGetLastError();
    return LSB_OK;
  }
  HIP_TRY(e);
  *count = n;
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
  // Every rank's streams first: a loopback rank's stream reads the other
  // ranks' buffers (exchange copies), and VMM record buffers are unmapped
  // without the implicit device synchronisation hipFree has.  (Debug builds
  // check it, and LSB_TEARDOWN_LEGACY there restores the old order, one rank's
  // own stream at a time, to show the check firing: free_rank.)
#ifdef LSB_DEBUG
  const bool legacy = getenv("LSB_TEARDOWN_LEGACY") != nullptr;
#else
  const bool legacy = false;
#endif
  for (Rank& r : c->ranks) {
    if (legacy) break;
    (void)hipSetDevice(r.dev);
    if (r.stream) (void)hipStreamSynchronize(r.stream);
    if (r.pstream) (void)hipStreamSynchronize(r.pstream);
    if (r.xstream) (void)hipStreamSynchronize(r.xstream);
  }
  for (Rank& r : c->ranks) free_rank(r, c);
  for (auto& e : c->event_pool) (void)hipEventDestroy(e.second);
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
    case LSB_OPT_REGION_FIRST:
      c->region = value != 0;
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
    case LSB_OPT_FAIL_ONESWEEP:
      if (value < 0 || value > (1 << 30)) return fail(LSB_ERR_INVALID, "lsb_set_option", "fail count");
      c->fail_onesweep = (int)value;
      return LSB_OK;
    case LSB_OPT_HYBRID:
      if (value < 0 || value > 2) return fail(LSB_ERR_INVALID, "lsb_set_option", "hybrid must be 0, 1 or 2");
      c->hybrid = (int)value;
      return LSB_OK;
    case LSB_OPT_ONESWEEP_SPLIT:
      if (value < 0 || value > 2) return fail(LSB_ERR_INVALID, "lsb_set_option", "split must be 0..2");
      c->os_split = (int)value;
      return LSB_OK;
    case LSB_OPT_EXCHANGE_CHUNKS:
      if (value != 0 && value != 2 && value != 4 && value != 8)
        return fail(LSB_ERR_INVALID, "lsb_set_option", "exchange chunks must be 0, 2, 4 or 8");
      c->xchunks = (int)value;
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

namespace {

// A sort that failed part-way may leave work queued on a rank's placement
// or wire stream (an exchange's placements, the chunked exchange's
// transfers) that reads or writes the record buffers; the next call on the
// context queues on the rank's stream only.  Wait for all of it before the
// error goes back, so no later sort races with it.
void quiesce(lsb_ctx* c) {
  for (Rank& r : c->ranks) {
    (void)hipSetDevice(r.dev);
    for (hipStream_t s : {r.stream, r.pstream, r.xstream})
      if (s) (void)hipStreamSynchronize(s);
  }
}

}  // namespace

int lsb_pass(lsb_ctx_t* c, int digit) {
  LSB_TRY(check_ctx(c));
  if (digit < 0 || digit >= 64 / c->bits) return fail(LSB_ERR_INVALID, "lsb_pass", "digit");
  // Filed under the digit's own local passes (a 64-bit digit: the whole sort).
  c->pass_cursor = c->bits == 64 ? 0 : digit * (c->bits / lsb::kDigitBits);
  const int rc = do_pass(c, digit);
  if (rc != LSB_OK) quiesce(c);
  return rc;
}

namespace {

int sort_body(lsb_ctx* c) {
  std::vector<Timer> sort_timers;
  sort_timers.reserve(c->ranks.size());
  for (Rank& r : c->ranks) sort_timers.emplace_back(c, &r, LSB_K_SORT);
  const int passes = 64 / c->bits;
  c->last_local_passes = c->last_exchanges = 0;
  c->last_varying = ~0ull;
  c->last_first = LSB_FIRST_COUNT;
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

}  // namespace

int lsb_sort(lsb_ctx_t* c) {
  LSB_TRY(check_ctx(c));
  const int rc = sort_body(c);
  if (rc != LSB_OK) quiesce(c);
  return rc;
}

int lsb_get_last_sort(lsb_ctx_t* c, int* local_passes, int* exchanges, uint64_t* varying_bits) {
  LSB_TRY(check_ctx(c));
  if (local_passes) *local_passes = c->last_local_passes;
  if (exchanges) *exchanges = c->last_exchanges;
  if (varying_bits) *varying_bits = c->last_varying;
  return LSB_OK;
}

int lsb_get_first_pass(lsb_ctx_t* c, int* form) {
  LSB_TRY(check_ctx(c));
  if (!form) return fail(LSB_ERR_INVALID, "lsb_get_first_pass", "null");
  *form = c->last_first;
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
    c->pass_xbytes[p] = 0;
  }
  c->xs_exchanges = c->xs_calls = 0;
  for (int q = 0; q < LSB_MAX_RANKS; ++q) c->xs_sent[q] = c->xs_recv[q] = 0;
  c->xs_place_bytes = c->xs_placed = c->xs_counted = 0;
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
  // The exchange: counts all-gather, plan and the all-to-all (wire) together.
  if (ms_exchange) *ms_exchange = c->pass_ms[pass][LSB_K_EXCHANGE] + c->pass_ms[pass][LSB_K_WIRE];
  if (ms_place) *ms_place = c->pass_ms[pass][LSB_K_PLACE];
  return LSB_OK;
}

int lsb_get_pass_exchange(lsb_ctx_t* c, int pass, int64_t* bytes, double* wire_ms, double* place_tail_ms) {
  LSB_TRY(check_ctx(c));
  if (pass < 0 || pass >= LSB_MAX_PASSES) return fail(LSB_ERR_INVALID, "lsb_get_pass_exchange", "pass");
  LSB_TRY(resolve_timing(c));
  if (bytes) *bytes = c->pass_xbytes[pass];
  if (wire_ms) *wire_ms = c->pass_ms[pass][LSB_K_WIRE];
  if (place_tail_ms) *place_tail_ms = c->pass_ms[pass][LSB_K_PLACE_TAIL];
  return LSB_OK;
}

int lsb_get_exchange_stats(lsb_ctx_t* c, lsb_exchange_stats_t* out) {
  LSB_TRY(check_ctx(c));
  if (!out) return fail(LSB_ERR_INVALID, "lsb_get_exchange_stats", "null out");
  LSB_TRY(resolve_timing(c));
  memset(out, 0, sizeof *out);
  out->exchanges = c->xs_exchanges;
  out->calls = c->xs_calls;
  for (int q = 0; q < LSB_MAX_RANKS; ++q) {
    out->sent_bytes[q] = c->xs_sent[q];
    out->recv_bytes[q] = c->xs_recv[q];
  }
  out->wire_ms = c->total_ms[LSB_K_WIRE];
  out->plan_ms = c->total_ms[LSB_K_EXCHANGE];
  out->place_ms = c->total_ms[LSB_K_PLACE];
  out->place_tail_ms = c->total_ms[LSB_K_PLACE_TAIL];
  out->place_bytes = c->xs_place_bytes;
  out->placed_records = c->xs_placed;
  out->counted_records = c->xs_counted;
  return LSB_OK;
}

int lsb_get_placement(lsb_ctx_t* c, int rank, int* candidates, double* chosen_ms, double* first_pair_ms,
                      double* worst_ms) {
  LSB_TRY(check_ctx(c));
  Rank* r = local_rank(c, rank);
  if (!r) return fail(LSB_ERR_INVALID, "lsb_get_placement", "rank");
  if (candidates) *candidates = r->placement_k;
  if (chosen_ms) *chosen_ms = r->placement_ms[0];
  if (first_pair_ms) *first_pair_ms = r->placement_ms[1];
  if (worst_ms) *worst_ms = r->placement_ms[2];
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
const char* lsb_build_info(void) {
  // The RCCL the process loaded (ncclGetVersion touches no device): its large
  // calls are cut at 1 GiB per peer (coll_alltoallv_u64).
  static const std::string info = [] {
    int v = 0;
    (void)ncclGetVersion(&v);
    return std::string("sha256=" LSB_SOURCE_DIGEST " host=" LSB_BUILD_HOST " rccl=") + std::to_string(v);
  }();
  return info.c_str();
}

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

