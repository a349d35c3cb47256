// The whole-key exchange (radix_bits = 64, lsb_sort / lsb_pass(0) on an
// exchanging context): every rank sorts its block on the whole key, a
// splitter search finds the owner (and slice) boundaries, ONE sliced
// all-to-all moves each record to its owner, which merges the P runs.
#include "lsb_rt.h"

namespace lsb_rt {

// ---- whole-key exchange (radix_bits = 64) ----------------------------------
// globalShuffle with a 64-bit digit (mpi/mpi_lsbsort.cpp:481-577 with one
// pass): each rank sorts its block locally on the whole key, the ranks find
// where the global positions q * per fall (a splitter search over the sorted
// blocks, in place of the count transposes and scan of :327-479), every rank
// sends each owner one contiguous range (one all-to-all-v for the whole sort,
// :316-324), and each owner merges its P sorted runs in rank order (the
// placement of :568-575).  Same output as 64 / 8 or 64 / 16 exchanges: the
// stable order by key, ties by input position.


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
  if (!r.R) LSB_TRY(ensure_recv(c, r));
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
  // 32 algorithmic bytes per record per level (and per copy)
  c->xs_place_bytes += 32 * (hi - lo) * (L + (fin != F ? 1 : 0));
  c->xs_placed += hi - lo;
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
  ++c->xs_exchanges;
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
  // The longest range any source sends to any (owner, slice): every rank holds
  // every source's cuts, so all cut their RCCL calls alike (coll_alltoallv_u64).
  int64_t run_max = 0;
  {
    const std::vector<int64_t>& mc = c->ranks[0].mcut;
    for (size_t s = 0; s < (size_t)P; ++s)
      for (size_t k = 0; k + 1 < K1; ++k) run_max = std::max(run_max, mc[s * K1 + k + 1] - mc[s * K1 + k]);
  }
  for (int j = 0; j < g.S; ++j) {
    if (c->mode == Mode::kLoopback) {
      for (Rank& q : c->ranks) {
        HIP_TRY(hipSetDevice(q.dev));
        Timer t(c, &q, LSB_K_WIRE);
        slice_runs(c, q, g, j, sr, &lo, &hi);
        for (Rank& s : c->ranks) {
          if (s.rank == q.rank || sr[s.rank].len == 0) continue;
          LSB_TRY(copy_range(c, q, q.R + sr[s.rank].roff, s, s.A + q.mcut[s.rank * K1 + (size_t)q.rank * g.S + j],
                             sr[s.rank].len, q.stream));
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
        Timer t(c, &r, LSB_K_WIRE);
        LSB_TRY(coll_alltoallv_u64(c, r, reinterpret_cast<const uint64_t*>(r.A), sc.data(), sd.data(),
                                   reinterpret_cast<uint64_t*>(r.R), rc.data(), rdp.data(),
                                   (size_t)run_max * 2));
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
    LSB_TRY(join_place_timed(c, r));
    std::swap(r.A, final_b ? r.B : r.R);
  }
  return LSB_OK;
}

// lsb_sort / lsb_pass(0) with a 64-bit exchange digit on an exchanging context.
int merge_sort(lsb_ctx* c) {
  LSB_TRY(sort_local_ranks(c));
  c->last_exchanges = 1;
  return exchange_merge(c);
}

}  // namespace lsb_rt
