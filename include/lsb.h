/*
 * lsb.h — C ABI of the MI355X-native distributed LSD radix sort.
 *
 * The reference (ronawho/distributed-lsb) has no library or FFI: every
 * variant is one program whose in-process seams are
 *   mySort(A, B)              mpi/mpi_lsbsort.cpp:580-585, shmem/shmem_lsbsort.cpp:460-472
 *   globalShuffle(A, B, d)    mpi/mpi_lsbsort.cpp:481-577, shmem/shmem_lsbsort.cpp:388-457
 *   DistributedArray::create  mpi/mpi_lsbsort.cpp:137-161
 *   checkSorted()             shmem/shmem_lsbsort.cpp:180-219
 *   PCG input init            mpi/mpi_lsbsort.cpp:643-666
 *   verify (gather + stable_sort + ==)  mpi/mpi_lsbsort.cpp:673-679,710-738
 * Each entry point below names the seam it replaces.  Plain C types only;
 * no C++ exception crosses this boundary; every function returning int
 * returns LSB_OK (0) or an LSB_ERR_* code (lsb_strerror() describes it).
 *
 * A context is one "world" of P ranks (P = num_ranks) over the block
 * partition per = ceil(n/P) (mpi/mpi_lsbsort.cpp:144-149):
 *   - lsb_create():      one process drives all P ranks (logical ranks, each
 *                        with its own buffers; several may share one GPU).
 *                        The per-pass exchange is a device-to-device copy
 *                        with exactly the all-to-all-v semantics of RCCL.
 *   - lsb_create_rank(): one process per GPU (torchrun / hip_lsbsort --gpus);
 *                        this process is rank `rank`; the exchange is RCCL
 *                        (AllGather of bucket counts + AllToAllv)
 *                        over xGMI.  Collective calls must be made by all
 *                        ranks in the same order, as in the MPI reference.
 * The context owns every device buffer (A, B, send/recv, histograms, RCCL
 * communicator), as DistributedArray owns localPart_.  A context is driven
 * by one host thread and is not re-entrant.
 */
#ifndef LSB_H
#define LSB_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LSB_OK                 0
#define LSB_ERR_INVALID        1  /* bad argument (rank, range, digit, radix) */
#define LSB_ERR_HIP            2  /* a HIP runtime call failed */
#define LSB_ERR_RCCL           3  /* an RCCL call failed */
#define LSB_ERR_NOMEM          4  /* device or host allocation failed */
#define LSB_ERR_VERIFY         5  /* lsb_verify found a mismatch */
#define LSB_ERR_UNSUPPORTED    6  /* valid request this build does not do */
#define LSB_ERR_STATE          7  /* call not valid in this context state */

#define LSB_UNIQUE_ID_BYTES  128  /* == NCCL_UNIQUE_ID_BYTES */

/* == struct SortElement (mpi/mpi_lsbsort.cpp:29-32): 16 B, little-endian,
 * key then val, no padding.  Order of the sort: key only, stable. */
typedef struct lsb_elem {
  uint64_t key;
  uint64_t val;
} lsb_elem_t;

typedef struct lsb_ctx lsb_ctx_t;

/* Kernel / phase ids for lsb_get_kernel_stats(). */
#define LSB_K_UPSWEEP   0  /* per-chunk digit histogram (count)           */
#define LSB_K_SCAN      1  /* chunk x bucket exclusive scan               */
#define LSB_K_SCATTER   2  /* stable LDS-staged scatter (shuffle)         */
#define LSB_K_EXCHANGE  3  /* bucket-count allgather + element all-to-all */
#define LSB_K_PLACE     4  /* received runs -> final local slots          */
#define LSB_K_SORT      5  /* whole lsb_sort()                            */
#define LSB_K_SEGSORT   6  /* segmented local sort (LSB_OPT_HYBRID)       */
#define LSB_K_WIRE      7  /* the element all-to-all calls alone (RCCL,
                              host ops, or loopback device copies)        */
#define LSB_K_PLACE_TAIL 8 /* placement still running after the last slice
                              arrived (rank's stream waiting on it)       */
#define LSB_K_COUNT     9
#define LSB_MAX_RANKS  64  /* ranks of a context */

/* Options for lsb_set_option(). */
#define LSB_OPT_TIMING          0  /* 1: record HIP events around every kernel */
#define LSB_OPT_FORCE_EXCHANGE  1  /* 1: run the exchange path even when P == 1 */
#define LSB_OPT_SKIP_CONSTANT_DIGITS 2  /* 1 (default): lsb_sort skips every digit after
                                           the first on which all keys agree */
#define LSB_OPT_EXCHANGE_SLICES 3  /* 1..64 (default 5; 8 for radix_bits = 64): the all-to-all of a pass is cut into
                                      this many groups; each slice is placed while the next
                                      is in flight.  Per-digit exchanges cut each peer segment
                                      in halving parts (1/2, 1/4, ..., the last two equal), so
                                      the placement left after the wire is 1/2^(slices-1) of it;
                                      the whole-key exchange in equal parts */
#define LSB_OPT_EXCHANGE_P2P    4  /* RCCL contexts: 0 (default) ncclAllToAllv per slice,
                                      1 the same as grouped ncclSend/ncclRecv */
#define LSB_OPT_EXCHANGE_PEER   5  /* 1: exchange by direct stores into the owners' buffers
                                      (shmem_putmem / MPI_Put form; IPC-mapped across
                                      processes); no receive buffer, no placement pass.
                                      Opt-in: set on every rank before the first sort. */
#define LSB_OPT_ONESWEEP        6  /* 1 (default): lsb_sort reads each record once per
                                      local pass (P == 1, the per-digit exchange forms and
                                      the whole-key form's local sort): offsets by decoupled
                                      look-back, histograms carried from pass to pass (or
                                      counted by the exchange's placement); 0: reduce-then-
                                      scan (count, scan, scatter), as lsb_pass always is */
#define LSB_OPT_EXCHANGE_SELF   7  /* one-rank-per-process contexts: 1 sends the rank's own
                                      segment through the element collective as well
                                      (ncclAllToAllv / ncclSend+ncclRecv to itself, or the
                                      caller's alltoallv) and places it from the receive
                                      buffer like every other source; 0 (default) places it
                                      straight out of A.  Same output; lets a world of one
                                      carry the whole payload through RCCL (tests). */
#define LSB_OPT_ONESWEEP_SPLIT  8  /* single-read passes' LDS stage: 0 (default) chosen per
                                      sort from the first digit's histogram (one bucket over
                                      1/32 of a rank's records: the tile is staged in two
                                      halves, 3 workgroups per CU); 1 never split; 2 always
                                      split.  Same output. */
#define LSB_OPT_HYBRID          9  /* local sorts without an exchange between digits (P == 1,
                                      and each rank's block in the whole-key form): 0 (default)
                                      the LSD passes; 1 the hybrid: stable 8-bit passes on the k
                                      most significant varying bytes only (k = 4 at 2^30 records),
                                      the last of which also orders every segment (run of records
                                      equal on those bytes, ~0.25 records on average) by the whole
                                      key inside its tile, and k_segfix merges the segments split
                                      between two tiles; 2 the same passes, then a separate
                                      segmented sort (k_segsort) orders the segments.  Same output
                                      (the stable sort by key) from k passes over HBM instead of up
                                      to 8.  Skewed keys (one bucket of the first byte over 1/32 of
                                      the records) take the LSD passes; runs too long for k_segfix
                                      take k_segsort, and segments longer than 64 records
                                      (kSegMax) make the sort redo the kept input by the LSD
                                      passes.  Needs a third record buffer. */
#define LSB_OPT_EXCHANGE_GATHER 10 /* per-digit exchange forms with single-read local passes:
                                      1 (default) every exchange but the last only counts
                                      the next byte as the records arrive, and the next local
                                      pass reads its tiles from where they arrived (the
                                      receive buffer, the rank's own segment in A) through
                                      the plan's piece table: no placement pass (k_place's
                                      16 B of writes per record) before it; 0 places every
                                      exchange.  Same output. */
#define LSB_OPT_FAIL_ONESWEEP   11 /* tests (fault injection): n >= 1 makes the n-th k_onesweep
                                      launch from now (the chunked exchange's chunk passes
                                      included) fail with LSB_ERR_HIP before it is queued, as a
                                      failed launch would; 0 (default) off.  The context stays
                                      usable: its buffers keep their roles and the next sort
                                      starts from the records in A (the input, or after an
                                      exchange's local pass a permutation of it).  lsb_sort
                                      returns any error only once every rank's streams are
                                      idle. */
#define LSB_OPT_REGION_FIRST    12 /* P == 1 sorts of >= 2^27 records by the LSD passes:
                                      1 (default) the first pass takes no histogram read: it
                                      writes each (digit, sub-array) class of records into a
                                      slot range of its own, sized with slack over a uniform
                                      class (A and B hold 1.6 % more slots at 2^30), and the
                                      second pass reads that layout back to a dense one.  A
                                      2^20-record sample sends skewed or structured low bytes
                                      to the usual start (a histogram read), and a range that
                                      overflows all the same makes the sort start over from
                                      its input.  0: every sort starts with the histogram
                                      read.  Same output. */
#define LSB_OPT_EXCHANGE_CHUNKS 13 /* radix_bits = 16 exchanges (P > 1 or forced; RCCL or loopback):
                                      C = 2, 4 or 8 sends each digit's records in C chunks of
                                      its low byte while the high-byte pass runs chunk by chunk
                                      (chunk k's records on the wire during chunk k + 1's pass;
                                      mpi/mpi_lsbsort.cpp:481-577 runs localShuffle, then the
                                      whole exchange).  One read after the low-byte pass counts
                                      the digit first.  0 (default; the
                                      environment's LSB_EXCHANGE_CHUNKS sets a context's start
                                      value) sends after the whole pass.  Same output. */

/* ---- geometry: DistributedArray::create (mpi/mpi_lsbsort.cpp:144-149) ---- */
int64_t lsb_per_rank(int64_t n_total, int num_ranks);            /* ceil(n/P) */
int64_t lsb_here(int64_t n_total, int num_ranks, int rank);      /* clamp(n - r*per, 0, per) */

/* ---- lifecycle ---------------------------------------------------------- */
/* One process, `num_ranks` logical ranks; rank r lives on device dev_ids[r]
 * (dev_ids == NULL: every rank on device 0).  Up to 64 ranks.
 * radix_bits is the width of the digit the ranks exchange on: 8 (256
 * buckets, 8 passes) or 16 (65536 buckets, 4 passes: the reference's own
 * RADIX, mpi/mpi_lsbsort.cpp:21).  On device every digit is sorted by
 * stable 8-bit local passes (a 16-bit digit = low byte, then high byte), so
 * the output is the same for both; 16 halves the all-to-alls when P > 1.
 * radix_bits = 64 makes the whole key one digit: each rank sorts its block
 * (all 8 local passes), then ONE all-to-all moves every record to its owner,
 * which merges the P sorted runs in rank order (lsb_plan_merge).  Same
 * output again; one exchange per sort instead of 64 / radix_bits.
 * Device memory per rank: lsb_rank_footprint (A and B here; R, the receive
 * buffer, at the first exchange or hybrid sort; record buffers of >= 1 GiB
 * are whole 1 GiB VMM pieces).  While its placement probe runs
 * (lsb_get_placement) a rank alone on its device holds K - 2 more record
 * buffers for a moment: by default K = 4 for buffers of >= 4 GiB, as many as
 * fit in half the free memory at that moment (2^30 records: 34 GiB more for
 * ~0.2 s); LSB_PLACEMENT_CANDIDATES = K sets K (0: no probe; at most 8,
 * within 90 % of the free memory). */
int  lsb_create(lsb_ctx_t** ctx, int64_t n_total, int num_ranks,
                const int* dev_ids, int radix_bits);
/* HIP devices this process can see (hipGetDeviceCount; 0 when there is
 * none).  For a binding that maps one rank per GPU, e.g. the mySort stub of
 * INTEGRATION.md (rank r on device r % count). */
int  lsb_device_count(int* count);
/* RCCL bootstrap: rank 0 calls this and ships the bytes to the other ranks
 * (bench.py uses torch.distributed; hip_lsbsort uses a pipe). */
int  lsb_get_unique_id(unsigned char id[LSB_UNIQUE_ID_BYTES]);
/* One process per GPU: this process is `rank` of `num_ranks`, on `dev_id`. */
int  lsb_create_rank(lsb_ctx_t** ctx, int64_t n_total, int num_ranks, int rank,
                     int dev_id, int radix_bits,
                     const unsigned char id[LSB_UNIQUE_ID_BYTES]);
/* One process per rank with caller-supplied collectives instead of RCCL (any
 * transport: MPI, gloo, sockets).  The runtime runs exactly the per-rank code
 * of lsb_create_rank; around each collective it synchronizes its stream and
 * stages the data through host memory.  All pointers are host pointers, all
 * sizes are bytes; every rank makes the same calls in the same order (as
 * MPI requires); a callback returns 0 on success.  `user` is passed back. */
typedef struct lsb_comm_ops {
  void* user;
  /* recv[r * bytes .. (r+1) * bytes) = send of rank r */
  int (*allgather)(void* user, const void* send, void* recv, size_t bytes);
  /* MPI_Alltoallv on bytes */
  int (*alltoallv)(void* user, const void* send, const size_t* send_bytes,
                   const size_t* send_displs, void* recv, const size_t* recv_bytes,
                   const size_t* recv_displs);
  /* *value = min over ranks */
  int (*allreduce_min_i64)(void* user, int64_t* value);
  int (*barrier)(void* user);
} lsb_comm_ops_t;
int  lsb_create_rank_ops(lsb_ctx_t** ctx, int64_t n_total, int num_ranks, int rank,
                         int dev_id, int radix_bits, const lsb_comm_ops_t* ops);
void lsb_destroy(lsb_ctx_t* ctx);
int  lsb_set_option(lsb_ctx_t* ctx, int option, int64_t value);
/* Ranks owned by this context: [*first_rank, *first_rank + *num_local). */
int  lsb_local_ranks(const lsb_ctx_t* ctx, int* first_rank, int* num_local);

/* ---- data --------------------------------------------------------------- */
/* PCG input init (mpi/mpi_lsbsort.cpp:650-656), on device: for every local
 * rank r and every one of its `per` slots i: key = i-th output of pcg64(r),
 * val = r*per + i.  Untimed in the reference; untimed here. */
int  lsb_generate(lsb_ctx_t* ctx);
/* Same stream, other key distributions (build-defined):
 *   LSB_DIST_UNIFORM         == lsb_generate
 *   LSB_DIST_ZIPF, param = s key = mix64(k), k = floor of a power law with
 *                            exponent s on [1, 2^30], drawn by inverse CDF
 *                            from the same pcg64(r) draw (heavy duplicates).
 * lsb_verify() recomputes keys with the distribution last generated. */
#define LSB_DIST_UNIFORM 0
#define LSB_DIST_ZIPF    1
int  lsb_generate_ex(lsb_ctx_t* ctx, int dist, double param);
/* Host <-> A of a local rank, slots [off, off+cnt) of that rank's per slots. */
int  lsb_copy_in(lsb_ctx_t* ctx, int rank, int64_t off, int64_t cnt, const lsb_elem_t* host);
int  lsb_copy_out(lsb_ctx_t* ctx, int rank, int64_t off, int64_t cnt, lsb_elem_t* host);

/* ---- the hot path ------------------------------------------------------- */
/* == mySort(A, B): all 64/radix_bits passes; result in A.  Asynchronous
 * with respect to the host except for the per-pass count exchange when
 * P > 1 and one 16-byte key-span read after the first pass; call
 * lsb_sync() to wait.
 * The first pass's count kernel also reduces the OR of all keys and of their
 * complements (all-gathered when P > 1).  A later digit on which every key
 * agrees is skipped: its stable pass and its exchange are the identity, so
 * the output is unchanged (keys < 2^32 take 4 of 8 passes).  Uniform 64-bit
 * keys run every pass.  LSB_OPT_SKIP_CONSTANT_DIGITS = 0 turns this off. */
int  lsb_sort(lsb_ctx_t* ctx);
/* What the last lsb_sort ran: 8-bit local passes, exchanges (0 when P == 1
 * and not forced) and the key bits that vary (~0 when skipping is off). */
int  lsb_get_last_sort(lsb_ctx_t* ctx, int* local_passes, int* exchanges,
                       uint64_t* varying_bits);
/* How the last lsb_sort began (LSB_OPT_REGION_FIRST): LSB_FIRST_COUNT a
 * histogram read (k_subhist / k_upsweep) before the first pass, or none ran;
 * LSB_FIRST_REGIONAL the regional first pass; LSB_FIRST_REGIONAL_REDONE the
 * regional pass overflowed a region, and the sort started over from its
 * input with the histogram read.  With LSB_FIRST_REGIONAL the varying bits
 * of lsb_get_last_sort are those of a 2^20-record sample (every byte varies
 * there, so every pass runs). */
#define LSB_FIRST_COUNT           0
#define LSB_FIRST_REGIONAL        1
#define LSB_FIRST_REGIONAL_REDONE 2
int  lsb_get_first_pass(lsb_ctx_t* ctx, int* form);
/* == globalShuffle(A, B, digit): one pass, result in A. */
int  lsb_pass(lsb_ctx_t* ctx, int digit);
int  lsb_sync(lsb_ctx_t* ctx);
/* lsb_sync, then (RCCL contexts) a device all-reduce across the ranks:
 * the MPI_Barrier around the timed region (mpi/mpi_lsbsort.cpp:688,693). */
int  lsb_barrier(lsb_ctx_t* ctx);

/* ---- checks ------------------------------------------------------------- */
/* Bit-exact check equivalent to the MPI verify (stable_sort + ==), in O(n)
 * on device, valid for PCG input from lsb_generate(): for every global i,
 * out[i].val < n, out[i].key == pcg64(val / per)[val % per] and
 * (key, val)[i] < (key, val)[i+1] strictly, across rank boundaries too.
 * Returns LSB_OK when all hold, LSB_ERR_VERIFY otherwise; *first_bad gets
 * the smallest failing global index (or -1). */
int  lsb_verify(lsb_ctx_t* ctx, int64_t* first_bad);
/* == checkSorted (shmem/shmem_lsbsort.cpp:180-219): key order inside every
 * rank and across rank boundaries.  *sorted = 1 / 0. */
int  lsb_check_sorted(lsb_ctx_t* ctx, int* sorted);

/* ---- measurement -------------------------------------------------------- */
/* With LSB_OPT_TIMING on: launches recorded and their summed device time
 * (HIP events on the stream each kernel runs on) since the last reset. */
int  lsb_get_kernel_stats(lsb_ctx_t* ctx, int kernel_id, int64_t* launches, double* total_ms);
int  lsb_reset_kernel_stats(lsb_ctx_t* ctx);
/* Elements one launch of the scatter kernel processed, summed like the stats. */
int  lsb_get_scatter_elems(lsb_ctx_t* ctx, int64_t* elems);
/* The same stats per local pass (the reference times only the
 * whole sort, mpi/mpi_lsbsort.cpp:688-699).  Pass p is the p-th 8-bit local
 * pass a sort ran (0-based; constant digits are skipped, so p counts passes
 * that ran, not digits; lsb_pass files a digit's passes under its own index).
 * A sort's first count read is filed under its first pass, and an exchange
 * (all-gather, plan, all-to-all, placement or merge) under the local pass
 * before it.  Summed over the launches since the last reset, every local
 * rank included: *shift = the pass's key shift (-1: no launch), *launches /
 * *elems = scatter launches and the records they processed, and the device
 * milliseconds of its count kernels (k_subhist / k_upsweep + k_scan), its
 * scatter (k_onesweep or k_scatter), its exchange and its placement. */
#define LSB_MAX_PASSES 16
int  lsb_get_pass_stats(lsb_ctx_t* ctx, int pass, int* shift, int64_t* launches, int64_t* elems,
                        double* ms_count, double* ms_scatter, double* ms_exchange, double* ms_place);
/* Element payload this context handed to its all-to-all collective
 * (ncclAllToAllv, grouped ncclSend/ncclRecv or the caller's alltoallv) since
 * the context was created: calls, bytes sent (self segment included when
 * LSB_OPT_EXCHANGE_SELF is on) and the largest one call sent.  Loopback
 * contexts (device copies) report 0. */
int  lsb_get_exchange_bytes(lsb_ctx_t* ctx, int64_t* calls, int64_t* bytes, int64_t* max_call_bytes);
/* The exchange steps since the last lsb_reset_kernel_stats, this context's
 * local ranks summed: the xGMI side of a pass that SURVEY §8(d) asks to
 * report beside the local passes (the reference's all-to-all and placement,
 * mpi/mpi_lsbsort.cpp:562-575).  Bytes are the element collective's payload
 * (ncclAllToAllv / grouped send-recv / the caller's alltoallv; the self
 * segment only with LSB_OPT_EXCHANGE_SELF; loopback device copies count 0),
 * per peer.  Times need LSB_OPT_TIMING (HIP events):
 *   wire_ms       the all-to-all calls on the rank's stream (LSB_K_WIRE);
 *   plan_ms       counts all-gather + device plan + tile descriptors, or the
 *                 whole key's splitter search (LSB_K_EXCHANGE);
 *   place_ms      the placement stream: k_place, or the merge (LSB_K_PLACE);
 *   place_tail_ms placement still running once the last slice had arrived
 *                 (LSB_K_PLACE_TAIL): the part not overlapped with the wire.
 * place_bytes: algorithmic bytes of the placement kernels: 32 per placed
 * record (16 read + 16 written), 16 per record a count-only k_place reads,
 * 32 per record per merge level. */
typedef struct lsb_exchange_stats {
  int64_t exchanges;                   /* exchange steps (digits, or 1 per whole-key sort) */
  int64_t calls;                       /* all-to-all calls (slices) */
  int64_t sent_bytes[LSB_MAX_RANKS];   /* payload to each destination rank */
  int64_t recv_bytes[LSB_MAX_RANKS];   /* payload from each source rank */
  double wire_ms, plan_ms, place_ms, place_tail_ms;
  int64_t place_bytes;
  int64_t placed_records;              /* records written by the placement */
  int64_t counted_records;             /* records only counted (gathered passes follow) */
} lsb_exchange_stats_t;
int  lsb_get_exchange_stats(lsb_ctx_t* ctx, lsb_exchange_stats_t* out);
/* Per local pass (as lsb_get_pass_stats files an exchange under the local
 * pass before it): payload bytes handed to the all-to-all, its wire time and
 * the placement tail, summed since the last reset. */
int  lsb_get_pass_exchange(lsb_ctx_t* ctx, int pass, int64_t* bytes, double* wire_ms,
                           double* place_tail_ms);

/* How the local rank's record buffers A and B were placed.  Record buffers of
 * at least 1 GiB are built from 1 GiB physical pieces (HIP virtual memory;
 * LSB_RECORD_ALLOC=malloc: hipMalloc) -- except in an RCCL context created
 * after an earlier RCCL context of the process released such buffers: such
 * contexts returned wrong data over pieces mapped at reused addresses (a
 * HIP VMM fault, reproduced with a copy kernel alone), so those take
 * hipMalloc'd buffers (LSB_RCCL_VMM=1: pieces regardless).
 * Such a buffer can still be a slow
 * pass destination as a whole, so a rank whose buffers hold
 * >= 4 GiB and that shares its device with no other rank of the context
 * tries 4 candidate buffers (LSB_PLACEMENT_CANDIDATES = K: K of them, at
 * most 8, for buffers of >= 1 GiB; 0: none) when three fit in half the free
 * memory (90 % when K is set).  Each candidate is timed once as the
 * destination of one k_onesweep pass over uniform keys (the speed that
 * differs); the two fastest destinations are kept and every other candidate
 * is freed as soon as it loses, so the probe holds at most one record buffer
 * more than A and B (see lsb_rank_footprint).  candidates = the candidates
 * timed, 0: no probe ran.  Milliseconds per pass as a destination: the mean
 * of the chosen two, the mean of the first two allocated (what a plain
 * allocation would have kept) and the slowest candidate. */
int  lsb_get_placement(lsb_ctx_t* ctx, int rank, int* candidates, double* chosen_ms,
                       double* first_pair_ms, double* worst_ms);

/* ---- device memory ------------------------------------------------------ */
/* Device bytes one rank of a context lsb_create(n_total, num_ranks,
 * radix_bits) holds (pure host arithmetic, no device needed): A and B (each
 * `per` records, rounded up to whole 1 GiB pieces when built from them), the
 * receive buffer R when with_recv (any exchange: num_ranks > 1 or forced; the
 * hybrid local sort), the single-read passes' look-back rows (4 B per bucket
 * per 4096-record tile), the gathered passes' tile descriptors (exchanges),
 * and the count and plan tables.  *probe_bytes: what the placement probe
 * (by default 4 candidates for buffers of >= 4 GiB; LSB_PLACEMENT_CANDIDATES,
 * read from the environment now) holds on top while it runs, at most: one
 * record buffer (a rank
 * that shares its device with another rank of its context runs none); 0 when
 * no probe would run.  A model of
 * init_rank's allocations, checked against the device's own free-memory
 * count by tests/test_footprint_gpu.py. */
int  lsb_rank_footprint(int64_t n_total, int num_ranks, int radix_bits, int with_recv,
                        int64_t* bytes, int64_t* probe_bytes);

/* Free and total device memory of device dev (hipMemGetInfo). */
int  lsb_device_memory(int dev, int64_t* free_bytes, int64_t* total_bytes);

/* ---- build --------------------------------------------------------------- */
/* "sha256=<digest of the sources the library was built from> host=<build
 * host> rccl=<ncclGetVersion of the RCCL loaded>" (static string).  tests/
 * compare the digest with the tree. */
const char* lsb_build_info(void);

/* ---- host planner (pure host code; used by the runtime when P > 1) ------- */
/* Given hist[s*nbuckets + b] = number of elements of bucket b that rank s
 * holds after its local stable pass (bucket order), compute rank `rank`'s
 * side of the exchange under the digit-major, rank-minor global order of
 * copyCountsToGlobalCounts / exclusiveScan (mpi/mpi_lsbsort.cpp:350,378,401):
 *   send_counts[q], send_displs[q]  elements of my bucket-ordered buffer for q
 *   recv_counts[s], recv_displs[s]  elements arriving from s, in s order
 *   place_off[s*nbuckets + b]       local slot = place_off[s][b] + recv index
 * All arrays are caller-allocated (P or P*nbuckets int64). */
int  lsb_plan_exchange(int64_t n_total, int num_ranks, int rank, int nbuckets,
                       const int64_t* hist,
                       int64_t* send_counts, int64_t* send_displs,
                       int64_t* recv_counts, int64_t* recv_displs,
                       int64_t* place_off);

/* The same plan computed by the device kernels the runtime uses (it keeps
 * place_off on the GPU and fetches only the 2P counts); host arrays in and
 * out, on device `dev_id`.  For testing the two planners against each other. */
int  lsb_plan_exchange_device(int dev_id, int64_t n_total, int num_ranks, int rank, int nbuckets,
                              const int64_t* hist,
                              int64_t* send_counts, int64_t* send_displs,
                              int64_t* recv_counts, int64_t* recv_displs,
                              int64_t* place_off);

/* Plan of the whole-key exchange (radix_bits = 64), host side.  After every
 * rank has sorted its block on the whole key, let k*_q be the key at global
 * position T_q = q * per (q = 1 .. P-1, the q with T_q < n) and
 *   below[s * (P-1) + q-1] = #records of rank s with key <  k*_q
 *   upto [s * (P-1) + q-1] = #records of rank s with key <= k*_q
 * (entries of targets T_q >= n are ignored).  Records of equal key keep rank
 * order, so source s's cut at T_q is below + min(equal, what T_q still
 * needs after the lower ranks).  Rank `rank` then sends its sorted range
 * [cut_q, cut_{q+1}) to q and receives [cut_rank, cut_{rank+1}) of every s:
 * counts and displacements (records) as for lsb_plan_exchange.  This is the
 * rule the runtime applies to the all-gathered counts of its device splitter
 * search (k_split_*), replacing copyCountsToGlobalCounts / exclusiveScan /
 * copyStartsFromGlobalStarts (mpi/mpi_lsbsort.cpp:327-479) for a digit of
 * 2^64 buckets.  LSB_ERR_INVALID when the counts do not bracket a target. */
int  lsb_plan_merge(int64_t n_total, int num_ranks, int rank, const int64_t* below,
                    const int64_t* upto, int64_t* send_counts, int64_t* send_displs,
                    int64_t* recv_counts, int64_t* recv_displs);

const char* lsb_strerror(int code);

#ifdef __cplusplus
}
#endif

#endif /* LSB_H */
