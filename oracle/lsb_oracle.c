/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the reference's distributed LSD radix sort
 * (ronawho/distributed-lsb, mpi/mpi_lsbsort.cpp) and of its PCG64 input
 * generator.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker: the
 * product path (distributed-lsb_amd/) never links or calls it.
 *
 * Parity pins (see oracle/README.md and tests/test_oracle.py):
 *   - pcg64 known answers recorded from the reference binary;
 *   - SHA-256 digests of input and sorted output of the reference binary
 *     for five (n, P) configurations (tests/golden/digests.json);
 *   - full small-n input/output vectors printed by the reference binary
 *     itself (tests/golden/ref_print_vectors.json, made by
 *     tests/golden/make_golden.py from oracle/_ref/mpi_lsbsort).
 *
 * pcg-cpp (imneme/pcg-cpp, header-only; the reference fetches it with
 * mpi/getpcg.sh:3) is not vendored by the reference; its published
 * algorithm for `pcg64` = setseq_xsl_rr_128_64 is restated below.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;

typedef struct {
  uint64_t key; /* to sort by   (mpi/mpi_lsbsort.cpp:30) */
  uint64_t val; /* carried along (mpi/mpi_lsbsort.cpp:31) */
} oracle_elem_t;

/* pcg-cpp default_multiplier<uint128> / default_increment<uint128>. */
#define PCG_MULT ((((u128)0x2360ED051FC65DA4ULL) << 64) | 0x4385DF649FCCF645ULL)
#define PCG_INC  ((((u128)0x5851F42D4C957F2DULL) << 64) | 0x14057B7EF767814FULL)

/* xsl_rr output of a 128-bit state: rotr64(hi ^ lo, state >> 122). */
static inline uint64_t pcg_out(u128 s) {
  uint64_t x = (uint64_t)(s >> 64) ^ (uint64_t)s;
  unsigned rot = (unsigned)(s >> 122);
  return (x >> rot) | (x << ((64u - rot) & 63u));
}

/* engine(seed): state = bump(seed + inc) where bump(s) = s*mult + inc. */
static inline u128 pcg_seed(uint64_t seed) {
  return ((u128)seed + PCG_INC) * PCG_MULT + PCG_INC;
}

/* LCG jump-ahead by `delta` steps (Brown, "Random number generation with
 * arbitrary strides"), as pcg-cpp's engine::advance. */
static u128 pcg_advance(u128 state, uint64_t delta) {
  u128 acc_mult = 1, acc_plus = 0, cur_mult = PCG_MULT, cur_plus = PCG_INC;
  while (delta) {
    if (delta & 1) {
      acc_mult *= cur_mult;
      acc_plus = acc_plus * cur_mult + cur_plus;
    }
    cur_plus = (cur_mult + 1) * cur_plus;
    cur_mult *= cur_mult;
    delta >>= 1;
  }
  return acc_mult * state + acc_plus;
}

/* k-th output (k = 0, 1, ...) of pcg64(seed): operator() bumps then outputs
 * the new state (output_previous = false for 128-bit state). */
uint64_t oracle_pcg64_at(uint64_t seed, uint64_t k) {
  return pcg_out(pcg_advance(pcg_seed(seed), k + 1));
}

/* Fill `count` consecutive outputs of pcg64(seed) starting at output k0. */
void oracle_pcg64_fill(uint64_t seed, uint64_t k0, int64_t count, uint64_t* out) {
  u128 s = pcg_advance(pcg_seed(seed), k0);
  for (int64_t i = 0; i < count; i++) {
    s = s * PCG_MULT + PCG_INC;
    out[i] = pcg_out(s);
  }
}

static inline int64_t div_ceil(int64_t x, int64_t y) { return (x + y - 1) / y; }

/* DistributedArray::create block partition (mpi/mpi_lsbsort.cpp:144-149). */
int64_t oracle_per_rank(int64_t n, int P) { return P > 0 ? div_ceil(n, P) : 0; }
int64_t oracle_here(int64_t n, int P, int r) {
  int64_t per = oracle_per_rank(n, P);
  int64_t here = per;
  if (per * r + here > n) here = n - per * r;
  if (here < 0) here = 0;
  return here;
}

/* Input of the reference (mpi/mpi_lsbsort.cpp:650-656): rng = pcg64(rank);
 * every one of the `per` local slots gets key = rng(), val = global index.
 * Writes the P*per slot image (tail padding of the last ranks included). */
void oracle_generate(int64_t n, int P, oracle_elem_t* slots) {
  int64_t per = oracle_per_rank(n, P);
  for (int r = 0; r < P; r++) {
    u128 s = pcg_seed((uint64_t)r);
    for (int64_t i = 0; i < per; i++) {
      s = s * PCG_MULT + PCG_INC;
      slots[r * per + i].key = pcg_out(s);
      slots[r * per + i].val = (uint64_t)(r * per + i);
    }
  }
}

/*
 * mySort with P logical ranks (mpi/mpi_lsbsort.cpp:580-585), digit width
 * `bits` (the reference uses RADIX 16, mpi/mpi_lsbsort.cpp:21).  `slots` is
 * the P*per image; each rank sorts its first here_r slots.  Per digit this
 * restates globalShuffle (mpi/mpi_lsbsort.cpp:481-577):
 *   localShuffle            :213-247  count, exclusive scan, stable scatter A->B
 *   copyCountsToGlobalCounts :327-383  GlobalCounts[digit*P + rank]
 *   exclusiveScan            :385-414  global exclusive prefix
 *   copyStartsFromGlobalStarts :416-479 starts[digit] for this rank
 *   element exchange         :527-576  dst = starts[bucket]++ over bucket-ordered B
 * The exchange is an in-memory placement into the owner's slot.
 * Returns 0, or -1 on allocation failure.
 */
int oracle_mpi_sort(int64_t n, int P, int bits, oracle_elem_t* slots) {
  if (P <= 0 || bits <= 0 || bits > 16 || 64 % bits) return -1;
  const int64_t per = oracle_per_rank(n, P);
  const int64_t nb = (int64_t)1 << bits;
  const uint64_t mask = (uint64_t)nb - 1;
  const int ndig = 64 / bits;
  if (per == 0) return 0;
  oracle_elem_t* B = (oracle_elem_t*)malloc(sizeof(oracle_elem_t) * (size_t)(P * per));
  int64_t* counts = (int64_t*)calloc((size_t)(nb * P), sizeof(int64_t));
  int64_t* lstart = (int64_t*)malloc(sizeof(int64_t) * (size_t)nb);
  int64_t* gstart = (int64_t*)malloc(sizeof(int64_t) * (size_t)(nb * P));
  if (!B || !counts || !lstart || !gstart) {
    free(B); free(counts); free(lstart); free(gstart);
    return -1;
  }
  for (int d = 0; d < ndig; d++) {
    const int sh = d * bits;
    memset(counts, 0, sizeof(int64_t) * (size_t)(nb * P));
    for (int r = 0; r < P; r++) {
      const int64_t here = oracle_here(n, P, r);
      oracle_elem_t* A_r = slots + r * per;
      oracle_elem_t* B_r = B + r * per;
      int64_t* c = counts + r * nb;
      for (int64_t i = 0; i < here; i++) c[(A_r[i].key >> sh) & mask]++;
      int64_t sum = 0;
      for (int64_t b = 0; b < nb; b++) { lstart[b] = sum; sum += c[b]; }
      for (int64_t i = 0; i < here; i++) B_r[lstart[(A_r[i].key >> sh) & mask]++] = A_r[i];
    }
    /* digit-major, rank-minor exclusive scan */
    int64_t sum = 0;
    for (int64_t b = 0; b < nb; b++)
      for (int r = 0; r < P; r++) {
        gstart[b * P + r] = sum;
        sum += counts[r * nb + b];
      }
    for (int r = 0; r < P; r++) {
      const int64_t here = oracle_here(n, P, r);
      const oracle_elem_t* B_r = B + r * per;
      for (int64_t i = 0; i < here; i++) {
        const int64_t b = (int64_t)((B_r[i].key >> sh) & mask);
        const int64_t dst = gstart[b * P + r]++;
        /* globalIdxToLocalIdx (mpi/mpi_lsbsort.cpp:113-120): the P*per
         * image is laid out rank-major, so the slot index is dst itself. */
        slots[dst] = B_r[i];
      }
    }
  }
  free(B); free(counts); free(lstart); free(gstart);
  return 0;
}

/* One local stable counting-sort pass, in -> out, on digit `digit` of width
 * `bits` (localShuffle, mpi/mpi_lsbsort.cpp:213-247).  Used as the checker
 * of a single HIP pass.  `hist` (2^bits entries) receives the counts. */
int oracle_local_pass(const oracle_elem_t* in, oracle_elem_t* out, int64_t m,
                      int bits, int digit, int64_t* hist) {
  const int64_t nb = (int64_t)1 << bits;
  const uint64_t mask = (uint64_t)nb - 1;
  const int sh = digit * bits;
  int64_t* start = (int64_t*)malloc(sizeof(int64_t) * (size_t)nb);
  if (!start) return -1;
  memset(hist, 0, sizeof(int64_t) * (size_t)nb);
  for (int64_t i = 0; i < m; i++) hist[(in[i].key >> sh) & mask]++;
  int64_t sum = 0;
  for (int64_t b = 0; b < nb; b++) { start[b] = sum; sum += hist[b]; }
  for (int64_t i = 0; i < m; i++) out[start[(in[i].key >> sh) & mask]++] = in[i];
  free(start);
  return 0;
}

/* std::stable_sort by key (mpi/mpi_lsbsort.cpp:722-726), as a bottom-up
 * merge sort.  Independent of the radix restatement above. */
int oracle_stable_sort(oracle_elem_t* a, int64_t n) {
  if (n < 2) return 0;
  oracle_elem_t* t = (oracle_elem_t*)malloc(sizeof(oracle_elem_t) * (size_t)n);
  if (!t) return -1;
  oracle_elem_t *src = a, *dst = t;
  for (int64_t w = 1; w < n; w *= 2) {
    for (int64_t lo = 0; lo < n; lo += 2 * w) {
      int64_t mid = lo + w < n ? lo + w : n;
      int64_t hi = lo + 2 * w < n ? lo + 2 * w : n;
      int64_t i = lo, j = mid, k = lo;
      while (i < mid && j < hi) dst[k++] = (src[j].key < src[i].key) ? src[j++] : src[i++];
      while (i < mid) dst[k++] = src[i++];
      while (j < hi) dst[k++] = src[j++];
    }
    oracle_elem_t* x = src; src = dst; dst = x;
  }
  if (src != a) memcpy(a, src, sizeof(oracle_elem_t) * (size_t)n);
  free(t);
  return 0;
}

/* SHMEM checkSorted semantics (shmem/shmem_lsbsort.cpp:180-219): key order
 * within each rank's here-part and across the first/last boundary records. */
int oracle_check_sorted(int64_t n, int P, const oracle_elem_t* slots) {
  const int64_t per = oracle_per_rank(n, P);
  uint64_t prev = 0;
  int have = 0;
  for (int r = 0; r < P; r++) {
    const int64_t here = oracle_here(n, P, r);
    for (int64_t i = 0; i < here; i++) {
      uint64_t k = slots[r * per + i].key;
      if (have && k < prev) return 0;
      prev = k;
      have = 1;
    }
  }
  return 1;
}
