/*
 * ASan/UBSan driver for the oracle (test infrastructure only; SURVEY §5:
 * "host ASan/UBSan on the CPU restatement").  `make -C oracle sanitize`
 * builds it with -fsanitize=address,undefined and runs it:
 *   - pcg64 known answers (pcg-cpp setseq_xsl_rr_128_64);
 *   - oracle_mpi_sort at 8 and 16 bits over ragged and tiny (n, P) equals the
 *     independent merge sort of the same input (mpi/mpi_lsbsort.cpp:722-737);
 *   - oracle_check_sorted on the result, and on a broken one.
 * Exit status 0 = all passed; any sanitizer report aborts with non-zero.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  uint64_t key, val;
} oracle_elem_t;

uint64_t oracle_pcg64_at(uint64_t seed, uint64_t k);
int64_t oracle_per_rank(int64_t n, int P);
int64_t oracle_here(int64_t n, int P, int r);
void oracle_generate(int64_t n, int P, oracle_elem_t* slots);
int oracle_mpi_sort(int64_t n, int P, int bits, oracle_elem_t* slots);
int oracle_stable_sort(oracle_elem_t* a, int64_t n);
int oracle_check_sorted(int64_t n, int P, const oracle_elem_t* slots);

static int fails = 0;
#define CHECK(c, ...)                 \
  do {                                \
    if (!(c)) {                       \
      fprintf(stderr, __VA_ARGS__);   \
      fputc('\n', stderr);            \
      ++fails;                        \
    }                                 \
  } while (0)

/* here-parts of the P*per slot image, in rank order */
static int64_t gather(int64_t n, int P, const oracle_elem_t* slots, oracle_elem_t* out) {
  int64_t per = oracle_per_rank(n, P), k = 0;
  for (int r = 0; r < P; r++) {
    int64_t h = oracle_here(n, P, r);
    memcpy(out + k, slots + r * per, sizeof(oracle_elem_t) * (size_t)h);
    k += h;
  }
  return k;
}

int main(void) {
  const uint64_t ka[2][3] = {{0x01070196e695f8f1ull, 0x703ec840c59f4493ull, 0xe54954914b3a44faull},
                             {0xe175e32ed3507bfaull, 0xc0bf922a0b283109ull, 0x140bfa21e68785bbull}};
  for (int s = 0; s < 2; s++)
    for (int i = 0; i < 3; i++)
      CHECK(oracle_pcg64_at((uint64_t)s, (uint64_t)i) == ka[s][i], "pcg64(%d)[%d]", s, i);

  const int64_t ns[] = {0, 1, 2, 3, 17, 20, 4097, 100003};
  const int Ps[] = {1, 2, 3, 4, 8};
  const int bitss[] = {8, 16};
  for (size_t a = 0; a < sizeof ns / sizeof *ns; a++)
    for (size_t b = 0; b < sizeof Ps / sizeof *Ps; b++)
      for (size_t c = 0; c < 2; c++) {
        const int64_t n = ns[a];
        const int P = Ps[b], bits = bitss[c];
        const int64_t per = oracle_per_rank(n, P);
        const size_t cap = (size_t)(P * per) + 1;
        oracle_elem_t* slots = malloc(sizeof(oracle_elem_t) * cap);
        oracle_elem_t* want = malloc(sizeof(oracle_elem_t) * cap);
        oracle_elem_t* got = malloc(sizeof(oracle_elem_t) * cap);
        if (!slots || !want || !got) return 2;
        oracle_generate(n, P, slots);
        const int64_t m = gather(n, P, slots, want);
        CHECK(m == n, "gather n=%lld P=%d", (long long)n, P);
        CHECK(oracle_stable_sort(want, m) == 0, "stable_sort");
        CHECK(oracle_mpi_sort(n, P, bits, slots) == 0, "mpi_sort");
        gather(n, P, slots, got);
        CHECK(memcmp(want, got, sizeof(oracle_elem_t) * (size_t)m) == 0,
              "mpi_sort != stable_sort at n=%lld P=%d bits=%d", (long long)n, P, bits);
        CHECK(oracle_check_sorted(n, P, slots) == 1, "check_sorted n=%lld P=%d", (long long)n, P);
        if (n >= 2) {  /* a descent must be caught */
          oracle_elem_t t = slots[0];
          int r1 = 0;
          while (oracle_here(n, P, r1) < 1) r1++;
          int64_t last = (int64_t)P * per - 1;
          while (last > 0 && oracle_here(n, P, (int)(last / per)) <= last % per) last--;
          slots[0] = slots[last];
          slots[last] = t;
          CHECK(slots[0].key == slots[last].key || oracle_check_sorted(n, P, slots) == 0,
                "check_sorted missed a descent n=%lld P=%d", (long long)n, P);
        }
        free(slots);
        free(want);
        free(got);
      }
  printf("oracle sanitizer driver: %s\n", fails ? "FAILED" : "ok");
  return fails ? 1 : 0;
}
