// ASan/UBSan driver for the C ABI's host code (sanitizers on host
// code).  `make -C distributed-lsb_amd asan` links it against an ASan/UBSan
// build of the runtime units (csrc/lsb_*.cpp; device code unchanged) and runs it without a GPU:
//   - lsb_plan_exchange on random, skewed, empty and n < P count matrices:
//     conservation (sum send = sum recv = here), displacement prefix sums,
//     every live placement offset inside [0, here);
//   - every argument check that returns before a device call;
//   - lsb_create / lsb_create_rank_ops with no usable device: the failure
//     path tears down a half-built context (no leak, no double free).
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

#include "lsb.h"

static int fails = 0;
#define CHECK(c, what)                                    \
  do {                                                    \
    if (!(c)) {                                           \
      std::fprintf(stderr, "FAILED: %s (%s:%d)\n", what, __FILE__, __LINE__); \
      ++fails;                                            \
    }                                                     \
  } while (0)

static void plan_case(std::mt19937_64& rng, int64_t n, int P, int nb, bool skew) {
  std::vector<int64_t> hist((size_t)P * nb, 0);
  for (int s = 0; s < P; ++s) {
    int64_t h = lsb_here(n, P, s);
    for (int64_t i = 0; i < h; ++i) {
      int b = skew ? (int)((rng() % 7 == 0) ? rng() % nb : 3) : (int)(rng() % nb);
      ++hist[(size_t)s * nb + b];
    }
  }
  // every rank's plan
  std::vector<std::vector<int64_t>> sc(P), sd(P), rc(P), rd(P), place(P);
  for (int me = 0; me < P; ++me) {
    sc[me].resize(P), sd[me].resize(P), rc[me].resize(P), rd[me].resize(P);
    place[me].assign((size_t)P * nb, -7);
    int rcode = lsb_plan_exchange(n, P, me, nb, hist.data(), sc[me].data(), sd[me].data(),
                                  rc[me].data(), rd[me].data(), place[me].data());
    CHECK(rcode == LSB_OK, "plan ok");
    int64_t ss = 0, rs = 0;
    for (int q = 0; q < P; ++q) {
      CHECK(sd[me][q] == ss && rd[me][q] == rs, "displacements are prefix sums");
      ss += sc[me][q];
      rs += rc[me][q];
    }
    CHECK(ss == lsb_here(n, P, me), "send total = here");
    CHECK(rs == lsb_here(n, P, me), "recv total = here");
  }
  // Receiver me: record k of the segment from s is record sd[s][me] + (k - rd[me][s])
  // of s's bucket-ordered buffer; its slot place[me][s][bucket] + k must
  // cover [0, here) exactly once.
  for (int me = 0; me < P; ++me) {
    const int64_t here = lsb_here(n, P, me);
    std::vector<char> seen((size_t)here + 1, 0);
    for (int s = 0; s < P; ++s) {
      CHECK(sc[s][me] == rc[me][s], "send/recv counts agree");
      int b = 0;
      int64_t bend = hist[(size_t)s * nb];  // end of bucket b in s's buffer
      for (int64_t i = 0; i < rc[me][s]; ++i) {
        const int64_t pos = sd[s][me] + i;
        while (b < nb - 1 && pos >= bend) bend += hist[(size_t)s * nb + ++b];
        const int64_t k = rd[me][s] + i;
        const int64_t slot = place[me][(size_t)s * nb + b] + k;
        const bool in = slot >= 0 && slot < here;
        CHECK(in, "slot inside here-part");
        if (in) {
          CHECK(!seen[(size_t)slot], "slot used once");
          seen[(size_t)slot] = 1;
        }
      }
    }
  }
}

static int noop_ag(void*, const void*, void*, size_t) { return 0; }
static int noop_a2a(void*, const void*, const size_t*, const size_t*, void*, const size_t*,
                    const size_t*) { return 0; }
static int noop_min(void*, int64_t*) { return 0; }
static int noop_bar(void*) { return 0; }

int main() {
  std::mt19937_64 rng(12345);
  const int64_t ns[] = {0, 1, 7, 1000, 100003};
  const int Ps[] = {1, 2, 3, 8, 64};
  for (int64_t n : ns)
    for (int P : Ps)
      for (int nb : {256, 65536})
        for (bool skew : {false, true})
          if (!(nb == 65536 && P == 64)) plan_case(rng, n, P, nb, skew);

  // argument checks
  std::vector<int64_t> h(2 * 256, 0), o(2), pl(2 * 256);
  CHECK(lsb_plan_exchange(0, 2, 2, 256, h.data(), o.data(), o.data(), o.data(), o.data(),
                          pl.data()) == LSB_ERR_INVALID, "rank >= P");
  h[5] = -1;
  CHECK(lsb_plan_exchange(10, 2, 0, 256, h.data(), o.data(), o.data(), o.data(), o.data(),
                          pl.data()) == LSB_ERR_INVALID, "negative count");
  lsb_ctx_t* c = nullptr;
  CHECK(lsb_create(nullptr, 1, 1, nullptr, 8) == LSB_ERR_INVALID, "null out");
  CHECK(lsb_create(&c, 1, 0, nullptr, 8) == LSB_ERR_INVALID, "P = 0");
  CHECK(lsb_create(&c, 1, 1, nullptr, 12) == LSB_ERR_UNSUPPORTED, "radix 12");
  CHECK(lsb_sort(nullptr) == LSB_ERR_INVALID, "null ctx");
  CHECK(lsb_set_option(nullptr, 0, 0) == LSB_ERR_INVALID, "null ctx option");
  for (int code = 0; code < 8; ++code) CHECK(lsb_strerror(code) != nullptr, "strerror");
  CHECK(lsb_per_rank(10, 3) == 4 && lsb_here(10, 3, 2) == 2 && lsb_here(10, 3, 3) == 0, "geometry");

  // no usable device in this container: creation fails cleanly
  int rc1 = lsb_create(&c, 1 << 20, 3, nullptr, 16);
  CHECK((rc1 == LSB_OK) == (c != nullptr), "create result consistent");
  if (c) lsb_destroy(c);
  lsb_comm_ops_t ops = {nullptr, noop_ag, noop_a2a, noop_min, noop_bar};
  c = nullptr;
  int rc2 = lsb_create_rank_ops(&c, 1 << 20, 2, 0, 0, 8, &ops);
  CHECK((rc2 == LSB_OK) == (c != nullptr), "create_rank_ops result consistent");
  if (c) lsb_destroy(c);
  lsb_destroy(nullptr);

  std::printf("host ABI sanitizer driver: %s (create without device: %d, %d)\n",
              fails ? "FAILED" : "ok", rc1, rc2);
  return fails ? 1 : 0;
}
