// hip_lsbsort — the MI355X peer of mpi/mpi_lsbsort.cpp and shmem/shmem_lsbsort.cpp.
//
// Same command line (--n N, --print, --verify, --no-verify; verify defaults
// to on iff n < 128Mi, mpi/mpi_lsbsort.cpp:591-611), same input (pcg64(rank),
// val = global index), same timing window (sort only, between barriers,
// :688-699) and the same output lines; the sort itself runs on GPUs through
// the C ABI in include/lsb.h.
//
// Ranks:
//   --gpus P   one process per GPU (rank r on device r), exchange over RCCL;
//              this program forks the P rank processes itself, before any HIP
//              call, the way mpirun would start them.
//   --ranks P  P logical ranks driven by this one process on --device D
//              (default 0), exchange by device copies; same results as
//              `mpirun -n P mpi_lsbsort` on one GPU.
//   --json     also print one machine-readable line.
//   --radix-bits 8|16|64  exchange digit width (local passes are always 8-bit):
//              16 (the reference's RADIX, one RCCL all-to-all per 16-bit digit;
//              the default with --gpus P > 1, as in bench.py), 8 (8 all-to-alls;
//              the default otherwise), or 64: local sort, ONE all-to-all, merge
//              of the P runs
//   --test-corrupt I  test hook: overwrite sorted record I before verifying
//              (the failure report: every mismatch, Expected/Got, status 134)
//   --dist uniform|zipf [--zipf-s S]   key distribution of the same pcg64 stream
//   --exchange alltoallv|p2p|peer  element exchange (default RCCL AllToAllv in
//              slices; grouped Send/Recv; direct peer stores, the shmem_putmem form)
//   --slices S  all-to-all slices whose placement overlaps the next slice
//   --hybrid 0|1|2  local sort by the hybrid (LSB_OPT_HYBRID: k top-byte passes,
//              then the segments ordered inside the last pass (1) or by a
//              k_segsort pass (2)); the same output; 0 (default) = LSD passes
//   --share-gpus G  with --gpus P: rank r runs on device r % G and is its own
//              RCCL "host" (NCCL_HOSTID), so RCCL links ranks that share a GPU
//              by its socket transport -- a rehearsal of the multi-GPU path on
//              fewer GPUs (RCCL refuses two ranks of one host on one device)
//   --shmem    the lines and semantics of shmem/shmem_lsbsort.cpp's main
//              (:474-584) instead of the MPI program's: "Total number of shmem
//              PEs", verify on unless --no-verify, printed elements tagged
//              "(rank r)", the check is checkSorted alone (key order within and
//              across ranks, :180-219: "Array is sorted" / "Array is NOT
//              sorted") and the exit status is !sorted (:583)
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "lsb.h"

namespace {

struct Options {
  int64_t n = 100LL * 1000 * 1000;
  bool print = false;
  bool verify = false;
  bool verify_set = false;
  int gpus = 0;
  int ranks = 1;
  int device = 0;
  bool json = false;
  int radix_bits = 0;        // --radix-bits (0: 16 with --gpus > 1, else 8)
  int dist = LSB_DIST_UNIFORM;
  double zipf_s = 1.1;
  int exchange_option = -1;  // --exchange: LSB_OPT_EXCHANGE_P2P / _PEER, or -1 (AllToAllv)
  int slices = 0;            // --slices S (0: library default)
  int hybrid = 0;            // --hybrid 0|1|2 (LSB_OPT_HYBRID)
  int64_t test_corrupt = -1; // --test-corrupt I: overwrite sorted record I (tests the report)
  int share_gpus = 0;        // --share-gpus G: rank r on device r % G, one RCCL host per rank
  bool shmem = false;        // --shmem: shmem_lsbsort.cpp's lines and exit status
};

void flush_output() {
  // mpi/mpi_lsbsort.cpp:163-169 flushes and sleeps so rank output interleaves
  // in order; here ranks are ordered by barriers, a flush is enough.
  fflush(stdout);
}

void die(const char* what, int rc) {
  fprintf(stderr, "hip_lsbsort: %s failed: %s\n", what, lsb_strerror(rc));
  fflush(stderr);
  _exit(2);
}

#define CHECK(call)                 \
  do {                              \
    int _rc = (call);               \
    if (_rc != LSB_OK) die(#call, _rc); \
  } while (0)

struct World {
  lsb_ctx_t* ctx = nullptr;
  int P = 1;
  int first = 0;
  int nlocal = 1;
  int64_t n = 0;
  int64_t per = 0;
  int dev = 0;  // device of this process's ranks
  // --gpus P: the failure report's gather to the root (MPI_Gather of the
  // output, mpi/mpi_lsbsort.cpp:717-719): report_fd[r] is the root's read end
  // of rank r's pipe; report_fd[first] a non-root rank's write end.
  std::vector<int> report_fd;
  bool root() const { return first == 0; }
  bool is_local(int r) const { return r >= first && r < first + nlocal; }
};

// DistributedArray::print (mpi/mpi_lsbsort.cpp:171-200; shmem: each element
// tagged with its rank, shmem/shmem_lsbsort.cpp:149-177).
void print_array(World& w, const char* name, int64_t n_per_rank, bool shmem) {
  CHECK(lsb_barrier(w.ctx));
  if (w.root()) {
    if (n_per_rank * w.P >= w.n)
      printf("%s: displaying all %" PRId64 " elements\n", name, w.n);
    else
      printf("%s: displaying first %" PRId64 " elements on each rank out of %" PRId64
             " elements\n", name, n_per_rank, w.n);
  }
  std::vector<lsb_elem_t> buf(n_per_rank);
  for (int r = 0; r < w.P; ++r) {
    if (w.is_local(r)) {
      const int64_t here = lsb_here(w.n, w.P, r);
      const int64_t k = here < n_per_rank ? here : n_per_rank;
      CHECK(lsb_copy_out(w.ctx, r, 0, k, buf.data()));
      for (int64_t i = 0; i < k; ++i) {
        printf("%s[%" PRId64 "] = (%016" PRIx64 ",%" PRIu64 ")", name, r * w.per + i, buf[i].key,
               buf[i].val);
        if (shmem) printf(" (rank %d)", r);
        printf("\n");
      }
      if (k < here) printf("...\n");
      flush_output();
    }
    CHECK(lsb_barrier(w.ctx));
  }
}

// Whole-buffer pipe I/O (the report's gather).
bool write_all(int fd, const void* p, size_t bytes) {
  const char* c = static_cast<const char*>(p);
  while (bytes > 0) {
    const ssize_t k = write(fd, c, bytes);
    if (k <= 0) return false;
    c += k;
    bytes -= (size_t)k;
  }
  return true;
}

bool read_all(int fd, void* p, size_t bytes) {
  char* c = static_cast<char*>(p);
  while (bytes > 0) {
    const ssize_t k = read(fd, c, bytes);
    if (k <= 0) return false;
    c += k;
    bytes -= (size_t)k;
  }
  return true;
}

constexpr int64_t kReportChunk = 1 << 20;  // records per pipe transfer

// The reference's failure report (mpi/mpi_lsbsort.cpp:715-737): the output
// is gathered to the root, which compares every index with std::stable_sort
// of the input by key and prints each mismatch with the expected and the
// actual record.  Only the root regenerates the input (a loopback context of
// the same n, P and key distribution on its device: the on-device PCG stream
// the sort started from) and sorts it on the host: host memory O(n) once, as
// the reference's rank 0.  The other rank processes stream their records to
// it through pipes, in rank order; there is no collective in the report.
void report_mismatches(World& w, const Options& o) {
  std::vector<lsb_elem_t> got;
  if (!w.root()) {  // --gpus: send my part to the root
    const int64_t here = lsb_here(o.n, w.P, w.first);
    const int fd = w.report_fd[w.first];
    if (!write_all(fd, &here, sizeof here)) die("report: write", LSB_ERR_STATE);
    for (int64_t off = 0; off < here; off += kReportChunk) {
      const int64_t k = std::min(kReportChunk, here - off);
      got.resize((size_t)k);
      CHECK(lsb_copy_out(w.ctx, w.first, off, k, got.data()));
      if (!write_all(fd, got.data(), (size_t)k * sizeof(lsb_elem_t))) die("report: write", LSB_ERR_STATE);
    }
    close(fd);
    return;
  }
  std::vector<lsb_elem_t> expect((size_t)o.n);
  {
    lsb_ctx_t* gen = nullptr;
    std::vector<int> devs(w.P, w.dev);
    CHECK(lsb_create(&gen, o.n, w.P, devs.data(), 8));
    CHECK(lsb_generate_ex(gen, o.dist, o.zipf_s));
    for (int r = 0; r < w.P; ++r)
      CHECK(lsb_copy_out(gen, r, 0, lsb_here(o.n, w.P, r), expect.data() + (size_t)r * w.per));
    lsb_destroy(gen);
  }
  std::stable_sort(expect.begin(), expect.end(),
                   [](const lsb_elem_t& a, const lsb_elem_t& b) { return a.key < b.key; });
  for (int r = 0; r < w.P; ++r) {
    const int64_t here = lsb_here(o.n, w.P, r);
    int64_t sent = here;
    if (!w.is_local(r) && !read_all(w.report_fd[r], &sent, sizeof sent)) {
      printf("Rank %d sent no records\n", r);
      continue;
    }
    if (sent != here) die("report: record count", LSB_ERR_STATE);
    for (int64_t off = 0; off < here; off += kReportChunk) {
      const int64_t k = std::min(kReportChunk, here - off);
      got.resize((size_t)k);
      if (w.is_local(r)) CHECK(lsb_copy_out(w.ctx, r, off, k, got.data()));
      else if (!read_all(w.report_fd[r], got.data(), (size_t)k * sizeof(lsb_elem_t)))
        die("report: read", LSB_ERR_STATE);
      for (int64_t i = 0; i < k; ++i) {
        const int64_t gi = r * w.per + off + i;
        const lsb_elem_t& e = expect[(size_t)gi];
        const lsb_elem_t& g = got[(size_t)i];
        if (e.key == g.key && e.val == g.val) continue;
        printf("Sorted element %" PRId64 " did not match\n", gi);
        printf("Expected: (%016" PRIx64 ",%" PRIu64 ")\n", e.key, e.val);
        printf("Got:      (%016" PRIx64 ",%" PRIu64 ")\n", g.key, g.val);
      }
    }
    if (!w.is_local(r)) close(w.report_fd[r]);
  }
  flush_output();
}

int run(World& w, const Options& o) {
  if (o.exchange_option >= 0) CHECK(lsb_set_option(w.ctx, o.exchange_option, 1));
  if (o.slices > 0) CHECK(lsb_set_option(w.ctx, LSB_OPT_EXCHANGE_SLICES, o.slices));
  if (o.hybrid > 0) CHECK(lsb_set_option(w.ctx, LSB_OPT_HYBRID, o.hybrid));
  if (w.root()) {
    // the reference's own line (mpi/mpi_lsbsort.cpp:619, shmem/shmem_lsbsort.cpp:498):
    // a rank here is one GPU
    if (o.shmem) printf("Total number of shmem PEs: %d\n", w.P);
    else printf("Total number of MPI ranks: %d\n", w.P);
    printf("Problem size: %" PRId64 "\n", o.n);
    flush_output();
  }
  {
    auto start = std::chrono::steady_clock::now();
    if (w.root()) {
      printf("Generating random values\n");
      flush_output();
    }
    CHECK(lsb_generate_ex(w.ctx, o.dist, o.zipf_s));
    CHECK(lsb_barrier(w.ctx));
    auto end = std::chrono::steady_clock::now();
    if (w.root()) {
      printf("Generated random values in %g s\n", std::chrono::duration<double>(end - start).count());
      flush_output();
    }
    CHECK(lsb_barrier(w.ctx));
  }
  if (o.print) print_array(w, "A", 10, o.shmem);

  double elapsed = 0;
  {
    if (w.root()) {
      printf("Sorting\n");
      flush_output();
    }
    CHECK(lsb_barrier(w.ctx));
    auto start = std::chrono::steady_clock::now();
    CHECK(lsb_sort(w.ctx));
    CHECK(lsb_barrier(w.ctx));
    auto end = std::chrono::steady_clock::now();
    elapsed = std::chrono::duration<double>(end - start).count();
    if (w.root()) {
      printf("Sorted %" PRId64 " values in %g\n", o.n, elapsed);
      printf("That's %g M elements sorted / s\n", o.n / elapsed / 1000.0 / 1000.0);
      flush_output();
    }
    CHECK(lsb_barrier(w.ctx));
  }
  if (o.print) print_array(w, "A", 10, o.shmem);
  if (o.test_corrupt >= 0 && o.test_corrupt < o.n) {
    // Test hook: overwrite one sorted record so the failure report can be checked.
    const int r = (int)(o.test_corrupt / w.per);
    if (w.is_local(r)) {
      lsb_elem_t bad = {0x0123456789abcdefull, (uint64_t)o.n + 7};
      CHECK(lsb_copy_in(w.ctx, r, o.test_corrupt - r * w.per, 1, &bad));
    }
    CHECK(lsb_barrier(w.ctx));
  }

  int status = 0;
  if (o.verify && o.shmem) {
    // shmem_lsbsort's check (:568-583): checkSorted only, exit status !sorted
    int sorted = 0;
    CHECK(lsb_check_sorted(w.ctx, &sorted));
    if (w.root()) printf(sorted ? "Array is sorted\n" : "Array is NOT sorted\n");
    flush_output();
    status = sorted ? 0 : 1;
  } else if (o.verify) {
    if (w.root()) {
      printf("Verifying\n");
      flush_output();
    }
    int64_t first_bad = -1;
    const int rc = lsb_verify(w.ctx, &first_bad);
    if (rc == LSB_ERR_VERIFY) {
      status = 1;
    } else if (rc != LSB_OK) {
      die("lsb_verify", rc);
    }
    int sorted = 0;
    CHECK(lsb_check_sorted(w.ctx, &sorted));
    if (w.root()) printf(sorted ? "Array is sorted\n" : "Array is NOT sorted\n");
    if (!sorted) status = 1;
    flush_output();
    if (status) {
      // The reference then fails `assert(!failures)` (:737): exit with the
      // status such an abort gives (134) after a clean teardown.
      report_mismatches(w, o);
      if (w.root()) fprintf(stderr, "hip_lsbsort: Assertion `!failures' failed.\n");
      fflush(stderr);
      lsb_destroy(w.ctx);
      _exit(134);
    }
  }
  if (o.json && w.root()) {
    printf("{\"n\": %" PRId64 ", \"ranks\": %d, \"sort_s\": %.9g, \"melem_per_s\": %.6g, "
           "\"verified\": %s}\n", o.n, w.P, elapsed, o.n / elapsed / 1e6,
           o.verify ? (status == 0 ? "true" : "false") : "null");
    flush_output();
  }
  return status;
}

int run_rank_process(const Options& o, int rank, int read_fd, const std::vector<int>& write_fds,
                     const std::vector<int>& report_fd) {
  int dev = rank;
  if (o.share_gpus > 0) {
    // Before anything touches RCCL: one host per rank, linked over loopback.
    char host[64];
    snprintf(host, sizeof host, "hip-lsbsort-rank-%d", rank);
    setenv("NCCL_HOSTID", host, 1);
    setenv("NCCL_SOCKET_IFNAME", "lo", 0);
    setenv("NCCL_IB_DISABLE", "1", 0);
    dev = rank % o.share_gpus;
  }
  unsigned char id[LSB_UNIQUE_ID_BYTES];
  if (rank == 0) {
    CHECK(lsb_get_unique_id(id));
    for (int fd : write_fds)
      if (write(fd, id, sizeof id) != (ssize_t)sizeof id) die("write unique id", LSB_ERR_STATE);
  } else {
    size_t got = 0;
    while (got < sizeof id) {
      ssize_t k = read(read_fd, id + got, sizeof id - got);
      if (k <= 0) die("read unique id", LSB_ERR_STATE);
      got += (size_t)k;
    }
  }
  World w;
  w.P = o.gpus;
  w.n = o.n;
  w.per = lsb_per_rank(o.n, o.gpus);
  w.first = rank;
  w.nlocal = 1;
  w.dev = dev;
  w.report_fd = report_fd;
  CHECK(lsb_create_rank(&w.ctx, o.n, o.gpus, rank, dev, o.radix_bits, id));
  const int status = run(w, o);
  lsb_destroy(w.ctx);
  return status;
}

}  // namespace

int main(int argc, char* argv[]) {
  Options o;
  for (int i = 1; i < argc; i++) {
    const std::string a = argv[i];
    auto next = [&](void) -> const char* {
      if (i + 1 >= argc) {
        fprintf(stderr, "missing value for %s\n", a.c_str());
        exit(2);
      }
      return argv[++i];
    };
    if (a == "--n") o.n = std::stoll(next());
    else if (a == "--print") o.print = true;
    else if (a == "--verify") { o.verify = true; o.verify_set = true; }
    else if (a == "--no-verify") { o.verify = false; o.verify_set = true; }
    else if (a == "--gpus") o.gpus = std::stoi(next());
    else if (a == "--ranks") o.ranks = std::stoi(next());
    else if (a == "--device") o.device = std::stoi(next());
    else if (a == "--json") o.json = true;
    else if (a == "--radix-bits") o.radix_bits = std::stoi(next());
    else if (a == "--zipf-s") o.zipf_s = std::stod(next());
    else if (a == "--slices") o.slices = std::stoi(next());
    else if (a == "--hybrid") o.hybrid = std::stoi(next());
    else if (a == "--test-corrupt") o.test_corrupt = std::stoll(next());
    else if (a == "--share-gpus") o.share_gpus = std::stoi(next());
    else if (a == "--shmem") o.shmem = true;
    else if (a == "--exchange") {
      const std::string x = next();
      if (x == "alltoallv") o.exchange_option = -1;
      else if (x == "p2p") o.exchange_option = LSB_OPT_EXCHANGE_P2P;
      else if (x == "peer") o.exchange_option = LSB_OPT_EXCHANGE_PEER;
      else { fprintf(stderr, "unknown --exchange %s\n", x.c_str()); return 2; }
    }
    else if (a == "--dist") {
      const std::string d = next();
      if (d == "zipf") o.dist = LSB_DIST_ZIPF;
      else if (d == "uniform") o.dist = LSB_DIST_UNIFORM;
      else { fprintf(stderr, "unknown --dist %s\n", d.c_str()); return 2; }
    }
  }
  // MPI: verify iff n < 128Mi (mpi/mpi_lsbsort.cpp:609-611); SHMEM: always (:479)
  if (!o.verify_set) o.verify = o.shmem || (o.n < 128LL * 1024 * 1024);
  if (o.radix_bits == 0) o.radix_bits = o.gpus > 1 ? 16 : 8;
  if (o.n < 0 || o.ranks < 1 || o.gpus < 0 || o.share_gpus < 0 || o.hybrid < 0 || o.hybrid > 2) {
    fprintf(stderr, "invalid arguments\n");
    return 2;
  }

  if (o.gpus >= 1) {
    // One process per GPU.  Fork every rank before anything touches HIP;
    // rank 0 sends the RCCL unique id to the others through pipes.
    std::vector<int> rd(o.gpus, -1), wr(o.gpus, -1);
    for (int r = 1; r < o.gpus; ++r) {
      int fds[2];
      if (pipe(fds) != 0) {
        perror("pipe");
        return 2;
      }
      rd[r] = fds[0];
      wr[r] = fds[1];
    }
    // Report pipes (verify failure only): rank q > 0 -> the root.
    std::vector<int> rep_rd(o.gpus, -1), rep_wr(o.gpus, -1);
    for (int r = 1; r < o.gpus; ++r) {
      int fds[2];
      if (pipe(fds) != 0) {
        perror("pipe");
        return 2;
      }
      rep_rd[r] = fds[0];
      rep_wr[r] = fds[1];
    }
    std::vector<pid_t> kids;
    for (int r = 0; r < o.gpus; ++r) {
      pid_t pid = fork();
      if (pid < 0) {
        perror("fork");
        return 2;
      }
      if (pid == 0) {
        std::vector<int> mine;
        if (r == 0)
          for (int q = 1; q < o.gpus; ++q) mine.push_back(wr[q]);
        // Keep only my ends of the report pipes, so the root sees EOF from a
        // rank that died instead of waiting on it.
        std::vector<int> rep(o.gpus, -1);
        for (int q = 1; q < o.gpus; ++q) {
          if (r == 0) rep[q] = rep_rd[q];
          else close(rep_rd[q]);
          if (q == r) rep[q] = rep_wr[q];
          else close(rep_wr[q]);
        }
        const int st = run_rank_process(o, r, rd[r], mine, rep);
        fflush(stdout);
        _exit(st);
      }
      kids.push_back(pid);
    }
    for (int q = 1; q < o.gpus; ++q) {
      close(rep_rd[q]);
      close(rep_wr[q]);
    }
    int worst = 0;
    for (pid_t pid : kids) {
      int st = 0;
      int code = 2;
      if (waitpid(pid, &st, 0) >= 0) {
        if (WIFEXITED(st)) code = WEXITSTATUS(st);
        else if (WIFSIGNALED(st)) code = 128 + WTERMSIG(st);  // e.g. 134: a rank's assert
      }
      worst = code > worst ? code : worst;
    }
    return worst;
  }

  World w;
  w.P = o.ranks;
  w.n = o.n;
  w.per = lsb_per_rank(o.n, o.ranks);
  w.first = 0;
  w.nlocal = o.ranks;
  w.dev = o.device;
  std::vector<int> devs(o.ranks, o.device);
  CHECK(lsb_create(&w.ctx, o.n, o.ranks, devs.data(), o.radix_bits));
  const int status = run(w, o);
  lsb_destroy(w.ctx);
  return status;
}
