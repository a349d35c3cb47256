// Pure-RCCL check of large per-peer ranges: no liblsb.
//
// The runtime cuts every RCCL call at 1 GiB per peer (lsb_context.cpp,
// coll_alltoallv_u64) because a world-of-one exchange of 2 GiB or more in one
// call came back wrong (profiles/r05/x16dbg_probe.log).  This program asks
// RCCL alone: W ranks (one process each, forked before any HIP call; on one
// GPU each rank gets its own NCCL_HOSTID, so RCCL links them by its socket
// transport) exchange S bytes with every peer, itself included, in ONE call:
// ncclAllToAllv, or grouped ncclSend / ncclRecv.  Every u64 carries a value
// derived from (source, destination, index); the receiver counts mismatches on
// the device and reports the first.  One JSON line per (form, size) from
// rank 0, with ncclGetVersion.
//
//   tools/rccl_big_call WORLD FORM SIZE_MIB...     FORM: a2a | p2p | both
//
// Build: hipcc --offload-arch=gfx950 -O2 tools/rccl_big_call.cpp -lrccl (tools/rccl_big_call.sh).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <sys/wait.h>
#include <unistd.h>

#include <array>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace {

__host__ __device__ inline uint64_t value_of(uint64_t src, uint64_t dst, uint64_t i) {
  uint64_t x = (src << 56) ^ (dst << 48) ^ i;
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  return x;
}

// seg[i] = value_of(src, dst, i) for the segment this rank sends to dst.
__global__ void k_fill(uint64_t* seg, uint64_t n, uint64_t src, uint64_t dst) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    seg[i] = value_of(src, dst, i);
}

// Mismatches of a received segment from src (bad[0]: count, bad[1]: first index + 1, min).
__global__ void k_check(const uint64_t* seg, uint64_t n, uint64_t src, uint64_t dst,
                        unsigned long long* bad) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    if (seg[i] != value_of(src, dst, i)) {
      atomicAdd(&bad[0], 1ull);
      atomicMin(&bad[1], (unsigned long long)(i + 1));
    }
}

#define CHECK_HIP(x)                                                              \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "rank %d: %s: %s\n", rank, #x, hipGetErrorString(e_));       \
      return 2;                                                                   \
    }                                                                             \
  } while (0)
#define CHECK_NCCL(x)                                                             \
  do {                                                                            \
    ncclResult_t r_ = (x);                                                        \
    if (r_ != ncclSuccess) {                                                      \
      fprintf(stderr, "rank %d: %s: %s\n", rank, #x, ncclGetErrorString(r_));      \
      return 3;                                                                   \
    }                                                                             \
  } while (0)

int run_rank(int rank, int world, const ncclUniqueId& id, const std::vector<std::string>& forms,
             const std::vector<size_t>& mib, int out_fd) {
  CHECK_HIP(hipSetDevice(0));
  ncclComm_t comm;
  CHECK_NCCL(ncclCommInitRank(&comm, world, id, rank));
  hipStream_t s;
  CHECK_HIP(hipStreamCreate(&s));
  unsigned long long* bad = nullptr;
  CHECK_HIP(hipMalloc(&bad, 2 * sizeof(unsigned long long)));
  for (size_t m : mib) {
    const uint64_t n = (uint64_t)(m << 20) / 8;  // u64 per peer
    uint64_t *send = nullptr, *recv = nullptr;
    CHECK_HIP(hipMalloc(&send, n * 8 * world));
    CHECK_HIP(hipMalloc(&recv, n * 8 * world));
    for (const std::string& form : forms) {
      for (int q = 0; q < world; ++q) k_fill<<<1024, 256, 0, s>>>(send + (size_t)q * n, n, rank, q);
      CHECK_HIP(hipMemsetAsync(recv, 0xab, n * 8 * world, s));
      std::vector<size_t> cnt(world, n), displ(world);
      for (int q = 0; q < world; ++q) displ[q] = (size_t)q * n;
      CHECK_HIP(hipStreamSynchronize(s));
      hipEvent_t e0, e1;
      CHECK_HIP(hipEventCreate(&e0));
      CHECK_HIP(hipEventCreate(&e1));
      CHECK_HIP(hipEventRecord(e0, s));
      if (form == "a2a") {
        CHECK_NCCL(ncclAllToAllv(send, cnt.data(), displ.data(), recv, cnt.data(), displ.data(), ncclUint64, comm, s));
      } else {
        CHECK_NCCL(ncclGroupStart());
        for (int q = 0; q < world; ++q) {
          CHECK_NCCL(ncclSend(send + displ[q], n, ncclUint64, q, comm, s));
          CHECK_NCCL(ncclRecv(recv + displ[q], n, ncclUint64, q, comm, s));
        }
        CHECK_NCCL(ncclGroupEnd());
      }
      CHECK_HIP(hipEventRecord(e1, s));
      const unsigned long long init[2] = {0ull, ~0ull};
      CHECK_HIP(hipMemcpyAsync(bad, init, sizeof init, hipMemcpyHostToDevice, s));
      for (int q = 0; q < world; ++q) k_check<<<1024, 256, 0, s>>>(recv + displ[q], n, q, rank, bad);
      unsigned long long hb[2];
      CHECK_HIP(hipMemcpyAsync(hb, bad, sizeof hb, hipMemcpyDeviceToHost, s));
      CHECK_HIP(hipStreamSynchronize(s));
      float ms = 0.f;
      CHECK_HIP(hipEventElapsedTime(&ms, e0, e1));
      (void)hipEventDestroy(e0);
      (void)hipEventDestroy(e1);
      char line[512];
      const int len = snprintf(line, sizeof line,
                               "{\"rank\": %d, \"world\": %d, \"form\": \"%s\", \"mib_per_peer\": %zu, "
                               "\"bytes_per_peer\": %llu, \"wrong_u64\": %llu, \"first_wrong\": %lld, \"ms\": %.2f}\n",
                               rank, world, form.c_str(), m, (unsigned long long)n * 8, hb[0],
                               hb[0] ? (long long)hb[1] - 1 : -1ll, ms);
      if (write(out_fd, line, (size_t)len) != len) return 4;
    }
    (void)hipFree(send);
    (void)hipFree(recv);
  }
  (void)ncclCommDestroy(comm);
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: %s WORLD a2a|p2p|both SIZE_MIB...\n", argv[0]);
    return 1;
  }
  const int world = atoi(argv[1]);
  std::vector<std::string> forms;
  if (!strcmp(argv[2], "both")) forms = {"a2a", "p2p"};
  else forms = {argv[2]};
  std::vector<size_t> mib;
  for (int i = 3; i < argc; ++i) mib.push_back((size_t)atoll(argv[i]));
  // No RCCL or HIP call in the parent (ncclGetUniqueId initialises the
  // runtime, and a forked child of an initialised parent cannot use the
  // GPU): rank 0 makes the id and hands it to the others through pipes.
  int fds[2];
  if (pipe(fds) != 0) return 1;
  std::vector<std::array<int, 2>> idp(world);
  for (auto& p : idp)
    if (pipe(p.data()) != 0) return 1;
  std::vector<pid_t> kids;
  for (int r = 0; r < world; ++r) {
    const pid_t p = fork();
    if (p == 0) {
      close(fds[0]);
      char host[64];
      snprintf(host, sizeof host, "rccl-big-call-%d", r);
      setenv("NCCL_HOSTID", host, 1);
      setenv("NCCL_SOCKET_IFNAME", "lo", 0);
      setenv("NCCL_IB_DISABLE", "1", 0);
      ncclUniqueId id;
      if (r == 0) {
        if (ncclGetUniqueId(&id) != ncclSuccess) _exit(5);
        for (int q = 1; q < world; ++q)
          if (write(idp[q][1], &id, sizeof id) != (ssize_t)sizeof id) _exit(5);
      } else if (read(idp[r][0], &id, sizeof id) != (ssize_t)sizeof id) {
        _exit(5);
      }
      if (r == 0) {
        int version = 0;
        (void)ncclGetVersion(&version);
        char line[128];
        const int len = snprintf(line, sizeof line, "{\"rccl_version\": %d, \"world\": %d}\n", version, world);
        if (write(fds[1], line, (size_t)len) != len) _exit(4);
      }
      const int rank = r;
      const int rc = run_rank(rank, world, id, forms, mib, fds[1]);
      _exit(rc);
    }
    kids.push_back(p);
  }
  close(fds[1]);
  char buf[4096];
  ssize_t k;
  while ((k = read(fds[0], buf, sizeof buf)) > 0) fwrite(buf, 1, (size_t)k, stdout);
  int worst = 0;
  for (pid_t p : kids) {
    int st = 0;
    waitpid(p, &st, 0);
    const int rc = WIFEXITED(st) ? WEXITSTATUS(st) : 128;
    if (rc > worst) worst = rc;
  }
  return worst;
}
