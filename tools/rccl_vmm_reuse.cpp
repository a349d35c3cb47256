// Pure-RCCL check of VMM buffers at reused addresses (no liblsb): the round-6
// wrong answer of test_world_of_one_large_calls[28-8-1] came from world-of-one
// RCCL contexts whose record buffers (HIP VMM: reserved address range, 1 GiB
// physical pieces) were mapped at addresses an earlier context's released
// buffers had used (profiles/r06/large_call/).  This program
// does what those contexts did, with RCCL alone: per iteration a fresh
// world-of-one communicator, a send and a receive buffer of S GiB built from
// 1 GiB pieces, D decoy buffers allocated and released first (the placement
// probe's losing candidates), then R rounds of ncclAllToAllv of the whole
// buffer to the rank itself, cut into 1 GiB calls (coll_alltoallv_u64), each
// checked on the device; then everything released.  One JSON line per
// iteration with the buffers' addresses and the wrong u64 count.
//
//   tools/rccl_vmm_reuse ITERS SIZE_GIB DECOYS ROUNDS [malloc|swap|late|chain|vmm] [rccl|memcpy|kernel] [nofill|nomemset]
//   (swap: odd iterations back the reused ranges with other physical pieces;
//    late: decoys written, released, then the receive buffer allocated;
//    chain: the placement probe's candidates, each written, checked and
//    released before the next is mapped)
//
// Build: hipcc --offload-arch=gfx950 -O2 tools/rccl_vmm_reuse.cpp -lrccl (tools/rccl_vmm_reuse.sh).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace {

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
      exit(2);                                                                 \
    }                                                                          \
  } while (0)
#define CN(x)                                                                  \
  do {                                                                         \
    ncclResult_t r_ = (x);                                                     \
    if (r_ != ncclSuccess) {                                                   \
      fprintf(stderr, "%s: %s\n", #x, ncclGetErrorString(r_));                 \
      exit(3);                                                                 \
    }                                                                          \
  } while (0)

constexpr size_t kPiece = size_t(1) << 30;

__host__ __device__ inline uint64_t value_of(uint64_t it, uint64_t round, uint64_t i) {
  uint64_t x = (it << 56) ^ (round << 48) ^ i;
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  return x;
}

__global__ void k_fill(uint64_t* p, uint64_t n, uint64_t it, uint64_t round) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = value_of(it, round, i);
}

__global__ void k_check(const uint64_t* p, uint64_t n, uint64_t it, uint64_t round, unsigned long long* bad) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    if (p[i] != value_of(it, round, i)) atomicAdd(bad, 1ull);
}

__global__ void k_copy(uint64_t* dst, const uint64_t* src, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

struct Buf {
  void* base = nullptr;
  size_t bytes = 0;
  std::vector<hipMemGenericAllocationHandle_t> pieces;
  bool vmm = true;
};

Buf reserve_buf(size_t bytes, bool vmm) {
  Buf b;
  b.bytes = bytes;
  b.vmm = vmm;
  if (!vmm) {
    CK(hipMalloc(&b.base, bytes));
    return b;
  }
  CK(hipMemAddressReserve(&b.base, bytes, kPiece, nullptr, 0));
  return b;
}

hipMemGenericAllocationHandle_t make_piece() {
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  hipMemGenericAllocationHandle_t h;
  CK(hipMemCreate(&h, kPiece, &prop, 0));
  return h;
}

void back_buf(Buf& b) {  // physical pieces for a reserved range, mapped in order
  if (!b.vmm) return;
  for (size_t off = 0; off < b.bytes; off += kPiece) {
    hipMemGenericAllocationHandle_t h = make_piece();
    CK(hipMemMap(static_cast<char*>(b.base) + off, kPiece, 0, h, 0));
    b.pieces.push_back(h);
  }
  hipMemAccessDesc a = {};
  a.location.type = hipMemLocationTypeDevice;
  a.location.id = 0;
  a.flags = hipMemAccessFlagsProtReadWrite;
  CK(hipMemSetAccess(b.base, b.bytes, &a, 1));
}

Buf alloc_buf(size_t bytes, bool vmm) {
  Buf b = reserve_buf(bytes, vmm);
  back_buf(b);
  return b;
}

void free_buf(Buf& b) {
  CK(hipDeviceSynchronize());
  if (!b.vmm) {
    CK(hipFree(b.base));
  } else {
    for (size_t k = 0; k < b.pieces.size(); ++k) CK(hipMemUnmap(static_cast<char*>(b.base) + k * kPiece, kPiece));
    for (auto h : b.pieces) CK(hipMemRelease(h));
    CK(hipMemAddressFree(b.base, b.bytes));
  }
  b = Buf();
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: %s ITERS SIZE_GIB DECOYS ROUNDS [malloc|swap|late|chain|vmm] [rccl|memcpy|kernel] [nofill|nomemset]\n", argv[0]);
    return 1;
  }
  const int iters = atoi(argv[1]), decoys = atoi(argv[3]), rounds = atoi(argv[4]);
  const size_t bytes = (size_t)atoi(argv[2]) * kPiece;
  const bool vmm = !(argc > 5 && !strcmp(argv[5], "malloc"));
  const bool swap = argc > 5 && !strcmp(argv[5], "swap");
  const bool late = argc > 5 && !strcmp(argv[5], "late");
  const bool chain = argc > 5 && !strcmp(argv[5], "chain");
  const bool nomemset = argc > 7 && !strcmp(argv[7], "nomemset");  // chain: no hipMemsetAsync of a candidate
  // transport (argv[6]): rccl (default) | memcpy (hipMemcpyAsync) | kernel (a copy kernel)
  const bool nofill = argc > 7 && !strcmp(argv[7], "nofill");  // late: decoys never written
  const int transport = argc > 6 ? (!strcmp(argv[6], "memcpy") ? 1 : !strcmp(argv[6], "kernel") ? 2 : 0) : 0;
  const uint64_t n = bytes / 8, call = kPiece / 8;  // u64 in all, per call
  CK(hipSetDevice(0));
  int version = 0;
  (void)ncclGetVersion(&version);
  printf("{\"rccl_version\": %d, \"gib\": %zu, \"decoys\": %d, \"rounds\": %d, \"vmm\": %s, \"swap\": %s, \"late\": %s, \"transport\": %d, \"nofill\": %s}\n", version,
         bytes >> 30, decoys, rounds, vmm ? "true" : "false", swap ? "true" : "false", late ? "true" : "false", transport, nofill ? "true" : "false");
  fflush(stdout);
  unsigned long long* bad = nullptr;
  CK(hipMalloc(&bad, sizeof(unsigned long long)));
  int worst = 0;
  for (int it = 0; it < iters; ++it) {
    ncclUniqueId id;
    CN(ncclGetUniqueId(&id));
    ncclComm_t comm;
    CN(ncclCommInitRank(&comm, 1, id, 0));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    if (chain) {
      // The placement probe's pattern (lsb_alloc.cpp Chain / alloc_third):
      // candidate k is mapped, written (copy of the send buffer), checked and
      // released, and candidate k + 1 is mapped at once -- DECOYS + 1 times.
      Buf src = alloc_buf(bytes, vmm);
      unsigned long long wrong = 0;
      void* first = nullptr;
      int same = 0;
      for (int k = 0; k <= decoys; ++k) {
        Buf cand = alloc_buf(bytes, vmm);
        if (k == 0) first = cand.base;
        else same += cand.base == first;
        k_fill<<<4096, 256, 0, s>>>(static_cast<uint64_t*>(src.base), n, it, k);
        if (!nomemset) CK(hipMemsetAsync(cand.base, 0, bytes, s));  // the probe never clears a candidate
        k_copy<<<4096, 256, 0, s>>>(static_cast<uint64_t*>(cand.base), static_cast<const uint64_t*>(src.base), n);
        CK(hipMemsetAsync(bad, 0, sizeof(unsigned long long), s));
        k_check<<<4096, 256, 0, s>>>(static_cast<const uint64_t*>(cand.base), n, it, k, bad);
        unsigned long long h = 0;
        CK(hipMemcpyAsync(&h, bad, sizeof h, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        wrong += h;
        free_buf(cand);
      }
      printf("{\"iter\": %d, \"chain\": %d, \"same_address\": %d, \"wrong_u64\": %llu}\n", it, decoys + 1, same, wrong);
      fflush(stdout);
      if (wrong) worst = 1;
      free_buf(src);
      CK(hipStreamDestroy(s));
      CN(ncclCommDestroy(comm));
      continue;
    }
    std::vector<Buf> decoy;
    for (int d = 0; d < decoys; ++d) decoy.push_back(alloc_buf(bytes, vmm));
    // swap: on odd iterations the ranges are backed in the other order, after
    // a held spacer piece, so a reused address range gets other physical
    // memory than it had (as when the placement probe picks another candidate).
    Buf snd, rcv;
    std::vector<hipMemGenericAllocationHandle_t> spacer;
    if (late) {
      // liblsb's order: the probe's candidates (the send buffer among them)
      // are written by timed passes, the losers released, and the receive
      // buffer is allocated at the first exchange, onto a released range.
      snd = alloc_buf(bytes, vmm);
      if (!nofill)
        for (Buf& d : decoy) k_fill<<<4096, 256, 0, s>>>(static_cast<uint64_t*>(d.base), n, it, 99);
      CK(hipStreamSynchronize(s));
      for (Buf& d : decoy) free_buf(d);
      decoy.clear();
      rcv = alloc_buf(bytes, vmm);
    } else if (swap && vmm && (it & 1)) {
      snd = reserve_buf(bytes, vmm);
      rcv = reserve_buf(bytes, vmm);
      spacer.push_back(make_piece());
      back_buf(rcv);
      back_buf(snd);
    } else {
      snd = reserve_buf(bytes, vmm);
      rcv = reserve_buf(bytes, vmm);
      back_buf(snd);
      back_buf(rcv);
    }
    for (Buf& d : decoy) free_buf(d);
    unsigned long long wrong = 0;
    for (int r = 0; r < rounds; ++r) {
      k_fill<<<4096, 256, 0, s>>>(static_cast<uint64_t*>(snd.base), n, it, r);
      CK(hipMemsetAsync(rcv.base, 0, bytes, s));
      for (uint64_t off = 0; off < n; off += call) {  // calls of at most 1 GiB, as the runtime cuts them
        size_t cnt = n - off < call ? n - off : call, zero = 0;
        uint64_t* src = static_cast<uint64_t*>(snd.base) + off;
        uint64_t* dst = static_cast<uint64_t*>(rcv.base) + off;
        if (transport == 1) {
          CK(hipMemcpyAsync(dst, src, cnt * 8, hipMemcpyDeviceToDevice, s));
        } else if (transport == 2) {
          k_copy<<<4096, 256, 0, s>>>(dst, src, cnt);
        } else {
          CN(ncclAllToAllv(src, &cnt, &zero, dst, &cnt, &zero, ncclUint64, comm, s));
        }
      }
      CK(hipMemsetAsync(bad, 0, sizeof(unsigned long long), s));
      k_check<<<4096, 256, 0, s>>>(static_cast<const uint64_t*>(rcv.base), n, it, r, bad);
      unsigned long long h = 0;
      CK(hipMemcpyAsync(&h, bad, sizeof h, hipMemcpyDeviceToHost, s));
      CK(hipStreamSynchronize(s));
      wrong += h;
    }
    printf("{\"iter\": %d, \"send\": \"%p\", \"recv\": \"%p\", \"wrong_u64\": %llu}\n", it, snd.base, rcv.base, wrong);
    fflush(stdout);
    if (wrong) worst = 1;
    free_buf(snd);
    free_buf(rcv);
    for (auto h : spacer) CK(hipMemRelease(h));
    CK(hipStreamDestroy(s));
    CN(ncclCommDestroy(comm));
  }
  CK(hipFree(bad));
  return worst;
}
