// Device helpers shared by the kernels of lsb_kernels.hip and lsb_segsort.hip.
#pragma once
#include "lsb_kernels.h"

namespace lsb {

// k_onesweep's look-back granules: bits 0-29 the value (a bucket's count
// within one sub-array), bit 30 the prefix flag, bit 31 the epoch parity.
constexpr uint32_t kStatusValMask = (1u << 30) - 1u;

// The k_onesweep sub-arrays: sub-array x holds tiles [x * TT / 8, (x + 1) * TT / 8).
__device__ __forceinline__ int64_t sub_first_tile(int x, int64_t TT) { return (int64_t)x * TT / kOnesweepSubs; }
// Sub-array of tile t without a division: the number of x in 1..kSub-1
// with x * TT <= kSub * t + kSub - 1, i.e. floor(x * TT / kSub) <= t
// (32-bit exact: TT < 2^22, see kOnesweepMaxElems).
__device__ __forceinline__ int sub_of_tile(int64_t t, int64_t TT) {
  const uint32_t num = (uint32_t)kOnesweepSubs * (uint32_t)t + (uint32_t)(kOnesweepSubs - 1), tt = (uint32_t)TT;
  int x = 0;
#pragma unroll
  for (int k = 1; k < kOnesweepSubs; ++k) x += num >= (uint32_t)k * tt ? 1 : 0;
  return x;
}

}  // namespace lsb
