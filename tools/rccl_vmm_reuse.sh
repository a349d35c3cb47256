#!/bin/bash
# Builds tools/rccl_vmm_reuse (pure RCCL, no liblsb) and runs it: 6
# world-of-one iterations of 4 GiB send / receive buffers from 1 GiB VMM
# pieces, 8 rounds of ncclAllToAllv to self each.  Default (round 6, first
# run): with 2 decoy buffers released first (as the placement probe's
# losers), without decoys, and with hipMalloc'd buffers.  MODE=swap: odd
# iterations back the reused ranges with other physical pieces, with 0 and 2
# decoys.  MODE=late: the decoys written and released, then the receive
# buffer allocated (liblsb's order), with 2 and 3 decoys.  MODE=transport:
# late with hipMemcpyAsync, a copy kernel, RCCL without local registration,
# and hipMalloc'd buffers.  MODE=nofill: late with decoys never written (copy
# kernel, RCCL), and the written case again.  MODE=chain: the placement
# probe's pattern (4 and 8 candidates), and late with a copy kernel again.
# MODE=chain_nomemset: 8 candidates without and with the hipMemsetAsync.  Stops at the first run that ends other than 0 (right) or 1 (wrong).
#   tools/rccl_vmm_reuse.sh OUT_DIR [build]
set -uo pipefail
cd "$(dirname "$0")/.."
O=${1:-gpurun_out/rccl_vmm_reuse}
mkdir -p "$O"
if [ "${2:-}" = build ] || [ ! -x tools/rccl_vmm_reuse ]; then
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/rccl_vmm_reuse.cpp -o tools/rccl_vmm_reuse \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib || exit 1
fi
[ "${2:-}" = build ] && exit 0
run() {  # NAME ARGS...
  local name=$1; shift
  timeout -k 10 300 tools/rccl_vmm_reuse "$@" > "$O/$name.jsonl" 2> "$O/$name.err"
  local rc=$?
  cat "$O/$name.jsonl"
  echo "{\"run\": \"$name\", \"rc\": $rc}"
  [ $rc -le 1 ]
}
if [ "${MODE:-}" = chain_nomemset ]; then
  run chain8_nomemset 4 4 7 1 chain kernel nomemset && run chain8_memset 4 4 7 1 chain kernel memset
elif [ "${MODE:-}" = chain ]; then
  run chain4 4 4 3 1 chain && run chain8 4 4 7 1 chain && run late_kernel_again 4 4 2 8 late kernel
elif [ "${MODE:-}" = nofill ]; then
  run late_kernel_nofill 4 4 2 8 late kernel nofill && run late_rccl_nofill 4 4 2 8 late rccl nofill &&
    run late_kernel_fill 4 4 2 8 late kernel fill
elif [ "${MODE:-}" = transport ]; then
  run late_memcpy 4 4 2 8 late memcpy && run late_kernel 4 4 2 8 late kernel &&
    NCCL_LOCAL_REGISTER=0 run late_noreg 4 4 2 8 late rccl && run late_malloc 4 4 2 8 malloc rccl
elif [ "${MODE:-}" = late ]; then
  run late_decoys2 6 4 2 8 late && run late_decoys3 6 4 3 8 late
elif [ "${MODE:-}" = swap ]; then
  run swap_plain 6 4 0 8 swap && run swap_decoys 6 4 2 8 swap
else
  run vmm_decoys 6 4 2 8 && run vmm_plain 6 4 0 8 && run malloc 6 4 2 8 malloc
fi
