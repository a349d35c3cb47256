#!/bin/bash
# Builds tools/rccl_vmm_reuse (pure RCCL, no liblsb) and runs it: 6
# world-of-one iterations of 4 GiB send / receive buffers from 1 GiB VMM
# pieces, 8 rounds of ncclAllToAllv to self each, with 2 decoy buffers
# released first (as the placement probe's losers), without decoys, and with
# hipMalloc'd buffers.
#   tools/rccl_vmm_reuse.sh OUT_DIR [build]
set -euo pipefail
cd "$(dirname "$0")/.."
O=${1:-gpurun_out/rccl_vmm_reuse}
mkdir -p "$O"
if [ "${2:-}" = build ] || [ ! -x tools/rccl_vmm_reuse ]; then
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/rccl_vmm_reuse.cpp -o tools/rccl_vmm_reuse \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
fi
[ "${2:-}" = build ] && exit 0
timeout -k 10 300 tools/rccl_vmm_reuse 6 4 2 8 > "$O/vmm_decoys.jsonl" 2> "$O/vmm_decoys.err" || true
cat "$O/vmm_decoys.jsonl"
timeout -k 10 300 tools/rccl_vmm_reuse 6 4 0 8 > "$O/vmm_plain.jsonl" 2> "$O/vmm_plain.err" || true
cat "$O/vmm_plain.jsonl"
timeout -k 10 300 tools/rccl_vmm_reuse 6 4 2 8 malloc > "$O/malloc.jsonl" 2> "$O/malloc.err" || true
cat "$O/malloc.jsonl"
