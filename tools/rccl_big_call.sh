#!/bin/bash
# Builds tools/rccl_big_call (pure RCCL, no liblsb) and runs it at world 1 and
# world 2 (two processes on the one GPU, RCCL's socket transport) for 1, 2
# and 4 GiB per peer in one call, ncclAllToAllv and grouped send/recv.
#   tools/rccl_big_call.sh OUT_DIR [build]
set -euo pipefail
cd "$(dirname "$0")/.."
O=${1:-gpurun_out/rccl_big}
mkdir -p "$O"
if [ "${2:-}" = build ] || [ ! -x tools/rccl_big_call ]; then
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/rccl_big_call.cpp -o tools/rccl_big_call \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
fi
[ "${2:-}" = build ] && exit 0
timeout -k 10 240 tools/rccl_big_call 1 both 512 1024 2048 4096 > "$O/world1.jsonl"
timeout -k 10 300 tools/rccl_big_call 2 both 512 1024 2048 4096 > "$O/world2.jsonl"
cat "$O"/world1.jsonl "$O"/world2.jsonl
