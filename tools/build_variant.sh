#!/bin/bash
# Build liblsb.so with extra compile flags into its own directory, for A/B
# runs (tools/ab.sh) and profiling builds:
#   bash tools/build_variant.sh abtest/prof -DLSB_OS_PROFILE
set -euo pipefail
out=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$out"
H=/opt/rocm/bin/hipcc
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$R/include -I$R/distributed-lsb_amd/csrc $*"
objs=()
for src in "$R"/distributed-lsb_amd/csrc/*.hip "$R"/distributed-lsb_amd/csrc/*.cpp; do
  o="$out/$(basename "${src%.*}").o"
  $H $F -c "$src" -o "$o" &
  objs+=("$o")
done
wait
$H --offload-arch=gfx950 -shared -o "$out/liblsb.so" "${objs[@]}" -L/opt/rocm/lib -lrccl \
  -Wl,-rpath,/opt/rocm/lib
