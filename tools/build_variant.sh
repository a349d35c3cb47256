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
$H $F -c "$R/distributed-lsb_amd/csrc/lsb_kernels.hip" -o "$out/k.o"
$H $F -c "$R/distributed-lsb_amd/csrc/lsb_merge.hip" -o "$out/m.o"
$H $F -c "$R/distributed-lsb_amd/csrc/lsb_segsort.hip" -o "$out/s.o"
$H $F -c "$R/distributed-lsb_amd/csrc/lsb_runtime.cpp" -o "$out/r.o"
$H --offload-arch=gfx950 -shared -o "$out/liblsb.so" "$out/k.o" "$out/m.o" "$out/s.o" "$out/r.o" -L/opt/rocm/lib -lrccl \
  -Wl,-rpath,/opt/rocm/lib
