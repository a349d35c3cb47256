#!/bin/bash
# Build liblsb.so from the library sources as they are at git revision REV
# (the A side of an A/B run against the working tree), plus optional extra
# compile flags:
#   bash tools/build_at.sh HEAD abtest/base [-DFLAG ...]
# Output: OUT/liblsb.so (OUT/src holds the exported sources).
set -euo pipefail
rev=$1; out=$2; shift 2
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$out/src/distributed-lsb_amd/csrc" "$out/src/include"
for f in distributed-lsb_amd/csrc/lsb_kernels.hip distributed-lsb_amd/csrc/lsb_merge.hip \
         distributed-lsb_amd/csrc/lsb_segsort.hip \
         distributed-lsb_amd/csrc/lsb_runtime.cpp distributed-lsb_amd/csrc/lsb_kernels.h distributed-lsb_amd/csrc/lsb_device.h include/lsb.h; do
  git -C "$R" show "$rev:$f" > "$out/src/$f" 2>/dev/null || rm -f "$out/src/$f"  # older revisions lack some
done
S=$out/src
H=/opt/rocm/bin/hipcc
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$S/include -I$S/distributed-lsb_amd/csrc $*"
$H $F -c "$S/distributed-lsb_amd/csrc/lsb_kernels.hip" -o "$out/k.o"
$H $F -c "$S/distributed-lsb_amd/csrc/lsb_merge.hip" -o "$out/m.o"
objs=("$out/k.o" "$out/m.o")
if [ -f "$S/distributed-lsb_amd/csrc/lsb_segsort.hip" ]; then
  $H $F -c "$S/distributed-lsb_amd/csrc/lsb_segsort.hip" -o "$out/s.o"
  objs+=("$out/s.o")
fi
$H $F -c "$S/distributed-lsb_amd/csrc/lsb_runtime.cpp" -o "$out/r.o"
$H --offload-arch=gfx950 -shared -o "$out/liblsb.so" "${objs[@]}" "$out/r.o" -L/opt/rocm/lib -lrccl \
  -Wl,-rpath,/opt/rocm/lib
