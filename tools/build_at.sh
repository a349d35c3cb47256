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
git -C "$R" show "$rev:include/lsb.h" > "$out/src/include/lsb.h"
for f in $(git -C "$R" ls-tree --name-only "$rev" distributed-lsb_amd/csrc/); do
  git -C "$R" show "$rev:$f" > "$out/src/$f"
done
S=$out/src
H=/opt/rocm/bin/hipcc
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$S/include -I$S/distributed-lsb_amd/csrc $*"
objs=()
for src in "$S"/distributed-lsb_amd/csrc/*.hip "$S"/distributed-lsb_amd/csrc/*.cpp; do
  o="$out/$(basename "${src%.*}").o"
  $H $F -c "$src" -o "$o" &
  objs+=("$o")
done
wait
$H --offload-arch=gfx950 -shared -o "$out/liblsb.so" "${objs[@]}" -L/opt/rocm/lib -lrccl \
  -Wl,-rpath,/opt/rocm/lib
