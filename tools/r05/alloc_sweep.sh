#!/bin/bash
# record buffers from VMM pieces vs hipMalloc, with the
# real sort (tools/alloc_probe.py: one context per fresh process, 3 sorts,
# per-pass k_onesweep ms) and the kbench copy at other piece sizes.
set -e
out=gpurun_out/r05_alloc
mkdir -p $out
kb() {  # name mode chunk_mib
  timeout -k 10 120 tools/kbench/vmmbw $2 4 30 5 $3 > $out/kb_$1.log 2>&1
  grep SUMMARY $out/kb_$1.log
}
ap() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python3 tools/alloc_probe.py 30 1 3 > $out/ap_$name.log 2>&1
  echo "$name: $(python3 tools/r05/ap_summary.py $out/ap_$name.log)"
}
for i in 1 2; do kb m2_256_$i 2 256; done
for i in 1 2; do kb m2_4096_$i 2 4096; done
for i in 1 2 3; do ap malloc_$i LSB_RECORD_ALLOC=malloc LSB_PLACEMENT_CANDIDATES=2; done
for i in 1 2 3 4 5; do ap vmm1g_$i LSB_PLACEMENT_CANDIDATES=2; done
for i in 1 2; do ap vmm256_$i LSB_VMM_CHUNK_MIB=256 LSB_PLACEMENT_CANDIDATES=2; done
for i in 1 2; do ap vmm4g_$i LSB_VMM_CHUNK_MIB=4096 LSB_PLACEMENT_CANDIDATES=2; done
