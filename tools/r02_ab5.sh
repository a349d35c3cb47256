#!/bin/bash
# Skewed write-out next-digit adds, Zipf and uniform keys at P = 1:
#   base = HEAD, z0 = run heads by DPP (add_slot_runs), z3 = lane 0's slot
#   counted by one ballot + one add, other lanes plain adds.
# Then the direct 65536-bucket write ceiling (tools/kbench/scatter16, C5).
set -euo pipefail
O=gpurun_out/ab5
mkdir -p $O
LSB_DIST=zipf AB_LOG=$O/zipf.log ROUNDS=5 bash tools/ab.sh abtest/base/liblsb.so abtest/z0/liblsb.so abtest/z3/liblsb.so
AB_LOG=$O/uniform.log ROUNDS=3 bash tools/ab.sh abtest/base/liblsb.so abtest/z3/liblsb.so
for f in zipf uniform; do echo "== $f"; python tools/ab_summary.py $O/$f.log; done
timeout -k 10 300 tools/kbench/scatter16 30 > $O/scatter16.log 2>&1
cat $O/scatter16.log
