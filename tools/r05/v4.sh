#!/bin/bash
# round 5 check 4: rocprofv3 evidence of the bench, and the DRAM-side /
# per-channel write counters of hipMalloc vs VMM record buffers.
set -u
O=gpurun_out/r05_v4
mkdir -p $O
bash tools/profile.sh > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }
cp $(find gpurun_out/prof/stats -name "*kernel_stats.csv" -print -quit) $O/kernel_stats.csv
TAG=r05_allocpmc2 SETS="dram inst" bash tools/r05/alloc_counters.sh > $O/allocpmc2.log 2>&1 || { tail -20 $O/allocpmc2.log; exit 1; }
cat $O/allocpmc2.log
