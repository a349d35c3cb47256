#!/bin/bash
# Exchange forms on one GPU (P logical ranks, device-copy all-to-all) with
# the current build: per-digit (tools/exchange_profile.py) and whole-key
# (tools/merge_profile.py at P = 2 and 8), 2^30 records in all.
set -euo pipefail
O=gpurun_out/loopback
mkdir -p $O
timeout -k 10 600 python -u tools/exchange_profile.py > $O/exchange_profile.log 2>&1
cat $O/exchange_profile.log | cut -c1-200
for P in 2 8; do
  timeout -k 10 300 python -u tools/merge_profile.py --ranks $P --n-per-rank $((1073741824 / P)) > $O/merge_p$P.log 2>&1
  tail -3 $O/merge_p$P.log
done
