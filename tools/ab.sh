#!/bin/bash
# A/B timing of two builds of liblsb.so on one GPU box, interleaved:
#   bash tools/ab.sh abtest/liblsb_old.so abtest/liblsb_new.so [log2 n] [rounds]
set -euo pipefail
A=$1; B=$2; LG=${3:-30}; R=${4:-3}
mkdir -p gpurun_out
for i in $(seq 1 $R); do
  for lib in $A $B; do
    echo "lib=$lib" >> gpurun_out/ab.log
    LSB_LIBRARY=$lib timeout -k 10 120 python tools/digit_probe.py $LG >> gpurun_out/ab.log 2>&1
  done
done
