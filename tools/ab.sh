#!/bin/bash
# A/B timing of several builds of liblsb.so on one GPU box, interleaved so
# that clock/thermal drift hits every build alike:
#   ROUNDS=3 LG=30 bash tools/ab.sh abtest/a.so abtest/b/liblsb.so ...
# Appends to gpurun_out/ab.log; summarise with tools/ab_summary.py.
set -euo pipefail
LG=${LG:-30}; R=${ROUNDS:-3}
mkdir -p gpurun_out
for i in $(seq 1 $R); do
  for lib in "$@"; do
    echo "lib=$lib" >> gpurun_out/ab.log
    LSB_LIBRARY=$lib timeout -k 10 120 python tools/digit_probe.py $LG >> gpurun_out/ab.log 2>&1
  done
done
