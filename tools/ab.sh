#!/bin/bash
# A/B timing of several builds of liblsb.so on one GPU box, interleaved so
# that clock/thermal drift hits every build alike:
#   ROUNDS=3 LG=30 bash tools/ab.sh abtest/a.so abtest/b/liblsb.so ...
# Appends to ${AB_LOG:-gpurun_out/ab.log}; summarise with tools/ab_summary.py.
# LSB_DIST=zipf times Zipf keys (tools/digit_probe.py).
set -euo pipefail
LG=${LG:-30}; R=${ROUNDS:-3}; LOG=${AB_LOG:-gpurun_out/ab.log}
mkdir -p gpurun_out
for i in $(seq 1 $R); do
  for lib in "$@"; do
    echo "lib=$lib" >> $LOG
    LSB_LIBRARY=$lib timeout -k 10 120 python tools/digit_probe.py $LG >> $LOG 2>&1
  done
done
