#!/bin/bash
# Uniform keys, P = 1: 8192-record tiles through a half stage (t8s) against
# the shipped 4096-record whole stage (auto), 8 rounds, order alternating.
set -euo pipefail
O=gpurun_out/ab19
mkdir -p $O
rm -f $O/*.log
LSB_LIBRARY=abtest/auto/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 > /dev/null 2>&1
run() { echo "lib=$1" >> $O/uniform.log; LSB_LIBRARY=abtest/$1/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 >> $O/uniform.log 2>&1; }
for i in 1 2 3 4 5 6 7 8; do
  if [ $((i % 2)) = 1 ]; then run auto; run t8s; else run t8s; run auto; fi
done
python tools/ab_summary.py $O/uniform.log
