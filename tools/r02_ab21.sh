#!/bin/bash
# Uniform keys, P = 1: the tile shape chosen per sort (big: 8192-record
# tiles for unskewed keys) against HEAD (auto: 4096 staged whole), 10
# rounds with the order alternating.
set -euo pipefail
O=gpurun_out/ab21
mkdir -p $O
rm -f $O/*.log
LSB_LIBRARY=abtest/auto/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 > /dev/null 2>&1
run() { echo "lib=$1" >> $O/uniform.log; LSB_LIBRARY=abtest/$1/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 >> $O/uniform.log 2>&1; }
for i in 1 2 3 4 5 6 7 8 9 10; do
  if [ $((i % 2)) = 1 ]; then run auto; run big; else run big; run auto; fi
done
python tools/ab_summary.py $O/uniform.log
