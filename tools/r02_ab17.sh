#!/bin/bash
# 8192-record tiles through a 4096-record (64 KiB) stage in two halves (t8,
# split forced) against the shipped build (auto): one warm-up run, then 5
# rounds with the order alternating, uniform and Zipf keys.
set -euo pipefail
O=gpurun_out/ab17
mkdir -p $O
rm -f $O/*.log
LSB_LIBRARY=abtest/auto/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 > /dev/null 2>&1
run() {  # lib-tag dist
  echo "lib=$1" >> $O/$2.log
  if [ $1 = t8 ]; then
    LSB_DIST=$2 LSB_SPLIT=2 LSB_LIBRARY=abtest/t8/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 >> $O/$2.log 2>&1
  else
    LSB_DIST=$2 LSB_LIBRARY=abtest/auto/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 >> $O/$2.log 2>&1
  fi
}
for dist in uniform zipf; do
  for i in 1 2 3 4 5; do
    if [ $((i % 2)) = 1 ]; then run auto $dist; run t8 $dist; else run t8 $dist; run auto $dist; fi
  done
  echo "== $dist"; python tools/ab_summary.py $O/$dist.log
done
