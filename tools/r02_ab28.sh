#!/bin/bash
# Zipf keys with the 512-thread whole stage: auto (split stage at 256 x 16),
# the whole stage forced (LSB_SPLIT=1, 512 x 8), and the split stage at
# 512 x 8 (spills).  Interleaved, 2^30 records.
set -euo pipefail
O=gpurun_out/ab28
mkdir -p $O
rm -f $O/*.log
LSB_LIBRARY=abtest/mix/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 > /dev/null 2>&1
run() { echo "lib=$1$3" >> $O/$2.log; LSB_LIBRARY=abtest/$1/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 >> $O/$2.log 2>&1; }
for i in 1 2 3 4; do
  LSB_DIST=zipf run mix zipf ""
  LSB_DIST=zipf LSB_SPLIT=1 run mix zipf "-whole"
  LSB_DIST=zipf run split512 zipf ""
done
python tools/ab_summary.py $O/zipf.log
grep -c "verify=(True" $O/zipf.log || true
