#!/bin/bash
# Tile shape chosen per sort (abtest/big = working tree: unskewed keys take
# 8192-record tiles, skewed keys 4096 split) against HEAD (abtest/auto:
# unskewed 4096 whole): GPU suite, then P = 1 uniform / Zipf and the forced
# 16-bit exchange, orders alternating.
set -euo pipefail
O=gpurun_out/ab20
mkdir -p $O
rm -f $O/*.log
timeout -k 10 300 python -u -m pytest tests/test_dist_ops_gpu.py -x -q --timeout 120 --timeout-method thread > $O/gputests_dist.log 2>&1 || { tail -40 $O/gputests_dist.log; exit 1; }
tail -2 $O/gputests_dist.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 \
  || { tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
LSB_LIBRARY=abtest/auto/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 > /dev/null 2>&1
run() { echo "lib=$1" >> $O/$2.log; LSB_LIBRARY=abtest/$1/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 >> $O/$2.log 2>&1; }
for i in 1 2 3 4 5 6; do
  if [ $((i % 2)) = 1 ]; then run auto uniform; run big uniform; else run big uniform; run auto uniform; fi
done
export LSB_DIST=zipf
for i in 1 2 3 4; do
  if [ $((i % 2)) = 1 ]; then run auto zipf; run big zipf; else run big zipf; run auto zipf; fi
done
unset LSB_DIST
export LSB_RADIX_BITS=16 LSB_FORCE_EXCHANGE=1
for i in 1 2 3; do
  if [ $((i % 2)) = 1 ]; then run auto x16; run big x16; else run big x16; run auto x16; fi
done
for f in uniform zipf x16; do echo "== $f"; python tools/ab_summary.py $O/$f.log; done
