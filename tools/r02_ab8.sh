#!/bin/bash
# Look-back window: W predecessor rows in flight per round trip (abtest/wW,
# W = 1 is the shipped walk) against HEAD; then the phase profile at W = 4.
set -euo pipefail
O=gpurun_out/ab8
mkdir -p $O
AB_LOG=$O/uniform.log ROUNDS=4 bash tools/ab.sh abtest/base/liblsb.so abtest/w1/liblsb.so abtest/w2/liblsb.so abtest/w4/liblsb.so abtest/w8/liblsb.so
LSB_DIST=zipf AB_LOG=$O/zipf.log ROUNDS=2 bash tools/ab.sh abtest/base/liblsb.so abtest/w2/liblsb.so abtest/w4/liblsb.so abtest/w8/liblsb.so
for f in uniform zipf; do echo "== $f"; python tools/ab_summary.py $O/$f.log; done
LSB_LIBRARY=abtest/prof4/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 > $O/prof4.log 2>&1
cat $O/prof4.log
