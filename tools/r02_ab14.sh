#!/bin/bash
# k_onesweep stage split chosen per sort (auto), forced off (never, LSB_SPLIT=1)
# and on (always, LSB_SPLIT=2) in the working-tree build, against HEAD~ (w1);
# uniform and Zipf keys, interleaved; GPU suite first.
set -euo pipefail
O=gpurun_out/ab14
mkdir -p $O
rm -f $O/*.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 \
  || { tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
for dist in uniform zipf; do
  for i in 1 2 3; do
    echo "lib=w1" >> $O/$dist.log; LSB_DIST=$dist LSB_LIBRARY=abtest/w1/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 >> $O/$dist.log 2>&1
    for sp in auto:0 never:1 always:2; do
      echo "lib=${sp%%:*}" >> $O/$dist.log
      LSB_DIST=$dist LSB_SPLIT=${sp#*:} LSB_LIBRARY=abtest/auto/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 >> $O/$dist.log 2>&1
    done
  done
  echo "== $dist"; python tools/ab_summary.py $O/$dist.log
done
