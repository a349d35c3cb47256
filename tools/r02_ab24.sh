#!/bin/bash
# Bounded tile-load window (LSB_LOAD_WINDOW = 4 / 8 / 12 loads in flight per
# wave, s_waitcnt before each further load) against all IPT loads at once
# (w0 = the shipped kernel).  Uniform keys, then Zipf.
set -euo pipefail
O=gpurun_out/ab24
mkdir -p $O
rm -f $O/*.log
LSB_LIBRARY=abtest/w0/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 > /dev/null 2>&1
run() { echo "lib=$1" >> $O/$2.log; LSB_LIBRARY=abtest/$1/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 >> $O/$2.log 2>&1; }
for i in 1 2 3 4 5; do
  if [ $((i % 2)) = 1 ]; then for v in w0 w4 w8 w12; do run $v uniform; done
  else for v in w12 w8 w4 w0; do run $v uniform; done; fi
done
python tools/ab_summary.py $O/uniform.log
grep -c "verify=(True" $O/uniform.log || true
for i in 1 2; do for v in w0 w4 w8; do LSB_DIST=zipf run $v zipf; done; done
python tools/ab_summary.py $O/zipf.log
