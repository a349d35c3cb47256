#!/bin/bash
# k_onesweep at 512 threads (8 waves x 8 records) for the whole stage, the
# split stage kept at 256 x 16 ("mix"), against the shipped 256 x 16 ("base"):
# uniform, Zipf (split stage), and the 16-bit exchange path at P = 1 (the
# C16 counting pass and k_place's next-digit counts).
set -euo pipefail
O=gpurun_out/ab27
mkdir -p $O
rm -f $O/*.log
LSB_LIBRARY=abtest/base/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 > /dev/null 2>&1
run() { echo "lib=$1" >> $O/$2.log; LSB_LIBRARY=abtest/$1/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 >> $O/$2.log 2>&1; }
for i in 1 2 3 4 5 6; do
  if [ $((i % 2)) = 1 ]; then for v in base mix; do run $v uniform; done
  else for v in mix base; do run $v uniform; done; fi
done
for i in 1 2 3 4; do for v in base mix; do LSB_DIST=zipf run $v zipf; done; done
for i in 1 2 3; do for v in base mix; do LSB_FORCE_EXCHANGE=1 LSB_RADIX_BITS=16 run $v x16; done; done
for f in uniform zipf x16; do echo "== $f"; python tools/ab_summary.py $O/$f.log; grep -c "verify=(True" $O/$f.log || true; done
