#!/bin/bash
# k_onesweep look-back: wave 0 alone polls each predecessor row with 16-byte
# loads (4 buckets per lane, "rowpoll", -DLSB_OS_ROWPOLL) vs 4 waves polling
# 8-byte pairs (HEAD).  Uniform + Zipf + 16-bit exchange at 2^30, then the
# single-read tests on "rowpoll".
set -euo pipefail
O=gpurun_out/ab30
mkdir -p $O
rm -f $O/*.log
LSB_LIBRARY=abtest/base/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 > /dev/null 2>&1
run() { echo "lib=$1" >> $O/$2.log; LSB_LIBRARY=abtest/$1/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 >> $O/$2.log 2>&1; }
for i in 1 2 3 4 5 6; do
  if [ $((i % 2)) = 1 ]; then for v in base rowpoll; do run $v uniform; done
  else for v in rowpoll base; do run $v uniform; done; fi
done
for f in uniform; do echo "== $f"; python tools/ab_summary.py $O/$f.log; grep -c "verify=(True" $O/$f.log || true; done
for i in 1 2 3; do for v in base rowpoll; do LSB_DIST=zipf run $v zipf; done; done
for i in 1 2; do for v in base rowpoll; do LSB_FORCE_EXCHANGE=1 LSB_RADIX_BITS=16 run $v x16; done; done
for f in zipf x16; do echo "== $f"; python tools/ab_summary.py $O/$f.log; grep -c "verify=(True" $O/$f.log || true; done
LSB_LIBRARY=abtest/rowpoll/liblsb.so timeout -k 10 400 python -u -m pytest tests/test_onesweep_gpu.py tests/test_exchange_onesweep_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || true
tail -1 $O/tests.log
