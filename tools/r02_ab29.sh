#!/bin/bash
# k_onesweep: bucket t's per-wave counts kept in registers across the tile
# scan, each wave's start written once ("fused") vs the column scan written
# twice (HEAD).  Uniform + Zipf 2^30, then the single-read tests on "fused".
set -euo pipefail
O=gpurun_out/ab29
mkdir -p $O
rm -f $O/*.log
LSB_LIBRARY=abtest/base/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 > /dev/null 2>&1
run() { echo "lib=$1" >> $O/$2.log; LSB_LIBRARY=abtest/$1/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 >> $O/$2.log 2>&1; }
for i in 1 2 3 4 5 6; do
  if [ $((i % 2)) = 1 ]; then for v in base fused; do run $v uniform; done
  else for v in fused base; do run $v uniform; done; fi
done
for i in 1 2 3; do for v in base fused; do LSB_DIST=zipf run $v zipf; done; done
for f in uniform zipf; do echo "== $f"; python tools/ab_summary.py $O/$f.log; grep -c "verify=(True" $O/$f.log || true; done
LSB_LIBRARY=abtest/fused/liblsb.so timeout -k 10 400 python -u -m pytest tests/test_onesweep_gpu.py tests/test_exchange_onesweep_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || true
tail -1 $O/tests.log
