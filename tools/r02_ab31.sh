#!/bin/bash
# k_onesweep look-back walked at raised wave priority (s_setprio 2 / 3 from
# the first poll to the inclusive store, -DLSB_OS_PRIO=N) vs HEAD.
# Uniform + Zipf at 2^30, then the single-read tests on the better variant.
set -euo pipefail
O=gpurun_out/ab31
mkdir -p $O
rm -f $O/*.log
LSB_LIBRARY=abtest/base/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 > /dev/null 2>&1
run() { echo "lib=$1" >> $O/$2.log; LSB_LIBRARY=abtest/$1/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 >> $O/$2.log 2>&1; }
for i in 1 2 3 4 5 6; do
  if [ $((i % 2)) = 1 ]; then for v in base prio2 prio3; do run $v uniform; done
  else for v in prio3 prio2 base; do run $v uniform; done; fi
done
echo "== uniform"; python tools/ab_summary.py $O/uniform.log; grep -c "verify=(True" $O/uniform.log || true
for i in 1 2; do for v in base prio2 prio3; do LSB_DIST=zipf run $v zipf; done; done
echo "== zipf"; python tools/ab_summary.py $O/zipf.log; grep -c "verify=(True" $O/zipf.log || true
LSB_LIBRARY=abtest/prio3/liblsb.so timeout -k 10 400 python -u -m pytest tests/test_onesweep_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || true
tail -1 $O/tests.log
