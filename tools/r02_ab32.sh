#!/bin/bash
# k_onesweep whole stage at 16 waves x 4 records (1024 threads, -DLSB_OS_BLOCK=1024;
# the compiler caps it at 64 VGPRs and spills 53) against the shipped 8 x 8:
# the onesweep GPU tests on the variant, then interleaved uniform sorts of 2^30.
set -euo pipefail
O=gpurun_out/ab32
mkdir -p $O
rm -f $O/*.log
LSB_LIBRARY=abtest/b1024/liblsb.so timeout -k 10 400 python -u -m pytest tests/test_onesweep_gpu.py -x -q \
  --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
LSB_LIBRARY=abtest/base/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 > /dev/null 2>&1
run() { echo "lib=$1" >> $O/$2.log; LSB_LIBRARY=abtest/$1/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 >> $O/$2.log 2>&1; }
for i in 1 2 3 4; do
  if [ $((i % 2)) = 1 ]; then for v in base b1024; do run $v uniform; done
  else for v in b1024 base; do run $v uniform; done; fi
done
echo "== uniform"; python tools/ab_summary.py $O/uniform.log; grep -c "verify=(True" $O/uniform.log || true
