#!/bin/bash
# k_onesweep with 512-thread workgroups (8 waves, 8 records per thread, same
# 4096-record tile and 64 KiB stage; threads >= 256 take no bucket role;
# 16-bit per-wave counters) against the shipped 256 x 16.  Uniform 2^30
# sorts interleaved, then the variant through the onesweep GPU tests.
set -euo pipefail
O=gpurun_out/ab26
mkdir -p $O
rm -f $O/*.log
LSB_LIBRARY=abtest/base/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 > /dev/null 2>&1
run() { echo "lib=$1" >> $O/$2.log; LSB_LIBRARY=abtest/$1/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 >> $O/$2.log 2>&1; }
for i in 1 2 3 4 5; do
  if [ $((i % 2)) = 1 ]; then for v in base os256 os512; do run $v uniform; done
  else for v in os512 os256 base; do run $v uniform; done; fi
done
python tools/ab_summary.py $O/uniform.log
grep -c "verify=(True" $O/uniform.log || true
LSB_LIBRARY=abtest/os512/liblsb.so timeout -k 10 400 python -u -m pytest tests/test_onesweep_gpu.py tests/test_exchange_onesweep_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests512.log 2>&1 || true
tail -3 $O/tests512.log
