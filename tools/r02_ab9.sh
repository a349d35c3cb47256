#!/bin/bash
# Look-back chain length vs sub-array count: every pass counts its own digit
# (k_subhist per pass, no fused next-digit histogram: LSB_NOFUSE) with 8, 16
# or 32 sub-arrays, so only the chains differ; phase profiles at 8 and 16.
set -euo pipefail
O=gpurun_out/ab9
mkdir -p $O
AB_LOG=$O/uniform.log ROUNDS=3 bash tools/ab.sh abtest/base/liblsb.so abtest/nf8/liblsb.so abtest/nf16/liblsb.so abtest/nf32/liblsb.so
python tools/ab_summary.py $O/uniform.log
for v in pnf8 pnf16; do
  LSB_LIBRARY=abtest/$v/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 > $O/$v.log 2>&1
  echo $v; cat $O/$v.log
done
