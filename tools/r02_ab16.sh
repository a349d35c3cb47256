#!/bin/bash
# Bigger register-held tiles through a half-tile LDS stage, 2 workgroups per
# CU: 6144-record tiles (t6, 48 KiB stage) and 8192-record tiles (t8, 64 KiB
# stage), split stage forced (LSB_SPLIT=2), against the shipped build (auto).
set -euo pipefail
O=gpurun_out/ab16
mkdir -p $O
rm -f $O/*.log
for dist in uniform zipf; do
  for i in 1 2 3; do
    echo "lib=auto" >> $O/$dist.log; LSB_DIST=$dist LSB_LIBRARY=abtest/auto/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 >> $O/$dist.log 2>&1
    for v in t6 t8; do
      echo "lib=$v" >> $O/$dist.log
      LSB_DIST=$dist LSB_SPLIT=2 LSB_LIBRARY=abtest/$v/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 >> $O/$dist.log 2>&1 || true
    done
  done
  echo "== $dist"; python tools/ab_summary.py $O/$dist.log
done
grep -c "verify=(True" $O/uniform.log $O/zipf.log || true
