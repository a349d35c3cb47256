#!/bin/bash
# k_onesweep with the ranked tile staged in two halves (32 KiB of LDS), so 3
# workgroups fit a CU (abtest/h2), against the shipped one-stage form (h1).
set -euo pipefail
O=gpurun_out/ab12
mkdir -p $O
AB_LOG=$O/uniform.log ROUNDS=3 bash tools/ab.sh abtest/h1/liblsb.so abtest/h2/liblsb.so
LSB_DIST=zipf AB_LOG=$O/zipf.log ROUNDS=2 bash tools/ab.sh abtest/h1/liblsb.so abtest/h2/liblsb.so
for f in uniform zipf; do echo "== $f"; python tools/ab_summary.py $O/$f.log; done
grep -c "verify=(True" $O/uniform.log
