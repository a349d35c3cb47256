#!/bin/bash
# A/B of the skewed write-out's next-digit adds (Zipf keys, P = 1):
#   z0 add_slot_runs on every wave-instruction (DPP run heads)
#   z1 add_slot_runs only where the 64 records share one bucket, else plain adds
#   z2 one add where the 64 records share one slot, else plain adds
# base = HEAD (run heads through ds_bpermute).  Then uniform keys and the forced
# 16-bit exchange (k_place's run-aggregated adds), base vs z0.
set -euo pipefail
O=gpurun_out/ab4
mkdir -p $O
LSB_DIST=zipf AB_LOG=$O/zipf.log ROUNDS=5 bash tools/ab.sh abtest/base/liblsb.so abtest/z0/liblsb.so abtest/z1/liblsb.so abtest/z2/liblsb.so
AB_LOG=$O/uniform.log ROUNDS=4 bash tools/ab.sh abtest/base/liblsb.so abtest/z0/liblsb.so
LSB_RADIX_BITS=16 LSB_FORCE_EXCHANGE=1 LSB_DIST=zipf AB_LOG=$O/x16_zipf.log ROUNDS=3 bash tools/ab.sh abtest/base/liblsb.so abtest/z0/liblsb.so
LSB_RADIX_BITS=16 LSB_FORCE_EXCHANGE=1 AB_LOG=$O/x16_uniform.log ROUNDS=3 bash tools/ab.sh abtest/base/liblsb.so abtest/z0/liblsb.so
for f in zipf uniform x16_zipf x16_uniform; do echo "== $f"; python tools/ab_summary.py $O/$f.log; done
