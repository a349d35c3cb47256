#!/bin/bash
# A/B of HEAD (abtest/base) against two working-tree builds:
#   abtest/dpp   run-aggregated next-digit adds through DPP (no ds_bpermute),
#                also in k_place
#   abtest/full  the same + full-tile instantiation of k_onesweep's load + rank
# uniform and Zipf keys at P = 1, then the forced 16-bit exchange path (k_place).
set -euo pipefail
O=gpurun_out/ab3
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 \
  || { tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
AB_LOG=$O/uniform.log ROUNDS=4 bash tools/ab.sh abtest/base/liblsb.so abtest/dpp/liblsb.so abtest/full/liblsb.so
LSB_DIST=zipf AB_LOG=$O/zipf.log ROUNDS=3 bash tools/ab.sh abtest/base/liblsb.so abtest/dpp/liblsb.so abtest/full/liblsb.so
LSB_RADIX_BITS=16 LSB_FORCE_EXCHANGE=1 LSB_DIST=zipf AB_LOG=$O/x16_zipf.log ROUNDS=2 bash tools/ab.sh abtest/base/liblsb.so abtest/full/liblsb.so
LSB_RADIX_BITS=16 LSB_FORCE_EXCHANGE=1 AB_LOG=$O/x16_uniform.log ROUNDS=2 bash tools/ab.sh abtest/base/liblsb.so abtest/full/liblsb.so
for f in uniform zipf x16_zipf x16_uniform; do echo "== $f"; python tools/ab_summary.py $O/$f.log; done
