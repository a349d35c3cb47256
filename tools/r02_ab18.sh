#!/bin/bash
# The 8192-record-tile build (abtest/t8s = working tree) against the
# previous one (abtest/auto): GPU suite; uniform and Zipf at P = 1; the
# forced 16-bit exchange (the high-byte pass's 65536 counts, k_place).
set -euo pipefail
O=gpurun_out/ab18
mkdir -p $O
rm -f $O/*.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 \
  || { tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
LSB_LIBRARY=abtest/auto/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 > /dev/null 2>&1
AB_LOG=$O/uniform.log ROUNDS=4 bash tools/ab.sh abtest/auto/liblsb.so abtest/t8s/liblsb.so
LSB_DIST=zipf AB_LOG=$O/zipf.log ROUNDS=3 bash tools/ab.sh abtest/auto/liblsb.so abtest/t8s/liblsb.so
LSB_RADIX_BITS=16 LSB_FORCE_EXCHANGE=1 AB_LOG=$O/x16_uniform.log ROUNDS=2 bash tools/ab.sh abtest/auto/liblsb.so abtest/t8s/liblsb.so
LSB_RADIX_BITS=16 LSB_FORCE_EXCHANGE=1 LSB_DIST=zipf AB_LOG=$O/x16_zipf.log ROUNDS=2 bash tools/ab.sh abtest/auto/liblsb.so abtest/t8s/liblsb.so
for f in uniform zipf x16_uniform x16_zipf; do echo "== $f"; python tools/ab_summary.py $O/$f.log; done
