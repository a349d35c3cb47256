#!/bin/bash
# Hot next-digit slot counted in registers in skewed launches (abtest/hs = working tree) against HEAD
# (base) and the DPP run-head write-out adds (z0); GPU suite on the tree first.
set -euo pipefail
O=gpurun_out/ab7
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 \
  || { tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
LSB_DIST=zipf AB_LOG=$O/zipf.log ROUNDS=5 bash tools/ab.sh abtest/base/liblsb.so abtest/z0/liblsb.so abtest/hs/liblsb.so
AB_LOG=$O/uniform.log ROUNDS=5 bash tools/ab.sh abtest/base/liblsb.so abtest/z0/liblsb.so abtest/hs/liblsb.so
for f in zipf uniform; do echo "== $f"; python tools/ab_summary.py $O/$f.log; done
