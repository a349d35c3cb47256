#!/bin/bash
# Split-stage k_onesweep chosen per sort (abtest/auto = working tree) against
# the whole-stage build (abtest/h1): GPU suite first, then uniform and Zipf.
set -euo pipefail
O=gpurun_out/ab13
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 \
  || { tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
AB_LOG=$O/uniform.log ROUNDS=3 bash tools/ab.sh abtest/h1/liblsb.so abtest/auto/liblsb.so
LSB_DIST=zipf AB_LOG=$O/zipf.log ROUNDS=3 bash tools/ab.sh abtest/h1/liblsb.so abtest/auto/liblsb.so
for f in uniform zipf; do echo "== $f"; python tools/ab_summary.py $O/$f.log; done
