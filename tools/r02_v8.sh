#!/bin/bash
# Round-2 check of the final round-2 tree (container rebuilt): full GPU suite, bench.py
# (live PMC traffic + CPU baseline), rocprofv3 stats + FETCH/WRITE passes,
# then the single-read tests against the LSB_DEBUG (bounds-assert) build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02v8
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 \
  || { tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
STEPS=3 bash tools/profile.sh > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }
LSB_LIBRARY=distributed-lsb_amd/build/debug/liblsb.so timeout -k 10 600 python -u -m pytest tests/test_onesweep_gpu.py \
  tests/test_exchange_onesweep_gpu.py -x -q --timeout 300 --timeout-method thread > $O/debugtests.log 2>&1 \
  || { tail -30 $O/debugtests.log; exit 1; }
tail -1 $O/debugtests.log
echo done
