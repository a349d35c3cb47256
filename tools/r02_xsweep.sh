#!/bin/bash
# Per-digit exchange with single-read local passes: the new GPU tests, then the
# whole GPU suite, then per-kernel times of the exchange path (loopback and
# forced exchange, single-read vs reduce-then-scan local passes).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02x
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_exchange_onesweep_gpu.py tests/test_dist_ops_gpu.py -x -v --timeout 120 --timeout-method thread > $O/xtests.log 2>&1 \
  || { tail -40 $O/xtests.log; exit 1; }
tail -2 $O/xtests.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 \
  || { tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
timeout -k 10 300 python -u tools/exchange_profile.py > $O/exchange_profile.log 2>&1 || { tail -20 $O/exchange_profile.log; exit 1; }
cat $O/exchange_profile.log
