#!/bin/bash
# The gathered pass's per-wave scalar descriptor loads (+ L2 prefetch of the
# descriptor 64 tiles ahead) against the last commit: interleaved A/B of the
# LSD sort and the forced 16-bit exchange (tools/ab.sh), the per-pass rows
# (tools/r06/gather_probe.py), then the exchange-path GPU suites on the new
# build, and the gathered exchange tests under the debug build (bounds
# asserts on every gathered read).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=$R/gpurun_out/r06_g15; mkdir -p $O
B=$R/distributed-lsb_amd/build
TAG=r06_g15 ROUNDS=4 FORMS="uniform x16 x16zipf" bash tools/ab.sh head=$B/ab_head/liblsb.so new=$B/liblsb.so > $O/ab.log 2>&1 \
  || { tail -20 $O/ab.log; exit 1; }
tail -14 $O/ab.log
GP_FORMS="gather placed plain" timeout -k 10 300 python -u tools/r06/gather_probe.py 30 3 > $O/gather_probe.log 2>&1 \
  || { tail -20 $O/gather_probe.log; exit 1; }
cat $O/gather_probe.log
timeout -k 10 900 python -u -m pytest tests/test_exchange_onesweep_gpu.py tests/test_chunked_exchange_gpu.py \
  tests/test_rccl_multirank_gpu.py tests/test_gpu_sort.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
LSB_LIBRARY=$B/debug/liblsb.so timeout -k 10 600 python -u -m pytest tests/test_exchange_onesweep_gpu.py \
  tests/test_chunked_exchange_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "not real_rccl" \
  > $O/tests_debug.log 2>&1 || { tail -30 $O/tests_debug.log; exit 1; }
tail -2 $O/tests_debug.log
