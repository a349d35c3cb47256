#!/bin/bash
# The gathered pass back on wave 0's descriptor hand-over through LDS (the
# per-wave scalar descriptor loads of ba33369 gave one wrong answer in three
# full suites: test_world_of_one_large_calls[28-8-1], profiles/r06/gather/
# sdesc_failure.log), kept: the L2 prefetch of the descriptor 64 tiles ahead
# and the LDS slot recomputed at the loop top (no spill reload).  A/B against
# the commit before ba33369, then the exchange-path suites, the large-call
# test three times, and the gathered tests under the debug build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=$R/gpurun_out/r06_g19; mkdir -p $O
B=$R/distributed-lsb_amd/build
TAG=r06_g19 ROUNDS=4 FORMS="uniform x16 x16zipf" bash tools/ab.sh pre=$B/ab_pre/liblsb.so new=$B/liblsb.so > $O/ab.log 2>&1 \
  || { tail -20 $O/ab.log; exit 1; }
tail -14 $O/ab.log
timeout -k 10 900 python -u -m pytest tests/test_exchange_onesweep_gpu.py tests/test_chunked_exchange_gpu.py \
  tests/test_rccl_multirank_gpu.py tests/test_gpu_sort.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 2 3; do
  timeout -k 10 300 python -u -m pytest "tests/test_gpu_sort.py::test_world_of_one_large_calls" -m gpu -x -q \
    --timeout 300 --timeout-method thread >> $O/large_calls.log 2>&1 || { tail -30 $O/large_calls.log; exit 1; }
done
grep -c passed $O/large_calls.log
LSB_LIBRARY=$B/debug/liblsb.so timeout -k 10 600 python -u -m pytest tests/test_exchange_onesweep_gpu.py \
  tests/test_chunked_exchange_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "not real_rccl" \
  > $O/tests_debug.log 2>&1 || { tail -30 $O/tests_debug.log; exit 1; }
tail -1 $O/tests_debug.log
