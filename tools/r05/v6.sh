#!/bin/bash
# round 5 check 6: RCCL call cutting by the exchange's largest segment
set -u
O=gpurun_out/r05_v6
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_sort.py tests/test_rccl_multirank_gpu.py tests/test_merge_exchange_gpu.py \
  tests/test_dist_ops_gpu.py -m gpu -x -q -k "world_of_one or rccl or merge or processes" --timeout 300 \
  --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python3 tools/r05/x16_probe.py 30 0 0 1 > $O/x16.log 2>&1 || { cat $O/x16.log; exit 1; }
cat $O/x16.log
