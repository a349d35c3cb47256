#!/bin/bash
# round 5 check 3: the RCCL call cap between real ranks, the bench, the
# allocation counters.
set -u
O=gpurun_out/r05_v3
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_rccl_multirank_gpu.py -m gpu -x -q -k "two_gib or vmm" \
  --timeout 300 --timeout-method thread > $O/rccl_tests.log 2>&1 || { tail -30 $O/rccl_tests.log; exit 1; }
tail -1 $O/rccl_tests.log
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { tail -c 3000 $O/bench.log; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('$O/bench.log') if l.startswith('{')][-1])
print(d['value'], d['roofline']['avg_launch_ms'], [p['ms'] for p in d['per_pass']], d.get('hybrid_melem_s'), d.get('x16_melem_s'), d.get('x16_verified'), d.get('x16_error'))"
TAG=r05_allocpmc bash tools/r05/alloc_counters.sh > $O/allocpmc.log 2>&1 || { tail -20 $O/allocpmc.log; exit 1; }
cat $O/allocpmc.log
