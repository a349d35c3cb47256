#!/bin/bash
# Round-2 evidence for the current build (split stage for skewed sorts):
#   GPU parity suite, bench.py at N = 1 (live --pmc traffic + CPU baseline),
#   rocprofv3 kernel stats + FETCH/WRITE passes (tools/profile.sh), and the SQ
#   counters (LDS bank conflicts, wait/issue shares) of k_onesweep at 2^28.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02v4
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 \
  || { tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
STEPS=3 bash tools/profile.sh > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }
SQ_TAG=_r02v4 bash tools/sq_counters.sh > $O/sq.log 2>&1 || { tail -20 $O/sq.log; exit 1; }

GRAFT_REPO_ROOT=$R bash tools/table_runs.sh > $O/table.log 2>&1 || { tail -20 $O/table.log; exit 1; }
cat $O/table.log | tail -6
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --transport gloo --n-per-gpu 16777216 --steps 2 --warmup 1 \
  --no-cpu-baseline > $O/bench_n2_gloo.log 2>&1 || { tail -20 $O/bench_n2_gloo.log; exit 1; }
tail -1 $O/bench_n2_gloo.log
