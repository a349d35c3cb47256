#!/bin/bash
# Round-2 GPU check: the parity suite, bench.py at N = 1 (live rocprofv3
# traffic passes + CPU baseline), and a gloo-transport rehearsal of the
# N > 1 bench line (2 ranks sharing the one GPU).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 \
  || { tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --transport gloo --n-per-gpu 16777216 --steps 2 --warmup 1 \
  --no-cpu-baseline > $O/bench_n2_gloo.log 2>&1 || { tail -20 $O/bench_n2_gloo.log; exit 1; }
tail -1 $O/bench_n2_gloo.log
