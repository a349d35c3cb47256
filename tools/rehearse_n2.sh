#!/bin/bash
# N = 2 rehearsal of bench.py on one GPU: two processes, gloo host collectives
# (lsb_create_rank_ops), default exchange form; usage: bash tools/rehearse_n2.sh [n_per_gpu]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
N=${1:-67108864}
mkdir -p $R/gpurun_out
timeout -k 10 240 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29511 $R/bench.py --gpus 2 --transport gloo --n-per-gpu $N --steps 2 --warmup 1 \
  > $R/gpurun_out/bench2g.log 2>&1 || { grep -v "^\[W" $R/gpurun_out/bench2g.log | grep -i "error\|lsb" | head -20; exit 1; }
tail -1 $R/gpurun_out/bench2g.log | cut -c1-600
