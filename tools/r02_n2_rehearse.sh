#!/bin/bash
# N = 2 bench lines over gloo on one GPU (shape checks, not measurements):
# configs[3] (Zipf keys) and 8-bit exchange digits.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/n2
mkdir -p $O
cd $R
for args in "--dist zipf" "--radix-bits 8"; do
  tag=$(echo $args | tr -d ' -')
  timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --transport gloo --n-per-gpu 16777216 --steps 2 --warmup 1 \
    --no-cpu-baseline $args > $O/bench_$tag.log 2>&1 || { tail -20 $O/bench_$tag.log; exit 1; }
  tail -1 $O/bench_$tag.log | cut -c1-400
done
