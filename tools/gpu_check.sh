#!/bin/bash
# GPU check: full parity suite, bench (N=1), 2-process gloo rehearsal of the N>1 bench (radix 64).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 700 python -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/gputests.log 2>&1 || { tail -40 $R/gpurun_out/gputests.log; exit 1; }
tail -2 $R/gpurun_out/gputests.log
timeout -k 10 240 python -u $R/bench.py --no-cpu-baseline > $R/gpurun_out/bench1.log 2>&1 || { tail -20 $R/gpurun_out/bench1.log; exit 1; }
tail -1 $R/gpurun_out/bench1.log
timeout -k 10 240 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 $R/bench.py --gpus 2 --transport gloo --n-per-gpu 67108864 --steps 2 --warmup 1 > $R/gpurun_out/bench2g.log 2>&1 || { tail -30 $R/gpurun_out/bench2g.log; exit 1; }
tail -1 $R/gpurun_out/bench2g.log
