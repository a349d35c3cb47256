#!/bin/bash
# Robustness of the round-2 build: the GPU suite against the LSB_DEBUG build
# (device bounds asserts on every scattered store), then two processes
# sorting at once on one GPU, uniform keys and Zipf keys (split stage), every
# sort verified.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/robust
mkdir -p $O
cd $R
LSB_LIBRARY=distributed-lsb_amd/build/debug/liblsb.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q \
  --timeout 300 --timeout-method thread > $O/gputests_debug.log 2>&1 || { tail -40 $O/gputests_debug.log; exit 1; }
tail -2 $O/gputests_debug.log
bash tools/stress_two.sh 67108864 20 > $O/stress_uniform.log 2>&1 || { cat $O/stress_uniform.log; exit 1; }
tail -3 $O/stress_uniform.log
STRESS_ARGS="--dist zipf" bash tools/stress_two.sh 67108864 20 > $O/stress_zipf.log 2>&1 || { cat $O/stress_zipf.log; exit 1; }
tail -3 $O/stress_zipf.log
