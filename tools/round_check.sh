#!/bin/bash
# Full GPU parity suite, then the rocprofv3 evidence of bench.py (stats +
# FETCH_SIZE + WRITE_SIZE passes, tools/profile.sh), then bench.py itself
# with its CPU baseline.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 700 python -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/gputests.log 2>&1 || { tail -40 $R/gpurun_out/gputests.log; exit 1; }
tail -2 $R/gpurun_out/gputests.log
bash $R/tools/profile.sh > $R/gpurun_out/profile.log 2>&1 || { tail -20 $R/gpurun_out/profile.log; exit 1; }
cd $R && timeout -k 10 400 python -u bench.py > $R/gpurun_out/bench_full.log 2>&1 || { tail -20 $R/gpurun_out/bench_full.log; exit 1; }
tail -1 $R/gpurun_out/bench_full.log
