#!/bin/bash
# rocprofv3 evidence (tools/profile.sh) and the bench line, back to back on one box.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
bash $R/tools/profile.sh > $R/gpurun_out/profile.log 2>&1 || { tail -20 $R/gpurun_out/profile.log; exit 1; }
cd $R && timeout -k 10 400 python -u bench.py > $R/gpurun_out/bench_full.log 2>&1 || { tail -20 $R/gpurun_out/bench_full.log; exit 1; }
tail -1 $R/gpurun_out/bench_full.log | cut -c1-200
