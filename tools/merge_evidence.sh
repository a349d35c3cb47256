#!/bin/bash
# rocprofv3 evidence of the whole-key exchange in loopback (P logical ranks
# on one GPU): kernel stats at P = 2 and P = 8 (2^30 records in total), and
# the merge kernels' HBM bytes (tools/merge_pmc.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/ev2 $R/gpurun_out/ev8
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ev2 -o run -- python3 $R/tools/merge_profile.py --ranks 2 --n-per-rank 536870912 --reps 2 > $R/gpurun_out/ev2/log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ev8 -o run -- python3 $R/tools/merge_profile.py --ranks 8 --n-per-rank 134217728 --reps 2 > $R/gpurun_out/ev8/log 2>&1 || exit 1
grep -h "sort\|verify" $R/gpurun_out/ev2/log $R/gpurun_out/ev8/log
bash $R/tools/merge_pmc.sh
