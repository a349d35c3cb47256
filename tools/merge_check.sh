#!/bin/bash
# Whole-key exchange on the GPU box: its parity tests, then rocprofv3 kernel traces of
# tools/merge_profile.py at P = 2 and P = 8 logical ranks (gpurun_out/m2, m8).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/m2 $R/gpurun_out/m8
timeout -k 10 300 python -u -m pytest $R/tests/test_merge_exchange_gpu.py -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/merge_tests.log 2>&1 || { tail -30 $R/gpurun_out/merge_tests.log; exit 1; }
tail -2 $R/gpurun_out/merge_tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/m2 -o run -- python3 $R/tools/merge_profile.py --ranks 2 --n-per-rank 536870912 --reps 2 > $R/gpurun_out/m2/log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/m8 -o run -- python3 $R/tools/merge_profile.py --ranks 8 --n-per-rank 134217728 --reps 2 > $R/gpurun_out/m8/log 2>&1 || exit 1
grep -h "sort\|verify" $R/gpurun_out/m2/log $R/gpurun_out/m8/log
