#!/bin/bash
# rocprofv3 evidence for bench.py (run on the GPU box from the repo root):
#   1. kernel trace + stats   -> gpurun_out/prof/stats/
#   2. FETCH_SIZE pass        -> gpurun_out/prof/fetch/
#   3. WRITE_SIZE pass        -> gpurun_out/prof/write/
# Counter passes are separate runs with --kernel-trace only (no sys/runtime trace).
# --no-traffic: bench.py must not start its own rocprofv3 passes under this one.
# PROF=<dir under gpurun_out> (default prof), BENCH_ARGS="--passes hybrid" etc.
set -euo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${PROF:-prof}
STEPS=${STEPS:-3}
EXTRA=${BENCH_ARGS:-}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
# --no-extras: no second GPU process (the hybrid extra) under the profiler;
# profile the hybrid explicitly with BENCH_ARGS="--passes hybrid".
BENCH="$REPO/bench.py --steps $STEPS --warmup 1 --no-cpu-baseline --no-traffic --no-extras $EXTRA"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- python3 $BENCH > "$OUT/stats.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 $REPO/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-traffic --no-extras $EXTRA > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 $REPO/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-traffic --no-extras $EXTRA > "$OUT/write.log" 2>&1
find "$OUT" -name "*.csv" | sort
