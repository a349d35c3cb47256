#!/bin/bash
# Round 6, after the host range checks on exchange copies, the debug-build
# bounds asserts on gathered reads and the probe without back passes: the GPU
# suite, smoke, creation time (off / default, alternated) and three default
# bench processes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=$R/gpurun_out/r06_g8; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/gputests.log 2>&1 || { tail -30 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 200 python -u tools/r05/create_time.py 3 > $O/create_time.log 2>&1 || { tail -30 $O/create_time.log; exit 1; }
cat $O/create_time.log
for k in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --steps 10 --warmup 3 > $O/bench_$k.log 2>&1 \
    || { tail -20 $O/bench_$k.log; exit 1; }
  tail -1 $O/bench_$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['placement'])"
done
