#!/bin/bash
# Why a bench right after the whole GPU suite runs ~8 % slower (all passes
# 7.2-7.4 ms, every candidate buffer alike): the copy ceiling, the bench and
# the GPU's temperatures and clocks, fresh and again after the suite.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=$R/gpurun_out/r06_g17; mkdir -p $O
state() {
  (rocm-smi --showtemp --showclocks --showpower 2>&1 || true) > $O/smi_$1.txt
  timeout -k 10 120 tools/kbench/copybw 30 > $O/copybw_$1.txt 2>&1 || return 1
  timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --no-traffic --steps 5 --warmup 2 > $O/bench_$1.log 2>&1 || return 1
  echo "$1: $(grep -m3 'copy1 b256\|copyP8 g2048\|copy8 b256' $O/copybw_$1.txt | tr -s ' ' | tr '\n' ';') bench $(tail -1 $O/bench_$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["placement"]["chosen_ms"], d["placement"]["worst_ms"])')"
}
state fresh || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 \
  || { tail -20 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
state after_suite || exit 1
sleep 60
state after_60s || exit 1
