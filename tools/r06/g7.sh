#!/bin/bash
# Round 6: the SEG A/B (tools/r06/seg_ab3.sh), then three default bench
# processes (the headline's range on this box), then the N > 1 rehearsals
# over RCCL's socket transport with the chunked_* extra (gpu_round.sh n2 n4zipf n8).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=$R/gpurun_out/r06_g7; mkdir -p $O
bash tools/r06/seg_ab3.sh || exit 1
for k in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --steps 10 --warmup 3 > $O/bench_$k.log 2>&1 \
    || { tail -20 $O/bench_$k.log; exit 1; }
  tail -1 $O/bench_$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['placement']['chosen_ms'])"
done
TAG=r06_g7 RUN="n2 n4zipf n8" bash tools/gpu_round.sh
