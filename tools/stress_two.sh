#!/bin/bash
# Two processes sorting on one GPU at once (tools/stress_onesweep.py).
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 150 python -u $R/tools/stress_onesweep.py --n ${1:-67108864} --iters ${2:-20} --tag A ${STRESS_ARGS:-} > $R/gpurun_out/stressA.log 2>&1 &
PA=$!
timeout -k 10 150 python -u $R/tools/stress_onesweep.py --n ${1:-67108864} --iters ${2:-20} --tag B ${STRESS_ARGS:-} > $R/gpurun_out/stressB.log 2>&1 &
PB=$!
wait $PA; RA=$?
wait $PB; RB=$?
tail -n 3 $R/gpurun_out/stressA.log $R/gpurun_out/stressB.log
echo "rc A=$RA B=$RB"
[ $RA -eq 0 ] && [ $RB -eq 0 ]
