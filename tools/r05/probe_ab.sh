#!/bin/bash
# The opt-in placement probe over VMM record buffers against no probe (run
# from the repo root on the GPU box).  tools/kbench/pairbw2.hip found that a
# buffer of 1 GiB pieces can be a slow LSD-pass destination as a whole (8-piece
# buffers: 3.7-3.9 against 2.9 ms; 16-piece: 5.71-5.96 ms), so choosing A and
# B among K candidates may remove the slow direction some boxes show.
# FORMS: "k0" (no probe, the default) and "kN" (LSB_PLACEMENT_CANDIDATES=N).
# bench.py per form in fresh processes, ROUNDS rounds in alternating order;
# prints the sort ms, the mean of the passes into B (even) and into A (odd),
# and the probe's own figures.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r05_probe}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
F=${FORMS:-"k0 k4"}
for k in $(seq 1 ${ROUNDS:-4}); do
  list=$F; [ $((k % 2)) = 0 ] && list=$(echo $F | tr ' ' '\n' | tac | tr '\n' ' ')
  for f in $list; do
    envs="LSB_PLACEMENT_CANDIDATES=${f#k}"
    env $envs timeout -k 10 200 python -u bench.py --steps ${STEPS:-10} --warmup 2 --no-extras \
      --no-traffic --no-cpu-baseline > $O/bench_${f}_$k.log 2>&1 || { echo "FAILED $f"; tail -30 $O/bench_${f}_$k.log; exit 1; }
    echo "$f round $k: $(grep '^{' $O/bench_${f}_$k.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); p=[x["ms"] for x in d["per_pass"]]; pl=d.get("placement", {}); print(d["ms_per_step"], d["verified"], "toB %.3f toA %.3f" % (sum(p[0::2]) / 4, sum(p[1::2]) / 4), {k: v for k, v in pl.items() if k in ("candidates", "chosen_ms", "first_pair_ms", "worst_ms")})')"
  done
done
