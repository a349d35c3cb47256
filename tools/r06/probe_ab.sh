#!/bin/bash
# Round 6 placement probe (each candidate timed once as a destination, losers
# freed at once) against round 5's (a timed pass between every ordered pair
# of 4 candidates): bench.py at N = 1 in fresh processes, alternated.  The
# round-5 library is built from git revision 860dbc9 by tools/build_at.sh
# into distributed-lsb_amd/build/ab_r05; r06a (one timed pass per candidate,
# a histogram read before each) from commit 1220170 into build/ab_r06a;
# head: the last commit (FORMS="head r06": a working-tree change against it).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=$R/gpurun_out/${TAG:-r06_probe}; mkdir -p $O
declare -A LIB=([r05]=$R/distributed-lsb_amd/build/ab_r05/liblsb.so [r06]=$R/distributed-lsb_amd/build/liblsb.so
               [r06a]=$R/distributed-lsb_amd/build/ab_r06a/liblsb.so [head]=$R/distributed-lsb_amd/build/ab_head/liblsb.so)
F=${FORMS:-"r05 r06"}
for k in $(seq 1 ${ROUNDS:-4}); do
  list=$F; [ $((k % 2)) = 0 ] && list=$(echo $F | tr ' ' '\n' | tac | tr '\n' ' ')
  for f in $list; do
    LSB_LIBRARY=${LIB[$f]} timeout -k 10 200 python -u bench.py --steps ${STEPS:-10} --warmup 2 --no-extras \
      --no-traffic --no-cpu-baseline > $O/bench_${f}_$k.log 2>&1 || { echo "FAILED $f"; tail -30 $O/bench_${f}_$k.log; exit 1; }
    echo "$f round $k: $(grep '^{' $O/bench_${f}_$k.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); p=[x["ms"] for x in d["per_pass"]]; pl=d.get("placement", {}); print(d["ms_per_step"], d["verified"], "toB %.3f toA %.3f" % (sum(p[0::2]) / 4, sum(p[1::2]) / 4), {k: v for k, v in pl.items() if k in ("candidates", "chosen_ms", "first_pair_ms", "worst_ms")})')"
  done
done
