#!/bin/bash
# Region slack vs the pass over the regional layout (run from the repo root on
# the GPU box).  Builds (tools/build_variant.sh, made on the CPU side):
#   abtest/s16  -DLSB_REGION_SIGMA=16          (131 tiles per region at 2^30)
#   abtest/s6   the default                    (130)
#   abtest/s5   -DLSB_REGION_SIGMA=5 -DLSB_REGION_DIV=1024   (129)
# plus the default build with LSB_REGION_FIRST=0 (the k_subhist start).
# bench.py per build, ROUNDS rounds in alternating order; prints the sort
# ms, the first two passes' ms and the count kernel's.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r05_slack}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
B="s16 s6 s5 rf0"
for k in $(seq 1 ${ROUNDS:-3}); do
  list=$B; [ $((k % 2)) = 0 ] && list=$(echo $B | tr ' ' '\n' | tac | tr '\n' ' ')
  for b in $list; do
    lib=abtest/$b/liblsb.so; envs=""
    [ $b = rf0 ] && { lib=distributed-lsb_amd/build/liblsb.so; envs="LSB_REGION_FIRST=0"; }
    env $envs LSB_LIBRARY=$lib timeout -k 10 200 python -u bench.py --steps ${STEPS:-10} --warmup 2 --no-extras \
      --no-traffic --no-cpu-baseline > $O/bench_${b}_$k.log 2>&1 || { echo "FAILED $b"; tail -30 $O/bench_${b}_$k.log; exit 1; }
    echo "$b round $k: $(grep '^{' $O/bench_${b}_$k.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); p=[x["ms"] for x in d["per_pass"]]; print(d["ms_per_step"], d["verified"], "count", d["kernel_ms_per_step"]["upsweep"], "p0 %.3f p1 %.3f rest %.3f" % (p[0], p[1], sum(p[2:]) / len(p[2:])))')"
  done
done
