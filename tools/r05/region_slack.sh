#!/bin/bash
# Builds of the regional first pass against each other (run from the repo
# root on the GPU box).  BUILDS: names of abtest/<name> builds
# (tools/build_variant.sh, made on the CPU side); "cur" is the tree's build,
# "rf0" the tree's build with LSB_REGION_FIRST=0 (the k_subhist start).
# Round 5: s16 = -DLSB_REGION_SIGMA=16 (131 tiles per region at 2^30), s6 =
# the default (130), s5 = -DLSB_REGION_SIGMA=5 -DLSB_REGION_DIV=1024 (129);
# stag = -DLSB_REGION_STAGGER=1.  TESTS=1: tests/test_region_gpu.py against
# every abtest build first.  bench.py per build, ROUNDS rounds in alternating
# order; prints the sort ms, the first two passes' ms and the count kernel's.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r05_slack}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
B=${BUILDS:-"s16 s6 s5 rf0"}
lib_of() { case $1 in cur|rf0) echo distributed-lsb_amd/build/liblsb.so ;; *) echo abtest/$1/liblsb.so ;; esac; }
if [ -n "${TESTS:-}" ]; then
  for b in $B; do
    case $b in cur|rf0) continue ;; esac
    LSB_LIBRARY=$(lib_of $b) timeout -k 10 600 python -u -m pytest tests/test_region_gpu.py -x -q --timeout 200 \
      --timeout-method thread > $O/tests_$b.log 2>&1 || { echo "FAILED tests $b"; tail -30 $O/tests_$b.log; exit 1; }
    echo "tests $b: $(tail -1 $O/tests_$b.log)"
  done
fi
for k in $(seq 1 ${ROUNDS:-3}); do
  list=$B; [ $((k % 2)) = 0 ] && list=$(echo $B | tr ' ' '\n' | tac | tr '\n' ' ')
  for b in $list; do
    envs=""; [ $b = rf0 ] && envs="LSB_REGION_FIRST=0"
    env $envs LSB_LIBRARY=$(lib_of $b) timeout -k 10 200 python -u bench.py --steps ${STEPS:-10} --warmup 2 --no-extras \
      --no-traffic --no-cpu-baseline > $O/bench_${b}_$k.log 2>&1 || { echo "FAILED $b"; tail -30 $O/bench_${b}_$k.log; exit 1; }
    echo "$b round $k: $(grep '^{' $O/bench_${b}_$k.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); p=[x["ms"] for x in d["per_pass"]]; print(d["ms_per_step"], d["verified"], "count", d["kernel_ms_per_step"]["upsweep"], "p0 %.3f p1 %.3f rest %.3f" % (p[0], p[1], sum(p[2:]) / len(p[2:])))')"
  done
done
