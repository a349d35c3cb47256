#!/bin/bash
# The probe without back passes (working tree) against the last commit's:
# bench.py in fresh processes, alternated, then creation time of each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=$R/gpurun_out/r06_g9; mkdir -p $O
TAG=r06_g9 FORMS="head r06" ROUNDS=${ROUNDS:-4} bash tools/r06/probe_ab.sh || exit 1
for k in 1 2; do
  for f in head r06; do
    L=$R/distributed-lsb_amd/build/liblsb.so; [ $f = head ] && L=$R/distributed-lsb_amd/build/ab_head/liblsb.so
    LSB_LIBRARY=$L timeout -k 10 200 python -u tools/r05/create_time.py 1 > $O/create_${f}_$k.log 2>&1 || { tail -20 $O/create_${f}_$k.log; exit 1; }
    echo "$f $k: $(tr '\n' ' ' < $O/create_${f}_$k.log)"
  done
done
