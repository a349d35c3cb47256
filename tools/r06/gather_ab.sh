#!/bin/bash
# A/B of the gathered pass's write-out / descriptor variants:
# tools/r06/gather_probe.py's gathered form (16-bit, exchange forced at P = 1,
# 2^30) per build, in fresh processes, the build order alternating per round.
# The variants were compile-time flags of lsb_kernels.hip in the working tree
# before commit ba33369, never committed (LSB_GATHER_BATCH, LSB_GATHER_EARLY_DESC, LSB_GATHER_LANESEL,
# LSB_GATHER_SDESC, LSB_GATHER_PF, LSB_GRAB_ASYNC; built by
# tools/build_variant.sh into build/ab_g_*); the shipped form is SDESC + PF 64,
# and LSB_GATHER_IDENTITY (build/ab_g_id) is still there.  Results:
# profiles/r06/gather/ (DESIGN.md §0).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=$R/gpurun_out/${TAG:-r06_gab}; mkdir -p $O
B=$R/distributed-lsb_amd/build
declare -A LIB=([base]=$B/liblsb.so [pre]=$B/ab_pre/liblsb.so [sdesc]=$B/ab_sdesc/liblsb.so [lid]=$B/ab_lid/liblsb.so)
F=${FORMS:-"pre base lid sdesc"}
for k in $(seq 1 ${ROUNDS:-3}); do
  list=$F; [ $((k % 2)) = 0 ] && list=$(echo $F | tr ' ' '\n' | tac | tr '\n' ' ')
  for f in $list; do
    GP_FORMS=gather LSB_LIBRARY=${LIB[$f]} timeout -k 10 200 python -u tools/r06/gather_probe.py 30 3 \
      > $O/${f}_$k.log 2>&1 || { echo "FAILED $f"; tail -20 $O/${f}_$k.log; exit 1; }
    echo "$f $k $(tail -1 $O/${f}_$k.log)"
  done
done
