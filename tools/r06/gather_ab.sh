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
declare -A LIB=([base]=$B/liblsb.so [e1]=$B/ab_g_e1/liblsb.so [b4]=$B/ab_g_b4/liblsb.so [b8]=$B/ab_g_b8/liblsb.so
               [b4l]=$B/ab_g_b4l/liblsb.so [id]=$B/ab_g_id/liblsb.so [ls]=$B/ab_g_ls/liblsb.so [sd]=$B/ab_g_sd/liblsb.so [pf64]=$B/ab_g_pf64/liblsb.so [pf128]=$B/ab_g_pf128/liblsb.so [pf256]=$B/ab_g_pf256/liblsb.so)
F=${FORMS:-"base e1 b4 b8 b4l"}
for k in $(seq 1 ${ROUNDS:-3}); do
  list=$F; [ $((k % 2)) = 0 ] && list=$(echo $F | tr ' ' '\n' | tac | tr '\n' ' ')
  for f in $list; do
    GP_FORMS=gather LSB_LIBRARY=${LIB[$f]} timeout -k 10 200 python -u tools/r06/gather_probe.py 30 3 \
      > $O/${f}_$k.log 2>&1 || { echo "FAILED $f"; tail -20 $O/${f}_$k.log; exit 1; }
    echo "$f $k $(tail -1 $O/${f}_$k.log)"
  done
done
