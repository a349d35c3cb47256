#!/bin/bash
# Is RCCL involved at all (g25: call size, grouped send/recv and copy engines
# change nothing; 2 placement candidates: 6 of 6 right)?  All with
# LSB_RCCL_VMM=1: the same sort in loopback contexts (self segment through the
# copy kernel, no RCCL); RCCL contexts without the forced exchange (no record
# goes through RCCL); the control again.
# Stops at the first run that ends other than 0.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=$R/gpurun_out/r06_g26; mkdir -p $O
run() {  # tag env...
  local tag=$1; shift
  echo "== $tag"
  env LP_QUICK=1 LSB_RCCL_VMM=1 "$@" timeout -k 10 300 python -u tools/r06/large_call_probe.py 28 8 1 8 > $O/$tag.log 2>&1
  local rc=$?
  grep '^{' $O/$tag.log | cut -c1-200
  echo "rc=$rc"
  return $rc
}
run loopback LP_LOOPBACK=1 &&
run noforce LP_NOFORCE=1 &&
run control LSB_X=0
