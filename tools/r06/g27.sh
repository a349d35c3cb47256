#!/bin/bash
# g26: loopback contexts 8 of 8 right, RCCL contexts with no records through
# RCCL 8 of 8 right, the control 6 of 8 wrong.  generate() gives every
# repetition the same input, so a buffer's leftovers from an earlier context
# can hide a read of stale data.  Here: the current allocation (later RCCL
# contexts hipMalloc'd) with other input per repetition; LSB_RCCL_VMM=1 with
# the device drained around every RCCL call (LSB_RCCL_SYNC=1), same input and
# other input.  Stops at the first run that ends other than 0.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=$R/gpurun_out/r06_g27; mkdir -p $O
run() {  # tag env...
  local tag=$1; shift
  echo "== $tag"
  env LP_QUICK=1 "$@" timeout -k 10 400 python -u tools/r06/large_call_probe.py 28 8 1 8 > $O/$tag.log 2>&1
  local rc=$?
  grep '^{' $O/$tag.log | cut -c1-300
  echo "rc=$rc"
  return $rc
}
run current_seeded LP_SEED=1 &&
run vmm_sync LSB_RCCL_VMM=1 LSB_RCCL_SYNC=1 &&
run vmm_sync_seeded LSB_RCCL_VMM=1 LSB_RCCL_SYNC=1 LP_SEED=1 &&
run vmm_seeded LSB_RCCL_VMM=1 LP_SEED=1
