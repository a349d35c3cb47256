#!/bin/bash
# g27's seeded runs were checked by lsb_verify, which checks against
# generate()'s input: invalid.  Again with the host check (keys with their
# values, values a permutation, stable order): the current allocation (later
# RCCL contexts hipMalloc'd), hipMalloc everywhere, LSB_RCCL_VMM=1, and
# LSB_RCCL_VMM=1 with the device drained around every RCCL call.
# Stops at the first run that ends other than 0.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=$R/gpurun_out/r06_g28; mkdir -p $O
run() {  # tag env...
  local tag=$1; shift
  echo "== $tag"
  env LP_QUICK=1 LP_SEED=1 "$@" timeout -k 10 400 python -u tools/r06/large_call_probe.py 28 8 1 8 > $O/$tag.log 2>&1
  local rc=$?
  grep '^{' $O/$tag.log | cut -c1-300
  echo "rc=$rc"
  return $rc
}
run current_seeded LSB_X=0 &&
run malloc_seeded LSB_RECORD_ALLOC=malloc &&
run vmm_seeded LSB_RCCL_VMM=1 &&
run vmm_sync_seeded LSB_RCCL_VMM=1 LSB_RCCL_SYNC=1
