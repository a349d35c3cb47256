#!/bin/bash
# test_world_of_one_large_calls[28-8-1]: after two good sorts in a process the
# third and fourth come back as garbage (zeros at the head, records lost;
# profiles/r06/large_call/g20).  Which allocation: the default (1 GiB VMM
# pieces, placement probe), hipMalloc'd record buffers, VMM without the
# probe, RCCL's local registration off.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=$R/gpurun_out/r06_g21; mkdir -p $O
run() {  # tag env...
  local tag=$1; shift
  echo "== $tag"
  env LP_QUICK=1 "$@" timeout -k 10 300 python -u tools/r06/large_call_probe.py 28 8 1 5 2>&1 | tee $O/$tag.log | grep '^{' | cut -c1-160
}
run default LSB_X=0
run malloc LSB_RECORD_ALLOC=malloc
run noprobe LSB_PLACEMENT_CANDIDATES=0
run noreg NCCL_LOCAL_REGISTER=0
