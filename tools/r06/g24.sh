#!/bin/bash
# RCCL contexts after released VMM buffers take hipMalloc'd ones: the probe
# (6 contexts per process) with the fix and with LSB_RCCL_VMM=1, the
# large-call test three times, then the whole GPU suite.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=$R/gpurun_out/r06_g24; mkdir -p $O
run() {  # tag env...
  local tag=$1; shift
  echo "== $tag"
  env LP_QUICK=1 "$@" timeout -k 10 300 python -u tools/r06/large_call_probe.py 28 8 1 6 2>&1 | tee $O/$tag.log | grep '^{' | cut -c1-120
}
run fixed LSB_X=0
run forced_vmm LSB_RCCL_VMM=1
for k in 1 2 3; do
  timeout -k 10 300 python -u -m pytest "tests/test_gpu_sort.py::test_world_of_one_large_calls" -m gpu -x -q \
    --timeout 300 --timeout-method thread > $O/large_calls_$k.log 2>&1 || { tail -30 $O/large_calls_$k.log; exit 1; }
  tail -1 $O/large_calls_$k.log
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 \
  || { tail -30 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
