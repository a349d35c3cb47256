#!/bin/bash
# The fix for the world-of-one large-call wrong answer: VMM address ranges
# retired instead of reused.  tools/r06/large_call_probe.py, 6 contexts per
# process, with the fix and with LSB_VMM_REUSE_VA=1 (the old behaviour);
# then the test itself three times, and tests/test_gpu_sort.py.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=$R/gpurun_out/r06_g22; mkdir -p $O
run() {  # tag env...
  local tag=$1; shift
  echo "== $tag"
  env LP_QUICK=1 "$@" timeout -k 10 300 python -u tools/r06/large_call_probe.py 28 8 1 6 2>&1 | tee $O/$tag.log | grep '^{' | cut -c1-150
}
run retired LSB_X=0
run reuse LSB_VMM_REUSE_VA=1
for k in 1 2 3; do
  timeout -k 10 300 python -u -m pytest "tests/test_gpu_sort.py::test_world_of_one_large_calls" -m gpu -x -q \
    --timeout 300 --timeout-method thread > $O/large_calls_$k.log 2>&1 || { tail -30 $O/large_calls_$k.log; exit 1; }
  tail -1 $O/large_calls_$k.log
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_sort.py tests/test_rccl_multirank_gpu.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
