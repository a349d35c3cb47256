#!/bin/bash
# Round 6, first GPU check: the new teardown / advisor tests, the pure-RCCL
# big-call probe, the stress pair replay under the debug build, creation time
# and the default bench (new placement probe).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=$R/gpurun_out/r06_g1; mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
echo "== tests $(date +%T)"
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_teardown_gpu.py tests/test_region_gpu.py tests/test_footprint_gpu.py \
  "tests/test_rccl_multirank_gpu.py::test_real_rccl_ranks_cut_calls" -k "not default_threshold" \
  > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
fi
echo "== rccl_big $(date +%T)"
tools/rccl_big_call.sh $O/rccl_big > $O/rccl_big.log 2>&1 || { tail -30 $O/rccl_big.log; exit 1; }
cat $O/rccl_big.log
echo "== replay $(date +%T)"
LSB_LIBRARY=$R/distributed-lsb_amd/build/debug/liblsb.so timeout -k 10 300 python -u tools/teardown_probe.py --replay 3 \
  > $O/replay.log 2>&1 || { tail -30 $O/replay.log; exit 1; }
tail -3 $O/replay.log; grep -c "teardown check" $O/replay.log || true
echo "== legacy $(date +%T)"
LSB_TEARDOWN_LEGACY=1 LSB_LIBRARY=$R/distributed-lsb_amd/build/debug/liblsb.so timeout -k 10 200 python -u tools/teardown_probe.py --per 33554432 \
  > $O/legacy.log 2>&1 || { tail -30 $O/legacy.log; exit 1; }
tail -1 $O/legacy.log; echo "legacy check lines: $(grep -c 'teardown check' $O/legacy.log || true)"
echo "== create $(date +%T)"
timeout -k 10 200 python -u tools/r05/create_time.py 2 > $O/create_time.log 2>&1 || { tail -30 $O/create_time.log; exit 1; }
cat $O/create_time.log
echo "== bench $(date +%T)"
timeout -k 10 500 python -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-600
