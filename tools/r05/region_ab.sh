#!/bin/bash
# The regional first pass on the GPU box (run from the repo root):
#   its GPU tests, then bench.py alternating LSB_REGION_FIRST=1 / 0 in fresh
#   processes (ROUNDS pairs, --no-extras --no-traffic --no-cpu-baseline).
# Output: gpurun_out/$TAG/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r05_rg}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_region_gpu.py -x -v --timeout 200 --timeout-method thread \
    > $O/region_tests.log 2>&1 || { echo "FAILED region tests"; tail -40 $O/region_tests.log; exit 1; }
  tail -2 $O/region_tests.log
fi
for k in $(seq 1 ${ROUNDS:-3}); do
  for f in 1 0; do
    LSB_REGION_FIRST=$f timeout -k 10 200 python -u bench.py --steps ${STEPS:-10} --warmup 2 --no-extras \
      --no-traffic --no-cpu-baseline > $O/bench_rf${f}_$k.log 2>&1 || { echo "FAILED bench rf$f"; tail -30 $O/bench_rf${f}_$k.log; exit 1; }
    echo "rf=$f round $k: $(grep '^{' $O/bench_rf${f}_$k.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["verified"] if "verified" in d else "", d["kernel_ms_per_step"]["upsweep"], [p["ms"] for p in d["per_pass"]])')"
  done
done
