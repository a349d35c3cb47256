#!/bin/bash
# The hybrid with and without the regional first pass (run from the repo
# root on the GPU box): the region tests, then bench.py --passes hybrid
# alternating LSB_REGION_FIRST=1 / 0 in fresh processes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r05_hyb}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_region_gpu.py -x -v --timeout 200 --timeout-method thread \
  > $O/region_tests.log 2>&1 || { echo "FAILED region tests"; tail -40 $O/region_tests.log; exit 1; }
tail -1 $O/region_tests.log
for k in $(seq 1 ${ROUNDS:-3}); do
  for f in 1 0; do
    LSB_REGION_FIRST=$f timeout -k 10 200 python -u bench.py --passes hybrid --steps 10 --warmup 2 --no-extras \
      --no-traffic --no-cpu-baseline > $O/bench_h_rf${f}_$k.log 2>&1 || { echo "FAILED rf$f"; tail -30 $O/bench_h_rf${f}_$k.log; exit 1; }
    echo "hybrid rf=$f round $k: $(grep '^{' $O/bench_h_rf${f}_$k.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["verified"], d["config"]["first_pass"], [p["ms"] for p in d["per_pass"]])')"
  done
done
