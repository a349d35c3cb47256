#!/bin/bash
# Diagnose test_world_of_one_large_calls[28-8-1]: two default bench processes
# first (the two failing runs had GPU work before the suite, the passing ones
# mostly not), then tools/r06/large_call_probe.py with the default 1 GiB call
# bound, with 512 MiB calls, and with every exchange placed.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=$R/gpurun_out/r06_g20; mkdir -p $O
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --no-traffic --steps 3 --warmup 1 > $O/churn_$k.log 2>&1 \
    || { tail -5 $O/churn_$k.log; exit 1; }
done
echo churned
timeout -k 10 500 python -u tools/r06/large_call_probe.py 28 8 1 4 2>&1 | tee $O/probe_default.log | cut -c1-600
