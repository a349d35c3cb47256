#!/bin/bash
# Released VMM buffers: memory returned? addresses reused?  (tools/r06/va_check.py
# in the three address modes), then the large-call probe in the hint mode.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=$R/gpurun_out/r06_g23; mkdir -p $O
for m in retire reuse hint; do
  echo "== $m"
  LSB_VMM_TRACE=1 LSB_VMM_VA_MODE=$m timeout -k 10 300 python -u tools/r06/va_check.py 28 4 > $O/va_$m.log 2>&1 \
    || { tail -20 $O/va_$m.log; exit 1; }
  grep "context" $O/va_$m.log
  grep "reserve" $O/va_$m.log | awk '{print $3}' | sort | uniq -c | sort -rn | head -3
  echo "distinct reserved addresses: $(grep reserve $O/va_$m.log | awk '{print $3}' | sort -u | wc -l) of $(grep -c reserve $O/va_$m.log)"
done
echo "== probe hint"
LP_QUICK=1 LSB_VMM_VA_MODE=hint timeout -k 10 300 python -u tools/r06/large_call_probe.py 28 8 1 6 2>&1 | tee $O/probe_hint.log | grep '^{' | cut -c1-140
